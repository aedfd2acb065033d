"""The DP product path on the GPU: siren_amd.training.train with the fused kernels (sine SingleBVPNet 5x256) and
fused_adam=True (FusedAdam.allreduce_grad: one count-weighted all-reduce of the flat bucket, then clip + Adam in
siren_adam_step), world size 2 with BOTH ranks on cuda:0 over gloo (gloo reduces CUDA tensors; RCCL is the same
code with the "nccl" backend, bench.py --gpus N). Parameters after 3 steps must equal single-process full-batch
training (training.py:95-104: clip after the reduced gradient). Needs an MI355X.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N, STEPS = 4096 + 37, 3


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch():
    g = torch.Generator().manual_seed(2)
    x = torch.rand(1, N, 2, generator=g) * 2 - 1
    return x, torch.sin(4 * x[..., :1]) * torch.cos(3 * x[..., 1:])


def _img_loss(out, gt):
    return {'img_loss': ((out['model_out'] - gt['img']) ** 2).mean()}


def _run(model, x, t, d):
    from siren_amd.training import train
    return train(model, [({'coords': x}, {'img': t})], epochs=STEPS, lr=1e-4, steps_til_summary=1000,
                 epochs_til_checkpoint=1000, model_dir=d, loss_fn=_img_loss, clip_grad=True, device='cuda',
                 log=lambda *a: None, fused_adam=True)


def _worker(rank, world, port, ret):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK='0')
    torch.cuda.set_device(0)
    from siren_amd import distributed as sd
    from siren_amd.modules import SingleBVPNet
    sd.init('gloo')
    torch.manual_seed(0)
    m = SingleBVPNet(verbose=False).cuda()
    x, t = _batch()
    a, b = sd.shard(N, world, rank)
    ret['n%d' % rank] = b - a
    with tempfile.TemporaryDirectory() as d:
        ret['loss%d' % rank] = _run(m, x[:, a:b], t[:, a:b], d)
    ret['p%d' % rank] = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().clone()
    torch.distributed.destroy_process_group()


def test_dp_world2_fused_adam_on_one_gpu_equals_full_batch(cuda):
    world, port = 2, _free_port()
    ret = mp.Manager().dict()
    mp.spawn(_worker, args=(world, port, ret), nprocs=world, join=True)
    assert ret['n0'] != ret['n1'] and ret['n0'] + ret['n1'] == N   # unequal shards (2048, 2085)
    assert torch.equal(ret['p0'], ret['p1'])
    from siren_amd.modules import SingleBVPNet
    torch.manual_seed(0)
    m = SingleBVPNet(verbose=False).to(cuda)
    p0 = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu()
    x, t = _batch()
    with tempfile.TemporaryDirectory() as d:
        _run(m, x, t, d)
    ref = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu()
    assert float((ref - p0).abs().max()) > 1e-5                      # the steps moved the weights
    assert float((ret['p0'] - ref).abs().max()) <= 1e-6 * float(ref.abs().max())
