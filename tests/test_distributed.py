"""Data parallelism over coordinates with world_size 2 on the gloo backend (CPU).

The sharded path must reproduce the single-process full-batch gradient: each rank takes a coordinate shard,
computes its local mean-loss gradient, and ONE all-reduce of the flat bucket combines them weighted by the ranks'
coordinate counts (exact for unequal and empty shards); the clip then runs on the reduced gradient
(training.py:95-104 semantics). The models here are the non-sine FCBlock (plain torch layers run on CPU); the
fused-kernel DP path with FusedAdam is tests/test_gpu_distributed.py.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank, world, port):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))


def _worker(rank, world, port, ret):
    _env(rank, world, port)
    import torch.distributed as dist
    from siren_amd import distributed as sd
    from siren_amd.modules import SingleBVPNet
    sd.init('gloo')
    torch.manual_seed(rank + 5)        # deliberately different init per rank: broadcast must fix it
    m = SingleBVPNet(type='tanh', hidden_features=32, num_hidden_layers=2, verbose=False)
    sd.broadcast_parameters(m)
    g = torch.Generator().manual_seed(0)
    x = torch.rand(1, 1000, 2, generator=g) * 2 - 1
    t = torch.sin(3 * x[..., :1])
    a, b = sd.shard(1000, world, rank, align=100)
    out = m({'coords': x[:, a:b]})
    loss = ((out['model_out'] - t[:, a:b]) ** 2).mean()
    loss.backward()
    sd.allreduce_gradients(list(m.parameters()))
    torch.nn.utils.clip_grad_norm_(m.parameters(), max_norm=1e-3)
    ret[rank] = torch.cat([p.grad.reshape(-1) for p in m.parameters()]).clone()
    ret['p%d' % rank] = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).clone()
    dist.barrier()
    dist.destroy_process_group()


def test_dp_gloo_world2_matches_full_batch():
    world, port = 2, _free_port()
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, port, ret), nprocs=world, join=True)
    assert torch.equal(ret['p0'], ret['p1'])
    assert torch.allclose(ret[0], ret[1])
    from siren_amd.modules import SingleBVPNet
    torch.manual_seed(5)
    m = SingleBVPNet(type='tanh', hidden_features=32, num_hidden_layers=2, verbose=False)
    with torch.no_grad():
        off = 0
        for p in m.parameters():
            p.copy_(ret['p0'][off:off + p.numel()].view_as(p))
            off += p.numel()
    g = torch.Generator().manual_seed(0)
    x = torch.rand(1, 1000, 2, generator=g) * 2 - 1
    t = torch.sin(3 * x[..., :1])
    loss = ((m({'coords': x})['model_out'] - t) ** 2).mean()
    loss.backward()
    torch.nn.utils.clip_grad_norm_(m.parameters(), max_norm=1e-3)
    ref = torch.cat([p.grad.reshape(-1) for p in m.parameters()])
    assert torch.allclose(ret[0], ref, atol=1e-7, rtol=1e-5)


# ---- the product path: siren_amd.training.train under DP ----------------------------------------------------------
N_TRAIN, STEPS = 1000, 3


def _batch(n):
    g = torch.Generator().manual_seed(1)
    x = torch.rand(1, n, 2, generator=g) * 2 - 1
    return x, torch.sin(3 * x[..., :1]) * torch.cos(2 * x[..., 1:])


def _img_loss(out, gt):
    return {'img_loss': ((out['model_out'] - gt['img']) ** 2).mean()}


def _train(model, x, t, model_dir, device='cpu', fused_adam=False):
    from siren_amd.training import train
    loader = [({'coords': x}, {'img': t})]
    return train(model, loader, epochs=STEPS, lr=1e-3, steps_til_summary=1000, epochs_til_checkpoint=1000,
                 model_dir=model_dir, loss_fn=_img_loss, clip_grad=True, device=device, log=lambda *a: None,
                 fused_adam=fused_adam)


def _train_worker(rank, world, port, n, align, ret):
    _env(rank, world, port)
    from siren_amd import distributed as sd
    from siren_amd.modules import SingleBVPNet
    sd.init('gloo')
    torch.manual_seed(0)
    m = SingleBVPNet(type='tanh', hidden_features=32, num_hidden_layers=2, verbose=False)
    x, t = _batch(n)
    a, b = sd.shard(n, world, rank, align=align)
    ret['n%d' % rank] = b - a
    with tempfile.TemporaryDirectory() as d:
        _train(m, x[:, a:b], t[:, a:b], d)
    ret['p%d' % rank] = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).clone()
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize('n,align', [(1000, 64), (100, 64)])
def test_training_train_dp_world2_equals_full_batch(n, align):
    """training.train (Adam + clip) on 2 gloo ranks with UNEQUAL shards ((448, 552) coordinates) and with an EMPTY
    shard ((0, 100)): parameters after 3 steps equal single-process full-batch training."""
    world, port = 2, _free_port()
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_train_worker, args=(world, port, n, align, ret), nprocs=world, join=True)
    assert ret['n0'] != ret['n1']
    assert torch.equal(ret['p0'], ret['p1'])
    from siren_amd.modules import SingleBVPNet
    torch.manual_seed(0)
    m = SingleBVPNet(type='tanh', hidden_features=32, num_hidden_layers=2, verbose=False)
    x, t = _batch(n)
    with tempfile.TemporaryDirectory() as d:
        _train(m, x, t, d)
    ref = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    assert float((ret['p0'] - ref).abs().max()) <= 1e-6 * float(ref.abs().max())


def test_shard_covers_range():
    from siren_amd.distributed import shard
    for n in (1, 63, 64, 1000, 1 << 20, (1 << 20) + 5):
        for world in (1, 2, 3, 8):
            parts = [shard(n, world, r) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            for (a, b), (c, d) in zip(parts[:-1], parts[1:]):
                assert b == c and a <= b and a % 64 == 0
            sizes = [b - a for a, b in parts]
            if n >= 64 * world:
                assert max(sizes) - min(sizes) < 64 + n % 64 + 64


def _loss_worker(rank, world, port, ret):
    _env(rank, world, port)
    from siren_amd import distributed as sd
    sd.init('gloo')
    torch.manual_seed(0)
    p = torch.nn.Parameter(torch.randn(5))
    x, t = _batch(100)
    a, b = sd.shard(100, world, rank, align=64)  # (64, 36): unequal shares
    loss = ((x[0, a:b, 0] * p.sum() - t[0, a:b, 0]) ** 2).mean()
    loss.backward()
    g = sd.allreduce_gradients([p], world, b - a, loss=loss)
    ret['l%d' % rank] = float(g)
    ret['g%d' % rank] = p.grad.clone()
    torch.distributed.destroy_process_group()


def test_dp_closure_loss_is_global():
    """The LBFGS closure under DP (training.train, use_lbfgs) returns the count-weighted GLOBAL loss from the same
    all-reduce as the gradient, so every rank's strong-Wolfe line search sees the same function:
    with unequal shards both ranks get the full-batch loss and gradient."""
    world, port = 2, _free_port()
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_loss_worker, args=(world, port, ret), nprocs=world, join=True)
    torch.manual_seed(0)
    p = torch.nn.Parameter(torch.randn(5))
    x, t = _batch(100)
    loss = ((x[0, :, 0] * p.sum() - t[0, :, 0]) ** 2).mean()
    loss.backward()
    lf = float(loss.detach())
    assert ret['l0'] == ret['l1'] and abs(ret['l0'] - lf) <= 1e-6 * lf
    assert torch.equal(ret['g0'], ret['g1']) and torch.allclose(ret['g0'], p.grad, rtol=1e-5, atol=0)
