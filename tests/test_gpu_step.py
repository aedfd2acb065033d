"""The per-step kernels: the device PointCloud sampler against the oracle's restatement of
its counter RNG (bit-exact), and FusedAdam (clip + Adam, siren_adam_step) against torch.optim.Adam +
clip_grad_norm_ and the oracle. Needs an MI355X."""
import numpy as np
import pytest
import torch

from oracle import siren_oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('m,k,seed,step', [(1000, 4096, 0, 0), (3, 7, 123, 5), (50000, 1000, 2 ** 63 + 11, 99)])
def test_sample_sdf_bit_exact(cuda, m, k, seed, step):
    from siren_amd.dataio import PointCloud
    rng = np.random.default_rng(m)
    pts = np.concatenate([rng.uniform(-3, 5, (m, 3)), rng.normal(size=(m, 3))], 1)
    pcd = PointCloud(points=pts, on_surface_points=k, device=cuda, seed=seed)
    inp, gt = pcd.sample(step)
    pc, pn = pcd.coords.cpu().numpy(), pcd.normals.cpu().numpy()
    c, nrm, sdf, _ = O.sample_sdf(pc, pn, k, seed, step)
    assert np.array_equal(inp['coords'].cpu().numpy(), c)
    assert np.array_equal(gt['normals'].cpu().numpy(), nrm)
    assert np.array_equal(gt['sdf'].cpu().numpy(), sdf)


def test_point_cloud_dataset_steps(cuda):
    from siren_amd.dataio import PointCloud
    rng = np.random.default_rng(3)
    pts = np.concatenate([rng.normal(size=(5000, 3)), rng.normal(size=(5000, 3))], 1)
    pcd = PointCloud(points=pts, on_surface_points=1000, device=cuda)
    assert len(pcd) == 5
    a, b = pcd[0], pcd[0]
    assert not torch.equal(a[0]['coords'], b[0]['coords'])  # a fresh draw per call, as np.random
    assert a[0]['coords'].shape == (2000, 3) and a[1]['sdf'].shape == (2000, 1)


@pytest.mark.parametrize('n,max_norm', [(198401, None), (198401, 1.), (13, 0.5), (4, None)])
def test_fused_adam_vs_torch(cuda, n, max_norm):
    from siren_amd.optim import FusedAdam
    rng = np.random.default_rng(n)
    p0 = rng.normal(size=n).astype(np.float32) * 0.05
    grads = [(rng.normal(size=n) * s).astype(np.float32) for s in (1., 10., 0.1, 3., 1.)]
    a = torch.nn.Parameter(torch.tensor(p0, device=cuda))
    b = torch.nn.Parameter(torch.tensor(p0, device=cuda))
    fa = FusedAdam([a], lr=1e-4, max_norm=max_norm)
    tb = torch.optim.Adam([b], lr=1e-4)
    for g in grads:
        fa.zero_grad()
        a.grad.copy_(torch.tensor(g, device=cuda))
        fa.step()
        b.grad = torch.tensor(g, device=cuda)
        if max_norm:
            torch.nn.utils.clip_grad_norm_([b], max_norm)
        tb.step()
    pa, pb = a.detach().cpu().numpy(), b.detach().cpu().numpy()
    ref = O.adam_steps(p0, grads, lr=1e-4, max_norm=max_norm)
    assert np.max(np.abs(pa - pb)) <= 2e-7
    assert np.max(np.abs(pa - ref)) <= 2e-7
    if max_norm:
        assert abs(float(fa.grad_norm()) - np.sqrt(np.sum(grads[-1].astype(np.float64) ** 2))) <= \
            1e-5 * np.sqrt(np.sum(grads[-1].astype(np.float64) ** 2))


def test_fused_adam_trains_like_torch_adam(cuda):
    """image_mse training through the drop-in modules: FusedAdam (autograd accumulating into the flat bucket)
    tracks torch.optim.Adam step for step."""
    from siren_amd.modules import SingleBVPNet
    from siren_amd import loss_functions as LF
    from siren_amd.dataio import get_mgrid, synthetic_image
    from siren_amd.optim import FusedAdam
    x = get_mgrid(64).to(cuda)[None]
    gt = {'img': synthetic_image(x)}
    models = []
    for _ in range(2):
        torch.manual_seed(0)
        models.append(SingleBVPNet(verbose=False).to(cuda))
    fa = FusedAdam(models[0].parameters(), lr=1e-4)
    tb = torch.optim.Adam(models[1].parameters(), lr=1e-4)
    for _ in range(10):
        for m, opt in ((models[0], fa), (models[1], tb)):
            opt.zero_grad()
            loss = LF.image_mse(None, m({'coords': x}), gt)['img_loss']
            loss.backward()
            opt.step()
    for (k, pa), (_, pb) in zip(models[0].named_parameters(), models[1].named_parameters()):
        assert torch.max(torch.abs(pa - pb)).item() <= 1e-6, k


@pytest.mark.parametrize('clip', [False, True])
def test_train_loop_fused_adam_matches_torch_adam(cuda, tmp_path, clip):
    """siren_amd.training.train (training.py:14-129 semantics) with fused_adam=True and the device PointCloud
    sampler against the same loop on torch.optim.Adam: identical loss trajectories and weights to fp32 rounding."""
    from siren_amd.modules import SingleBVPNet
    from siren_amd import loss_functions as LF, training
    from siren_amd.dataio import PointCloud
    rng = np.random.default_rng(4)
    d = rng.normal(size=(4000, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    pcd = PointCloud(points=np.concatenate([d * 0.5, d], 1), on_surface_points=2048, device=cuda, seed=9)
    batches = [pcd.sample(s) for s in range(4)]
    res = []
    for fused in (True, False):
        torch.manual_seed(0)
        m = SingleBVPNet(in_features=3, verbose=False).to(cuda)
        losses = training.train(m, batches, epochs=2, lr=1e-4, steps_til_summary=100, epochs_til_checkpoint=100,
                                model_dir=str(tmp_path / ('f%d' % fused)), loss_fn=LF.sdf, clip_grad=clip,
                                log=lambda *a: None, fused_adam=fused)
        res.append((losses, torch.cat([p.detach().reshape(-1) for p in m.parameters()])))
    (la, pa), (lb, pb) = res
    assert len(la) == len(lb) == 8
    assert np.allclose(la, lb, rtol=1e-4, atol=0)
    assert torch.max(torch.abs(pa - pb)).item() <= 1e-6
