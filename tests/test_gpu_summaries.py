"""Summary-grid evaluation (siren_amd/utils.py; SURVEY.md §8f row 1: the reference's utils.py:40-64 wave frames,
249-284 SDF slices, 300-325 video frames) on the fused W0 kernel: the grids follow the reference's coordinate
construction (checked on CPU against a restatement of it) and the dense values match the fp64 oracle on sampled
points (model_out tolerance 1e-4). Needs an MI355X."""
import numpy as np
import pytest
import torch

from oracle import siren_oracle as O

pytestmark = pytest.mark.gpu


class Recorder:
    def __init__(self):
        self.scalars, self.images, self.figures = {}, {}, {}

    def add_scalar(self, k, v, step):
        self.scalars[k] = float(v)

    def add_image(self, k, v, global_step=None):
        self.images[k] = v

    def add_figure(self, k, v, global_step=None):
        self.figures[k] = v


def layers_of(m):
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy().astype(np.float64)
    return O.layers_from_state({k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}, prefix=''), flat


def check_dense(m, coords, vals, k=4096):
    layers, _ = layers_of(m)
    idx = np.random.default_rng(0).choice(coords.shape[0], size=min(k, coords.shape[0]), replace=False)
    ref = O.forward(coords[idx].astype(np.float64), layers)
    assert np.max(np.abs(vals[idx] - ref)) <= 1e-4 * max(1., np.max(np.abs(ref)))


def test_sdf_slices_and_summary(cuda):
    from siren_amd import utils
    from siren_amd.modules import SingleBVPNet
    torch.manual_seed(0)
    m = SingleBVPNet(in_features=3, verbose=False).to(cuda)
    sl = utils.sdf_slices(m, 128)
    coords = utils.sdf_slice_coords(128)
    for k in ('yz', 'xz', 'xy'):
        assert sl[k].shape == (128, 128)
        # lin2img of a (1, N, 1) row-major grid: image[i, j] = value of grid point i * 128 + j
        check_dense(m, coords[k].numpy(), sl[k].reshape(-1).cpu().numpy().reshape(-1, 1))
    rec = Recorder()
    out = m({'coords': coords['xy'][None].to(cuda)})
    utils.write_sdf_summary(m, {'coords': coords['xy'][None]}, None, out, rec, 1)
    assert set(rec.figures) == {'train_yz_sdf_slice', 'train_xz_sdf_slice', 'train_xy_sdf_slice'}
    assert 'train_model_out_min_max_min' in rec.scalars


def test_video_frames_and_summary(cuda):
    from siren_amd import utils
    from siren_amd.modules import SingleBVPNet
    torch.manual_seed(1)
    m = SingleBVPNet(in_features=3, out_features=3, hidden_features=512, verbose=False).to(cuda)
    res = (201, 64, 48)
    pred = utils.video_frames(m, res)
    assert pred.shape == (4, 64, 48, 3) and float(pred.min()) >= 0 and float(pred.max()) <= 1
    c = utils.video_frame_coords(res).reshape(-1, 3).numpy()
    assert np.allclose(c[:64 * 48, 0], -1.) and np.allclose(c[-1, 0], (200 / 200 - 0.5) * 2)
    layers, _ = layers_of(m)
    idx = np.random.default_rng(1).choice(c.shape[0], size=2048, replace=False)
    ref = np.clip(O.forward(c[idx].astype(np.float64), layers) / 2 + 0.5, 0, 1)
    assert np.max(np.abs(pred.reshape(-1, 3).cpu().numpy()[idx] - ref)) <= 1e-4

    class Vid:
        shape = res
        vid = np.random.default_rng(2).uniform(0, 1, (201, 64, 48, 3)).astype(np.float32)
    rec = Recorder()
    x = c[None, :16]
    utils.write_video_summary(Vid, m, {'coords': torch.tensor(x)}, None, None, rec, 3)
    assert rec.images['train_output_vs_gt'].shape == (3, 128, 4 * 48) and np.isfinite(rec.scalars['train_psnr'])


def test_wave_frames(cuda):
    from siren_amd import utils
    from siren_amd.modules import SingleBVPNet
    torch.manual_seed(2)
    m = SingleBVPNet(in_features=3, verbose=False).to(cuda)
    w = utils.wave_frames(m, sl=64)
    assert w.shape == (5, 64, 64)
    c = utils.wave_frame_coords(sl=64).reshape(-1, 3).numpy()
    check_dense(m, c, w.reshape(-1, 1).cpu().numpy())
    rec = Recorder()
    utils.write_wave_summary(m, None, None, None, rec, 0)
    assert len([k for k in rec.images if k.startswith('train_pred_img_')]) == 5
