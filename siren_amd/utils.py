"""Summary-grid evaluation (utils.py:40-63 wave frames, 249-284 SDF slices, 300-325 video
frames) on the device.

The reference's summary functions evaluate the model densely on fixed grids — three 512² SDF slices, four video
frames in 10 slices, five wave frames — and then plot them for TensorBoard. Here the grids are built with the
reference's own coordinate construction (dataio.get_mgrid, the same slice planes and frame times) and evaluated
under no_grad by the fused W0 kernel in one launch per grid (the reference splits the frames into Nslice chunks to
bound CUDA memory; 288 GB of HBM makes that unnecessary). `*_frames` / `sdf_slices` return the tensors; the
`write_*` functions keep the reference's signatures and log them through `writer` (contour figures need
matplotlib; image grids are concatenated with torch instead of torchvision.make_grid, which is absent here).
"""
import numpy as np
import torch

from . import dataio


def lin2img(tensor, image_resolution=None):
    """(B, N, C) -> (B, C, H, W) (dataio.py:43-52)."""
    return dataio.lin2img(tensor, image_resolution)


def min_max_summary(name, tensor, writer, total_steps):
    """utils.py:565-567."""
    writer.add_scalar(name + '_min', tensor.min().detach().cpu().numpy(), total_steps)
    writer.add_scalar(name + '_max', tensor.max().detach().cpu().numpy(), total_steps)


def _device_of(model):
    try:
        return next(iter(model.parameters())).device
    except (StopIteration, AttributeError, TypeError):
        return torch.device('cuda')


def _eval(model, coords):
    with torch.no_grad():
        return model({'coords': coords})['model_out']


def sdf_slice_coords(resolution=512):
    """The three planes of write_sdf_summary (utils.py:249-276): yz at x = 0, xz at y = 0, xy at z = -0.75."""
    s2 = dataio.get_mgrid(resolution)
    zero = torch.zeros_like(s2[:, :1])
    return {'yz': torch.cat((zero, s2), dim=-1),
            'xz': torch.cat((s2[:, :1], zero, s2[:, -1:]), dim=-1),
            'xy': torch.cat((s2[:, :2], -0.75 * torch.ones_like(s2[:, :1])), dim=-1)}


def sdf_slices(model, resolution=512):
    """{'yz', 'xz', 'xy'}: (resolution, resolution) SDF images of the three summary planes (lin2img order)."""
    dev = _device_of(model)
    out = {}
    for k, c in sdf_slice_coords(resolution).items():
        y = _eval(model, c.to(dev)[None])
        out[k] = lin2img(y).squeeze()
    return out


def make_contour_plot(array_2d, mode='log'):
    """Filled-contour figure of a 2-D SDF slice for write_sdf_summary (the reference's helper, utils.py:225-246, drawn
    with the same figure): symmetric levels — 'log': +-10^-2 .. 10^0 in six magnitudes per sign, 13 palette entries;
    otherwise ten linear levels on [-0.5, 0.5] — from the 'Spectral' map, thin black isolines plus a heavier zero
    level set, rows flipped so that the slice's first row is drawn at the bottom."""
    import matplotlib
    matplotlib.use('agg')
    import matplotlib.pyplot as plt
    field = np.asarray(array_2d)[::-1]
    if mode == 'log':
        mags = np.logspace(-2, 0, 6)
        levels, n_colors = np.concatenate([-mags[::-1], mags]), 13
    else:
        levels, n_colors = np.linspace(-.5, .5, 10), 10
    palette = plt.get_cmap('Spectral')(np.linspace(0., 1., n_colors))
    fig = plt.figure(figsize=(2.75, 2.75), dpi=300)
    ax = fig.add_subplot()
    fig.colorbar(ax.contourf(field, levels=levels, colors=palette))
    for lv, lw in ((levels, 0.1), ([0.], 0.3)):
        ax.contour(field, levels=lv, colors='k', linewidths=lw)
    ax.set_axis_off()
    return fig


def write_sdf_summary(model, model_input, gt, model_output, writer, total_steps, prefix='train_'):
    """utils.py:249-284: contour plots of the three SDF slices + min / max summaries."""
    for k, img in sdf_slices(model).items():
        writer.add_figure(prefix + '%s_sdf_slice' % k, make_contour_plot(img.cpu().numpy()), global_step=total_steps)
    min_max_summary(prefix + 'model_out_min_max', model_output['model_out'], writer, total_steps)
    min_max_summary(prefix + 'coords', model_input['coords'], writer, total_steps)


def video_frame_coords(resolution, frames=(0, 60, 120, 200)):
    """write_video_summary's frames (utils.py:300-307): (len(frames), H*W, 3), t = (f / (T - 1) - 0.5) * 2."""
    coords = dataio.get_mgrid((1, resolution[1], resolution[2]), dim=3)[None].repeat(len(frames), 1, 1)
    for i, f in enumerate(frames):
        coords[i, :, 0] = (f / (resolution[0] - 1) - 0.5) * 2
    return coords


def video_frames(model, resolution, frames=(0, 60, 120, 200)):
    """(len(frames), H, W, 3) predicted frames in [0, 1] (pred / 2 + 0.5, clamped; utils.py:309-313)."""
    dev = _device_of(model)
    c = video_frame_coords(resolution, frames).to(dev)
    y = _eval(model, c.reshape(1, -1, 3)).reshape(len(frames), resolution[1], resolution[2], -1)
    return torch.clamp(y / 2 + 0.5, 0, 1)


def write_video_summary(vid_dataset, model, model_input, gt, model_output, writer, total_steps, prefix='train_'):
    """utils.py:300-325: predicted vs ground-truth frames, PSNR over the four frames."""
    frames = [0, 60, 120, 200]
    pred = video_frames(model, vid_dataset.shape, frames)
    gt_vid = torch.as_tensor(np.asarray(vid_dataset.vid)[frames], dtype=torch.float32, device=pred.device)
    psnr = 10 * torch.log10(1 / torch.mean((gt_vid - pred) ** 2))
    grid = torch.cat((gt_vid, pred), dim=1).permute(0, 3, 1, 2)  # gt above prediction, frames side by side
    grid = torch.cat(list(grid), dim=-1)
    writer.add_image(prefix + 'output_vs_gt', grid, global_step=total_steps)
    min_max_summary(prefix + 'coords', model_input['coords'], writer, total_steps)
    min_max_summary(prefix + 'pred_vid', pred, writer, total_steps)
    writer.add_scalar(prefix + 'psnr', float(psnr), total_steps)


def wave_frame_coords(frames=(0.0, 0.05, 0.1, 0.15, 0.25), sl=256):
    """write_wave_summary's grids (utils.py:50-55): (len(frames), sl*sl, 3) with coords[..., 0] = t."""
    coords = dataio.get_mgrid((1, sl, sl), dim=3)[None].repeat(len(frames), 1, 1)
    for i, f in enumerate(frames):
        coords[i, :, 0] = f
    return coords


def wave_frames(model, frames=(0.0, 0.05, 0.1, 0.15, 0.25), sl=256):
    """(len(frames), sl, sl) wave field at the summary times (utils.py:57-64)."""
    dev = _device_of(model)
    c = wave_frame_coords(frames, sl).to(dev)
    return _eval(model, c.reshape(1, -1, 3))[..., 0].reshape(len(frames), sl, sl)


def write_wave_summary(model, model_input, gt, model_output, writer, total_steps, prefix='train_'):
    """utils.py:40-110 (the evaluation and its images; the matplotlib line plots of the reference are omitted)."""
    pred = wave_frames(model)
    min_max_summary(prefix + 'pred', pred, writer, total_steps)
    for i in range(pred.shape[0]):
        img = pred[i]
        lo, hi = torch.quantile(img.flatten(), 0.01), torch.quantile(img.flatten(), 0.99)
        writer.add_image(prefix + 'pred_img_%d' % i, ((img.clamp(lo, hi) - lo) / (hi - lo + 1e-12))[None],
                         global_step=total_steps)
