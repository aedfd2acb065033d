"""Dense SDF evaluation and surface extraction (sdf_meshing.py:13-138).

create_mesh(decoder, filename, N, max_batch, offset, scale) keeps the reference's signature and output: the
decoder is evaluated on the N^3 voxel grid of [-1, 1]^3 (voxel_origin (-1, -1, -1), voxel_size 2/(N-1), the
index order of sdf_meshing.py:24-38: axis 0 slowest), the zero level set is extracted and written as a binary
.ply with float x/y/z vertices and int vertex_indices faces (sdf_meshing.py:120-138).

What differs, and why:
  * the grid is generated on the device chunk by chunk (the reference materialises an (N^3, 4) fp32 host tensor,
    65 GB at N = 1600, and copies every chunk to the GPU and back); the decoder runs under no_grad on the fused
    W0 kernel when it is one of siren_amd's SIREN modules, with chunks as large as `max_batch` (HBM is 288 GB, so
    the default here is 2^22 coordinates per launch instead of 64^3);
  * surface extraction: the reference calls skimage.measure.marching_cubes_lewiner inside a bare try/except
    (sdf_meshing.py:97-102). skimage is not installed in this image; when it is importable its marching_cubes is
    used, otherwise the device marching cubes (`marching_cubes` below: HIP kernels in marching.hip, cube-case
    table from tools/gen_mc_table.py) meshes the volume where the W0 kernel left it. Both interpolate the zero
    crossing linearly along grid edges (the same vertex set); Lewiner's variant resolves the interior ambiguity of
    a few cube cases differently, so triangle lists can differ there — mesh parity vs the reference is unpinned
    (no skimage here); tests pin the kernels to oracle/mc_oracle.py and check closedness / orientation.
  * plyfile is not installed either: write_ply writes the same binary_little_endian layout plyfile produces for
    the reference's element descriptions.
"""
import os
import time

import numpy as np
import torch


def voxel_grid_chunk(N, start, stop, device, voxel_origin=(-1., -1., -1.), voxel_size=None):
    """Coordinates of flat voxel indices [start, stop) in the reference's order (sdf_meshing.py:24-38):
    column 0 = idx // N^2 (slowest), column 2 = idx % N, each scaled by voxel_size and offset by the origin."""
    if voxel_size is None:
        voxel_size = 2.0 / (N - 1)
    idx = torch.arange(start, stop, device=device, dtype=torch.int64)
    out = torch.empty(stop - start, 3, device=device, dtype=torch.float32)
    out[:, 2] = (idx % N).float()
    out[:, 1] = ((idx // N) % N).float()
    out[:, 0] = ((idx // N // N) % N).float()
    # the reference scales column 0 with voxel_origin[2] and column 2 with voxel_origin[0] (all -1)
    out[:, 0] = out[:, 0] * voxel_size + voxel_origin[2]
    out[:, 1] = out[:, 1] * voxel_size + voxel_origin[1]
    out[:, 2] = out[:, 2] * voxel_size + voxel_origin[0]
    return out


def evaluate_sdf_grid(decoder, N=256, max_batch=1 << 22, device=None, out_device='cpu'):
    """The decoder on the N^3 voxel grid, reshaped (N, N, N) (axis 0 = the slowest voxel index)."""
    if device is None:
        device = next(iter(decoder.parameters())).device if hasattr(decoder, 'parameters') else torch.device('cuda')
    total = N ** 3
    sdf = torch.empty(total, dtype=torch.float32, device=out_device)
    if hasattr(decoder, 'eval'):
        decoder.eval()
    with torch.no_grad():
        head = 0
        while head < total:
            stop = min(head + max_batch, total)
            pts = voxel_grid_chunk(N, head, stop, device)
            val = decoder(pts)
            if isinstance(val, dict):
                val = val['model_out']
            sdf[head:stop] = val.reshape(-1).to(out_device, non_blocking=False)
            head = stop
    return sdf.view(N, N, N)


# --------------------------------------------------------------------------------------------------------
# device marching cubes (stand-in for skimage.measure.marching_cubes_lewiner, which this image lacks)
# --------------------------------------------------------------------------------------------------------
def marching_cubes(volume, level=0.0, spacing=(1., 1., 1.)):
    """Zero level set of an (X, Y, Z) volume on the device (siren_mc_count / siren_mc_emit, marching.hip) ->
    (verts (V, 3) float32 in index units * spacing, faces (F, 3) int32), both on the volume's device. Cube-case
    marching cubes: vertices welded per grid edge, crack-free on ambiguous faces, normals towards increasing value."""
    import ctypes
    from . import _lib
    if not isinstance(volume, torch.Tensor) or volume.dim() != 3:
        raise ValueError('volume must be an (X, Y, Z) tensor')
    if volume.device.type != 'cuda':
        raise RuntimeError('siren_amd marching cubes runs on ROCm devices (MI355X) only; got a %s tensor'
                           % volume.device.type)
    vol = volume.detach().float().contiguous()
    dev = vol.device
    lib = _lib.load()
    X, Y, Z = vol.shape
    nb = ctypes.c_int64()
    _lib.check(lib.siren_mc_ws_bytes(X, Y, Z, ctypes.byref(nb)), 'siren_mc_ws_bytes')
    ws = torch.empty(max(1, nb.value // 4), dtype=torch.int32, device=dev)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    nv, nf = ctypes.c_int64(), ctypes.c_int64()
    _lib.check(lib.siren_mc_count(ctypes.c_void_p(vol.data_ptr()), X, Y, Z, ctypes.c_float(level),
                                  ctypes.c_void_p(ws.data_ptr()), ctypes.byref(nv), ctypes.byref(nf), stream),
               'siren_mc_count')
    verts = torch.empty(nv.value, 3, dtype=torch.float32, device=dev)
    faces = torch.empty(nf.value, 3, dtype=torch.int32, device=dev)
    if nv.value == 0 and nf.value == 0:
        return verts, faces
    sp = (ctypes.c_float * 3)(*[float(t) for t in spacing])
    _lib.check(lib.siren_mc_emit(ctypes.c_void_p(vol.data_ptr()), X, Y, Z, ctypes.c_float(level),
                                 ctypes.cast(sp, ctypes.c_void_p),
                                 ctypes.c_void_p(ws.data_ptr()), ctypes.c_void_p(verts.data_ptr()),
                                 ctypes.c_void_p(faces.data_ptr()), stream), 'siren_mc_emit')
    return verts, faces


def extract_surface(sdf_volume, voxel_size, level=0.0):
    """(verts, faces) in voxel units * voxel_size: skimage's marching_cubes when importable, else the device
    marching cubes (a host volume — the reference passes sdf_values.cpu() — is moved to the current device)."""
    try:
        import skimage.measure  # noqa: F401
        v = sdf_volume.detach().cpu().numpy()
        verts, faces, _, _ = skimage.measure.marching_cubes(v, level=level, spacing=[voxel_size] * 3)
        return np.asarray(verts, np.float64), np.asarray(faces, np.int64)
    except ImportError:
        vol = torch.as_tensor(sdf_volume)
        if vol.device.type != 'cuda':
            if not torch.cuda.is_available():
                raise RuntimeError('siren_amd marching cubes needs a ROCm device (MI355X); there is no CPU path')
            vol = vol.cuda()
        verts, faces = marching_cubes(vol, level, (voxel_size,) * 3)
        return verts.double().cpu().numpy(), faces.long().cpu().numpy()


def write_ply(path, verts, faces):
    """Binary PLY exactly as plyfile writes the reference's elements (sdf_meshing.py:120-138): vertex x, y, z
    float32; face 'vertex_indices' as list uchar int."""
    verts = np.ascontiguousarray(verts, dtype='<f4').reshape(-1, 3)
    faces = np.ascontiguousarray(faces, dtype='<i4').reshape(-1, 3)
    header = ('ply\nformat binary_little_endian 1.0\nelement vertex %d\nproperty float x\nproperty float y\n'
              'property float z\nelement face %d\nproperty list uchar int vertex_indices\nend_header\n'
              % (verts.shape[0], faces.shape[0]))
    rec = np.empty(faces.shape[0], dtype=[('n', 'u1'), ('idx', '<i4', (3,))])
    rec['n'] = 3
    rec['idx'] = faces
    with open(path, 'wb') as fh:
        fh.write(header.encode('ascii'))
        fh.write(verts.tobytes())
        fh.write(rec.tobytes())


def read_ply(path):
    """Inverse of write_ply (tests / inspection)."""
    with open(path, 'rb') as fh:
        data = fh.read()
    end = data.index(b'end_header\n') + len(b'end_header\n')
    head = data[:end].decode('ascii').split('\n')
    nv = int([h for h in head if h.startswith('element vertex')][0].split()[-1])
    nf = int([h for h in head if h.startswith('element face')][0].split()[-1])
    verts = np.frombuffer(data, dtype='<f4', count=3 * nv, offset=end).reshape(nv, 3)
    rec = np.frombuffer(data, dtype=[('n', 'u1'), ('idx', '<i4', (3,))], count=nf, offset=end + 12 * nv)
    return verts.copy(), rec['idx'].copy()


def convert_sdf_samples_to_ply(pytorch_3d_sdf_tensor, voxel_grid_origin, voxel_size, ply_filename_out,
                               offset=None, scale=None):
    """sdf_meshing.py:74-138: level-0 surface of an (n, n, n) volume, shifted to the voxel origin, then
    /scale and -offset, written as .ply."""
    verts, faces = extract_surface(pytorch_3d_sdf_tensor, voxel_size)
    mesh_points = np.zeros_like(verts)
    mesh_points[:, 0] = voxel_grid_origin[0] + verts[:, 0]
    mesh_points[:, 1] = voxel_grid_origin[1] + verts[:, 1]
    mesh_points[:, 2] = voxel_grid_origin[2] + verts[:, 2]
    if scale is not None:
        mesh_points = mesh_points / scale
    if offset is not None:
        mesh_points = mesh_points - offset
    write_ply(ply_filename_out, mesh_points, faces)
    return mesh_points, faces


def create_mesh(decoder, filename, N=256, max_batch=64 ** 3, offset=None, scale=None):
    """sdf_meshing.py:13-71 on the device: decoder.eval(), dense decoder evaluation in max_batch chunks (the reference's
    defaults; a larger max_batch means fewer, larger W0 launches) + level-0 surface -> filename + '.ply'."""
    start = time.time()
    if hasattr(decoder, 'eval'):
        decoder.eval()
    voxel_origin = [-1, -1, -1]
    voxel_size = 2.0 / (N - 1)
    dev = next(iter(decoder.parameters())).device if hasattr(decoder, 'parameters') else torch.device('cuda')
    sdf = evaluate_sdf_grid(decoder, N, max_batch, device=dev, out_device=dev)
    print('sampling takes: %f' % (time.time() - start))
    return convert_sdf_samples_to_ply(sdf, voxel_origin, voxel_size, os.fspath(filename) + '.ply', offset, scale)
