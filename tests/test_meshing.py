"""sdf_meshing: voxel-grid order, surface extraction and the .ply writer on CPU, and the
dense decoder evaluation on the fused W0 kernel on the GPU."""
import os

import numpy as np
import pytest
import torch

from siren_amd import sdf_meshing as M


def reference_grid(N):
    """The reference's sample construction (sdf_meshing.py:24-38) restated with integer (floor) division."""
    voxel_origin = [-1, -1, -1]
    voxel_size = 2.0 / (N - 1)
    idx = torch.arange(0, N ** 3, 1, dtype=torch.int64)
    s = torch.zeros(N ** 3, 4)
    s[:, 2] = idx % N
    s[:, 1] = (idx // N) % N
    s[:, 0] = ((idx // N) // N) % N
    s[:, 0] = (s[:, 0] * voxel_size) + voxel_origin[2]
    s[:, 1] = (s[:, 1] * voxel_size) + voxel_origin[1]
    s[:, 2] = (s[:, 2] * voxel_size) + voxel_origin[0]
    return s[:, :3]


def test_voxel_grid_matches_reference_order():
    N = 9
    ref = reference_grid(N)
    got = torch.cat([M.voxel_grid_chunk(N, a, min(a + 100, N ** 3), 'cpu') for a in range(0, N ** 3, 100)])
    assert torch.equal(got, ref)


def sphere_volume(N, r=0.5):
    g = torch.linspace(-1, 1, N)
    x, y, z = torch.meshgrid(g, g, g, indexing='ij')
    return torch.sqrt(x ** 2 + y ** 2 + z ** 2) - r


def edge_counts(faces):
    e = np.sort(np.concatenate([faces[:, [0, 1]], faces[:, [1, 2]], faces[:, [2, 0]]]), axis=1)
    _, counts = np.unique(e, axis=0, return_counts=True)
    return counts


@pytest.mark.parametrize('N', [16, 33])
def test_marching_tetrahedra_sphere_closed_oriented(N):
    vol = sphere_volume(N)
    h = 2.0 / (N - 1)
    verts, faces = M.marching_tetrahedra(vol, 0.0, (h, h, h))
    v = verts.double().numpy() - 1.0
    f = faces.numpy()
    assert f.shape[0] > 0
    # vertices on the sphere (linear interpolation of a smooth SDF: error O(h^2))
    rad = np.linalg.norm(v, axis=1)
    assert np.max(np.abs(rad - 0.5)) < 0.5 * h
    # closed 2-manifold: every edge shared by exactly two faces
    assert np.all(edge_counts(f) == 2)
    # consistently oriented outwards: positive enclosed volume close to 4/3 pi r^3
    a, b, c = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
    vol6 = np.einsum('ij,ij->i', a, np.cross(b, c)).sum()
    assert abs(vol6 / 6 - 4 / 3 * np.pi * 0.125) < 0.05 * (4 / 3 * np.pi * 0.125)


def test_marching_tetrahedra_empty_and_tiny():
    v, f = M.marching_tetrahedra(torch.ones(5, 5, 5))
    assert v.shape == (0, 3) and f.shape == (0, 3)
    v, f = M.marching_tetrahedra(torch.ones(1, 5, 5))
    assert f.shape == (0, 3)


def test_ply_roundtrip(tmp_path):
    verts = np.random.default_rng(0).normal(size=(10, 3)).astype(np.float32)
    faces = np.random.default_rng(1).integers(0, 10, size=(7, 3))
    p = os.path.join(tmp_path, 'm.ply')
    M.write_ply(p, verts, faces)
    v2, f2 = M.read_ply(p)
    assert np.array_equal(v2, verts) and np.array_equal(f2, faces)
    head = open(p, 'rb').read(200).split(b'end_header')[0].decode()
    assert 'element vertex 10' in head and 'element face 7' in head and 'property list uchar int vertex_indices' in head


def test_convert_sdf_samples_to_ply_offset_scale(tmp_path):
    N = 17
    vol = sphere_volume(N)
    p = os.path.join(tmp_path, 's.ply')
    pts, faces = M.convert_sdf_samples_to_ply(vol, [-1, -1, -1], 2.0 / (N - 1), p, offset=np.array([0.1, 0., 0.]),
                                              scale=2.0)
    v, f = M.read_ply(p)
    assert np.allclose(v, pts.astype(np.float32)) and np.array_equal(f, faces)
    rad = np.linalg.norm((v + np.array([0.1, 0, 0])) * 2.0, axis=1)
    assert np.max(np.abs(rad - 0.5)) < 0.1


@pytest.mark.gpu
def test_create_mesh_on_fused_kernel(cuda, tmp_path):
    """Dense evaluation of a SingleBVPNet (d_in 3) through the W0 kernel matches the oracle on sampled voxels and
    the mesh of a SIREN fitted... (untrained weights: any level set; the check is evaluation parity + a valid
    .ply)."""
    from oracle import siren_oracle as O
    from siren_amd.modules import SingleBVPNet
    torch.manual_seed(0)
    m = SingleBVPNet(in_features=3, verbose=False).to(cuda)

    class Decoder(torch.nn.Module):
        def __init__(self, model):
            super().__init__()
            self.model = model

        def forward(self, coords):
            return self.model({'coords': coords})['model_out']

    dec = Decoder(m)
    N = 48
    sdf = M.evaluate_sdf_grid(dec, N, max_batch=10000, device=cuda, out_device=cuda)
    pts = reference_grid(N)
    idx = torch.randperm(N ** 3)[:4096]
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu().numpy().astype(np.float64)
    layers = O.unflatten(flat, 3, 256, 3, 1)
    ry = O.forward(pts[idx].numpy().astype(np.float64), layers)
    assert np.max(np.abs(sdf.reshape(-1)[idx.to(cuda)].cpu().numpy() - ry[:, 0])) <= 1e-4
    # shift the level so it crosses the volume, then mesh
    level = float(sdf.median())
    dec2 = lambda c: dec(c) - level  # noqa: E731
    dec2.parameters = m.parameters
    pts_out, faces = M.create_mesh(dec2, os.path.join(tmp_path, 'mesh'), N=N, max_batch=1 << 16, log=None)
    v, f = M.read_ply(os.path.join(tmp_path, 'mesh.ply'))
    assert f.shape[0] > 0 and v.shape[0] > 0 and f.max() < v.shape[0]
