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


def closed_oriented(v, f, r=0.5, h=None):
    """Every undirected edge in exactly two faces, the two uses opposite (consistent winding), enclosed volume
    positive and close to the sphere's."""
    assert f.shape[0] > 0
    assert np.all(edge_counts(f) == 2)
    d = np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]])
    assert np.unique(d, axis=0).shape[0] == d.shape[0]  # no directed edge twice
    a, b, c = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
    vol6 = np.einsum('ij,ij->i', a, np.cross(b, c)).sum()
    assert abs(vol6 / 6 - 4 / 3 * np.pi * r ** 3) < 0.05 * (4 / 3 * np.pi * r ** 3)


@pytest.mark.parametrize('N', [16, 25])
def test_oracle_marching_cubes_sphere(N):
    """The CPU restatement of the device marching cubes (oracle/mc_oracle.py): a sphere SDF gives a closed,
    outward-oriented mesh whose vertices lie on the sphere to O(h^2)."""
    from oracle import mc_oracle as MC
    h = 2.0 / (N - 1)
    v, f = MC.marching_cubes(sphere_volume(N).numpy(), 0.0, (h, h, h))
    v = v - 1.0
    assert np.max(np.abs(np.linalg.norm(v, axis=1) - 0.5)) < 0.5 * h
    closed_oriented(v, f)


def test_oracle_marching_cubes_noise_is_manifold():
    """Random volumes (every ambiguous face and cube case): still a closed consistently wound 2-manifold inside
    the volume — ambiguous faces are resolved identically by both cells, and no triangle chord lies on a face."""
    from oracle import mc_oracle as MC
    rng = np.random.default_rng(0)
    for _ in range(6):
        vol = rng.normal(size=(7, 6, 8))
        vol[[0, -1]] = 1.
        vol[:, [0, -1]] = 1.
        vol[:, :, [0, -1]] = 1.
        v, f = MC.marching_cubes(vol)
        assert np.all(edge_counts(f) == 2)
        d = np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]])
        assert np.unique(d, axis=0).shape[0] == d.shape[0]


def test_mc_table_header_matches_derivation():
    """siren_amd/csrc/mc_table.h (tools/gen_mc_table.py) == the oracle's independent derivation, case by case."""
    import re
    from oracle import mc_oracle as MC
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'siren_amd', 'csrc',
                            'mc_table.h')).read()
    counts = [int(t) for t in re.findall(r'-?\d+', src.split('kMcCount[256] = {')[1].split('};')[0])]
    rows = re.findall(r'\{([-0-9, ]+)\},', src.split('kMcTri[256]')[1])
    table = MC.case_table()
    assert len(counts) == 256 and len(rows) == 256
    for m in range(256):
        got = [int(t) for t in rows[m].split(',') if int(t) >= 0]
        assert got == [e for tri in table[m] for e in tri] and counts[m] == len(table[m]), m
    assert max(counts) == 5 and counts[0] == 0 and counts[255] == 0


def test_ply_roundtrip(tmp_path):
    verts = np.random.default_rng(0).normal(size=(10, 3)).astype(np.float32)
    faces = np.random.default_rng(1).integers(0, 10, size=(7, 3))
    p = os.path.join(tmp_path, 'm.ply')
    M.write_ply(p, verts, faces)
    v2, f2 = M.read_ply(p)
    assert np.array_equal(v2, verts) and np.array_equal(f2, faces)
    head = open(p, 'rb').read(200).split(b'end_header')[0].decode()
    assert 'element vertex 10' in head and 'element face 7' in head and 'property list uchar int vertex_indices' in head


@pytest.mark.gpu
def test_convert_sdf_samples_to_ply_offset_scale(cuda, tmp_path):
    """The reference passes a host tensor (sdf_values.cpu(), sdf_meshing.py:64-71): it is meshed on the device."""
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
    pts_out, faces = M.create_mesh(dec2, os.path.join(tmp_path, 'mesh'), N=N, max_batch=1 << 16)
    v, f = M.read_ply(os.path.join(tmp_path, 'mesh.ply'))
    assert f.shape[0] > 0 and v.shape[0] > 0 and f.max() < v.shape[0]


@pytest.mark.gpu
@pytest.mark.parametrize('shape,seed', [((7, 6, 8), 0), ((2, 2, 2), 1), ((3, 9, 4), 2), ((11, 11, 11), 3)])
def test_device_marching_cubes_matches_oracle(cuda, shape, seed):
    """siren_mc_count / siren_mc_emit (marching.hip) == oracle/mc_oracle.py: the same vertex numbering (grid point,
    axis), the same faces bit for bit, vertex positions to fp32 rounding — on noise volumes (every cube case)."""
    from oracle import mc_oracle as MC
    vol = np.random.default_rng(seed).normal(size=shape).astype(np.float32)
    sp = (0.5, 1.0, 2.0)
    v, f = M.marching_cubes(torch.tensor(vol, device=cuda), 0.1, sp)
    rv, rf = MC.marching_cubes(vol.astype(np.float64), 0.1, sp)
    assert f.shape == rf.shape and v.shape == rv.shape
    assert np.array_equal(f.cpu().numpy(), rf)
    assert np.max(np.abs(v.cpu().numpy() - rv), initial=0.) <= 1e-5


@pytest.mark.gpu
def test_device_marching_cubes_empty_and_tiny(cuda):
    for shape in [(5, 5, 5), (1, 5, 5), (5, 0, 5)]:
        v, f = M.marching_cubes(torch.ones(shape, device=cuda))
        assert v.shape == (0, 3) and f.shape == (0, 3)


@pytest.mark.gpu
@pytest.mark.parametrize('N', [33, 256])
def test_device_marching_cubes_sphere(cuda, N):
    """A sphere SDF at the reference's default resolution (create_mesh N = 256): closed, outward, on the sphere."""
    h = 2.0 / (N - 1)
    v, f = M.marching_cubes(sphere_volume(N).to(cuda), 0.0, (h, h, h))
    v = v.double().cpu().numpy() - 1.0
    f = f.long().cpu().numpy()
    assert np.max(np.abs(np.linalg.norm(v, axis=1) - 0.5)) < 0.5 * h
    closed_oriented(v, f)
    # Euler characteristic of a sphere
    e = np.unique(np.sort(np.concatenate([f[:, [0, 1]], f[:, [1, 2]], f[:, [2, 0]]]), axis=1), axis=0).shape[0]
    assert v.shape[0] - e + f.shape[0] == 2
