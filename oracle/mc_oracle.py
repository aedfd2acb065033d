"""CPU restatement of the device marching cubes (siren_amd/csrc/marching.hip) — TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module, as the checker of the HIP kernels. The product path never imports it.

The reference extracts the SDF zero level set with skimage.measure.marching_cubes_lewiner (sdf_meshing.py:97-102).
skimage is not installed in this image, so the reference's own output cannot be produced here: parity of the
mesh against the reference is UNPINNED. What this module pins is the engine's algorithm itself — classic cube-case
marching cubes with the case table derived, not typed in:

  * corners c = x | y << 1 | z << 2 over the volume axes (0, 1, 2); inside = value < level;
  * cube edge e = 4 a + k runs along axis a from its lower corner (bit (a+1)%3 = k & 1, bit (a+2)%3 = k >> 1);
  * on each of the 6 faces, walked counter-clockwise seen from outside the cube, every maximal run of inside
    corners yields one directed segment from the crossing where the walk leaves the run to the crossing where it
    entered it (face ambiguity resolved by separating inside corners — the same rule in both cells that share the
    face, so the surface is crack-free);
  * every crossing then has one outgoing and one incoming segment: the segments close into loops, each loop is
    fanned into triangles (v0, v_i, v_i+1), and the winding is chosen once so that normals point towards
    increasing value (outside of an SDF);
  * vertices are welded per grid edge: a crossing on the edge from grid point p along axis a sits at
    p + t e_a, t = (level - v(p)) / (v(p + e_a) - v(p)), numbered in (point index, axis) order.

The result is a closed oriented 2-manifold away from the volume boundary for any input (tests check it).
"""
import numpy as np


def corner_bits(c):
    return (c & 1, (c >> 1) & 1, (c >> 2) & 1)


def edge_corners(e):
    """(lower corner, upper corner, axis) of cube edge e."""
    a, k = e // 4, e % 4
    lo = [0, 0, 0]
    lo[(a + 1) % 3] = k & 1
    lo[(a + 2) % 3] = k >> 1
    c0 = lo[0] | lo[1] << 1 | lo[2] << 2
    return c0, c0 | 1 << a, a


def edge_between(c0, c1):
    d = c0 ^ c1
    a = d.bit_length() - 1
    lo = min(c0, c1)
    b = corner_bits(lo)
    return 4 * a + (b[(a + 1) % 3] | b[(a + 2) % 3] << 1)


def face_rings():
    """The 6 cube faces as corner rings, counter-clockwise seen from outside."""
    rings = []
    for a in range(3):
        b, c = (a + 1) % 3, (a + 2) % 3
        for s in (0, 1):
            ring = []
            for (u, v) in ((0, 0), (1, 0), (1, 1), (0, 1)):
                p = [0, 0, 0]
                p[a], p[b], p[c] = s, u, v
                ring.append(p[0] | p[1] << 1 | p[2] << 2)
            rings.append(ring if s == 1 else ring[::-1])
    return rings


def case_triangles(mask):
    """Triangles (as cube-edge triples) of inside mask `mask`, wound so normals point to increasing value."""
    inside = [(mask >> c) & 1 for c in range(8)]
    nxt = {}
    for ring in face_rings():
        for i in range(4):
            if inside[ring[i]] and not inside[ring[i - 1]]:  # a run of inside corners starts at i
                enter = edge_between(ring[i - 1], ring[i])
                j = i
                while inside[ring[(j + 1) % 4]]:
                    j += 1
                leave = edge_between(ring[j % 4], ring[(j + 1) % 4])
                nxt[leave] = enter
    tris, seen = [], set()
    for start in sorted(nxt):
        if start in seen:
            continue
        loop, e = [], start
        while e not in seen:
            seen.add(e)
            loop.append(e)
            e = nxt[e]
        # the segment walk winds the loop clockwise about the outward direction: reversed triangles
        tris += [(t[0], t[2], t[1]) for t in triangulate(loop)]
    return tris


def share_face(e1, e2):
    """Whether cube edges e1, e2 lie in one cube face (a chord between them would run along that face)."""
    for f in range(3):
        for side in (0, 1):
            if all(e // 4 != f and corner_bits(edge_corners(e)[0])[f] == side for e in (e1, e2)):
                return True
    return False


def triangulations(poly):
    """Every triangulation of the convex polygon `poly` (vertex list), fans from poly[0] first."""
    if len(poly) < 3:
        yield []
        return
    a, b = poly[0], poly[-1]
    for m in range(len(poly) - 2, 0, -1):  # the triangle on edge (poly[-1], poly[0]) has apex poly[m]
        for left in triangulations(poly[:m + 1]):
            for right in triangulations(poly[m:]):
                yield left + right + [(a, poly[m], b)]


def triangulate(loop):
    """The first triangulation (over every rotation of the loop) none of whose chords runs along a cube face: two
    cells that share an ambiguous face then never both put a chord on it, so every mesh edge has exactly two
    faces."""
    n = len(loop)
    for r in range(n):
        rot = loop[r:] + loop[:r]
        for tri in triangulations(rot):
            chords = set()
            for t in tri:
                for i in range(3):
                    u, v = t[i], t[(i + 1) % 3]
                    if (rot.index(u) - rot.index(v)) % n not in (1, n - 1):
                        chords.add((min(u, v), max(u, v)))
            if not any(share_face(u, v) for u, v in chords):
                return [tuple(t) for t in tri]
    raise AssertionError('no face-free triangulation for loop %s' % loop)


def case_table():
    return [case_triangles(m) for m in range(256)]


def marching_cubes(vol, level=0.0, spacing=(1., 1., 1.)):
    """(verts (V, 3) float64 in index units * spacing, faces (F, 3) int64) — the device kernels' numbering:
    vertices in (grid point, axis) order, faces in (cell, table) order."""
    v = np.asarray(vol, np.float64)
    X, Y, Z = v.shape
    ins = v < level
    table = case_table()
    vid = {}
    verts = []
    for i in range(X):
        for j in range(Y):
            for k in range(Z):
                for a in range(3):
                    q = [i, j, k]
                    q[a] += 1
                    if q[a] >= v.shape[a]:
                        continue
                    if ins[i, j, k] != ins[q[0], q[1], q[2]]:
                        v0, v1 = v[i, j, k], v[q[0], q[1], q[2]]
                        t = (level - v0) / (v1 - v0)
                        p = [float(i), float(j), float(k)]
                        p[a] += t
                        vid[(i, j, k, a)] = len(verts)
                        verts.append([p[0] * spacing[0], p[1] * spacing[1], p[2] * spacing[2]])
    faces = []
    for i in range(X - 1):
        for j in range(Y - 1):
            for k in range(Z - 1):
                m = 0
                for c in range(8):
                    b = corner_bits(c)
                    if ins[i + b[0], j + b[1], k + b[2]]:
                        m |= 1 << c
                for tri in table[m]:
                    f = []
                    for e in tri:
                        c0, _, a = edge_corners(e)
                        b = corner_bits(c0)
                        f.append(vid[(i + b[0], j + b[1], k + b[2], a)])
                    faces.append(f)
    return np.array(verts, np.float64).reshape(-1, 3), np.array(faces, np.int64).reshape(-1, 3)
