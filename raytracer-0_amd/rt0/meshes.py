"""Procedural triangle models for TRIANGLE scene entries.

BASELINE config 5 names a ~100k-triangle model (the reference's Happy Buddha
OBJ is git-ignored and absent): `icosphere(6)` (81,920 triangles)
stands in for it, as SURVEY suggests.  `wavy_icosphere` displaces the sphere
so that rays graze many triangles at different depths (a harder BVH case).
"""
import numpy as np


def icosphere(level, radius=1.0):
    """Unit icosahedron subdivided `level` times, projected onto the sphere:
    20 * 4**level triangles, counter-clockwise seen from outside.
    Returns (positions float32 [nv, 3], triangles int32 [nt, 3])."""
    t = (1.0 + 5.0 ** 0.5) / 2.0
    v = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
         (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    f = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2), (10, 7, 6),
         (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11), (6, 2, 10),
         (8, 6, 7), (9, 8, 1)]
    verts = [np.array(p, np.float64) / np.linalg.norm(p) for p in v]
    faces = list(f)
    for _ in range(level):
        mid = {}

        def midpoint(a, b):
            key = (min(a, b), max(a, b))
            if key not in mid:
                m = verts[a] + verts[b]
                verts.append(m / np.linalg.norm(m))
                mid[key] = len(verts) - 1
            return mid[key]

        nf = []
        for a, b, c in faces:
            ab, bc, ca = midpoint(a, b), midpoint(b, c), midpoint(c, a)
            nf += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        faces = nf
    return (np.array(verts) * radius).astype(np.float32), np.array(faces, np.int32)


def wavy_icosphere(level, radius=1.0, amp=0.08, freq=6.0):
    """icosphere displaced along the normal by amp*sin(freq*x)*sin(freq*y)*sin(freq*z)."""
    v, f = icosphere(level)
    p = v.astype(np.float64)
    s = 1.0 + amp * np.sin(freq * p[:, 0]) * np.sin(freq * p[:, 1]) * np.sin(freq * p[:, 2])
    return (p * (s * radius)[:, None]).astype(np.float32), f


def world_triangles(positions, triangles, pos, scale):
    """World-space triangle vertices [nt, 9] of an instance (pos + scale * v), in
    the float32 arithmetic of librt0's BVH input (rt0_host.cpp build_bvh)."""
    v = np.asarray(positions, np.float32)[np.asarray(triangles).reshape(-1)]
    w = np.asarray(pos, np.float32)[None, :] + np.float32(scale) * v
    return w.astype(np.float32).reshape(-1, 9)
