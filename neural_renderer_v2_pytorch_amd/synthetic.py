"""Synthetic meshes and batched scenes for parity tests and the benchmark.

Meshes:
  * icosphere(level)  -- level 4: V=2562, F=5120 (the headline "~5k-face mesh"), radius 0.9
  * torus(nu, nv)     -- 250x100: V=25000, F=50000 (config 5)
  * subdivide(v, f, vt, ft) -- one midpoint subdivision (the ShapeNet car 3644 -> 14576 faces, config 3)
Scenes: per-item Gaussian vertex jitter (seed 1000+b) and per-item viewpoint
get_points_from_angles(2.732, U(-30,30), U(0,360)) (seed 2000+b); faces shared across the batch.
"""
import math

import numpy as np
import torch


def icosphere(level=4, radius=0.9):
    t = (1.0 + 5.0 ** 0.5) / 2.0
    verts = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t),
             (0, 1, -t), (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    verts = [np.array(v, np.float64) / np.linalg.norm(v) for v in verts]
    faces = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4),
             (11, 10, 2), (10, 7, 6), (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8),
             (3, 8, 9), (4, 9, 5), (2, 4, 11), (6, 2, 10), (8, 6, 7), (9, 8, 1)]
    for _ in range(level):
        cache = {}

        def mid(a, b):
            key = (min(a, b), max(a, b))
            if key not in cache:
                m = verts[a] + verts[b]
                verts.append(m / np.linalg.norm(m))
                cache[key] = len(verts) - 1
            return cache[key]

        nf = []
        for a, b, c in faces:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            nf += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        faces = nf
    v = (np.stack(verts) * radius).astype(np.float32)
    f = np.asarray(faces, np.int32)
    return v, f


def torus(nu=250, nv=100, major=0.65, minor=0.25):
    u = np.arange(nu) * (2 * math.pi / nu)
    w = np.arange(nv) * (2 * math.pi / nv)
    uu, ww = np.meshgrid(u, w, indexing="ij")
    x = (major + minor * np.cos(ww)) * np.cos(uu)
    y = minor * np.sin(ww)
    z = (major + minor * np.cos(ww)) * np.sin(uu)
    v = np.stack([x, y, z], -1).reshape(-1, 3).astype(np.float32)
    i = np.arange(nu)[:, None]
    j = np.arange(nv)[None, :]
    a = i * nv + j
    b = ((i + 1) % nu) * nv + j
    c = ((i + 1) % nu) * nv + (j + 1) % nv
    d = i * nv + (j + 1) % nv
    f = np.concatenate([np.stack([a, b, c], -1).reshape(-1, 3), np.stack([a, c, d], -1).reshape(-1, 3)], 0)
    return v, f.astype(np.int32)


def subdivide(v, f, vt=None, ft=None):
    """Midpoint subdivision: every triangle into 4 (shared edge midpoints, computed in float64);
    the same on the uv mesh when given.  SURVEY.md section 8d: the car 4e49873... (F=3644) once
    subdivided is the "ShapeNet car ~15k faces" of BASELINE config 3 (F=14576)."""
    def split(verts, faces):
        cache, out_v, nf = {}, [tuple(x) for x in verts], []

        def mid(a, b):
            key = (min(a, b), max(a, b))
            if key not in cache:
                out_v.append(tuple((np.asarray(out_v[a], np.float64) + np.asarray(out_v[b], np.float64)) / 2))
                cache[key] = len(out_v) - 1
            return cache[key]
        for a, b, c in faces:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            nf += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        return np.asarray(out_v, np.float32), np.asarray(nf, np.int32)
    v2, f2 = split(v, f)
    if vt is None:
        return v2, f2
    vt2, ft2 = split(vt, ft)
    return v2, f2, vt2, ft2


def viewpoints(batch_size, distance=2.732, seed_base=2000):
    out = []
    for b in range(batch_size):
        r = np.random.RandomState(seed_base + b)
        el = r.uniform(-30, 30)
        az = r.uniform(0, 360)
        el, az = np.radians(el), np.radians(az)
        out.append((distance * np.cos(el) * np.sin(az), distance * np.sin(el),
                    -distance * np.cos(el) * np.cos(az)))
    return np.asarray(out, np.float32)


def jittered(vertices, batch_size, sigma=0.01, seed_base=1000):
    out = np.empty((batch_size,) + vertices.shape, np.float32)
    for b in range(batch_size):
        r = np.random.RandomState(seed_base + b)
        out[b] = vertices + r.normal(0, sigma, vertices.shape).astype(np.float32)
    return out


def project(vertices, eyes, viewing_angle=30.0):
    """look_at (at=0, up=+y) + perspective, per item, float32 torch ops on the input's device.
    Equivalent to the reference Renderer.transform_vertices (renderer.py:24-35) for B != 3."""
    from .look_at import look_at
    from .perspective import perspective
    return perspective(look_at(vertices, eyes), angle=viewing_angle)
