"""Adversarial geometry for the triangle walk's distance pruning.

A flat grid of triangles in a random plane (coordinates not representable exactly, so
the reference's f32 distance and barycentrics carry rounding), and rays that lie
nearly in that plane close to their origin: the regime where the reference's own
test is dominated by rounding and a pruning slack that is not derived from the
error bound can skip the triangle the sweep accepts. Shared by the CPU harness tests
(tests/test_tri_accel_cpu.py) and the GPU parity tests (tests/test_gpu_parity.py)."""
from __future__ import annotations

import numpy as np

from rust_gpu_raytracing_amd import buffers as B
from rust_gpu_raytracing_amd.scene import SceneObject


def tilted_plane_grid(seed, n=200, size=0.1):
    """2 n^2 triangles on an n x n grid of `size` cells in a random plane through a random
    point: (objects, sub_objects, triangles, SceneObject, frame=(p0, e1, e2, normal))."""
    rng = np.random.default_rng(seed)
    m, _ = np.linalg.qr(rng.standard_normal((3, 3)))
    e1, e2, nrm = m[:, 0], m[:, 1], m[:, 2]
    p0 = rng.uniform(-3, 3, 3)
    g = (np.arange(n + 1) - n / 2) * size
    u, v = np.meshgrid(g, g)
    p = (p0 + u[..., None] * e1 + v[..., None] * e2).astype(np.float32)
    p00, p10, p01, p11 = p[:-1, :-1], p[:-1, 1:], p[1:, :-1], p[1:, 1:]
    t = B.scene_triangles(np.concatenate([p00.reshape(-1, 3), p10.reshape(-1, 3)]),
                          np.concatenate([p10.reshape(-1, 3), p11.reshape(-1, 3)]),
                          np.concatenate([p01.reshape(-1, 3), p01.reshape(-1, 3)]))
    info = np.zeros((), B.OBJECT_INFO)
    info["min_bounds"] = p.reshape(-1, 3).min(0)
    info["max_bounds"] = p.reshape(-1, 3).max(0)
    o = SceneObject(info, t)
    o.create_sub_objects(0, 0)
    objs = np.stack([np.asarray(o.object_info)]).astype(B.OBJECT_INFO)
    return objs, o.sub_object_info.astype(B.SUB_OBJECT_INFO), t, o, (p0, e1, e2, nrm)


def grazing_directions(frame, n, c_range, rng):
    """Unit directions meeting the plane at cos c (log-uniform in c_range), heading into it
    from the side opposite its normal, with random in-plane azimuths."""
    p0, e1, e2, nrm = frame
    c = 10 ** rng.uniform(*np.log10(c_range), n)
    phi = rng.uniform(0, 2 * np.pi, n)
    return (np.cos(phi)[:, None] * e1 + np.sin(phi)[:, None] * e2) * np.sqrt(1 - c * c)[:, None] + c[:, None] * nrm


def grazing_rays(frame, n, h_range, c_range, seed, span=8.0):
    """(n, 6) rays: origins h (log-uniform) from the plane, grazing directions."""
    p0, e1, e2, nrm = frame
    rng = np.random.default_rng(seed)
    h = 10 ** rng.uniform(*np.log10(h_range), n)
    u, v = rng.uniform(-span, span, n), rng.uniform(-span, span, n)
    o = p0 + u[:, None] * e1 + v[:, None] * e2 - h[:, None] * nrm
    return np.concatenate([o, grazing_directions(frame, n, c_range, rng)], 1)
