"""Host camera: per-pixel primary-ray directions (the kernel's ``camera_rays`` input).

Restates ``Camera`` from src/camera.rs:28-194: ``perspective_rh_gl`` with the
reference's integer-division aspect ratio (src/camera.rs:123, SURVEY Appendix A
item 15), ``look_at_rh`` with +Y up, and ``recalculate_ray_directions``
(src/camera.rs:139-182), whose per-pixel arithmetic is done here in f32 in glam's
operation order. The 4x4 inverses are taken in float64 and rounded to f32 (glam's
SSE2 cofactor inverse is not restated bit for bit: camera rays are an input to
the hot path, handed identically to the HIP kernel and the oracle, so they do not
affect parity; device-side ray generation is SURVEY §8f-1).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

from . import buffers as B

f32 = np.float32


def _normalize64(v):
    v = np.asarray(v, np.float64)
    return v / np.linalg.norm(v)


def perspective_rh_gl(fov_y_rad: float, aspect: float, near: float, far: float) -> np.ndarray:
    """glam ``Mat4::perspective_rh_gl`` as a column-major (4 cols x 4) f32 array."""
    fov_y_rad, aspect, near, far = f32(fov_y_rad), f32(aspect), f32(near), f32(far)
    inv_length = f32(1.0) / (near - far)
    f = f32(1.0) / f32(math.tan(float(f32(0.5) * fov_y_rad)))
    a = f / aspect
    b = (near + far) * inv_length
    c = (f32(2.0) * near * far) * inv_length
    cols = np.zeros((4, 4), np.float32)
    cols[0] = [a, 0, 0, 0]
    cols[1] = [0, f, 0, 0]
    cols[2] = [0, 0, b, -1]
    cols[3] = [0, 0, c, 0]
    return cols


def look_at_rh(eye, center, up) -> np.ndarray:
    """glam ``Mat4::look_at_rh`` (column-major)."""
    eye = np.asarray(eye, np.float64)
    f = _normalize64(np.asarray(center, np.float64) - eye)
    s = _normalize64(np.cross(f, np.asarray(up, np.float64)))
    u = np.cross(s, f)
    cols = np.zeros((4, 4), np.float64)
    cols[0] = [s[0], u[0], -f[0], 0]
    cols[1] = [s[1], u[1], -f[1], 0]
    cols[2] = [s[2], u[2], -f[2], 0]
    cols[3] = [-s.dot(eye), -u.dot(eye), f.dot(eye), 1]
    return cols.astype(np.float32)


def inverse_cols(cols: np.ndarray) -> np.ndarray:
    """Inverse of a column-major 4x4, in float64, rounded to f32."""
    m = cols.astype(np.float64).T  # row-major matrix
    return np.linalg.inv(m).T.astype(np.float32)


def mat_vec_cols(cols: np.ndarray, v: np.ndarray) -> np.ndarray:
    """glam Mat4 * Vec4 in f32: ((c0*x + c1*y) + c2*z) + c3*w, for (n, 4) v."""
    cols = cols.astype(np.float32)
    v = v.astype(np.float32)
    r = cols[0][None, :] * v[:, 0:1]
    r = r + cols[1][None, :] * v[:, 1:2]
    r = r + cols[2][None, :] * v[:, 2:3]
    r = r + cols[3][None, :] * v[:, 3:4]
    return r.astype(np.float32)


@dataclass
class Camera:
    """src/camera.rs:7-25 (movement/turning state omitted: input handling is off-path)."""

    viewport_width: int
    viewport_height: int
    position: np.ndarray = field(default_factory=lambda: np.array([0.0, -6.0, 25.0], np.float32))
    direction: np.ndarray = field(default_factory=lambda: np.array([0.0, 0.0, -1.0], np.float32))
    vertical_fov: float = 45.0
    near_clip: float = 0.1
    far_clip: float = 100.0

    def __post_init__(self):
        self.position = np.asarray(self.position, np.float32)
        self.direction = np.asarray(self.direction, np.float32)
        self.recalculate_view()
        self.recalculate_projection()

    def recalculate_projection(self) -> None:  # src/camera.rs:121-128
        fov_rad = f32(self.vertical_fov) * f32(math.pi / 180.0)
        aspect = float(self.viewport_width // self.viewport_height)  # integer division, :123
        self.projection = perspective_rh_gl(fov_rad, aspect, self.near_clip, self.far_clip)
        self.inverse_projection = inverse_cols(self.projection)

    def recalculate_view(self) -> None:  # src/camera.rs:130-137
        self.view = look_at_rh(self.position, self.position + self.direction, [0.0, 1.0, 0.0])
        self.inverse_view = inverse_cols(self.view)

    def ray_camera(self) -> np.ndarray:
        rc = np.zeros((), B.RAY_CAMERA)
        rc["origin"] = self.position
        return rc

    def recalculate_ray_directions(self) -> np.ndarray:
        """src/camera.rs:139-182: one ``Ray`` per pixel, row-major (row 0 first)."""
        w, h = self.viewport_width, self.viewport_height
        aspect = f32(w) / f32(h)
        ys, xs = np.meshgrid(np.arange(h, dtype=np.float32), np.arange(w, dtype=np.float32), indexing="ij")
        xc = (xs / f32(w)).reshape(-1)
        yc = (ys / f32(h)).reshape(-1)
        nx = xc * f32(2.0) - f32(1.0)
        ny = yc * f32(2.0) - f32(1.0)
        ax = nx * aspect
        v = np.stack([ax, ny, np.ones_like(ax), np.ones_like(ax)], axis=1)
        target = mat_vec_cols(self.inverse_projection, v)
        t3 = target[:, :3] / target[:, 3:4]
        wst = B.normalize_f32(t3)
        wst4 = np.concatenate([wst, np.zeros((wst.shape[0], 1), np.float32)], axis=1)
        d = mat_vec_cols(self.inverse_view, wst4)[:, :3]
        rays = np.zeros(w * h, B.RAY)
        rays["direction"] = d
        return rays
