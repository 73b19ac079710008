"""GPU-visible POD layouts, as numpy structured dtypes.

Mirrors the reference's ``#[repr(C)]`` bytemuck structs in
``src/buffers.rs:7-129`` byte for byte, so arrays built here can be handed to
the C ABI (``include/rt_abi.h``) without conversion, exactly as the reference
hands ``bytemuck::cast_slice`` views to ``wgpu::Queue::write_buffer``.
"""
from __future__ import annotations

import numpy as np

# src/buffers.rs:9-22 -- Params (48 B)
PARAMS = np.dtype(
    [
        ("screen_width", "<u4"),
        ("accumulation_index", "<u4"),
        ("accumulate", "<u4"),
        ("sphere_count", "<u4"),
        ("object_count", "<u4"),
        ("compute_per_frame", "<u4"),
        ("texture_width", "<u4"),
        ("texture_height", "<u4"),
        ("texture_count", "<u4"),  # `textue_count` in the reference
        ("env_map_width", "<u4"),
        ("env_map_height", "<u4"),
        ("_padding", "<u4"),
    ]
)

# src/buffers.rs:26-29 / :33-36 -- RayCamera, Ray (16 B)
RAY_CAMERA = np.dtype([("origin", "<f4", 3), ("_padding", "<u4")])
RAY = np.dtype([("direction", "<f4", 3), ("_padding", "<u4")])

# src/buffers.rs:40-45 -- SceneSphere (32 B)
SPHERE = np.dtype(
    [("position", "<f4", 3), ("radius", "<f4"), ("material_index", "<u4"), ("_padding", "<u4", 3)]
)

# src/buffers.rs:49-64 -- SceneTriangle (112 B)
TRIANGLE = np.dtype(
    [
        ("a", "<f4", 3), ("_p0", "<u4"),
        ("edge_ab", "<f4", 3), ("_p1", "<u4"),
        ("edge_ac", "<f4", 3), ("_p2", "<u4"),
        ("calc_normal", "<f4", 3), ("_p3", "<u4"),
        ("face_normal", "<f4", 3), ("_p4", "<u4"),
        ("min_bounds", "<f4", 3), ("_p5", "<u4"),
        ("max_bounds", "<f4", 3), ("_p6", "<u4"),
    ]
)

# src/buffers.rs:100-109 -- SceneMaterial (32 B)
MATERIAL = np.dtype(
    [
        ("texture_index", "<u4"),
        ("roughness", "<f4"),
        ("emission_power", "<f4"),
        ("specular", "<f4"),
        ("specular_scatter", "<f4"),
        ("glass", "<f4"),
        ("refraction_index", "<f4"),
        ("_padding", "<u4"),
    ]
)

# src/buffers.rs:113-120 -- ObjectInfo (48 B)
OBJECT_INFO = np.dtype(
    [
        ("min_bounds", "<f4", 3),
        ("first_sub_object_index", "<u4"),
        ("max_bounds", "<f4", 3),
        ("sub_object_count", "<u4"),
        ("material_index", "<u4"),
        ("_padding", "<u4", 3),
    ]
)

# src/buffers.rs:124-129 -- SubObjectInfo (32 B)
SUB_OBJECT_INFO = np.dtype(
    [
        ("min_bounds", "<f4", 3),
        ("first_triangle_index", "<u4"),
        ("max_bounds", "<f4", 3),
        ("triangle_count", "<u4"),
    ]
)

# include/rt_abi.h rt_object_transform -- SceneObject's edit state
# (rotation in degrees, scale, transformation; src/triangle_object.rs:39-52), 32 B
OBJECT_TRANSFORM = np.dtype(
    [("rotation", "<f4", 3), ("scale", "<f4"), ("transformation", "<f4", 3), ("_padding", "<u4")]
)

for _dt, _size in (
    (PARAMS, 48), (RAY_CAMERA, 16), (RAY, 16), (SPHERE, 32), (TRIANGLE, 112),
    (MATERIAL, 32), (OBJECT_INFO, 48), (SUB_OBJECT_INFO, 32), (OBJECT_TRANSFORM, 32),
):
    assert _dt.itemsize == _size, (_dt, _size)


def cross_f32(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """glam ``Vec3A::cross`` in f32: (y*bz - z*by, z*bx - x*bz, x*by - y*bx)."""
    a = a.astype(np.float32, copy=False)
    b = b.astype(np.float32, copy=False)
    x = a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1]
    y = a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2]
    z = a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]
    return np.stack([x, y, z], axis=-1).astype(np.float32)


def dot_f32(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """glam ``dot3``: ((x*x' + y*y') + z*z') in f32."""
    a = a.astype(np.float32, copy=False)
    b = b.astype(np.float32, copy=False)
    return ((a[..., 0] * b[..., 0] + a[..., 1] * b[..., 1]) + a[..., 2] * b[..., 2]).astype(np.float32)


def normalize_f32(v: np.ndarray) -> np.ndarray:
    """glam ``Vec3A::normalize``: v * (1 / sqrt(dot(v, v))) in f32."""
    v = v.astype(np.float32, copy=False)
    with np.errstate(divide="ignore", invalid="ignore"):
        recip = np.float32(1.0) / np.sqrt(dot_f32(v, v))
    return (v * recip[..., None]).astype(np.float32)


def scene_triangles(a: np.ndarray, b: np.ndarray, c: np.ndarray) -> np.ndarray:
    """Vectorised ``SceneTriangle::new`` (src/buffers.rs:66-95).

    ``a``, ``b``, ``c`` are (n, 3) float32 vertex arrays.
    """
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    c = np.asarray(c, np.float32)
    out = np.zeros(a.shape[0], TRIANGLE)
    edge_ab = (b - a).astype(np.float32)
    edge_ac = (c - a).astype(np.float32)
    calc_normal = cross_f32(edge_ab, edge_ac)
    out["a"] = a
    out["edge_ab"] = edge_ab
    out["edge_ac"] = edge_ac
    out["calc_normal"] = calc_normal
    out["face_normal"] = normalize_f32(calc_normal)
    # Vec3A::min/max (SSE minps/maxps: `x < y ? x : y`, the second operand on
    # ties and NaN), chained as a.min(b).min(c)
    mn = np.where(a < b, a, b)
    out["min_bounds"] = np.where(mn < c, mn, c)
    mx = np.where(a > b, a, b)
    out["max_bounds"] = np.where(mx > c, mx, c)
    return out


def make_params(
    screen_width: int,
    *,
    accumulation_index: int = 1,
    accumulate: int = 1,
    sphere_count: int = 0,
    object_count: int = 0,
    compute_per_frame: int = 1,
    texture_width: int = 1,
    texture_height: int = 1,
    texture_count: int = 1,
    env_map_width: int = 1,
    env_map_height: int = 1,
) -> np.ndarray:
    """One ``Params`` record (built the way src/main.rs:131-144 builds it)."""
    p = np.zeros((), PARAMS)
    p["screen_width"] = screen_width
    p["accumulation_index"] = accumulation_index
    p["accumulate"] = accumulate
    p["sphere_count"] = sphere_count
    p["object_count"] = object_count
    p["compute_per_frame"] = compute_per_frame
    p["texture_width"] = texture_width
    p["texture_height"] = texture_height
    p["texture_count"] = texture_count
    p["env_map_width"] = env_map_width
    p["env_map_height"] = env_map_height
    return p
