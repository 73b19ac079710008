"""Native scene building: the C++ restatement of
src/triangle_object.rs behind the C ABI (``csrc/scene_build.cpp``), returning the
same :class:`~rust_gpu_raytracing_amd.scene.SceneObject` records as the Python
restatement in ``scene.py``.

=================================================  =====================================
reference (src/triangle_object.rs)                 here
=================================================  =====================================
``stl_io::read_stl`` :69                           ``read_stl(data)`` -> ``rt_stl_read``
``SceneObject::new`` :55-127                       ``object_new(...)`` -> ``rt_scene_object_new``
``create_sub_objects`` :160-197                    ``create_sub_objects(obj, ...)``
``update_triangles`` + ``update_sub_objects``      ``update_object(obj)`` (host) or
:129-150, :199-220                                 ``Renderer.update_objects`` (device)
``load_stl_files`` :16-37                          ``load_stl_files(creations, meshes)``
=================================================  =====================================
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N
from . import buffers as B
from .scene import SUB_OBJECT_TRIANGLES, SceneObject

_F3 = ctypes.c_float * 3


def _check(rc: int, lib) -> None:
    N.check(None, rc, lib)


def read_stl(data: bytes, lib=None) -> np.ndarray:
    """Binary or ASCII STL bytes -> (n, 3, 3) f32 vertices (facet normals ignored, as the reference does)."""
    lib = lib or N.load_library()
    buf = (ctypes.c_uint8 * len(data)).from_buffer_copy(data) if data else (ctypes.c_uint8 * 1)()
    n = ctypes.c_uint32()
    _check(lib.rt_stl_triangle_count(buf, len(data), ctypes.byref(n)), lib)
    out = np.zeros((n.value, 3, 3), np.float32)
    if n.value:
        _check(lib.rt_stl_read(buf, len(data), N.ptr(out), n.value), lib)
    return out


def write_binary_stl(vertices: np.ndarray) -> bytes:
    """(n, 3, 3) vertices -> binary STL bytes (zero normals, zero attributes); for tests and tools."""
    v = np.ascontiguousarray(vertices, np.float32).reshape(-1, 9)
    rec = np.zeros(v.shape[0], np.dtype([("n", "<f4", 3), ("v", "<f4", 9), ("attr", "<u2")]))
    rec["v"] = v
    return b"\0" * 80 + np.uint32(v.shape[0]).tobytes() + rec.tobytes()


def object_new(vertices: np.ndarray, scale: float, coordinates, rotation, material_index: int, lib=None) -> SceneObject:
    """SceneObject::new (src/triangle_object.rs:55-127) in native code."""
    lib = lib or N.load_library()
    v = np.ascontiguousarray(vertices, np.float32).reshape(-1, 9)
    n = v.shape[0]
    pts = np.zeros((3 * n, 3), np.float32)
    tris = np.zeros(n, B.TRIANGLE)
    info = np.zeros((), B.OBJECT_INFO)
    state = np.zeros((), B.OBJECT_TRANSFORM)
    _check(lib.rt_scene_object_new(N.ptr(v) if n else None, n, float(np.float32(scale)),
                                   _F3(*np.asarray(coordinates, np.float32)), _F3(*np.asarray(rotation, np.float32)),
                                   int(material_index), N.ptr(pts), N.ptr(tris), info.ctypes.data, state.ctypes.data),
           lib)
    return SceneObject(info, tris, normalized_points=pts, rotation=state["rotation"].copy(),
                       scale=np.float32(state["scale"]), transformation=state["transformation"].copy())


def create_sub_objects(obj: SceneObject, start_sub: int, start_tri: int, lib=None):
    """create_sub_objects (src/triangle_object.rs:160-197) in native code; returns (next_sub, next_tri)."""
    lib = lib or N.load_library()
    n = obj.triangles.shape[0]
    subs = np.zeros((n + SUB_OBJECT_TRIANGLES - 1) // SUB_OBJECT_TRIANGLES, B.SUB_OBJECT_INFO)
    tris = np.ascontiguousarray(obj.triangles)
    _check(lib.rt_scene_object_create_sub_objects(N.ptr(tris), n, start_sub, start_tri, obj.object_info.ctypes.data,
                                                  N.ptr(subs)), lib)
    obj.sub_object_info = subs
    return start_sub + subs.shape[0], start_tri + n


def transform_of(obj: SceneObject) -> np.ndarray:
    t = np.zeros((), B.OBJECT_TRANSFORM)
    t["rotation"] = obj.rotation
    t["scale"] = obj.scale
    t["transformation"] = obj.transformation
    return t


def update_object(obj: SceneObject, lib=None) -> None:
    """update_triangles + update_sub_objects (src/triangle_object.rs:129-150, :199-220) in native code."""
    lib = lib or N.load_library()
    n = obj.triangles.shape[0]
    pts = np.ascontiguousarray(obj.normalized_points, np.float32)
    t = transform_of(obj)
    tris = np.zeros(n, B.TRIANGLE)
    subs = np.ascontiguousarray(obj.sub_object_info).copy()
    _check(lib.rt_scene_object_update(N.ptr(pts), n, t.ctypes.data, obj.object_info.ctypes.data, N.ptr(tris),
                                      N.ptr(subs)), lib)
    obj.triangles = tris
    obj.sub_object_info = subs


def load_stl_files(creations, meshes, lib=None) -> list:
    """load_stl_files (src/triangle_object.rs:16-37) in native code; arguments as scene.load_stl_files."""
    objs = []
    sub_i = tri_i = 0
    for model, scale, coords, rot, mat in creations:
        o = object_new(meshes[model], scale, coords, rot, mat, lib=lib)
        sub_i, tri_i = create_sub_objects(o, sub_i, tri_i, lib=lib)
        objs.append(o)
    return objs
