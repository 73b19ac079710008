"""ctypes binding of the C ABI in ``include/rt_abi.h``.

The shared library ``librt_pathtrace.so`` (HIP kernel + host runtime) is built
in-tree by ``rust_gpu_raytracing_amd.build``. There is no fallback: if the
library is missing or fails to load, every entry point raises
:class:`NativeLibraryError`.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

from . import buffers as B

LIB_NAME = "librt_pathtrace.so"
LIB_PATH = Path(__file__).resolve().parent / LIB_NAME

RT_OK = 0
RT_E_INVALID = -1
RT_E_HIP = -2
RT_E_NOMEM = -3
RT_E_CAPACITY = -4
RT_E_NODEVICE = -5

_ERR_NAMES = {
    RT_E_INVALID: "RT_E_INVALID",
    RT_E_HIP: "RT_E_HIP",
    RT_E_NOMEM: "RT_E_NOMEM",
    RT_E_CAPACITY: "RT_E_CAPACITY",
    RT_E_NODEVICE: "RT_E_NODEVICE",
}


class NativeLibraryError(RuntimeError):
    """The HIP extension is missing or could not be loaded."""


class RtError(RuntimeError):
    """A C-ABI call returned a negative status."""

    def __init__(self, code: int, message: str):
        super().__init__(f"{_ERR_NAMES.get(code, code)}: {message}")
        self.code = code


class rt_ray_camera(ctypes.Structure):
    _fields_ = [("origin", ctypes.c_float * 3), ("_padding", ctypes.c_uint32)]


class rt_params(ctypes.Structure):
    _fields_ = [(name, ctypes.c_uint32) for name in B.PARAMS.names]


class rt_create_info(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_uint32),
        ("height", ctypes.c_uint32),
        ("device", ctypes.c_int32),
        ("_reserved", ctypes.c_uint32),
        ("camera", rt_ray_camera),
        ("camera_rays", ctypes.c_void_p),
        ("materials", ctypes.c_void_p),
        ("material_count", ctypes.c_uint32),
        ("spheres", ctypes.c_void_p),
        ("sphere_count", ctypes.c_uint32),
        ("triangles", ctypes.c_void_p),
        ("triangle_count", ctypes.c_uint32),
        ("objects", ctypes.c_void_p),
        ("object_count", ctypes.c_uint32),
        ("sub_objects", ctypes.c_void_p),
        ("sub_object_count", ctypes.c_uint32),
        ("params", rt_params),
        ("rank", ctypes.c_uint32),
        ("world_size", ctypes.c_uint32),
    ]


assert ctypes.sizeof(rt_params) == 48
assert ctypes.sizeof(rt_ray_camera) == 16

# name -> (restype, argtypes)
_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
SIGNATURES = {
    "rt_create": (ctypes.c_int, [ctypes.POINTER(rt_create_info), ctypes.POINTER(_P)]),
    "rt_destroy": (None, [_P]),
    "rt_last_error": (ctypes.c_char_p, [_P]),
    "rt_abi_version": (ctypes.c_int, []),
    "rt_build_hash": (ctypes.c_char_p, []),
    "rt_upload_textures": (ctypes.c_int, [_P, _P, _U32, _U32, _U32]),
    "rt_upload_env_map": (ctypes.c_int, [_P, _P, _U32, _U32]),
    "rt_update_params": (ctypes.c_int, [_P, ctypes.POINTER(rt_params)]),
    "rt_reset_accumulation": (ctypes.c_int, [_P, ctypes.POINTER(rt_params)]),
    "rt_update_ray_directions": (ctypes.c_int, [_P, _P, _U32]),
    "rt_update_camera": (ctypes.c_int, [_P, ctypes.POINTER(rt_ray_camera)]),
    "rt_update_camera_matrices": (ctypes.c_int, [_P, _P, _P]),
    "rt_update_spheres": (ctypes.c_int, [_P, _P, _U32]),
    "rt_update_triangles": (ctypes.c_int, [_P, _P, _U32]),
    "rt_update_object_info": (ctypes.c_int, [_P, _P, _U32]),
    "rt_update_sub_object_info": (ctypes.c_int, [_P, _P, _U32]),
    "rt_update_materials": (ctypes.c_int, [_P, _P, _U32]),
    "rt_dispatch": (ctypes.c_int, [_P, _U32]),
    "rt_compute_frame": (ctypes.c_int, [_P, _U32]),
    "rt_compute_frames": (ctypes.c_int, [_P, _U32, _U32]),
    "rt_submit_frames": (ctypes.c_int, [_P, _U32, _U32]),
    "rt_set_frame_batch": (ctypes.c_int, [_P, _U32]),
    "rt_frame_batch": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
    "rt_flush": (ctypes.c_int, [_P]),
    "rt_synchronize": (ctypes.c_int, [_P]),
    "rt_read_output": (ctypes.c_int, [_P, _P]),
    "rt_copy_output_to_device": (ctypes.c_int, [_P, _P, _U32]),
    "rt_read_accumulation": (ctypes.c_int, [_P, _P]),
    "rt_read_output_pitched": (ctypes.c_int, [_P, _P, _U32]),
    "rt_bytes_per_row": (_U32, [_U32, _U32]),
    "rt_ray_count": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64)]),
    "rt_reset_ray_count": (ctypes.c_int, [_P]),
    "rt_accumulation_index": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint32)]),
    "rt_set_brute_force": (ctypes.c_int, [_P, ctypes.c_int]),
    "rt_set_triangle_pruning": (ctypes.c_int, [_P, ctypes.c_int]),
    "rt_streamed_bytes": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64)]),
    "rt_streamed_bytes_l2": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64)]),
    "rt_set_tuning": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_int32]),
    "rt_set_tile_schedule": (ctypes.c_int, [_P, _U32]),
    "rt_tile_schedule_state": (ctypes.c_int, [_P, _P, _P]),
    "rt_set_timing": (ctypes.c_int, [_P, ctypes.c_int]),
    "rt_last_dispatch_ms": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_float)]),
    "rt_dispatch_time_total": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]),
    "rt_resolve_time_total": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]),
    "rt_reset_timing": (ctypes.c_int, [_P]),
    "rt_owned_pixel_count": (ctypes.c_int, [_P, _U32, _U32, ctypes.POINTER(ctypes.c_uint64)]),
    "rt_pack_owned_accumulation": (ctypes.c_int, [_P, _P]),
    "rt_unpack_accumulation": (ctypes.c_int, [_P, _P, _U32, _U32, _U32]),
    "rt_pack_owned_output": (ctypes.c_int, [_P, _P]),
    "rt_unpack_output": (ctypes.c_int, [_P, _P, _U32, _U32]),
    "rt_unpack_accumulation_ranks": (ctypes.c_int, [_P, _P, ctypes.c_uint64, _U32, _U32, _U32]),
    "rt_unpack_output_ranks": (ctypes.c_int, [_P, _P, ctypes.c_uint64, _U32, _U32]),
    "rt_launch_config": (ctypes.c_int, [_P] + [ctypes.POINTER(ctypes.c_uint32)] * 4),
    "rt_last_launch_passes": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint32)]),
    "rt_debug_counters": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), _U32]),
    "rt_debug_check_leaf_certificates": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint32),
                                                        ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
    "rt_math_selftest": (ctypes.c_int, [_U32, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32)]),
    "rt_stream": (_P, [_P]),
    "rt_srgb_table": (ctypes.c_int, [ctypes.POINTER(ctypes.c_float)]),
    "rt_stl_triangle_count": (ctypes.c_int, [_P, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32)]),
    "rt_stl_read": (ctypes.c_int, [_P, ctypes.c_size_t, _P, _U32]),
    "rt_scene_object_new": (ctypes.c_int, [_P, _U32, ctypes.c_float, _P, _P, _U32, _P, _P, _P, _P]),
    "rt_scene_object_create_sub_objects": (ctypes.c_int, [_P, _U32, _U32, _U32, _P, _P]),
    "rt_scene_object_update": (ctypes.c_int, [_P, _U32, _P, _P, _P, _P]),
    "rt_set_object_models": (ctypes.c_int, [_P, _P, _U32]),
    "rt_update_objects": (ctypes.c_int, [_P, _P, _U32]),
    "rt_read_triangles": (ctypes.c_int, [_P, _P, _U32]),
    "rt_read_object_info": (ctypes.c_int, [_P, _P, _U32]),
    "rt_read_sub_object_info": (ctypes.c_int, [_P, _P, _U32]),
    # several GPUs in one process (rt_multi.cpp)
    "rt_create_multi": (ctypes.c_int, [ctypes.POINTER(rt_create_info), ctypes.POINTER(ctypes.c_int32), _U32,
                                       ctypes.POINTER(_P)]),
    "rt_create_multi_ex": (ctypes.c_int, [ctypes.POINTER(rt_create_info), ctypes.POINTER(ctypes.c_int32), _U32, _U32,
                                          ctypes.POINTER(_P)]),
    "rt_destroy_multi": (None, [_P]),
    "rt_group_last_error": (ctypes.c_char_p, [_P]),
    "rt_group_size": (_U32, [_P]),
    "rt_group_context": (_P, [_P, _U32]),
    "rt_group_compute_frame": (ctypes.c_int, [_P, _U32]),
    "rt_group_set_frame_batch": (ctypes.c_int, [_P, _U32]),
    "rt_group_flush": (ctypes.c_int, [_P]),
    "rt_group_synchronize": (ctypes.c_int, [_P]),
    "rt_group_update_params": (ctypes.c_int, [_P, ctypes.POINTER(rt_params)]),
    "rt_group_reset_accumulation": (ctypes.c_int, [_P, ctypes.POINTER(rt_params)]),
    "rt_group_update_camera": (ctypes.c_int, [_P, ctypes.POINTER(rt_ray_camera)]),
    "rt_group_update_camera_matrices": (ctypes.c_int, [_P, _P, _P]),
    "rt_group_update_ray_directions": (ctypes.c_int, [_P, _P, _U32]),
    "rt_group_update_spheres": (ctypes.c_int, [_P, _P, _U32]),
    "rt_group_update_triangles": (ctypes.c_int, [_P, _P, _U32]),
    "rt_group_update_object_info": (ctypes.c_int, [_P, _P, _U32]),
    "rt_group_update_sub_object_info": (ctypes.c_int, [_P, _P, _U32]),
    "rt_group_update_materials": (ctypes.c_int, [_P, _P, _U32]),
    "rt_group_upload_textures": (ctypes.c_int, [_P, _P, _U32, _U32, _U32]),
    "rt_group_upload_env_map": (ctypes.c_int, [_P, _P, _U32, _U32]),
    "rt_group_ray_count": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64)]),
    "rt_group_reset_ray_count": (ctypes.c_int, [_P]),
    "rt_gather_frame": (ctypes.c_int, [_P, _U32, _U32]),
    "rt_group_read_output": (ctypes.c_int, [_P, _U32, _P]),
    "rt_group_read_accumulation": (ctypes.c_int, [_P, _U32, _P]),
}

RT_DEFAULT_FRAME_BATCH = 16  # include/rt_abi.h (ABI 11)
RT_PASS_PATH, RT_PASS_PRIMARY, RT_PASS_RESOLVE, RT_PASS_BRUTE, RT_PASS_BRUTE_STREAM = 1, 2, 4, 8, 16
RT_GROUP_COPY_TRANSPORT = 1  # rt_create_multi_ex flags
RT_GATHER_IMAGE = 0
RT_GATHER_ACCUMULATION = 1

_lib = None


def load_library(path: os.PathLike | str | None = None) -> ctypes.CDLL:
    """Load and return the HIP extension; raise if it is unavailable.

    With no argument: the in-tree build (cached), or the build named by the
    RT_LIB environment variable (experiment builds for A/B runs; it must exist
    too — there is no fallback). With a path: that build, uncached."""
    global _lib
    if path is None:
        if _lib is not None:
            return _lib
        _lib = _open(Path(os.environ.get("RT_LIB") or LIB_PATH))
        return _lib
    return _open(Path(path), strict=False)


def _open(p: Path, strict: bool = True) -> ctypes.CDLL:
    if not p.exists():
        raise NativeLibraryError(
            f"{p} not found: build the HIP extension first "
            "(python -c 'import __graft_entry__ as g; g.build()')"
        )
    try:
        lib = ctypes.CDLL(str(p), mode=ctypes.RTLD_LOCAL)
    except OSError as exc:  # pragma: no cover - depends on the box
        raise NativeLibraryError(f"could not load {p}: {exc}") from exc
    for name, (res, args) in SIGNATURES.items():
        if not strict and not hasattr(lib, name):  # older experiment builds may predate an entry point
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def check(ctx, rc: int, lib=None) -> None:
    if rc != RT_OK:
        msg = (lib or load_library()).rt_last_error(ctx)
        raise RtError(rc, msg.decode() if msg else "")


def ptr(a: np.ndarray | None) -> int | None:
    if a is None or a.size == 0:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays handed to the C ABI must be C-contiguous"
    return a.ctypes.data


def params_struct(p: np.ndarray) -> rt_params:
    s = rt_params()
    for name in B.PARAMS.names:
        setattr(s, name, int(p[name]))
    return s


def srgb_table() -> np.ndarray:
    out = np.zeros(256, np.float32)
    rc = load_library().rt_srgb_table(out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    if rc != RT_OK:
        raise RtError(rc, "rt_srgb_table")
    return out
