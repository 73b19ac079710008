"""The C-ABI library: builds, loads, exports exactly what include/rt_abi.h declares.

No kernel launches here (no GPU in the CPU suite); host-only entry points only.
"""
import ctypes
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

from rust_gpu_raytracing_amd import _native as N
from rust_gpu_raytracing_amd import buffers as B

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "rt_abi.h"


def declared_functions():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"^RT_API\s+[\w\s\*]+?\b(rt_\w+)\s*\(", text, re.M)))


def test_header_declares_expected_surface():
    fns = declared_functions()
    for must in ("rt_create", "rt_destroy", "rt_compute_frame", "rt_dispatch", "rt_update_spheres",
                 "rt_update_triangles", "rt_reset_accumulation", "rt_read_accumulation", "rt_ray_count"):
        assert must in fns
    assert set(fns) == set(N.SIGNATURES), set(fns) ^ set(N.SIGNATURES)


def test_library_exports_every_declared_symbol(native_lib):
    out = subprocess.run(["nm", "-D", "--defined-only", str(N.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (rt_\w+)", out))
    # exactly the declared surface: internal helpers stay hidden (-fvisibility=hidden)
    assert set(declared_functions()) == exported
    for name in declared_functions():
        assert hasattr(native_lib, name)


def test_abi_version(native_lib):
    assert native_lib.rt_abi_version() == 12


def test_library_reads_no_environment():
    """The product library takes no input from the process environment (ABI 12: the round-1..5
    RT_* A/B switches became rt_set_tuning keys, the inexact pruning mode only
    rt_set_triangle_pruning(ctx, 2)): it imports neither getenv nor secure_getenv, so no
    environment can change what it renders (tests/test_gpu_parity.py checks the same on the GPU)."""
    out = subprocess.run(["nm", "-D", "--undefined-only", str(N.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    assert not re.search(r"\b(secure_)?getenv\b", out), out


def test_tuning_keys_documented():
    """Every rt_set_tuning key the library accepts is listed in include/rt_abi.h."""
    src = (ROOT / "rust_gpu_raytracing_amd" / "csrc" / "rt_abi.cpp").read_text()
    body = src[src.index("int rt_set_tuning("):]
    body = body[:body.index("\n}\n")]
    keys = set(re.findall(r'k == "(\w+)"', body))
    assert len(keys) >= 25
    header = HEADER.read_text()
    doc = header[header.index("Exact variants of the launch schedule"):header.index("RT_API int rt_set_tuning")]
    assert keys == set(re.findall(r'"(\w+)"', doc)), keys ^ set(re.findall(r'"(\w+)"', doc))


def test_library_built_from_these_sources(native_lib):
    """The loaded library embeds the hash of the sources + flags it was compiled from
    (build.py: content-gated, not mtime-gated): it must be this tree's."""
    from rust_gpu_raytracing_amd import build as nb

    assert native_lib.rt_build_hash().decode() == nb.source_hash() == nb.build_info()["hash"]


def test_ctypes_layouts_match_header():
    assert ctypes.sizeof(N.rt_params) == B.PARAMS.itemsize == 48
    # rt_create_info: 4 u32, camera 16 B, rays pointer, then 5 (pointer, u32 count + pad) pairs
    assert N.rt_create_info.camera.offset == 16
    assert N.rt_create_info.camera_rays.offset == 32
    assert N.rt_create_info.materials.offset == 40
    assert N.rt_create_info.sub_objects.offset == 40 + 4 * 16


def test_create_info_layout_against_compiled_header(tmp_path):
    # compile a tiny C program against the real header and compare offsets
    src = tmp_path / "off.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "rt_abi.h"\n'
        "int main(void){printf(\"%zu %zu %zu %zu %zu\\n\", sizeof(rt_create_info),"
        " offsetof(rt_create_info, camera_rays), offsetof(rt_create_info, params),"
        " offsetof(rt_create_info, rank), sizeof(rt_scene_triangle)); return 0;}\n"
    )
    exe = tmp_path / "off"
    subprocess.run(["gcc", f"-I{ROOT / 'include'}", str(src), "-o", str(exe)], check=True)
    size, rays, params, rank, tri = map(int, subprocess.run([str(exe)], capture_output=True, text=True,
                                                             check=True).stdout.split())
    assert size == ctypes.sizeof(N.rt_create_info)
    assert rays == N.rt_create_info.camera_rays.offset
    assert params == N.rt_create_info.params.offset
    assert rank == N.rt_create_info.rank.offset
    assert tri == 112


def test_srgb_table_matches_oracle(native_lib, oracle_lib):
    prod = N.srgb_table()
    ref = np.zeros(256, np.float32)
    oracle_lib.lib().oracle_srgb_table(ref.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    assert np.array_equal(prod.view(np.uint32), ref.view(np.uint32))


def test_invalid_create_is_rejected_without_device(native_lib):
    info = N.rt_create_info()  # width = height = 0
    ctx = ctypes.c_void_p()
    rc = native_lib.rt_create(ctypes.byref(info), ctypes.byref(ctx))
    assert rc == N.RT_E_INVALID and not ctx.value
    assert b"width" in native_lib.rt_last_error(None)


def test_null_context_calls_fail_cleanly(native_lib):
    assert native_lib.rt_compute_frame(None, 8) == N.RT_E_INVALID
    assert native_lib.rt_submit_frames(None, 8, 3) == N.RT_E_INVALID
    assert native_lib.rt_synchronize(None) == N.RT_E_INVALID
    z = ctypes.c_uint32()
    assert native_lib.rt_debug_check_leaf_certificates(None, z, z, z) == N.RT_E_INVALID
    native_lib.rt_destroy(None)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(N.NativeLibraryError):
        N.load_library(tmp_path / "nope.so")


def _multi(native_lib, info, devices):
    devs = (ctypes.c_int32 * max(len(devices), 1))(*devices)
    g = ctypes.c_void_p()
    rc = native_lib.rt_create_multi(ctypes.byref(info) if info is not None else None, devs,
                                    len(devices), ctypes.byref(g))
    return rc, g


def test_create_multi_validates_arguments_without_device(native_lib):
    """rt_create_multi (rt_multi.cpp): argument checks come before any device or RCCL
    call, with the reason in rt_last_error(NULL); a valid request on a machine with
    no GPU is RT_E_NODEVICE. No group is returned on failure."""
    info = N.rt_create_info()
    info.width, info.height = 16, 8
    rc, g = _multi(native_lib, None, [0])
    assert rc == N.RT_E_INVALID and not g.value
    rc, g = _multi(native_lib, info, [])
    assert rc == N.RT_E_INVALID and not g.value and b"n_devices" in native_lib.rt_last_error(None)
    rc, g = _multi(native_lib, info, [0, 1, 0])
    assert rc == N.RT_E_INVALID and not g.value and b"twice" in native_lib.rt_last_error(None)
    info.world_size, info.rank = 2, 1
    rc, g = _multi(native_lib, info, [0, 1])
    assert rc == N.RT_E_INVALID and not g.value and b"whole frame" in native_lib.rt_last_error(None)
    info.world_size, info.rank = 1, 0
    rc, g = _multi(native_lib, info, [0])
    assert rc in (N.RT_E_NODEVICE, N.RT_OK)  # no GPU in the CPU suite: NODEVICE
    if rc == N.RT_OK:  # pragma: no cover - a box with a GPU
        native_lib.rt_destroy_multi(g)


def test_null_group_calls_fail_cleanly(native_lib):
    assert native_lib.rt_group_compute_frame(None, 8) == N.RT_E_INVALID
    assert native_lib.rt_group_synchronize(None) == N.RT_E_INVALID
    assert native_lib.rt_gather_frame(None, 0, 0) == N.RT_E_INVALID
    assert native_lib.rt_group_size(None) == 0
    assert native_lib.rt_group_context(None, 0) is None
    native_lib.rt_destroy_multi(None)


def test_create_multi_ex_flags_without_device(native_lib):
    """rt_create_multi_ex: unknown flags are refused; with RT_GROUP_COPY_TRANSPORT a device may
    repeat (several ranks on one GPU), so [0, 0, 0] passes the argument checks and, with no GPU
    in the CPU suite, stops at RT_E_NODEVICE instead of the "listed twice" refusal."""
    info = N.rt_create_info()
    info.width, info.height = 16, 8
    devs = (ctypes.c_int32 * 3)(0, 0, 0)
    g = ctypes.c_void_p()
    rc = native_lib.rt_create_multi_ex(ctypes.byref(info), devs, 3, 0x80, ctypes.byref(g))
    assert rc == N.RT_E_INVALID and not g.value and b"flags" in native_lib.rt_last_error(None)
    rc = native_lib.rt_create_multi_ex(ctypes.byref(info), devs, 3, 0, ctypes.byref(g))
    assert rc == N.RT_E_INVALID and b"twice" in native_lib.rt_last_error(None)
    rc = native_lib.rt_create_multi_ex(ctypes.byref(info), devs, 3, N.RT_GROUP_COPY_TRANSPORT, ctypes.byref(g))
    assert rc in (N.RT_E_NODEVICE, N.RT_OK)
    if rc == N.RT_OK:  # pragma: no cover - a box with a GPU
        native_lib.rt_destroy_multi(g)


def test_header_constants_match_binding():
    text = HEADER.read_text()
    assert re.search(r"#define RT_DEFAULT_FRAME_BATCH (\d+)", text).group(1) == str(N.RT_DEFAULT_FRAME_BATCH)
    assert re.search(r"#define RT_GROUP_COPY_TRANSPORT (\d+)u", text).group(1) == str(N.RT_GROUP_COPY_TRANSPORT)
    for name in ("PATH", "PRIMARY", "RESOLVE", "BRUTE", "BRUTE_STREAM"):
        assert re.search(rf"#define RT_PASS_{name} (\d+)u", text).group(1) == str(getattr(N, f"RT_PASS_{name}"))
