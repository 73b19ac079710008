"""Python handle on the CPU oracle (oracle/pathtrace_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg — never by the product package. Parity against the
reference itself is UNPINNED (see the header of pathtrace_oracle.c).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
SRC = HERE / "pathtrace_oracle.c"
LIB = HERE / "build" / "liboracle.so"

CFLAGS = ["-O2", "-ffp-contract=off", "-fno-fast-math", "-fopenmp", "-fPIC", "-shared", "-std=c11", "-Wall"]


# bench.py's cpu_baseline leg times a build tuned for the host it runs on (SURVEY §8d:
# -O3 -march=native); same IEEE semantics (no FMA contraction, no fast-math), so the
# same results bit for bit -- cpu_baseline checks that on a crop before timing.
BASELINE_CFLAGS = ["-O3", "-march=native", *CFLAGS[1:]]


def build_baseline() -> Path:
    """Compile the -O3 -march=native variant on this host (not shipped: built where it runs)."""
    out = HERE / "build" / f"liboracle_native.{os.getpid()}.so"
    out.parent.mkdir(parents=True, exist_ok=True)
    subprocess.run(["gcc", *BASELINE_CFLAGS, "-o", str(out), str(SRC), "-lm"], check=True)
    return out


def use_library(path: Path) -> None:
    """Make lib() (and every Oracle) use the oracle built at ``path`` from here on."""
    global _lib
    _lib = None
    lib(path)


def build(force: bool = False) -> Path:
    """Compile the oracle with gcc (strict IEEE: no FMA contraction, no fast-math)."""
    if LIB.exists() and not force and LIB.stat().st_mtime >= SRC.stat().st_mtime:
        return LIB
    LIB.parent.mkdir(parents=True, exist_ok=True)
    tmp = LIB.with_suffix(f".{os.getpid()}.tmp")
    subprocess.run(["gcc", *CFLAGS, "-o", str(tmp), str(SRC), "-lm"], check=True)
    os.replace(tmp, LIB)
    return LIB


class OScene(ctypes.Structure):
    _fields_ = [
        ("camera_origin", ctypes.c_void_p),
        ("camera_rays", ctypes.c_void_p),
        ("materials", ctypes.c_void_p), ("material_count", ctypes.c_uint32),
        ("spheres", ctypes.c_void_p), ("sphere_capacity", ctypes.c_uint32),
        ("triangles", ctypes.c_void_p), ("triangle_count", ctypes.c_uint32),
        ("objects", ctypes.c_void_p), ("object_capacity", ctypes.c_uint32),
        ("subs", ctypes.c_void_p), ("sub_count", ctypes.c_uint32),
        ("textures", ctypes.c_void_p), ("tex_w", ctypes.c_uint32), ("tex_h", ctypes.c_uint32),
        ("tex_layers", ctypes.c_uint32),
        ("env", ctypes.c_void_p), ("env_w", ctypes.c_uint32), ("env_h", ctypes.c_uint32),
    ]


class OHitOut(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in ("t", "px", "py", "pz", "nx", "ny", "nz", "u", "v")] + [
        ("material_index", ctypes.c_uint32), ("front_face", ctypes.c_int32)]


_lib = None


def lib(path: Path | None = None) -> ctypes.CDLL:
    global _lib
    if _lib is None:
        L = ctypes.CDLL(str(path or build()))
        for n in ("oracle_logf", "oracle_cosf", "oracle_asinf", "oracle_acosf", "oracle_atanf"):
            getattr(L, n).restype = ctypes.c_float
            getattr(L, n).argtypes = [ctypes.c_float]
        L.oracle_atan2f.restype = ctypes.c_float
        L.oracle_atan2f.argtypes = [ctypes.c_float, ctypes.c_float]
        L.oracle_random.restype = ctypes.c_float
        L.oracle_random.argtypes = [ctypes.POINTER(ctypes.c_uint32)]
        L.oracle_pack.restype = ctypes.c_uint32
        L.oracle_pack.argtypes = [ctypes.POINTER(ctypes.c_float)]
        L.oracle_srgb_table.restype = None
        L.oracle_srgb_table.argtypes = [ctypes.POINTER(ctypes.c_float)]
        L.oracle_trace.restype = None
        L.oracle_trace.argtypes = [ctypes.POINTER(OScene), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                   ctypes.POINTER(OHitOut)]
        L.oracle_render_frame.restype = ctypes.c_uint64
        L.oracle_render_frame.argtypes = [ctypes.POINTER(OScene), ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_int]
        L.oracle_render_pixels.restype = ctypes.c_uint64
        L.oracle_render_pixels.argtypes = [ctypes.POINTER(OScene), ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                           ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oracle_num_threads.restype = ctypes.c_int
        L.oracle_set_trace_log.restype = None
        L.oracle_set_trace_log.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.oracle_trace_log_count.restype = ctypes.c_uint64
        _lib = L
    return _lib


def _p(a):
    return None if a is None or a.size == 0 else a.ctypes.data


class Oracle:
    """Holds one scene's arrays (the 12 bindings of compute_shader.wgsl:12-23) for the C oracle."""

    def __init__(self, scene, camera_rays=None):
        self.scene = scene
        objs, subs, tris = scene.flatten()
        rays = scene.camera.recalculate_ray_directions() if camera_rays is None else camera_rays
        self.width = scene.camera.viewport_width
        self.height = scene.camera.viewport_height
        self._arrays = dict(
            origin=np.ascontiguousarray(scene.camera.position, np.float32),
            rays=np.ascontiguousarray(rays),
            mats=np.ascontiguousarray(scene.materials),
            sph=np.ascontiguousarray(scene.spheres),
            tris=tris, objs=objs, subs=subs,
            tex=np.ascontiguousarray(scene.textures, np.uint8),
            env=np.ascontiguousarray(scene.environment_map, np.uint8),
        )
        a = self._arrays
        s = OScene()
        s.camera_origin = _p(a["origin"])
        s.camera_rays = _p(a["rays"])
        s.materials, s.material_count = _p(a["mats"]), a["mats"].shape[0]
        s.spheres, s.sphere_capacity = _p(a["sph"]), a["sph"].shape[0]
        s.triangles, s.triangle_count = _p(tris), tris.shape[0]
        s.objects, s.object_capacity = _p(objs), objs.shape[0]
        s.subs, s.sub_count = _p(subs), subs.shape[0]
        s.textures = _p(a["tex"])
        s.tex_layers, s.tex_h, s.tex_w = a["tex"].shape[:3]
        s.env = _p(a["env"])
        s.env_h, s.env_w = a["env"].shape[:2]
        self._s = s

    def render_frame(self, params, bounces, accum, out, rank=0, world_size=1, threads=0) -> int:
        """One dispatch (compute_shader.wgsl:146-189) over the pixels this rank owns.
        ``accum`` (H, W, 4) f32 and ``out`` (H, W) u32 are updated in place."""
        assert accum.dtype == np.float32 and accum.flags["C_CONTIGUOUS"]
        assert out.dtype == np.uint32 and out.flags["C_CONTIGUOUS"]
        p = np.ascontiguousarray(params)
        return int(lib().oracle_render_frame(ctypes.byref(self._s), p.ctypes.data, self.height, bounces, rank,
                                             world_size, accum.ctypes.data, out.ctypes.data, threads))

    def render_pixels(self, params, bounces, pixels, accum_in=None, threads=0):
        """Shade an explicit list of pixel indices; returns (accum (n,4), out (n,), rays)."""
        pixels = np.ascontiguousarray(pixels, np.uint32)
        n = pixels.shape[0]
        acc = np.zeros((n, 4), np.float32) if accum_in is None else np.ascontiguousarray(accum_in, np.float32).copy()
        out = np.zeros(n, np.uint32)
        p = np.ascontiguousarray(params)
        rays = int(lib().oracle_render_pixels(ctypes.byref(self._s), p.ctypes.data, bounces, pixels.ctypes.data, n,
                                              acc.ctypes.data, out.ctypes.data, threads))
        return acc, out, rays

    def trace(self, params, origin, direction) -> OHitOut:
        h = OHitOut()
        o = np.ascontiguousarray(origin, np.float32)
        d = np.ascontiguousarray(direction, np.float32)
        p = np.ascontiguousarray(params)
        lib().oracle_trace(ctypes.byref(self._s), p.ctypes.data, o.ctypes.data, d.ctypes.data, ctypes.byref(h))
        return h


def render_frames(scene, bounces, frames, *, compute_per_frame=1, accumulate=1, rank=0, world_size=1, threads=0):
    """Render `frames` frames the way Renderer::compute_frame sequences them
    (k = 1, 2, ...; src/renderer.rs:216-234). Returns (accum, out, rays)."""
    o = Oracle(scene)
    accum = np.zeros((o.height, o.width, 4), np.float32)
    out = np.zeros((o.height, o.width), np.uint32)
    rays = 0
    for k in range(1, frames + 1):
        p = scene.params(accumulate=accumulate, compute_per_frame=compute_per_frame, accumulation_index=k)
        rays += o.render_frame(p, bounces, accum, out, rank=rank, world_size=world_size, threads=threads)
    return accum, out, rays
