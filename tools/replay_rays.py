"""Dump the rays of a real frame for traversal experiments (analysis tool, CPU only).

Renders a sample of a BASELINE configuration's pixels with the CPU oracle (one
thread, trace log on) and writes every traced ray (o, d as 6 f32) plus the
scene's spheres (rt_scene_sphere records) -- the inputs of
`tests/cpp/bvh_exactness --replay <rays> <spheres>`.

usage: python tools/replay_rays.py [config] [stride] [out_prefix]
       (default c2_rtiow, every 6th pixel, /tmp/replay_c2)
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from oracle.oracle import Oracle, lib  # noqa: E402  (analysis tool: the oracle is the ray source)
from rust_gpu_raytracing_amd.scene import build_config  # noqa: E402


def main() -> None:
    name = sys.argv[1] if len(sys.argv) > 1 else "c2_rtiow"
    stride = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    prefix = sys.argv[3] if len(sys.argv) > 3 else "/tmp/replay_c2"
    scene, bounces = build_config(name)
    o = Oracle(scene)
    pixels = np.arange(0, o.width * o.height, stride, dtype=np.uint32)
    cap = len(pixels) * (bounces + 1)
    log = np.zeros((cap, 6), np.float32)
    lib().oracle_set_trace_log(log.ctypes.data, cap)
    p = scene.params(accumulate=1, compute_per_frame=1, accumulation_index=1)
    _, _, rays = o.render_pixels(p, bounces, pixels, threads=1)
    n = int(lib().oracle_trace_log_count())
    lib().oracle_set_trace_log(None, 0)
    assert n == rays, (n, rays)
    log[:n].tofile(prefix + "_rays.bin")
    np.ascontiguousarray(scene.spheres).tofile(prefix + "_spheres.bin")
    print(f"{name}: {len(pixels)} pixels, {n} rays -> {prefix}_rays.bin, {len(scene.spheres)} spheres")


if __name__ == "__main__":
    main()
