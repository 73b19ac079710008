"""Replay a real frame's rays through the triangle-walk harness (analysis tool, CPU only).

Renders a sample of a BASELINE configuration's pixels with the CPU oracle (trace log on),
dumps the scene's object / sub-object / triangle records and every traced ray, and runs
tests/cpp/tri_exactness on them: every walk (binary, quantized, octant layouts with the
relative slack, leaf certificates, the kernel's default) checked ray by ray against the
reference's sweep, with node visits and triangle tests per ray.

usage: python tools/tri_replay.py [config] [stride] [extra env VAR=VAL ...]
       (default c5_heightfield, every 997th pixel)
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from oracle.oracle import Oracle, lib  # noqa: E402  (analysis tool: the oracle is the ray source)
from rust_gpu_raytracing_amd.scene import build_config  # noqa: E402


def harness(out: Path) -> Path:
    csrc = ROOT / "rust_gpu_raytracing_amd" / "csrc"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", f"-I{ROOT / 'include'}", f"-I{csrc}",
                    str(ROOT / "tests" / "cpp" / "tri_exactness.cpp"), str(csrc / "sphere_bvh.cpp"), "-o", str(out)],
                   check=True)
    return out


def main() -> None:
    name = sys.argv[1] if len(sys.argv) > 1 else "c5_heightfield"
    stride = int(sys.argv[2]) if len(sys.argv) > 2 else 997
    env = dict(os.environ)
    for kv in sys.argv[3:]:
        k, v = kv.split("=", 1)
        env[k] = v
    scene, bounces = build_config(name)
    o = Oracle(scene)
    pixels = np.arange(0, o.width * o.height, stride, dtype=np.uint32)
    cap = len(pixels) * (bounces + 1)
    log = np.zeros((cap, 6), np.float32)
    lib().oracle_set_trace_log(log.ctypes.data, cap)
    p = scene.params(accumulate=1, compute_per_frame=1, accumulation_index=1)
    _, _, rays = o.render_pixels(p, bounces, pixels, threads=8)
    n = int(lib().oracle_trace_log_count())
    lib().oracle_set_trace_log(None, 0)
    objs, subs, tris = scene.flatten()
    with tempfile.TemporaryDirectory() as td:
        t = Path(td)
        for key, arr in (("o", objs), ("s", subs), ("t", tris), ("r", log[:n])):
            np.ascontiguousarray(arr).tofile(t / f"{key}.bin")
        exe = harness(t / "tri_exactness")
        out = subprocess.run([str(exe)] + [str(t / f"{k}.bin") for k in "ostr"], capture_output=True, text=True,
                             env=env)
    print(f"{name}: {len(pixels)} pixels, {n} rays (rc {out.returncode})")
    print(out.stdout, out.stderr, sep="")


if __name__ == "__main__":
    main()
