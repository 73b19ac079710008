"""Wall time of one timed batch launch against its device-clock span (analysis tool).

usage: python tools/launch_gap.py lib_a.so [lib_b.so ...] [--config c2_rtiow] [--reps 15] [--frames 20]
For each build, `reps` times: synchronize, submit `frames` frames (one launch), synchronize --
the bench's timed region -- and the launch's device span (rt_set_timing: path kernel + resolve).
The difference is what the host and the launch path add to a bench step.
"""
import argparse
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from rust_gpu_raytracing_amd import Renderer, _native as N  # noqa: E402
from rust_gpu_raytracing_amd.scene import build_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--config", default="c2_rtiow")
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--frames", type=int, default=20)
    args = ap.parse_args()
    scene, bounces = build_config(args.config)
    rays = scene.camera.recalculate_ray_directions()
    rs = [Renderer(scene, camera_rays=rays, lib=N.load_library(Path(p).resolve()), frame_batch=args.frames)
          for p in args.libs]
    for r in rs:  # warm up and settle the clocks
        for _ in range(20 * args.frames):
            r.compute_frame(bounces)
        r.synchronize()
    walls = {p: [] for p in args.libs}
    spans = {p: [] for p in args.libs}
    for _ in range(args.reps):
        for p, r in zip(args.libs, rs):
            r.reset_timing()
            r.set_timing(True)
            r.synchronize()
            t0 = time.perf_counter()
            r.submit_frames(bounces, args.frames)
            r.synchronize()
            walls[p].append((time.perf_counter() - t0) * 1e3)
            r.set_timing(False)
            ms, n = r.dispatch_time_total()
            rms, _ = r.resolve_time_total()
            spans[p].append(ms + rms)
    for p in args.libs:
        w, s = statistics.median(walls[p]), statistics.median(spans[p])
        print(json.dumps({"lib": Path(p).name, "wall_ms": round(w, 4), "span_ms": round(s, 4), "gap_ms": round(w - s, 4),
                          "wall_min_ms": round(min(walls[p]), 4)}))
    for r in rs:
        r.close()


if __name__ == "__main__":
    main()
