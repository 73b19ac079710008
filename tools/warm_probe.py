"""Per-launch time of consecutive 20-frame launches after a short warmup (analysis tool).

usage: python tools/warm_probe.py [--warmup 5] [--launches 8] [--config c2_rtiow]
Prints, per launch, the device-clock span and the host wall time: shows how long the
GPU takes to reach its steady per-frame rate after the process starts rendering.
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from rust_gpu_raytracing_amd import Renderer  # noqa: E402
from rust_gpu_raytracing_amd.scene import build_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2_rtiow")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--launches", type=int, default=8)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--gap-ms", type=float, default=0.0, help="host sleep between launches")
    args = ap.parse_args()
    scene, bounces = build_config(args.config, width=1920, height=1080)
    r = Renderer(scene, frame_batch=args.frames)
    t0 = time.perf_counter()
    for _ in range(args.warmup):
        r.compute_frame(bounces)
    r.synchronize()
    out = {"config": args.config, "warmup": args.warmup, "warmup_ms": (time.perf_counter() - t0) * 1e3, "launches": []}
    for i in range(args.launches):
        if args.gap_ms:
            time.sleep(args.gap_ms / 1e3)
        r.reset_timing()
        r.set_timing(True)
        r.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.frames):
            r.compute_frame(bounces)
        r.synchronize()
        wall = (time.perf_counter() - t1) * 1e3
        r.set_timing(False)
        ms, n = r.dispatch_time_total()
        out["launches"].append({"i": i, "span_ms": round(ms, 4), "wall_ms": round(wall, 4)})
    print(json.dumps(out))
    r.close()


if __name__ == "__main__":
    main()
