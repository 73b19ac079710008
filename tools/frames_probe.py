"""Per-frame kernel time of single-frame launches vs fused multi-frame launches
(rt_compute_frames) on one GPU: how much of a launch is ramp and tail.

usage: python tools/frames_probe.py [--config c2_rtiow] [--fused 1 2 4 8]
"""
import argparse
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from rust_gpu_raytracing_amd import Renderer  # noqa: E402
from rust_gpu_raytracing_amd.scene import build_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2_rtiow")
    ap.add_argument("--fused", type=int, nargs="*", default=[1, 2, 4, 8])
    ap.add_argument("--frames", type=int, default=16)
    args = ap.parse_args()
    scene, bounces = build_config(args.config)
    with Renderer(scene) as r:
        r.compute_frame(bounces)
        r.synchronize()
        for f in args.fused:
            r.reset_timing()
            r.reset_ray_count()
            r.set_timing(True)
            for _ in range(args.frames // f):
                r.compute_frames(bounces, f)
            r.synchronize()
            r.set_timing(False)
            ms, n = r.dispatch_time_total()
            per_frame = ms / (n * f)
            rays = r.ray_count() / (n * f)
            print(json.dumps({"config": args.config, "fused": f, "ms_per_frame": round(per_frame, 4),
                              "mray_s": round(rays / per_frame / 1e3, 1), "env": {k: v for k, v in os.environ.items()
                                                                                  if k.startswith("RT_")}}))


if __name__ == "__main__":
    main()
