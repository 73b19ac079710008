"""Measure every BASELINE.json configuration on one GPU (+ the CPU oracle on a sample).

usage: python tools/bench_all.py [--frames 10] [--configs c1_four_spheres c2_rtiow ...] [--cpu-seconds 8]
Prints one JSON object per config: GPU Mray/s (wall time of the timed frames; the
device-clock span of each launch is reported too),
rays per frame, algorithmic HBM bytes per launch and fraction of 8 TB/s, and the
CPU oracle's Mray/s on a tile sample of the same frame.
C4 is the 8-GPU configuration; here it runs whole on one GPU (the per-GPU share is
1/8 of it).
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import bench  # noqa: E402
from rust_gpu_raytracing_amd import Renderer  # noqa: E402
from rust_gpu_raytracing_amd.scene import CONFIGS, build_config  # noqa: E402

SIZES = {  # BASELINE.json configs
    "c1_four_spheres": (800, 600),
    "c2_rtiow": (1920, 1080),
    "c3_chess": (1920, 1080),
    "c4_mixed": (3840, 2160),
    "c5_heightfield": (1920, 1080),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="*", default=list(CONFIGS))
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-seconds", type=float, default=6.0)
    ap.add_argument("--settle-ms", type=float, default=150.0, help="as bench.py --settle-ms")
    ap.add_argument("--cpu-sample-world", type=int, default=64)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--kw", default="{}", help="JSON builder kwargs applied to every config, e.g. '{\"env_size\": [1024, 512]}'")
    ap.add_argument("--size", default=None, help="WxH override")
    ap.add_argument("--frame-batch", type=int, default=0,
                    help="rt_set_frame_batch (frames per launch at most); 0 = bench.default_frame_batch(1, frames)")
    args = ap.parse_args()
    for name in args.configs:
        w, h = SIZES[name] if args.size is None else map(int, args.size.split("x"))
        t0 = time.perf_counter()
        scene, bounces = build_config(name, width=w, height=h, **json.loads(args.kw))
        t_build = time.perf_counter() - t0
        fb = args.frame_batch or bench.default_frame_batch(1, args.frames)
        with Renderer(scene, frame_batch=fb) as r:
            for _ in range(args.warmup):
                r.compute_frame(bounces)
            r.synchronize()
            t_settle = time.perf_counter()  # as bench.py: untimed frames until the clocks settle
            while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
                for _ in range(fb):
                    r.compute_frame(bounces)
                r.synchronize()
            r.reset_ray_count()
            r.reset_timing()
            r.set_timing(True)
            t0 = time.perf_counter()
            for _ in range(args.frames):
                r.compute_frame(bounces)
            r.synchronize()
            wall = time.perf_counter() - t0
            r.set_timing(False)
            ms, n = r.dispatch_time_total()
            rays = r.ray_count()
            launch = r.launch_config()
        # per frame: wall time of the timed frames (batches overlap on two streams, so the
        # sum of the launches' device spans exceeds it); spans reported per launch
        kern_s = wall / args.frames
        span_ms = ms / max(n, 1)
        rpf = rays / args.frames
        fpl = args.frames / max(n, 1)  # frames per launch
        b = bench.algorithmic_bytes(w * h, rpf * fpl, bench.scene_bytes(scene), fpl) / fpl  # per frame
        res = {
            "config": name, "width": w, "height": h, "bounces": bounces,
            "spheres": int(scene.spheres.shape[0]), "triangles": int(scene.flatten()[2].shape[0]),
            "gpu_mray_s": rpf / kern_s / 1e6, "gpu_mray_s_wall": rays / wall / 1e6,
            "ms_per_frame": kern_s * 1e3, "kernel_span_ms_per_launch": span_ms, "launches": n, "frame_batch": fb, "rays_per_frame": rpf, "nominal_rays_per_frame": w * h * bounces,
            "hbm_bytes_per_frame": b, "hbm_frac": b / kern_s / 8e12, "launch": launch,
            "scene_build_s": round(t_build, 2),
        }
        if not args.no_cpu:
            res["cpu"] = bench.cpu_baseline(scene, bounces, args.cpu_seconds, args.cpu_sample_world)
            res["gpu_over_cpu"] = res["gpu_mray_s"] / res["cpu"]["value"]
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
