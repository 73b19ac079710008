"""Interleaved A/B timing of several builds of librt_pathtrace.so in ONE process.

usage: python tools/ab_bench.py lib_a.so lib_b.so ... [--config c2_rtiow] [--rounds 5] [--frames 10]
Each round times `frames` frames of every build (HIP events around each launch)
in turn; prints per-build median/min kernel ms and Mray/s, and checks that all
builds produce bit-identical accumulations.
"""
import argparse
import json
import statistics
import time
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from rust_gpu_raytracing_amd import Renderer, _native as N  # noqa: E402
from rust_gpu_raytracing_amd.scene import build_config  # noqa: E402


def launch_of(r):
    try:
        return r.launch_config()
    except AttributeError:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--config", default="c2_rtiow")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--tune", nargs="*", default=[], help="key=v rt_set_tuning settings for every build (before its own)")
    ap.add_argument("--device-rays", action="store_true", help="generate primary rays on the device")
    ap.add_argument("--frame-batch", type=int, default=8, help="rt_set_frame_batch (frames is rounded to a multiple)")
    ap.add_argument("--world", type=int, default=1, help="time rank --rank's share of an N-way tile split")
    ap.add_argument("--rank", type=int, default=0)
    args = ap.parse_args()
    scene, bounces = build_config(args.config, width=args.width, height=args.height)
    rays_dirs = scene.camera.recalculate_ray_directions()
    rs = []
    for spec in args.libs:
        # "path.so" or "path.so:key=v,key2=v": rt_set_tuning settings of that build's context
        p, _, knobs = spec.partition(":")
        tuning = {k: int(v) for k, v in (kv.split("=", 1) for kv in [*args.tune, *filter(None, knobs.split(","))])}
        lib = N.load_library(Path(p).resolve())
        kw = dict(lib=lib, frame_batch=args.frame_batch, rank=args.rank, world_size=args.world)
        if tuning:  # (older builds predate rt_set_tuning: pass none to them)
            kw["tuning"] = tuning
        if args.device_rays:
            rs.append(Renderer(scene, device_rays=True, **kw))
        else:
            rs.append(Renderer(scene, camera_rays=rays_dirs, **kw))
    args.frames = max(1, args.frames // args.frame_batch) * args.frame_batch
    for r in rs:  # warmup
        for _ in range(args.frame_batch):
            r.compute_frame(bounces)
        r.synchronize()
    times = {p: [] for p in args.libs}
    walls = {p: [] for p in args.libs}
    rays = {}
    for _ in range(args.rounds):
        for p, r in zip(args.libs, rs):
            r.reset_timing()
            r.reset_ray_count()
            r.set_timing(True)
            r.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.frames):
                r.compute_frame(bounces)
            r.synchronize()
            walls[p].append((time.perf_counter() - t0) * 1e3 / args.frames)
            r.set_timing(False)
            ms, n = r.dispatch_time_total()
            times[p].append(ms / args.frames)  # kernel time per frame (a launch renders a batch)
            rays[p] = r.ray_count() / args.frames
    ref = rs[0].read_accumulation().view(np.uint32)
    same = [bool(np.array_equal(r.read_accumulation().view(np.uint32), ref)) for r in rs]
    out = []
    for (p, t), s in zip(times.items(), same):
        med = statistics.median(t)
        out.append({"lib": Path(p).name, "median_ms": round(med, 4), "min_ms": round(min(t), 4),
                    "wall_ms": round(statistics.median(walls[p]), 4),
                    "mray_s": round(rays[p] / med / 1e3, 1), "bit_identical_to_first": s,
                    "launch": launch_of(rs[list(times).index(p)])})
    print(json.dumps({"config": args.config, "bounces": bounces, "results": out}, indent=1))
    for r in rs:
        r.close()


if __name__ == "__main__":
    main()
