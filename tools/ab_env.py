"""Interleaved A/B of ONE build under different per-context tunings (rt_set_tuning).

usage: python tools/ab_env.py "block_threads=256" "block_threads=512 leaf_batch=4" ... [--config ...]
Each spec is a space-separated list of KEY=VALUE tuning settings (include/rt_abi.h lists the
keys; "prune=N" calls rt_set_triangle_pruning) for that variant's context; "" is the default.
"""
import argparse
import json
import statistics
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from rust_gpu_raytracing_amd import Renderer  # noqa: E402
from rust_gpu_raytracing_amd.scene import build_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("specs", nargs="+")
    ap.add_argument("--config", default="c2_rtiow")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--frame-batch", type=int, default=1, help="frames per launch (rt_set_frame_batch)")
    ap.add_argument("--split", default="0/1", help="R/N: rank R's share of an N-way tile split (the strong bench)")
    args = ap.parse_args()
    scene, bounces = build_config(args.config, width=args.width, height=args.height)
    dirs = scene.camera.recalculate_ray_directions()
    rs = []
    for spec in args.specs:
        tuning = {k: int(v) for k, v in (kv.split("=", 1) for kv in spec.split())}
        prune = tuning.pop("prune", None)
        rank, world = map(int, args.split.split("/"))
        r = Renderer(scene, camera_rays=dirs, frame_batch=args.frame_batch, rank=rank, world_size=world, tuning=tuning)
        if prune is not None:
            r.set_triangle_pruning(prune)
        rs.append(r)
    for r in rs:
        for _ in range(args.frame_batch):
            r.compute_frame(bounces)
        r.synchronize()
    times = {s: [] for s in args.specs}  # wall ms per frame: every kernel of the launches counts
    dev = {s: [] for s in args.specs}
    rays = {}
    for _ in range(args.rounds):
        for s, r in zip(args.specs, rs):
            r.reset_timing()
            r.reset_ray_count()
            r.set_timing(True)
            t0 = time.perf_counter()
            for _ in range(args.frames):
                r.compute_frame(bounces)
            r.synchronize()
            times[s].append((time.perf_counter() - t0) * 1e3 / args.frames)
            r.set_timing(False)
            ms, n = r.dispatch_time_total()
            rms, _ = r.resolve_time_total()
            # path kernel + resolve spans only (an auxiliary pass such as the primary
            # pre-pass is not in them: compare variants on the wall time)
            dev[s].append((ms + rms) / args.frames)
            rays[s] = r.ray_count() / args.frames
    ref = rs[0].read_accumulation().view(np.uint32)
    for (s, t), r in zip(times.items(), rs):
        med = statistics.median(t)
        print(json.dumps({"config": args.config, "split": args.split, "spec": s, "median_ms": round(med, 4), "min_ms": round(min(t), 4),
                          "path_kernel_ms": round(statistics.median(dev[s]), 4),
                          "mray_s": round(rays[s] / med / 1e3, 1),
                          "bit_identical_to_first": bool(np.array_equal(r.read_accumulation().view(np.uint32), ref)),
                          "launch": r.launch_config()}))
    for r in rs:
        r.close()


if __name__ == "__main__":
    main()
