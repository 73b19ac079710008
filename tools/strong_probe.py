"""Predict the strong-scaling curve of bench.py from one GPU.

On an N-GPU node every rank renders only its own 8x8 tiles (tile t -> rank t % N)
with no communication until the final gather, so a rank's timed loop on its own
GPU is the same program whether or not the other ranks exist. This tool runs
each rank's share of the bench workload alone on the one GPU of the box, in
turn, with the bench's settings (bench.default_frame_batch(N, steps), same steps), and reports per N:
the slowest rank's render time per frame, the predicted whole-job Mray/s (all
ranks' rays / the slowest rank's time, as bench.py computes `value`), and the
predicted parallel efficiency against N=1 without and with a measured estimate
of the gather (pack + unpack + the bytes rank 0 receives, priced at --link-gbs,
+ 2 x 50 us of collective latency), for the payload bench.py gathers (--gather).

usage: python tools/strong_probe.py [--steps 20] [--warmup 3] [--settle-ms 150] [--ns 1 2 4 8]
"""
import argparse
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import bench  # noqa: E402
from rust_gpu_raytracing_amd import Renderer  # noqa: E402
from rust_gpu_raytracing_amd.scene import build_config  # noqa: E402


def time_rank(scene, bounces, rank, world, steps, warmup, fb, settle_ms, what="image", tuning=None):
    import torch

    with Renderer(scene, rank=rank, world_size=world, frame_batch=fb, tuning=tuning or {}) as r:
        for _ in range(warmup):
            r.compute_frame(bounces)
        r.synchronize()
        t_settle = time.perf_counter()  # as bench.py: untimed frames until the clocks settle
        while (time.perf_counter() - t_settle) * 1e3 < settle_ms:
            for _ in range(fb):
                r.compute_frame(bounces)
            r.synchronize()
        r.reset_ray_count()
        r.reset_timing()
        r.set_timing(True)
        t0 = time.perf_counter()
        done = 0
        while done < steps:  # as bench.py: a launch's worth of compute_frame calls per rt_submit_frames
            n = min(fb, steps - done)
            r.submit_frames(bounces, n)
            done += n
        t_submit = time.perf_counter() - t0
        r.synchronize()
        t = time.perf_counter() - t0
        r.set_timing(False)
        span_ms, n_launch = r.dispatch_time_total()
        rays = r.ray_count()
        launch = r.launch_config()
        # the device half of the gather: pack this rank's share (the bench's payload: the RGBA8
        # image, 4 B/px, or the accumulation, 16 B/px), averaged over 20 back-to-back packs so the
        # host round trip of one synchronize does not count as pack time
        n = r.owned_pixel_count()
        words = 4 if what == "accumulation" else 1
        buf = torch.empty((n, words), dtype=torch.float32 if words == 4 else torch.int32, device="cuda")
        pack = r.pack_owned_accumulation if what == "accumulation" else r.pack_owned_output
        pack(buf.data_ptr())
        r.synchronize()
        p0 = time.perf_counter()
        for _ in range(20):
            pack(buf.data_ptr())
        r.synchronize()
        t_pack = (time.perf_counter() - p0) / 20
    return t, rays, t_pack, n * 4 * words, t_submit, span_ms, n_launch, launch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2_rtiow")
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--ns", type=int, nargs="*", default=[1, 2, 4, 8])
    ap.add_argument("--settle-ms", type=float, default=150.0, help="as bench.py --settle-ms")
    ap.add_argument("--frame-batch", type=int, default=0, help="override bench.default_frame_batch(N)")
    ap.add_argument("--tune", nargs="*", default=[], help="key=value rt_set_tuning settings of every rank's context")
    ap.add_argument("--repeats", type=int, default=3, help="timed runs per rank (the median is used)")
    ap.add_argument("--gather", choices=["image", "accumulation"], default="image",
                    help="the gather payload priced (bench.py --gather; default image, 4 B/px)")
    ap.add_argument("--link-gbs", type=float, default=50.0,
                    help="xGMI bandwidth one peer achieves into rank 0 (GB/s, per link; 7 links)")
    args = ap.parse_args()
    tuning = {k: int(v) for k, v in (kv.split("=", 1) for kv in args.tune)}
    scene, bounces = build_config(args.config)
    base = None
    for n in args.ns:
        fb = args.frame_batch or bench.default_frame_batch(n, args.steps)
        per = []
        for r in range(n):
            # the median of --repeats timed runs per rank (one 20-frame run is under 1 ms at N=8:
            # a single launch-latency hiccup would move it by several percent)
            runs = sorted((time_rank(scene, bounces, r, n, args.steps, args.warmup, fb, args.settle_ms, args.gather, tuning)
                           for _ in range(args.repeats)), key=lambda x: x[0])
            per.append(runs[len(runs) // 2])
        t_max = max(p[0] for p in per)
        rays = sum(p[1] for p in per)
        # gather estimate: packs run in parallel (max), rank 0 receives N-1 blocks over N-1 links
        # (pack on every rank, then rank 0's unpack of about as many bytes: priced as a second pack)
        t_gather = (2 * max(p[2] for p in per) + (max(p[3] for p in per) / (args.link_gbs * 1e9)) + 2 * 50e-6) if n > 1 else 0.0
        v = rays / t_max / 1e6
        vg = rays / (t_max + t_gather) / 1e6
        if base is None:
            base = v
        print(json.dumps({
            "n": n, "frame_batch": fb, "ms_per_frame_slowest_rank": t_max / args.steps * 1e3,
            "ms_per_frame_per_rank": [round(p[0] / args.steps * 1e3, 4) for p in per],
            "pred_mray_s": v, "pred_eff": v / (n * base),
            "gather_est_ms": t_gather * 1e3, "pred_mray_s_with_gather": vg, "pred_eff_with_gather": vg / (n * base),
            "host_submit_ms_max": max(p[4] for p in per) * 1e3,
            "kernel_span_ms_per_rank": [round(p[5], 4) for p in per], "launches": per[0][6],
            "wall_ms_per_rank": [round(p[0] * 1e3, 4) for p in per],
            "steps": args.steps, "launch": per[0][7], "gather_payload": args.gather,
            "pack_ms_max": max(p[2] for p in per) * 1e3,
            "rays_per_rank": [p[1] for p in per], "repeats": args.repeats,
        }), flush=True)


if __name__ == "__main__":
    main()
