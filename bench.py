#!/usr/bin/env python3
"""Headline benchmark: Mray/s of the path-tracing kernel, 1920x1080, 8 bounces.

Workload (BASELINE.json configs[1]): the RTIOW cover scene (488 spheres),
1920x1080, 8 bounces, 1 sample per pixel per frame, accumulation on. One
"step" = one Renderer.compute_frame (one kernel launch over the frame). Inputs
are resident in HBM before timing; the timed region holds exactly `--steps`
frames bracketed by barrier + device synchronize.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
the 1920x1080 image is tile-split across ranks (8x8 tile t -> rank t % N,
SURVEY §8e). Default "--scaling weak": the same view rendered at N times the
pixels -- (1920*sqrt(N)) x (1080*sqrt(N)) rounded to whole 8x8 tiles (N=4 is
3840x2160) -- so every GPU owns one 1920x1080 frame's worth of tiles at every N
and each step is still one single-frame launch per GPU (one frame of the job's
image). "--scaling strong": the 1920x1080 frame split N ways (0.1 ms of work
per GPU at N=8). No collective runs in the timed loop; one RCCL gather of the
accumulated RGBA32F tiles to rank 0 runs afterwards and is reported separately
as gather_ms.

roofline.traffic: HBM bytes per launch from the committed rocprofv3 PMC summary
(profiles/pmc_traffic.json, FETCH_SIZE x2 per the gfx950 note + WRITE_SIZE), when
it was measured on this workload; null otherwise.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "Mray/s (primary+bounce) at 1920x1080, 8 bounces; 1/2/4/8-GPU scaling"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def algorithmic_bytes(owned_pixels: int, rays: float, scene_bytes: int, frames: float = 1.0) -> float:
    """SURVEY §8d, per launch: B = 52 B/px/frame (ray dir 16 + accum 16 read + 16 write +
    RGBA8 4) + 4 B per counted ray (one RGBA8 texel: texture on hit, env map on miss)
    + the scene arrays read once. A launch rendering F batched frames reads each
    pixel's accumulation once and keeps it in a register between its frames:
    16 + 36 F B/px (F = 1: the 52 B above)."""
    return (16.0 + 36.0 * frames) * owned_pixels + 4.0 * rays + scene_bytes


def scene_bytes(scene) -> int:
    objs, subs, tris = scene.flatten()
    return int(scene.spheres.nbytes + scene.materials.nbytes + objs.nbytes + subs.nbytes + tris.shape[0] * 64)


def pmc_traffic(workload: str):
    """HBM bytes per launch measured by rocprofv3 PMC for this workload (tools/profile.sh ->
    profiles/pmc_traffic.json), or None when no committed measurement matches."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    if not f.exists():
        return None, None
    d = json.loads(f.read_text())
    e = d.get(workload)
    if not e:
        return None, None
    return float(e["fetch_bytes_x2"] + e["write_bytes"]), e.get("source")


def pmc_issue(workload: str):
    """VALU issue and lane utilisation of the same committed PMC run (SQ counters): the
    resource this branchy f32 path is actually bound by, or None."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    e = json.loads(f.read_text()).get(workload) if f.exists() else None
    if not e or e.get("valu_issue_util") is None:
        return None
    return {"valu_issue_util": e["valu_issue_util"], "valu_lane_util": e["valu_lane_util"], "source": e.get("source")}


def cpu_baseline(scene, bounces, min_seconds: float, sample_world: int):
    """The CPU oracle (scalar C restatement, OpenMP over the host cores) on a bounded
    sample of the same workload: the tiles t % sample_world == 0, frames k = 1, 2, ...
    until min_seconds have elapsed."""
    from oracle import oracle as O

    O.build()
    o = O.Oracle(scene)
    threads = O.lib().oracle_num_threads()
    accum = np.zeros((o.height, o.width, 4), np.float32)
    out = np.zeros((o.height, o.width), np.uint32)
    rays = 0
    frames = 0
    t0 = time.perf_counter()
    while True:
        frames += 1
        p = scene.params(accumulation_index=frames)
        rays += o.render_frame(p, bounces, accum, out, rank=0, world_size=sample_world, threads=threads)
        el = time.perf_counter() - t0
        if el >= min_seconds or frames >= 512:
            break
    return {
        "value": rays / el / 1e6,
        "unit": "Mray/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"CPU oracle (oracle/pathtrace_oracle.c, -O2 scalar f32, OpenMP {threads} threads) on "
                   f"1/{sample_world} of the 8x8 tiles of the same {o.width}x{o.height} {bounces}-bounce frame, "
                   f"{frames} frame(s), {rays} rays in {el:.1f} s"),
    }


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2_rtiow")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--bounces", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-sample-world", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--frame-batch", type=int, default=int(os.environ.get("RT_FRAME_BATCH", "1")),
                    help="frames one launch may render (rt_set_frame_batch); 1 = one launch per frame")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="N>1: weak = N frames per step (1/N of the tiles each, per-GPU work fixed); "
                         "strong = one frame per step split N ways")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    assert torch.cuda.is_available(), "bench.py needs a HIP device"
    # RT_BENCH_ONE_DEVICE=1 + RT_DIST_BACKEND=gloo: rehearse the N-rank path with
    # every rank on GPU 0 (single-GPU test boxes); the real run is one rank per GPU
    # over RCCL (backend "nccl").
    device = 0 if os.environ.get("RT_BENCH_ONE_DEVICE") == "1" else local_rank
    backend = os.environ.get("RT_DIST_BACKEND", "nccl")
    torch.cuda.set_device(device)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)

    from rust_gpu_raytracing_amd import Renderer
    from rust_gpu_raytracing_amd import build as native_build
    from rust_gpu_raytracing_amd.scene import build_config

    if rank == 0:
        native_build.build(verbose=False)
    if world > 1:
        dist.barrier()

    width, height = args.width, args.height
    if world > 1 and args.scaling == "weak":
        scale = world ** 0.5  # same view, N x the pixels: per-GPU work fixed
        width = int(round(args.width * scale / 8.0)) * 8
        height = int(round(args.height * scale / 8.0)) * 8
    scene, default_bounces = build_config(args.config, width=width, height=height)
    bounces = args.bounces or default_bounces
    r = Renderer(scene, device=device, rank=rank, world_size=world, frame_batch=args.frame_batch)
    owned_px = r.owned_pixel_count()

    def step():
        r.compute_frame(bounces)

    def barrier_sync():
        r.synchronize()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    barrier_sync()
    r.reset_ray_count()
    r.reset_timing()
    r.set_timing(True)
    barrier_sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
        if rank == 0 and args.steps >= 50 and (i + 1) % 50 == 0:
            log(f"step {i + 1}/{args.steps}")
    barrier_sync()
    elapsed = time.perf_counter() - t0
    r.set_timing(False)
    launch = r.launch_config()
    rays = r.ray_count()
    kern_ms, n_timed = r.dispatch_time_total()

    stats = torch.tensor([elapsed, float(rays)], dtype=torch.float64,
                         device="cuda" if backend == "nccl" else "cpu")
    if world > 1:
        t_max = stats[0:1].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        tot = stats[1:2].clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed_max, rays_total = float(t_max.item()), float(tot.item())
    else:
        elapsed_max, rays_total = elapsed, float(rays)

    gather_ms = None
    if world > 1 and not args.no_gather:
        from rust_gpu_raytracing_amd.distributed import gather_accumulation

        barrier_sync()
        g0 = time.perf_counter()
        gather_accumulation(r, dst=0)
        barrier_sync()
        gather_ms = (time.perf_counter() - g0) * 1e3
        if os.environ.get("RT_BENCH_VERIFY_GATHER") == "1" and rank == 0:
            # the assembled tile-split image must equal a 1-GPU render of the same frames
            with Renderer(scene, device=device) as ref:
                for _ in range(args.warmup + args.steps):
                    ref.compute_frame(bounces)
                same = np.array_equal(ref.read_accumulation().view(np.uint32), r.read_accumulation().view(np.uint32))
                same = same and np.array_equal(ref.read_output(), r.read_output())
            log(f"gather verify: assembled image {'==' if same else '!='} 1-GPU render")
            if not same:
                return 3

    if rank == 0:
        avg_kernel_s = kern_ms / max(n_timed, 1) / 1e3
        frames_per_launch = args.steps / max(n_timed, 1)
        rays_per_launch = rays / max(n_timed, 1)
        b_launch = algorithmic_bytes(owned_px, rays_per_launch, scene_bytes(scene), frames_per_launch)
        achieved = b_launch / avg_kernel_s / 1e9
        workload = f"{args.config} {width}x{height}, {bounces} bounces, 1 spp/frame, accumulate"
        traffic, traffic_src = pmc_traffic(workload) if world == 1 else (None, None)
        result = {
            "metric": METRIC,
            "value": rays_total / elapsed_max / 1e6,
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if args.scaling == "weak" else "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": {
                "workload": workload,
                "width": width,
                "height": height,
                "bounces": bounces,
                "spheres": int(scene.spheres.shape[0]),
                "triangles": int(scene.flatten()[2].shape[0]),
                "parallelism": f"tile{world}" if world > 1 else "single",
                "pixels_per_gpu": owned_px,
                "rays_per_step": rays_total / args.steps,
                "nominal_rays_per_step": width * height * bounces,
                "frame_batch": args.frame_batch,
                "launches": n_timed,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": "rt_pathtrace_kernel",
                "kernel_ms_avg": avg_kernel_s * 1e3,
                "launch": launch,
                "bytes_per_launch": b_launch,
                "note": "branchy f32 VALU-bound path (SURVEY §7); HBM fraction is low by construction",
                "valu": pmc_issue(workload) if world == 1 else None,
            },
        }
        if gather_ms is not None:
            result["gather_ms"] = gather_ms
        if world == 1 and not args.no_cpu_baseline:
            log("cpu baseline ...")
            result["cpu_baseline"] = cpu_baseline(scene, bounces, args.cpu_seconds, args.cpu_sample_world)
        print(json.dumps(result), flush=True)
    r.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
