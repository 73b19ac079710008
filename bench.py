#!/usr/bin/env python3
"""Headline benchmark: Mray/s of the path-tracing kernel, 1920x1080, 8 bounces.

Workload (BASELINE.json configs[1]): the RTIOW cover scene (484 spheres),
1920x1080, 8 bounces, 1 sample per pixel per frame, accumulation on. One
"step" = one Renderer.compute_frame (one frame: every pixel traced, its
accumulation and RGBA8 output written). Frames are launched in batches of
--frame-batch (rt_set_frame_batch; default: the steps split evenly into launches
of at most 32N frames, default_frame_batch: the persistent grid's fill and drain
are paid once per launch; every frame is traced in full and added to the
accumulation in the reference's order). Inputs are resident in
HBM before timing; the timed region holds exactly `--steps` frames bracketed by
barrier + device synchronize.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
default "--scaling strong", the metric's config: the 1920x1080 frame is
tile-split across ranks (8x8 tile t -> rank t % N), launches of up
to 32N frames (a GPU's launch holds the units of an N=1 launch), and the timed region also
assembles the frame on rank 0 once (device pack -> RCCL gather -> unpack), so `value`
includes the gather (also reported as gather_ms). --gather accumulation (default, the
north star's "RCCL gather of the accumulated RGBA buffer") moves the RGBA32F accumulation
(16 B/px, the whole renderer state on rank 0, which rebuilds the RGBA8 output from it);
--gather image the displayed RGBA8 frame (4 B/px; accumulations stay sharded on their
owners). Both gathers are also timed alone after the timed region (gather_image_ms,
gather_accum_ms), and value_with_image_gather / value_with_accum_gather price the run
with either payload. A secondary "weak" object measures the same view at N x the pixels
((1920*sqrt(N)) x (1080*sqrt(N)) in whole tiles, one 1920x1080 frame's worth
of tiles per GPU). `value` = all ranks' rays / the slowest rank's time.

roofline: algorithmic bytes per launch (bench.algorithmic_bytes) /
the average launch span on the device clock (rt_set_timing: first workgroup start
to last workgroup end, what rocprofv3's kernel trace reports); consecutive batches
overlap on two streams, so `achieved_effective` also divides by the wall time per
launch. traffic and
valu: the committed rocprofv3 PMC entry (profiles/pmc_traffic.json, FETCH_SIZE x2
per the gfx950 note + WRITE_SIZE; SQ counters) of this workload, frame batch and
kernel build hash; null (with the reason, and a warning) when stale.

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
# f32 VALU lane peak for this path's scalar (non-packed, non-FMA-counted) code: 256 CUs x 4 SIMDs x
# 16 lanes x 2.4 GHz (a wave64 instruction issues over 4 cycles of a SIMD16)
VALU_LANE_PEAK_TOPS = 256 * 4 * 16 * 2.4e9 / 1e12
KERNEL_NAMES = {"path": "rt_pathtrace_kernel", "primary": "rt_primary_kernel", "resolve": "rt_resolve_frames_kernel",
                "brute": "rt_brute_wf_kernel", "brute_stream": "(its records through the scalar cache)"}
# The reference computes a frame every >= 0.8 ms and displays every >= 5 ms
# (src/main.rs:88-92, 365-375): about 6 computed frames per displayed image.
DISPLAY_CADENCE_FRAMES = 6


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def algorithmic_bytes(owned_pixels: int, rays: float, scene_bytes: int, frames: float = 1.0) -> float:
    """SURVEY §8d's per-frame figure x the frames one launch renders: B = 52 B/px/frame
    (ray dir 16 + accum 16 read + 16 write + RGBA8 4) + 4 B per counted ray (one RGBA8
    texel: texture on hit, env map on miss) + the scene arrays read once. (A batched
    launch moves less -- each pixel's accumulation once per batch, plus its lights:
    roofline.traffic is what the counters see.)"""
    return 52.0 * frames * owned_pixels + 4.0 * rays + scene_bytes


def scene_bytes(scene) -> int:
    objs, subs, tris = scene.flatten()
    return int(scene.spheres.nbytes + scene.materials.nbytes + objs.nbytes + subs.nbytes + tris.shape[0] * 64)


def pmc_entry(key: str, build_hash: str):
    """The committed rocprofv3 PMC measurement (tools/profile.sh -> tools/update_traffic.py ->
    profiles/pmc_traffic.json) of this workload AND this kernel build: (entry, None), or
    (None, reason) when there is none or it was measured on another build (stale)."""
    f = ROOT / "profiles" / "pmc_traffic.json"
    e = json.loads(f.read_text()).get(key) if f.exists() else None
    if not e:
        return None, f"no PMC entry for '{key}'"
    if e.get("build_hash") != build_hash:
        msg = f"PMC entry for '{key}' was measured on build {e.get('build_hash')}, this is {build_hash}: stale, not used"
        log("WARNING: " + msg)
        return None, msg
    return e, None


def pmc_traffic(e):
    """HBM bytes per launch: FETCH_SIZE x2 (gfx950 note) + WRITE_SIZE."""
    return None if e is None else float(e["fetch_bytes_x2"] + e["write_bytes"])


def pmc_issue(e):
    """VALU issue and lane utilisation of the same PMC run (SQ counters): the resource
    this branchy f32 path is actually bound by."""
    if e is None or e.get("valu_issue_util") is None:
        return None
    return {"valu_issue_util": e["valu_issue_util"], "valu_lane_util": e["valu_lane_util"], "source": e.get("source")}


def cpu_baseline(scene, bounces, min_seconds: float, sample_world: int):
    """The CPU oracle (scalar C restatement, OpenMP over the host cores) on a bounded
    sample of the same workload: the tiles t % sample_world == 0, frames k = 1, 2, ...
    until min_seconds have elapsed. SURVEY §8d also asks for a 1-thread figure: the
    same loop on one thread over 1/64 of the tiles, for a quarter of the time."""
    from oracle import oracle as O

    # the restatement at -O3 -march=native for this host; checked bit-identical to
    # the tests' -O2 build on a crop of the same frame before anything is timed
    O.build()
    crop = np.arange(0, scene.camera.viewport_width * scene.camera.viewport_height, 997, dtype=np.uint32)
    p1 = scene.params(accumulation_index=1)
    ref = O.Oracle(scene).render_pixels(p1, bounces, crop)
    native = O.build_baseline()
    O.use_library(native)
    native.unlink()  # loaded; the per-process build leaves nothing behind
    got = O.Oracle(scene).render_pixels(p1, bounces, crop)
    assert np.array_equal(ref[0].view(np.uint32), got[0].view(np.uint32)) and np.array_equal(ref[1], got[1])
    o = O.Oracle(scene)

    def run(threads, world, seconds):
        accum = np.zeros((o.height, o.width, 4), np.float32)
        out = np.zeros((o.height, o.width), np.uint32)
        rays = frames = 0
        t0 = time.perf_counter()
        while True:
            frames += 1
            p = scene.params(accumulation_index=frames)
            rays += o.render_frame(p, bounces, accum, out, rank=0, world_size=world, threads=threads)
            el = time.perf_counter() - t0
            if el >= seconds or frames >= 512:
                return rays, frames, el

    threads = O.lib().oracle_num_threads()
    rays, frames, el = run(threads, sample_world, min_seconds)
    rays1, frames1, el1 = run(1, 64, min_seconds / 4)
    return {
        "value": rays / el / 1e6,
        "unit": "Mray/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"CPU oracle (oracle/pathtrace_oracle.c, -O3 -march=native f32, OpenMP {threads} threads) on "
                   f"1/{sample_world} of the 8x8 tiles of the same {o.width}x{o.height} {bounces}-bounce frame, "
                   f"{frames} frame(s), {rays} rays in {el:.1f} s"),
        "build": " ".join(["gcc", *O.BASELINE_CFLAGS]),
        "single_thread": {"value": rays1 / el1 / 1e6, "unit": "Mray/s", "cores": 1,
                          "sample": f"1/64 of the tiles, {frames1} frame(s), {rays1} rays in {el1:.1f} s"},
    }


def default_frame_batch(world: int, steps: int) -> int:
    """Frames per launch: the timed steps split into launches of at most 32N frames
    (64 at most), as evenly as they go -- 20 steps at N=1 are one 20-frame launch,
    64 steps two of 32. A persistent launch pays one fill and one drain (about one
    path at full iteration cost) whatever its size, and a tile split
    over N GPUs needs N x the frames per launch for the same units per GPU. Measured
    at 20 steps, per frame (profiles/archive/r02_s3/r02_s3n, r02_s3o): C2 8 -> 20 frames
    0.337 -> 0.329 ms, C3 0.333 -> 0.290, C5 17.5 -> 15.5; 64 steps, C2 batches of
    8 -> 32: 0.318 -> 0.310."""
    cap = min(64, 32 * world)
    launches = -(-max(steps, 1) // cap)
    return -(-max(steps, 1) // launches)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2_rtiow")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--bounces", type=int, default=None)
    ap.add_argument("--settle-ms", type=float, default=150.0,
                    help="after the warmup steps, keep rendering untimed frames for this long (GPU clock ramp)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-sample-world", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true",
                    help="N>1: leave the RCCL gather of the image to rank 0 out of the timed region")
    ap.add_argument("--no-weak", action="store_true", help="N>1: skip the secondary weak-scaling measurement")
    ap.add_argument("--no-cadences", action="store_true",
                    help="N=1: skip the secondary single-frame and display-cadence timings")
    ap.add_argument("--gather", choices=["image", "accumulation"], default="accumulation",
                    help="N>1: the payload of the gather in the timed region: the RGBA32F accumulation "
                         "(16 B/px, the north star's 'RCCL gather of the accumulated RGBA buffer'; default) or "
                         "the displayed RGBA8 frame (4 B/px)")
    ap.add_argument("--driver", choices=["torch", "group"], default="torch",
                    help="N>1 route: torch = one process per GPU (torch.distributed.run, RCCL via ProcessGroupNCCL); "
                         "group = one process driving --gpus devices through the C ABI (rt_create_multi, "
                         "rt_gather_frame: RCCL send/recv), the Rust host's route")
    ap.add_argument("--brute-force", nargs="?", const="tiled", default=None, choices=["tiled", "stream"],
                    help="the reference's own sweeps (rt_set_brute_force; BASELINE config 5's stress mode) instead "
                         "of the acceleration structures: the sub-object records LDS-tiled (default) or streamed "
                         "through the scalar cache ('stream', rt_set_brute_force(ctx, 2))")
    ap.add_argument("--frame-batch", type=int, default=0,
                    help="frames one launch may render (rt_set_frame_batch); 0 = default_frame_batch(N, steps)")
    ap.add_argument("--triangle-pruning", type=int, choices=[0, 1, 2], default=1,
                    help="rt_set_triangle_pruning: 1 certified (default, exact), 0 box culling, 2 the round-3 "
                         "relative slack (not exact)")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="rt_set_tuning: an exact variant of the schedule or acceleration structures (A/B runs; "
                         "include/rt_abi.h lists the keys); repeatable")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong",
                    help="N>1: strong = the 1920x1080 frame split N ways (the metric's config, `value`); "
                         "weak = N x the pixels (per-GPU work fixed)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # RT_BENCH_DIST=1: take the N > 1 code path (process group, gather in the timed
    # region, weak run) even with one rank -- the one-GPU test box's check of the RCCL path
    dist_run = world > 1 or os.environ.get("RT_BENCH_DIST") == "1"
    if world != args.gpus:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    assert torch.cuda.is_available(), "bench.py needs a HIP device"
    # RT_BENCH_ONE_DEVICE=1 + RT_DIST_BACKEND=gloo: rehearse the N-rank path with
    # every rank on GPU 0 (single-GPU test boxes); the real run is one rank per GPU
    # over RCCL (backend "nccl").
    device = 0 if os.environ.get("RT_BENCH_ONE_DEVICE") == "1" else local_rank
    backend = os.environ.get("RT_DIST_BACKEND", "nccl")
    torch.cuda.set_device(device)
    if dist_run:
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
    if dist_run:
        dist.barrier()

    def size_for(scaling):
        if world > 1 and scaling == "weak":
            scale = world ** 0.5  # same view, N x the pixels: per-GPU work fixed
            return int(round(args.width * scale / 8.0)) * 8, int(round(args.height * scale / 8.0)) * 8
        return args.width, args.height

    def run(scaling, frame_batch, pattern="submit"):
        """Warmup, then exactly args.steps frames between barrier + sync; with N > 1 the
        timed region also assembles the image on rank 0 (pack -> RCCL gather -> unpack),
        once per run (a readback after the last frame, amortised over the steps).
        pattern "reference" (N=1 secondary): the reference's event loop through the default
        ABI -- no rt_set_frame_batch (frame_batch None), one rt_compute_frame call per frame
        and every DISPLAY_CADENCE_FRAMES frames the display copy (rt_copy_output_to_device,
        update_texture's buffer-to-texture copy on the device) into a display buffer."""
        width, height = size_for(scaling)
        scene, default_bounces = build_config(args.config, width=width, height=height)
        bounces = args.bounces or default_bounces
        r = Renderer(scene, device=device, rank=rank, world_size=world, frame_batch=frame_batch,
                     tuning={k: int(v) for k, v in (t.split("=", 1) for t in args.tune)})
        if args.triangle_pruning != 1:
            r.set_triangle_pruning(args.triangle_pruning)
        if frame_batch is None:
            frame_batch = r.frame_batch()[0]
        display = None
        if pattern == "reference":
            bpr = int(r._lib.rt_bytes_per_row(width, 256))
            display = (torch.zeros(height * bpr, dtype=torch.uint8, device=torch.device("cuda", device)), bpr)
        if args.brute_force:
            r.set_brute_force(2 if args.brute_force == "stream" else 1)

        def barrier_sync():
            r.synchronize()
            torch.cuda.synchronize()
            if dist_run:
                dist.barrier()

        gathered = dist_run and not args.no_gather
        if gathered:
            from rust_gpu_raytracing_amd.distributed import gather_frame
        for _ in range(args.warmup):
            r.compute_frame(bounces)
        # Clock settle: the GPU's power management raises its clocks only after tens of
        # ms of sustained load (a 20-frame C2 launch: 6.2 ms right after a 5-frame
        # warmup, 5.75 ms from the fourth launch on, 6.2 ms again after a 100 ms idle
        # gap; DESIGN.md §6, profiles/archive/r02_s4d). A display loop renders continuously, so
        # the steady rate is the one to time: after the W warmup steps, more untimed
        # frames until --settle-ms of wall time have passed (on every rank alike).
        settle_frames = 0
        r.synchronize()
        t_settle = time.perf_counter()
        while args.settle_ms > 0:
            go = torch.tensor([1.0 if (time.perf_counter() - t_settle) * 1e3 < args.settle_ms else 0.0],
                              device="cuda" if backend == "nccl" else "cpu")
            if dist_run:
                dist.all_reduce(go, op=dist.ReduceOp.MIN)
            if go.item() == 0.0:
                break
            for _ in range(frame_batch):
                r.compute_frame(bounces)
            settle_frames += frame_batch
            r.synchronize()
        if gathered:
            # untimed readbacks: allocate the gathers' buffers and let RCCL set up its
            # peer connections (made lazily on a pair's first transfer), as any display
            # loop has done by its second frame
            gather_frame(r, 0, "accumulation")
            gather_frame(r, 0, "image")
        barrier_sync()
        r.reset_ray_count()
        r.reset_timing()
        r.set_timing(True)
        barrier_sync()
        t0 = time.perf_counter()
        # the steps' compute_frame calls, a launch's worth per C call (rt_submit_frames: the
        # host loop a native caller runs, without a Python round trip per frame)
        done = 0
        if pattern == "reference":
            for i in range(args.steps):
                r.compute_frame(bounces)
                if (i + 1) % DISPLAY_CADENCE_FRAMES == 0:
                    r.copy_output_to_device(display[0].data_ptr(), display[1])
            done = args.steps
        while done < args.steps:
            n = min(frame_batch, args.steps - done)
            r.submit_frames(bounces, n)
            done += n
            if rank == 0 and args.steps >= 50 and done % 50 < n:
                log(f"step {done}/{args.steps}")
        t_gather_in_region = 0.0
        if gathered:
            # the frame assembled on rank 0 (pack -> RCCL gather -> unpack), stream-ordered
            # after the last frame; the closing barrier + sync waits for it. The gather's
            # share of the timed region is measured in place (events on the renderer's
            # stream around it; gloo: the host-side span after the frames are done), so
            # render time = timed region - that share is positive by construction.
            r.flush()
            if backend == "nccl":
                stream = torch.cuda.ExternalStream(r.stream_handle, device=torch.device("cuda", device))
                ev_frames = torch.cuda.Event(enable_timing=True)
                ev_gather = torch.cuda.Event(enable_timing=True)
                ev_frames.record(stream)
                gather_frame(r, 0, args.gather, sync=False)
                ev_gather.record(stream)
            else:
                r.synchronize()
                t_frames = time.perf_counter()
                gather_frame(r, 0, args.gather, sync=False)
                r.synchronize()
                t_gather_in_region = time.perf_counter() - t_frames
        barrier_sync()
        t_total = time.perf_counter() - t0
        if gathered and backend == "nccl":
            t_gather_in_region = ev_frames.elapsed_time(ev_gather) / 1e3
        r.set_timing(False)  # (reads the launch events back: outside the timed region)
        t_gather = t_gather_accum = t_gather_image = 0.0
        if gathered:
            # the gathers' own cost, reported beside `value` (which already includes the
            # --gather one): one more readback of the same frame per payload, timed alone
            # (the accumulation first, so that rank 0's output ends as the image gather
            # left it and the gather verify checks both payloads)
            def timed_gather(what):
                barrier_sync()
                t1 = time.perf_counter()
                gather_frame(r, 0, what, sync=False)
                barrier_sync()
                return time.perf_counter() - t1

            t_gather_accum = timed_gather("accumulation")
            t_gather_image = timed_gather("image")
            t_gather = t_gather_image if args.gather == "image" else t_gather_accum
        # render time: the timed region minus the gather it contains, measured in that
        # region (not the separately timed gathers above, which can take longer)
        t_render = t_total - t_gather_in_region
        assert 0.0 < t_render <= t_total, (t_render, t_total, t_gather_in_region)
        res = dict(r=r, scene=scene, bounces=bounces, width=width, height=height, rays=r.ray_count(),
                   streamed=r.streamed_bytes(), streamed_l2=r.streamed_bytes_l2(),
                   settle_frames=settle_frames,
                   t_render=t_render, t_gather=t_gather, gathered=gathered, launch=r.launch_config(),
                   passes=r.last_launch_passes(),
                   timing=r.dispatch_time_total(), resolve_timing=r.resolve_time_total(),
                   owned_px=r.owned_pixel_count())
        res["t_gather_in_region"] = t_gather_in_region
        stats = torch.tensor([t_total, t_render, t_gather, t_gather_accum, t_gather_image, float(res["rays"])],
                             dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        if dist_run:
            mx = stats[0:5].clone()
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            tot = stats[5:6].clone()
            dist.all_reduce(tot, op=dist.ReduceOp.SUM)
            stats = torch.cat([mx, tot])
        (res["t_total_max"], res["t_render_max"], res["t_gather_max"], res["t_gather_accum_max"],
         res["t_gather_image_max"], res["rays_total"]) = map(float, stats.tolist())
        return res

    def run_group(frame_batch):
        """--driver group: this one process drives args.gpus devices through the C ABI
        (rt_create_multi: a context and a host thread per device, RCCL communicators from
        ncclCommInitAll) -- the route a Rust host takes to several GPUs. Same timed
        region as run(): warmup, settle, then exactly args.steps frames and the frame
        assembled on device 0 (rt_gather_frame: pack -> grouped ncclSend/ncclRecv ->
        unpack), bracketed by a device synchronize of every device."""
        from rust_gpu_raytracing_amd.group import RendererGroup

        n = args.gpus
        scene, default_bounces = build_config(args.config, width=args.width, height=args.height)
        bounces = args.bounces or default_bounces
        g = RendererGroup(scene, list(range(n)), frame_batch=frame_batch)
        for _ in range(args.warmup):
            g.compute_frame(bounces)
        g.synchronize()
        settle_frames = 0
        t_settle = time.perf_counter()
        while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
            for _ in range(frame_batch):
                g.compute_frame(bounces)
            settle_frames += frame_batch
            g.synchronize()
        g.gather(0, args.gather)  # untimed: buffers, RCCL peer connections
        g.synchronize()
        g.reset_ray_count()
        views = [g.context_view(i) for i in range(n)]
        for v in views:
            v.reset_timing()
            v.set_timing(True)
        g.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            g.compute_frame(bounces)
        g.synchronize()  # the frames done on every device: the render share of the timed region
        t_frames = time.perf_counter() - t0
        g.gather(0, args.gather)
        g.synchronize()
        t_total = time.perf_counter() - t0
        t1 = time.perf_counter()
        g.gather(0, args.gather)
        g.synchronize()
        t_gather = time.perf_counter() - t1
        for v in views:
            v.set_timing(False)
        v0 = views[0]
        rays_total = g.ray_count()
        return dict(r=g, scene=scene, bounces=bounces, width=args.width, height=args.height,
                    rays=rays_total / n, settle_frames=settle_frames, t_render=t_frames,
                    t_gather=t_gather, gathered=True, launch=v0.launch_config(), passes=v0.last_launch_passes(),
                    timing=v0.dispatch_time_total(),
                    resolve_timing=v0.resolve_time_total(), owned_px=v0.owned_pixel_count(),
                    t_total_max=t_total, t_render_max=t_frames, t_gather_max=t_gather,
                    t_gather_accum_max=t_gather if args.gather == "accumulation" else 0.0,
                    t_gather_image_max=t_gather if args.gather == "image" else 0.0, rays_total=float(rays_total))

    if args.driver == "group":
        if world != 1:
            log("--driver group drives every device from one process: run it without torch.distributed.run")
            return 2
        world = args.gpus  # the group's ranks, for default_frame_batch and the report
        dist_run = True
    fb = args.frame_batch or default_frame_batch(world, args.steps)
    main_run = run_group(fb) if args.driver == "group" else run(args.scaling, fb)
    r = main_run["r"]
    if (main_run["gathered"] and os.environ.get("RT_BENCH_VERIFY_GATHER") == "1" and rank == 0
            and args.driver != "group"):
        # the assembled tile-split image must equal a 1-GPU render of the same frames
        with Renderer(main_run["scene"], device=device) as ref:
            for _ in range(args.warmup + main_run["settle_frames"] + args.steps):
                ref.compute_frame(main_run["bounces"])
            same = np.array_equal(ref.read_accumulation().view(np.uint32), r.read_accumulation().view(np.uint32))
            same = same and np.array_equal(ref.read_output(), r.read_output())
        log(f"gather verify: assembled image {'==' if same else '!='} 1-GPU render")
        if not same:
            return 3
    r.close()
    # Secondary cadences (N=1): the reference's call pattern through the default ABI (one
    # rt_compute_frame per frame, no rt_set_frame_batch, the display copy every 6 frames:
    # src/renderer.rs:201-283, src/main.rs:88-92, 365-375 -- a frame computed every >= 0.8 ms,
    # displayed every >= 5 ms); one launch per frame (rt_set_frame_batch(1), the reference's
    # one dispatch per compute_frame); launches of 6 frames (the display pacing, submitted).
    cadences = {}
    if world == 1 and not args.no_cadences and args.driver != "group":
        for key, batch, pattern in (("ms_per_step_reference_pattern", None, "reference"),
                                    ("ms_per_step_f1", 1, "submit"),
                                    ("ms_per_step_display_cadence", DISPLAY_CADENCE_FRAMES, "submit")):
            c_run = run(args.scaling, batch, pattern)
            c_run["r"].close()
            cadences[key] = c_run["t_total_max"] / args.steps * 1e3
    weak = None
    if dist_run and args.scaling == "strong" and not args.no_weak and args.driver != "group":
        w_run = run("weak", args.frame_batch or default_frame_batch(1, args.steps))
        w_run["r"].close()
        weak = {
            "value": w_run["rays_total"] / w_run["t_total_max"] / 1e6,
            "ms_per_step": w_run["t_total_max"] / args.steps * 1e3,
            "render_ms_per_step": w_run["t_render_max"] / args.steps * 1e3,
            "gather_ms": w_run["t_gather_max"] * 1e3,
            "gather_accum_ms": w_run["t_gather_accum_max"] * 1e3,
            "width": w_run["width"], "height": w_run["height"], "frame_batch": args.frame_batch or default_frame_batch(1, args.steps),
            "note": "secondary: the same view at N x the pixels, every GPU owning one 1920x1080 frame's worth of tiles",
        }

    if rank == 0:
        m = main_run
        scene, bounces, width, height = m["scene"], m["bounces"], m["width"], m["height"]
        kern_ms, n_timed = m["timing"]
        resolve_ms, _ = m["resolve_timing"]
        # the frame's work is the path kernel plus, in frame-parallel batches, the
        # resolve pass that adds the lights to the accumulation and packs the output:
        # SURVEY §8d's bytes are priced against both kernels' device time
        avg_path_s = kern_ms / max(n_timed, 1) / 1e3
        avg_resolve_s = resolve_ms / max(n_timed, 1) / 1e3
        avg_kernel_s = avg_path_s + avg_resolve_s
        frames_per_launch = args.steps / max(n_timed, 1)
        rays_per_launch = m["rays"] / max(n_timed, 1)
        b_launch = algorithmic_bytes(m["owned_px"], rays_per_launch, scene_bytes(scene), frames_per_launch)
        # brute-force launches also stream the sub-object records: SURVEY §8d's tile-streaming
        # term with its fixed convention (32 B x the sub-objects per started 256 rays of each
        # bounce level), counted by the kernel; what the sweeps actually read from L2 (per LDS
        # tile and workgroup, or per wave in the scalar-cache mode) is reported beside it
        stream_launch = m.get("streamed", 0) / max(n_timed, 1)
        stream_l2_launch = m.get("streamed_l2", 0) / max(n_timed, 1)
        b_launch += stream_launch
        achieved = b_launch / avg_kernel_s / 1e9
        eff_launch_s = m["t_render"] / max(n_timed, 1)  # wall time per launch: overlapped launches pipeline
        workload = f"{args.config} {width}x{height}, {bounces} bounces, 1 spp/frame, accumulate"
        if args.brute_force:
            # named by the kernel that ran (rt_last_launch_passes): mode 2 streams the records only
            # where the scene has triangles to sweep, else the LDS tiles run
            streamed = "brute_stream" in m.get("passes", [])
            workload += (", brute-force sweeps streamed through the scalar cache" if streamed
                         else ", brute-force LDS-tiled sweeps")
        # a non-default triangle walk is another workload for the PMC table (its counters are
        # not the default walk's): --triangle-pruning 0 = box culling, 2 = the round-3 slack (not exact)
        if args.triangle_pruning != 1 and int(scene.flatten()[2].shape[0]) > 0:
            workload += f", triangle pruning mode {args.triangle_pruning}"
        if args.tune:
            workload += ", tuning " + " ".join(sorted(args.tune))
        build_hash = native_build.source_hash()
        pmc, pmc_why = pmc_entry(f"{workload} | frame_batch {fb}", build_hash) if world == 1 else (None, "N>1")
        result = {
            "metric": METRIC,
            "value": m["rays_total"] / m["t_total_max"] / 1e6,
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle": {"ms": args.settle_ms, "frames": m["settle_frames"],
                       "note": "untimed frames after the warmup steps until the GPU clocks settle (DESIGN.md §6)"},
            "ms_per_step": m["t_total_max"] / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling if world > 1 else "strong",
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
                "pixels_per_gpu": m["owned_px"],
                "rays_per_step": m["rays_total"] / args.steps,
                "nominal_rays_per_step": width * height * bounces,
                "frame_batch": fb,
                "launches": n_timed,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": pmc_traffic(pmc),
                "traffic_source": pmc["source"] if pmc else pmc_why,
                "kernel": " + ".join(KERNEL_NAMES[p] for p in m.get("passes", ["path", "resolve"])),
                "kernel_ms_avg": avg_kernel_s * 1e3,
                "path_kernel_ms_avg": avg_path_s * 1e3,
                "resolve_ms_avg": avg_resolve_s * 1e3,
                "kernel_timing": ("device-clock span per launch (first workgroup start to last end, the primary "
                                  "pre-pass included when it runs), rt_set_timing, plus the batch's resolve pass"),
                "counter_frac": (pmc_traffic(pmc) / avg_path_s / 1e9 / HBM_PEAK_GBS) if pmc else None,  # PMC: path kernel
                "valu_frac": ((pmc["valu_issue_util"] * pmc["valu_lane_util"])
                              if pmc and pmc.get("valu_issue_util") is not None else None),
                "effective_ms_per_launch": eff_launch_s * 1e3,
                "achieved_effective": b_launch / eff_launch_s / 1e9,
                "frames_per_launch": frames_per_launch,
                "launch": m["launch"],
                "bytes_per_launch": b_launch,
                "tile_stream_bytes_per_launch": stream_launch,
                "l2_stream_bytes_per_launch": stream_l2_launch,
                "note": ("the reference's sweeps: VALU-bound on sub-object box tests (DESIGN §5.5). "
                         "bytes_per_launch carries SURVEY §8d's tile-streaming term, the sub-object "
                         "records (32 B each) delivered once per started 256-ray tile of every bounce "
                         "level: a fixed convention for bytes moved to the CUs, which the L2 and MALL "
                         "serve (the whole record array is a few MB), so it exceeds the HBM traffic the "
                         "PMC counters see (`traffic`); l2_stream_bytes_per_launch is what the kernel's "
                         "own tiles (mode 1) or waves (mode 2) actually read from L2"
                         if args.brute_force else
                         "branchy f32 VALU-bound path (SURVEY §7); HBM fraction is low by construction"),
                "valu": pmc_issue(pmc),
                # the roofline this path is actually bound by: VALU issue x lane utilisation of the
                # same PMC run against the f32 lane peak
                "valu_lane_roofline": ({"bound": "valu", "unit": "T lane-op/s",
                                        "achieved": pmc["valu_issue_util"] * pmc["valu_lane_util"] * VALU_LANE_PEAK_TOPS,
                                        "peak": VALU_LANE_PEAK_TOPS,
                                        "frac": pmc["valu_issue_util"] * pmc["valu_lane_util"]}
                                       if pmc and pmc.get("valu_issue_util") is not None else None),
                "build_hash": build_hash,
            },
        }
        result.update(cadences)
        if cadences:
            result["cadence_note"] = (f"secondary: the same {args.steps} steps as the reference's loop calls the "
                                      "default ABI (one rt_compute_frame per frame, no rt_set_frame_batch, "
                                      f"rt_copy_output_to_device every {DISPLAY_CADENCE_FRAMES} frames), in "
                                      "single-frame launches (rt_set_frame_batch(1)), and in submitted launches of "
                                      f"{DISPLAY_CADENCE_FRAMES}; `value` uses frame_batch")
            result["reference_pattern_vs_headline"] = cadences["ms_per_step_reference_pattern"] / result["ms_per_step"]
        if args.driver == "group":
            result["driver"] = "c-abi group (rt_create_multi + rt_gather_frame, one process)"
        # the gather's payload in `value` (the default moved from the RGBA8 image to
        # the accumulation in round 5; None when no gather is timed, N = 1)
        result["gather_payload"] = args.gather if (dist_run and m["gathered"]) else None
        if dist_run:
            result["render_ms_per_step"] = m["t_render_max"] / args.steps * 1e3
            result["gather_ms"] = m["t_gather_max"] * 1e3
            result["gather_in_value"] = m["gathered"]
            if m["gathered"]:
                result["gather_image_ms"] = m["t_gather_image_max"] * 1e3
                result["gather_accum_ms"] = m["t_gather_accum_max"] * 1e3
                # the same run priced with the other payload's gather in place of the --gather
                # one: rays / (render time + that gather's time, timed alone)
                result["value_with_accum_gather"] = m["rays_total"] / (m["t_render_max"] + m["t_gather_accum_max"]) / 1e6
                result["value_with_image_gather"] = m["rays_total"] / (m["t_render_max"] + m["t_gather_image_max"]) / 1e6
            if weak is not None:
                result["weak"] = weak
        if world == 1 and not args.no_cpu_baseline:
            log("cpu baseline ...")
            result["cpu_baseline"] = cpu_baseline(scene, bounces, args.cpu_seconds, args.cpu_sample_world)
        print(json.dumps(result), flush=True)
    if dist_run and args.driver != "group":
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
