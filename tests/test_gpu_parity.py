"""GPU parity: the HIP kernel through the C ABI against the CPU oracle and the goldens.

The bar is bit-exact (accumulation f32 bits, packed RGBA8, counted rays), which
implies the north star's <= 1e-4 per-channel RMS; the RMS is asserted too.
"""
import numpy as np
import pytest

from rust_gpu_raytracing_amd import Renderer, RtError
from rust_gpu_raytracing_amd import _native as N
from rust_gpu_raytracing_amd import buffers as B
from rust_gpu_raytracing_amd.scene import build_config
from tests.golden.fixtures import CASES, load, params_for, render_case_with_oracle, scene_from_inputs

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-4  # north_star: <= 1e-4 per-channel RMS


def rms_per_channel(a, b):
    a = np.nan_to_num(a.reshape(-1, 4).astype(np.float64), nan=0.0)
    b = np.nan_to_num(b.reshape(-1, 4).astype(np.float64), nan=0.0)
    return np.sqrt(((a - b) ** 2).mean(axis=0))


def assert_same(acc_g, out_g, rays_g, acc_o, out_o, rays_o):
    assert rays_g == rays_o
    assert rms_per_channel(acc_g, acc_o).max() <= RMS_TOL
    assert np.array_equal(out_g, out_o)
    assert np.array_equal(acc_g.view(np.uint32), acc_o.view(np.uint32))


def gpu_render(scene, bounces, frames, *, spp=1, accumulate=1, rays=None, prune=None, **kw):
    with Renderer(scene, accumulate=bool(accumulate), compute_per_frame=spp, camera_rays=rays, **kw) as r:
        if prune is not None:
            r.set_triangle_pruning(prune)
        for _ in range(frames):
            r.compute_frame(bounces)
        return r.read_accumulation(), r.read_output(), r.ray_count()


# frame_batch None: the library default (frames queued, launched at the readback: batched
# launches); 1: one launch per compute_frame, the reference's dispatch pattern
@pytest.mark.parametrize("batch", [None, 1])
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_matches_golden(gpu, name, batch):
    g = load(name)
    case = CASES[name]
    scene = scene_from_inputs(g)
    acc, out, rays = gpu_render(scene, case["bounces"], case["frames"], spp=case["spp"],
                                accumulate=case["accumulate"], rays=g["camera_rays"].astype(B.RAY),
                                frame_batch=batch)
    assert_same(acc, out, rays, g["accum"], g["out"], int(g["rays"]))


@pytest.mark.parametrize("config,w,h,frames,kw", [
    ("c1_four_spheres", 200, 152, 4, {}),
    ("c2_rtiow", 320, 180, 2, {}),
    ("c3_chess", 320, 184, 2, dict(env_size=(2048, 1024))),
    ("c4_mixed", 256, 144, 2, dict(env_size=(1024, 512))),
    ("c5_heightfield", 192, 112, 2, dict(nx=160, nz=80)),
])
@pytest.mark.parametrize("batch", [None, 1])
def test_gpu_matches_oracle_full_frame(gpu, oracle_lib, config, w, h, frames, kw, batch):
    scene, bounces = build_config(config, width=w, height=h, **kw)
    acc_o, out_o, rays_o = oracle_lib.render_frames(scene, bounces, frames)
    acc, out, rays = gpu_render(scene, bounces, frames, frame_batch=batch)
    assert_same(acc, out, rays, acc_o, out_o, rays_o)


@pytest.mark.parametrize("kind", ["cols_uniform", "rows_uniform", "both_uniform", "one_texel_off", "random"])
def test_gpu_env_map_uniform_rows_columns(gpu, oracle_lib, kind):
    """sample_env skips u (v) when every row (column) of the env map is one colour
    (rt_upload_env_map detects it): each case, and a map one texel away from
    uniform rows, must equal the oracle, which always computes both coordinates."""
    scene, bounces = build_config("c2_rtiow", width=160, height=96)
    rng = np.random.default_rng(11)
    eh, ew = 64, 128
    if kind == "cols_uniform":
        env = np.broadcast_to(rng.integers(0, 256, (1, ew, 4), dtype=np.uint8), (eh, ew, 4))
    elif kind in ("rows_uniform", "one_texel_off"):
        env = np.broadcast_to(rng.integers(0, 256, (eh, 1, 4), dtype=np.uint8), (eh, ew, 4))
    elif kind == "both_uniform":
        env = np.broadcast_to(np.array([40, 90, 200, 255], np.uint8), (eh, ew, 4))
    else:
        env = rng.integers(0, 256, (eh, ew, 4), dtype=np.uint8)
    env = np.ascontiguousarray(env)
    if kind == "one_texel_off":
        env[eh // 2, ew // 3, 0] ^= 0x40
    scene.environment_map = env
    acc_o, out_o, rays_o = oracle_lib.render_frames(scene, bounces, 2)
    acc, out, rays = gpu_render(scene, bounces, 2)
    assert_same(acc, out, rays, acc_o, out_o, rays_o)


def oracle_frames(oracle_lib, scene, bounces, frames, rays, **kw):
    """The oracle's accumulation, output and rays after `frames` frames (k = 1..frames)."""
    o = oracle_lib.Oracle(scene, camera_rays=rays)
    acc = np.zeros((o.height, o.width, 4), np.float32)
    out = np.zeros((o.height, o.width), np.uint32)
    n = 0
    for k in range(1, frames + 1):
        n += o.render_frame(scene.params(accumulation_index=k, **kw), bounces, acc, out)
    return acc, out, n


@pytest.mark.parametrize("config", ["c1_four_spheres", "c2_rtiow", "c3_chess", "c4_mixed"])
def test_gpu_full_frame_baseline_size(gpu, oracle_lib, config):
    """BASELINE.json sizes, every pixel: C1 800x600x4, C2 and C3 1920x1080x8 (C3 with its
    8192x4096 env map), C4 3840x2160x16 -- 2 accumulated frames each (k = 1, 2;
    compute_shader.wgsl:146-189), accumulation bits, RGBA8 and ray count against the oracle."""
    scene, bounces = build_config(config)
    rays = scene.camera.recalculate_ray_directions()
    acc, out, n = gpu_render(scene, bounces, 2, rays=rays)
    assert_same(acc, out, n, *oracle_frames(oracle_lib, scene, bounces, 2, rays))


_C5_SAMPLE = {}


def _c5_full_size_oracle_sample(oracle_lib):
    """C5 at its BASELINE size with the oracle's result on 20,000 random pixels of 2 frames
    (the oracle sweeps all 142,858 sub-objects per ray, ~10^4 rays/s per thread); built once
    and shared by the accelerator and brute-force tests."""
    if not _C5_SAMPLE:
        scene, bounces = build_config("c5_heightfield")
        rays = scene.camera.recalculate_ray_directions()
        o = oracle_lib.Oracle(scene, camera_rays=rays)
        rng = np.random.default_rng(11)
        pix = rng.choice(1920 * 1080, 20000, replace=False).astype(np.uint32)
        a = None
        for k in (1, 2):
            a, o_out, _ = o.render_pixels(scene.params(accumulation_index=k), bounces, pix, accum_in=a)
        _C5_SAMPLE.update(scene=scene, bounces=bounces, rays=rays, pix=pix, acc=a, out=o_out)
    return _C5_SAMPLE


def _check_c5_sample(smp, acc, out):
    g_acc = acc.reshape(-1, 4)[smp["pix"]]
    g_out = out.reshape(-1)[smp["pix"]]
    assert rms_per_channel(g_acc, smp["acc"]).max() <= RMS_TOL
    assert np.array_equal(g_out, smp["out"])
    assert np.array_equal(g_acc.view(np.uint32), smp["acc"].view(np.uint32))


def test_gpu_full_size_sampled_c5(gpu, oracle_lib):
    """C5 (1M triangles, 1920x1080x8) on the default path: 20,000 random pixels of 2
    frames against the oracle."""
    smp = _c5_full_size_oracle_sample(oracle_lib)
    acc, out, _ = gpu_render(smp["scene"], smp["bounces"], 2, rays=smp["rays"])
    _check_c5_sample(smp, acc, out)


@pytest.mark.parametrize("mode", [1, 2])
def test_gpu_full_size_brute_force_c5(gpu, oracle_lib, mode):
    """BASELINE config 5 as named -- the 1,000,000-triangle mesh at 1920x1080x8 in the
    brute-force mode (rt_brute_wf_kernel: the reference's own object -> sub-object ->
    triangle sweep for every ray; the records LDS-tiled, 1, or streamed through the scalar
    cache, 2): the oracle's 20,000 sampled pixels, and every pixel of both frames
    bit-identical to the accelerated default path."""
    smp = _c5_full_size_oracle_sample(oracle_lib)
    scene, bounces, rays = smp["scene"], smp["bounces"], smp["rays"]
    with Renderer(scene, camera_rays=rays, frame_batch=2) as r:
        r.set_brute_force(mode)
        for _ in range(2):
            r.compute_frame(bounces)
        acc, out, n = r.read_accumulation(), r.read_output(), r.ray_count()
        # SURVEY §8d's tile-streaming term: 32 B x 142,858 sub-objects per started 256 rays of
        # each bounce level -- at least the first level's whole frame of rays, per frame
        n_sub = sum(len(o.sub_object_info) for o in scene.objects)
        assert r.streamed_bytes() >= 2 * -(-1920 * 1080 // 256) * 32 * n_sub
        assert r.streamed_bytes() % (32 * n_sub) == 0
        assert r.streamed_bytes_l2() > 0
        assert "brute" in r.last_launch_passes()
    _check_c5_sample(smp, acc, out)
    acc_d, out_d, n_d = gpu_render(scene, bounces, 2, rays=rays)
    assert n == n_d
    assert np.array_equal(out, out_d)
    assert np.array_equal(acc.view(np.uint32), acc_d.view(np.uint32))


def test_gpu_reference_bounce_default(gpu, oracle_lib):
    # the reference hard-codes 10 bounces (compute_shader.wgsl:150); Renderer's default
    scene, _ = build_config("c3_chess", width=96, height=64, env_size=(512, 256))
    acc_o, out_o, rays_o = oracle_lib.render_frames(scene, 10, 2, compute_per_frame=5)
    with Renderer(scene, compute_per_frame=5) as r:
        r.compute_frame()
        r.compute_frame()
        assert_same(r.read_accumulation(), r.read_output(), r.ray_count(), acc_o, out_o, rays_o)


def owned_mask(w, h, rank, world):
    """Pixels of the 8x8 tiles t with t % world == rank."""
    ty, tx = np.divmod(np.arange(h * w), w)
    tile = (ty // 8) * ((w + 7) // 8) + tx // 8
    return (tile % world == rank).reshape(h, w)


@pytest.mark.parametrize("config,w,h,world,kw", [
    ("c3_chess", 256, 136, 4, dict(env_size=(1024, 512))),
    ("c2_rtiow", 1920, 1080, 8, {}),
    ("c4_mixed", 3840, 2160, 8, {}),
])
def test_gpu_tile_split_bitwise(gpu, config, w, h, world, kw):
    """Seeds depend only on the global pixel index (:217): N tile-ranks == 1 GPU, bit for
    bit, including the 8-way split of the BASELINE C2 and C4 frames."""
    scene, bounces = build_config(config, width=w, height=h, **kw)
    rays = scene.camera.recalculate_ray_directions()
    acc1, out1, rays1 = gpu_render(scene, bounces, 2, rays=rays)
    acc = np.zeros_like(acc1)
    out = np.zeros_like(out1)
    total = 0
    for rank in range(world):
        a, o, r = gpu_render(scene, bounces, 2, rays=rays, rank=rank, world_size=world)
        mask = owned_mask(w, h, rank, world)
        acc[mask] = a[mask]
        out[mask] = o[mask]
        assert not a[~mask].any() and not o[~mask].any()  # nothing written outside the rank's tiles
        total += r
    assert total == rays1
    assert np.array_equal(out, out1) and np.array_equal(acc.view(np.uint32), acc1.view(np.uint32))


@pytest.mark.parametrize("rank,world,w,h", [(0, 1, 1920, 1080), (1, 3, 3840, 2160)])
def test_gpu_cost_ordered_schedule(gpu, rank, world, w, h):
    """The cost-ordered tile schedule (rt_set_tile_schedule) changes only the
    claim order: bit-identical to index order. Each launch records every ray
    of its tiles; the next launch's first idle workgroup sorts them into a
    permutation, most rays first, which the launch after that claims in."""
    scene, bounces = build_config("c2_rtiow", width=w, height=h)
    res = []
    for schedule in (0, 1):
        with Renderer(scene, rank=rank, world_size=world) as r:
            r.set_tile_schedule(schedule)
            n_tiles = r.owned_pixel_count() // 64
            prev_costs = None
            for f in range(5):
                before = r.ray_count()
                r.compute_frame(bounces)
                order, costs = r.tile_schedule_state()
                assert np.array_equal(np.sort(order), np.arange(n_tiles))  # always a permutation
                if schedule == 0:
                    assert np.array_equal(order, np.arange(n_tiles)) and not costs.any()
                    continue
                assert costs.sum() == r.ray_count() - before  # every ray of this launch, by tile
                if f == 0:
                    assert np.array_equal(order, np.arange(n_tiles))  # nothing recorded before launch 0
                else:  # a stable sort of the previous launch's costs into 16 buckets, most rays first
                    c = prev_costs.astype(np.uint64)
                    key = 15 - (c * 16) // (c.max() + 1)
                    assert np.array_equal(order, np.argsort(key, kind="stable"))
                prev_costs = costs
            res.append((r.read_accumulation(), r.read_output(), r.ray_count()))
    (a0, o0, n0), (a1, o1, n1) = res
    assert n0 == n1
    assert np.array_equal(o0, o1) and np.array_equal(a0.view(np.uint32), a1.view(np.uint32))


def test_gpu_cost_ordered_schedule_inactive_on_small_frames(gpu):
    """With about one tile per resident wave the schedule stays off: index order, nothing recorded."""
    scene, bounces = build_config("c1_four_spheres", width=320, height=184)
    with Renderer(scene) as r:
        r.set_tile_schedule(1)
        for _ in range(3):
            r.compute_frame(bounces)
        order, costs = r.tile_schedule_state()
        assert np.array_equal(order, np.arange(order.size)) and not costs.any()


@pytest.mark.parametrize("accumulate,payload", [(1, "accumulation"), (0, "image"), (1, "image")])
def test_gpu_pack_unpack_gather(gpu, accumulate, payload):
    """The multi-GPU readback path on one device: ranks pack their tiles into device
    buffers, rank 0 unpacks them; the assembled frame equals a 1-GPU render. The
    "image" payload (bench.py's default at N > 1, and the only one of a
    non-accumulating render, which never writes the accumulation, :171-178) moves the
    RGBA8 words: rank 0's output is the whole frame, its accumulation keeps its own
    tiles only."""
    import torch

    from rust_gpu_raytracing_amd.distributed import owned_pixel_indices

    scene, bounces = build_config("c2_rtiow", width=200, height=104)
    acc1, out1, _ = gpu_render(scene, bounces, 3, accumulate=accumulate)
    world = 3
    rs = [Renderer(scene, rank=r, world_size=world, accumulate=bool(accumulate)) for r in range(world)]
    try:
        for r in rs:
            for _ in range(3):
                r.compute_frame(bounces)
        bufs = []
        if payload == "image" and accumulate:
            for r in rs:
                t = torch.empty((r.owned_pixel_count(),), dtype=torch.int32, device=gpu)
                r.pack_owned_output(t.data_ptr())
                r.synchronize()
                bufs.append(t)
            root = rs[0]
            for src in range(1, world):
                root.unpack_output(bufs[src].data_ptr(), src, world)
            root.synchronize()
            assert np.array_equal(root.read_output(), out1)
            acc0 = root.read_accumulation().reshape(-1, 4)
            own = owned_pixel_indices(200, 104, 0, world)
            own = own[own >= 0]
            mine = np.zeros(acc0.shape[0], bool)
            mine[own] = True
            assert np.array_equal(acc0[mine].view(np.uint32), acc1.reshape(-1, 4)[mine].view(np.uint32))
            assert not acc0[~mine].any()  # the other ranks' accumulations stay on their owners
            return
        for r in rs:
            n = r.owned_pixel_count()
            if accumulate:
                t = torch.empty((n, 4), dtype=torch.float32, device=gpu)
                r.pack_owned_accumulation(t.data_ptr())
            else:
                t = torch.empty((n,), dtype=torch.int32, device=gpu)
                r.pack_owned_output(t.data_ptr())
            r.synchronize()
            bufs.append(t)
        root = rs[0]
        k = root.accumulation_index - 1
        for src in range(1, world):
            if accumulate:
                root.unpack_accumulation(bufs[src].data_ptr(), src, world, k * 1)
            else:
                root.unpack_output(bufs[src].data_ptr(), src, world)
        root.synchronize()
        assert np.array_equal(root.read_accumulation().view(np.uint32), acc1.view(np.uint32))
        assert np.array_equal(root.read_output(), out1)
        if not accumulate:
            assert out1.any() and not acc1.any()
    finally:
        for r in rs:
            r.close()


@pytest.mark.parametrize("accumulate,world,dst", [(1, 3, 0), (1, 5, 2), (0, 4, 3)])
def test_gpu_unpack_all_ranks_one_launch(gpu, accumulate, world, dst):
    """rt_unpack_{accumulation,output}_ranks: the gather's blocks laid out in one
    (world, cap) buffer, every rank's but the destination's unpacked by one launch;
    the destination's frame equals a 1-GPU render. 200x104 is 25x13 = 325 tiles, so
    the ranks own unequal tile counts and the padded blocks carry unused rows."""
    import torch

    scene, bounces = build_config("c2_rtiow", width=200, height=104)
    acc1, out1, _ = gpu_render(scene, bounces, 3, accumulate=accumulate)
    rs = [Renderer(scene, rank=r, world_size=world, accumulate=bool(accumulate)) for r in range(world)]
    try:
        cap = rs[0].owned_pixel_count()  # rank 0 owns the most tiles
        shape = (world, cap, 4) if accumulate else (world, cap)
        dtype = torch.float32 if accumulate else torch.int32
        allb = torch.full(shape, -1, dtype=dtype, device=gpu)  # garbage in the padding rows
        for r in rs:
            for _ in range(3):
                r.compute_frame(bounces)
            (r.pack_owned_accumulation if accumulate else r.pack_owned_output)(allb[r.rank].data_ptr())
            r.synchronize()
        root = rs[dst]
        if accumulate:
            root.unpack_accumulation_ranks(allb.data_ptr(), cap, world, dst, root.accumulation_index - 1)
        else:
            root.unpack_output_ranks(allb.data_ptr(), cap, world, dst)
        root.synchronize()
        assert np.array_equal(root.read_accumulation().view(np.uint32), acc1.view(np.uint32))
        assert np.array_equal(root.read_output(), out1)
    finally:
        for r in rs:
            r.close()


@pytest.mark.parametrize("config,spp,accumulate,batch,parallel,kw", [
    ("c2_rtiow", 1, 1, 4, "1", {}),
    ("c2_rtiow", 1, 1, 4, "0", {}),
    ("c3_chess", 2, 1, 3, "1", dict(env_size=(512, 256))),
    ("c3_chess", 2, 1, 3, "0", dict(env_size=(512, 256))),
    ("c1_four_spheres", 1, 0, 4, "1", {}),
    ("c5_heightfield", 1, 1, 2, "1", dict(nx=80, nz=40)),
    ("c2_rtiow", 1, 1, 20, "1", {}),  # the bench's launch at its default 20 steps
    ("c3_chess", 1, 1, 64, "1", dict(env_size=(512, 256))),  # the largest batch
])
def test_gpu_frame_batch(gpu, oracle_lib, config, spp, accumulate, batch, parallel, kw):
    """rt_set_frame_batch: queued frames launched F at a time give, after every
    observable point, exactly the single-frame sequence (the oracle's): a readback
    in the middle of a batch, a bounce change, and a tail shorter than F (frames queued
    one call at a time and through rt_submit_frames). Both batch
    kernels: frame-parallel (a queue unit per (frame, tile), lights resolved in order,
    the default) and tuning "frame_parallel" 0 (each pixel's frames back to back on a lane)."""
    scene, bounces = build_config(config, width=96, height=56, **kw)
    rays = scene.camera.recalculate_ray_directions()
    with Renderer(scene, accumulate=bool(accumulate), compute_per_frame=spp, camera_rays=rays,
                  frame_batch=batch, tuning={"frame_parallel": int(parallel)}) as r:
        assert r.frame_batch() == (batch, 0)
        for f in range(batch - 1):
            r.compute_frame(bounces)
        assert r.frame_batch() == (batch, batch - 1)  # queued, k advanced already
        assert r.accumulation_index == (batch if accumulate else 1)
        mid = r.read_accumulation(), r.read_output(), r.ray_count()  # flushes the partial batch
        assert r.frame_batch() == (batch, 0)
        r.submit_frames(bounces, batch + 1)  # a full batch, then one queued frame (rt_submit_frames)
        r.compute_frame(bounces + 1)  # bounce change: the queued frame is launched first
        end = r.read_accumulation(), r.read_output(), r.ray_count()
    o = oracle_lib.Oracle(scene, camera_rays=rays)
    acc = np.zeros((56, 96, 4), np.float32)
    out = np.zeros((56, 96), np.uint32)
    n = 0
    seq = [bounces] * (batch - 1 + batch + 1) + [bounces + 1]
    for i, b in enumerate(seq):
        k = i + 1 if accumulate else 1
        n += o.render_frame(scene.params(accumulate=accumulate, compute_per_frame=spp, accumulation_index=k), b,
                            acc, out)
        if i == batch - 2:
            assert_same(*mid, acc, out, n)
    assert_same(*end, acc, out, n)


@pytest.mark.parametrize("stage", ["0", "1"])
def test_gpu_sub_objects_in_lds(gpu, oracle_lib, stage):
    """Mode 2 stages the leaves' sub-object records in LDS when they fit (tuning "stage_subs");
    both ways, and through the in-plane sweep fallback that reads them too, the result is
    the oracle's."""
    tuning = {"stage_subs": int(stage)}
    scene, bounces = build_config("c3_chess", width=96, height=64, env_size=(512, 256))
    rays = scene.camera.recalculate_ray_directions()
    acc, out, n = gpu_render(scene, bounces, 3, rays=rays, tuning=tuning)
    with Renderer(scene, camera_rays=rays, tuning=tuning) as r:
        r.compute_frame(bounces)
        assert r.launch_config()["scene_in_lds"] == 2
    o = oracle_lib.Oracle(scene, camera_rays=rays)
    acc_o = np.zeros((64, 96, 4), np.float32)
    out_o = np.zeros((64, 96), np.uint32)
    n_o = sum(o.render_frame(scene.params(accumulation_index=k), bounces, acc_o, out_o) for k in (1, 2, 3))
    assert_same(acc, out, n, acc_o, out_o, n_o)


def test_gpu_default_batch_at_4k_with_many_samples(gpu):
    """the default frame batch (RT_DEFAULT_FRAME_BATCH) sizes its light
    buffer per batch -- 3840x2160 at 24 samples per frame is 16 x 24 x 8.3 M x 16 B = 51 GB for
    one 16-frame batch, more than the context's budget (an eighth of the device's memory), so
    the library renders it as consecutive launches. The default context renders 16 frames
    bit-identical to single-frame launches."""
    scene, bounces = build_config("c2_rtiow", width=3840, height=2160)
    rays = scene.camera.recalculate_ray_directions()
    res = []
    for fb in (None, 1):
        with Renderer(scene, camera_rays=rays, compute_per_frame=24, frame_batch=fb) as r:
            if fb is None:
                assert r.frame_batch()[0] == N.RT_DEFAULT_FRAME_BATCH
            r.submit_frames(bounces, 16)
            r.synchronize()
            res.append((r.read_accumulation(), r.read_output(), r.ray_count()))
    (a0, o0, n0), (a1, o1, n1) = res
    assert n0 == n1 and np.array_equal(o0, o1) and np.array_equal(a0.view(np.uint32), a1.view(np.uint32))


def test_gpu_default_batching_and_device_display_copy(gpu, oracle_lib):
    """ABI 11: by default rt_compute_frame queues its frame (RT_DEFAULT_FRAME_BATCH) and the
    next observation launches the queue. The reference's loop -- one compute_frame per frame,
    a display copy every ~6 frames (src/renderer.rs:201-283, src/main.rs:88-92) -- through
    rt_copy_output_to_device (update_texture's buffer-to-texture copy, on the device, with
    the 256-B row pitch): every displayed image equals the oracle's output after that frame."""
    import torch

    scene, bounces = build_config("c2_rtiow", width=200, height=112)
    rays = scene.camera.recalculate_ray_directions()
    o = oracle_lib.Oracle(scene, camera_rays=rays)
    acc_o = np.zeros((o.height, o.width, 4), np.float32)
    out_o = np.zeros((o.height, o.width), np.uint32)
    with Renderer(scene, camera_rays=rays) as r:
        assert r.frame_batch() == (N.RT_DEFAULT_FRAME_BATCH, 0)
        lib = r._lib
        bpr = int(lib.rt_bytes_per_row(r.width, 256))
        disp = torch.full((r.height * bpr,), 0xAB, dtype=torch.uint8, device="cuda")
        shown = 0
        for k in range(1, 21):
            r.compute_frame(bounces)
            o.render_frame(scene.params(accumulation_index=k), bounces, acc_o, out_o)
            assert r.frame_batch()[1] == k - 6 * shown  # queued, nothing launched yet
            if k % 6 == 0:
                r.copy_output_to_device(disp.data_ptr(), bpr)
                shown += 1
                assert r.frame_batch()[1] == 0
                r.synchronize()  # the copy is ordered on the renderer's stream, not torch's
                img = disp.cpu().numpy().reshape(r.height, bpr)
                assert np.array_equal(img[:, : 4 * r.width].copy().view(np.uint32), out_o)
                assert (img[:, 4 * r.width:] == 0xAB).all()  # the pitch padding untouched
        with pytest.raises(RtError):
            r.copy_output_to_device(disp.data_ptr(), 4 * r.width - 4)
        assert np.array_equal(r.read_accumulation().view(np.uint32), acc_o.view(np.uint32))


def test_gpu_last_launch_passes(gpu):
    """rt_last_launch_passes names the kernels a dispatch ran (the bench's roofline uses it)."""
    scene, bounces = build_config("c2_rtiow", width=64, height=48)
    with Renderer(scene, frame_batch=2) as r:
        r.compute_frame(bounces)
        r.synchronize()
        assert r.last_launch_passes() == ["path"]  # a single frame: no resolve pass
        r.compute_frame(bounces)
        r.compute_frame(bounces)
        r.synchronize()
        assert r.last_launch_passes() == ["path", "resolve"]
    scene, bounces = build_config("c5_heightfield", width=64, height=48, nx=200, nz=100)
    with Renderer(scene) as r:
        r.compute_frame(bounces)
        r.synchronize()
        assert r.last_launch_passes() == ["path", "primary"]  # accelerator in global memory
        r.set_brute_force(True)
        r.compute_frame(bounces)
        r.synchronize()
        assert r.last_launch_passes() == ["brute"]
        r.set_brute_force(2)
        r.compute_frame(bounces)
        r.synchronize()
        assert r.last_launch_passes() == ["brute", "brute_stream"]
    scene, bounces = build_config("c2_rtiow", width=64, height=48)
    with Renderer(scene) as r:  # no triangles: mode 2 has no records to stream and runs mode 1's sweep
        r.set_brute_force(2)
        r.compute_frame(bounces)
        r.synchronize()
        assert r.last_launch_passes() == ["brute"]


@pytest.mark.parametrize("qnodes,primary", [("1", "0"), ("0", "0"), ("1", "1")])
def test_gpu_quantized_triangle_nodes(gpu, oracle_lib, qnodes, primary):
    """Walks of the binary triangle accelerator from global memory read its 16-B quantized
    copy (tri_qnode.h: boxes rounded outward onto an exact f32 grid). Per-lane walk, and the
    primary pre-pass beside it: the oracle's result either way."""
    tuning = {"tri_qnodes": int(qnodes), "primary_pass": int(primary)}
    scene, bounces = build_config("c5_heightfield", width=64, height=48, nx=200, nz=100)
    rays = scene.camera.recalculate_ray_directions()
    acc, out, n = gpu_render(scene, bounces, 2, rays=rays, tuning=tuning)
    with Renderer(scene, camera_rays=rays, tuning=tuning) as r:
        r.compute_frame(bounces)
        assert r.launch_config()["scene_in_lds"] <= 1  # the accelerator in global memory
    o = oracle_lib.Oracle(scene, camera_rays=rays)
    acc_o = np.zeros((48, 64, 4), np.float32)
    out_o = np.zeros((48, 64), np.uint32)
    n_o = sum(o.render_frame(scene.params(accumulation_index=k), bounces, acc_o, out_o) for k in (1, 2))
    assert_same(acc, out, n, acc_o, out_o, n_o)


@pytest.mark.parametrize("prune,octants,primary", [("1", "1", "0"), ("1", "0", "0"), ("1", "1", "1"),
                                                   ("0", "1", "0"), ("2", "1", "0"), ("2", "1", "1")])
def test_gpu_triangle_pruning(gpu, oracle_lib, prune, octants, primary):
    """Distance pruning of the triangle walk over the direction-ordered layouts (DESIGN.md
    §5.3c): certified (1, default), none (0), the round-3 relative slack (2); per-lane walk
    and primary pre-pass, and each switch alone: the oracle's result on this scene."""
    scene, bounces = build_config("c5_heightfield", width=64, height=48, nx=200, nz=100)
    rays = scene.camera.recalculate_ray_directions()
    acc, out, n = gpu_render(scene, bounces, 2, rays=rays, prune=int(prune),
                             tuning={"tri_octants": int(octants), "primary_pass": int(primary)})
    o = oracle_lib.Oracle(scene, camera_rays=rays)
    acc_o = np.zeros((48, 64, 4), np.float32)
    out_o = np.zeros((48, 64), np.uint32)
    n_o = sum(o.render_frame(scene.params(accumulation_index=k), bounces, acc_o, out_o) for k in (1, 2))
    assert_same(acc, out, n, acc_o, out_o, n_o)


def test_gpu_environment_has_no_effect(gpu, oracle_lib, monkeypatch):
    """The library reads no environment (ABI 12): with the round-1..5 switches set
    -- among them RT_TRI_PRUNE=2, the inexact pruning, and RT_BRUTE_FORCE=1 -- a default context
    on a small C5 heightfield launches the default kernels (the path kernel and the primary
    pre-pass, scene in LDS mode 1) and renders the oracle's bits."""
    for k, v in {"RT_TRI_PRUNE": "2", "RT_BRUTE_FORCE": "1", "RT_LDS_MODE": "0", "RT_PRIMARY_PASS": "0",
                 "RT_FRAME_BATCH": "1", "RT_TRI_OCTANTS": "0", "RT_COOP_LEAVES": "0", "RT_TRI_BVH": "0"}.items():
        monkeypatch.setenv(k, v)
    scene, bounces = build_config("c5_heightfield", width=64, height=48, nx=200, nz=100)
    rays = scene.camera.recalculate_ray_directions()
    with Renderer(scene, camera_rays=rays) as r:
        assert r.frame_batch()[0] == N.RT_DEFAULT_FRAME_BATCH
        r.compute_frame(bounces)
        r.synchronize()
        assert r.last_launch_passes() == ["path", "primary"]
        assert r.launch_config()["scene_in_lds"] == 1
        r.compute_frame(bounces)
        acc, out, n = r.read_accumulation(), r.read_output(), r.ray_count()
    assert_same(acc, out, n, *oracle_frames(oracle_lib, scene, bounces, 2, rays))


def test_gpu_tuning_keys_refuse_bad_input(gpu):
    """rt_set_tuning refuses unknown keys and out-of-range values (RT_E_INVALID), and
    rt_copy_output_to_device refuses host memory and rank contexts."""
    scene, bounces = build_config("c2_rtiow", width=64, height=48)
    with Renderer(scene) as r:
        for key, value in (("no_such_key", 1), ("lds_mode", 3), ("block_threads", 300), ("queue_stripes", 0),
                           ("primary_pass", 2), ("batch_memory_mb", 0)):
            with pytest.raises(RtError) as e:
                r.set_tuning(key, value)
            assert e.value.code == N.RT_E_INVALID
        host = np.zeros(64 * 48, np.uint32)
        with pytest.raises(RtError):
            r.copy_output_to_device(host.ctypes.data, 4 * 64)
    with Renderer(scene, rank=1, world_size=2) as r:
        import torch

        dev = torch.zeros(64 * 48, dtype=torch.int32, device="cuda")
        with pytest.raises(RtError):
            r.copy_output_to_device(dev.data_ptr(), 4 * 64)


def test_gpu_leaf_certificates_match_host(gpu):
    """The leaf certificates the device builds (rt_tri_leafcert_kernel) are bit for bit the
    host's (tri_cone.h, the CPU harness's builder), and every C5 leaf carries one."""
    scene, bounces = build_config("c5_heightfield", width=64, height=48, nx=200, nz=100)
    with Renderer(scene) as r:
        r.set_triangle_pruning(1)
        r.compute_frame(bounces)
        r.synchronize()
        mism, valid, total = r.check_leaf_certificates()
        assert total == len(scene.flatten()[1]) and mism == 0 and valid == total, (mism, valid, total)


@pytest.mark.parametrize("config,kw,frames", [
    ("c5_heightfield", {}, 6),
    ("c3_chess", {}, 20),
    ("c4_mixed", dict(width=1920, height=1080), 10),
])
def test_gpu_triangle_pruning_full_frames(gpu, config, kw, frames):
    """At BASELINE size the certified pruned walk (default), box culling alone
    (rt_set_triangle_pruning 0) and the round-3 relative slack (2) give the same
    accumulation bit for bit, frame after frame, on these scenes."""
    scene, bounces = build_config(config, **kw)
    res = []
    for prune in (0, 1, 2):
        with Renderer(scene, frame_batch=frames) as r:
            r.set_triangle_pruning(prune)
            for _ in range(frames):
                r.compute_frame(bounces)
            res.append((r.read_accumulation(), r.read_output(), r.ray_count()))
    a0, o0, n0 = res[0]
    for a1, o1, n1 in res[1:]:
        assert n1 == n0
        assert np.array_equal(o1, o0)
        assert np.array_equal(a1.view(np.uint32), a0.view(np.uint32))


@pytest.mark.parametrize("prune,primary", [("1", "0"), ("1", "1"), ("0", "0")])
def test_gpu_grazing_rays_certified_pruning(gpu, oracle_lib, prune, primary):
    """Adversarial primary rays (tests/adversarial.py): the camera 1e-4 from a tilted plane
    of 12,800 triangles, every direction within 1e-6..1e-3 rad of that plane after the
    kernel's own jitter (:217-219, cancelled per pixel), so the reference's f32 distances and
    barycentrics are rounding-dominated; then the paths' bounces. The certified walk
    (default) and box culling must give the oracle's result bit for bit, with and without
    the primary pre-pass."""
    from rust_gpu_raytracing_amd.camera import Camera
    from tests.adversarial import grazing_directions, tilted_plane_grid

    w, h = 64, 48
    scene, bounces = build_config("c1_four_spheres", width=w, height=h)
    _, _, _, obj, frame = tilted_plane_grid(3, n=80, size=0.1)
    scene.objects = [obj]
    p0, e1, e2, nrm = frame
    origin = (p0 - 1e-4 * nrm).astype(np.float32)
    scene.camera = Camera(w, h, position=origin)
    rays = scene.camera.recalculate_ray_directions()
    want = grazing_directions(frame, w * h, (1e-6, 1e-3), np.random.default_rng(4)).astype(np.float32)
    for i in range(w * h):  # frame k = 1: seed = index * 1 * 326624; jitter x, y, z (:219)
        s = (i * 326624) & 0xFFFFFFFF
        jit = []
        for _ in range(3):
            s, r01 = _pcg_f32(s)
            jit.append((r01 * np.float32(2.0) - np.float32(1.0)) * np.float32(0.0005))
        rays["direction"][i] = want[i] - np.array(jit, np.float32)
    o = oracle_lib.Oracle(scene, camera_rays=rays)
    acc_o = np.zeros((h, w, 4), np.float32)
    out_o = np.zeros((h, w), np.uint32)
    rays_o = o.render_frame(scene.params(accumulation_index=1), bounces, acc_o, out_o)
    acc, out, n = gpu_render(scene, bounces, 1, rays=rays, prune=int(prune), tuning={"primary_pass": int(primary)})
    assert_same(acc, out, n, acc_o, out_o, rays_o)


def test_gpu_update_scene_and_reset(gpu, oracle_lib):
    scene, bounces = build_config("c3_chess", width=96, height=64, env_size=(512, 256))
    with Renderer(scene) as r:
        r.compute_frame(bounces)
        r.compute_frame(bounces)
        assert r.accumulation_index == 3
        scene.spheres["position"][:, 1] -= np.float32(0.5)
        scene.materials["emission_power"][2] = np.float32(9.0)
        scene.objects[3].object_info["material_index"] = 5
        r.update_scene()  # resets accumulation to k = 1 (src/renderer.rs:153-154)
        assert r.accumulation_index == 1
        r.reset_ray_count()
        r.compute_frame(bounces)
        acc, out, rays = r.read_accumulation(), r.read_output(), r.ray_count()
    acc_o, out_o, rays_o = oracle_lib.render_frames(scene, bounces, 1)
    assert_same(acc, out, rays, acc_o, out_o, rays_o)


@pytest.mark.parametrize("config,kw", [
    ("c3_chess", dict(width=96, height=64, env_size=(512, 256))),
    ("c5_heightfield", dict(width=64, height=48, nx=60, nz=30)),
])
def test_gpu_device_scene_edit(gpu, oracle_lib, config, kw):
    """update_scene on the device: every object rotated, scaled and
    moved; triangles, object and sub-object bounds rebuilt by scene_edit.hip and
    the accelerator refitted. Geometry must equal the host rebuild bit for bit
    (update_triangles + update_sub_objects, src/triangle_object.rs:129-150,
    :199-220) and the frames must equal the oracle's on the edited scene."""
    from rust_gpu_raytracing_amd import builder

    scene, bounces = build_config(config, **kw)
    rng = np.random.default_rng(5)
    with Renderer(scene) as r:
        r.compute_frame(bounces)
        for step in range(2):  # two edits in a row: the second refits a refitted tree
            for o in scene.objects:
                o.rotation = (rng.random(3) * 40 - 20).astype(np.float32)
                o.scale = np.float32(0.8 + 0.4 * rng.random())
                o.transformation = (np.asarray(o.transformation) + rng.random(3) - 0.5).astype(np.float32)
            # a non-geometry ObjectInfo field must reach the device too (src/renderer.rs:188-193)
            scene.objects[0].object_info["material_index"] = (int(scene.objects[0].object_info["material_index"])
                                                              + 1 + step) % scene.materials.shape[0]
            r.update_scene(device=True)
            r.compute_frame(bounces)
        geo = r.read_geometry()
        r.reset_accumulation()
        r.reset_ray_count()
        for _ in range(2):
            r.compute_frame(bounces)
        acc, out, rays = r.read_accumulation(), r.read_output(), r.ray_count()
    for o in scene.objects:
        builder.update_object(o)
    objs, subs, tris = scene.flatten()
    assert geo[0].tobytes() == objs.tobytes()
    assert geo[1].tobytes() == subs.tobytes()
    assert geo[2].tobytes() == tris.tobytes()
    acc_o, out_o, rays_o = oracle_lib.render_frames(scene, bounces, 2)
    assert_same(acc, out, rays, acc_o, out_o, rays_o)


def test_gpu_device_edit_then_host_rebuild(gpu, oracle_lib):
    """A device edit followed by a change that forces the host to rebuild the
    accelerator (fewer objects in Params): the host reads the device geometry
    back first."""
    from rust_gpu_raytracing_amd import builder

    scene, bounces = build_config("c3_chess", width=64, height=48, env_size=(512, 256))
    with Renderer(scene) as r:
        for o in scene.objects[:5]:
            o.rotation = np.array([0.0, 30.0, 0.0], np.float32)
        r.update_scene(device=True)
        scene.objects = scene.objects[:20]  # Params.object_count 34 -> 20
        r.reset_accumulation()
        r.reset_ray_count()
        r.compute_frame(bounces)
        acc, out, rays = r.read_accumulation(), r.read_output(), r.ray_count()
    for o in scene.objects:
        builder.update_object(o)
    acc_o, out_o, rays_o = oracle_lib.render_frames(scene, bounces, 1)
    assert_same(acc, out, rays, acc_o, out_o, rays_o)


def test_gpu_device_edit_full_size_heightfield(gpu):
    """C5 at full size (1M triangles): the device rebuild equals the host one bit for bit."""
    from rust_gpu_raytracing_amd import builder

    scene, _ = build_config("c5_heightfield", width=64, height=32)
    o = scene.objects[0]
    o.rotation = np.array([3.0, -7.0, 11.0], np.float32)
    o.scale = np.float32(1.5)
    o.transformation = np.array([0.25, -1.0, 2.0], np.float32)
    with Renderer(scene) as r:
        r.update_objects()
        geo = r.read_geometry()
    builder.update_object(o)
    objs, subs, tris = scene.flatten()
    assert geo[0].tobytes() == objs.tobytes()
    assert geo[1].tobytes() == subs.tobytes()
    assert geo[2].tobytes() == tris.tobytes()


def test_gpu_camera_move(gpu, oracle_lib):
    from rust_gpu_raytracing_amd.camera import Camera

    scene, bounces = build_config("c1_four_spheres", width=80, height=64)
    with Renderer(scene) as r:
        r.compute_frame(bounces)
        cam = Camera(80, 64, position=np.array([1.0, -5.0, 20.0], np.float32))
        r.update_camera(cam)
        r.reset_ray_count()
        r.compute_frame(bounces)
        acc, out, rays = r.read_accumulation(), r.read_output(), r.ray_count()
    acc_o, out_o, rays_o = oracle_lib.render_frames(scene, bounces, 1)
    assert_same(acc, out, rays, acc_o, out_o, rays_o)


def test_gpu_empty_scene_and_ragged_size(gpu, oracle_lib):
    scene, _ = build_config("c1_four_spheres", width=13, height=7)
    scene.spheres = scene.spheres[:0]
    acc_o, out_o, rays_o = oracle_lib.render_frames(scene, 4, 2)
    acc, out, rays = gpu_render(scene, 4, 2)
    assert rays == rays_o == 2 * 13 * 7  # every path escapes on its first segment
    assert_same(acc, out, rays, acc_o, out_o, rays_o)


def test_gpu_display_readback_any_width(gpu, tmp_path):
    """update_texture/calculate_bytes_per_row (src/renderer.rs:254-295) headless: a
    width that is not a multiple of 64 px (the reference's constraint,
    src/main.rs:51-53), each row at the 256-B pitch, padding untouched."""
    from rust_gpu_raytracing_amd import image_io
    scene, bounces = build_config("c1_four_spheres", width=100, height=37)
    with Renderer(scene) as r:
        r.compute_frame(bounces)
        out = r.read_output()
        staged = r.update_texture()
        img = r.image()
        odd = r.update_texture(alignment=4)
        with pytest.raises(ValueError):
            r.update_texture(alignment=100)
    assert staged.shape == (37, 512)
    assert np.array_equal(staged[:, :400].copy().view("<u4"), out)
    assert not staged[:, 400:].any()
    assert np.array_equal(odd.view("<u4"), out)
    assert np.array_equal(img, image_io.unpack_rgba8(out))
    assert np.array_equal(image_io.load_png(image_io.save_png(tmp_path / "f.png", img)), img)


def test_gpu_one_pixel(gpu, oracle_lib):
    scene, bounces = build_config("c1_four_spheres", width=1, height=1)
    acc_o, out_o, rays_o = oracle_lib.render_frames(scene, bounces, 3)
    assert_same(*gpu_render(scene, bounces, 3), acc_o, out_o, rays_o)


def test_gpu_scene_beyond_lds_budget(gpu, oracle_lib):
    """Scenes whose spheres+materials+objects exceed the 64 KiB LDS budget take the
    global-memory variant of the kernel; results are unchanged."""
    scene, bounces = build_config("c2_rtiow", width=64, height=40)
    reps = 8
    sph = np.concatenate([scene.spheres] * reps)
    for i in range(1, reps):  # copies far behind the camera: same image, 5x the sphere loop
        seg = slice(i * scene.spheres.shape[0], (i + 1) * scene.spheres.shape[0])
        sph["position"][seg, 2] -= np.float32(200.0 * i)
    scene.spheres = sph
    assert scene.spheres.shape[0] * 16 + scene.materials.shape[0] * 32 > 64 * 1024
    acc_o, out_o, rays_o = oracle_lib.render_frames(scene, bounces, 1)
    assert_same(*gpu_render(scene, bounces, 1), acc_o, out_o, rays_o)


def test_gpu_capacity_and_validation(gpu):
    scene, _ = build_config("c1_four_spheres", width=16, height=16)
    with Renderer(scene) as r:
        more = np.concatenate([scene.spheres, scene.spheres])
        with pytest.raises(RtError) as e:
            r._call("rt_update_spheres", N.ptr(more), more.shape[0])
        assert e.value.code == N.RT_E_CAPACITY
        p = scene.params()
        p["sphere_count"] = 99
        with pytest.raises(RtError) as e:
            r._call("rt_update_params", N.params_struct(p))
        assert e.value.code == N.RT_E_INVALID


def test_gpu_determinism_and_timing(gpu):
    scene, bounces = build_config("c2_rtiow", width=256, height=144)
    with Renderer(scene, frame_batch=1) as r:  # one timed launch per frame
        r.set_timing(True)
        for _ in range(3):
            r.compute_frame(bounces)
        ms, n = r.dispatch_time_total()
        a1 = r.read_accumulation()
    assert n == 3 and ms > 0
    a2, _, _ = gpu_render(scene, bounces, 3)
    assert np.array_equal(a1.view(np.uint32), a2.view(np.uint32))


@pytest.mark.parametrize("config,spp,accumulate,frames,kw", [
    ("c2_rtiow", 1, 1, 4, {}),
    ("c3_chess", 3, 1, 3, dict(env_size=(512, 256))),
    ("c1_four_spheres", 1, 0, 3, {}),
])
def test_gpu_multi_frame_launch(gpu, config, spp, accumulate, frames, kw):
    """rt_compute_frames(b, F) == F x rt_compute_frame(b), bit for bit (the fused launch the
    multi-GPU bench uses), also after ordinary frames and with a tile split."""
    scene, bounces = build_config(config, width=96, height=56, **kw)
    acc1, out1, rays1 = gpu_render(scene, bounces, 1 + frames, spp=spp, accumulate=accumulate)
    with Renderer(scene, accumulate=bool(accumulate), compute_per_frame=spp) as r:
        r.compute_frame(bounces)
        r.compute_frames(bounces, frames)
        assert r.accumulation_index == (1 + (1 + frames) if accumulate else 1)
        acc, out, rays = r.read_accumulation(), r.read_output(), r.ray_count()
    assert rays == rays1
    assert np.array_equal(out, out1) and np.array_equal(acc.view(np.uint32), acc1.view(np.uint32))
    world, total = 2, 0
    for rank in range(world):
        with Renderer(scene, accumulate=bool(accumulate), compute_per_frame=spp, rank=rank, world_size=world) as r:
            r.compute_frames(bounces, 1 + frames)
            total += r.ray_count()
    assert total == rays1


@pytest.mark.parametrize("config,w,h", [("c2_rtiow", 1920, 1080), ("c3_chess", 13, 7), ("c1_four_spheres", 800, 600)])
def test_gpu_device_camera_rays(gpu, config, w, h):
    """Device-side primary rays (rt_update_camera_matrices) == the host generator's ray buffer
    (src/camera.rs:139-182 restated in camera.py), bit for bit, through a whole frame."""
    kw = dict(env_size=(256, 128)) if config == "c3_chess" else {}
    scene, bounces = build_config(config, width=w, height=h, **kw)
    host = scene.camera.recalculate_ray_directions()
    a1, o1, r1 = gpu_render(scene, bounces, 1, rays=host)
    with Renderer(scene, device_rays=True) as r:
        r.compute_frame(bounces)
        a2, o2, r2 = r.read_accumulation(), r.read_output(), r.ray_count()
    assert r1 == r2
    assert np.array_equal(o1, o2) and np.array_equal(a1.view(np.uint32), a2.view(np.uint32))


@pytest.mark.parametrize("config,kw", [("c3_chess", dict(env_size=(512, 256))), ("c5_heightfield", dict(nx=40, nz=20))])
def test_gpu_reference_sweep_without_accelerator(gpu, oracle_lib, config, kw):
    """Tuning "tri_bvh" 0: the kernel walks the reference's own object -> sub-object -> triangle
    sweep, same results as the oracle."""
    scene, bounces = build_config(config, width=64, height=40, **kw)
    acc_o, out_o, rays_o = oracle_lib.render_frames(scene, bounces, 2)
    assert_same(*gpu_render(scene, bounces, 2, tuning={"tri_bvh": 0}), acc_o, out_o, rays_o)


@pytest.mark.parametrize("tuning", [
    {"coop_leaves": 0},
    {"block_threads": 256},
    {"primary_pass": 0, "prune": 0},
    {"tri_octants": 0, "tri_qnodes": 0},
    {"leaf_batch": 8, "trav_threshold": 63, "drain_threshold": 0},
])
@pytest.mark.parametrize("config,kw", [("c4_mixed", dict(env_size=(256, 128))), ("c5_heightfield", dict(nx=60, nz=30)),
                                       ("c3_chess", dict(env_size=(512, 256)))])
def test_gpu_global_walk_variants(gpu, oracle_lib, config, kw, tuning):
    """The walks from global memory (scene not staged in LDS: tuning "lds_mode" 1): per-lane leaf
    tests instead of the cooperative leaf batches, 256-thread workgroups, box culling without the
    primary pre-pass, one layout of 32-B nodes, extreme schedule thresholds: the oracle's images
    and ray counts."""
    scene, bounces = build_config(config, width=96, height=64, **kw)
    tuning = dict(tuning, lds_mode=1)
    prune = tuning.pop("prune", None)
    with Renderer(scene, tuning=tuning) as r:
        r.compute_frame(bounces)
        assert r.launch_config()["scene_in_lds"] <= 1
    acc_o, out_o, rays_o = oracle_lib.render_frames(scene, bounces, 2)
    assert_same(*gpu_render(scene, bounces, 2, prune=prune, tuning=tuning), acc_o, out_o, rays_o)


@pytest.mark.parametrize("tuning", [
    {},
    {"trav_threshold": 1},            # traverse (almost) to the end before shading
    {"trav_threshold": 63},           # back to shading after every block
    {"leaf_batch": 1},                # triangle leaf batches as soon as one lane waits
    {"leaf_batch": 8},                # ... only once every traversing lane waits
    {"sphere_leaf": 1},               # one sphere per BVH leaf: a leaf at nearly every step
    {"block_threads": 256, "batch_overlap": 0},
])
@pytest.mark.parametrize("config,kw", [("c1_four_spheres", {}), ("c2_rtiow", {}),
                                       ("c3_chess", dict(env_size=(512, 256))),
                                       ("c4_mixed", dict(env_size=(256, 128)))])
def test_gpu_leaf_scheduling_extremes(gpu, oracle_lib, config, kw, tuning):
    """Round 6's leaf scheduling: sphere-only walks wait at a leaf and test the waiting lanes'
    groups after a block of node steps (kBlockLeaves), and LDS-resident triangle walks run their
    leaf batch in the node-step iteration (kFusedLeaves). Under extreme shading and batch
    thresholds, one-sphere leaves and small workgroups, no lane waits forever (the launch
    ends) and every image and ray count is the oracle's."""
    scene, bounces = build_config(config, width=96, height=64, **kw)
    acc_o, out_o, rays_o = oracle_lib.render_frames(scene, bounces, 3)
    assert_same(*gpu_render(scene, bounces, 3, tuning=tuning, frame_batch=3), acc_o, out_o, rays_o)


@pytest.mark.parametrize("config,kw,spp,accumulate,batch,world,env", [
    ("c3_chess", dict(env_size=(512, 256)), 2, 1, 3, 1, {"primary_pass": 1}),
    ("c3_chess", dict(env_size=(512, 256)), 1, 0, 3, 1, {"primary_pass": 1}),  # non-accumulating batch
    ("c4_mixed", dict(env_size=(256, 128)), 1, 1, 4, 3, {"primary_pass": 1}),  # tile split
    ("c5_heightfield", dict(nx=60, nz=30), 1, 1, 2, 1, {"frame_parallel": 0, "primary_pass": 1}),
    ("c5_heightfield", dict(nx=60, nz=30), 1, 1, 1, 1, {"primary_pass": 1, "lds_mode": 1}),
    ("c5_heightfield", dict(nx=200, nz=100), 1, 1, 2, 1, {}),       # default: on (accelerator in global memory)
    # pre-pass workgroup sizes and unit orders (the default is 256 threads held to 64 VGPRs)
    ("c5_heightfield", dict(nx=200, nz=100), 1, 1, 3, 1, {"primary_threads": 64, "primary_tile_major": 0}),
    ("c5_heightfield", dict(nx=200, nz=100), 2, 1, 3, 2, {"primary_threads": 1024, "primary_tile_major": 1}),
    ("c5_heightfield", dict(nx=200, nz=100), 1, 1, 3, 1, {"primary_waves": 0}),
    # a batch budget of 1 MB: the batches run as consecutive launches of the
    # frames whose lights and primary records fit
    ("c5_heightfield", dict(nx=200, nz=100), 2, 1, 3, 1, {"batch_memory_mb": 1}),
    ("c3_chess", dict(env_size=(512, 256)), 1, 1, 4, 3, {"batch_memory_mb": 1}),
])
def test_gpu_primary_pass(gpu, oracle_lib, config, kw, spp, accumulate, batch, world, env):
    """rt_primary_kernel traces every path's first segment as 8x8 packets (wave-uniform
    node walk, per-lane culling and exact leaf tests); the path kernel starts from its
    records. Results must equal the oracle's (and therefore the per-lane walk's) in
    batches, with several samples, without accumulation and in tile splits."""
    scene, bounces = build_config(config, width=96, height=64, **kw)
    rays = scene.camera.recalculate_ray_directions()
    o = oracle_lib.Oracle(scene, camera_rays=rays)
    acc_o = np.zeros((64, 96, 4), np.float32)
    out_o = np.zeros((64, 96), np.uint32)
    n_o = 0
    for k in range(1, 5):
        n_o += o.render_frame(scene.params(accumulate=accumulate, compute_per_frame=spp,
                                           accumulation_index=k if accumulate else 1), bounces, acc_o, out_o)
    acc = np.zeros_like(acc_o)
    out = np.zeros_like(out_o)
    n = 0
    for rank in range(world):
        with Renderer(scene, camera_rays=rays, frame_batch=batch, rank=rank, world_size=world,
                      compute_per_frame=spp, accumulate=bool(accumulate), tuning=env) as r:
            for _ in range(4):
                r.compute_frame(bounces)
            a, oo, k = r.read_accumulation(), r.read_output(), r.ray_count()
        mask = owned_mask(96, 64, rank, world)
        acc[mask] = a[mask]
        out[mask] = oo[mask]
        n += k
    if accumulate:
        assert_same(acc, out, n, acc_o, out_o, n_o)
    else:
        assert n == n_o and np.array_equal(out, out_o)


@pytest.mark.parametrize("config,kw,batch,world", [
    ("c1_four_spheres", {}, 1, 1),
    ("c2_rtiow", {}, 3, 1),
    ("c3_chess", dict(env_size=(512, 256)), 1, 1),
    ("c4_mixed", dict(env_size=(256, 128)), 2, 3),
    ("c5_heightfield", dict(nx=60, nz=30), 2, 1),
])
@pytest.mark.parametrize("mode", [1, 2])
def test_gpu_brute_force_mode(gpu, oracle_lib, config, kw, batch, world, mode):
    """rt_set_brute_force: the reference's own sphere and object -> sub-object ->
    triangle sweeps, sub-objects streamed through LDS tiles (BASELINE config 5's
    stress mode) -- bit-identical to the oracle, in frame batches and tile splits: the
    wavefront over compacted queues of live paths (rt_brute_wf_kernel), the sub-object records
    LDS-tiled, or streamed through the scalar cache with rt_set_brute_force(ctx, 2)."""
    scene, bounces = build_config(config, width=96, height=64, **kw)
    rays = scene.camera.recalculate_ray_directions()
    acc_o, out_o, n_o = oracle_frames(oracle_lib, scene, bounces, 4, rays)
    acc = np.zeros_like(acc_o)
    out = np.zeros_like(out_o)
    n = 0
    streamed = 0
    for rank in range(world):
        with Renderer(scene, camera_rays=rays, frame_batch=batch, rank=rank, world_size=world) as r:
            r.set_brute_force(mode)
            for _ in range(4):
                r.compute_frame(bounces)
            a, o, k = r.read_accumulation(), r.read_output(), r.ray_count()
            streamed += r.streamed_bytes()
        mask = owned_mask(96, 64, rank, world)
        acc[mask] = a[mask]
        out[mask] = o[mask]
        n += k
    assert_same(acc, out, n, acc_o, out_o, n_o)
    assert (streamed > 0) == bool(scene.objects)


@pytest.mark.parametrize("config,kw,spp,accumulate,batch,bounces,mode", [
    ("c2_rtiow", {}, 3, 1, 2, None, 1),
    ("c5_heightfield", dict(nx=40, nz=20), 2, 1, 3, None, 1),
    ("c5_heightfield", dict(nx=40, nz=20), 2, 1, 3, None, 2),
    ("c3_chess", dict(env_size=(512, 256)), 1, 0, 3, None, 2),
    ("c4_mixed", dict(env_size=(256, 128)), 1, 1, 1, 0, 1),
    ("c1_four_spheres", {}, 1, 1, 2, 40, 1),
    ("c5_heightfield", dict(nx=40, nz=20), 1, 1, 2, 80, 2),  # beyond round 5's 62-bounce limit
    ("c2_rtiow", {}, 1, 1, 2, None, 2),  # no triangles: mode 2 runs mode 1's sweep
])
def test_gpu_brute_force_samples_and_modes(gpu, oracle_lib, config, kw, spp, accumulate, batch, bounces, mode):
    """The brute-force wavefront's passes: several samples per frame (each pass = one (frame,
    sample), summed in that order per pixel), accumulation off (the last frame's image), zero
    bounces (no launch traces; the image is written from the empty paths), and a deep bounce
    limit (the queue levels): the oracle's images and ray counts."""
    scene, b0 = build_config(config, width=80, height=48, **kw)
    bounces = b0 if bounces is None else bounces
    rays = scene.camera.recalculate_ray_directions()
    with Renderer(scene, accumulate=bool(accumulate), compute_per_frame=spp, camera_rays=rays,
                  frame_batch=batch) as r:
        r.set_brute_force(mode)
        with pytest.raises(Exception):
            r.set_brute_force(3)  # RT_E_INVALID
        for _ in range(3):
            r.compute_frame(bounces)
        got = r.read_accumulation(), r.read_output(), r.ray_count()
        assert r.last_launch_passes() == (["brute", "brute_stream"] if mode == 2 and scene.objects else ["brute"])
    o = oracle_lib.Oracle(scene, camera_rays=rays)
    acc = np.zeros((48, 80, 4), np.float32)
    out = np.zeros((48, 80), np.uint32)
    n = 0
    for i in range(3):
        k = i + 1 if accumulate else 1
        n += o.render_frame(scene.params(accumulate=accumulate, compute_per_frame=spp, accumulation_index=k),
                            bounces, acc, out)
    if accumulate:
        assert_same(*got, acc, out, n)
    else:
        assert got[2] == n and np.array_equal(got[1], out)


def _pcg_f32(seed):
    state = (seed * 747796405 + 2891336453) & 0xFFFFFFFF
    word = (((state >> ((state >> 28) + 4)) ^ state) * 277803737) & 0xFFFFFFFF
    seed = ((word >> 22) ^ word) & 0xFFFFFFFF
    return seed, np.float32(seed) / np.float32(4294967296.0)


@pytest.mark.parametrize("primary", ["0", "1"])
def test_gpu_in_plane_rays_nan_distance(gpu, oracle_lib, primary):
    """Rays lying exactly in a triangle's plane (det == 0, origin on the plane) give a NaN
    distance that the reference's sweep accepts (:449-481, :457); the accelerator hands such
    lanes to the sweep itself. Primary directions are chosen so that d.y + jitter.y == 0
    exactly (the jitter is the kernel's own PCG draw, :217-219). Such a hit has NaN
    barycentrics too, which pass the reference's `< 0` rejections (:467-481). With and
    without the primary pre-pass."""
    from rust_gpu_raytracing_amd.camera import Camera
    from rust_gpu_raytracing_amd.scene import SceneObject

    scene, bounces = build_config("c1_four_spheres", width=48, height=32)
    y0 = np.float32(0.5)
    a = np.array([[-1, y0, -1], [1, y0, -1]], np.float32)
    b = np.array([[1, y0, -1], [1, y0, 1]], np.float32)
    c = np.array([[-1, y0, 1], [-1, y0, 1]], np.float32)
    info = np.zeros((), B.OBJECT_INFO)
    info["min_bounds"] = [-1, y0, -1]
    info["max_bounds"] = [1, y0, 1]
    obj = SceneObject(info, B.scene_triangles(a, b, c))
    obj.create_sub_objects(0, 0)
    scene.objects = [obj]
    scene.camera = Camera(48, 32, position=np.array([0.0, y0, 4.0], np.float32))
    rays = scene.camera.recalculate_ray_directions()
    for i in range(rays.shape[0]):  # frame k = 1: seed = index * 1 * 326624
        s = (i * 326624) & 0xFFFFFFFF
        s, _ = _pcg_f32(s)
        s, ry = _pcg_f32(s)
        jy = (ry * np.float32(2.0) - np.float32(1.0)) * np.float32(0.0005)
        rays["direction"][i, 1] = -jy
    o = oracle_lib.Oracle(scene, camera_rays=rays)
    acc_o = np.zeros((32, 48, 4), np.float32)
    out_o = np.zeros((32, 48), np.uint32)
    rays_o = o.render_frame(scene.params(accumulation_index=1), bounces, acc_o, out_o)
    acc, out, n = gpu_render(scene, bounces, 1, rays=rays, tuning={"primary_pass": int(primary)})
    assert_same(acc, out, n, acc_o, out_o, rays_o)


@pytest.mark.parametrize("which,name", [(0, "sqrt on {0} U [2^-96, inf]"), (1, "x / 2pi"), (2, "x / pi"),
                                        (3, "x / 255"), (4, "x / 10"), (5, "Box-Muller log on random01's range"),
                                        (6, "Box-Muller cos on 2pi * random01's range")])
def test_gpu_fast_exact_math_selftest(gpu, which, name):
    """The kernel's short correctly-rounded sqrt and constant divisions equal the IEEE
    operations bit for bit over every f32 input of their domain (exhaustive, on the device)."""
    import ctypes

    lib = N.load_library()
    bad, first = ctypes.c_uint64(), ctypes.c_uint32()
    assert lib.rt_math_selftest(which, ctypes.byref(bad), ctypes.byref(first)) == 0
    assert bad.value == 0, (name, bad.value, hex(first.value))


def test_gpu_device_edit_models_invalidated_by_range_change(gpu):
    """rt_set_object_models' triangle maps follow the object / sub-object ranges: once
    rt_update_sub_object_info changes a range, rt_update_objects refuses until the models
    are set again (rather than writing the wrong triangles)."""
    from rust_gpu_raytracing_amd import builder

    scene, bounces = build_config("c3_chess", width=32, height=24, env_size=(256, 128))
    with Renderer(scene) as r:
        r.update_objects()  # uploads the models
        _, subs, _ = scene.flatten()
        same = np.ascontiguousarray(subs.copy())
        r._call("rt_update_sub_object_info", N.ptr(same), same.shape[0])  # ranges unchanged: still valid
        r.update_objects()
        changed = same.copy()
        changed["triangle_count"][-1] -= 1
        r._call("rt_update_sub_object_info", N.ptr(changed), changed.shape[0])
        t = np.ascontiguousarray(np.stack([builder.transform_of(o) for o in scene.objects]))
        with pytest.raises(RtError):
            r._call("rt_update_objects", N.ptr(t), t.shape[0])


@pytest.mark.parametrize("overlap", ["1", "0"])
def test_gpu_overlapped_batches_with_updates(gpu, oracle_lib, overlap):
    """Consecutive frame-parallel batches alternate between two HIP streams (the path
    kernel of batch i overlaps batch i-1's drain; only its resolve waits for batch
    i-1's): results must equal the one-frame-at-a-time sequence, including when
    scene updates, a reset and readbacks are interleaved with queued batches."""
    scene, bounces = build_config("c2_rtiow", width=128, height=72)
    rays = scene.camera.recalculate_ray_directions()

    def run(batch):
        with Renderer(scene, camera_rays=rays, frame_batch=batch, tuning={"batch_overlap": int(overlap)}) as r:
            for _ in range(7):
                r.compute_frame(bounces)
            a1 = r.read_accumulation()
            scene.materials["emission_power"][1] = np.float32(3.0)
            r._call("rt_update_materials", N.ptr(scene.materials), scene.materials.shape[0])
            for _ in range(5):
                r.compute_frame(bounces)
            r.reset_accumulation()
            for _ in range(6):
                r.compute_frame(bounces)
            out = r.read_accumulation(), r.read_output(), r.ray_count()
        scene.materials["emission_power"][1] = base_e
        return a1, out

    base_e = scene.materials["emission_power"][1].copy()
    a1_ref, ref = run(1)
    a1, got = run(2)
    assert np.array_equal(a1.view(np.uint32), a1_ref.view(np.uint32))
    assert got[2] == ref[2] and np.array_equal(got[1], ref[1])
    assert np.array_equal(got[0].view(np.uint32), ref[0].view(np.uint32))
    # and the last six frames against the oracle (after the reset: k = 1..6, new material)
    scene.materials["emission_power"][1] = np.float32(3.0)
    try:
        acc_o, out_o, _ = oracle_frames(oracle_lib, scene, bounces, 6, rays)
    finally:
        scene.materials["emission_power"][1] = base_e
    assert np.array_equal(got[1], out_o) and np.array_equal(got[0].view(np.uint32), acc_o.view(np.uint32))


def test_gpu_overlapped_batch_after_plain_launch(gpu, oracle_lib):
    """A one-frame flush (a bounce change flushing a single queued frame) is a plain
    launch on the primary stream that reads and writes the accumulation; the next
    batch lands on the auxiliary stream and its resolve must wait for that launch too
    (primary_dirty after a plain launch). Sequence: batches on primary,
    aux, primary, then 1 frame at b, compute_frame(b + 1) flushing it alone, then a
    full batch at b + 1 on aux -- against the oracle's single frames."""
    scene, b = build_config("c2_rtiow", width=320, height=184)
    rays = scene.camera.recalculate_ray_directions()
    seq = [b] * 13 + [b + 1] * 4
    with Renderer(scene, camera_rays=rays, frame_batch=4, tuning={"batch_overlap": 1}) as r:
        for bb in seq:
            r.compute_frame(bb)
        got = r.read_accumulation(), r.read_output(), r.ray_count()
    o = oracle_lib.Oracle(scene, camera_rays=rays)
    acc = np.zeros((184, 320, 4), np.float32)
    out = np.zeros((184, 320), np.uint32)
    n = 0
    for i, bb in enumerate(seq):
        n += o.render_frame(scene.params(accumulation_index=i + 1), bb, acc, out)
    assert_same(*got, acc, out, n)


def _fuzz_scene(seed, w, h, with_tris):
    """A random scene that leans on the culling: clustered and far spheres, tiny and huge
    radii, duplicates and overlaps, every material kind, emitters; camera rays with exact
    zero, denormal and axis-aligned components next to random ones."""
    from rust_gpu_raytracing_amd.scene import RenderScene, _material, _sphere, solid_color_image
    from rust_gpu_raytracing_amd.camera import Camera

    rng = np.random.default_rng(seed)
    n = int(rng.integers(5, 600))
    pos = np.concatenate([rng.uniform(-8, 8, (n // 2, 3)),                          # a cluster
                          rng.normal(0, 40, (n - n // 2, 3))]).astype(np.float32)   # far ones
    rad = np.exp(rng.uniform(np.log(1e-3), np.log(3.0), n)).astype(np.float32)
    pos[0], rad[0] = (0.0, 1000.5, 0.0), 1000.0                                      # a ground
    if n > 8:
        pos[1], rad[1] = pos[2], rad[2]                                               # a duplicate (tie)
    n_mat = int(rng.integers(1, 12))
    mats = np.stack([_material(int(rng.integers(0, 3)), float(rng.uniform(0, 1)),
                               float(rng.choice([0.0, 0.0, 0.0, rng.uniform(0, 8)])),
                               float(rng.uniform(0, 1)), float(rng.uniform(0, 1)),
                               float(rng.choice([0.0, 1.0, rng.uniform(0, 1)])),
                               float(rng.uniform(1.0, 2.4))) for _ in range(n_mat)])
    spheres = np.stack([_sphere(pos[i], rad[i], int(rng.integers(0, n_mat))) for i in range(n)])
    tex = np.stack([solid_color_image(rng.uniform(0, 1, 3), (1, 1)) for _ in range(3)])
    env = np.ascontiguousarray((rng.uniform(0, 255, (16, 32, 4))).astype(np.uint8))
    objects = []
    if with_tris:
        hf, _ = build_config("c5_heightfield", width=w, height=h, nx=24, nz=12, seed=int(seed))
        objects = hf.objects
    cam = Camera(w, h, position=np.array(rng.uniform(-15, 15, 3), np.float32))
    scene = RenderScene(spheres.astype(B.SPHERE), mats.astype(B.MATERIAL), objects, tex, env, cam, name="fuzz")
    d = rng.normal(0, 1, (w * h, 3)).astype(np.float32)
    k = w * h // 8
    d[:k, int(seed) % 3] = 0.0                    # exact zero components
    d[k:2 * k, :2] = 0.0                          # axis-aligned
    d[2 * k:3 * k, 1] = np.float32(1e-40)         # denormal component
    rays = np.zeros(w * h, B.RAY)
    rays["direction"] = d
    return scene, rays


@pytest.mark.parametrize("seed,with_tris", [(s, False) for s in range(1, 25)] + [(s, True) for s in range(25, 35)])
def test_gpu_fuzz_scenes(gpu, oracle_lib, seed, with_tris):
    """Random scenes (see _fuzz_scene) rendered for 2 accumulated frames of 6 bounces:
    accumulation, output and ray count bit-identical to the oracle. Exercises the
    culling margins and the sphere-only kernels' v_rcp_f32 1/d on inputs no config has."""
    w, h = 48, 32
    scene, rays = _fuzz_scene(seed, w, h, with_tris)
    acc_o, out_o, rays_o = oracle_frames(oracle_lib, scene, 6, 2, rays)
    acc, out, n = gpu_render(scene, 6, 2, rays=rays)
    assert_same(acc, out, n, acc_o, out_o, rays_o)
