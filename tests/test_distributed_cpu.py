"""The N>1 path on CPU: world_size-2 (and 3) gloo process groups.

Each rank renders only its 8x8 tiles (oracle stands in for the kernel on CPU),
packs them exactly as rt_pack_tiles_kernel does, and the gather used by bench.py
(`gather_packed`) assembles them on rank 0; the result must equal a one-process
render bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from rust_gpu_raytracing_amd import distributed as D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, config, w, h, frames, q):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from rust_gpu_raytracing_amd.scene import build_config

        scene, bounces = build_config(config, width=w, height=h)
        acc, out, rays = O.render_frames(scene, bounces, frames, rank=rank, world_size=world, threads=2)
        packed = torch.from_numpy(D.pack_owned_host(acc, rank, world))
        tx, ty = D.tile_grid(w, h)
        parts = D.gather_packed(packed, tx * ty, rank, world, dst=0)
        # the "image" payload: the RGBA8 output words (as int32: gloo has no uint32)
        words = torch.from_numpy(D.pack_owned_host(out.view(np.int32), rank, world))
        word_parts = D.gather_packed(words, tx * ty, rank, world, dst=0)
        tot = torch.tensor([rays], dtype=torch.int64)
        dist.all_reduce(tot)
        if rank == 0:
            full = np.zeros_like(acc)
            for src, part in enumerate(parts):
                D.unpack_host(full, part.numpy(), src, world)
            image = np.zeros(out.shape, np.int32)
            for src, part in enumerate(word_parts):
                D.unpack_host(image, part.numpy(), src, world)
            q.put((full, image.view(np.uint32), int(tot.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,config,w,h", [(2, "c2_rtiow", 72, 40), (3, "c1_four_spheres", 61, 35)])
def test_gloo_tile_gather_matches_single_render(oracle_lib, world, config, w, h):
    from rust_gpu_raytracing_amd.scene import build_config

    frames = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, config, w, h, frames, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, image, rays = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    scene, bounces = build_config(config, width=w, height=h)
    acc1, out1, rays1 = oracle_lib.render_frames(scene, bounces, frames)
    assert rays == rays1
    assert np.array_equal(full.view(np.uint32), acc1.view(np.uint32))
    assert out1.any() and np.array_equal(image, out1)


def test_owned_pixels_partition_the_image():
    w, h = 45, 29  # ragged: partial edge tiles
    seen = np.zeros(w * h, int)
    for rank in range(4):
        idx = D.owned_pixel_indices(w, h, rank, 4)
        assert idx.shape[0] % 64 == 0
        seen[idx[idx >= 0]] += 1
    assert (seen == 1).all()


def test_pack_unpack_roundtrip_host():
    rng = np.random.default_rng(0)
    acc = rng.random((20, 33, 4)).astype(np.float32)
    out = np.zeros_like(acc)
    for r in range(3):
        D.unpack_host(out, D.pack_owned_host(acc, r, 3), r, 3)
    assert np.array_equal(out, acc)
    words = rng.integers(0, 2**32, (20, 33), dtype=np.uint64).astype(np.uint32)
    img = np.zeros_like(words)
    for r in range(3):
        packed = D.pack_owned_host(words, r, 3)
        assert packed.dtype == np.uint32 and packed.shape == (D.owned_pixel_indices(33, 20, r, 3).shape[0],)
        D.unpack_host(img, packed, r, 3)
    assert np.array_equal(img, words)


def test_tile_gather_payload_checks():
    """TileGather refuses an accumulation gather of a render that never writes one."""
    class FakeRenderer:
        accumulate = False
    with pytest.raises(ValueError):
        D.TileGather(FakeRenderer(), 0, "accumulation")
    with pytest.raises(ValueError):
        D.TileGather(FakeRenderer(), 0, "pixels")
