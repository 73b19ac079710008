"""Multi-GPU tile partition and the readback gather.

The reference renders on one adapter (src/main.rs:636-665). Here one process
drives one GPU; the frame is cut into 8x8-pixel tiles and tile t belongs to rank
t % world_size. Each rank's kernel launch renders only its tiles, using global
pixel indices for the RNG seeds (compute_shader.wgsl:217), so the assembled image
is bitwise identical to a 1-GPU render. Rendering needs no communication; at
readback every rank packs its tiles' RGBA32F accumulation into one contiguous
buffer (tile order, 64 pixels per tile) and one RCCL gather (torch.distributed,
backend "nccl") moves them to the destination rank, which unpacks them into its
framebuffer and re-packs the RGBA8 output.
"""
from __future__ import annotations

import numpy as np

TILE = 8


def tile_grid(width: int, height: int):
    return (width + TILE - 1) // TILE, (height + TILE - 1) // TILE


def owned_tiles(n_tiles: int, rank: int, world_size: int) -> np.ndarray:
    """Global tile ids of `rank`, in local order (local l -> global l * world + rank)."""
    return np.arange(rank, n_tiles, world_size, dtype=np.int64)


def max_owned_tiles(n_tiles: int, world_size: int) -> int:
    return (n_tiles + world_size - 1) // world_size


def owned_pixel_indices(width: int, height: int, rank: int, world_size: int) -> np.ndarray:
    """Row-major pixel index of every slot of the packed buffer (-1 outside the image)."""
    tx_n, ty_n = tile_grid(width, height)
    tiles = owned_tiles(tx_n * ty_n, rank, world_size)
    lane = np.arange(64)
    x = (tiles[:, None] % tx_n) * TILE + (lane[None, :] & 7)
    y = (tiles[:, None] // tx_n) * TILE + (lane[None, :] >> 3)
    idx = y * width + x
    idx[(x >= width) | (y >= height)] = -1
    return idx.reshape(-1)


def pack_owned_host(accum: np.ndarray, rank: int, world_size: int) -> np.ndarray:
    """Host mirror of rt_pack_tiles_kernel: (H, W, 4) f32 -> (owned_tiles*64, 4)."""
    h, w, _ = accum.shape
    idx = owned_pixel_indices(w, h, rank, world_size)
    out = np.zeros((idx.shape[0], 4), np.float32)
    ok = idx >= 0
    out[ok] = accum.reshape(-1, 4)[idx[ok]]
    return out


def unpack_host(accum: np.ndarray, packed: np.ndarray, src_rank: int, world_size: int) -> None:
    h, w, _ = accum.shape
    idx = owned_pixel_indices(w, h, src_rank, world_size)
    ok = idx >= 0
    accum.reshape(-1, 4)[idx[ok]] = packed[: idx.shape[0]][ok]


def gather_packed(packed, n_tiles: int, rank: int, world_size: int, dst: int = 0):
    """Gather every rank's packed tile buffer (torch tensor, owned*64 rows: (n, 4) f32
    accumulation or (n,) int32 RGBA8 words) to `dst`.

    Buffers are padded to the largest rank's size so one collective moves them
    all. Returns the list of per-rank tensors (trimmed) on `dst`, None elsewhere.
    Works with any torch.distributed backend (nccl = RCCL on ROCm, or gloo)."""
    import torch
    import torch.distributed as dist

    cap = max_owned_tiles(n_tiles, world_size) * 64
    if packed.shape[0] < cap:
        pad = torch.zeros((cap - packed.shape[0], *packed.shape[1:]), dtype=packed.dtype, device=packed.device)
        packed = torch.cat([packed, pad])
    device = packed.device
    if dist.get_backend() == "gloo" and packed.is_cuda:  # gloo moves host tensors only
        packed = packed.cpu()
    bufs = [torch.empty_like(packed) for _ in range(world_size)] if rank == dst else None
    dist.gather(packed, gather_list=bufs, dst=dst)
    if rank != dst:
        return None
    return [b[: owned_tiles(n_tiles, r, world_size).shape[0] * 64].to(device) for r, b in enumerate(bufs)]


def gather_accumulation(renderer, dst: int = 0):
    """Assemble the whole frame of a tile-split render on rank `dst`'s Renderer:
    device pack -> RCCL gather -> device unpack. Accumulating renders move the
    RGBA32F accumulation (16 B/px) and rebuild the RGBA8 output from it with the
    last frame's divisor k*c (compute_shader.wgsl:166); non-accumulating ones
    (which never write the accumulation, :171-178) move the RGBA8 words as is."""
    import torch

    rank, world = renderer.rank, renderer.world_size
    tx_n, ty_n = tile_grid(renderer.width, renderer.height)
    n_tiles = tx_n * ty_n
    cap = max_owned_tiles(n_tiles, world) * 64
    device = torch.device("cuda", renderer.device)  # the renderer's GPU, whatever torch's current device is
    if renderer.accumulate:
        packed = torch.zeros((cap, 4), dtype=torch.float32, device=device)
        renderer.pack_owned_accumulation(packed.data_ptr())
    else:
        packed = torch.zeros((cap,), dtype=torch.int32, device=device)
        renderer.pack_owned_output(packed.data_ptr())
    renderer.synchronize()
    parts = gather_packed(packed, n_tiles, rank, world, dst)
    if parts is None:
        return
    torch.cuda.synchronize(device)
    k = renderer.accumulation_index - 1  # the last frame's accumulation_index
    divisor = max(k, 1) * renderer.compute_per_frame
    for src, part in enumerate(parts):
        if src != rank and part.shape[0]:
            if renderer.accumulate:
                renderer.unpack_accumulation(part.data_ptr(), src, world, divisor)
            else:
                renderer.unpack_output(part.data_ptr(), src, world)
    renderer.synchronize()
