"""Multi-GPU tile partition and the readback gather.

The reference renders on one adapter (src/main.rs:636-665). Here one process
drives one GPU; the frame is cut into 8x8-pixel tiles and tile t belongs to rank
t % world_size. Each rank's kernel launch renders only its tiles, using global
pixel indices for the RNG seeds (compute_shader.wgsl:217), so the assembled image
is bitwise identical to a 1-GPU render. Rendering needs no communication; at
readback every rank packs its tiles into one contiguous buffer (tile order, 64
pixels per tile) and one RCCL gather (torch.distributed, backend "nccl") moves them
to the destination rank, which unpacks them into its framebuffer. Two payloads:

* "image": the packed RGBA8 output words (4 B/px) -- the frame as the reference
  displays it (the output buffer its render pass blits, src/renderer.rs:237-249,
  src/render_shader.wgsl). The accumulation stays sharded on its owner ranks, which
  keep accumulating their own tiles frame after frame; this is the per-frame
  readback of an interactive multi-GPU loop.
* "accumulation": the RGBA32F accumulation (16 B/px), from which the destination
  also rebuilds the RGBA8 output: the whole renderer state on one rank (a
  checkpoint, or a switch back to one GPU).
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
    """Host mirror of rt_pack_tiles_kernel: (H, W, 4) f32 -> (owned_tiles*64, 4), or of
    rt_pack_owned_output: (H, W) RGBA8 words -> (owned_tiles*64,). Padding slots are 0."""
    h, w = accum.shape[:2]
    idx = owned_pixel_indices(w, h, rank, world_size)
    flat = accum.reshape(h * w, *accum.shape[2:])
    out = np.zeros((idx.shape[0], *accum.shape[2:]), accum.dtype)
    ok = idx >= 0
    out[ok] = flat[idx[ok]]
    return out


def unpack_host(accum: np.ndarray, packed: np.ndarray, src_rank: int, world_size: int) -> None:
    h, w = accum.shape[:2]
    idx = owned_pixel_indices(w, h, src_rank, world_size)
    ok = idx >= 0
    accum.reshape(h * w, *accum.shape[2:])[idx[ok]] = packed[: idx.shape[0]][ok]


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


GATHER_PAYLOADS = ("image", "accumulation")


class TileGather:
    """Reusable readback gather for a tile-split Renderer: the pack buffer and (on
    `dst`) the receive buffers are allocated once, so repeated gathers (one per
    displayed frame in an interactive loop, once per run in bench.py) allocate
    nothing. The first gather also makes RCCL set up its peer connections, which it
    does lazily on a pair's first transfer; bench.py runs one during warmup.

    what="image" moves the RGBA8 output words (4 B/px) as is: the destination's
    output buffer then holds the whole frame, bit-identical to a 1-GPU render's,
    while its accumulation keeps only its own tiles. what="accumulation" (only for
    accumulating renders) moves the RGBA32F accumulation (16 B/px) and rebuilds the
    RGBA8 output from it with the last frame's divisor k*c (compute_shader.wgsl:166),
    so both buffers equal a 1-GPU render's. Default: the accumulation when the
    renderer accumulates (non-accumulating renders never write it, :171-178)."""

    def __init__(self, renderer, dst: int = 0, what: str | None = None):
        import torch
        import torch.distributed as dist

        if what is None:
            what = "accumulation" if renderer.accumulate else "image"
        if what not in GATHER_PAYLOADS:
            raise ValueError(f"TileGather: what must be one of {GATHER_PAYLOADS}, got {what!r}")
        if what == "accumulation" and not renderer.accumulate:
            raise ValueError("TileGather: a non-accumulating render never writes its accumulation; gather the image")
        self.what = what
        self.accum = what == "accumulation"
        self.r, self.dst = renderer, dst
        self.rank, self.world = renderer.rank, renderer.world_size
        tx_n, ty_n = tile_grid(renderer.width, renderer.height)
        self.n_tiles = tx_n * ty_n
        cap = max_owned_tiles(self.n_tiles, self.world) * 64
        self.device = torch.device("cuda", renderer.device)  # the renderer's GPU, whatever torch's current device is
        shape, dtype = ((cap, 4), torch.float32) if self.accum else ((cap,), torch.int32)
        self.cap = cap
        self.packed = torch.zeros(shape, dtype=dtype, device=self.device)
        # gloo moves host tensors only
        self.host = dist.get_backend() == "gloo"
        send_dev = "cpu" if self.host else self.device
        self.send = torch.zeros(shape, dtype=dtype, device=send_dev) if self.host else self.packed
        # the destination receives into one contiguous (world, cap, ...) buffer, so a
        # single unpack launch covers every rank's block
        self.recv_all = torch.empty((self.world, *shape), dtype=dtype, device=send_dev) if self.rank == dst else None
        self.recv = list(self.recv_all.unbind(0)) if self.rank == dst else None
        self.recv_dev_all = (torch.empty((self.world, *shape), dtype=dtype, device=self.device)
                             if self.rank == dst and self.host else self.recv_all)

    def __call__(self) -> None:
        import torch
        import torch.distributed as dist

        r = self.r
        if self.host:  # gloo: through host memory, synchronously
            self._pack()
            r.synchronize()
            self.send.copy_(self.packed)
            dist.gather(self.send, gather_list=self.recv, dst=self.dst)
            if self.rank == self.dst:
                self.recv_dev_all.copy_(self.recv_all)
                torch.cuda.synchronize(self.device)
                self._unpack()
            r.synchronize()
            return
        # RCCL: everything stream-ordered on the renderer's own HIP stream (no host
        # waits): the pack kernel, the gather (ProcessGroupNCCL orders its stream
        # after the current stream, and the current stream after the collective),
        # then the unpack kernels on the destination.
        stream = torch.cuda.ExternalStream(r.stream_handle, device=self.device)
        with torch.cuda.device(self.device), torch.cuda.stream(stream):
            self._pack()
            dist.gather(self.send, gather_list=self.recv, dst=self.dst)
            if self.rank == self.dst:
                self._unpack()

    def _pack(self) -> None:
        if self.accum:
            self.r.pack_owned_accumulation(self.packed.data_ptr())
        else:
            self.r.pack_owned_output(self.packed.data_ptr())

    def _unpack(self) -> None:
        """Every other rank's block in one launch (the own block is already in place)."""
        r = self.r
        if self.accum:
            divisor = max(r.accumulation_index - 1, 1) * r.compute_per_frame  # the last frame's k*c
            r.unpack_accumulation_ranks(self.recv_dev_all.data_ptr(), self.cap, self.world, self.rank, divisor)
        else:
            r.unpack_output_ranks(self.recv_dev_all.data_ptr(), self.cap, self.world, self.rank)


def gather_frame(renderer, dst: int = 0, what: str | None = None, sync: bool = True):
    """Assemble the frame of a tile-split render on rank `dst`'s Renderer: device
    pack -> RCCL gather -> device unpack, of the payload `what` (TileGather). The
    TileGather is cached on the renderer per (dst, payload), so a second call
    allocates nothing. sync=False leaves the RCCL path stream-ordered (no host wait)."""
    cache = renderer.__dict__.setdefault("_tile_gathers", {})
    what = what or ("accumulation" if renderer.accumulate else "image")
    g = cache.get((dst, what))
    if g is None:
        g = cache[(dst, what)] = TileGather(renderer, dst, what)
    g()
    if sync:
        renderer.synchronize()


def gather_accumulation(renderer, dst: int = 0):
    """The whole renderer state on `dst`: the accumulation when the render
    accumulates (plus the output rebuilt from it), else the RGBA8 image."""
    gather_frame(renderer, dst)


def gather_image(renderer, dst: int = 0):
    """The displayed frame (RGBA8 words) on `dst`; accumulations stay on their owners."""
    gather_frame(renderer, dst, "image")
