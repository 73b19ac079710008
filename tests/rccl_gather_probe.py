"""RCCL leg of the tile gather on one GPU (run by tests/test_gpu_rccl.py).

Launched as `python -m torch.distributed.run --nproc-per-node 1 ... tests/rccl_gather_probe.py`:
one rank, backend "nccl" (RCCL on ROCm), so the code path bench.py takes at N > 1 --
the TileGather on the renderer's own stream (torch.cuda.ExternalStream), dist.gather
into one (world, cap) buffer, the one-launch unpack -- runs for real. (RCCL refuses two
ranks on one device, so the N-rank layout itself is covered by the gloo tests.)
Prints "ok" when the gathered image equals the render it came from.
"""
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main() -> int:
    import torch
    import torch.distributed as dist

    from rust_gpu_raytracing_amd import Renderer
    from rust_gpu_raytracing_amd.distributed import TileGather, pack_owned_host
    from rust_gpu_raytracing_amd.scene import build_config

    rank = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    scene, bounces = build_config("c2_rtiow", width=200, height=104)
    with Renderer(scene, rank=rank, world_size=dist.get_world_size(), frame_batch=4) as r:
        for _ in range(6):
            r.compute_frame(bounces)
        r.synchronize()
        before = r.read_accumulation(), r.read_output()
        g = TileGather(r, dst=0)
        assert not g.host, "expected the RCCL path"
        g()
        g()  # reused buffers
        r.synchronize()
        after = r.read_accumulation(), r.read_output()
        recv = g.recv_all[rank].cpu().numpy()
        gi = TileGather(r, dst=0, what="image")  # bench.py's default payload at N > 1
        gi()
        r.synchronize()
        after_image = r.read_accumulation(), r.read_output()
        recv_words = gi.recv_all[rank].cpu().numpy().view(np.uint32)
    dist.destroy_process_group()
    same = np.array_equal(before[0].view(np.uint32), after[0].view(np.uint32)) and np.array_equal(before[1], after[1])
    # the block RCCL delivered is this rank's packed accumulation, bit for bit
    want = pack_owned_host(before[0], rank, 1)
    packed_ok = np.array_equal(recv[: want.shape[0]].view(np.uint32), want.view(np.uint32))
    same_image = (np.array_equal(before[0].view(np.uint32), after_image[0].view(np.uint32))
                  and np.array_equal(before[1], after_image[1]))
    want_words = pack_owned_host(before[1], rank, 1)
    words_ok = np.array_equal(recv_words[: want_words.shape[0]], want_words)
    ok = same and packed_ok and same_image and words_ok and before[0].any() and before[1].any()
    print("ok" if ok else f"MISMATCH same={same} packed={packed_ok} image={same_image} words={words_ok}", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
