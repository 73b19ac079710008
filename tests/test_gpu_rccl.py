"""The RCCL (backend "nccl") leg of the multi-GPU gather, on the box's one GPU.

tests/rccl_gather_probe.py runs under torch.distributed.run with one rank: the
TileGather's stream-ordered RCCL path (the one bench.py takes at N > 1) gathers a
render's accumulation and must hand back exactly what was packed.
"""
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gpu_rccl_tile_gather(gpu):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(ROOT / "tests" / "rccl_gather_probe.py")]
    out = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=240, cwd=ROOT)
    assert out.returncode == 0 and "ok" in out.stdout.split(), out.stdout[-2000:] + out.stderr[-2000:]


def test_gpu_bench_distributed_path_rccl(gpu):
    """bench.py's N > 1 code path (process group over RCCL, gather inside the timed
    region, gather verify, the weak run) with one rank (RT_BENCH_DIST=1)."""
    import json

    env = dict(os.environ, MASTER_ADDR="127.0.0.1", RT_BENCH_DIST="1", RT_BENCH_VERIFY_GATHER="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(ROOT / "bench.py"),
           "--gpus", "1", "--steps", "4", "--warmup", "2", "--settle-ms", "20", "--no-cpu-baseline"]
    out = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=280, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    line = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert line["gather_in_value"] is True and line["value"] > 0 and "weak" in line
    assert "gather verify: assembled image == 1-GPU render" in out.stderr
