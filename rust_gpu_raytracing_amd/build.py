"""Build the HIP extension in-tree: ``librt_pathtrace.so`` for gfx950.

The numeric-contract flags are load-bearing: no FMA contraction,
correctly rounded f32 division and sqrt, denormals preserved. Without them the
kernel still runs but is no longer bit-exact against the oracle.
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = ROOT / "include"
OUT = PKG / "librt_pathtrace.so"
SOURCES = [CSRC / "pathtrace.hip", CSRC / "scene_edit.hip", CSRC / "rt_abi.cpp", CSRC / "sphere_bvh.cpp",
           CSRC / "scene_build.cpp"]
HEADERS = [CSRC / "rt_bvh_slab.h", CSRC / "rt_device_math.h", CSRC / "rt_kernel_args.h", CSRC / "sphere_bvh.h",
           CSRC / "rt_scene_math.h", INCLUDE / "rt_abi.h"]

ARCH = os.environ.get("RT_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

NUMERIC_FLAGS = [
    "-ffp-contract=off",
    "-fno-fast-math",
    "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-fno-gpu-flush-denormals-to-zero",
]
# gfx950 runs v_pk_{mul,add}_f32 at about a third of the scalar wave-instruction
# rate (tools/microbench/valu_rate.hip), so the SLP vectorizer's packed f32
# code is slower than scalar code here: measured -21% kernel time without it.
PERF_FLAGS = ["-fno-slp-vectorize"]


def hipcc_command(out: Path = OUT, extra: list[str] | None = None) -> list[str]:
    return [
        HIPCC,
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++17",
        *NUMERIC_FLAGS,
        *PERF_FLAGS,
        "-fPIC",
        "-shared",
        "-fvisibility=hidden",
        "-Wall",
        f"-I{INCLUDE}",
        f"-I{CSRC}",
        *(extra or []),
        *map(str, SOURCES),
        "-o",
        str(out),
    ]


def up_to_date(out: Path = OUT) -> bool:
    if not out.exists():
        return False
    t = out.stat().st_mtime
    return all(p.stat().st_mtime <= t for p in SOURCES + HEADERS + [Path(__file__)])


def build(force: bool = False, verbose: bool = True) -> Path:
    if not force and up_to_date():
        return OUT
    tmp = OUT.with_suffix(f".{os.getpid()}.tmp.so")
    cmd = hipcc_command(tmp)
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
