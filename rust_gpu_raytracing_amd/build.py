"""Build the HIP extension in-tree: ``librt_pathtrace.so`` for gfx950.

The numeric-contract flags are load-bearing: no FMA contraction,
correctly rounded f32 division and sqrt, denormals preserved. Without them the
kernel still runs but is no longer bit-exact against the oracle.
"""
from __future__ import annotations

import hashlib
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = ROOT / "include"
OUT = PKG / "librt_pathtrace.so"
SOURCES = [CSRC / "pathtrace.hip", CSRC / "scene_edit.hip", CSRC / "rt_abi.cpp", CSRC / "sphere_bvh.cpp",
           CSRC / "scene_build.cpp", CSRC / "rt_multi.cpp"]
HEADERS = [CSRC / "rt_bvh_slab.h", CSRC / "rt_device_math.h", CSRC / "rt_kernel_args.h", CSRC / "sphere_bvh.h",
           CSRC / "rt_scene_math.h", CSRC / "tri_qnode.h", CSRC / "tri_cone.h", CSRC / "rt_path_common.h",
           INCLUDE / "rt_abi.h"]

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


STAMP = PKG / "librt_pathtrace.build.json"  # what built OUT: source hash, hipcc command, host, time


def source_hash() -> str:
    """SHA-256 over the compiler, the flags and every source and header: the identity of
    a build. The library embeds it (rt_build_hash) and build() rebuilds when it differs."""
    h = hashlib.sha256()
    h.update(" ".join([HIPCC, ARCH, *NUMERIC_FLAGS, *PERF_FLAGS]).encode())
    for f in SOURCES + HEADERS + [Path(__file__)]:
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()[:16]


def hipcc_command(out: Path = OUT, extra: list[str] | None = None, build_hash: str | None = None) -> list[str]:
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
        f'-DRT_BUILD_HASH="{build_hash or source_hash()}"',
        *(extra or []),
        *map(str, SOURCES),
        "-ldl",  # rt_multi.cpp opens librccl at run time (dlopen), only for rt_create_multi
        "-pthread",  # rt_multi.cpp: one host thread per device of a group
        "-o",
        str(out),
    ]


def build_info() -> dict:
    """The stamp of the library on disk ({} if none) plus the current source hash."""
    info = json.loads(STAMP.read_text()) if STAMP.exists() and OUT.exists() else {}
    info["sources_hash"] = source_hash()
    return info


def up_to_date(out: Path = OUT) -> bool:
    if not out.exists() or not STAMP.exists():
        return False
    try:
        return json.loads(STAMP.read_text()).get("hash") == source_hash()
    except (ValueError, OSError):
        return False


def build(force: bool = False, verbose: bool = True) -> Path:
    """Compile when the sources' hash differs from the one the library was built
    from (content, not mtime: a copied tree with fresh timestamps does not rebuild,
    an edited header does)."""
    if not force and up_to_date():
        return OUT
    digest = source_hash()
    tmp = OUT.with_suffix(f".{os.getpid()}.tmp.so")
    cmd = hipcc_command(tmp, build_hash=digest)
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    t0 = time.time()
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    STAMP.write_text(json.dumps({"hash": digest, "host": socket.gethostname(),
                                 "built_at": time.strftime("%Y-%m-%dT%H:%M:%S"), "seconds": round(time.time() - t0, 1),
                                 "command": " ".join(hipcc_command(OUT, build_hash=digest))}, indent=1))
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
