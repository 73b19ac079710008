"""Build librt_pathtrace.so from the kernel sources of an earlier commit (analysis tool).

usage: python tools/build_at_commit.py <commit> <out.so> [-DFLAG ...]
Extracts rust_gpu_raytracing_amd/csrc and include/ at <commit> (git archive) into a
temporary directory and compiles the sources that commit's build.py lists, with today's
numeric and performance flags. Used for same-process A/B runs (tools/ab_bench.py) that
locate a change in kernel time between commits.
"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from rust_gpu_raytracing_amd import build as B  # noqa: E402


def main():
    commit, out = sys.argv[1], Path(sys.argv[2]).resolve()
    extra = sys.argv[3:]
    out.parent.mkdir(parents=True, exist_ok=True)
    with tempfile.TemporaryDirectory() as tmp:
        t = Path(tmp)
        arch = subprocess.run(["git", "-C", str(ROOT), "archive", commit, "rust_gpu_raytracing_amd/csrc",
                               "include", "rust_gpu_raytracing_amd/build.py"], check=True, capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", str(t)], input=arch, check=True)
        build_py = (t / "rust_gpu_raytracing_amd/build.py").read_text()
        src_line = re.search(r"SOURCES = \[(.*?)\]", build_py, re.S).group(1)
        sources = [t / "rust_gpu_raytracing_amd/csrc" / s for s in re.findall(r'CSRC / "([^"]+)"', src_line)]
        short = subprocess.run(["git", "-C", str(ROOT), "rev-parse", "--short=8", commit], check=True,
                               capture_output=True, text=True).stdout.strip()
        cmd = [B.HIPCC, f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", *B.NUMERIC_FLAGS, *B.PERF_FLAGS, "-fPIC",
               "-shared", "-fvisibility=hidden", f"-I{t / 'include'}", f"-I{t / 'rust_gpu_raytracing_amd/csrc'}",
               f'-DRT_BUILD_HASH="commit-{short}"', *extra, *map(str, sources), "-ldl", "-pthread", "-o", str(out)]
        subprocess.run(cmd, check=True)
    print(out)


if __name__ == "__main__":
    main()
