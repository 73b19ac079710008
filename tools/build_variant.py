"""Build an experiment variant of librt_pathtrace.so (analysis tool).

usage: python tools/build_variant.py <out.so> [-DFLAG ...]
Same sources and numeric flags as the product build (rust_gpu_raytracing_amd/build.py)
plus the given extra compiler arguments; load it with RT_LIB=<out.so> or
tools/ab_bench.py.
"""
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from rust_gpu_raytracing_amd.build import hipcc_command  # noqa: E402

out = Path(sys.argv[1]).resolve()
out.parent.mkdir(parents=True, exist_ok=True)
subprocess.run(hipcc_command(out, sys.argv[2:]), check=True)
print(out)
