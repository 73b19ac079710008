#!/bin/bash
# One GPU-box pass: parity tests, smoke, headline bench, all configs, profile.
# usage (via gpurun): bash tools/gpu_check.sh <tag> [steps...]
#   steps: any of tests smoke bench all prof multi (default: all of them)
# Every GPU step has its own time limit; the script stops at the first failure.
set -e -o pipefail
TAG=${1:-r01}; shift || true
STEPS=${*:-tests smoke bench all prof multi strong}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1
for s in $STEPS; do
  echo "== $s $(date +%T)"
  case $s in
    tests) timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 ;;
    smoke) timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench) timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    all)   timeout -k 10 600 python3 tools/bench_all.py --no-cpu --frames 20 > "$OUT/bench_all.jsonl" 2> "$OUT/bench_all.err" ;;
    strong) timeout -k 10 300 python3 tools/strong_probe.py --steps 20 > "$OUT/strong_probe.jsonl" 2> "$OUT/strong_probe.err" ;;
    prof)  bash tools/profile.sh "$TAG" ;;  # then locally: python tools/update_traffic.py gpurun_out/prof_<tag> profiles/<tag>
    srcbuild) # provenance: compile the library from source on this box (its own hipcc) into a
           # scratch path and run the golden + smoke-size parity tests against that build
           timeout -k 10 600 python3 -c "
import subprocess, sys
from rust_gpu_raytracing_amd import build as b
out = '/tmp/librt_srcbuild.so'
subprocess.run(b.hipcc_command(__import__('pathlib').Path(out)), check=True)
print('built', out, 'hash', b.source_hash())" > "$OUT/srcbuild.log" 2>&1 &&
           RT_LIB=/tmp/librt_srcbuild.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v \
             --timeout 200 --timeout-method thread -k "golden or full_frame_baseline_size" >> "$OUT/srcbuild.log" 2>&1 &&
           RT_LIB=/tmp/librt_srcbuild.so python3 -c "
from rust_gpu_raytracing_amd import _native as N, build as b
lib = N.load_library(); import socket
print('srcbuild library hash', lib.rt_build_hash().decode(), '== tree', b.source_hash(), 'on', socket.gethostname())" >> "$OUT/srcbuild.log" 2>&1 ;;
    multi) # N-rank rehearsal on the one GPU of the box (gloo; the real run is RCCL, one GPU per rank)
           for n in 2 4 8; do
             RT_BENCH_ONE_DEVICE=1 RT_DIST_BACKEND=gloo RT_BENCH_VERIFY_GATHER=1 timeout -k 10 300 \
               python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
               --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 2 > "$OUT/multi_$n.json" 2> "$OUT/multi_$n.err"
           done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  tail -3 "$OUT"/*.log 2>/dev/null | tail -3 || true
done
echo "== done $(date +%T)"
