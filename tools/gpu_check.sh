#!/bin/bash
# One GPU-box pass: parity tests, smoke, headline bench, all configs, profile.
# usage (via gpurun): bash tools/gpu_check.sh <tag> [steps...]
#   steps: any of tests smoke bench all prof (default: all of them)
# Every GPU step has its own time limit; the script stops at the first failure.
set -e -o pipefail
TAG=${1:-r01}; shift || true
STEPS=${*:-tests smoke bench all prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1
for s in $STEPS; do
  echo "== $s $(date +%T)"
  case $s in
    tests) timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > "$OUT/tests.log" 2>&1 ;;
    smoke) timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench) timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    all)   timeout -k 10 600 python3 tools/bench_all.py --no-cpu > "$OUT/bench_all.jsonl" 2> "$OUT/bench_all.err" ;;
    prof)  bash tools/profile.sh "$TAG" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  tail -3 "$OUT"/*.log 2>/dev/null | tail -3 || true
done
echo "== done $(date +%T)"
