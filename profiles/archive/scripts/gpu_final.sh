#!/bin/bash
# Round-4 final passes (via gpurun), split in two calls so each fits the box's time limit.
#   bash tools/gpu_final.sh <tag> A   tests, smoke, rocprofv3 stats + PMC for C2, C3 and brute-force C5
#                                     (then locally: tools/update_traffic.py per profile dir)
#   bash tools/gpu_final.sh <tag> B   headline bench, all configs, C3 / C5 / C5 relative-slack / brute
#                                     C5 bench lines (their PMC entries committed by then), strong probe,
#                                     the source build on the box, the 2/4/8-rank gloo rehearsal
set -e -o pipefail
TAG=${1:-r04_f}; PART=${2:-A}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$PART" = A ]; then
  bash tools/gpu_check.sh "$TAG" tests smoke
  bash tools/profile.sh "$TAG"
  bash tools/profile.sh "${TAG}_c3" --config c3_chess
  bash tools/profile.sh "${TAG}_c5b" --config c5_heightfield --brute-force --steps 2 --warmup 2 --settle-ms 0
else
  bash tools/gpu_check.sh "$TAG" bench all
  timeout -k 10 300 python3 bench.py --config c3_chess --no-cpu-baseline --no-cadences > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
  timeout -k 10 300 python3 bench.py --config c5_heightfield --no-cpu-baseline --no-cadences > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err"
  RT_TRI_PRUNE=2 timeout -k 10 300 python3 bench.py --config c5_heightfield --no-cpu-baseline --no-cadences > "$OUT/bench_c5_slack.json" 2> "$OUT/bench_c5_slack.err"
  timeout -k 10 400 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --settle-ms 0 --no-cpu-baseline --no-cadences > "$OUT/bench_c5_brute.json" 2> "$OUT/bench_c5_brute.err"
  bash tools/gpu_check.sh "$TAG" strong srcbuild multi
fi
echo "== final $PART done $(date +%T)"
