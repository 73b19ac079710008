#!/bin/bash
# Counter A/B of one build under per-run environment settings (run via gpurun).
#   bash tools/pmc_ab.sh <tag> <config> "<spec>" ["<spec>" ...]
# spec = space-separated VAR=VALUE exported for that variant's runs. Per variant:
# one rocprofv3 --kernel-trace --stats pass and three --pmc passes (each within the
# per-block counter limits), on bench.py --config <config> (20 frames in one launch,
# 20 warmup frames: every profiled launch is a 20-frame launch).
set -e -o pipefail
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --config $CFG --steps 20 --warmup 20 --settle-ms 0 --no-cpu-baseline --no-cadences"
i=0
for spec in "$@"; do
  i=$((i + 1))
  D="$OUT/v$i"
  mkdir -p "$D"
  echo "$spec" > "$D/spec.txt"
  (
    for kv in $spec; do export "$kv"; done
    echo "== v$i [$spec] $(date +%T)"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/trace" -o run -- python3 $BENCH > "$D/bench.json" 2> "$D/trace.err"
    timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$D/fetch" -o run -- python3 $BENCH > /dev/null 2> "$D/fetch.err"
    timeout -s KILL 180 rocprofv3 --pmc TA_BUSY_avr GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$D/mem" -o run -- python3 $BENCH > /dev/null 2> "$D/mem.err"
    timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d "$D/sq" -o run -- python3 $BENCH > /dev/null 2> "$D/sq.err"
  )
done
echo "== done $(date +%T)"
