#!/bin/bash
# Instruction-cache counters of the path kernel per build (run via gpurun): one --pmc pass of
# 8 SQ-block counters per library on bench.py's C2 launch (20 frames, 20 warmup frames).
#   bash tools/pmc_icache.sh <tag> <lib.so> [<lib.so> ...]
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
CFG=${RT_PMC_CONFIG:-c2_rtiow}
BENCH="bench.py --config $CFG --steps 20 --warmup 20 --settle-ms 0 --no-cpu-baseline --no-cadences"
i=0
for lib in "$@"; do
  i=$((i + 1))
  D="$OUT/v$i"
  mkdir -p "$D"
  echo "$lib" > "$D/lib.txt"
  echo "== v$i $lib $(date +%T)"
  RT_LIB=$lib timeout -s KILL 180 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d "$D/ic" -o run -- python3 $BENCH > "$D/bench.json" 2> "$D/ic.err"
done
echo "== done $(date +%T)"
