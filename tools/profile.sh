#!/bin/bash
# Profile the headline bench on the GPU box (run via gpurun).
# usage: tools/profile.sh <tag> [extra bench args]
# Writes gpurun_out/prof_<tag>/: kernel-trace stats, then one PMC pass per
# counter group (counters are never combined with sys/runtime traces).
set -e -o pipefail
TAG=${1:-r01}; shift || true
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --steps 20 --warmup 20 --no-cpu-baseline --no-cadences $*"  # warmup = steps: every launch renders 20 frames, so per-launch averages are the timed launches
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH > "$OUT/trace_bench.json" 2> "$OUT/trace.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 $BENCH > /dev/null 2> "$OUT/pmc_fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 $BENCH > /dev/null 2> "$OUT/pmc_write.err"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$OUT/pmc_sq" -o run -- python3 $BENCH > /dev/null 2> "$OUT/pmc_sq.err"
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_valu" -o run -- python3 $BENCH > /dev/null 2> "$OUT/pmc_valu.err"
echo done
