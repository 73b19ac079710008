#!/bin/bash
# L1 (TCP) / texture-address (TA) counters of one bench workload (run via gpurun): is the walk
# bound by the L1's tag lookups? usage: tools/pmc_tcp.sh <tag> [bench args]
# Environment switches (RT_*) are inherited by the profiled bench. One counter group per pass.
set -e -o pipefail
TAG=${1:-tcp}; shift || true
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --steps 20 --warmup 20 --no-cpu-baseline --no-cadences $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH > "$OUT/trace_bench.json" 2> "$OUT/trace.err"
timeout -k 10 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TAGRAM0_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_tcp1" -o run -- python3 $BENCH > /dev/null 2> "$OUT/pmc_tcp1.err"
timeout -k 10 300 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum --output-format csv -d "$OUT/pmc_ta" -o run -- python3 $BENCH > /dev/null 2> "$OUT/pmc_ta.err"
timeout -k 10 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum --output-format csv -d "$OUT/pmc_tcp2" -o run -- python3 $BENCH > /dev/null 2> "$OUT/pmc_tcp2.err"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$OUT/pmc_sq" -o run -- python3 $BENCH > /dev/null 2> "$OUT/pmc_sq.err"
echo done
