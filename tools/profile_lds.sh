#!/bin/bash
# LDS / instruction-mix counters for the bench, one PMC pass per group.
# usage: tools/profile_lds.sh <tag>   (env vars such as RT_BLOCK_THREADS pass through)
set -e -o pipefail
TAG=${1:-lds}; shift || true
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --steps 10 --warmup 2 --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH > /dev/null 2> "$OUT/trace.err"
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_lds" -o run -- python3 $BENCH > /dev/null 2> "$OUT/pmc_lds.err"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQC_ICACHE_MISSES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d "$OUT/pmc_mix" -o run -- python3 $BENCH > /dev/null 2> "$OUT/pmc_mix.err"
echo done
