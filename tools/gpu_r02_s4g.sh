#!/bin/bash
# Session 4: SQ counters (LDS instructions, bank conflicts, waits) of the skip-link and pair walks.
set -e -o pipefail
OUT=gpurun_out/r02_s4g
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
for l in lib_base lib_pairs; do
  RT_LIB=$V/$l.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU --output-format csv -d $OUT/pmc_$l -o run -- python3 bench.py --steps 20 --warmup 20 --no-cpu-baseline --settle-ms 0 > $OUT/pmc_$l.json 2> $OUT/pmc_$l.err
done
echo done
