#!/bin/bash
# Session 4: bench with the clock settle; SQ counters of the group-leaf and sphere-step builds.
set -e -o pipefail
OUT=gpurun_out/r02_s4e
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
for l in lib_base lib_step; do
  RT_LIB=$V/$l.so timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_$l -o run -- python3 bench.py --steps 20 --warmup 20 --no-cpu-baseline > $OUT/pmc_$l.json 2> $OUT/pmc_$l.err
done
echo done
