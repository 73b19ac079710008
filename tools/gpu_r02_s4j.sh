#!/bin/bash
# Session 4: split tail (last units claimed in parts) -- tests + A/B + N=8 share.
set -e -o pipefail
OUT=gpurun_out/r02_s4j
mkdir -p $OUT
export TMPDIR=/tmp
L=build/variants/lib_tail.so
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
A="--frames 20 --rounds 6 --frame-batch 20"
for c in c2_rtiow c3_chess; do
  timeout -k 10 300 python3 tools/ab_bench.py $L:RT_TAIL_SHIFT=0 $L $L:RT_TAIL_SHIFT=3 $L:RT_TAIL_WAVES=4 --config $c $A > $OUT/ab_$c.json 2>> $OUT/err.log
done
for v in 0 2 3 0 2; do
  RT_LIB=$L RT_TAIL_SHIFT=$v timeout -k 10 200 python3 tools/strong_probe.py --ns 8 --steps 20 >> $OUT/strong_shift$v.jsonl 2>> $OUT/err.log
done
echo done
