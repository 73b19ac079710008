#!/bin/bash
# Session 3: paired triangle loads in the leaf (RT_TRI_PAIR) vs current.
set -e -o pipefail
OUT=gpurun_out/r02_s3e
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
A="--frames 16 --rounds 3 --frame-batch 8"
for c in c3_chess c4_mixed; do
  timeout -k 10 300 python3 tools/ab_bench.py $V/lib_cur.so $V/lib_pair.so --config $c $A > $OUT/ab_$c.json 2>> $OUT/err.log
done
timeout -k 10 300 python3 tools/ab_bench.py $V/lib_cur.so $V/lib_pair.so --config c5_heightfield --frames 8 --rounds 2 --frame-batch 8 > $OUT/ab_c5_heightfield.json 2>> $OUT/err.log
echo done
