#!/bin/bash
# Session 3: HEAD vs the session's starting build (regression check).
set -e -o pipefail
OUT=gpurun_out/r02_s3k2
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
A="--frames 32 --rounds 4 --frame-batch 8"
for c in c2_rtiow c3_chess c4_mixed; do
  timeout -k 10 300 python3 tools/ab_bench.py $V/lib_s3start.so $V/lib_head2.so $V/lib_s3start.so $V/lib_head2.so --config $c $A > $OUT/ab_$c.json 2>> $OUT/err.log
done
timeout -k 10 300 python3 tools/ab_bench.py $V/lib_s3start.so $V/lib_head2.so --config c5_heightfield --frames 8 --rounds 2 --frame-batch 8 > $OUT/ab_c5_heightfield.json 2>> $OUT/err.log
echo done
