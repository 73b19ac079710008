#!/bin/bash
# Session 3: exact-sweep SAH builds (sphere BVH + triangle accelerator) -- tests + A/B.
set -e -o pipefail
OUT=gpurun_out/r02_s3m
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
A="--frames 32 --rounds 4 --frame-batch 8"
for c in c2_rtiow c3_chess c4_mixed c1_four_spheres; do
  timeout -k 10 300 python3 tools/ab_bench.py $V/lib_rcp2.so $V/lib_sweep.so --config $c $A > $OUT/ab_$c.json 2>> $OUT/err.log
done
timeout -k 10 300 python3 tools/ab_bench.py $V/lib_rcp2.so $V/lib_sweep.so --config c5_heightfield --frames 8 --rounds 2 --frame-batch 8 > $OUT/ab_c5_heightfield.json 2>> $OUT/err.log
echo done
