#!/bin/bash
# Session 3: v_rcp_f32 for sphere-only culling, margin-only sqrt/rcp upper bounds -- tests + A/B.
set -e -o pipefail
OUT=gpurun_out/r02_s3l
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
A="--frames 32 --rounds 4 --frame-batch 8"
for c in c2_rtiow c1_four_spheres c3_chess c4_mixed; do
  timeout -k 10 300 python3 tools/ab_bench.py $V/lib_head2.so $V/lib_rcp.so $V/lib_rcp2.so --config $c $A > $OUT/ab_$c.json 2>> $OUT/err.log
done
echo done
