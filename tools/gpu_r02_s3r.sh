#!/bin/bash
# Session 3: decoded 1x1 texels in the LDS material table -- tests + A/B.
set -e -o pipefail
OUT=gpurun_out/r02_s3r
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
A="--frames 40 --rounds 4 --frame-batch 20"
for c in c2_rtiow c1_four_spheres c3_chess; do
  timeout -k 10 300 python3 tools/ab_bench.py $V/lib_aux.so $V/lib_tex1.so $V/lib_aux.so $V/lib_tex1.so --config $c $A > $OUT/ab_$c.json 2>> $OUT/err.log
done
echo done
