#!/bin/bash
# Session 4: sphere leaves tested once per group of node steps (RT_SPHERE_LEAF_END) -- A/B.
set -e -o pipefail
OUT=gpurun_out/r02_s4o
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
A="--frames 20 --rounds 5 --frame-batch 20"
for c in c2_rtiow c1_four_spheres; do
  timeout -k 10 300 python3 tools/ab_bench.py $V/lib_cur.so $V/lib_lend.so $V/lib_lend_u4.so $V/lib_lend_u2.so $V/lib_defer.so --config $c $A > $OUT/ab_$c.json 2>> $OUT/err.log
done
echo done
