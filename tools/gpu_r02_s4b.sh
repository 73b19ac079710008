#!/bin/bash
# Session 4: sphere leaves tested one sphere per traversal step -- tests + A/B.
set -e -o pipefail
OUT=gpurun_out/r02_s4b
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
A="--frames 40 --rounds 4 --frame-batch 20"
for c in c2_rtiow c1_four_spheres; do
  timeout -k 10 300 python3 tools/ab_bench.py $V/lib_base.so $V/lib_step.so $V/lib_step_u2.so $V/lib_step_u4.so $V/lib_base.so $V/lib_step.so --config $c $A > $OUT/ab_$c.json 2>> $OUT/err.log
done
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
echo done
