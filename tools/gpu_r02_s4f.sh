#!/bin/bash
# Session 4: child-pair sphere BVH walk with a register stack -- tests + A/B + N=8 share.
set -e -o pipefail
OUT=gpurun_out/r02_s4f
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
A="--frames 40 --rounds 4 --frame-batch 20"
for c in c2_rtiow c1_four_spheres; do
  timeout -k 10 300 python3 tools/ab_bench.py $V/lib_base.so $V/lib_step.so $V/lib_pairs.so --config $c $A > $OUT/ab_$c.json 2>> $OUT/err.log
done
for l in lib_base lib_pairs; do
  RT_LIB=$V/$l.so timeout -k 10 200 python3 tools/strong_probe.py --ns 1 8 --steps 20 > $OUT/strong_$l.jsonl 2>> $OUT/err.log
done
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
echo done
