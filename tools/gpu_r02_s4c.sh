#!/bin/bash
# Session 4: issue priority in the drain -- A/B (C2/C3 20-frame launches) and the N=8 share.
set -e -o pipefail
OUT=gpurun_out/r02_s4c
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
A="--frames 20 --rounds 5 --frame-batch 20"
for c in c2_rtiow c3_chess; do
  timeout -k 10 300 python3 tools/ab_bench.py $V/lib_step.so $V/lib_prio2.so $V/lib_prioall.so --config $c $A > $OUT/ab_$c.json 2>> $OUT/err.log
done
for l in lib_step lib_prio2 lib_prioall lib_step; do
  RT_LIB=$V/$l.so timeout -k 10 200 python3 tools/strong_probe.py --ns 8 --steps 20 > $OUT/strong_$l.jsonl 2>> $OUT/err.log
done
echo done
