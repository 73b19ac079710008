#!/bin/bash
# Session 3: one-round-trip stripe scan in claim_tile -- tests, A/B, 8-way share.
set -e -o pipefail
OUT=gpurun_out/r02_s3h
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
A="--frames 32 --rounds 4 --frame-batch 8"
for c in c2_rtiow c3_chess c1_four_spheres; do
  timeout -k 10 300 python3 tools/ab_bench.py $V/lib_cur.so $V/lib_scan.so --config $c $A > $OUT/ab_$c.json 2>> $OUT/err.log
done
for lib in lib_cur lib_scan lib_cur lib_scan; do
  RT_LIB=$V/$lib.so timeout -k 10 300 python3 tools/strong_probe.py --steps 20 --ns 1 8 >> $OUT/strong_$lib.jsonl 2>> $OUT/err.log
done
echo done
