#!/bin/bash
# Session 3: wave-cooperative triangle leaves -- GPU parity tests, then A/B against RT_TRI_COOP=0.
set -e -o pipefail
OUT=gpurun_out/r02_s3d
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
A="--frames 16 --rounds 3 --frame-batch 8"
for c in c3_chess c4_mixed; do
  timeout -k 10 300 python3 tools/ab_bench.py $V/lib_coop.so $V/lib_coop.so:RT_TRI_COOP=0 --config $c $A > $OUT/ab_$c.json 2>> $OUT/err.log
done
timeout -k 10 300 python3 tools/ab_bench.py $V/lib_coop.so $V/lib_coop.so:RT_TRI_COOP=0 --config c5_heightfield --frames 8 --rounds 2 --frame-batch 8 > $OUT/ab_c5_heightfield.json 2>> $OUT/err.log
echo done
