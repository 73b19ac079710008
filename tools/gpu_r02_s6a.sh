#!/bin/bash
# Session 6: drain pool (RT_POOL_PUSH) -- A/B of push thresholds against the pool-off build and the
# previous build on C2 (whole frame and an 8-way share) and C3, then the GPU suite with the pool on.
set -e -o pipefail
echo start
OUT=gpurun_out/r02_s6a
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
L="$V/lib_cur.so $V/lib_pool.so $V/lib_pool.so:RT_POOL_PUSH=8 $V/lib_pool.so:RT_POOL_PUSH=16 $V/lib_pool.so:RT_POOL_PUSH=32"
timeout -k 10 200 python3 -u tools/ab_bench.py $L --config c2_rtiow --frames 20 --rounds 7 --frame-batch 20 --world 8 > $OUT/ab_c2_w8.json 2>> $OUT/err.log
echo w8 done
timeout -k 10 200 python3 -u tools/ab_bench.py $L --config c2_rtiow --frames 20 --rounds 7 --frame-batch 20 > $OUT/ab_c2.json 2>> $OUT/err.log
echo c2 done
timeout -k 10 200 python3 -u tools/ab_bench.py $L --config c3_chess --frames 20 --rounds 5 --frame-batch 20 > $OUT/ab_c3.json 2>> $OUT/err.log
echo ab done
RT_POOL_PUSH=16 timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests_pool16.log 2>&1
echo done
