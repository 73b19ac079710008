#!/bin/bash
# Session 6: node steps per wave-wide check (RT_TRAV_UNROLL 2/3/4/5) and the traversal threshold
# (RT_TRAV_THRESHOLD) re-measured on the box-ordered build, C2 whole frame and 8-way share, C1.
set -e -o pipefail
echo start
OUT=gpurun_out/r02_s6c
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
L="$V/lib_cur.so $V/lib_u2.so $V/lib_u4.so $V/lib_u5.so $V/lib_cur.so:RT_TRAV_THRESHOLD=6 $V/lib_cur.so:RT_TRAV_THRESHOLD=10 $V/lib_cur.so:RT_TRAV_THRESHOLD=12"
timeout -k 10 200 python3 -u tools/ab_bench.py $L --config c2_rtiow --frames 20 --rounds 9 --frame-batch 20 > $OUT/ab_c2.json 2>> $OUT/err.log
echo c2 done
timeout -k 10 200 python3 -u tools/ab_bench.py $L --config c2_rtiow --frames 20 --rounds 9 --frame-batch 20 --world 8 > $OUT/ab_c2_w8.json 2>> $OUT/err.log
echo w8 done
timeout -k 10 200 python3 -u tools/ab_bench.py $L --config c1_four_spheres --frames 20 --rounds 9 --frame-batch 20 > $OUT/ab_c1.json 2>> $OUT/err.log
echo done
