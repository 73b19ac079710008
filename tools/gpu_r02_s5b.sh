#!/bin/bash
# Session 5: traversal threshold during the drain for the LDS-resident instances (RT_DRAIN_PLAIN) -- A/B,
# full C2 frame and an 8-way share (rank 0), 20-frame launches.
set -e -o pipefail
echo start
OUT=gpurun_out/r02_s5b
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
L="$V/lib_cur.so $V/lib_dp4.so $V/lib_dp8.so $V/lib_dp16.so"
timeout -k 10 150 python3 -u tools/ab_bench.py $L --config c2_rtiow --frames 20 --rounds 7 --frame-batch 20 > $OUT/ab_c2.json 2>> $OUT/err.log
timeout -k 10 150 python3 -u tools/ab_bench.py $L --config c2_rtiow --frames 20 --rounds 9 --frame-batch 20 --world 8 > $OUT/ab_c2_w8.json 2>> $OUT/err.log
timeout -k 10 150 python3 -u tools/ab_bench.py $L --config c3_chess --frames 20 --rounds 5 --frame-batch 20 > $OUT/ab_c3.json 2>> $OUT/err.log
echo done
