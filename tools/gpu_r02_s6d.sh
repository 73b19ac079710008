#!/bin/bash
# Session 6: device scheduler strategy / optimisation level (same sources, numerics flags unchanged):
# gcn-max-ilp, occupancy-only metric bias, -O2, against the product flags; C2, C2 8-way share, C3.
set -e -o pipefail
echo start
OUT=gpurun_out/r02_s6d
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
L="$V/lib_cur.so $V/lib_ilp.so $V/lib_bias100.so $V/lib_o2.so"
timeout -k 10 200 python3 -u tools/ab_bench.py $L --config c2_rtiow --frames 20 --rounds 9 --frame-batch 20 > $OUT/ab_c2.json 2>> $OUT/err.log
echo c2 done
timeout -k 10 200 python3 -u tools/ab_bench.py $L --config c2_rtiow --frames 20 --rounds 9 --frame-batch 20 --world 8 > $OUT/ab_c2_w8.json 2>> $OUT/err.log
timeout -k 10 200 python3 -u tools/ab_bench.py $L --config c3_chess --frames 20 --rounds 7 --frame-batch 20 > $OUT/ab_c3.json 2>> $OUT/err.log
echo done
