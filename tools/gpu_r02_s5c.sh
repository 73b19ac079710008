#!/bin/bash
# Session 5: box-ordered sphere layouts (slab_hit_ordered in the sphere-only kernels) -- A/B against the
# same build with RT_SPHERE_BOX_ORDER=0 and against the previous build, then the GPU test suite.
set -e -o pipefail
echo start
OUT=gpurun_out/r02_s5c
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
L="$V/lib_box.so $V/lib_box.so:RT_SPHERE_BOX_ORDER=0 $V/lib_cur.so"
timeout -k 10 150 python3 -u tools/ab_bench.py $L --config c2_rtiow --frames 20 --rounds 9 --frame-batch 20 > $OUT/ab_c2.json 2>> $OUT/err.log
timeout -k 10 150 python3 -u tools/ab_bench.py $L --config c2_rtiow --frames 20 --rounds 9 --frame-batch 20 --world 8 > $OUT/ab_c2_w8.json 2>> $OUT/err.log
timeout -k 10 150 python3 -u tools/ab_bench.py $L --config c1_four_spheres --frames 20 --rounds 9 --frame-batch 20 > $OUT/ab_c1.json 2>> $OUT/err.log
timeout -k 10 150 python3 -u tools/ab_bench.py $L --config c3_chess --frames 20 --rounds 5 --frame-batch 20 > $OUT/ab_c3.json 2>> $OUT/err.log
echo ab done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
echo done
