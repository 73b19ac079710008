#!/bin/bash
# Session 4: knob sweep 2 -- leaf batch and traversal threshold combinations (20-frame launches).
set -e -o pipefail
OUT=gpurun_out/r02_s4l
mkdir -p $OUT
export TMPDIR=/tmp
L=rust_gpu_raytracing_amd/librt_pathtrace.so
A="--frames 20 --rounds 5 --frame-batch 20"
timeout -k 10 300 python3 tools/ab_bench.py $L $L:RT_LEAF_BATCH=6 $L:RT_LEAF_BATCH=5 $L:RT_LEAF_BATCH=4 $L:RT_TRAV_THRESHOLD=32,RT_LEAF_BATCH=6 $L:RT_TRAV_THRESHOLD=32,RT_LEAF_BATCH=5 $L:RT_TRAV_THRESHOLD=40,RT_LEAF_BATCH=6 --config c3_chess $A > $OUT/ab_c3.json 2>> $OUT/err.log
timeout -k 10 300 python3 tools/ab_bench.py $L $L:RT_LEAF_BATCH=6 $L:RT_LEAF_BATCH=5 $L:RT_LEAF_BATCH=4 $L:RT_TRAV_THRESHOLD=16,RT_LEAF_BATCH=6 $L:RT_TRAV_THRESHOLD=16,RT_LEAF_BATCH=5 --config c4_mixed --width 3840 --height 2160 --frames 20 --rounds 3 --frame-batch 20 > $OUT/ab_c4.json 2>> $OUT/err.log
timeout -k 10 300 python3 tools/ab_bench.py $L $L:RT_LEAF_BATCH=5 $L:RT_LEAF_BATCH=4 $L:RT_LEAF_BATCH=3 --config c5_heightfield --frames 20 --rounds 3 --frame-batch 20 > $OUT/ab_c5.json 2>> $OUT/err.log
echo done
