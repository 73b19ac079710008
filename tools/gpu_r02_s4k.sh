#!/bin/bash
# Session 4: knob sweep at the bench's launch shape (20-frame launches).
set -e -o pipefail
OUT=gpurun_out/r02_s4k
mkdir -p $OUT
export TMPDIR=/tmp
L=rust_gpu_raytracing_amd/librt_pathtrace.so
A="--frames 20 --rounds 5 --frame-batch 20"
timeout -k 10 300 python3 tools/ab_bench.py $L $L:RT_TRAV_THRESHOLD=4 $L:RT_TRAV_THRESHOLD=12 $L:RT_TRAV_THRESHOLD=16 $L:RT_QUEUE_STRIPES=16 $L:RT_QUEUE_STRIPES=64 --config c2_rtiow $A > $OUT/ab_c2.json 2>> $OUT/err.log
timeout -k 10 300 python3 tools/ab_bench.py $L $L:RT_TRAV_THRESHOLD=16 $L:RT_TRAV_THRESHOLD=32 $L:RT_LEAF_BATCH=5 $L:RT_LEAF_BATCH=6 $L:RT_LEAF_BATCH=8 --config c3_chess $A > $OUT/ab_c3.json 2>> $OUT/err.log
timeout -k 10 300 python3 tools/ab_bench.py $L $L:RT_TRAV_THRESHOLD=16 $L:RT_TRAV_THRESHOLD=32 $L:RT_LEAF_BATCH=6 $L:RT_LEAF_BATCH=8 --config c4_mixed --width 3840 --height 2160 --frames 20 --rounds 3 --frame-batch 20 > $OUT/ab_c4.json 2>> $OUT/err.log
timeout -k 10 300 python3 tools/ab_bench.py $L $L:RT_LEAF_BATCH=5 $L:RT_LEAF_BATCH=7 $L:RT_DRAIN_THRESHOLD=16 $L:RT_DRAIN_THRESHOLD=48 --config c5_heightfield --frames 20 --rounds 3 --frame-batch 20 > $OUT/ab_c5.json 2>> $OUT/err.log
echo done
