#!/bin/bash
# Session 6: claim order for the strong split's drain -- cost-ordered claims in frame-parallel
# batches (RT_BATCH_SCHEDULE=1), tile-major or frame-major units, on the 8-way C2 share and whole C2.
set -e -o pipefail
echo start
OUT=gpurun_out/r02_s6b
mkdir -p $OUT
export TMPDIR=/tmp
L="rust_gpu_raytracing_amd/librt_pathtrace.so rust_gpu_raytracing_amd/librt_pathtrace.so:RT_BATCH_SCHEDULE=1 rust_gpu_raytracing_amd/librt_pathtrace.so:RT_BATCH_SCHEDULE=1,RT_UNIT_TILE_MAJOR=0 rust_gpu_raytracing_amd/librt_pathtrace.so:RT_UNIT_TILE_MAJOR=0"
timeout -k 10 200 python3 -u tools/ab_bench.py $L --config c2_rtiow --frames 20 --rounds 9 --frame-batch 20 --world 8 > $OUT/ab_c2_w8.json 2>> $OUT/err.log
timeout -k 10 200 python3 -u tools/ab_bench.py $L --config c2_rtiow --frames 20 --rounds 9 --frame-batch 20 --world 4 > $OUT/ab_c2_w4.json 2>> $OUT/err.log
timeout -k 10 200 python3 -u tools/ab_bench.py $L --config c2_rtiow --frames 20 --rounds 7 --frame-batch 20 > $OUT/ab_c2.json 2>> $OUT/err.log
echo done
