#!/bin/bash
# Session 6: waves per CU for the strong split's small shares (RT_WAVES_PER_CU 8 = 512-thread
# workgroups, 2 waves per SIMD, against the default 16): a shorter drain per launch against a
# slower steady state. 8-way and 4-way C2 shares and the whole frame.
set -e -o pipefail
echo start
OUT=gpurun_out/r02_s6e
mkdir -p $OUT
export TMPDIR=/tmp
P=rust_gpu_raytracing_amd/librt_pathtrace.so
L="$P $P:RT_WAVES_PER_CU=8 $P:RT_WAVES_PER_CU=4"
for w in 8 4 1; do
  timeout -k 10 200 python3 -u tools/ab_bench.py $L --config c2_rtiow --frames 20 --rounds 9 --frame-batch 20 --world $w > $OUT/ab_c2_w$w.json 2>> $OUT/err.log
  echo "w$w done"
done
