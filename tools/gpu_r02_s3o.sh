#!/bin/bash
# Session 3: frame batch size for longer runs at N=1 (64 steps).
set -e -o pipefail
OUT=gpurun_out/r02_s3o
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for fb in 8 16 32 64; do
    timeout -k 10 300 python3 tools/strong_probe.py --steps 64 --ns 1 --frame-batch $fb >> $OUT/n1_s64_fb$fb.jsonl 2>> $OUT/err.log
  done
done
for c in c3_chess c5_heightfield; do
  for fb in 8 20; do
    timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 3 --frame-batch $fb --no-cpu-baseline >> $OUT/bench_${c}_fb$fb.jsonl 2>> $OUT/err.log
  done
done
echo done
