#!/bin/bash
# Session 3: frame batch size at the driver's 20 steps, N=1 and the 2-way share.
set -e -o pipefail
OUT=gpurun_out/r02_s3n
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  for fb in 7 8 10 20; do
    timeout -k 10 300 python3 tools/strong_probe.py --steps 20 --ns 1 --frame-batch $fb >> $OUT/n1_fb$fb.jsonl 2>> $OUT/err.log
  done
  for fb in 10 16 20; do
    timeout -k 10 300 python3 tools/strong_probe.py --steps 20 --ns 2 --frame-batch $fb >> $OUT/n2_fb$fb.jsonl 2>> $OUT/err.log
  done
done
echo done
