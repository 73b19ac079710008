#!/bin/bash
# Session 3: 8-way share at 20 steps with the cost-ordered claim schedule for batches.
set -e -o pipefail
OUT=gpurun_out/r02_s3i
mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python3 tools/strong_probe.py --steps 20 --ns 8 >> $OUT/strong_default.jsonl 2>> $OUT/err.log
  RT_BATCH_SCHEDULE=1 timeout -k 10 300 python3 tools/strong_probe.py --steps 20 --ns 8 >> $OUT/strong_sched.jsonl 2>> $OUT/err.log
  RT_BATCH_SCHEDULE=1 timeout -k 10 300 python3 tools/strong_probe.py --steps 20 --ns 1 >> $OUT/strong_sched.jsonl 2>> $OUT/err.log
done
RT_BATCH_SCHEDULE=1 RT_LIB=build/variants/lib_tail.so timeout -k 10 300 python3 tools/tail_probe.py --frame-batch 20 --split 0/8 c2_rtiow > $OUT/tail_split8_fb20_sched.jsonl 2>> $OUT/err.log
echo done
