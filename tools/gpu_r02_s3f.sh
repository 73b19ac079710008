#!/bin/bash
# Session 3: strong-scaling batch size at the driver's 20 steps (one rank's share timed alone).
set -e -o pipefail
OUT=gpurun_out/r02_s3f
mkdir -p $OUT
export TMPDIR=/tmp
for fb in 10 20; do
  timeout -k 10 300 python3 tools/strong_probe.py --steps 20 --ns 2 4 8 --frame-batch $fb > $OUT/strong_fb$fb.jsonl 2>> $OUT/err.log
done
timeout -k 10 300 python3 tools/strong_probe.py --steps 20 --ns 1 8 > $OUT/strong_default.jsonl 2>> $OUT/err.log
echo done
