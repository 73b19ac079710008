#!/bin/bash
# Session 3: reverse claim order (ends launches on the sky bands of C2) -- A/B at N=1 and the 8-way share.
set -e -o pipefail
OUT=gpurun_out/r02_s3j
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
A="--frames 32 --rounds 4 --frame-batch 8"
for c in c2_rtiow c3_chess c4_mixed; do
  timeout -k 10 300 python3 tools/ab_bench.py $V/lib_rev.so $V/lib_rev.so:RT_CLAIM_REVERSE=1 --config $c $A > $OUT/ab_$c.json 2>> $OUT/err.log
done
for i in 1 2; do
  timeout -k 10 300 python3 tools/strong_probe.py --steps 20 --ns 1 8 >> $OUT/strong_fwd.jsonl 2>> $OUT/err.log
  RT_CLAIM_REVERSE=1 timeout -k 10 300 python3 tools/strong_probe.py --steps 20 --ns 1 8 >> $OUT/strong_rev.jsonl 2>> $OUT/err.log
done
RT_CLAIM_REVERSE=1 RT_LIB=$V/lib_tail.so timeout -k 10 300 python3 tools/tail_probe.py --frame-batch 20 --split 0/8 c2_rtiow > $OUT/tail_split8_fb20_rev.jsonl 2>> $OUT/err.log
echo done
