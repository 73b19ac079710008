#!/bin/bash
# Session 3: where an 8-way share's time goes at the driver's 20 steps (kernel span vs wall; ramp/dry/drain).
set -e -o pipefail
OUT=gpurun_out/r02_s3g
mkdir -p $OUT
export TMPDIR=/tmp
python3 -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1
timeout -k 10 300 python3 tools/strong_probe.py --steps 20 --ns 1 8 > $OUT/strong_spans.jsonl 2>> $OUT/err.log
RT_LIB=build/variants/lib_tail.so timeout -k 10 300 python3 tools/tail_probe.py --frame-batch 20 --split 0/8 c2_rtiow > $OUT/tail_split8_fb20.jsonl 2>> $OUT/err.log
RT_LIB=build/variants/lib_tail.so timeout -k 10 300 python3 tools/tail_probe.py --frame-batch 8 c2_rtiow > $OUT/tail_fb8.jsonl 2>> $OUT/err.log
echo done
