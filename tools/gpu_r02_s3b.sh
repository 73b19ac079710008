#!/bin/bash
# Session 3: RT_DIAG split with leaf-step time (C2, C3, C5; batches of 8).
set -e -o pipefail
OUT=gpurun_out/r02_s3b
mkdir -p $OUT
export TMPDIR=/tmp
RT_LIB=build/variants/lib_diag.so timeout -k 10 300 python3 tools/diag_split.py --frame-batch 8 c2_rtiow c3_chess c5_heightfield > $OUT/diag_split_fb8.jsonl 2> $OUT/diag.err
echo done
