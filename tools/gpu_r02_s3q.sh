#!/bin/bash
# Session 3: C5 PMC profile of the current build + RT_DIAG split at 20-frame launches.
set -e -o pipefail
OUT=gpurun_out/r02_s3q
mkdir -p $OUT
export TMPDIR=/tmp
RT_LIB=build/variants/lib_diag.so timeout -k 10 300 python3 tools/diag_split.py --frame-batch 20 c2_rtiow c3_chess c5_heightfield > $OUT/diag_split_fb20.jsonl 2> $OUT/diag.err
bash tools/profile.sh r02_c5v6 --config c5_heightfield
echo done
