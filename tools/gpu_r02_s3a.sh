#!/bin/bash
# Session 3 check: strong-scaling probe at the driver's 20 steps, gather rehearsal (gloo, 2/4/8 ranks on one GPU).
set -e -o pipefail
OUT=gpurun_out/r02_s3a
mkdir -p $OUT
export TMPDIR=/tmp
python3 -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1
timeout -k 10 300 python3 tools/strong_probe.py --steps 20 > $OUT/strong_probe_s20.jsonl 2> $OUT/strong_probe.err
timeout -k 10 300 python3 tools/strong_probe.py --steps 40 --ns 1 8 > $OUT/strong_probe_s40.jsonl 2>> $OUT/strong_probe.err
bash tools/gpu_check.sh r02_s3a_m multi
echo done
