#!/bin/bash
# Session 4: kernel timeline of the N=8 share (20 steps) -- gaps around the path and resolve kernels.
set -e -o pipefail
OUT=gpurun_out/r02_s4h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/trace8 -o run -- python3 tools/strong_probe.py --ns 8 --steps 20 > $OUT/strong8.jsonl 2> $OUT/trace8.err
echo done
