#!/bin/bash
# Session 4: per-launch times after a short warmup (clock ramp?), bench twice.
set -e -o pipefail
OUT=gpurun_out/r02_s4d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/warm_probe.py --warmup 5 --launches 10 > $OUT/warm5.json 2>> $OUT/err.log
timeout -k 10 120 python3 tools/warm_probe.py --warmup 5 --launches 6 --gap-ms 100 > $OUT/warm5_gap100.json 2>> $OUT/err.log
timeout -k 10 120 python3 tools/warm_probe.py --warmup 5 --launches 6 --config c3_chess > $OUT/warm5_c3.json 2>> $OUT/err.log
timeout -k 10 300 python3 bench.py --warmup 5 --no-cpu-baseline > $OUT/bench_w5.json 2>> $OUT/err.log
timeout -k 10 300 python3 bench.py --warmup 100 --no-cpu-baseline > $OUT/bench_w100.json 2>> $OUT/err.log
echo done
