#!/bin/bash
# Interleaved A/B of one build under per-context environment settings, on several configs
# (tools/ab_env.py), each config under its own time limit. Run via gpurun:
#   bash tools/gpu_ab.sh <tag> "<config> ..." "<spec>" "<spec>" ...
# e.g. bash tools/gpu_ab.sh r03_w "c3_chess c5_heightfield" "RT_TRI_WIDE=0" "RT_TRI_WIDE=1"
# Env: AB_FRAMES (20), AB_BATCH (20), AB_ROUNDS (3).
set -e -o pipefail
TAG=$1; CONFIGS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in $CONFIGS; do
  echo "== ab $c $(date +%T)"
  timeout -k 10 300 python3 tools/ab_env.py --config "$c" --frames "${AB_FRAMES:-20}" \
    --frame-batch "${AB_BATCH:-20}" --rounds "${AB_ROUNDS:-3}" "$@" >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err"
done
echo "== done $(date +%T)"
