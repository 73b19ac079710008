#!/bin/bash
# Round-4 measurement pass (via gpurun): triangle pruning modes A/B (certified default, box
# culling, the round-3 relative slack), the persistent grid's ramp/drain at the 8-way share
# (RT_DIAG_TAIL variant in abvar/), the strong probe.
# usage: bash tools/gpu_r04.sh <tag> [steps...]  (steps: prune tail strong diag)
set -e -o pipefail
TAG=${1:-r04_m}; shift || true
STEPS=${*:-prune tail strong}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for s in $STEPS; do
  echo "== $s $(date +%T)"
  case $s in
    prune)
      for c in c5_heightfield c3_chess c4_mixed; do
        timeout -k 10 300 python3 tools/ab_env.py "RT_TRI_PRUNE=1" "RT_TRI_PRUNE=0" "RT_TRI_PRUNE=2" \
          --config $c --frames 20 --frame-batch 20 --rounds 5 >> "$OUT/ab_prune.jsonl" 2>> "$OUT/ab_prune.err"
      done ;;
    knobs5)  # C5 under the certified default: layouts, pre-pass, thresholds re-tuned for an unpruned walk
      timeout -k 10 400 python3 tools/ab_env.py "RT_TRI_PRUNE=1" "RT_TRI_PRUNE=1 RT_TRI_OCTANTS=0" \
        "RT_TRI_PRUNE=1 RT_PRIMARY_PASS=0" "RT_TRI_PRUNE=1 RT_TRAV_THRESHOLD=32" "RT_TRI_PRUNE=1 RT_TRAV_THRESHOLD=24" \
        "RT_TRI_PRUNE=1 RT_LEAF_BATCH=4" "RT_TRI_PRUNE=1 RT_LEAF_BATCH=6" \
        --config c5_heightfield --frames 20 --frame-batch 20 --rounds 3 >> "$OUT/ab_knobs5.jsonl" 2>> "$OUT/ab_knobs5.err" ;;
    c3)  # the LDS vertex table (mode 2) on C3 and C4 at 1080p, certified default
      for c in c3_chess c4_mixed; do
        timeout -k 10 300 python3 tools/ab_env.py "RT_TRI_LDS_COMPACT=1" "RT_TRI_LDS_COMPACT=0" \
          "RT_TRI_LDS_COMPACT=0 RT_STAGE_SUBS=0" --config $c --frames 20 --frame-batch 20 --rounds 5 \
          >> "$OUT/ab_compact.jsonl" 2>> "$OUT/ab_compact.err"
      done ;;
    tail)
      RT_LIB=abvar/lib_tail.so timeout -k 10 300 python3 tools/tail_probe.py --frame-batch 20 --split 0/8 c2_rtiow \
        > "$OUT/tail_8way.jsonl" 2> "$OUT/tail.err"
      RT_LIB=abvar/lib_tail.so timeout -k 10 300 python3 tools/tail_probe.py --frame-batch 20 c2_rtiow \
        > "$OUT/tail_full.jsonl" 2>> "$OUT/tail.err" ;;
    diag)
      RT_LIB=abvar/lib_diag.so timeout -k 10 300 python3 tools/diag_split.py --frame-batch 20 c2_rtiow c3_chess \
        > "$OUT/diag.jsonl" 2> "$OUT/diag.err" ;;
    share8)  # the 8-way share (N=8 strong bench per rank): LDS image and threshold knobs
      timeout -k 10 300 python3 tools/ab_env.py "RT_TILE_SCHEDULE=1" "RT_SPHERE_OCTANTS=0" "RT_TRAV_THRESHOLD=4" \
        "RT_TRAV_THRESHOLD=12" "RT_TILE_SCHEDULE=0" "RT_BLOCK_THREADS=512" --split 0/8 --config c2_rtiow \
        --frames 20 --frame-batch 20 --rounds 7 >> "$OUT/ab_share8.jsonl" 2>> "$OUT/ab_share8.err" ;;
    strong) timeout -k 10 300 python3 tools/strong_probe.py --steps 20 > "$OUT/strong_probe.jsonl" 2> "$OUT/strong_probe.err" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
