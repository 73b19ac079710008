#!/bin/bash
# Round-4 leaf-certificate A/B (via gpurun): the certified walk with leaf certificates against
# box culling and the round-3 relative slack, and the mode-2 build switches
# (abvar/lib_lc0.so: -DRT_LEAFCERT_LDS=0, lib_cp0.so: -DRT_LDS_COMPACT=0, lib_both0.so: both),
# then the GPU parity tests of the triangle paths.
# usage: bash tools/gpu_lcert.sh <tag> [steps...]   (steps: ab5 ab3 abr03 diag tests)
set -e -o pipefail
TAG=${1:-r04_c}; shift || true
STEPS=${*:-ab5 ab3 tests}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
L=rust_gpu_raytracing_amd/librt_pathtrace.so
for s in $STEPS; do
  echo "== $s $(date +%T)"
  case $s in
    ab5)
      timeout -k 10 300 python3 tools/ab_bench.py "$L:RT_TRI_PRUNE=1" "$L:RT_TRI_PRUNE=0" "$L:RT_TRI_PRUNE=2" \
        --config c5_heightfield --frames 20 --frame-batch 20 --rounds 3 > "$OUT/ab_c5.json" 2> "$OUT/ab_c5.err" ;;
    ab3)
      for c in c3_chess c4_mixed; do
        timeout -k 10 300 python3 tools/ab_bench.py "$L:RT_TRI_PRUNE=1" "$L:RT_TRI_PRUNE=0" "$L:RT_TRI_PRUNE=2" \
          "$L:RT_TRI_PRUNE=1,RT_TRI_LEAFCERT_LDS=0" abvar/lib_lc0.so "abvar/lib_cp0.so:RT_TRI_LDS_COMPACT=0" \
          "abvar/lib_both0.so:RT_TRI_LDS_COMPACT=0" "abvar/lib_both0.so:RT_TRI_LDS_COMPACT=0,RT_TRI_PRUNE=2" \
          --config $c --frames 20 --frame-batch 20 --rounds 5 > "$OUT/ab_$c.json" 2> "$OUT/ab_$c.err"
      done ;;
    abr03)  # round-3 final build (abvar/lib_r03.so, its relative-slack default) against this one
      for c in c2_rtiow c3_chess c4_mixed c5_heightfield; do
        timeout -k 10 300 python3 tools/ab_bench.py abvar/lib_r03.so "$L" "$L:RT_TRI_PRUNE=0" "$L:RT_TRI_PRUNE=2" \
          --config $c --frames 20 --frame-batch 20 --rounds 5 > "$OUT/abr03_$c.json" 2> "$OUT/abr03_$c.err"
      done ;;
    diag)
      RT_LIB=abvar/lib_diag.so timeout -k 10 300 python3 tools/diag_split.py --frame-batch 20 c5_heightfield c3_chess c2_rtiow \
        > "$OUT/diag.jsonl" 2> "$OUT/diag.err" ;;
    tests)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$OUT/tests.log" 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
