#!/bin/bash
# Round-5 GPU passes (run via gpurun). usage: bash tools/gpu_r05.sh <tag> <step>...
#   steps: t:<pytest -k expr> | tests | smoke | bench | all | strong[:config[:gather]] | prof[:args]
# Every GPU step runs under its own time limit; the script stops at the first failure.
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -c "import __graft_entry__ as g; g.build()" > "$OUT/build.log" 2>&1
i=0
for s in "$@"; do
  i=$((i+1))
  echo "== $s $(date +%T)"
  case $s in
    t:*) timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
           -k "${s#t:}" > "$OUT/tests_$i.log" 2>&1 ;;
    tests) timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
           > "$OUT/tests.log" 2>&1 ;;
    smoke) timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    bench) timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    bench:*) a=${s#bench:}; timeout -k 10 400 python3 bench.py ${a//,/ } > "$OUT/bench_$i.json" 2> "$OUT/bench_$i.err" ;;
    all) timeout -k 10 600 python3 tools/bench_all.py --no-cpu --frames 20 > "$OUT/bench_all.jsonl" 2> "$OUT/bench_all.err" ;;
    strong:*) IFS=: read -r _ cfg gat <<< "$s"
           timeout -k 10 600 python3 tools/strong_probe.py --steps 20 --config "${cfg:-c2_rtiow}" --gather "${gat:-accumulation}" \
             > "$OUT/strong_${cfg}_${gat}.jsonl" 2> "$OUT/strong_${cfg}_${gat}.err" ;;
    ab:*) a=${s#ab:}; timeout -k 10 900 python3 tools/ab_env.py ${a//,/ } > "$OUT/ab_$i.jsonl" 2> "$OUT/ab_$i.err" ;;
    prof) bash tools/profile.sh "$TAG" ;;
    prof:*) a=${s#prof:}; bash tools/profile.sh "${TAG}_$i" ${a//,/ } ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
