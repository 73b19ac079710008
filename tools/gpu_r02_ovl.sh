set -e -o pipefail
OUT=gpurun_out/r02_ovl
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
for c in c2_rtiow c3_chess c1_four_spheres; do
  timeout -k 10 300 python3 tools/ab_bench.py $V/lib_ovl.so:RT_BATCH_OVERLAP=0 $V/lib_ovl.so:RT_BATCH_OVERLAP=1 --config $c --frames 32 --rounds 5 --frame-batch 8 > $OUT/ab_$c.json 2>> $OUT/err.log
done
timeout -k 10 300 python3 tools/strong_probe.py > $OUT/strong_probe.jsonl 2> $OUT/strong.err
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
echo done
