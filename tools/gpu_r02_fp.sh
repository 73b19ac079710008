set -e -o pipefail
OUT=gpurun_out/r02_fp
mkdir -p $OUT
export TMPDIR=/tmp
python3 -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
for fb in 1 4 8; do
  timeout -k 10 300 python3 tools/bench_all.py --no-cpu --frames 16 --frame-batch $fb > $OUT/all_fb$fb.jsonl 2>> $OUT/all.err
done
timeout -k 10 300 python3 tools/strong_probe.py > $OUT/strong_probe.jsonl 2> $OUT/strong_probe.err
echo done
