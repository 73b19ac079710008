set -e -o pipefail
OUT=gpurun_out/r02_fp2
mkdir -p $OUT
export TMPDIR=/tmp
python3 -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1
timeout -k 10 300 python3 tools/strong_probe.py > $OUT/strong_probe.jsonl 2> $OUT/strong_probe.err
timeout -k 10 300 python3 tools/strong_probe.py --ns 1 8 --steps 96 > $OUT/strong_probe96.jsonl 2>> $OUT/strong_probe.err
for fb in 4 8; do
  timeout -k 10 300 python3 bench.py --frame-batch $fb --no-cpu-baseline > $OUT/bench_fb$fb.json 2> $OUT/bench_fb$fb.err
done
echo done
