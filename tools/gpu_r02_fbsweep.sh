set -e -o pipefail
OUT=gpurun_out/r02_fbsweep
mkdir -p $OUT
export TMPDIR=/tmp
for st in 20 40; do
for fb in 8 16 32 64; do
  timeout -k 10 300 python3 tools/strong_probe.py --ns 8 --steps $st --frame-batch $fb > $OUT/n8_s${st}_fb$fb.jsonl 2>> $OUT/err.log
done
timeout -k 10 300 python3 tools/strong_probe.py --ns 1 --steps $st --frame-batch 8 > $OUT/n1_s${st}_fb8.jsonl 2>> $OUT/err.log
done
echo done
