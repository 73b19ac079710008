set -e -o pipefail
OUT=gpurun_out/r02_diag
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/parity_budget.py build/variants/hw_transc.so > $OUT/parity_budget.jsonl 2> $OUT/parity_budget.err
for fb in 1 8; do
  RT_LIB=build/variants/lib_tail.so timeout -k 10 300 python3 tools/tail_probe.py --frame-batch $fb c2_rtiow c3_chess > $OUT/tail_fb$fb.jsonl 2> $OUT/tail.err
done
echo done
