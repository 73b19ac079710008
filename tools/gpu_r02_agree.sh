# rocprof kernel-trace vs the bench's device-clock spans, batches overlapped (default) and not
set -e -o pipefail
OUT=gpurun_out/r02_agree
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --steps 16 --warmup 8 --no-cpu-baseline"
timeout -k 10 300 python3 $B > $OUT/bench_ovl.json 2> $OUT/err.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_ovl -o run -- python3 $B > $OUT/trace_ovl_bench.json 2>> $OUT/err.log
RT_BATCH_OVERLAP=0 timeout -k 10 300 python3 $B > $OUT/bench_seq.json 2>> $OUT/err.log
RT_BATCH_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_seq -o run -- python3 $B > $OUT/trace_seq_bench.json 2>> $OUT/err.log
echo done
