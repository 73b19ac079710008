# round-5 session script (scratch): lazy triangle piece loads -- tests and A/B against the previous build
set -o pipefail
mkdir -p gpurun_out/r05o
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "triangle or chess or golden or pruning or walk" > gpurun_out/r05o/tests.log 2>&1 || exit 1
for c in c3_chess c4_mixed c5_heightfield; do
  timeout -k 10 300 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_nolazy.so abvar/lib_head.so --config $c --rounds 4 --frames 40 --frame-batch 20 > gpurun_out/r05o/ab_$c.json 2> gpurun_out/r05o/ab_$c.err || exit 1
done
