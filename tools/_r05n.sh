# round-5 session script (scratch): C5 regression check (ABI-11 commit build vs now, q4 compiled in/out)
set -o pipefail
mkdir -p gpurun_out/r05n
timeout -k 10 600 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_3e26.so abvar/lib_q4.so --config c5_heightfield --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/r05n/ab_c5.json 2> gpurun_out/r05n/ab_c5.err || exit 1
timeout -k 10 300 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_3e26.so --config c3_chess --rounds 5 --frames 40 --frame-batch 20 > gpurun_out/r05n/ab_c3.json 2> gpurun_out/r05n/ab_c3.err || exit 1
timeout -k 10 300 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_3e26.so --config c2_rtiow --rounds 5 --frames 40 --frame-batch 20 > gpurun_out/r05n/ab_c2.json 2> gpurun_out/r05n/ab_c2.err || exit 1
