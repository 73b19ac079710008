# round-5 session script (scratch): cooperative leaf batches in the LDS-resident walk (RT_COOP_LDS build)
set -o pipefail
mkdir -p gpurun_out/r05ab
RT_LIB=abvar/lib_cooplds.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "chess or c3 or c4 or mixed or golden or lds or full_frame" > gpurun_out/r05ab/tests.log 2>&1 || exit 1
timeout -k 10 400 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_cooplds.so --config c3_chess --rounds 5 --frames 40 --frame-batch 20 > gpurun_out/r05ab/ab_c3.json 2> gpurun_out/r05ab/ab_c3.err || exit 1
timeout -k 10 400 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_cooplds.so --config c4_mixed --width 3840 --height 2160 --rounds 3 --frames 20 --frame-batch 20 > gpurun_out/r05ab/ab_c4.json 2> gpurun_out/r05ab/ab_c4.err || exit 1
timeout -k 10 400 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_cooplds.so --config c2_rtiow --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/r05ab/ab_c2.json 2> gpurun_out/r05ab/ab_c2.err || exit 1
