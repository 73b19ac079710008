# round-5 session script (scratch): refill prologue tests + A/B
set -o pipefail
mkdir -p gpurun_out/r05m
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -x -v --timeout 120 --timeout-method thread -m gpu -k "golden or frame_batch or group or full_frame or sphere or determinism or camera or device" > gpurun_out/r05m/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_noprep.so --config c2_rtiow --rounds 5 --frames 40 --frame-batch 20 > gpurun_out/r05m/ab_c2.json 2> gpurun_out/r05m/ab_c2.err || exit 1
timeout -k 10 300 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_noprep.so --config c1_four_spheres --width 800 --height 600 --rounds 5 --frames 40 --frame-batch 20 > gpurun_out/r05m/ab_c1.json 2> gpurun_out/r05m/ab_c1.err || exit 1
