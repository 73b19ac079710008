# round-5 session script (scratch): node pairs in the global-memory walk
set -o pipefail
mkdir -p gpurun_out/r05r
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "heightfield or c5 or quantized or pruning or grazing or walk or certif or leaf or triangle_accel or device_scene" > gpurun_out/r05r/tests.log 2>&1 || exit 1
timeout -k 10 400 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_nopairs.so abvar/lib_pairs_u3.so --config c5_heightfield --rounds 4 --frames 40 --frame-batch 20 > gpurun_out/r05r/ab_c5.json 2> gpurun_out/r05r/ab_c5.err || exit 1
