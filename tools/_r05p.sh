# round-5 session script (scratch): lazy triangle pieces on C5, three builds in one process
set -o pipefail
mkdir -p gpurun_out/r05p
timeout -k 10 400 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_nolazy.so abvar/lib_head.so --config c5_heightfield --rounds 4 --frames 40 --frame-batch 20 > gpurun_out/r05p/ab_c5.json 2> gpurun_out/r05p/ab_c5.err || exit 1
