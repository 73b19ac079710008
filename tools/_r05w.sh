# round-5 session script (scratch): C5 knobs at the final build
set -o pipefail
mkdir -p gpurun_out/r05w
timeout -k 10 500 python3 tools/ab_env.py "RT_LEAF_BATCH=4" "RT_LEAF_BATCH=3" "RT_LEAF_BATCH=5" "RT_TRAV_THRESHOLD=48" "RT_TRAV_THRESHOLD=60" "RT_DRAIN_THRESHOLD=24" --config c5_heightfield --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05w/ab_knobs.jsonl 2> gpurun_out/r05w/ab_knobs.err || exit 1
timeout -k 10 400 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_u4.so abvar/lib_u6.so --config c5_heightfield --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/r05w/ab_unroll.json 2> gpurun_out/r05w/ab_unroll.err || exit 1
