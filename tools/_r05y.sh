# round-5 session script (scratch): sphere pair leaves (RT_SPHERE_PAIRS) -- parity and A/B
set -o pipefail
mkdir -p gpurun_out/r05y
RT_SPHERE_PAIRS=1 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -x -v --timeout 200 --timeout-method thread -m gpu -k "golden or full_frame or c2 or c1 or four_spheres or rtiow or sphere or brute or frame_batch" > gpurun_out/r05y/tests.log 2>&1 || exit 1
timeout -k 10 500 python3 tools/ab_env.py "RT_SPHERE_PAIRS=0" "RT_SPHERE_PAIRS=1" "RT_SPHERE_PAIRS=1 RT_SPHERE_LEAF=1" --config c2_rtiow --frame-batch 20 --frames 40 --rounds 5 > gpurun_out/r05y/ab_c2.jsonl 2> gpurun_out/r05y/ab_c2.err || exit 1
timeout -k 10 300 python3 tools/ab_env.py "RT_SPHERE_PAIRS=0" "RT_SPHERE_PAIRS=1" --config c1_four_spheres --frame-batch 20 --frames 40 --rounds 5 > gpurun_out/r05y/ab_c1.jsonl 2> gpurun_out/r05y/ab_c1.err || exit 1
