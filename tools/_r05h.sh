# round-5 session script (scratch): walk-variant and brute-force tests, q4 A/B, brute A/B
set -o pipefail
mkdir -p gpurun_out/r05h
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "global_walk_variants or lds_vertex or brute" > gpurun_out/r05h/tests.log 2>&1 || exit 1
RT_BRUTE_WF=1 timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05h/brute_wf.json 2> gpurun_out/r05h/brute_wf.err || exit 1
RT_BRUTE_WF=0 timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05h/brute_old.json 2> gpurun_out/r05h/brute_old.err || exit 1
timeout -k 10 400 python3 tools/ab_env.py "RT_TRI_Q4=1" "RT_TRI_Q4=0" "RT_TRI_Q4=1 RT_BLOCK_THREADS=512" "RT_TRI_Q4=1 RT_BLOCK_THREADS=256" --config c5_heightfield --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05h/ab_threads.jsonl 2> gpurun_out/r05h/ab_threads.err || exit 1
RT_LIB=abvar/lib_diag.so RT_TRI_Q4=1 timeout -k 10 200 python3 tools/diag_split.py --frame-batch 20 c5_heightfield > gpurun_out/r05h/diag_q4.json 2>&1 || exit 1
RT_LIB=abvar/lib_diag.so RT_TRI_Q4=0 timeout -k 10 200 python3 tools/diag_split.py --frame-batch 20 c5_heightfield > gpurun_out/r05h/diag_bin.json 2>&1
