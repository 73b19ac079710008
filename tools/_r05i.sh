# round-5 session script (scratch): brute-force tests + bench, C5 layout A/B
set -o pipefail
mkdir -p gpurun_out/r05i
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "brute" > gpurun_out/r05i/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05i/brute_wf.json 2> gpurun_out/r05i/brute_wf.err || exit 1
timeout -k 10 400 python3 tools/ab_env.py "RT_TRI_OCTANTS=1" "RT_TRI_OCTANTS=0" "RT_TRI_OCTANTS=0 RT_TRI_QNODES=0" "RT_TRI_OCTANTS=1 RT_PRIMARY_PASS=0" "RT_TRI_OCTANTS=0 RT_PRIMARY_PASS=0" --config c5_heightfield --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05i/ab_oct.jsonl 2> gpurun_out/r05i/ab_oct.err
