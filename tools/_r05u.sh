# round-5 session script (scratch): brute-force modes (tiled / scalar-streamed)
set -o pipefail
mkdir -p gpurun_out/r05u
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "brute" > gpurun_out/r05u/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05u/brute_tiled.json 2> gpurun_out/r05u/brute_tiled.err || exit 1
timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force stream --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05u/brute_stream.json 2> gpurun_out/r05u/brute_stream.err || exit 1
