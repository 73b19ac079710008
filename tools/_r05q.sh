# round-5 session script (scratch): streamed brute-force sweep variant
set -o pipefail
mkdir -p gpurun_out/r05q
RT_LIB=abvar/lib_bstream.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "brute" > gpurun_out/r05q/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05q/brute_default.json 2> gpurun_out/r05q/brute_default.err || exit 1
RT_LIB=abvar/lib_bstream.so timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05q/brute_stream.json 2> gpurun_out/r05q/brute_stream.err || exit 1
