# round-5 session script (scratch): scalar loads in the primary pre-pass -- tests, bench A/B
set -o pipefail
mkdir -p gpurun_out/r05x
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "primary or heightfield or c5 or pruning or grazing or quantized or walk or full_size" > gpurun_out/r05x/tests.log 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 200 python3 bench.py --config c5_heightfield --no-cpu-baseline --no-cadences > gpurun_out/r05x/c5_new_$i.json 2> gpurun_out/r05x/c5_new_$i.err || exit 1
RT_LIB=abvar/lib_head.so timeout -k 10 200 python3 bench.py --config c5_heightfield --no-cpu-baseline --no-cadences > gpurun_out/r05x/c5_head_$i.json 2> gpurun_out/r05x/c5_head_$i.err || exit 1
done
