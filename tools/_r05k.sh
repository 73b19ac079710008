# round-5 session script (scratch): brute-force wavefront variants
set -o pipefail
mkdir -p gpurun_out/r05k
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "brute" > gpurun_out/r05k/tests.log 2>&1 || exit 1
for v in default abvar/lib_brh16.so abvar/lib_brg8.so abvar/lib_br2.so abvar/lib_brt1k.so; do
  if [ "$v" = default ]; then L=""; else L="RT_LIB=$v"; fi
  env $L timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05k/brute_$(basename $v .so).json 2> gpurun_out/r05k/brute_$(basename $v .so).err || exit 1
done
