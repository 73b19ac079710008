# round-5 session script (scratch): brute-force occupancy variants
set -o pipefail
mkdir -p gpurun_out/r05t
for v in default abvar/lib_bstream.so abvar/lib_bs_w6.so abvar/lib_bs_w8.so abvar/lib_bt_w6.so; do
  if [ "$v" = default ]; then L=""; else L="RT_LIB=$v"; fi
  env $L timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05t/brute_$(basename $v .so).json 2> gpurun_out/r05t/brute_$(basename $v .so).err || exit 1
done
