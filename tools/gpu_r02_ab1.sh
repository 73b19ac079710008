set -e -o pipefail
OUT=gpurun_out/r02_ab1
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
timeout -k 10 400 python3 tools/ab_bench.py $V/lib_base.so $V/lib_defer.so:RT_LEAF_BATCH=2 $V/lib_defer.so:RT_LEAF_BATCH=4 $V/lib_defer.so:RT_LEAF_BATCH=6 --frames 32 --rounds 5 > $OUT/defer_c2.json 2> $OUT/err.log
timeout -k 10 400 python3 tools/ab_bench.py $V/lib_base.so $V/lib_defer.so:RT_LEAF_BATCH=2 $V/lib_defer.so:RT_LEAF_BATCH=4 --config c1_four_spheres --width 800 --height 600 --frames 32 --rounds 5 > $OUT/defer_c1.json 2>> $OUT/err.log
echo done
