set -e -o pipefail
OUT=gpurun_out/r02_knobs2
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
A="--frames 32 --rounds 4 --frame-batch 8"
for c in c2_rtiow c3_chess c1_four_spheres; do
timeout -k 10 300 python3 tools/ab_bench.py $V/lib_cur.so $V/lib_cur.so:RT_BATCH_SCHEDULE=1 $V/lib_cur.so:RT_UNIT_TILE_MAJOR=1 --config $c $A > $OUT/$c.json 2>> $OUT/err.log
done
timeout -k 10 300 python3 tools/ab_bench.py $V/lib_cur.so $V/lib_cur.so:RT_BATCH_SCHEDULE=1 $V/lib_cur.so:RT_UNIT_TILE_MAJOR=1 --config c5_heightfield --frames 8 --rounds 2 --frame-batch 8 > $OUT/c5.json 2>> $OUT/err.log
timeout -k 10 300 python3 tools/ab_bench.py $V/lib_cur.so $V/lib_cur.so:RT_BATCH_SCHEDULE=1 $V/lib_cur.so:RT_UNIT_TILE_MAJOR=1 --config c4_mixed --width 3840 --height 2160 --frames 16 --rounds 3 --frame-batch 8 > $OUT/c4.json 2>> $OUT/err.log
echo done
