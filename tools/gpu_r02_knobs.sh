set -e -o pipefail
OUT=gpurun_out/r02_knobs
mkdir -p $OUT
export TMPDIR=/tmp
V=build/variants
A="--frames 32 --rounds 4 --frame-batch 8"
timeout -k 10 300 python3 tools/ab_bench.py $V/lib_cur.so $V/lib_unroll2.so $V/lib_unroll4.so $A > $OUT/unroll_c2.json 2>> $OUT/err.log
timeout -k 10 300 python3 tools/ab_bench.py $V/lib_cur.so $V/lib_cur.so:RT_TRAV_THRESHOLD=4 $V/lib_cur.so:RT_TRAV_THRESHOLD=12 $V/lib_cur.so:RT_TRAV_THRESHOLD=16 $A > $OUT/thresh_c2.json 2>> $OUT/err.log
timeout -k 10 300 python3 tools/ab_bench.py $V/lib_cur.so $V/lib_cur.so:RT_TILE_SCHEDULE=0 $V/lib_cur.so:RT_QUEUE_STRIPES=8 $V/lib_cur.so:RT_QUEUE_STRIPES=64 $A > $OUT/sched_c2.json 2>> $OUT/err.log
timeout -k 10 300 python3 tools/ab_bench.py $V/lib_cur.so $V/lib_cur.so:RT_WAVES_PER_CU=12 $V/lib_cur.so:RT_WAVES_PER_CU=20 $A > $OUT/waves_c2.json 2>> $OUT/err.log
timeout -k 10 300 python3 tools/ab_bench.py $V/lib_cur.so --frames 64 --rounds 4 --frame-batch 16 > $OUT/fb16_c2.json 2>> $OUT/err.log
timeout -k 10 300 python3 tools/ab_bench.py $V/lib_cur.so $V/lib_unroll2.so $V/lib_unroll4.so $V/lib_cur.so:RT_TRAV_THRESHOLD=16 $V/lib_cur.so:RT_TILE_SCHEDULE=0 --config c3_chess $A > $OUT/c3.json 2>> $OUT/err.log
echo done
