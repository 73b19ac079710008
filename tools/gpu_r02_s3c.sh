#!/bin/bash
# Session 3: counter list + TA/TD busy on C5 and C2 (is the leaf step bound by the L1 address path?).
set -e -o pipefail
OUT=gpurun_out/r02_s3c
mkdir -p $OUT
export TMPDIR=/tmp
python3 -c "import __graft_entry__ as g; g.build()" > $OUT/build.log 2>&1
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
for cfg in c5_heightfield c3_chess c2_rtiow; do
  st=4; [ $cfg = c5_heightfield ] || st=16
  timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE --output-format csv -d $OUT/ta_$cfg -o run -- python3 bench.py --config $cfg --steps $st --warmup 2 --no-cpu-baseline > /dev/null 2> $OUT/ta_$cfg.err
  timeout -s KILL 120 rocprofv3 --pmc TD_BUSY_avr TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $OUT/td_$cfg -o run -- python3 bench.py --config $cfg --steps $st --warmup 2 --no-cpu-baseline > /dev/null 2> $OUT/td_$cfg.err
done
echo done
