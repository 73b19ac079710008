#!/bin/bash
# Session 5: image-payload gather -- targeted GPU tests, then the 2/8-rank gloo rehearsal with the gather verify.
set -e -o pipefail
OUT=gpurun_out/r02_s5a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "pack_unpack_gather or rccl or unpack_all_ranks" > $OUT/tests.log 2>&1
for n in 2 8; do
  RT_BENCH_ONE_DEVICE=1 RT_DIST_BACKEND=gloo RT_BENCH_VERIFY_GATHER=1 timeout -k 10 300 \
    python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 2 > $OUT/multi_$n.json 2> $OUT/multi_$n.err
done
echo done
