#!/bin/bash
# bench.py at N=2 on a one-GPU box: two ranks share the GPU over gloo (PJ_BENCH_BACKEND),
# exercising the N>1 bookkeeping (root sharding, max/sum reductions, partitioned k28 over 2
# ranks, ms1024 sharding) that the driver's RCCL runs use.
set -o pipefail
OUT=gpurun_out/n2; mkdir -p $OUT
PJ_BENCH_BACKEND=gloo timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 8 --warmup 1 "$@" \
  > $OUT/bench.json 2> $OUT/bench.err || { echo bench n2 failed; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
