#!/bin/bash
# Round 5: bench.py's multi-process path rehearsed on one GPU (IPC transport, gloo collectives).
set -o pipefail
mkdir -p gpurun_out/r05l
for n in 2 4; do
    timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
        --master-port $((29500 + n)) bench.py --gpus $n --steps 10 --warmup 3 --rehearse-one-gpu \
        > gpurun_out/r05l/bench_rehearse$n.log 2>&1 || exit 1
done
