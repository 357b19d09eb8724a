#!/bin/bash
# round 4: full GPU suite, sharded bench paths (virtual ranks; 2-process rehearsal on one GPU), graph walk
set -o pipefail
mkdir -p gpurun_out/r04b
export PYTHONUNBUFFERED=1
GM_GRAPH_TRACE=1 timeout -k 10 300 python tools/graph_enum_time.py 16 16 > gpurun_out/r04b/graph_enum.log 2>&1
timeout -k 10 300 python bench.py --virtual-ranks 8 --no-toot --no-cpu-baseline --steps 10 > gpurun_out/r04b/bench_v8.log 2>&1 &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --rehearse-one-gpu --steps 10 > gpurun_out/r04b/bench_rehearse2.log 2>&1 &&
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04b/pytest_gpu.log 2>&1
