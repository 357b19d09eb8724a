#!/bin/bash
# box dataflow default for sharded solves: tests, per-rank times, bench rehearsal
mkdir -p gpurun_out/r04n
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py -m gpu -x -v --timeout 240 --timeout-method thread -k "box" > gpurun_out/r04n/pytest_box.log 2>&1 || exit 1
timeout -k 10 180 python tools/box_shard_time.py --ranks 1 2 4 8 --reps 10 > gpurun_out/r04n/shard_time.log 2>&1 || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --rehearse-one-gpu > gpurun_out/r04n/bench_rehearse2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --virtual-ranks 8 --steps 10 --warmup 3 --no-toot --no-cpu-baseline > gpurun_out/r04n/bench_v8.log 2>&1
