#!/bin/bash
# Round 5: the bench's two-solve IPC probe (ranks sharing one GPU): clean and forced failure;
# the bench GPU tests.
TAG=r05ab
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp PYTHONUNBUFFERED=1
steps=(
  "300:$TAG/pytest_bench:python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_bench.py"
  "400:$TAG/rehearse4:python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 4 --steps 10 --warmup 3 --rehearse-one-gpu"
  "400:$TAG/rehearse2_forced:GM_BENCH_PROBE_FAIL=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29516 bench.py --gpus 2 --steps 5 --warmup 1 --rehearse-one-gpu"
)
tools/gpu_steps.sh "${steps[@]}"
