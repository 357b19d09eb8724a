#!/bin/bash
# Round 5: the bench's IPC probe (ranks sharing one GPU): a clean probe, and a forced failure
# reported in the line (no RCCL to fall back to on one GPU); the IPC tests after the wait change.
TAG=r05y
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp PYTHONUNBUFFERED=1
steps=(
  "600:$TAG/pytest_ipc:python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multiproc.py -k ipc"
  "400:$TAG/rehearse2:python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 3 --rehearse-one-gpu"
  "400:$TAG/rehearse2_forced:GM_BENCH_PROBE_FAIL=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29516 bench.py --gpus 2 --steps 5 --warmup 1 --rehearse-one-gpu"
)
tools/gpu_steps.sh "${steps[@]}"
