#!/bin/bash
# Round 6: the two-process rehearsal now runs the side configs too (hash-sharded over the sparse
# IPC transport, the ranks sharing one GPU): the bench tests, then the rehearsal's line.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06aa
steps=(
  "900:r06aa/bench_tests:python3 -u -m pytest -v --timeout 400 --timeout-method thread tests/test_gpu_bench.py"
  "500:r06aa/rehearse2:python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 2 --rehearse-one-gpu"
)
tools/gpu_steps.sh "${steps[@]}"
