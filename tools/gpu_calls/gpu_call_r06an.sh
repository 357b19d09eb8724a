#!/bin/bash
# Round 6: the rehearsal with its side configs over the windowed sparse IPC transport: the bench
# tests, then the rehearsal's line.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06an
( for i in $(seq 1 60); do sleep 20; echo "tick $i" >> gpurun_out/r06an/ticks.txt; done ) &
T=$!
steps=(
  "900:r06an/bench_tests:python3 -u -m pytest -v --timeout 400 --timeout-method thread tests/test_gpu_bench.py"
  "500:r06an/rehearse2:python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 2 --rehearse-one-gpu"
)
tools/gpu_steps.sh "${steps[@]}"
rc=$?
kill $T
exit $rc
