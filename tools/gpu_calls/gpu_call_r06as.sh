#!/bin/bash
# Round 6: the whole GPU suite as the driver runs it, smoke, the default bench line (with the
# Othello 8x8 endgame side config) and the two-process rehearsal.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06as
steps=(
  "900:r06as/pytest_gpu:python3 -u -m pytest tests/ -x -v --timeout 300 --timeout-method thread -m gpu"
  "120:r06as/smoke:python3 -c 'import __graft_entry__ as g; g.smoke()'"
  "600:r06as/bench:python3 bench.py"
  "400:r06as/rehearse2:python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29545 bench.py --gpus 2 --steps 5 --warmup 2 --rehearse-one-gpu"
)
tools/gpu_steps.sh "${steps[@]}"
