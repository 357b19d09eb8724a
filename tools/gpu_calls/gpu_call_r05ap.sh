#!/bin/bash
# Round 5 rehearsal after the split graph replay: the whole GPU suite, smoke(), the default bench line and the
# multi-process bench rehearsed on one GPU (IPC transport).
TAG=r05ap
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
steps=(
  "900:$TAG/pytest_gpu:python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread"
  "200:$TAG/smoke:python3 -u -c \"import __graft_entry__ as g; g.smoke(); print('smoke ok')\""
  "400:$TAG/bench:python3 bench.py"
  "400:$TAG/rehearse2:python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 3 --rehearse-one-gpu"
  "400:$TAG/rehearse4:python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 4 --steps 10 --warmup 3 --rehearse-one-gpu"
)
tools/gpu_steps.sh "${steps[@]}"
