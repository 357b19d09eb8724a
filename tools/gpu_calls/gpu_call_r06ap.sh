#!/bin/bash
# Round 6: the bench as the driver runs it at N = 4 (torch.distributed.run, one process per rank),
# rehearsed with the four ranks sharing this one GPU: the box engine's halos and the side
# configs' exchanges over the IPC transports.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06ap
( for i in $(seq 1 60); do sleep 20; echo "tick $i" >> gpurun_out/r06ap/ticks.txt; done ) &
T=$!
steps=(
  "600:r06ap/rehearse4:python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 4 --steps 5 --warmup 2 --rehearse-one-gpu"
)
tools/gpu_steps.sh "${steps[@]}"
rc=$?
kill $T
exit $rc
