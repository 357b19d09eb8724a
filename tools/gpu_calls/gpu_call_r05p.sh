#!/bin/bash
# Round 5 profile round: the default bench line, its kernel trace and PMC passes, and the
# multi-process bench rehearsed on one GPU (IPC transport, direct halo stores).
TAG=r05p
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
steps=(
  "400:$TAG/bench:python3 bench.py"
  "300:$TAG/prof_kt:rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-toot"
  "120:$TAG/prof_fetch:timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-toot"
  "120:$TAG/prof_write:timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-toot"
  "400:$TAG/rehearse2:python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 3 --rehearse-one-gpu"
  "400:$TAG/rehearse4:python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 4 --steps 10 --warmup 3 --rehearse-one-gpu"
)
tools/gpu_steps.sh "${steps[@]}"
