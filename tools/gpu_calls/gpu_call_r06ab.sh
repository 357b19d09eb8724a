#!/bin/bash
# Round 6: the two-process rehearsal with the side configs over the sparse IPC transport, run on
# its own with every rank's Python stacks dumped every 60 s (GM_BENCH_STACKS) and a ticker, to
# see where the time goes (the bench test of r06aa went silent for 3 minutes).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06ab
( for i in $(seq 1 40); do sleep 20; echo "tick $i" >> gpurun_out/r06ab/ticks.txt; done ) &
T=$!
GM_BENCH_STACKS=60 timeout -k 10 420 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 2 --rehearse-one-gpu > gpurun_out/r06ab/rehearse2.log 2>&1
echo "rc=$?"
kill $T
tail -c 6000 gpurun_out/r06ab/rehearse2.log
