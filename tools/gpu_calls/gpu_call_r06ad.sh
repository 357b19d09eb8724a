#!/bin/bash
# Round 6: the two-process rehearsal traced (GM_TRACE=1): where the side configs' Toot 6x4 solves
# over the sparse IPC transport spend their time inside bench.py (r06ab: > 240 s; r06ac: the same
# solve outside bench.py takes 0.21 s).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06ad
GM_TRACE=1 GM_BENCH_STACKS=60 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 2 --warmup 1 --rehearse-one-gpu > gpurun_out/r06ad/rehearse2.log 2>&1
echo "rc=$?"
grep -n "sharded rank\|Timeout\|error" gpurun_out/r06ad/rehearse2.log | tail -60
