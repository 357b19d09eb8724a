#!/bin/bash
# sharded box engine, 8 virtual ranks: kernel trace of the dataflow launches (one per rank
# and solve) and the HBM PMC passes of one solve, beside the event-timed per-rank numbers
mkdir -p gpurun_out/r04x
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04x/kt -o run -- python3 tools/box_shard_time.py --ranks 8 --reps 5 > gpurun_out/r04x/kt.log 2>&1 || exit 1
timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r04x/fetch -o run -- python3 tools/box_shard_time.py --ranks 8 --reps 1 > gpurun_out/r04x/fetch.log 2>&1 || exit 1
timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r04x/write -o run -- python3 tools/box_shard_time.py --ranks 8 --reps 1 > gpurun_out/r04x/write.log 2>&1 || exit 1
