#!/bin/bash
# Round 5: direct halo writes (loopback and IPC): box tests, IPC processes, smoke, split timing.
set -o pipefail
mkdir -p gpurun_out/r05m
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_sharded.py -k "box" \
    > gpurun_out/r05m/pytest_box.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multiproc.py -k "ipc" \
    > gpurun_out/r05m/pytest_ipc.txt 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05m/smoke.txt 2>&1 || exit 1
for b in 1 2; do
    timeout -k 10 400 python -X faulthandler -u tools/box_split_time.py --ranks 2 4 8 --reps 3 --batch $b \
        --dump gpurun_out/r05m >> gpurun_out/r05m/split_time.txt 2>&1 || exit 1
done
