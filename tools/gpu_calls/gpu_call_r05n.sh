#!/bin/bash
# Round 5: the split dataflow (virtual ranks, IPC processes) and the box tests.
set -o pipefail
mkdir -p gpurun_out/r05n
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_sharded.py -k "box" \
    > gpurun_out/r05n/pytest_box.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multiproc.py -k "ipc" \
    > gpurun_out/r05n/pytest_ipc.txt 2>&1 || exit 1
timeout -k 10 400 python -X faulthandler -u tools/box_split_time.py --ranks 2 4 8 --reps 3 --flow >> gpurun_out/r05n/flow_time.txt 2>&1 || exit 1
