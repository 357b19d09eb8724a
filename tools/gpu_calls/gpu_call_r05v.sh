#!/bin/bash
# Round 5: split solves of virtual ranks and of the IPC transport replayed as one captured graph
# (GM_OPT_GRAPH, default on): the split parity tests (virtual ranks, IPC processes), then
# solo spans G = 2 / 4 / 8 with the graph and without it (GM_OPT_GRAPH 0 via GM_SPLIT_NO_GRAPH).
set -o pipefail
mkdir -p gpurun_out/r05v
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_sharded.py -k "box" \
    > gpurun_out/r05v/pytest_box.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multiproc.py -k "ipc" \
    > gpurun_out/r05v/pytest_ipc.txt 2>&1 || exit 1
timeout -k 10 300 python -X faulthandler -u tools/box_split_time.py --ranks 2 4 8 --reps 3 --batch 1 \
    > gpurun_out/r05v/graph.txt 2>&1 || exit 1
timeout -k 10 300 python -X faulthandler -u tools/box_split_time.py --ranks 2 4 8 --reps 3 --batch 1 --no-graph \
    > gpurun_out/r05v/eager.txt 2>&1 || exit 1
