#!/bin/bash
# Round 5: the split box engine with the halo messages written by the tier kernel.
set -o pipefail
mkdir -p gpurun_out/r05d
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_sharded.py -k "box" \
    > gpurun_out/r05d/gpu_box_tests.txt 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05d/smoke.txt 2>&1 || exit 1
for b in 1 2 4; do
    timeout -k 10 400 python -X faulthandler -u tools/box_split_time.py --ranks 2 4 8 --reps 3 --batch $b \
        >> gpurun_out/r05d/split_time.txt 2>&1 || exit 1
done
