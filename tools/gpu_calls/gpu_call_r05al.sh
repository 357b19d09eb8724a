#!/bin/bash
# Round 5: IPC hand-offs folded into the tier launches (GM_BOX_HANDOFF=1): the IPC tests and the
# one-GPU rehearsal with it, and the emulated model (virtual ranks, GM_BOX_SIGNAL_KERNELS=1).
TAG=r05al
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp PYTHONUNBUFFERED=1
steps=(
  "600:$TAG/pytest_ipc_handoff:GM_BOX_HANDOFF=1 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multiproc.py -k ipc"
  "300:$TAG/pytest_split_handoff:GM_BOX_HANDOFF=1 GM_BOX_SIGNAL_KERNELS=1 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_sharded.py -k box_split_2_32"
  "300:$TAG/split_time_handoff:GM_BOX_HANDOFF=1 GM_BOX_SIGNAL_KERNELS=1 python3 -X faulthandler -u tools/box_split_time.py --ranks 2 4 8 --reps 3 --batch 1"
  "300:$TAG/split_time_sigk:GM_BOX_SIGNAL_KERNELS=1 python3 -X faulthandler -u tools/box_split_time.py --ranks 2 4 8 --reps 3 --batch 1"
  "400:$TAG/rehearse4_handoff:GM_BOX_HANDOFF=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 4 --steps 10 --warmup 3 --rehearse-one-gpu"
)
tools/gpu_steps.sh "${steps[@]}"
