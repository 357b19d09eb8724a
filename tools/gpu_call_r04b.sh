#!/bin/bash
# round 4: full GPU suite, sharded bench paths (virtual ranks; 2-process rehearsal on one GPU), graph walk
set -o pipefail
mkdir -p gpurun_out/r04b
export PYTHONUNBUFFERED=1
GM_GRAPH_TRACE=1 timeout -k 10 300 python tools/graph_enum_time.py 16 16 > gpurun_out/r04b/graph_enum.log 2>&1
# sparse engine: batch kernels (default) against the round-3 kernels, Toot 6x4
timeout -k 10 300 python tools/solve_timed.py toot 6 4 5 > gpurun_out/r04b/toot_batch.log 2>&1 &&
GM_SPARSE_BATCH=0 timeout -k 10 300 python tools/solve_timed.py toot 6 4 5 > gpurun_out/r04b/toot_nobatch.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "batch or toot" -x -v --timeout 280 --timeout-method thread > gpurun_out/r04b/pytest_batch.log 2>&1
timeout -k 10 300 python bench.py --virtual-ranks 8 --no-toot --no-cpu-baseline --steps 10 > gpurun_out/r04b/bench_v8.log 2>&1 &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --rehearse-one-gpu --steps 10 > gpurun_out/r04b/bench_rehearse2.log 2>&1 &&
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04b/pytest_gpu.log 2>&1
# LDS image layout A/B: round 3's pitch 68 / a0 stride 16, pitch 72, and the new 76 / 20 (default)
timeout -k 10 400 python tools/box_variants.py _exp/libgm_p68.so _exp/libgm_p76s20.so _exp/libgm_p72.so _exp/libgm_p68.so _exp/libgm_p76s20.so > gpurun_out/r04b/layout_ab.log 2>&1 &&
bash tools/gpu_pmc_box.sh _exp/libgm_p68.so > gpurun_out/r04b/pmc_p68.txt 2>&1 &&
bash tools/gpu_pmc_box.sh _exp/libgm_p76s20.so > gpurun_out/r04b/pmc_p76s20.txt 2>&1
