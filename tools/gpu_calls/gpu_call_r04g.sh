#!/bin/bash
# round 4 profile round: the headline (bench line, plain kernel trace of the same
# command, FETCH/WRITE PMC passes, box counter passes) and the sparse engine's Toot 6x4
# counters with the sorted lists + plain kernels (GM_SPARSE_BATCH 1) and the LDS batch
# kernels (2), one solve per pass
TAG=r04g
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"
T1="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
steps=(
  "300:$TAG/bench:python bench.py --no-toot"
  "300:$TAG/prof_kt:rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python3 bench.py --no-cpu-baseline --no-toot"
  "120:$TAG/prof_fetch:timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-toot"
  "120:$TAG/prof_write:timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-toot"
)
for m in 1 2; do
  steps+=("150:$TAG/sp${m}_kt:GM_SPARSE_BATCH=$m rocprofv3 --kernel-trace --stats --output-format csv -d $O/sp${m}_kt -o run -- python3 tools/solve_timed.py toot 6 4 3")
  steps+=("150:$TAG/sp${m}_fetch:GM_SPARSE_BATCH=$m timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/sp${m}_fetch -o run -- python3 tools/solve_timed.py toot 6 4 1")
  steps+=("150:$TAG/sp${m}_write:GM_SPARSE_BATCH=$m timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/sp${m}_write -o run -- python3 tools/solve_timed.py toot 6 4 1")
  steps+=("150:$TAG/sp${m}_tcc:GM_SPARSE_BATCH=$m timeout -s KILL 140 rocprofv3 --pmc $T1 --output-format csv -d $O/sp${m}_tcc -o run -- python3 tools/solve_timed.py toot 6 4 1")
  steps+=("150:$TAG/sp${m}_sq:GM_SPARSE_BATCH=$m timeout -s KILL 140 rocprofv3 --pmc $S1 --output-format csv -d $O/sp${m}_sq -o run -- python3 tools/solve_timed.py toot 6 4 1")
done
steps+=("300:$TAG/pmc_box:bash tools/gpu_pmc_box.sh")
tools/gpu_steps.sh "${steps[@]}"
