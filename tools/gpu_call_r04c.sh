#!/bin/bash
# round 4 profile round of the headline: bench line, plain kernel trace of the same
# command, HBM PMC passes (separate runs), LDS/VALU counter passes
TAG=${1:-r04c}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "300:$TAG/bench:python bench.py --no-toot" \
  "300:$TAG/prof_kt:rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python3 bench.py --no-cpu-baseline --no-toot" \
  "120:$TAG/prof_fetch:timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-toot" \
  "120:$TAG/prof_write:timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-toot" \
  "300:$TAG/pmc_box:bash tools/gpu_pmc_box.sh"
