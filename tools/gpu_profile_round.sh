#!/bin/bash
# One GPU call: parity tests, the bench line, and the rocprofv3 evidence for it
# (kernel trace + stats, then one --pmc pass per counter), plus a kernel trace of
# the Toot-and-Otto 6x4 solve.  Each GPU step has its own time limit; the script
# stops at the first crash / abort / timeout (tools/gpu_steps.sh).
# usage: tools/gpu_profile_round.sh TAG
TAG=${1:-r01}
R=$(pwd)
O=$R/gpurun_out
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "900:pytest_gpu:python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
  "300:bench:python bench.py" \
  "300:prof_kt:rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-toot" \
  "120:prof_fetch:timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-toot" \
  "120:prof_write:timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-toot" \
  "300:prof_toot:rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_toot -o run -- python3 tools/solve_timed.py toot 6 4 3"
