#!/bin/bash
# round 3, box engine default: GPU suite, bench, kernel trace + FETCH/WRITE passes of the bench
R=$(pwd); O=$R/gpurun_out; export TMPDIR=/tmp
tools/gpu_steps.sh \
  "900:pytest_gpu:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "300:bench:python bench.py" \
  "300:prof_kt:rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-toot" \
  "120:prof_fetch:timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-toot" \
  "120:prof_write:timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-toot"
