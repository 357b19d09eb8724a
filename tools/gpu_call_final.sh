#!/bin/bash
# End-of-round check on one GPU: the GPU parity suite, smoke(), the bench line, and
# the bench's sharded path with 8 loopback ranks.
tools/gpu_steps.sh \
 "900:pytest_gpu:python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread" \
 "200:smoke:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "300:bench:python bench.py" \
 "300:bench_v8:python bench.py --virtual-ranks 8 --no-cpu-baseline --no-toot"
