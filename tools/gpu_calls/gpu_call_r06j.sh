#!/bin/bash
# Round 6: the CSR retro (GM_SPARSE_CSR=1): parity of every sparse test with
# it on, then Toot 6x4 solve times and a kernel trace against the default in the same run.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=$(pwd)/gpurun_out/r06j
mkdir -p $O
P="python3 -u -m pytest -v --timeout 300 --timeout-method thread"
steps=(
  "400:r06j/csr_everywhere:$P tests/test_gpu_parity.py -k csr_retro"
  "500:r06j/parity_csr:GM_SPARSE_CSR=1 $P tests/test_gpu_parity.py -k 'toot or othello or sparse or f2o or four'"
  "300:r06j/time_default:python3 -u tools/solve_timed.py toot 6 4 8"
  "300:r06j/time_csr:GM_SPARSE_CSR=1 python3 -u tools/solve_timed.py toot 6 4 8"
  "300:r06j/time_default2:python3 -u tools/solve_timed.py toot 6 4 8"
  "300:r06j/kt_csr:GM_SPARSE_CSR=1 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_csr -o run -- python3 tools/solve_timed.py toot 6 4 4"
  "300:r06j/kt_default:rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_default -o run -- python3 tools/solve_timed.py toot 6 4 4"
)
tools/gpu_steps.sh "${steps[@]}"
