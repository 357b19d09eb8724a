#!/bin/bash
# Round 5 sparse profile: Toot 6x4 (config 3) with the current engine -- kernel trace of 3
# solves (1 synced + 2 replays) and one-solve PMC passes -- and the locality home
# (GM_SPARSE_HOME_W=20) beside it: kernel trace, L2 pass, probe lengths.
TAG=r05g
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"
T1="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
P="python3 tools/solve_timed.py toot 6 4"
steps=(
  "150:$TAG/sp_kt:rocprofv3 --kernel-trace --stats --output-format csv -d $O/sp_kt -o run -- $P 3"
  "150:$TAG/sp_fetch:timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/sp_fetch -o run -- $P 1"
  "150:$TAG/sp_write:timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/sp_write -o run -- $P 1"
  "150:$TAG/sp_tcc:timeout -s KILL 140 rocprofv3 --pmc $T1 --output-format csv -d $O/sp_tcc -o run -- $P 1"
  "150:$TAG/sp_sq:timeout -s KILL 140 rocprofv3 --pmc $S1 --output-format csv -d $O/sp_sq -o run -- $P 1"
  "150:$TAG/probe_w0:GM_SPARSE_PROBE_STATS=1 $P 1"
  "150:$TAG/probe_w20:GM_SPARSE_PROBE_STATS=1 GM_SPARSE_HOME_W=20 $P 1"
  "150:$TAG/loc_kt:GM_SPARSE_HOME_W=20 rocprofv3 --kernel-trace --stats --output-format csv -d $O/loc_kt -o run -- $P 3"
  "150:$TAG/loc_fetch:GM_SPARSE_HOME_W=20 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/loc_fetch -o run -- $P 1"
  "150:$TAG/loc_write:GM_SPARSE_HOME_W=20 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/loc_write -o run -- $P 1"
  "150:$TAG/loc_tcc:GM_SPARSE_HOME_W=20 timeout -s KILL 140 rocprofv3 --pmc $T1 --output-format csv -d $O/loc_tcc -o run -- $P 1"
  "150:$TAG/loc_sq:GM_SPARSE_HOME_W=20 timeout -s KILL 140 rocprofv3 --pmc $S1 --output-format csv -d $O/loc_sq -o run -- $P 1"
)
tools/gpu_steps.sh "${steps[@]}"
