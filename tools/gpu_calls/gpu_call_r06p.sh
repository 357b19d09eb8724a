#!/bin/bash
# Round 6: Othello 8x8 (15- and 16-empty roots) counters per kernel, for its random-access roofline:
# a kernel trace of 3 solves, then one-solve PMC passes (FETCH_SIZE, WRITE_SIZE, the TCC request
# and hit counters, SQ instruction counts), each pass in a run of its own.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
E=${E:-15}
O=$(pwd)/gpurun_out/r06p$E
mkdir -p $O
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU"
T1="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
P="python3 tools/othello8_scale.py $E --repeats"
steps=(
  "200:r06p$E/kt:rocprofv3 --kernel-trace --stats --output-format csv -d $O/o8_kt -o run -- $P 3"
  "150:r06p$E/fetch:timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/o8_fetch -o run -- $P 1"
  "150:r06p$E/write:timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/o8_write -o run -- $P 1"
  "150:r06p$E/tcc:timeout -s KILL 140 rocprofv3 --pmc $T1 --output-format csv -d $O/o8_tcc -o run -- $P 1"
  "150:r06p$E/sq:timeout -s KILL 140 rocprofv3 --pmc $S1 --output-format csv -d $O/o8_sq -o run -- $P 1"
)
tools/gpu_steps.sh "${steps[@]}"
