#!/bin/bash
# PMC passes of the box engine (one solve each), each pass its own rocprofv3 run
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
lib=${1:-gamesmanmpi_amd/libgmsolve.so}
i=0
for pmc in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM SQ_BUSY_CYCLES" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  GM_LIB_PATH=$lib REPS=1 timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/pmc_box/p$i -o run -- python tools/box_check.py full > gpurun_out/pmc_box_p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  python tools/pmc_sum.py gpurun_out/pmc_box/p$i box_tier 41
done
