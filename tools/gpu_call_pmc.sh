# PMC evidence: LDS bank conflicts of the dense kernel, traffic / atomics / L2 of the sparse kernels
O=gpurun_out
B="python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --no-toot"
T="python3 tools/solve_timed.py toot 6 4 1"
tools/gpu_steps.sh \
  "120:pmc_lds:timeout -s KILL 100 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $O/pmc_lds -o run -- $B" \
  "120:pmc_t_fetch:timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_t_fetch -o run -- $T" \
  "120:pmc_t_write:timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_t_write -o run -- $T" \
  "120:pmc_t_atomic:timeout -s KILL 100 rocprofv3 --pmc TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum --output-format csv -d $O/pmc_t_atomic -o run -- $T" \
  "120:pmc_t_l2:timeout -s KILL 100 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_t_l2 -o run -- $T"
