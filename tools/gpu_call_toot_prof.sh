O=gpurun_out
T="python3 tools/solve_timed.py toot 6 4 1"
tools/gpu_steps.sh \
  "150:toot_trace:timeout -k 10 140 rocprofv3 --kernel-trace --stats --output-format csv -d $O/toot_trace -o run -- python3 tools/solve_timed.py toot 6 4 3" \
  "120:pmc_t_fetch:timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_t_fetch -o run -- $T" \
  "120:pmc_t_write:timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_t_write -o run -- $T" \
  "120:pmc_t_atomic:timeout -s KILL 100 rocprofv3 --pmc TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum --output-format csv -d $O/pmc_t_atomic -o run -- $T" \
  "120:pmc_t_l2:timeout -s KILL 100 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_t_l2 -o run -- $T"
