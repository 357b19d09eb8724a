#!/bin/bash
# Round 6: the drop-in launcher on the reference's unmodified 8x8 Othello plugin, endgame roots
# passed with --custom / --init_pos; wall time of the whole command (import, bind, solve, print).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06aq
out=gpurun_out/r06aq/launcher_othello8.txt
for e in 10 14 16; do
  echo "== endgame_$e" >> $out
  s=$(date +%s%N)
  timeout -k 10 240 python3 solver_launcher.py test_games/othello_bit_new.py --custom tools/othello8_roots.py \
      --init_pos endgame_$e >> $out 2>&1 || { echo "rc=$? at endgame_$e" >> $out; exit 1; }
  echo "wall $(( ($(date +%s%N) - s) / 1000000 )) ms" >> $out
done
GM_TRACE=0 timeout -k 10 240 python3 -c "
import time, importlib.util
from gamesmanmpi_amd import Solver
spec = importlib.util.spec_from_file_location('g', 'test_games/othello_bit_new.py'); g = importlib.util.module_from_spec(spec); spec.loader.exec_module(g)
spec = importlib.util.spec_from_file_location('r', 'tools/othello8_roots.py'); r = importlib.util.module_from_spec(spec); spec.loader.exec_module(r)
t0 = time.perf_counter(); s = Solver(g, root=r.endgame_16(), device=0); t1 = time.perf_counter()
n, rec = s.solve(); t2 = time.perf_counter()
print('endgame_16 in process: bind %.2f s, solve %.3f s, %d positions, root record %#x' % (t1 - t0, t2 - t1, n, rec))
" >> $out 2>&1
