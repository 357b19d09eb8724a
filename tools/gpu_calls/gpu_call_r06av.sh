#!/bin/bash
# Round 6: where the first 16-empty Othello 8x8 solve of a process spends its time (the scale
# tool's first solve took 3.7-3.8 s against 0.35 s repeated, r06au; the launcher's 0.36 s, r06aq).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06av
O=gpurun_out/r06av
for i in 1 2; do
  s=$(date +%s%N)
  GM_TRACE=1 timeout -k 10 120 python3 solver_launcher.py test_games/othello_bit_new.py --custom tools/othello8_roots.py \
      --init_pos endgame_16 > $O/launcher_$i.txt 2>&1 || exit 1
  echo "wall $(( ($(date +%s%N) - s) / 1000000 )) ms" >> $O/launcher_$i.txt
done
for i in 1 2; do
  GM_TRACE=1 timeout -k 10 120 python3 tools/othello8_scale.py 16 --repeats 2 > $O/scale_$i.txt 2>&1 || exit 1
done
