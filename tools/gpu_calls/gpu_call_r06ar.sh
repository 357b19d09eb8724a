#!/bin/bash
# Round 6: the launcher on the reference's 8x8 Othello plugin from its START position (no
# custom root): the reachable set is beyond one GPU's 288 GB, so the solve must end with a
# clean out-of-memory error, not a hang or a fault.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06ar
out=gpurun_out/r06ar/launcher_othello8_start.txt
s=$(date +%s%N)
GM_TRACE=1 timeout -k 10 240 python3 solver_launcher.py test_games/othello_bit_new.py --stats > $out 2>&1
rc=$?
echo "rc=$rc wall $(( ($(date +%s%N) - s) / 1000000 )) ms" >> $out
exit 0
