#!/bin/bash
# Round 6: the same allocation exported and imported again and again between two processes
# (tools/ipc_big_probe.hip with repeats), as a rank's cached send buffer is in every solve.
export TMPDIR=/tmp
mkdir -p gpurun_out/r06ag
for b in 100000000 2600000000; do
  d=$(mktemp -d)
  timeout -k 5 100 ./tools/ipc_big_probe_bin 0 $b $d 24 > gpurun_out/r06ag/exp_$b.txt 2>&1 &
  E=$!
  timeout -k 5 100 ./tools/ipc_big_probe_bin 1 $b $d 24 > gpurun_out/r06ag/imp_$b.txt 2>&1
  ri=$?
  wait $E; re=$?
  echo "$b: importer rc=$ri exporter rc=$re"; tail -3 gpurun_out/r06ag/imp_$b.txt; grep -c "open" gpurun_out/r06ag/imp_$b.txt
  if [ $ri -ge 124 ] || [ $re -ge 124 ]; then echo "stopping"; break; fi
done
