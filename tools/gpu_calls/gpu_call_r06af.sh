#!/bin/bash
# Round 6: HIP IPC mappings of one large allocation between two processes on one GPU
# (tools/ipc_big_probe.hip): 1.5 / 2.1 / 2.2 / 2.6 / 4.5 GB.
export TMPDIR=/tmp
mkdir -p gpurun_out/r06af
for b in 1500000000 2100000000 2200000000 2600000000 4500000000; do
  d=$(mktemp -d)
  timeout -k 5 70 ./tools/ipc_big_probe_bin 0 $b $d > gpurun_out/r06af/exp_$b.txt 2>&1 &
  E=$!
  timeout -k 5 70 ./tools/ipc_big_probe_bin 1 $b $d > gpurun_out/r06af/imp_$b.txt 2>&1
  ri=$?
  wait $E; re=$?
  echo "$b: importer rc=$ri exporter rc=$re"; cat gpurun_out/r06af/imp_$b.txt gpurun_out/r06af/exp_$b.txt
  if [ $ri -ge 124 ] || [ $re -ge 124 ]; then echo "stopping"; break; fi
done
