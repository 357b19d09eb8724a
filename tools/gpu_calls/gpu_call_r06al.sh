#!/bin/bash
# Round 6: a growing IPC-exported buffer as in a solve (tools/ipc_big_probe.hip roles 2/3): the sizes
# of the stalled solve's send buffers (r06ak), the importer keeping every mapping open.
export TMPDIR=/tmp
mkdir -p gpurun_out/r06al
S=100000000,300000000,600000000,1000000000,1559000000,1949000000,2605000000,3300000000
d=$(mktemp -d)
timeout -k 5 120 ./tools/ipc_big_probe_bin 2 0 $d 1 $S > gpurun_out/r06al/exp.txt 2>&1 &
E=$!
timeout -k 5 120 ./tools/ipc_big_probe_bin 3 0 $d 1 $S > gpurun_out/r06al/imp.txt 2>&1
ri=$?
wait $E; re=$?
echo "importer rc=$ri exporter rc=$re"; cat gpurun_out/r06al/imp.txt; tail -3 gpurun_out/r06al/exp.txt
