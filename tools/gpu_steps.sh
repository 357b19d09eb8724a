#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step
# that crashed, aborted or timed out (exit 124/134/137/139 or > 128).  Plain test
# failures (exit 1) do not stop later steps.
# usage: tools/gpu_steps.sh "<seconds>:<name>:<command>" ...
mkdir -p gpurun_out
for step in "$@"; do
  secs="${step%%:*}"; rest="${step#*:}"; name="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "=== stopping: $name ended with $rc"; exit $rc
  fi
done
