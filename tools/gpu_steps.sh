#!/bin/bash
# Run GPU steps in order, each under its own time limit; a step that FAILS
# (rc 1: a test failure) does not stop the chain, anything else (a fault,
# abort, segfault, time limit) ends the call there.
#   bash tools/gpu_steps.sh "<seconds> <command>" ["<seconds> <command>" ...]
mkdir -p gpurun_out
export TMPDIR=/tmp
for step in "$@"; do
  secs=${step%% *}
  cmd=${step#* }
  echo "== [$secs s] $cmd" >> gpurun_out/steps.log
  timeout -k 10 "$secs" bash -c "$cmd"
  rc=$?
  echo "== rc=$rc" >> gpurun_out/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: rc=$rc in: $cmd"; exit $rc; fi
done
