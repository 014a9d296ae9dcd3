#!/bin/bash
# Run GPU steps in order; each under its own time limit.  A step that ends in
# a fault/abort/segfault/timeout (exit >= 2, pytest's "tests failed" = 1 is
# allowed) stops the script: nothing more touches the GPU in this call.
# usage: tools/gpu_steps.sh "<name>:<seconds>:<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name exit $rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 2 ]; then echo "stopping after $name (exit $rc)"; exit $rc; fi
done
exit 0
