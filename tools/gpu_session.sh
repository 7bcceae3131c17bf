#!/bin/bash
# Run a sequence of GPU steps on the gpurun box; each step has its own time limit.
# A step that faults / aborts / times out (exit >= 124 or signal) ends the session;
# ordinary test failures (exit 1) do not.
# usage: tools/gpu_session.sh "<name>:<timeout_s>:<command>" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; tmo="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${tmo}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "=== stopping: step $name ended with rc=$rc"; exit $rc
  fi
done
