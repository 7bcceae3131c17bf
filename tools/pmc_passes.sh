#!/bin/bash
# Hardware-counter passes over the step's kernels (tools/kb_once.py launches each a few
# times): one rocprofv3 --pmc run per counter group (block limits: 8 SQ, 4 TCC, 4 TCP,
# 2 TA, 2 TD per run), each under its own time limit; stops at the first failure.
# usage: tools/pmc_passes.sh OUTDIR "name:COUNTER COUNTER ..." ...
out="$1"; shift
mkdir -p "$out"
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%:*}"; ctrs="${spec#*:}"
  echo "=== pmc pass $name: $ctrs"
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "$out/$name" -o "$name" -- python3 tools/kb_once.py > "$out/$name.log" 2>&1
  rc=$?
  echo "=== pass $name rc=$rc"; tail -n 3 "$out/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
