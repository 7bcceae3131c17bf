#!/bin/bash
# Headline bench (graph replay ms/step) for each libcfdj variant, alternating, $ROUNDS rounds.
# usage: tools/bench_ab.sh build/a/libcfdj.so build/b/libcfdj.so ...
for r in $(seq ${ROUNDS:-2}); do
  for lib in "$@"; do
    out=$(CFDJ_LIB=$lib timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-timing $BENCH_ARGS) || exit $?
    echo "$lib $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])')"
  done
done
