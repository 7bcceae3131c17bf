#!/bin/bash
# Per-rank ms/step of the y-slab code (--virtual P, one GPU) for each libcfdj variant.
# usage: tools/slab_ab.sh build/a/libcfdj.so ...   (env NX, P, STEPS)
for lib in "$@"; do
  out=$(CFDJ_LIB=$lib timeout -k 10 200 python bench.py --nx ${NX:-16384} --virtual ${P:-8} --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-timing) || exit $?
  echo "$lib $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["ms_per_step"], d["config"]["parallelism"])')"
done
