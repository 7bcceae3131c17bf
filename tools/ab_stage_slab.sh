#!/bin/bash
# Rows per wavefront of the marching stage kernel on one rank's slab (whole-step time).
set -e
for cfg in "8192 2" "4096 2" "4096 4" "4096 8" "2048 2" "2048 4"; do
  set -- $cfg
  for rpw in 8 16 32; do
    timeout -k 10 100 python3 tools/solo_run.py --nx $1 --ranks $2 --steps 40 --no-overlap --rpw $rpw
  done
done
