#!/bin/bash
# Half-length DST kernels (default) against the odd-extension ones (CFDJ_DST_HALF=0): cavity
# tests, then kernel stats of 22 steps at 2048^2 under rocprofv3 for both.
# usage: tools/ab_dsth.sh OUTDIR
out=$1; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cavity.py -m gpu > $out/pytest_cavity.log 2>&1; rc=$?
tail -5 $out/pytest_cavity.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
for v in half odd; do
  if [ $v = odd ]; then export CFDJ_DST_HALF=0; else unset CFDJ_DST_HALF; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$v -o p -- python3 tools/cav_prof.py dst > $out/$v.log 2>&1 || exit 1
  echo "== $v"; python3 tools/kstats.py $out/$v/p_kernel_stats.csv > $out/$v.txt; sed -n 1,6p $out/$v.txt
done
