#!/bin/bash
# A/B of variant libraries (build/<name>/libcfdj.so) on the cavity's DST passes: kernel stats of
# 22 steps at 2048^2 under rocprofv3.  usage: tools/ab_cav.sh OUTDIR name...  ("default" = in-tree)
out=$1; shift
mkdir -p $out; export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = default ]; then unset CFDJ_LIB; else export CFDJ_LIB=$PWD/build/$v/libcfdj.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$v -o p -- python3 tools/cav_prof.py dst > $out/$v.log 2>&1 || exit 1
  echo "== $v"; python3 tools/kstats.py $out/$v/p_kernel_stats.csv > $out/$v.txt; sed -n 1,6p $out/$v.txt
done
