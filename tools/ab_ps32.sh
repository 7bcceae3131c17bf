#!/bin/bash
# A/B of the 3/2-rule solver's 3 * 2^k transform variants (build/<name>/libcfdj.so from
# tools/build_variant.sh): kernel stats of 4 steps at 4096^2 under rocprofv3 for each library.
# usage: tools/ab_ps32.sh OUTDIR name...   ("default" = the in-tree library)
out=$1; shift
mkdir -p $out; export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = default ]; then unset CFDJ_LIB; else export CFDJ_LIB=$PWD/build/$v/libcfdj.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$v -o p -- python3 tools/spec_prof.py 3/2 4096 3 > $out/$v.log 2>&1 || exit 1
  echo "== $v"; python3 tools/kstats.py $out/$v/p_kernel_stats.csv | head -7
done
