#!/bin/bash
# Trace kernel of the substructured solve: modes per workgroup (library paths in LIBS).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/ab_trace; mkdir -p $out
for cfg in "8192 8" "8192 4" "8192 2" "4096 4"; do
  set -- $cfg
  i=0
  for lib in $LIBS; do
    i=$((i+1))
    d=$out/n$1p$2v$i
    CFDJ_LIB=$lib timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o t -- python3 tools/solo_run.py --nx $1 --ranks $2 --steps 20 --no-overlap > $d.log 2>&1
    echo "== $1 / $2 $lib"; python3 tools/kstats.py $d/t_kernel_stats.csv | grep -E "schur_trace" | cut -c1-100
  done
done
