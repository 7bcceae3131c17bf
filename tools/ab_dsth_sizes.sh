out=gpurun_out/r3h4; mkdir -p $out; export TMPDIR=/tmp
for n in 4096 1024; do
for v in half odd; do
  if [ $v = odd ]; then export CFDJ_DST_HALF=0; else unset CFDJ_DST_HALF; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$v$n -o p -- python3 tools/cav_prof.py dst $n > $out/$v$n.log 2>&1 || exit 1
  echo "== $v $n"; python3 tools/kstats.py $out/$v$n/p_kernel_stats.csv > $out/$v$n.txt; sed -n 1,4p $out/$v$n.txt
done
done
