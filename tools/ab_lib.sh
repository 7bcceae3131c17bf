#!/bin/bash
# A/B of a variant library (build/<name>/libcfdj.so from tools/build_variant.sh) against the
# in-tree one: the headline bench line, the kernel stats of the 3/2-rule solver, and the FFT
# parity tests under the variant.
# usage: tools/ab_lib.sh OUTDIR name
out=$1; v=$2
mkdir -p $out; export TMPDIR=/tmp
for lib in default $v; do
  if [ "$lib" = default ]; then unset CFDJ_LIB; else export CFDJ_LIB=$PWD/build/$lib/libcfdj.so; fi
  timeout -k 10 200 python3 bench.py --steps 50 --no-cpu-baseline --no-ladders > $out/bench_$lib.json 2> $out/bench_$lib.err || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/spec_$lib -o p -- python3 tools/spec_prof.py 3/2 4096 3 > $out/spec_$lib.log 2>&1 || exit 1
  echo "== $lib"; python3 tools/kstats.py $out/spec_$lib/p_kernel_stats.csv | head -8
done
python3 - $out $v <<'PY'
import json, sys
out, v = sys.argv[1:3]
for lib in ("default", v):
    d = json.load(open(f"{out}/bench_{lib}.json"))
    print(lib, d["ms_per_step"], {k: d["kernels"][k] for k in d["kernels"]})
PY
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_spectral.py tests/test_gpu_cavity.py tests/test_gpu_schur.py -m gpu > $out/pytest_$v.log 2>&1; echo "pytest($v) rc=$?"; tail -3 $out/pytest_$v.log
