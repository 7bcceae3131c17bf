set -e
for v in base g4 base g4; do
  if [ $v = base ]; then unset CFDJ_LIB; else export CFDJ_LIB=$PWD/tools/micro/variants/libcfdj_$v.so; fi
  echo "== $v"
  KB_IDS=1,2,3 KB_N=20 timeout -k 10 60 python tools/kb_once.py
  timeout -k 10 120 python bench.py --steps 50 --warmup 10 --no-cpu-baseline 2>/dev/null | python -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print(d['value'], d['ms_per_step'], d['roofline']['frac'], [s['avg_launch_us'] for s in d['roofline']['per_stage']])
"
done
