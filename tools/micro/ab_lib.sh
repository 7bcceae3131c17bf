# A/B of library variants under tools/micro/variants: kernel microbench of the ids in KB_IDS.
set -e
for v in base "$@"; do
  if [ $v = base ]; then unset CFDJ_LIB; else export CFDJ_LIB=$PWD/tools/micro/variants/libcfdj_$v.so; fi
  echo "== $v"
  KB_N=20 timeout -k 10 60 python tools/kb_once.py
done
