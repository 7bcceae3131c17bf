#!/bin/bash
# rocprofv3 evidence for the bench command: kernel-trace stats of the headline run, then the
# FETCH_SIZE and WRITE_SIZE counter passes (one run each), each step under its own limit.
# usage: tools/profile_bench.sh OUTDIR
out="${1:-gpurun_out/prof}"
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o bench -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$out/bench_under_rocprof.json" 2> "$out/stats.log" || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o fetch -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> "$out/fetch.log" || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o write -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> "$out/write.log" || exit $?
echo done
