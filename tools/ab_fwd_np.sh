mkdir -p gpurun_out/r3i
for v in 0 2 4 8; do
  CFDJ_FWD_NP=$v timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/r3i/bench_fwdnp$v.json 2> gpurun_out/r3i/bench_fwdnp$v.err || exit 1
done
CFDJ_FWD_NP=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "fused_fps or fused_vm" > gpurun_out/r3i/pytest_np4.log 2>&1; echo "np4 pytest rc=$?"
python - <<'PY'
import json
for v in (0,2,4,8):
    d=json.load(open(f"gpurun_out/r3i/bench_fwdnp{v}.json"))
    print(v, d["ms_per_step"], d["kernels"]["fft_fwd"], d["kernel_bench"]["rows_fwd_kernel"]["us_per_launch"], d["kernels"]["divide"]["ms_per_step"], d["kernels"]["stage"]["ms_per_step"])
PY
