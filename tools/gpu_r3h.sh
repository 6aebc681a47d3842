# Round 3 (h): vectorized fp16/bf16/fp64 stochastic kernels: parity tests + C3 timing.
set -o pipefail
echo "== pytest"; timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_stoch_dt.py > gpurun_out/dt_t.log 2>&1; rc=$?; tail -2 gpurun_out/dt_t.log; [ $rc -eq 0 ] || exit $rc
echo "== stoch"; timeout -k 10 300 python tools/bench_configs.py --mode stoch --steps 20 --warmup 3 --no-cpu > gpurun_out/stoch_r3h.json 2> gpurun_out/stoch_r3h.err || exit 1
python - <<'PY'
import json
d=json.load(open("gpurun_out/stoch_r3h.json"))
for k,v in d.items():
    if isinstance(v,dict) and ("float" in k or k.startswith("c3_bucket_") and "flushed" in k): print(k, v.get("encode_ms"), v.get("encode_frac"))
PY
