# Round 3 (e): tiled stochastic decode: stochastic GPU tests + stoch bench.
set -o pipefail
echo "== pytest"; timeout -k 10 500 python -u -m pytest tests/test_gpu_stoch.py tests/test_gpu_stoch_resident.py tests/test_gpu_channel.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r3e.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r3e.log; [ $rc -eq 0 ] || exit $rc
echo "== stoch"; timeout -k 10 300 python tools/bench_configs.py --mode stoch --steps 20 --warmup 3 > gpurun_out/stoch_r3e.json 2> gpurun_out/stoch_r3e.err || exit 1
python - <<'PY'
import json
d=json.load(open("gpurun_out/stoch_r3e.json"))
for k,v in d.items():
    if isinstance(v,dict) and "decode_ms" in v: print(k, "enc", v.get("encode_ms"), v.get("encode_frac"), "dec", v["decode_ms"], v.get("decode_frac"))
PY
