# Round 4 (n): host channel after the cached range plans / leaner entry loops: spread + phases; channel tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4n
mkdir -p $O
for rep in 1 2; do
timeout -k 10 200 python -u $R/tools/channel_timeline.py --calls 60 > $O/t$rep.json 2> $O/t$rep.err || exit 1
done
python - <<'PY'
import json
for rep in (1, 2):
    d = json.load(open(f"gpurun_out/r4n/t{rep}.json"))
    print(rep, {w: d["spread"][w]["p10_p50_p90_ms"] for w in ("encode", "decode")})
d = json.load(open("gpurun_out/r4n/t1.json"))
for w in ("encode", "decode"):
    for k, v in d["spread"][w]["fastest_quarter_phases"].items():
        if "native job wait" not in k or k.endswith("#0") or k.endswith("#7"):
            print("   ", w, k, v)
PY
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_channel.py tests/test_gpu_receive_mean.py tests/test_gpu_compression.py tests/test_gpu_aggregate_golden.py tests/test_gpu_parity.py tests/test_gpu_bucket_copy.py > $O/pytest.txt 2>&1; rc=$?; tail -3 $O/pytest.txt; exit $rc
