# Round 4 (h): host channel timeline with the pipelined output creation + async scatter; channel GPU tests.

set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4h
mkdir -p $O
timeout -k 10 200 python -u $R/tools/channel_timeline.py --calls 40 > $O/timeline.json 2> $O/timeline.err || exit 1
python - <<'PY'
import json
for f in ("timeline",):
    d = json.load(open(f"gpurun_out/r4h/{f}.json"))
    print(f, {k: (v["total_ms_median"], v["total_ms_min"]) for k, v in d.items()})
PY
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_channel.py tests/test_gpu_receive_mean.py tests/test_gpu_compression.py tests/test_gpu_stoch_receive_mean.py tests/test_gpu_aggregate_golden.py tests/test_gpu_stoch.py > gpurun_out/r4h/pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r4h/pytest.txt; exit $rc
