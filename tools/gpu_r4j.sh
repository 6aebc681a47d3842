# Round 4 (j): host channel timeline with host-side scales (fused gather+absmax) vs the previous path; channel GPU tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4j
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 200 python -u $R/tools/channel_timeline.py --calls 40 > $O/pipe_$rep.json 2> $O/pipe_$rep.err || exit 1
  timeout -k 10 200 python -u $R/tools/channel_timeline.py --calls 40 --no-pipeline > $O/nopipe_$rep.json 2> $O/nopipe_$rep.err || exit 1
done
python - <<'PY'
import json
for f in ("pipe_1", "nopipe_1", "pipe_2", "nopipe_2"):
    d = json.load(open(f"gpurun_out/r4j/{f}.json"))
    print(f, {k: (v["total_ms_median"], v["total_ms_min"], v["free_previous_result_ms_median"]) for k, v in d.items()})
PY
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_channel.py tests/test_gpu_receive_mean.py tests/test_gpu_compression.py tests/test_gpu_stoch_receive_mean.py tests/test_gpu_aggregate_golden.py tests/test_gpu_stoch.py tests/test_gpu_parity.py tests/test_gpu_bucket_copy.py > gpurun_out/r4j/pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r4j/pytest.txt; exit $rc
