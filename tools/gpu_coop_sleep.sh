# Poll back-off sweep of the cooperative encode (C3 config bench; coop and plain launches).
set -o pipefail
mkdir -p gpurun_out
echo "== tests"; timeout -k 10 200 python -u -m pytest tests/test_gpu_coop.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_coop2.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_coop2.log; [ $rc -eq 0 ] || exit $rc
for launch in coop plain; do for sl in 1 8 32 127; do
  ADFL_SLQ_COOP_LAUNCH=$launch ADFL_SLQ_COOP_SLEEP=$sl timeout -k 10 200 python tools/bench_configs.py --mode c3 > gpurun_out/c3_sleep.json 2> gpurun_out/c3_sleep.err || exit $?
  python -c "
import json; d=json.load(open('gpurun_out/c3_sleep.json'))
print('$launch', $sl, 'loguniform coop enc', d['loguniform_layout']['flushed']['encode_ms'], 'rt', d['loguniform_layout']['flushed']['round_trip_ms'], '| equal coop enc', d['equal_coop']['flushed']['encode_ms'], '| twopass enc', d['loguniform_twopass']['flushed']['encode_ms'])"
done; done
