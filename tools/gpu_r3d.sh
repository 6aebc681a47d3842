# Round 3 (d): int4 bucketed exchange + receive_mean: GPU tests, channel bench (aggregate), C3 bucket exchange int8 vs int4.
set -o pipefail
echo "== pytest"; timeout -k 10 400 python -u -m pytest tests/test_gpu_receive_mean.py tests/test_gpu_exchange_bucket.py tests/test_gpu_channel.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r3d.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r3d.log; [ $rc -eq 0 ] || exit $rc
echo "== channel"; timeout -k 10 300 python tools/bench_configs.py --mode channel --steps 20 --warmup 3 > gpurun_out/channel_r3d.json 2> gpurun_out/channel_r3d.err || exit 1; cat gpurun_out/channel_r3d.json
for L in c3_equal c3_loguniform; do
  for P in "" "--packed"; do
    echo "== exchange $L $P"; timeout -k 10 200 python tools/bench_configs.py --mode exchange --layout $L $P --steps 50 --warmup 10 2> gpurun_out/ex_err.txt | grep "^{" || exit 1
  done
done
exit 0
