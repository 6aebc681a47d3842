# Stochastic codec iteration: microbench, GPU stochastic tests, stoch config bench.
set -o pipefail
mkdir -p gpurun_out
echo "== microbench"; timeout -k 10 120 ./tools/microbench_stoch_bucket > gpurun_out/mb_sb.txt 2>&1; rc=$?; cat gpurun_out/mb_sb.txt; [ $rc -eq 0 ] || exit $rc
echo "== pytest stoch"; timeout -k 10 400 python -u -m pytest tests/test_gpu_stoch.py tests/test_gpu_channel.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_stoch.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_stoch.log; [ $rc -eq 0 ] || exit $rc
echo "== stoch"; timeout -k 10 300 python tools/bench_configs.py --mode stoch --steps 20 --warmup 3 > gpurun_out/stoch.json 2> gpurun_out/stoch.err; rc=$?; cat gpurun_out/stoch.json; exit $rc
