# C3 bucketed encode iteration: parity tests of the bucketed paths, the round-trip microbench, the config bench.
set -o pipefail
mkdir -p gpurun_out
echo "== parity"; timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_channel.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_c3.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_c3.log; [ $rc -eq 0 ] || exit $rc
echo "== c3"; timeout -k 10 300 python tools/bench_configs.py --mode c3 > gpurun_out/c3.json 2> gpurun_out/c3.err; rc=$?; cat gpurun_out/c3.json; exit $rc
