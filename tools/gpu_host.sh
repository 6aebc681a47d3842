# Host-path iteration: channel GPU tests, the per-phase breakdown, the C3 channel bench and the PCIe modes.
set -o pipefail
mkdir -p gpurun_out
echo "== pytest channel"; timeout -k 10 600 python -u -m pytest tests/test_gpu_channel.py tests/test_gpu_stoch.py tests/test_gpu_accumulate.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_channel.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_channel.log; [ $rc -eq 0 ] || exit $rc
echo "== breakdown"; timeout -k 10 200 python tools/channel_breakdown.py > gpurun_out/breakdown.json 2> gpurun_out/breakdown.err; rc=$?; cat gpurun_out/breakdown.json; [ $rc -eq 0 ] || exit $rc
echo "== channel"; timeout -k 10 300 python tools/bench_configs.py --mode channel --steps 20 --warmup 3 > gpurun_out/channel.json 2> gpurun_out/channel.err; rc=$?; cat gpurun_out/channel.json; [ $rc -eq 0 ] || exit $rc
echo "== pcie"; timeout -k 10 300 python tools/bench_configs.py --mode pcie --steps 10 --warmup 2 > gpurun_out/pcie.json 2> gpurun_out/pcie.err; rc=$?; cat gpurun_out/pcie.json; exit $rc
