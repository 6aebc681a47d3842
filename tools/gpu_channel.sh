set -o pipefail
mkdir -p gpurun_out
echo "== pytest channel"; timeout -k 10 600 python -m pytest tests/test_gpu_channel.py tests/test_gpu_exchange.py -x -q -p no:cacheprovider > gpurun_out/pytest_channel.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_channel.log; [ $rc -eq 0 ] || exit $rc
echo "== channel"; timeout -k 10 400 python tools/bench_configs.py --mode channel --steps 20 --warmup 3 > gpurun_out/channel.json 2> gpurun_out/channel.err; rc=$?; cat gpurun_out/channel.json; tail -3 gpurun_out/channel.err; exit $rc
