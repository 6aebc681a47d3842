# Full GPU check at HEAD: smoke, every -m gpu test, the config benches (channel, C3, stochastic) and bench.py.
set -o pipefail
mkdir -p gpurun_out
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== pytest gpu"; timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; grep -c PASSED gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== channel"; timeout -k 10 300 python tools/bench_configs.py --mode channel --steps 20 --warmup 3 > gpurun_out/channel.json 2> gpurun_out/channel.err; rc=$?; cat gpurun_out/channel.json; [ $rc -eq 0 ] || exit $rc
echo "== c3"; timeout -k 10 300 python tools/bench_configs.py --mode c3 > gpurun_out/c3.json 2> gpurun_out/c3.err; rc=$?; cat gpurun_out/c3.json; [ $rc -eq 0 ] || exit $rc
echo "== stoch"; timeout -k 10 300 python tools/bench_configs.py --mode stoch --steps 20 --warmup 3 > gpurun_out/stoch.json 2> gpurun_out/stoch.err; rc=$?; cat gpurun_out/stoch.json; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; cat gpurun_out/bench.json; exit $rc
