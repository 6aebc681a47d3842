# Iteration check: selected GPU tests, then C3 config bench and the headline bench (with the C4 leg).
set -o pipefail
mkdir -p gpurun_out
T=${TESTS:-tests/test_gpu_resident.py tests/test_gpu_parity.py}
echo "== pytest $T"; timeout -k 10 400 python -u -m pytest $T -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_iter.log; [ $rc -eq 0 ] || exit $rc
echo "== c3"; timeout -k 10 300 python tools/bench_configs.py --mode c3 > gpurun_out/c3.json 2> gpurun_out/c3.err; rc=$?; cat gpurun_out/c3.json; tail -3 gpurun_out/c3.err; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 300 python bench.py --steps 50 --warmup 10 --exchange on --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; exit $rc
