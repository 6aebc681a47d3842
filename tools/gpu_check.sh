set -o pipefail
mkdir -p gpurun_out
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== pytest gpu"; timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
if [ -x tools/microbench ]; then echo "== microbench"; timeout -k 10 300 ./tools/microbench 28 > gpurun_out/microbench.txt 2>&1; rc=$?; cat gpurun_out/microbench.txt; [ $rc -eq 0 ] || exit $rc; fi
echo "== bench"; timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; exit $rc
