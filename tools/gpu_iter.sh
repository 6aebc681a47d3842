# Iteration check: selected GPU tests, microbenches, config benches and the headline bench (+ C4 leg).
set -o pipefail
mkdir -p gpurun_out
T=${TESTS:-tests/test_gpu_parity.py}
echo "== pytest $T"; timeout -k 10 400 python -u -m pytest $T -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_iter.log; [ $rc -eq 0 ] || exit $rc
for mb in microbench_bucket microbench_stoch_bucket; do
  echo "== $mb"; timeout -k 10 120 ./tools/$mb > gpurun_out/$mb.txt 2>&1; rc=$?; cat gpurun_out/$mb.txt; [ $rc -eq 0 ] || exit $rc
done
for m in c3 stoch; do
  echo "== $m"; timeout -k 10 300 python tools/bench_configs.py --mode $m --steps 50 --warmup 5 > gpurun_out/$m.json 2> gpurun_out/$m.err; rc=$?; cat gpurun_out/$m.json; [ $rc -eq 0 ] || exit $rc
done
echo "== bench"; timeout -k 10 300 python bench.py --steps 50 --warmup 10 --exchange on --no-cpu-baseline --pmc off > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; cat gpurun_out/bench.json; exit $rc
