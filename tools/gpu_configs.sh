set -o pipefail
mkdir -p gpurun_out
echo "== pytest gpu"; timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for m in "c3" "c5_int4" "pcie" "exchange" "exchange --packed --chunks 8 --elems 1073741824"; do
  echo "== $m"; timeout -k 10 300 python tools/bench_configs.py --mode $m >> gpurun_out/configs.jsonl 2> gpurun_out/configs.err; rc=$?; tail -1 gpurun_out/configs.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/configs.err; exit $rc; }
done
echo "== bench"; timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; cat gpurun_out/bench.json; exit $rc
