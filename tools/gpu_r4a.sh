# Round 4 (a): torch-order mean kernels — new parity tests (mean order, reference-executed aggregate
# fixtures), the existing mean / exchange / receive_mean tests, then the exchange bench at world 1.
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_mean_order.py tests/test_gpu_aggregate_golden.py tests/test_gpu_receive_mean.py \
  tests/test_gpu_stoch_receive_mean.py tests/test_gpu_exchange.py tests/test_gpu_exchange_k2.py \
  tests/test_gpu_exchange_bucket.py tests/test_gpu_parity.py tests/test_gpu_custom_ops.py > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; grep -E "FAILED|Error" $O/pytest.txt | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_configs.py --mode exchange --steps 20 --warmup 3 --no-cpu > $O/exchange.json 2> $O/exchange.err; rc=$?; tail -c 1500 $O/exchange.json; exit $rc
