# Round 3: side-stream exchange (k2 + C4/C5 full size + bench leg), C5 overlap trace, resident timeline, coop repro control.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/trace_c5b
echo "== pytest"; timeout -k 10 900 python -u -m pytest tests/test_gpu_exchange_k2.py tests/test_gpu_exchange.py tests/test_gpu_exchange_full.py tests/test_gpu_bench_contract.py tests/test_gpu_parity.py tests/test_gpu_stoch.py tests/test_gpu_stoch_resident.py -m gpu -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r3c.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r3c.log; grep "^rank" gpurun_out/pytest_r3c.log | cut -c1-60; [ $rc -eq 0 ] || exit $rc
echo "== c5 trace"; (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/trace_c5b -o trace -- python $R/tools/exchange_trace.py --run > $R/gpurun_out/trace_c5b/run.log 2>&1); rc=$?; echo "rc=$rc"; tail -2 gpurun_out/trace_c5b/run.log; [ $rc -eq 0 ] || exit $rc
python tools/exchange_trace.py --report gpurun_out/trace_c5b > gpurun_out/trace_c5b/overlap.json || exit 1
echo "== resident timeline"; timeout -k 10 120 tools/microbench_resident_timeline 40 > gpurun_out/resident_timeline2.txt 2>&1; echo "rc=$?"; cat gpurun_out/resident_timeline2.txt
echo "== stoch bench"; timeout -k 10 300 python tools/bench_configs.py --mode stoch --steps 20 --warmup 3 > gpurun_out/stoch_r7.json 2> gpurun_out/stoch_r7.err; echo "rc=$?"; cat gpurun_out/stoch_r7.json
echo "== coop repro"; bash tools/gpu_coop_repro.sh > gpurun_out/coop_repro2.txt 2>&1; echo "rc=$?"; cat gpurun_out/coop_repro2.txt
exit 0
