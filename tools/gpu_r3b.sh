# Round 3: new GPU tests (custom ops, any-offset accumulate, bench self-check, C4/C5 at full size), the C5
# exchange overlap trace, and the cooperative-launch profiler repro. Each GPU step has its own time limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/trace_c5
echo "== pytest"; timeout -k 10 900 python -u -m pytest tests/test_gpu_custom_ops.py tests/test_gpu_accumulate.py tests/test_gpu_bench_contract.py tests/test_gpu_exchange_full.py -m gpu -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r3b.log 2>&1; rc=$?; tail -6 gpurun_out/pytest_r3b.log; grep "^rank" gpurun_out/pytest_r3b.log; [ $rc -eq 0 ] || exit $rc
echo "== c5 trace"; (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/trace_c5 -o trace -- python $R/tools/exchange_trace.py --run > $R/gpurun_out/trace_c5/run.log 2>&1); rc=$?; echo "rc=$rc"; tail -3 gpurun_out/trace_c5/run.log; [ $rc -eq 0 ] || exit $rc
python tools/exchange_trace.py --report gpurun_out/trace_c5 > gpurun_out/trace_c5/overlap.json; rc=$?; head -c 1500 gpurun_out/trace_c5/overlap.json; [ $rc -eq 0 ] || exit $rc
echo "== resident timeline"; timeout -k 10 120 tools/microbench_resident_timeline 40 > gpurun_out/resident_timeline.txt 2>&1; echo "rc=$?"; cat gpurun_out/resident_timeline.txt
echo "== coop repro"; bash tools/gpu_coop_repro.sh > gpurun_out/coop_repro.txt 2>&1; echo "rc=$?"
exit 0
