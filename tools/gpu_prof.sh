# rocprofv3 over the bench workload: kernel trace + stats (the bench line printed under the profiler is
# kept next to it), then FETCH_SIZE and WRITE_SIZE in separate PMC passes, then kernel traces of the
# C3 bucketed and stochastic config benches.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
echo "== trace"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_trace -o trace -- python3 $R/bench.py --steps 50 --warmup 10 --no-cpu-baseline --pmc off > $O/prof_trace.log 2>&1; rc=$?; grep '"metric"' $O/prof_trace.log; [ $rc -eq 0 ] || exit $rc
echo "== fetch"; timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/prof_fetch -o fetch -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --pmc off > $O/prof_fetch.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
echo "== write"; timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/prof_write -o write -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --pmc off > $O/prof_write.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
echo "== c3 trace"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o c3 -- python3 $R/tools/bench_configs.py --mode c3 --steps 50 --warmup 5 > $O/prof_c3.log 2>&1; rc=$?; grep '"metric"' $O/prof_c3.log; [ $rc -eq 0 ] || exit $rc
echo "== stoch trace"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_stoch -o stoch -- python3 $R/tools/bench_configs.py --mode stoch --steps 20 --warmup 3 > $O/prof_stoch.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
find $O/prof_trace $O/prof_fetch $O/prof_write $O/prof_c3 $O/prof_stoch -name "*.csv" | head -30
