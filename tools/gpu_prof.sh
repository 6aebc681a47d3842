# rocprofv3 kernel trace + separate PMC passes over the bench workload, plus the microbench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
echo "== microbench"; timeout -k 10 300 $R/tools/microbench 28 > $R/gpurun_out/microbench.txt 2>&1; rc=$?; cat $R/gpurun_out/microbench.txt; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
echo "== trace"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_trace -o trace -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/prof_trace.log 2>&1; rc=$?; grep -v "^W20" $R/gpurun_out/prof_trace.log | tail -2; [ $rc -eq 0 ] || exit $rc
echo "== fetch"; timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_fetch -o fetch -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_fetch.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
echo "== write"; timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_write -o write -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_write.log 2>&1; rc=$?
find $R/gpurun_out/prof_trace $R/gpurun_out/prof_fetch $R/gpurun_out/prof_write -name "*.csv" | head -20
exit $rc
