# rocprofv3 kernel trace + separate PMC passes (FETCH_SIZE, WRITE_SIZE) over the stochastic-codec bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
echo "== stoch"; timeout -k 10 300 python3 $R/tools/bench_configs.py --mode stoch --steps 20 --warmup 3 > $R/gpurun_out/stoch.json 2> $R/gpurun_out/stoch.err; rc=$?; cat $R/gpurun_out/stoch.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
B="$R/tools/bench_configs.py --mode stoch --steps 10 --warmup 2 --no-cpu"
echo "== trace"; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stoch_trace -o trace -- python3 $B > $R/gpurun_out/prof_stoch_trace.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
echo "== fetch"; timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_stoch_fetch -o fetch -- python3 $B > $R/gpurun_out/prof_stoch_fetch.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
echo "== write"; timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_stoch_write -o write -- python3 $B > $R/gpurun_out/prof_stoch_write.log 2>&1; rc=$?
find $R/gpurun_out/prof_stoch_trace -name "*stats*.csv" -exec cat {} \;
exit $rc
