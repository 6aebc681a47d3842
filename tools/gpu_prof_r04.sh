# Round-4 profile set at HEAD: rocprofv3 kernel-trace stats of the headline bench and of the C3 /
# stochastic config benches, FETCH_SIZE and WRITE_SIZE passes (each its own run) over the same three, and
# the PMC summaries (tools/pmc_kernels.py) written next to them.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_r04
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # name, seconds, rocprof args..., -- program args
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 $secs rocprofv3 "$@" > $O/$name.log 2>&1; local rc=$?; grep '"metric"' $O/$name.log | cut -c1-200; return $rc
}
run trace_bench 300 --kernel-trace --stats --output-format csv -d $O/trace_bench -o bench -- python3 $R/bench.py --steps 50 --warmup 10 --no-cpu-baseline --pmc off --extras off &&
run fetch_bench 150 --pmc FETCH_SIZE --output-format csv -d $O/fetch_bench -o fetch -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --pmc off --extras off &&
run write_bench 150 --pmc WRITE_SIZE --output-format csv -d $O/write_bench -o write -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --pmc off --extras off &&
run trace_c3 300 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o c3 -- python3 $R/tools/bench_configs.py --mode c3 --steps 50 --warmup 5 &&
run fetch_c3 150 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c3 -o fetch -- python3 $R/tools/bench_configs.py --mode c3 --steps 5 --warmup 1 &&
run write_c3 150 --pmc WRITE_SIZE --output-format csv -d $O/write_c3 -o write -- python3 $R/tools/bench_configs.py --mode c3 --steps 5 --warmup 1 &&
run trace_stoch 300 --kernel-trace --stats --output-format csv -d $O/trace_stoch -o stoch -- python3 $R/tools/bench_configs.py --mode stoch --steps 20 --warmup 3 --no-cpu &&
run fetch_stoch 150 --pmc FETCH_SIZE --output-format csv -d $O/fetch_stoch -o fetch -- python3 $R/tools/bench_configs.py --mode stoch --steps 3 --warmup 1 --no-cpu &&
run write_stoch 150 --pmc WRITE_SIZE --output-format csv -d $O/write_stoch -o write -- python3 $R/tools/bench_configs.py --mode stoch --steps 3 --warmup 1 --no-cpu
rc=$?
cd $R
for w in bench c3 stoch; do
  f=$(find $O/fetch_$w -name "*counter_collection.csv" | head -1); g=$(find $O/write_$w -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && [ -n "$g" ] && python3 tools/pmc_kernels.py "$f" "$g" > $O/pmc_${w}_traffic.json && echo "pmc_$w: $(python3 -c "import json;print(len(json.load(open('$O/pmc_${w}_traffic.json'))['kernels']))") kernels"
done
find $O -name "*kernel_stats.csv" | sort
exit $rc
