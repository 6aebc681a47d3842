# Round-3 profile set: rocprofv3 kernel-trace stats of the headline bench and of the C3 / stochastic config
# benches, FETCH_SIZE and WRITE_SIZE passes (separate runs) over the headline bench and the C3 bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_r03
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # name, seconds, rocprof args..., -- program args
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 $secs rocprofv3 "$@" > $O/$name.log 2>&1; local rc=$?; grep '"metric"' $O/$name.log | cut -c1-300; return $rc
}
run trace_bench 300 --kernel-trace --stats --output-format csv -d $O/trace_bench -o bench -- python3 $R/bench.py --steps 50 --warmup 10 --no-cpu-baseline --pmc off &&
run fetch_bench 120 --pmc FETCH_SIZE --output-format csv -d $O/fetch_bench -o fetch -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --pmc off &&
run write_bench 120 --pmc WRITE_SIZE --output-format csv -d $O/write_bench -o write -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --pmc off &&
run trace_c3 300 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o c3 -- python3 $R/tools/bench_configs.py --mode c3 --steps 50 --warmup 5 &&
run fetch_c3 120 --pmc FETCH_SIZE --output-format csv -d $O/fetch_c3 -o fetch -- python3 $R/tools/bench_configs.py --mode c3 --steps 5 --warmup 1 &&
run write_c3 120 --pmc WRITE_SIZE --output-format csv -d $O/write_c3 -o write -- python3 $R/tools/bench_configs.py --mode c3 --steps 5 --warmup 1 &&
run trace_stoch 300 --kernel-trace --stats --output-format csv -d $O/trace_stoch -o stoch -- python3 $R/tools/bench_configs.py --mode stoch --steps 20 --warmup 3 --no-cpu &&
run fetch_stoch 150 --pmc FETCH_SIZE --output-format csv -d $O/fetch_stoch -o fetch -- python3 $R/tools/bench_configs.py --mode stoch --steps 3 --warmup 1 --no-cpu &&
run write_stoch 150 --pmc WRITE_SIZE --output-format csv -d $O/write_stoch -o write -- python3 $R/tools/bench_configs.py --mode stoch --steps 3 --warmup 1 --no-cpu &&
run trace_c5 300 --kernel-trace --stats --output-format csv -d $O/trace_c5 -o c5 -- python3 $R/tools/bench_configs.py --mode c5_int4 --steps 20 --warmup 3
rc=$?
find $O -name "*.csv" | sort
exit $rc
