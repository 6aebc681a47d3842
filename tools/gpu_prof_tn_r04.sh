# Round-4 profile of the reference-order norm kernels (k_norm_walk on C3, k_norm_torch on C2, next to the
# default norm and the encodes): rocprofv3 kernel-trace stats and FETCH_SIZE / WRITE_SIZE passes over
# tools/torch_norm_bench.py, summarised per kernel by tools/pmc_kernels.py.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_tn_r04
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # name, seconds, rocprof args..., -- program args
  local name=$1 secs=$2; shift 2
  echo "== $name"; timeout -k 10 $secs rocprofv3 "$@" > $O/$name.log 2>&1; local rc=$?; grep '^C' $O/$name.log | cut -c1-160; return $rc
}
run trace_tn 300 --kernel-trace --stats --output-format csv -d $O/trace_tn -o tn -- python3 $R/tools/torch_norm_bench.py --reps 9 --no-seq &&
run fetch_tn 200 --pmc FETCH_SIZE --output-format csv -d $O/fetch_tn -o fetch -- python3 $R/tools/torch_norm_bench.py --reps 2 --no-seq &&
run write_tn 200 --pmc WRITE_SIZE --output-format csv -d $O/write_tn -o write -- python3 $R/tools/torch_norm_bench.py --reps 2 --no-seq
rc=$?
cd $R
f=$(find $O/fetch_tn -name "*counter_collection.csv" | head -1); g=$(find $O/write_tn -name "*counter_collection.csv" | head -1)
[ -n "$f" ] && [ -n "$g" ] && python3 tools/pmc_kernels.py "$f" "$g" > $O/pmc_tn_traffic.json && echo "pmc_tn: $(python3 -c "import json;print(len(json.load(open('$O/pmc_tn_traffic.json'))['kernels']))") kernels"
find $O -name "*kernel_stats.csv" | sort
exit $rc
