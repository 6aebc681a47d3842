#!/bin/bash
# Kernel trace and HBM traffic of any workload, on the GPU box: rocprofv3 --kernel-trace --stats, then separate
# FETCH_SIZE and WRITE_SIZE passes (counters only in their own runs), summarised per kernel and grid by
# tools/pmc_kernels.py (with the guide's gfx950 FETCH_SIZE correction).
#
#   tools/gpu_prof.sh NAME [--no-pmc] [--secs S] -- python3 tools/ref_norm_prof.py --cfg c2 --reps 3
#
# Writes gpurun_out/prof_NAME/{trace,fetch,write}/ and pmc_traffic.json; the program runs from the repo root
# (put it right after "--": python3 ..., never env / bash -c). Stops at the first failing step.
set -o pipefail
name=$1
shift
pmc=1
secs=300
while [ $# -gt 0 ] && [ "$1" != "--" ]; do
  case $1 in
    --no-pmc) pmc=0 ;;
    --secs) secs=$2; shift ;;
    *) echo "unknown option $1" >&2; exit 2 ;;
  esac
  shift
done
[ "$1" = "--" ] && shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_$name
mkdir -p "$O"
export TMPDIR=/tmp
cd "$R" || exit 1
timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o trace -- "$@" > "$O/trace.log" 2>&1 || exit $?
if [ $pmc = 1 ]; then
  timeout -k 10 "$secs" rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch" -o fetch -- "$@" > "$O/fetch.log" 2>&1 || exit $?
  timeout -k 10 "$secs" rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write" -o write -- "$@" > "$O/write.log" 2>&1 || exit $?
  f=$(find "$O/fetch" -name "*counter_collection.csv" | head -1)
  g=$(find "$O/write" -name "*counter_collection.csv" | head -1)
  python3 tools/pmc_kernels.py "$f" "$g" > "$O/pmc_traffic.json" || exit $?
fi
find "$O" -name "*kernel_stats.csv"
