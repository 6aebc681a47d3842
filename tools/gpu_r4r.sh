# Round 4 (r): full GPU suite (verbose) + the default bench line at HEAD.
set -o pipefail
O=gpurun_out/r4r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_verbose.txt 2>&1; rc=$?; tail -3 $O/pytest_gpu_verbose.txt; grep -E "FAILED|ERROR" $O/pytest_gpu_verbose.txt | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?; cut -c1-3000 $O/bench.json; exit $rc
