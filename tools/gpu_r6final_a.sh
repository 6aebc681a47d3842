# round 6 final, part A: the whole GPU suite, smoke(), then the default bench line (tests failing do not stop
# the bench; a crash or time limit does)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
rc=$?
echo "pytest rc=$rc" > $O/rc.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench_line.json 2> $O/bench.err
echo rc=$?
