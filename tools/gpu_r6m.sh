# round 6: the bench line with the new stochastic legs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r06m}
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench_line.json 2> $O/bench.err
echo rc=$?
