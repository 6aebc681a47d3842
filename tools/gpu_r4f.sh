# Round 4 (f): per-phase timeline of the host-to-host C3 channel calls at HEAD.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4f
mkdir -p $O
timeout -k 10 200 python -u $R/tools/channel_timeline.py --calls 30 > $O/timeline.json 2> $O/timeline.err; rc=$?; cat $O/timeline.json; tail -3 $O/timeline.err; exit $rc
