# Round 4 (e): where ADFL's host-to-host C3 call pattern spends its milliseconds at HEAD (cProfile + minima).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4e
mkdir -p $O
timeout -k 10 200 python -u $R/tools/prof_channel_py.py > $O/prof_channel_py.txt 2>&1; rc=$?; head -60 $O/prof_channel_py.txt; exit $rc
