# Round-3 item: is the rocprofv3 SIGSEGV at exit (round 2, C3 bench with the cooperative encode) the
# profiler's, the cooperative launch's or libadfl_slq's teardown? Each step records its exit status.
set -o pipefail
mkdir -p gpurun_out/coop_repro
cd /tmp && export TMPDIR=/tmp PYTHONFAULTHANDLER=1
R=$GRAFT_REPO_ROOT
echo "== plain repro"; timeout -k 10 60 $R/tools/coop_repro 3; echo "rc=$?"
echo "== repro under rocprofv3 --kernel-trace --stats"; timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/coop_repro/min -o run -- $R/tools/coop_repro 3 > $R/gpurun_out/coop_repro/min.log 2>&1; echo "rc=$?"; tail -25 $R/gpurun_out/coop_repro/min.log
echo "== python c3 --coop-ab plain"; timeout -k 10 180 python $R/tools/bench_configs.py --mode c3 --coop-ab > $R/gpurun_out/coop_repro/c3_plain.json 2> $R/gpurun_out/coop_repro/c3_plain.err; echo "rc=$?"
echo "== python c3 --coop-ab under rocprofv3 --kernel-trace --stats"; timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/coop_repro/c3 -o run -- python $R/tools/bench_configs.py --mode c3 --coop-ab > $R/gpurun_out/coop_repro/c3_prof.log 2>&1; echo "rc=$?"; tail -40 $R/gpurun_out/coop_repro/c3_prof.log
exit 0
