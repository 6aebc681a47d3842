# Round 3: the rocprofv3 SIGSEGV at exit (round 2, C3 bench with the cooperative encode). A torch-free,
# library-free program with one hipLaunchCooperativeKernel, plain and under rocprofv3 --kernel-trace, and the
# same program with ordinary launches only (the control). Each step records its exit status.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/coop_repro
cd /tmp && export TMPDIR=/tmp
echo "== plain repro"; timeout -k 10 60 $R/tools/coop_repro 3; echo "rc=$?"
echo "== repro under rocprofv3 --kernel-trace --stats"; timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/coop_repro/min -o run -- $R/tools/coop_repro 3 > $R/gpurun_out/coop_repro/min.log 2>&1; echo "rc=$?"; grep "^ok\|SIGSEGV\|PC:" $R/gpurun_out/coop_repro/min.log
echo "== control (ordinary launches) under rocprofv3 --kernel-trace --stats"; timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/coop_repro/ctl -o run -- $R/tools/coop_repro 3 plain > $R/gpurun_out/coop_repro/ctl.log 2>&1; echo "rc=$?"; grep "^ok\|SIGSEGV\|PC:" $R/gpurun_out/coop_repro/ctl.log
echo "== repro under rocprofv3 --kernel-trace (no --stats)"; timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/coop_repro/nostats -o run -- $R/tools/coop_repro 3 > $R/gpurun_out/coop_repro/nostats.log 2>&1; echo "rc=$?"; grep "^ok\|SIGSEGV\|PC:" $R/gpurun_out/coop_repro/nostats.log
exit 0
