# SQ issue/wait counters over the stochastic-codec bench (one PMC pass; no trace domains).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/rocprof_counters.txt 2>&1
echo "== sq"; timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES --output-format csv -d $R/gpurun_out/prof_stoch_sq -o sq -- python3 $R/tools/bench_configs.py --mode stoch --steps 5 --warmup 1 --no-cpu > $R/gpurun_out/prof_stoch_sq.log 2>&1; rc=$?
tail -3 $R/gpurun_out/prof_stoch_sq.log
exit $rc
