# SQ counter passes over the stochastic microbench (2 reps per variant): issue / wait breakdown per kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
echo "== sq1"; timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $O/prof_sq1 -o sq1 -- $R/tools/microbench_stoch_res 2 > $O/prof_sq1.log 2>&1; rc=$?; tail -2 $O/prof_sq1.log; [ $rc -eq 0 ] || exit $rc
echo "== sq2"; timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $O/prof_sq2 -o sq2 -- $R/tools/microbench_stoch_res 2 > $O/prof_sq2.log 2>&1; rc=$?; tail -2 $O/prof_sq2.log
find $O/prof_sq1 $O/prof_sq2 -name "*.csv"
exit $rc
