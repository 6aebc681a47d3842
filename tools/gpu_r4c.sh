# Round 4 (c): int8 quantize variants (the headline's dominant kernel) at C2 and C5 sizes; PMC passes over
# the int8 / int4 flat kernels on one input at 2^28 and 2^30.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4c
mkdir -p $O
timeout -k 10 120 $R/tools/microbench_q8var 28 21 > $O/q8var_28.txt 2>&1 && cat $O/q8var_28.txt &&
timeout -k 10 120 $R/tools/microbench_q8var 30 9 > $O/q8var_30.txt 2>&1 && cat $O/q8var_30.txt || exit 1
cd /tmp && export TMPDIR=/tmp
i=0
for lg in 28 30; do
  for set in "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_STALL_sum" \
             "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_BUSY_sum" \
             "TA_BUSY_avr TD_TD_BUSY_sum GRBM_GUI_ACTIVE" \
             "SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $set --output-format csv -d $O/pmc_$i -o p -- $R/tools/microbench_q8q4 $lg 3 > $O/pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/pmc_$i.log; exit 1; }
    echo "pass $i (2^$lg): $set" >> $O/pmc_index.txt
  done
done
echo "pmc passes done: $i"
