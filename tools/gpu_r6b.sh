# round 6: k_tn_short counters (stats build) on C3 equal / log-uniform
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
ADFL_LIB_VARIANT=tools/_variants/libadfl_stats.so timeout -k 10 120 python -u tools/ref_norm_prof.py --cfg c3,c3lu --reps 2 > $O/stats.txt 2>&1
echo rc=$?
