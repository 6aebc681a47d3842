# round 6: k_tn_short timeline (stats build), C3 equal
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r06g}
mkdir -p $O
ADFL_LIB_VARIANT=tools/_variants/libadfl_stats.so timeout -k 10 120 python -u tools/ref_norm_prof.py --cfg c3 --reps 2 > $O/stats.txt 2>&1
echo rc=$?
