# round 6: k_tn_short A/B of the serial chain start (64 / 128 / 256 product / 512 steps): C3 timing and trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r07m}
mkdir -p $O
for v in product ser64 ser128 ser512; do
  if [ $v = product ]; then L=; else L=tools/_variants/libadfl_$v.so; fi
  ADFL_LIB_VARIANT=$L timeout -k 10 200 python -u tools/ref_norm_bench.py --dtypes f32 --reps 21 --cfgs C3 > $O/bench_$v.txt 2>&1 || exit $?
  ADFL_LIB_VARIANT=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python tools/ref_norm_prof.py --cfg c3,c3lu --reps 10 > $O/prof_$v.log 2>&1 || exit $?
done
echo rc=0
