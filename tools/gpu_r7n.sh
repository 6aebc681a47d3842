# round 6: sampled phase A, chunks per wave A/B (2 / 4 product / 8): C2 per dtype under a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r07n}
mkdir -p $O
for v in product cpw2 cpw8; do
  if [ $v = product ]; then L=; else L=tools/_variants/libadfl_$v.so; fi
  for d in f32 bf16 f16; do
    ADFL_LIB_VARIANT=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_${v}_$d -o run -- python tools/ref_norm_prof.py --cfg c2 --dtype $d --reps 3 > $O/prof_${v}_$d.log 2>&1 || exit $?
  done
done
echo rc=0
