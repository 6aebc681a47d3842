#!/bin/bash
# round 4 final evidence at HEAD: the full GPU suite (verbose), smoke(), the default bench line with its wall time
set -o pipefail
O=gpurun_out/final_r04
mkdir -p $O
sha256sum ad-federatedlearning_amd/adfl_amd/lib/libadfl_slq.so > $O/lib_sha256.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_verbose.txt 2>&1
rc=$?
tail -3 $O/pytest_gpu_verbose.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || exit $?
tail -1 $O/smoke.txt
t0=$(date +%s.%N)
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?
t1=$(date +%s.%N)
echo "bench wall_s $(python3 -c "print(round($t1 - $t0, 1))")" | tee $O/bench_wall.txt
tail -c 600 $O/bench.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/torch_norm_bench.py --reps 9 > $O/torch_norm_bench.txt 2>&1
rc=$?
tail -1 $O/torch_norm_bench.txt | cut -c1-400
exit $rc
