# Stochastic encode iteration: stochastic GPU tests (resident vs multi-launch vs oracle), the stochastic
# microbench (tools/microbench_stoch_res.hip), then the config bench with the resident path on and off
# (ADFL_STOCH_RESIDENT=0: multi-launch A/B).
set -o pipefail
mkdir -p gpurun_out
echo "== tests"; timeout -k 10 400 python -u -m pytest tests/test_gpu_stoch_resident.py tests/test_gpu_stoch.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_stoch.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_stoch.log; [ $rc -eq 0 ] || exit $rc
echo "== microbench"; timeout -k 10 200 ./tools/microbench_stoch_res > gpurun_out/mb_res.txt 2>&1; rc=$?; cat gpurun_out/mb_res.txt; [ $rc -eq 0 ] || exit $rc
echo "== stoch resident"; timeout -k 10 300 python tools/bench_configs.py --mode stoch --steps 20 --warmup 3 --no-cpu > gpurun_out/stoch_res.json 2> gpurun_out/stoch_res.err; rc=$?; cat gpurun_out/stoch_res.json; [ $rc -eq 0 ] || exit $rc
echo "== stoch multi"; ADFL_STOCH_RESIDENT=0 timeout -k 10 300 python tools/bench_configs.py --mode stoch --steps 20 --warmup 3 --no-cpu > gpurun_out/stoch_multi.json 2> gpurun_out/stoch_multi.err; rc=$?; cat gpurun_out/stoch_multi.json; exit $rc
