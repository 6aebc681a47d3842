set -o pipefail
mkdir -p gpurun_out/r3n
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3n/pytest_gpu.log 2>&1 && tail -3 gpurun_out/r3n/pytest_gpu.log &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3n/smoke.log 2>&1 && tail -2 gpurun_out/r3n/smoke.log &&
timeout -k 10 300 python -u bench.py > gpurun_out/r3n/bench.json 2> gpurun_out/r3n/bench.err && cat gpurun_out/r3n/bench.json
