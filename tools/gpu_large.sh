set -o pipefail
mkdir -p gpurun_out
echo "== bigtest"; timeout -k 10 240 ./tools/bigtest > gpurun_out/bigtest.log 2>&1; rc=$?; cat gpurun_out/bigtest.log; exit $rc
