set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3 4 5 6; do for v in memcpy stream; do ADFL_HOST_LIB=tools/hc_$v.so timeout -k 10 120 python tools/hostcopy_ab.py pinned || exit 1; done; done > gpurun_out/hcab.txt 2>&1
cat gpurun_out/hcab.txt
