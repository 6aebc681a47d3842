# C5 int4 quantize: HIP-event timing with and without rocprofv3 kernel tracing, same box, same call.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c5_ab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/bench_configs.py --mode c5_int4 --steps 20 --warmup 3 > $O/plain1.json 2> $O/plain1.err && cat $O/plain1.json &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o c5 -- python3 $R/tools/bench_configs.py --mode c5_int4 --steps 20 --warmup 3 > $O/traced.log 2>&1 && grep '"metric"' $O/traced.log &&
timeout -k 10 120 python3 $R/tools/bench_configs.py --mode c5_int4 --steps 20 --warmup 3 > $O/plain2.json 2> $O/plain2.err && cat $O/plain2.json
