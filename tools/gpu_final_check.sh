# Round-end evidence: the in-tree library's SHA-256, the full GPU suite verbose (every test id and its
# outcome), smoke(), and the default bench line.
set -o pipefail
O=gpurun_out/final
mkdir -p $O
sha256sum ad-federatedlearning_amd/adfl_amd/lib/libadfl_slq.so > $O/lib_sha256.txt &&
timeout -k 10 300 python -u -m pytest tests -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_verbose.txt 2>&1 && tail -2 $O/pytest_gpu_verbose.txt &&
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && cat $O/smoke.txt &&
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err && cut -c1-400 $O/bench.json
