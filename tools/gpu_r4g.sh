# Round 4 (g): host channel timeline after the positional payload objects and 8 staging pieces; the same
# with glibc keeping freed memory (no trim, fixed 32 MiB mmap threshold) to size the page-fault share.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4g
mkdir -p $O
timeout -k 10 200 python -u $R/tools/channel_timeline.py --calls 40 > $O/timeline.json 2> $O/timeline.err || exit 1
MALLOC_TRIM_THRESHOLD_=4294967296 MALLOC_MMAP_THRESHOLD_=33554432 timeout -k 10 200 python -u $R/tools/channel_timeline.py --calls 40 > $O/timeline_keep.json 2> $O/timeline_keep.err || exit 1
python - <<'PY'
import json
for f in ("timeline", "timeline_keep"):
    d = json.load(open(f"gpurun_out/r4g/{f}.json"))
    print(f, {k: (v["total_ms_median"], v["total_ms_min"]) for k, v in d.items()})
PY
