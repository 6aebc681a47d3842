# Round 4 (o): host channel vs pool size (ADFL_HOST_THREADS 16 / 8 / 4), alternating processes; the box's
# CPU affinity and NUMA placement of the GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4o
mkdir -p $O
python -c "import os; print('affinity', len(os.sched_getaffinity(0)), sorted(os.sched_getaffinity(0))[:4], 'cpu_count', os.cpu_count())"
cat /sys/class/drm/card*/device/numa_node 2>/dev/null | head -3; ls /sys/devices/system/node | head; nproc
for rep in 1 2; do
  for th in 16 8 4; do
    ADFL_HOST_THREADS=$th timeout -k 10 200 python -u $R/tools/channel_timeline.py --calls 60 > $O/t${th}_$rep.json 2> $O/t${th}_$rep.err || exit 1
  done
done
python - <<'PY'
import json
for rep in (1, 2):
    for th in (16, 8, 4):
        d = json.load(open(f"gpurun_out/r4o/t{th}_{rep}.json"))
        print(th, rep, {w: d["spread"][w]["p10_p50_p90_ms"] for w in ("encode", "decode")})
PY
