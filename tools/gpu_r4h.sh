#!/bin/bash
# round 4: vectorized host absmax (target_clones) — host tests, C3 channel timeline, the bench line
set -o pipefail
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_hostcopy.py tests/test_gpu_channel.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1
rc=$?; tail -1 $O/pytest.txt; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 200 python -u tools/channel_timeline.py --calls 30 > $O/timeline_$i.json 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('$O/timeline_$i.json'));print('timeline', d['spread']['encode']['p10_p50_p90_ms'], d['spread']['decode']['p10_p50_p90_ms'])"
done
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'], d['pcie']['channel_c3_dict'], d['bench_wall_s'])"
