"""The bench line's host-to-host C3 dict leg (bench.channel_c3_dict) in a fresh process, optionally after other
bench legs, to tell the leg's own cost from the state earlier legs leave behind:

    python tools/host_dict_order.py head            # the leg alone
    python tools/host_dict_order.py c3+c5+pinned    # after the C3, C5 and pinned 1 GiB legs, as bench.py runs it
"""
import json, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench
dev = torch.device("cuda", 0)
from adfl_amd import _lib
lib = _lib.load()
mode = sys.argv[1]
for step in mode.split("+"):
    if step == "c3":
        bench.extra_c3(dev, lib, 20); torch.cuda.empty_cache()
    elif step == "c5":
        bench.extra_c5(dev, lib, 10); torch.cuda.empty_cache()
    elif step == "pinned":
        bench.extra_pcie(dev, lib, 5); torch.cuda.empty_cache()
    elif step == "head":
        pass
r = bench.channel_c3_dict(5)
print(mode, r["round_trip_ms"], r["encode_ms"], r["decode_ms"], json.dumps(r["phases_ms"]), flush=True)
