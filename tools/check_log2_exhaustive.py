"""Exhaustive check behind CNAT's log2 restatement (oracle/stoch_oracle.py): for EVERY fp32 v in
[2^-23, FLT_MAX] (the values fl(|x| + eps) can take), floor/ceil of torch's CPU fp32 log2 equal
floor/ceil of the correctly rounded fp32 log2. Run on the CPU (about a minute):

    python tools/check_log2_exhaustive.py
"""
import sys
import time

import numpy as np
import torch

lo = np.array([2.0 ** -23], np.float32).view(np.uint32)[0]
hi = np.array([np.finfo(np.float32).max], np.float32).view(np.uint32)[0]
step = 1 << 24
bad = 0
t0 = time.time()
for b in range(int(lo), int(hi) + 1, step):
    bits = np.arange(b, min(b + step, int(hi) + 1), dtype=np.uint32)
    v = bits.view(np.float32)
    lt = torch.log2(torch.from_numpy(v)).numpy()
    lc = np.log2(v.astype(np.float64)).astype(np.float32)
    d = (np.floor(lt) != np.floor(lc)) | (np.ceil(lt) != np.ceil(lc))
    if d.any():
        idx = np.nonzero(d)[0]
        bad += idx.size
        print("mismatch", v[idx[:5]], lt[idx[:5]], lc[idx[:5]])
print(f"checked {int(hi) - int(lo) + 1} values in {time.time() - t0:.0f} s, floor/ceil mismatches: {bad}")
sys.exit(1 if bad else 0)
