"""A/B of the native host-copy pool's copy routine on the C3 staging shapes (256 x 45,662 fp32): gather of
the tensors into one bucket and scatter back into fresh tensors. Run once per build of host_copy.cpp, the
library picked by ADFL_HOST_LIB (tools/hc_memcpy.so = plain memcpy, tools/hc_stream.so = streaming stores):

    g++ -O3 -fPIC -shared -Iinclude -o tools/hc_stream.so ad-federatedlearning_amd/csrc/host_copy.cpp -lpthread
    ADFL_HOST_LIB=tools/hc_stream.so python tools/hostcopy_ab.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ad-federatedlearning_amd"))
from adfl_amd import hostcopy  # noqa: E402

n = 45662
srcs = [torch.randn(n) for _ in range(256)]
pinned = len(sys.argv) > 1 and sys.argv[1] == "pinned"
buf = torch.empty(256 * n, pin_memory=pinned)
offs = [i * n for i in range(256)]
g, s = [], []
for k in range(22):
    t0 = time.perf_counter()
    hostcopy.gather(srcs, buf, offs)
    t1 = time.perf_counter()
    outs = [torch.empty(n) for _ in range(256)]
    t2 = time.perf_counter()
    hostcopy.scatter(buf, outs, offs)
    t3 = time.perf_counter()
    if k >= 2:
        g.append(t1 - t0)
        s.append(t3 - t2)
assert all(torch.equal(a, b) for a, b in zip(outs, srcs))
g.sort()
s.sort()
print(f"{os.path.basename(os.environ.get('ADFL_HOST_LIB', 'libadfl_slq.so'))} {'pinned' if pinned else 'pageable'} bucket: "
      f"gather best {1e3 * g[0]:.3f} med {1e3 * g[len(g) // 2]:.3f} ms, "
      f"scatter (fresh outputs) best {1e3 * s[0]:.3f} med {1e3 * s[len(s) // 2]:.3f} ms, threads {hostcopy.threads()}")
