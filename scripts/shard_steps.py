"""Step structure of one rank's shard: the middle shard of a
P-way cost split of the R=64 n=7 sweep, launched back to back on one stream
as a bench rank's steps are (launch + result copy to pinned memory), for
P = 1, 2, 4, 8, 64.  Per shard: wall time per step, the sweep kernel's event
time, and the difference (the per-step work outside the kernel: zeroing,
sample launch, seed, fix-up, merge, copy).  Run under rocprofv3 --kernel-trace
for the per-dispatch table.

  python scripts/shard_steps.py [steps=20]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fantoch_amd.bote import DEFAULT_OBJECTIVES, DEFAULT_RANKING, DevicePlanet, Sweep
from fantoch_amd.planet import Planet

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
p = Planet.synthetic(64)
dp = DevicePlanet(p)
srv = np.arange(64, dtype=np.uint32)
sw = Sweep(dp, srv, srv, 7, DEFAULT_OBJECTIVES, K=100, ranking=DEFAULT_RANKING, digest=True)
stream = torch.cuda.current_stream().cuda_stream
host = torch.empty(sw.result_bytes(), dtype=torch.uint8, pin_memory=True)
rows = []
for parts in (1, 2, 4, 8, 64):
    b = sw.split(0, sw.total, parts)
    i = parts // 2
    rb, re = b[i], b[i + 1]
    for _ in range(3):
        sw.launch(rb, re, stream)
        sw.result_device(host.data_ptr(), stream)
    torch.cuda.synchronize()
    sw.timing_reset()
    t0 = time.perf_counter()
    for _ in range(steps):
        sw.launch(rb, re, stream)
        sw.result_device(host.data_ptr(), stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps * 1e3
    kms, n = sw.timing()
    row = {"parts": parts, "shard": [rb, re], "configs": re - rb, "step_ms": round(dt, 4),
           "kernel_ms": round(kms / n, 4), "outside_ms": round(dt - kms / n, 4)}
    rows.append(row)
    print(json.dumps(row), flush=True)
