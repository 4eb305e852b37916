"""Timing diagnostics: kernel time of one shard of a P-way cost split of the
R=64 n=7 sweep, with sections switched off (BOTE_ABLATE mask, a library built
with -DBOTE_ABLATION; results are wrong when a bit is set).  Separates the
per-launch cost that does not shrink with the shard (the strong-scaling bound)
from the per-config work.

  BOTE_LIB_PATH=fantoch_amd/lib_abl/libbote_hip.so python scripts/shard_ablate.py 0 4
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch  # noqa: F401  (one HIP runtime)

from fantoch_amd.bote import DEFAULT_OBJECTIVES, DEFAULT_RANKING, DevicePlanet, Sweep
from fantoch_amd.planet import Planet

p = Planet.synthetic(64)
dp = DevicePlanet(p)
srv = np.arange(64, dtype=np.uint32)
for mask in [int(x, 0) for x in sys.argv[1:]] or [0, 4]:
    os.environ["BOTE_ABLATE"] = str(mask)
    sw = Sweep(dp, srv, srv, 7, DEFAULT_OBJECTIVES, K=100, ranking=DEFAULT_RANKING, digest=True)
    row = []
    for parts in (1, 2, 4, 8, 64):
        b = sw.split(0, sw.total, parts)
        i = parts // 2
        sw.launch(b[i], b[i + 1])
        sw.result()
        sw.timing_reset()
        for _ in range(3):
            sw.launch(b[i], b[i + 1])
        sw.result()
        ms, k = sw.timing()
        row.append(f"1/{parts}: {ms / k:7.3f} ms")
    print(f"ablate={mask:5d}  " + "  ".join(row), flush=True)
