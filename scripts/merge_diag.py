"""Diagnostics: one launch of the R=64 n=7 sweep over the full range and over
the middle 1/8 and 1/64 shards, with the merge's device printf build
(scripts/build_variant.sh mpr -DBOTE_MERGE_PRINTF): per objective the heads'
bound passes, head count and gathered records.

  BOTE_LIB_PATH=fantoch_amd/lib_mpr/libbote_hip.so python scripts/merge_diag.py
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
sw = Sweep(dp, srv, srv, 7, DEFAULT_OBJECTIVES, K=100, ranking=DEFAULT_RANKING, digest=True)
for parts in (1, 8, 64):
    b = sw.split(0, sw.total, parts)
    i = parts // 2
    print(f"--- 1/{parts}: [{b[i]}, {b[i + 1]})", flush=True)
    sw.launch(b[i], b[i + 1])
    r = sw.result()
    torch.cuda.synchronize()
    print(f"valid {r.valid}", flush=True)
