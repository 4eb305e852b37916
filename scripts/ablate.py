"""Timing diagnostics: kernel time of the fast sweep with sections skipped
(BOTE_ABLATE bit mask, see FastArgs::ablate).  Results are wrong when a bit is
set; only the times matter.  Needs a library built with -DBOTE_ABLATION
(scripts/build_variant.sh abl -DBOTE_ABLATION; BOTE_LIB_PATH=fantoch_amd/lib_abl/...):
the product library has no ablation switches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch  # noqa: F401  (one HIP runtime)

from fantoch_amd.bote import DEFAULT_OBJECTIVES, DEFAULT_RANKING, DevicePlanet, Sweep
from fantoch_amd.planet import Planet

R, n = int(os.environ.get("R", "64")), int(os.environ.get("N", "7"))
p = Planet.synthetic(R)
dp = DevicePlanet(p)
srv = np.arange(R, dtype=np.uint32)
for mask in [int(x, 0) for x in sys.argv[1:]] or [0, 1, 2, 4, 8, 16, 31]:
    os.environ["BOTE_ABLATE"] = str(mask)
    sw = Sweep(dp, srv, srv, n, DEFAULT_OBJECTIVES, K=100, ranking=DEFAULT_RANKING, digest=True)
    sw.launch()
    sw.result()
    sw.timing_reset()
    for _ in range(3):
        sw.launch()
    ms, k = sw.timing()
    print(f"ablate={mask:3d}  kernel {ms / k:8.2f} ms  fast={sw.is_fast()}", flush=True)
