"""How often each rare path of the group kernel runs for a whole wavefront
(any lane taking it), per 64-config wave-step, from the -DBOTE_PATHSTATS
library (diagnostics only; the counters cost instructions of their own):

  scripts/build_variant.sh pstats -DBOTE_PATHSTATS
  BOTE_LIB_PATH=fantoch_amd/lib_pstats/libbote_hip.so python scripts/pathstats.py [r64n7|r128n6|r128n6_base]

Counters (bote_group.hip PSTAT): 0 steps, 1 no client lines, 2 leader re-scan,
3 leader deferred, 4/5 f64 mean test f=1/2, 6 COV validity tests, 8 validity
deferred, 9 f64 score, 10 COV af1 key, 11 block top-K merge, 12 groups, 13 chunks."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NAMES = {0: "steps", 1: "no client lines", 2: "leader re-scan", 3: "leader deferred", 4: "f64 mean test f=1",
         5: "f64 mean test f=2", 6: "COV validity tests", 8: "validity deferred", 9: "f64 score",
         10: "COV af1 key", 11: "block top-K merge", 12: "groups", 13: "chunks"}


def main():
    import numpy as np

    from fantoch_amd import _lib
    from fantoch_amd.bote import CONFIG5_OBJECTIVES, DEFAULT_OBJECTIVES, DEFAULT_RANKING, DevicePlanet, Sweep
    from fantoch_amd.planet import Planet

    wl = sys.argv[1] if len(sys.argv) > 1 else "r64n7"
    R, n, keys = {"r64n7": (64, 7, 0), "r128n6": (128, 6, 1), "r128n6_base": (128, 6, 0)}[wl]
    p = Planet.synthetic(R)
    srv = np.arange(R, dtype=np.uint32)
    objs = CONFIG5_OBJECTIVES if keys else DEFAULT_OBJECTIVES
    sw = Sweep(DevicePlanet(p), srv, srv, n, objs, K=100, ranking=DEFAULT_RANKING, digest=True, keys=keys)
    f = _lib.lib().bote_sweep_pathstats
    f.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
    out = (C.c_uint64 * 64)()
    sw.launch()
    sw.result()
    _lib.check(f(sw.h, out))  # (the warm-up launch)
    sw.launch()
    r = sw.result()
    _lib.check(f(sw.h, out))
    steps = out[0]
    rep = {"workload": wl, "valid": r.valid, "digest": str(r.digest), "steps": steps,
           "per_step": {NAMES.get(k, str(k)): out[k] / steps for k in sorted(NAMES) if k},
           "raw": {NAMES.get(k, str(k)): out[k] for k in sorted(NAMES)}}
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
