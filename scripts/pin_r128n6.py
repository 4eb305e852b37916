"""Regression pin of BASELINE config 5 as stated at full size (R=128 n=6, the
extended key set, CONFIG5_OBJECTIVES, K=100): the valid count, digest and the
8 objectives' top-K of all 5,423,611,200 configs.

The oracle cannot sweep 5.4e9 configs here (about 2 days on 16 CPUs), so the
pin is NOT an oracle fixture.  It is what the device computes, under two
checks made here:
  * the group kernel (the bench path) equals the exact generic kernel
    (every slot's and every leader's moments through the digest, the valid
    count, the top-K lists);
  * every reported record (8 x 100 configs) is re-derived by the oracle
    (compute_stats_x + compute_score on those configs: per objective the
    oracle's ordered list over the reported configs equals the device's).
bench.py --workload r128n6 checks its result against this pin and says so.

  python scripts/pin_r128n6.py OUT.json [--base]     (on a GPU box)

--base: the same for the 10 compute_stats keys and DEFAULT_OBJECTIVES
(bench.py --workload r128n6_base), pinned as syn_r128n6_base_pin.json.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402
from fantoch_amd import _lib  # noqa: E402
from fantoch_amd.bote import CONFIG5_OBJECTIVES, DEFAULT_OBJECTIVES, DEFAULT_RANKING, DevicePlanet, Sweep  # noqa: E402
from fantoch_amd.planet import Planet  # noqa: E402


def main():
    out_path = sys.argv[1]
    base = "--base" in sys.argv[2:]
    keys = 0 if base else _lib.KEYS_TEMPO_ALL_LEADERS
    objectives = DEFAULT_OBJECTIVES if base else CONFIG5_OBJECTIVES
    p = Planet.synthetic(128)
    dp = DevicePlanet(p)
    srv = np.arange(128, dtype=np.uint32)
    res = {}
    for k in ("group", "generic"):
        sw = Sweep(dp, srv, srv, 6, objectives, K=100, ranking=DEFAULT_RANKING, digest=True, kernel=k, keys=keys)
        assert sw.kernel_path() == k
        t0 = time.time()
        sw.launch(0, sw.total)
        r = sw.result()
        print(k, r.valid, r.digest, round(time.time() - t0, 2), "s", flush=True)
        res[k] = (r.valid, r.digest, [[(int(kk), int(rk)) for kk, rk in t] for t in r.tops])
        total = sw.total
    if res["group"] != res["generic"]:
        sys.exit("group kernel differs from the generic kernel: no pin")
    valid, digest, tops = res["group"]
    o = O.OraclePlanet.of(p)
    rp = (DEFAULT_RANKING.min_mean_fpaxos_improv, DEFAULT_RANKING.min_mean_epaxos_improv,
          DEFAULT_RANKING.min_fairness_fpaxos_improv, DEFAULT_RANKING.min_mean_decrease)
    for oi, obj in enumerate(objectives):
        recs = tops[oi]
        t, _, _ = o.sweep_ranks(srv, srv, 6, [rk for _, rk in recs], [obj], 100, rp, DEFAULT_RANKING.ft_metric.value,
                                threads=16, keys=1 if keys else 0)
        if [(int(k), int(rk)) for k, rk in t[0]] != recs:
            sys.exit(f"objective {oi}: the oracle's re-derivation differs: no pin")
    pin = {
        "what": ("regression pin of BASELINE config 5 at full size: synthetic R=128 planet (seed 0x5EED0128), n=6, "
                 "all 5,423,611,200 configs, " +
                 ("the 10 compute_stats keys, DEFAULT_OBJECTIVES" if base else
                  "extended key set (BOTE_KEYS_TEMPO_ALL_LEADERS), CONFIG5_OBJECTIVES") +
                 ", K=100, RankingParams(110,35,0,15,F1F2)"),
        "source": ("GPU, NOT the oracle: the group kernel equals the exact generic kernel at full size, and every "
                   "reported record was re-derived by the oracle (keys and order); generator scripts/pin_r128n6.py"),
        "R": 128, "n": 6, "rank_begin": 0, "rank_end": total, "keys": 0 if base else 1, "K": 100,
        "objectives": [list(x) for x in objectives],
        "valid": valid, "digest": str(digest), "tops": [[[str(k), rk] for k, rk in t] for t in tops],
    }
    os.makedirs(os.path.dirname(os.path.abspath(out_path)), exist_ok=True)
    json.dump(pin, open(out_path, "w"))
    print("pinned", valid, digest, "->", out_path)


if __name__ == "__main__":
    main()
