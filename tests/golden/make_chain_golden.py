"""TEST INFRASTRUCTURE — golden chains of Search::sorted_evolving_configs
(search.rs:97-178) from the CPU oracle (oracle/bote_oracle.cpp,
oracle_search_chains), for the device chain search (bote_evolving_chains).

  python tests/golden/make_chain_golden.py   ->  tests/golden/chains.json

Cases: R13C13, R17C17, R20C20 (one client set each) and a sample of
R17CMaxN's client sets (every 20th of C(17, 13) = 2,380), at the reference's
test params (110, 35, 0, 15), at its original min_mean_fpaxos_improv = 30
(search.rs:684-686), and at two lenient sets (10, 5, 0, 5) and (0, 0, 0, 0)
that yield 10^3..10^7 chains (R20C20 only at the first two: the oracle's
nested loops cannot enumerate its lenient chain sets), FTMetric::F1F2.  Per
case: the total chain count, the first K chains (score, region names per
level) and an order-dependent digest of ALL chains.
"""
import itertools
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402
from fantoch_amd.bote import SearchInput  # noqa: E402
from fantoch_amd.planet import Planet  # noqa: E402

PARAMS = [(110.0, 35.0, 0.0, 15.0), (30.0, 35.0, 0.0, 15.0), (10.0, 5.0, 0.0, 5.0), (0.0, 0.0, 0.0, 0.0)]
K = 50
MAXN_EVERY = 20


def main():
    p = Planet.new()
    o = O.OraclePlanet.of(p)
    out = {"_doc": __doc__.strip().splitlines()[0], "K": K, "params": PARAMS, "cases": {}}
    for si in (SearchInput.R13C13, SearchInput.R17C17, SearchInput.R20C20):
        srv, clis = si.get_inputs(13, p)
        s, c = p.idxs(srv), p.idxs(clis[0])
        for pi, rp in enumerate(PARAMS):
            if si is SearchInput.R20C20 and pi >= 2:
                continue
            chains, n, dig = o.search_chains(s, c, rp, 2, K)
            out["cases"][f"{si}_{pi}"] = {"input": str(si), "params": list(rp), "nchains": n, "digest": str(dig),
                                          "chains": [[sc, [[p.names[r] for r in st] for st in sets]]
                                                     for sc, sets in chains]}
            print(si, rp, n, flush=True)
    # R17CMaxN: every client set is its own server list (search.rs:599-606)
    _, sets = SearchInput.R17CMaxN.get_inputs(13, p)
    for pi, rp in enumerate(PARAMS[:3]):
        per = []
        for ci in range(0, len(sets), MAXN_EVERY):
            ids = p.idxs(sets[ci])
            chains, n, dig = o.search_chains(ids, ids, rp, 2, 5)
            per.append({"set": ci, "nchains": n, "digest": str(dig),
                        "chains": [[sc, [[p.names[r] for r in st] for st in ss]] for sc, ss in chains]})
        out["cases"][f"R17CMaxN_{pi}"] = {"input": "R17CMaxN", "params": list(rp), "sets": len(sets),
                                          "every": MAXN_EVERY, "per_set": per}
        print("R17CMaxN", rp, sum(x["nchains"] for x in per), flush=True)
    json.dump(out, open(os.path.join(HERE, "chains.json"), "w"))


if __name__ == "__main__":
    main()
