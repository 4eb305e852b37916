"""`python -m fantoch_amd` — the reference's bote binary, and flags for the
search the reference hard-codes.

With no arguments it does what `fantoch_bote/src/main.rs:4-85` does: the
distance table of the 13 regions (`distance_table`, main.rs:9-30, through
`Planet::distance_matrix`, planet/mod.rs:144-177), then `Search::new(3, 13,
R13C13, save_search = true)`, `sorted_evolving_configs` under
`RankingParams::new(110, 35, 0, 15, 3, 13, F1F2)` and, for the best chain,
`score: {:?}` and one `Search::stats_fmt` line per configuration
(main.rs:32-85).  Everything is computed by the gfx950 kernels
(libbote_hip.so); there is no CPU path.

The reference has no CLI (parameters are hard-coded in
main.rs:31-60).  Subcommands expose them, and the sweep the hot path serves:

  python -m fantoch_amd [main] [--lat-dir D] [--input R13C13] [--min-n 3] [--max-n 13]
                        [--ranking 110,35,0,15] [--ft-metric F1F2] [--chains 1] [--no-save-search]
  python -m fantoch_amd distance-table [--lat-dir D] [--regions a,b,...]
  python -m fantoch_amd stats --config a,b,c [--clients ...] [--tempo] [--lat-dir D]
  python -m fantoch_amd sweep (--synthetic R [--seed S] | --lat-dir D) --n N [--K 100]
                        [--objectives default|config5|mean:af1,cov:af1,score,...]
                        [--keys base|tempo-all-leaders] [--gpus G] [--rank-begin B --rank-end E]
"""
from __future__ import annotations

import argparse
import json
import sys
from decimal import Decimal
from typing import List, Optional, Sequence

# main.rs:12-25
REGIONS13 = ("asia-southeast1", "europe-west4", "southamerica-east1", "australia-southeast1", "europe-west2",
             "asia-south1", "us-east1", "asia-northeast1", "europe-west1", "asia-east1", "us-west1", "europe-west3",
             "us-central1")


def rust_f64(x: float) -> str:
    """Rust's `{}` / `{:?}` of an f64 (float.rs:97-101 Debug = Display): the
    shortest round-trip digits, never in exponent form, integral values with
    no fractional part ("10360" for 10360.0, "-0" for -0.0)."""
    if x != x:
        return "NaN"
    if x in (float("inf"), float("-inf")):
        return "inf" if x > 0 else "-inf"
    s = format(Decimal(repr(float(x))), "f")
    if "." in s:
        s = s.rstrip("0").rstrip(".")
    return s


def _planet(args):
    from .planet import Planet

    if getattr(args, "synthetic", None):
        return Planet.synthetic(args.synthetic, args.seed)
    return Planet.from_dir(args.lat_dir) if args.lat_dir else Planet.new()


def distance_table(planet, regions: Sequence[str]) -> str:
    """main.rs:9-30: `if let Ok(matrix) = planet.distance_matrix(regions) { println!("{}", matrix) }`."""
    from .planet import Region

    return planet.distance_matrix([Region(r) for r in regions])


def best_chains(args, out=sys.stdout) -> int:
    """main.rs:32-85 (the search, then the best chain's score and stats).
    main.rs takes the best chain with `.next().unwrap()`, which panics (exit
    101) when no evolving chain exists: with no chain this prints an error to
    stderr and returns 101."""
    from .bote import FTMetric, RankingParams, Search, SearchInput

    planet = _planet(args)
    search = Search(args.min_n, args.max_n, SearchInput(args.input), save_search=args.save_search,
                    planet=planet, device=args.device)
    a, b, c, d = (int(x) for x in args.ranking.split(","))
    params = RankingParams.new(a, b, c, d, args.min_n, args.max_n, FTMetric[args.ft_metric])
    chains = search.sorted_evolving_configs(params, limit=args.chains)
    if not chains:
        print("error: no evolving config chain (main.rs:66-69 `.next().unwrap()` on None)", file=sys.stderr)
        return 101
    for score, css, _clients in chains[:args.chains]:
        print(f"score: {rust_f64(score.value())}", file=out)
        sorted_config: List = []
        for cs in css:
            for region in cs.config:
                if region not in sorted_config:
                    sorted_config.append(region)
            print(Search.stats_fmt(cs.stats, len(cs.config)), file=out)
        if args.show_order:  # (main.rs builds `sorted_config` but does not print it)
            print(f"sorted_config: {sorted_config!r}", file=out)
    return 0


def config_stats(args, out=sys.stdout) -> None:
    """`Search::compute_stats` (search.rs:262-319) of one config, printed as
    `Search::stats_fmt`, and Tempo's keys (config.rs:317-329) with --tempo."""
    from .bote import Bote, Search

    planet = _planet(args)
    bote = Bote.from_(planet, args.device)
    config = args.config.split(",")
    clients = args.clients.split(",") if args.clients else [r.name for r in planet.regions()]
    stats = Search.compute_stats(config, clients, bote, tempo=args.tempo)
    print(Search.stats_fmt(stats, len(config)), file=out)
    if args.tempo:
        for key in sorted(k for k in stats.map if k.startswith("t")):
            print(f"{key}={stats.map[key]!r}", file=out)


def _objectives(spec: str):
    from . import _lib
    from .bote import CONFIG5_OBJECTIVES, DEFAULT_OBJECTIVES

    if spec == "default":
        return list(DEFAULT_OBJECTIVES)
    if spec == "config5":
        return list(CONFIG5_OBJECTIVES)
    kinds = {"score": _lib.OBJ_SCORE, "mean": _lib.OBJ_MEAN, "cov": _lib.OBJ_COV}
    out = []
    for item in spec.split(","):
        if item == "score":
            out.append((_lib.OBJ_SCORE, 0))
            continue
        kind, slot = item.split(":")
        out.append((kinds[kind], _lib.SLOT_NAMES_X.index(slot)))
    return out


def sweep(args, out=sys.stdout) -> dict:
    """The exhaustive sweep of every n-subset (search.rs:199-319 + the ranking's
    compute_score, search.rs:421-472) streamed through the device top-K, sharded
    over --gpus devices (bote_search_*), as one JSON object: per objective the
    K best (key, colex rank, regions), the valid count and the digest."""
    import numpy as np

    from . import _lib
    from .bote import DEFAULT_RANKING, DevicePlanet, MultiDeviceSearch, Sweep

    planet = _planet(args)
    srv = np.arange(planet.R, dtype=np.uint32)
    objs = _objectives(args.objectives)
    keys = _lib.KEYS_TEMPO_ALL_LEADERS if args.keys == "tempo-all-leaders" else _lib.KEYS_BASE
    total = _lib.binomial(planet.R, args.n)
    rb = args.rank_begin or 0
    re = total if args.rank_end is None else args.rank_end
    if args.gpus > 1:
        dps = [DevicePlanet(planet, d) for d in range(args.gpus)]
        h = MultiDeviceSearch(dps, srv, srv, args.n, objectives=objs, K=args.K, ranking=DEFAULT_RANKING,
                              rank_begin=rb, rank_end=re, keys=keys)
        h.launch()
        res = h.result()
    else:
        sw = Sweep(DevicePlanet(planet, args.device), srv, srv, args.n, objs, K=args.K, ranking=DEFAULT_RANKING,
                   digest=True, keys=keys)
        sw.launch(rb, re)
        res = sw.result()

    def regions(rank):
        return [planet.names[i] for i in _lib.colex_unrank(int(rank), args.n, planet.R)]

    names = {_lib.OBJ_SCORE: "score", _lib.OBJ_MEAN: "mean", _lib.OBJ_COV: "cov"}
    doc = {"regions": planet.R, "n": args.n, "rank_begin": rb, "rank_end": re, "configs": re - rb,
           "keys": args.keys, "gpus": args.gpus, "valid": res.valid, "digest": str(res.digest),
           "objectives": [{"objective": names[k] + ("" if k == _lib.OBJ_SCORE else ":" + _lib.SLOT_NAMES_X[s]),
                           "top": [{"key": str(key), "rank": rank, "regions": regions(rank)}
                                   for key, rank in res.tops[o][:args.show]]}
                          for o, (k, s) in enumerate(objs)]}
    print(json.dumps(doc, indent=None if args.compact else 1), file=out)
    return doc


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="python -m fantoch_amd", description=__doc__.split("\n\n")[0], allow_abbrev=False)
    sub = ap.add_subparsers(dest="cmd")

    def planet_flags(p, synthetic=False):
        p.add_argument("--lat-dir", default=None, help="a directory of ping .dat files (default: latency_gcp)")
        if synthetic:
            p.add_argument("--synthetic", type=int, default=None, metavar="R", help="synthetic R-region planet")
            p.add_argument("--seed", type=int, default=None)
        p.add_argument("--device", type=int, default=0)

    def main_flags(p):
        planet_flags(p)
        p.add_argument("--input", default="R13C13", choices=["R13C13", "R17C17", "R20C20", "R17CMaxN"])
        p.add_argument("--min-n", type=int, default=3)
        p.add_argument("--max-n", type=int, default=13)
        p.add_argument("--ranking", default="110,35,0,15",
                       help="min_mean_fpaxos_improv,min_mean_epaxos_improv,min_fairness_fpaxos_improv,"
                            "min_mean_decrease")
        p.add_argument("--ft-metric", default="F1F2", choices=["F1", "F1F2"])
        p.add_argument("--chains", type=int, default=1, help="best chains to print (main.rs: 1)")
        p.add_argument("--no-save-search", dest="save_search", action="store_false",
                       help="do not write {min}_{max}_{input}.data (main.rs saves it)")
        p.add_argument("--no-distance-table", dest="distance_table", action="store_false")
        p.add_argument("--show-order", action="store_true", help="also print the chain's sorted_config")

    main_flags(ap)
    main_flags(sub.add_parser("main", allow_abbrev=False, help="main.rs: distance table + best evolving chain"))
    p = sub.add_parser("distance-table", allow_abbrev=False, help="Planet::distance_matrix of the given regions")
    planet_flags(p)
    p.add_argument("--regions", default=",".join(REGIONS13))
    p = sub.add_parser("stats", allow_abbrev=False, help="Search::compute_stats of one config (stats_fmt)")
    planet_flags(p, synthetic=True)
    p.add_argument("--config", required=True, help="comma-separated region names")
    p.add_argument("--clients", default=None, help="comma-separated region names (default: every region)")
    p.add_argument("--tempo", action="store_true", help="also Tempo's fast/tiny/write keys")
    p = sub.add_parser("sweep", allow_abbrev=False, help="exhaustive n-subset sweep with the device top-K")
    planet_flags(p, synthetic=True)
    p.add_argument("--n", type=int, required=True)
    p.add_argument("--K", type=int, default=100)
    p.add_argument("--show", type=int, default=10, help="records printed per objective")
    p.add_argument("--objectives", default="default")
    p.add_argument("--keys", default="base", choices=["base", "tempo-all-leaders"])
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--rank-begin", type=int, default=None)
    p.add_argument("--rank-end", type=int, default=None)
    p.add_argument("--compact", action="store_true")
    return ap


def main(argv: Optional[Sequence[str]] = None, out=sys.stdout) -> int:
    args = build_parser().parse_args(argv)
    cmd = args.cmd or "main"
    if cmd == "main":
        if args.distance_table:
            print(distance_table(_planet(args), REGIONS13), file=out)
        return best_chains(args, out)
    elif cmd == "distance-table":
        print(distance_table(_planet(args), args.regions.split(",")), file=out)
    elif cmd == "stats":
        config_stats(args, out)
    elif cmd == "sweep":
        sweep(args, out)
    return 0
