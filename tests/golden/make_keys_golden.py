"""Generate the oracle fixtures of the extended key set (BASELINE config 5:
"Tempo f=1,2 + FPaxos all leaders"; include/bote_hip.h
BOTE_KEYS_TEMPO_ALL_LEADERS) and the random R=128 n=6 windows, from the CPU
oracle (oracle/bote_oracle.cpp compute_stats_x, checked against the oracle's
reference-pinned single calls by tests/test_keys_oracle.py).

  python tests/golden/make_keys_golden.py [--threads T] [topk|windows|all]

Writes:
  topk_x.json   every GCP R20C20 config of n = 2..13 and the synthetic
                sub-ranges of topk.json, swept with the extended key set:
                valid count, digest and top-K (K=32) of the config-5
                objectives (bote.CONFIG5_OBJECTIVES; n < 4: tw1 for tw2)
  syn_r128n6_windows.json  (appends) 64 windows of 10^5 ranks at seeded
                random offsets of [0, C(128, 6)), each swept with the base
                key set (the 10 compute_stats keys, DEFAULT_OBJECTIVES, K=100)
                and with the extended one (CONFIG5_OBJECTIVES): "random": true
Resumable: finished windows are kept in oracle/build/keys_windows.jsonl.

Data only: inputs and expected outputs.
"""
import argparse
import json
import os
import sys
import time
from math import comb

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402
from fantoch_amd import _lib  # noqa: E402
from fantoch_amd.bote import CONFIG5_OBJECTIVES, DEFAULT_OBJECTIVES  # noqa: E402
from fantoch_amd.planet import Planet  # noqa: E402

RP = (110.0, 35.0, 0.0, 15.0)
K_TOPK = 32
SYN = {"r64n7": (64, 7, 310_608_096, 60_000), "r128n6": (128, 6, 2_711_805_600, 40_000)}
N_WINDOWS, WIN = 64, 100_000
SEED = 0x5EED0128


def objectives_x(n):
    objs = list(CONFIG5_OBJECTIVES)
    if min(n // 2, 2) < 2:  # tw2 (f = 2) does not exist at n < 4
        objs[6] = (_lib.OBJ_MEAN, _lib.SLOT_TW1)
    return objs


def sweep_case(planet, n, rb, re, objs, K, keys, threads):
    op = O.OraclePlanet.of(planet)
    s = np.arange(planet.R, dtype=np.uint32)
    tops, valid, digest = op.sweep(s, s, n, rb, re, objs, K, RP, 2, threads, keys=keys)
    return {"valid": valid, "digest": str(digest), "tops": [[[str(k), r] for k, r in t] for t in tops]}


def make_topk(threads):
    gcp = Planet.new()
    out = {"_doc": "oracle top-K (key, colex rank) per objective with the extended key set "
                   "(BOTE_KEYS_TEMPO_ALL_LEADERS); objectives per case; RankingParams(110,35,0,15,F1F2); K=%d"
                   % K_TOPK, "K": K_TOPK, "keys": 1, "cases": {}}
    for n in range(2, 14):
        c = sweep_case(gcp, n, 0, comb(gcp.R, n), objectives_x(n), K_TOPK, 1, threads)
        out["cases"][f"gcp_n{n}"] = dict(R=gcp.R, n=n, rank_begin=0, rank_end=comb(gcp.R, n),
                                         objectives=[list(x) for x in objectives_x(n)], **c)
        print("topk_x gcp n", n, flush=True)
    for name, (R, n, rb, cnt) in SYN.items():
        c = sweep_case(Planet.synthetic(R), n, rb, rb + cnt, objectives_x(n), K_TOPK, 1, threads)
        out["cases"][f"syn_{name}"] = dict(R=R, n=n, rank_begin=rb, rank_end=rb + cnt,
                                           objectives=[list(x) for x in objectives_x(n)], **c)
        print("topk_x", name, flush=True)
    json.dump(out, open(os.path.join(HERE, "topk_x.json"), "w"), indent=0)


def window_begins():
    total = comb(128, 6)
    rng = np.random.default_rng(SEED)
    return sorted(int(x) for x in rng.integers(0, total - WIN, size=N_WINDOWS))


def make_windows(threads):
    p = Planet.synthetic(128)
    scratch = os.path.join(ROOT, "oracle", "build", "keys_windows.jsonl")
    os.makedirs(os.path.dirname(scratch), exist_ok=True)
    done = {}
    if os.path.exists(scratch):
        for line in open(scratch):
            w = json.loads(line)
            done[w["rank_begin"]] = w
    for b in window_begins():
        if b in done:
            continue
        t0 = time.time()
        base = sweep_case(p, 6, b, b + WIN, DEFAULT_OBJECTIVES, 100, 0, threads)
        x = sweep_case(p, 6, b, b + WIN, objectives_x(6), 100, 1, threads)
        w = dict(R=128, n=6, rank_begin=b, rank_end=b + WIN, K=100, random=True,
                 objectives=[list(o) for o in DEFAULT_OBJECTIVES], ranking=list(RP), ft_metric=2, **base,
                 x=dict(keys=1, objectives=[list(o) for o in objectives_x(6)], **x),
                 cpu_seconds_wall=round(time.time() - t0, 1), threads=threads)
        with open(scratch, "a") as fh:
            fh.write(json.dumps(w) + "\n")
        done[b] = w
        print("window", b, len(done), "/", N_WINDOWS, round(time.time() - t0, 1), "s", flush=True)
    path = os.path.join(HERE, "syn_r128n6_windows.json")
    d = json.load(open(path))
    keep = [w for w in d["windows"] if not w.get("random")]
    d["windows"] = keep + [done[b] for b in window_begins()]
    d["what"] = ("oracle sweeps of windows of the synthetic R=128 planet, n=6: nine 10^6-rank windows (eight "
                 "straddling a colex boundary C(m, 6)) and 64 10^5-rank windows at seeded random offsets "
                 "(\"random\": true, also swept with the extended key set under \"x\")")
    d["generator"] = "scripts/oracle_fixtures.sh; tests/golden/make_keys_golden.py (random windows)"
    json.dump(d, open(path, "w"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="?", default="all", choices=["topk", "windows", "all", "refresh_x"])
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    if a.what in ("topk", "all"):
        make_topk(a.threads)
    if a.what in ("windows", "all"):
        make_windows(a.threads)
    if a.what == "refresh_x":
        make_topk(a.threads)
        refresh_x(a.threads)



def refresh_x(threads):
    """Recompute the extended-key part of every fixture with the current
    oracle and rewrite the entries that differ (used once after the digest's
    definition changed while a generation was running)."""
    p = Planet.synthetic(128)
    path = os.path.join(HERE, "syn_r128n6_windows.json")
    d = json.load(open(path))
    changed = 0
    for w in d["windows"]:
        if "x" not in w:
            continue
        b, e = w["rank_begin"], w["rank_end"]
        x = sweep_case(p, 6, b, e, objectives_x(6), 100, 1, threads)
        if (x["valid"], x["digest"], x["tops"]) != (w["valid"], w["x"]["digest"], w["x"]["tops"]):
            w["x"].update(digest=x["digest"], tops=x["tops"])
            changed += 1
        print("window", b, "x", "changed" if changed else "same", flush=True)
    json.dump(d, open(path, "w"))
    print("windows refreshed:", changed)


if __name__ == "__main__":
    main()
