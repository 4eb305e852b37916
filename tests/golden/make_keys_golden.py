"""Generate the oracle fixtures of the extended key set (BASELINE config 5:
"Tempo f=1,2 + FPaxos all leaders"; include/bote_hip.h
BOTE_KEYS_TEMPO_ALL_LEADERS) and the random R=128 n=6 windows, from the CPU
oracle (oracle/bote_oracle.cpp compute_stats_x, checked against the oracle's
reference-pinned single calls by tests/test_keys_oracle.py).

  python tests/golden/make_keys_golden.py [--threads T] [topk|windows|edges|around|around_base|all]

Writes:
  topk_x.json   every GCP R20C20 config of n = 2..13 and the synthetic
                sub-ranges of topk.json, swept with the extended key set:
                valid count, digest and top-K (K=32) of the config-5
                objectives (bote.CONFIG5_OBJECTIVES; n < 4: tw1 for tw2)
  syn_r128n6_windows.json  nine 10^6-rank windows, eight of them straddling
                a colex boundary C(m, 6) where every member changes (base key
                set: the 10 compute_stats keys, DEFAULT_OBJECTIVES, K=100);
                256 windows at seeded random offsets of [0, C(128, 6)),
                "random": true -- the first 64 draws of 10^5 ranks, each swept
                with the base key set and with the extended one
                (CONFIG5_OBJECTIVES, under "x"), the other 192 of 2.5 10^4
                ranks with the extended key set only ("x_only": true)
  syn_r128n6_edges.json  (round 6) a window of 10^4 ranks centred on EVERY
                colex boundary C(m, 6), m = 6..127, where the largest member
                changes from m - 1 to m and a new run of groups begins: each
                swept with the base key set (DEFAULT_OBJECTIVES) and with the
                extended one (CONFIG5_OBJECTIVES), K=32
  syn_r128n6_around_pin.json  (round 6) a window of 2 x 2,048 ranks around
                every record of the full-size regression pin
                (syn_r128n6_pin.json: 8 objectives x 100), overlapping ones
                merged, swept with the extended key set (CONFIG5_OBJECTIVES,
                K=100): the oracle's view of the pin's records and of their
                colex neighbours
  syn_r128n6_base_around_pin.json  (round 6) the same around the 10-key
                pin (syn_r128n6_base_pin.json: DEFAULT_OBJECTIVES, 5 x 100)
Resumable: finished windows are kept in oracle/build/keys_windows.jsonl
(edges: oracle/build/keys_edges.jsonl; around: keys_around.jsonl).

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
N_WINDOWS, WIN = 64, 100_000  # random windows with both key sets
N_WINDOWS_X, WIN_X = 192, 25_000  # more random windows, extended key set only
BOUNDARY = (0, 3338380, 49563860, 300000200, 1191552400, 2141351635, 3652245460, 5168879425, 5422611200)
WIN_B = 1_000_000
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


def window_begins(x_only=False):
    """The first N_WINDOWS draws (both key sets), or the next N_WINDOWS_X (the
    extended key set only), of one seeded stream."""
    total = comb(128, 6)
    rng = np.random.default_rng(SEED)
    b = [int(x) for x in rng.integers(0, total - WIN, size=N_WINDOWS + N_WINDOWS_X)]
    return sorted(b[N_WINDOWS:]) if x_only else sorted(b[:N_WINDOWS])


def make_windows(threads):
    p = Planet.synthetic(128)
    scratch = os.path.join(ROOT, "oracle", "build", "keys_windows.jsonl")
    os.makedirs(os.path.dirname(scratch), exist_ok=True)
    done = {}
    if os.path.exists(scratch):
        for line in open(scratch):
            w = json.loads(line)
            done[(w["rank_begin"], w.get("kind"))] = w
    jobs = [("boundary", b, WIN_B) for b in BOUNDARY] + [("random", b, WIN) for b in window_begins()] + \
           [("random_x", b, WIN_X) for b in window_begins(x_only=True)]
    for kind, b, win in jobs:
        if (b, kind) in done:
            continue
        t0 = time.time()
        w = dict(R=128, n=6, rank_begin=b, rank_end=b + win, K=100, kind=kind)
        if kind != "random_x":
            base = sweep_case(p, 6, b, b + win, DEFAULT_OBJECTIVES, 100, 0, threads)
            w.update(objectives=[list(o) for o in DEFAULT_OBJECTIVES], ranking=list(RP), ft_metric=2, **base)
        if kind != "boundary":
            x = sweep_case(p, 6, b, b + win, objectives_x(6), 100, 1, threads)
            w["random"] = True
            w["valid"] = x.pop("valid")
            w["x"] = dict(keys=1, objectives=[list(o) for o in objectives_x(6)], ranking=list(RP), ft_metric=2, **x)
        if kind == "random_x":
            w["x_only"] = True
        w.update(cpu_seconds_wall=round(time.time() - t0, 1), threads=threads)
        with open(scratch, "a") as fh:
            fh.write(json.dumps(w) + "\n")
        done[(b, kind)] = w
        print("window", kind, b, len(done), "/", len(jobs), round(time.time() - t0, 1), "s", flush=True)
    path = os.path.join(HERE, "syn_r128n6_windows.json")
    d = {"what": ("oracle sweeps of windows of the synthetic R=128 planet, n=6: nine 10^6-rank windows (eight "
                  "straddling a colex boundary C(m, 6)), 64 10^5-rank windows at seeded random offsets "
                  "(\"random\": true, also swept with the extended key set under \"x\") and 192 2.5 10^4-rank "
                  "windows at further seeded random offsets swept with the extended key set only "
                  "(\"x_only\": true)"),
         "generator": "tests/golden/make_keys_golden.py windows",
         "windows": [done[(b, k)] for k, b, _ in jobs]}
    json.dump(d, open(path, "w"))


WIN_E, K_E = 10_000, 32  # the edge windows: ranks per window, top-K


def edge_windows():
    """[C(m, 6) - WIN_E / 2, C(m, 6) + WIN_E / 2) clipped to the rank space, m = 6..127."""
    total = comb(128, 6)
    return [(m, max(0, comb(m, 6) - WIN_E // 2), min(total, comb(m, 6) + WIN_E // 2)) for m in range(6, 128)]


def make_edges(threads):
    p = Planet.synthetic(128)
    scratch = os.path.join(ROOT, "oracle", "build", "keys_edges.jsonl")
    os.makedirs(os.path.dirname(scratch), exist_ok=True)
    done = {}
    if os.path.exists(scratch):
        for line in open(scratch):
            w = json.loads(line)
            done[w["m"]] = w
    jobs = edge_windows()
    for m, b, e in jobs:
        if m in done:
            continue
        t0 = time.time()
        base = sweep_case(p, 6, b, e, DEFAULT_OBJECTIVES, K_E, 0, threads)
        x = sweep_case(p, 6, b, e, objectives_x(6), K_E, 1, threads)
        w = dict(m=m, boundary=comb(m, 6), R=128, n=6, rank_begin=b, rank_end=e, K=K_E,
                 objectives=[list(o) for o in DEFAULT_OBJECTIVES], ranking=list(RP), ft_metric=2, **base,
                 x=dict(keys=1, objectives=[list(o) for o in objectives_x(6)], **x))
        w.update(cpu_seconds_wall=round(time.time() - t0, 1), threads=threads)
        with open(scratch, "a") as fh:
            fh.write(json.dumps(w) + "\n")
        done[m] = w
        print("edge", m, b, e, len(done), "/", len(jobs), round(time.time() - t0, 1), "s", flush=True)
    d = {"what": ("oracle sweeps of 10^4-rank windows of the synthetic R=128 planet, n=6, one centred on every "
                  "colex boundary C(m, 6), m = 6..127 (the largest member changes from m - 1 to m), with the "
                  "base key set (DEFAULT_OBJECTIVES) and the extended key set (CONFIG5_OBJECTIVES, under \"x\"), "
                  "K=%d, RankingParams(110,35,0,15,F1F2)" % K_E),
         "generator": "tests/golden/make_keys_golden.py edges",
         "windows": [done[m] for m, _, _ in jobs]}
    json.dump(d, open(os.path.join(HERE, "syn_r128n6_edges.json"), "w"))


A_P = 2_048  # the windows around the pin's records: ranks on each side
KEEP_A = 8  # records kept per window list at least


def around_windows(pin_name="syn_r128n6_pin.json"):
    """[rank - A_P, rank + A_P) around every record of a pin (syn_r128n6_pin.json:
    8 objectives x 100), clipped to the rank space, overlapping ones merged."""
    pin = json.load(open(os.path.join(HERE, pin_name)))
    total = comb(128, 6)
    iv = sorted((max(0, r - A_P), min(total, r + A_P)) for t in pin["tops"] for _, r in t)
    out = []
    for b, e in iv:
        if out and b <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([b, e])
    return [tuple(x) for x in out]


def make_around(threads, base=False):
    """base: the 10-key pin (syn_r128n6_base_pin.json), DEFAULT_OBJECTIVES."""
    pin_name = "syn_r128n6_base_pin.json" if base else "syn_r128n6_pin.json"
    objs, keys = (DEFAULT_OBJECTIVES, 0) if base else (objectives_x(6), 1)
    p = Planet.synthetic(128)
    scratch = os.path.join(ROOT, "oracle", "build", "keys_around_base.jsonl" if base else "keys_around.jsonl")
    os.makedirs(os.path.dirname(scratch), exist_ok=True)
    done = {}
    if os.path.exists(scratch):
        for line in open(scratch):
            w = json.loads(line)
            done[(w["rank_begin"], w["rank_end"])] = w
    jobs = around_windows(pin_name)
    t_all = time.time()
    for b, e in jobs:
        if (b, e) in done:
            continue
        x = sweep_case(p, 6, b, e, objs, 100, keys, threads)
        w = dict(rank_begin=b, rank_end=e, **x)
        with open(scratch, "a") as fh:
            fh.write(json.dumps(w) + "\n")
        done[(b, e)] = w
        if len(done) % 50 == 0:
            print("around", len(done), "/", len(jobs), round(time.time() - t_all, 1), "s", flush=True)
    # each window's lists are kept up to one record past the pin's K-th
    # (key, rank) of the objective, and at least KEEP_A records: every window
    # config at or below that record is kept, and the rest of a K=100 list is
    # prefix-checked on the GPU
    pin = json.load(open(os.path.join(HERE, pin_name)))
    kth = [(int(t[-1][0]), t[-1][1]) for t in pin["tops"]]
    wins = []
    for b, e in jobs:
        w = dict(done[(b, e)])
        tops, full = [], []
        for o, t in enumerate(w["tops"]):
            below = sum(1 for k, r in t if (int(k), r) <= kth[o])
            full.append(below == len(t) == 100)  # (a K=100 list entirely at or below the K-th: more may exist)
            tops.append(t[:max(KEEP_A, below + 1)])
        w["tops"], w["full_below_kth"] = tops, full
        wins.append(w)
    d = {"what": ("oracle sweeps (%s, K=100, RankingParams(110,35,0,15,F1F2)) of "
                  "the synthetic R=128 planet, n=6, over a window of %d ranks on each side of every record of "
                  "%s (%d objectives x 100 records; overlapping windows merged): the pin's "
                  "records and their colex neighbours, where their closest competitors are.  Each objective's "
                  "K=100 list is kept up to one record past the pin's 100th (key, rank) and at least %d records "
                  "(a prefix of the oracle's list)" % (
                      "the 10 compute_stats keys, DEFAULT_OBJECTIVES" if base else
                      "extended key set, CONFIG5_OBJECTIVES", A_P, pin_name, len(objs), KEEP_A)),
         "generator": "tests/golden/make_keys_golden.py " + ("around_base" if base else "around"),
         "R": 128, "n": 6, "keys": keys, "K": 100, "objectives": [list(o) for o in objs], "pin": pin_name,
         "windows": wins}
    json.dump(d, open(os.path.join(HERE, "syn_r128n6_base_around_pin.json" if base else "syn_r128n6_around_pin.json"),
                      "w"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="?", default="all", choices=["topk", "windows", "edges", "around", "around_base",
                                                                 "all"])
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    if a.what in ("topk", "all"):
        make_topk(a.threads)
    if a.what in ("windows", "all"):
        make_windows(a.threads)
    if a.what in ("edges", "all"):
        make_edges(a.threads)
    if a.what in ("around", "all"):
        make_around(a.threads)
    if a.what in ("around_base", "all"):
        make_around(a.threads, base=True)


if __name__ == "__main__":
    main()
