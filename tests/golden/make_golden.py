"""Generate the committed golden fixtures under tests/golden/ from the CPU
oracle (oracle/bote_oracle.cpp, itself pinned to the reference's own
known-answer tests in reference_goldens.json by tests/test_oracle.py).

  python tests/golden/make_golden.py [topk]     (topk: only topk.json)

Writes:
  planets.npz            parsed GCP, AWS 2020_06_05 and AWS 2021_02_13
                         matrices (u16, name order) + names (dat.rs:21-75,
                         planet/mod.rs:38-54)
  gcp_n3_n5_stats.npz    every GCP R20C20 config of n=3 and n=5 (colex rank
                         order): FPaxos leader position, per-slot exact sum and
                         sum of squares (10 slots, search.rs:262-319), score and
                         validity under RankingParams(110,35,0,15,F1F2)
                         (search.rs:421-472); full per-client latency vectors
                         for every 37th config
  topk.json              top-K (K=32) per objective for GCP n=3..13, AWS 2021
                         n=3,5, and colex sub-ranges of the synthetic R=64 n=7
                         and R=128 n=6 planets, with valid counts and digests

Data only: inputs and expected outputs.
"""
import json
import os
import sys
from math import comb

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402
from fantoch_amd.bote import DEFAULT_OBJECTIVES  # noqa: E402
from fantoch_amd.planet import AWS_2020_DIR, AWS_2021_DIR, Planet  # noqa: E402

RP = (110.0, 35.0, 0.0, 15.0)
TOPK_K = 32
SAMPLE_EVERY = 37
# colex sub-ranges of the synthetic planets (start, count)
SYN = {"r64n7": (64, 7, 310_608_096, 60_000), "r128n6": (128, 6, 2_711_805_600, 40_000)}


def moments(vals, n, nc):
    """per-slot (sum, sum of squares) from oracle per-client values."""
    ncfg = vals.shape[0]
    s1 = np.zeros((ncfg, 10), np.uint64)
    s2 = np.zeros((ncfg, 10), np.uint64)
    for slot in range(10):
        if slot < 5:
            v = vals[:, slot * nc:(slot + 1) * nc]
        else:
            v = vals[:, 5 * nc + (slot - 5) * n:5 * nc + (slot - 4) * n]
        if min(n // 2, 2) < 2 and slot % 5 in (2, 3):  # af2/ff2 do not exist (search.rs:474-477)
            s1[:, slot] = 0xFFFFFFFF
            s2[:, slot] = 0xFFFFFFFFFFFFFFFF
            continue
        s1[:, slot] = v.sum(axis=1)
        s2[:, slot] = (v * v).sum(axis=1)
    return s1, s2


def main():
    gcp = Planet.new()
    aws20 = Planet.from_dir(AWS_2020_DIR)
    aws21 = Planet.from_dir(AWS_2021_DIR)
    only_topk = sys.argv[1:] == ["topk"]
    if not only_topk:
        write_stats(gcp, aws20, aws21)
    write_topk(gcp, aws21)


def write_stats(gcp, aws20, aws21):
    np.savez_compressed(os.path.join(HERE, "planets.npz"),
                        gcp_lat=gcp.lat.astype(np.uint16), gcp_names=np.array(gcp.names),
                        aws20_lat=aws20.lat.astype(np.uint16), aws20_names=np.array(aws20.names),
                        aws21_lat=aws21.lat.astype(np.uint16), aws21_names=np.array(aws21.names))

    o = O.OraclePlanet.of(gcp)
    srv = np.arange(gcp.R, dtype=np.uint32)
    out = {}
    for n in (3, 5):
        cfg = np.array([O.colex_unrank(r, n, gcp.R) for r in range(comb(gcp.R, n))], dtype=np.uint32)
        vals, lead = o.compute_stats(cfg, srv)
        s1, s2 = moments(vals, n, gcp.R)
        sc, va = o.scores(cfg, srv, RP, 2)
        out[f"n{n}_leader"] = lead.astype(np.uint8)
        out[f"n{n}_s1"] = s1.astype(np.uint32)
        out[f"n{n}_s2"] = s2
        out[f"n{n}_score"] = sc
        out[f"n{n}_valid"] = va
        out[f"n{n}_sample_ranks"] = np.arange(0, len(cfg), SAMPLE_EVERY, dtype=np.uint64)
        out[f"n{n}_sample_vals"] = vals[::SAMPLE_EVERY].astype(np.uint16)
    np.savez_compressed(os.path.join(HERE, "gcp_n3_n5_stats.npz"), **out)


def write_topk(gcp, aws21):
    topk = {"_doc": "oracle top-K (key, colex rank) per objective; objectives = DEFAULT_OBJECTIVES "
                    "(kind, slot); RankingParams(110,35,0,15,F1F2); K=%d" % TOPK_K,
            "objectives": [list(x) for x in DEFAULT_OBJECTIVES], "K": TOPK_K, "cases": {}}

    def add(name, planet, n, rb, re):
        op = O.OraclePlanet.of(planet)
        s = np.arange(planet.R, dtype=np.uint32)
        tops, valid, digest = op.sweep(s, s, n, rb, re, DEFAULT_OBJECTIVES, TOPK_K, RP, 2, 8)
        topk["cases"][name] = {"R": planet.R, "n": n, "rank_begin": rb, "rank_end": re,
                               "valid": valid, "digest": str(digest),
                               "tops": [[[str(k), r] for k, r in t] for t in tops]}

    for n in range(3, 14):
        add(f"gcp_n{n}", gcp, n, 0, comb(gcp.R, n))
    for n in (3, 5):
        add(f"aws21_n{n}", aws21, n, 0, comb(aws21.R, n))
    for name, (R, n, rb, cnt) in SYN.items():
        add(f"syn_{name}", Planet.synthetic(R), n, rb, rb + cnt)
    json.dump(topk, open(os.path.join(HERE, "topk.json"), "w"), indent=0)
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
