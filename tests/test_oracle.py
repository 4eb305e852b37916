"""Pin the CPU oracle against the reference's own known-answer tests.

Every expected value comes from tests/golden/reference_goldens.json, transcribed
from the reference's unit tests (file:line in each entry).  CPU only.
"""
import json
import math
import os

import numpy as np
import pytest

import oracle as O
from fantoch_amd.planet import Planet, Region, dat_latencies, dat_region, GCP_LAT_DIR

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_goldens.json")))


@pytest.fixture(scope="module")
def gcp():
    p = Planet.new()
    return p, O.OraclePlanet.of(p)


def ids(p, names):
    return p.idxs(names)


# lib.rs:193-222
def test_quorum_latencies(gcp):
    p, o = gcp
    g = GOLD["quorum_latencies"]
    regs = ids(p, g["regions"])
    for q, key in ((2, "q2"), (3, "q3")):
        got = [o.quorum_latency(int(r), regs, q) for r in regs]
        assert got == g[key]


# lib.rs:224-324
def test_leaderless(gcp):
    p, o = gcp
    g = GOLD["leaderless"]
    servers = ids(p, g["servers"])
    for case in g["cases"]:
        v = o.leaderless(servers, ids(p, case["clients"]), case["q"])
        st = O.hist_stats(v)
        assert O.f64_round(st[0]) == case["mean"]
        assert O.f64_round(st[2]) == case["cov"]
        assert O.f64_round(st[3]) == case["mdtm"]


# lib.rs:326-444
def test_leader(gcp):
    p, o = gcp
    g = GOLD["leader"]
    servers = ids(p, g["servers"])
    for case in g["cases"]:
        v = o.leader(p.idx(case["leader"]), servers, ids(p, case["clients"]), g["q"])
        st = O.hist_stats(v)
        assert (O.f64_round(st[0]), O.f64_round(st[2]), O.f64_round(st[3])) == (
            case["mean"], case["cov"], case["mdtm"])


# lib.rs:446-465
def test_best_latency_leader(gcp):
    p, o = gcp
    g = GOLD["best_latency_leader"]
    servers = ids(p, g["servers"])
    pos = o.best_leader(servers, servers, g["q"], 0)
    v = o.leader(int(servers[pos]), servers, servers, g["q"])
    st = O.hist_stats(v)
    assert (O.f64_round(st[0]), O.f64_round(st[2]), O.f64_round(st[3])) == (g["mean"], g["cov"], g["mdtm"])


# protocol.rs:122-137
def test_quorum_size():
    proto = {"FPaxos": O.FPAXOS, "EPaxos": O.EPAXOS, "Atlas": O.ATLAS}
    for name, n, f, want in GOLD["quorum_size"]["cases"]:
        assert O.quorum_size(proto[name], n, f) == want


# histogram.rs:390-463
def test_histogram_stats():
    g = GOLD["histogram"]
    for c in g["stats"]:
        st = O.hist_stats(c["values"])
        for i, k in enumerate(["mean", "stddev", "cov", "mdtm", "min", "max"]):
            if k in c:
                assert st[i] == c[k], (c, k)
    for c in g["stats_show"]:
        st = O.hist_stats(c["values"])
        assert (O.f64_round(st[0]), O.f64_round(st[2]), O.f64_round(st[3])) == (c["mean"], c["cov"], c["mdtm"])
    for c in g["improv"]:
        a, b = O.hist_stats(c["a"]), O.hist_stats(c["b"])
        if "mean_improv" in c:
            assert a[0] - b[0] == c["mean_improv"]
        if "cov_improv" in c:
            assert a[2] - b[2] == c["cov_improv"]
        if "mdtm_improv" in c:
            assert a[3] - b[3] == c["mdtm_improv"]
    pc = g["percentile"]
    st = O.hist_stats(pc["values"])
    assert st[4] == pc["min"] and st[5] == pc["max"]
    for p_, want in pc["p"]:
        assert O.hist_percentile(pc["values"], p_) == want


# float.rs:168-177
def test_f64_order():
    nan = float("nan")
    assert O.f64_cmp(5.2, 5.3) == -1
    assert O.f64_cmp(5.3, 5.2) == 1
    assert O.f64_cmp(5.2, 5.2) == 0
    assert O.f64_cmp(5.2, nan) == -1
    assert O.f64_cmp(nan, 5.3) == 1
    assert O.f64_cmp(nan, nan) == 0


def test_count_one_histogram_cov_is_nan():
    st = O.hist_stats([7])
    assert math.isnan(st[1]) and math.isnan(st[2])


# planet/mod.rs:190-254
def test_planet_symmetry_and_sorted(gcp):
    p, o = gcp
    g = GOLD["planet"]
    for a, b in g["symmetric"]:
        assert p.ping_latency(a, b) == p.ping_latency(b, a)
    for a, b in g["asymmetric"]:
        assert p.ping_latency(a, b) != p.ping_latency(b, a)
    frm = p.idx(g["sorted_from"])
    assert [p.names[r] for _, r in o.sorted(frm)] == g["sorted"]
    # the product planet agrees with the oracle's (latency, name) order
    assert [r.name for _, r in p.sorted(g["sorted_from"])] == g["sorted"]


# dat.rs:115-154
def test_dat():
    g = GOLD["planet"]
    f = os.path.join(GCP_LAT_DIR, "europe-west3.dat")
    assert dat_region(f) == Region(g["dat_region"])
    assert {k.name: v for k, v in dat_latencies(f).items()} == g["dat_latencies"]


# planet/mod.rs:257-277
def test_equidistant():
    regions, p = Planet.equidistant(10, 3)
    assert len(regions) == 3
    for a in regions:
        for b in regions:
            assert p.ping_latency(a, b) == (0 if a == b else 10)


# search.rs:671-751 — the end-to-end golden.
def test_search_r13c13(gcp):
    p, o = gcp
    g = GOLD["search"]
    regs = ids(p, g["regions13"])
    score, sets, fmts, nchains = o.search_best(regs, regs, tuple(float(x) for x in g["params"]), 2)
    assert O.f64_round(score) == g["score"]
    assert nchains >= 1
    n5 = [f for s, f in zip(sets, fmts) if len(s) == 5]
    assert n5 and n5[0] == g["stats_fmt_n5"]
    sorted_config = []
    for s in sets:
        for r in s:
            if p.names[r] not in sorted_config:
                sorted_config.append(p.names[r])
    assert sorted_config == g["sorted_config"]


def test_colex_unrank_roundtrip():
    from math import comb
    n, ns = 4, 9
    seen = set()
    for r in range(comb(ns, n)):
        c = O.colex_unrank(r, n, ns)
        assert c == sorted(c) and len(set(c)) == n and max(c) < ns
        assert sum(comb(x, j + 1) for j, x in enumerate(c)) == r
        seen.add(tuple(c))
    assert len(seen) == comb(ns, n)


def test_leaderless_batch_equals_single_calls():
    """oracle_leaderless_batch (the Tempo parity checker) is Bote::leaderless
    per config and quorum size (lib.rs:38-59)."""
    from fantoch_amd.planet import Planet
    p = Planet.new()
    o = O.OraclePlanet.of(p)
    rng = np.random.default_rng(3)
    cfgs = np.array([rng.choice(p.R, 7, replace=False) for _ in range(20)], dtype=np.uint32)
    cli = rng.choice(p.R, 9, replace=True)
    qs = [2, 3, 4, 5]
    got = o.leaderless_batch(cfgs, cli, qs, threads=2)
    for i, cfg in enumerate(cfgs):
        for qi, q in enumerate(qs):
            assert got[i, qi, :9].tolist() == o.leaderless(cfg, cli, q).tolist()
            assert got[i, qi, 9:].tolist() == o.leaderless(cfg, cfg, q).tolist()


def test_tempo_quorum_sizes_known_answers():
    """fantoch/src/config.rs:531-548 (tempo_parameters)."""
    from fantoch_amd.protocol import Protocol, tempo_quorum_sizes
    assert tempo_quorum_sizes(7, 1, False) == (4, 2, 4)
    assert tempo_quorum_sizes(7, 2, False) == (5, 3, 4)
    assert tempo_quorum_sizes(7, 1, True) == (2, 2, 6)
    assert tempo_quorum_sizes(7, 2, True) == (4, 3, 5)
    for n in range(3, 14):
        for f in (1, 2):
            assert Protocol.Tempo.quorum_size(n, f) == tempo_quorum_sizes(n, f, False)[0]
            assert Protocol.TempoTiny.quorum_size(n, f) == tempo_quorum_sizes(n, f, True)[0]
            assert Protocol.TempoWrite.quorum_size(n, f) == tempo_quorum_sizes(n, f, True)[1]


def test_write_dat_round_trip(tmp_path):
    """write_dat is the inverse of Dat::latencies (planet/dat.rs:33-75) on
    integral planets: every region's file re-read by Planet.from_dir gives the
    same matrix and name order (GCP, AWS 2021 and a synthetic planet with
    asymmetric pairs); each line is ping's `min/avg/max/mdev:zone` and the
    lines are in the order `sort -n` gives them (ping_exp_gcp/region_ping_loop.sh,
    run by fantoch_exp/src/bin/ping.rs:178-214)."""
    import subprocess

    from fantoch_amd.planet import AWS_2021_DIR, Planet, write_dat

    for name, p in (("gcp", Planet.new()), ("aws", Planet.from_dir(AWS_2021_DIR)),
                    ("syn", Planet.synthetic(24))):
        d = tmp_path / name
        for r in p.names:
            path = write_dat(p, r, str(d))
            lines = open(path).read().splitlines()
            assert len(lines) == p.R
            for ln in lines:
                stats, zone = ln.rsplit(":", 1)
                assert len(stats.split("/")) == 4 and zone in p.names
            srt = subprocess.run(["sort", "-n", path], capture_output=True, text=True, check=True,
                                 env={"LC_ALL": "C"}).stdout.splitlines()
            assert srt == lines
        q = Planet.from_dir(str(d))
        assert q.names == p.names
        assert np.array_equal(q.lat, p.lat)
