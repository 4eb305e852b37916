"""The committed fixtures (tests/golden/make_golden.py) against the planet
loader and the CPU oracle.  CPU only; tests/test_gpu_parity.py checks the HIP
path against the same files."""
import json
import os
from math import comb

import numpy as np
import pytest

import oracle as O
from fantoch_amd.bote import DEFAULT_OBJECTIVES
from fantoch_amd.planet import AWS_2020_DIR, AWS_2021_DIR, Planet

G = os.path.join(os.path.dirname(__file__), "golden")
RP = (110.0, 35.0, 0.0, 15.0)


@pytest.fixture(scope="module")
def stats():
    return np.load(os.path.join(G, "gcp_n3_n5_stats.npz"))


@pytest.fixture(scope="module")
def topk():
    return json.load(open(os.path.join(G, "topk.json")))


def test_planets_fixture_matches_loader():
    z = np.load(os.path.join(G, "planets.npz"))
    for key, p in (("gcp", Planet.new()), ("aws20", Planet.from_dir(AWS_2020_DIR)),
                   ("aws21", Planet.from_dir(AWS_2021_DIR))):
        assert list(z[f"{key}_names"]) == p.names
        assert np.array_equal(z[f"{key}_lat"], p.lat.astype(np.uint16))


@pytest.mark.parametrize("n,step", [(3, 1), (5, 7)])
def test_oracle_per_config_matches_fixture(stats, n, step):
    p = Planet.new()
    o = O.OraclePlanet.of(p)
    srv = np.arange(p.R, dtype=np.uint32)
    ranks = np.arange(0, comb(p.R, n), step)
    cfg = np.array([O.colex_unrank(int(r), n, p.R) for r in ranks], dtype=np.uint32)
    vals, lead = o.compute_stats(cfg, srv)
    assert np.array_equal(lead, stats[f"n{n}_leader"][ranks])
    nc = p.R
    for slot in range(10):
        if n < 4 and slot % 5 in (2, 3):
            continue
        v = vals[:, slot * nc:(slot + 1) * nc] if slot < 5 else vals[:, 5 * nc + (slot - 5) * n:5 * nc + (slot - 4) * n]
        assert np.array_equal(v.sum(axis=1), stats[f"n{n}_s1"][ranks, slot].astype(np.uint64))
        assert np.array_equal((v * v).sum(axis=1), stats[f"n{n}_s2"][ranks, slot])
    sc, va = o.scores(cfg, srv, RP, 2)
    assert np.array_equal(va, stats[f"n{n}_valid"][ranks])
    assert np.array_equal(sc.view(np.uint64), stats[f"n{n}_score"][ranks].view(np.uint64))


@pytest.mark.parametrize("case", ["gcp_n3", "gcp_n5", "gcp_n13", "aws21_n3", "aws21_n5"])
def test_oracle_topk_matches_fixture(topk, case):
    c = topk["cases"][case]
    p = Planet.new() if case.startswith("gcp") else Planet.from_dir(AWS_2021_DIR)
    o = O.OraclePlanet.of(p)
    s = np.arange(p.R, dtype=np.uint32)
    tops, valid, digest = o.sweep(s, s, c["n"], c["rank_begin"], c["rank_end"], DEFAULT_OBJECTIVES, topk["K"],
                                  RP, 2, 4)
    assert valid == c["valid"] and str(digest) == c["digest"]
    assert [[[str(k), r] for k, r in t] for t in tops] == c["tops"]


def test_full_r64n7_fixture_keys_rederived():
    """tests/golden/syn_r64n7_full.json (the oracle over all 621,216,192 ranks,
    scripts/oracle_full_sweep.py): every list is sorted by (key, rank) and the
    first 20 records of each objective carry the key the oracle computes for
    that single config."""
    fx = json.load(open(os.path.join(G, "syn_r64n7_full.json")))
    assert (fx["R"], fx["n"], fx["rank_begin"], fx["rank_end"]) == (64, 7, 0, comb(64, 7))
    p = Planet.synthetic(64)
    o = O.OraclePlanet.of(p)
    s = np.arange(64, dtype=np.uint32)
    for oi, t in enumerate(fx["tops"]):
        assert len(t) == fx["K"] and t == sorted(t)
        for key, rank in t[:20]:
            tops, _, _ = o.sweep(s, s, 7, rank, rank + 1, DEFAULT_OBJECTIVES, 1, RP, 2, 1)
            assert tops[oi] == [(key, rank)], (oi, rank)


@pytest.mark.parametrize("m", [6, 64, 127])
def test_r128n6_edge_windows_fixture_vs_oracle(m):
    """tests/golden/syn_r128n6_edges.json (make_keys_golden.py edges): a
    10^4-rank window on every colex boundary C(m, 6), m = 6..127, with both key
    sets; three of them swept again here by the oracle."""
    from fantoch_amd import _lib
    from fantoch_amd.bote import CONFIG5_OBJECTIVES

    fx = json.load(open(os.path.join(G, "syn_r128n6_edges.json")))
    ws = {w["m"]: w for w in fx["windows"]}
    assert sorted(ws) == list(range(6, 128))
    assert all(w["rank_begin"] <= comb(mm, 6) <= w["rank_end"] for mm, w in ws.items())
    w = ws[m]
    p = Planet.synthetic(128)
    o = O.OraclePlanet.of(p)
    s = np.arange(128, dtype=np.uint32)
    for keys, objs, c in ((0, DEFAULT_OBJECTIVES, w), (_lib.KEYS_TEMPO_ALL_LEADERS, CONFIG5_OBJECTIVES, w["x"])):
        assert [tuple(x) for x in c["objectives"]] == list(objs)
        tops, valid, digest = o.sweep(s, s, 6, w["rank_begin"], w["rank_end"], objs, w["K"], RP, 2, 4, keys=keys)
        assert valid == c["valid"] and str(digest) == c["digest"]
        assert [[[str(k), r] for k, r in t] for t in tops] == c["tops"]


AROUND = {"x": ("syn_r128n6_around_pin.json", "syn_r128n6_pin.json"),
          "base": ("syn_r128n6_base_around_pin.json", "syn_r128n6_base_pin.json")}


def _around_pin(kind="x"):
    fx_name, pin_name = AROUND[kind]
    path = os.path.join(G, fx_name)
    if not os.path.exists(path):
        pytest.skip(f"{fx_name} not generated yet (tests/golden/make_keys_golden.py around)")
    return json.load(open(path)), json.load(open(os.path.join(G, pin_name)))


@pytest.mark.parametrize("kind", ["x", "base"])
def test_r128n6_pin_records_in_their_oracle_neighbourhoods(kind):
    """Config 5's full-size pin (GPU: group == generic) against the oracle
    around its own records (syn_r128n6_around_pin.json): the oracle sweeps
    2 x 2,048 colex ranks around each of the 800 reported records, so
      * every reported record is among its window's 100 best in the oracle's
        own sweep, with the same key (its key and standing are the oracle's,
        not only its order among the reported records);
      * no config of those windows at or below an objective's 100th reported
        (key, rank) is missing from the pin (the records' closest colex
        neighbours, which share at least 3 of the 6 members, do not beat
        them unreported)."""
    fx, pin = _around_pin(kind)
    assert fx["K"] == pin["K"] == 100 and fx["objectives"] == pin["objectives"]
    wins = fx["windows"]
    found = 0
    for o, t in enumerate(pin["tops"]):
        recs = [(int(k), r) for k, r in t]
        kth, S = recs[-1], set(recs)
        for key, rank in recs:
            w = next(w for w in wins if w["rank_begin"] <= rank < w["rank_end"])
            lst = [(int(k), r) for k, r in w["tops"][o]]
            assert (key, rank) in lst, (o, rank)
            found += 1
        for w in wins:
            lst = [(int(k), r) for k, r in w["tops"][o]]
            assert all(rec in S for rec in lst if rec <= kth), (o, w["rank_begin"])
            # the fixture keeps every list up to one record past the K-th; a
            # window whose whole K=100 list is at or below it must end on the
            # K-th itself (objective 7's 100 records are 100 consecutive ranks
            # of one key), or configs would be left unchecked
            if w["full_below_kth"][o]:
                assert lst[-1] == kth, (o, w["rank_begin"])
    assert found == 100 * len(pin["tops"])


@pytest.mark.parametrize("kind,i", [("x", 0), ("x", 269), ("x", 537), ("base", 0), ("base", 371)])
def test_r128n6_around_pin_fixture_vs_oracle(kind, i):
    """Some of the around-pin windows swept again by the oracle here."""
    fx, _ = _around_pin(kind)
    w = fx["windows"][i]
    p = Planet.synthetic(128)
    o = O.OraclePlanet.of(p)
    s = np.arange(128, dtype=np.uint32)
    objs = [tuple(x) for x in fx["objectives"]]
    tops, valid, digest = o.sweep(s, s, 6, w["rank_begin"], w["rank_end"], objs, fx["K"], RP, 2, 4, keys=fx["keys"])
    assert valid == w["valid"] and str(digest) == w["digest"]
    assert [[[str(k), r] for k, r in t][:len(s_)] for t, s_ in zip(tops, w["tops"])] == w["tops"]


@pytest.mark.parametrize("fx_name,pin_name,least", [
    ("syn_r128n6_1700000000_1897132288.json", "syn_r128n6_base_pin.json", 30),
    ("syn_r128n6_x_2005000000_2035408704.json", "syn_r128n6_pin.json", 100),
    ("syn_r128n6_x_540000000_570408704.json", "syn_r128n6_pin.json", 100),
    ("syn_r128n6_x_1026000000_1056408704.json", "syn_r128n6_pin.json", 30),
    ("syn_r128n6_x_327000000_356360128.json", "syn_r128n6_pin.json", 20),
    ("syn_r128n6_x_1823000000_1852360128.json", "syn_r128n6_pin.json", 20),
    ("syn_r128n6_x_4963900000_4992211552.json", "syn_r128n6_pin.json", 15),
    ("syn_r128n6_x_4513400000_4542760128.json", "syn_r128n6_pin.json", 15),
    ("syn_r128n6_x_2400000000_2429360128.json", "syn_r128n6_pin.json", 15)])
def test_r128n6_oracle_range_agrees_with_the_pin(fx_name, pin_name, least):
    """The oracle's contiguous ranges of config 5 (the 10-key sweep over
    2.0e8 ranks; the extended keys over five ranges of ~3.0e7 ranks placed on
    clusters of the pin's records) against the GPU's full-size pins: every
    pin record inside a range is in the oracle's list for that range, and
    every record of the oracle's list at or below the pin's 100th is in the
    pin; at least `least` pin records lie inside."""
    path = os.path.join(G, fx_name)
    if not os.path.exists(path):
        pytest.skip("oracle range fixture not generated")
    fx = json.load(open(path))
    pin = json.load(open(os.path.join(G, pin_name)))
    assert fx["objectives"] == pin["objectives"] and fx["K"] == pin["K"]
    rb, re_ = fx["rank_begin"], fx["rank_end"]
    inside = 0
    for o, t in enumerate(pin["tops"]):
        recs = [(int(k), r) for k, r in t]
        lst = [tuple(x) for x in fx["tops"][o]]
        kth = recs[-1]
        for rec in recs:
            # (a global top-100 record inside the range is among the range's
            # 100 best: fewer than 100 configs of the range can beat it)
            if rb <= rec[1] < re_:
                assert rec in lst, (o, rec)
                inside += 1
        for rec in lst:
            if rec <= kth:
                assert rec in recs, (o, rec)
    assert inside >= least, inside
