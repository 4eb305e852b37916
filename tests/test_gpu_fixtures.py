"""GPU parity at full size against oracle-pinned fixtures (scripts/
oracle_full_sweep.py, tests/golden/make_keys_golden.py; the oracle is
oracle/bote_oracle.cpp):
  * BASELINE config 4, R=64 n=7: all 621,216,192 configs -- valid count,
    digest and the 5 x K=100 top-K lists (tests/golden/syn_r64n7_full.json);
  * BASELINE config 5, R=128 n=6: nine 10^6-rank windows, eight straddling a
    colex boundary C(m, 6) where every member changes, and the full sweep on
    the group kernel equal to the generic kernel;
  * BASELINE config 2: per-client latency vectors and leaders of EVERY GCP
    config of every n = 2..13 against the oracle's compute_stats."""
import json
import os
from math import comb

import numpy as np
import pytest

import oracle as O
from fantoch_amd import _lib
from fantoch_amd.bote import DEFAULT_OBJECTIVES, DEFAULT_RANKING, DevicePlanet, Sweep, eval_configs
from fantoch_amd.planet import Planet

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _fixture(name):
    path = os.path.join(GOLDEN, name)
    if not os.path.exists(path):
        pytest.skip(f"{name} not generated yet (scripts/oracle_fixtures.sh)")
    return json.load(open(path))


def _check(res, fx):
    # (u64 keys and digests are JSON strings in the make_keys_golden.py windows)
    assert res.valid == fx["valid"]
    assert res.digest == int(fx["digest"])
    assert res.tops == [[(int(k), int(r)) for k, r in t] for t in fx["tops"]]


def test_full_r64n7_vs_oracle_fixture():
    fx = _fixture("syn_r64n7_full.json")
    p = Planet.synthetic(64)
    srv = np.arange(64, dtype=np.uint32)
    sw = Sweep(DevicePlanet(p), srv, srv, 7, DEFAULT_OBJECTIVES, K=100, ranking=DEFAULT_RANKING, digest=True)
    assert (fx["rank_begin"], fx["rank_end"]) == (0, sw.total)
    sw.launch(0, sw.total)
    _check(sw.result(), fx)


def test_r128n6_windows_vs_oracle_fixture():
    """Nine 10^6-rank windows (eight straddling a colex boundary C(m, 6)) and
    64 10^5-rank windows at seeded random offsets, which begin and end inside
    groups (tests/golden/make_keys_golden.py)."""
    fx = _fixture("syn_r128n6_windows.json")
    p = Planet.synthetic(128)
    srv = np.arange(128, dtype=np.uint32)
    sw = Sweep(DevicePlanet(p), srv, srv, 6, DEFAULT_OBJECTIVES, K=100, ranking=DEFAULT_RANKING, digest=True)
    assert sw.kernel_path() == "group"
    ws = [w for w in fx["windows"] if not w.get("x_only")]
    assert len(ws) >= 73
    assert sum(1 for w in ws if w.get("random")) >= 64
    for w in ws:
        sw.launch(w["rank_begin"], w["rank_end"])
        _check(sw.result(), w)


def test_r128n6_full_group_equals_generic():
    """All 5,423,611,200 configs: the group kernel equals the exact generic
    kernel (every config's moments and leader through the digest, valid count,
    top-K)."""
    p = Planet.synthetic(128)
    dp = DevicePlanet(p)
    srv = np.arange(128, dtype=np.uint32)
    out = {}
    for k in ("group", "generic"):
        sw = Sweep(dp, srv, srv, 6, DEFAULT_OBJECTIVES, K=100, ranking=DEFAULT_RANKING, digest=True, kernel=k)
        sw.launch(0, sw.total)
        r = sw.result()
        out[k] = (r.valid, r.digest, r.tops)
    assert out["group"] == out["generic"]


@pytest.mark.parametrize("n", range(2, 14))
def test_gcp_every_config_per_client_vectors(n):
    """BASELINE config 2: for EVERY GCP config of size n, the device's
    per-client latencies of all 10 keys and its FPaxos leader equal the
    oracle's compute_stats (search.rs:262-319), bit for bit."""
    p = Planet.new()
    dp = DevicePlanet(p)
    o = O.OraclePlanet.of(p)
    srv = np.arange(p.R, dtype=np.uint32)
    total = comb(p.R, n)
    for rb in range(0, total, 50_000):
        cnt = min(50_000, total - rb)
        r = eval_configs(dp, srv, srv, n, rank_begin=rb, ncfg=cnt)
        cfg = np.array([_lib.colex_unrank(x, n, p.R) for x in range(rb, rb + cnt)], dtype=np.uint32)
        ov, ol = o.compute_stats(srv[cfg], srv, threads=16)
        want = np.where(ov == np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64(0xFFFFFFFF), ov)
        assert np.array_equal(r.vals.astype(np.uint64), want), (n, rb)
        assert np.array_equal(r.leader, ol), (n, rb)
