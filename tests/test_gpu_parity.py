"""GPU parity: the HIP path (libbote_hip.so through the C ABI) against the CPU
oracle (oracle/) and the reference's own golden values.  Bit-exact for
latencies, histograms, leaders, means, scores, validity and top-K identities;
COV outputs within 1e-12 relative (the tolerance north_star allows is 1e-9).
"""
import json
import math
import os

import numpy as np
import pytest

import oracle as O
from fantoch_amd import _lib
from fantoch_amd.bote import SLOT_KEYS as SLOT_KEYS_T
from fantoch_amd.bote import (DEFAULT_OBJECTIVES, DEFAULT_RANKING, Bote, DevicePlanet, FTMetric, RankingParams,
                              Search, SearchInput, Sweep, eval_configs)
from fantoch_amd.metrics import Stats
from fantoch_amd.planet import AWS_2021_DIR, Planet, Region

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_goldens.json")))
COV_RTOL = 1e-12


@pytest.fixture(scope="module")
def gcp():
    p = Planet.new()
    return p, DevicePlanet(p), O.OraclePlanet.of(p)


@pytest.fixture(scope="module")
def bote():
    return Bote.new()


# ------------------------------------------------ lib.rs known answers ----
def test_quorum_latencies(bote):
    g = GOLD["quorum_latencies"]
    for q, key in ((2, "q2"), (3, "q3")):
        assert [bote.quorum_latency(r, g["regions"], q) for r in g["regions"]] == g[key]


def test_leaderless(bote):
    g = GOLD["leaderless"]
    from fantoch_amd.metrics import Histogram
    for case in g["cases"]:
        h = Histogram.from_values(v for _, v in bote.leaderless(g["servers"], case["clients"], case["q"]))
        assert (h.mean().round(), h.cov().round(), h.mdtm().round()) == (case["mean"], case["cov"], case["mdtm"])


def test_leader(bote):
    g = GOLD["leader"]
    from fantoch_amd.metrics import Histogram
    for case in g["cases"]:
        h = Histogram.from_values(v for _, v in bote.leader(case["leader"], g["servers"], case["clients"], g["q"]))
        assert (h.mean().round(), h.cov().round(), h.mdtm().round()) == (case["mean"], case["cov"], case["mdtm"])
        stats = dict((r.name, hh) for r, hh in bote.all_leaders_stats(g["servers"], case["clients"], g["q"]))
        assert stats[case["leader"]] == h


def test_best_latency_leader(bote):
    g = GOLD["best_latency_leader"]
    _, h = bote.best_leader(g["servers"], g["servers"], g["q"], Stats.Mean)
    assert (h.mean().round(), h.cov().round(), h.mdtm().round()) == (g["mean"], g["cov"], g["mdtm"])


def test_tempo_fast_quorums_leaderless(gcp, bote):
    """BASELINE config 2's Tempo: fast quorums n/2+f and, tiny, 2f
    (fantoch/src/config.rs:317-329) through Bote::leaderless (lib.rs:38-59)."""
    p, _, o = gcp
    rng = np.random.default_rng(7)
    for n in (3, 5, 7, 9, 13):
        for f in range(1, min(n // 2, 2) + 1):
            for tiny, proto in ((False, _lib.TEMPO), (True, _lib.TEMPO_TINY)):
                q = _lib.lib().bote_quorum_size(proto, n, f)
                assert q == (2 * f if tiny else n // 2 + f)
                for _ in range(4):
                    srv = rng.choice(p.R, n, replace=False)
                    cli = rng.choice(p.R, 11, replace=False)
                    got = bote.leaderless([p.names[i] for i in srv], [p.names[i] for i in cli], q)
                    want = o.leaderless(srv, cli, q)
                    assert [r.name for r, _ in got] == [p.names[i] for i in cli]
                    assert [v for _, v in got] == want.tolist()


def test_single_config_api_vs_oracle(gcp):
    p, dp, o = gcp
    b = Bote(p)
    rng = np.random.default_rng(7)
    for _ in range(40):
        ns = int(rng.integers(2, 12))
        servers = rng.choice(p.R, ns, replace=False)
        clients = rng.choice(p.R, int(rng.integers(1, 20)), replace=True)
        q = int(rng.integers(1, ns + 1))
        sv = [p.names[i] for i in servers]
        cv = [p.names[i] for i in clients]
        assert [v for _, v in b.leaderless(sv, cv, q)] == o.leaderless(servers, clients, q).tolist()
        lead = int(rng.integers(0, p.R))
        assert [v for _, v in b.leader(p.names[lead], sv, cv, q)] == o.leader(lead, servers, clients, q).tolist()
        for stat in (Stats.Mean, Stats.COV, Stats.MDTM):
            r, _ = b.best_leader(sv, cv, q, stat)
            assert servers[o.best_leader(servers, clients, q, stat.value)] == p.idx(r)


# ------------------------------------------------ compute_stats parity ----
def _oracle_batch(o, srv, cli, cfg_pos):
    regs = srv[cfg_pos]
    return o.compute_stats(regs, cli)


def _check_eval(o, dp, srv, cli, n, cfg_pos, ranking=None):
    r = eval_configs(dp, srv, cli, n, configs=cfg_pos, ranking=ranking)
    ov, ol = _oracle_batch(o, srv, cli, cfg_pos)
    assert np.array_equal(r.vals.astype(np.uint64), np.where(ov == np.uint64(0xFFFFFFFFFFFFFFFF),
                                                                np.uint64(0xFFFFFFFF), ov))
    assert np.array_equal(r.leader, ol)
    # moments and means against the oracle histograms
    nc = len(cli)
    for i in range(0, len(cfg_pos), max(1, len(cfg_pos) // 64)):
        for slot in range(10):
            vals = r.slot_values(i, slot)
            if vals.size and vals[0] == 0xFFFFFFFF:
                continue
            st = O.hist_stats(vals)
            assert r.mean[i, slot] == st[0]
            if math.isnan(st[2]):
                assert math.isnan(r.cov[i, slot])
            else:
                assert abs(r.cov[i, slot] - st[2]) <= COV_RTOL * abs(st[2])
    return r


def test_gcp_r20c20_n3_n5_all_configs(gcp):
    """BASELINE config 1: GCP R=20, n=3,5, clients = all 20 — every config bit-exact."""
    p, dp, o = gcp
    srv = np.arange(p.R, dtype=np.uint32)
    for n in (3, 5):
        total = _lib.binomial(p.R, n)
        cfg = np.array([_lib.colex_unrank(r, n, p.R) for r in range(total)], dtype=np.uint32)
        _check_eval(o, dp, srv, srv, n, cfg)


def test_gcp_all_n_sampled(gcp):
    """BASELINE config 2: GCP n=2..13 (odd = reference, even = extension), sampled."""
    p, dp, o = gcp
    srv = np.arange(p.R, dtype=np.uint32)
    rng = np.random.default_rng(11)
    for n in range(2, 14):
        total = _lib.binomial(p.R, n)
        ranks = rng.choice(total, min(total, 1500), replace=False)
        cfg = np.array([_lib.colex_unrank(int(r), n, p.R) for r in ranks], dtype=np.uint32)
        _check_eval(o, dp, srv, srv, n, cfg)


def test_rank_mode_equals_explicit(gcp):
    p, dp, o = gcp
    srv = np.arange(p.R, dtype=np.uint32)
    n, rb, cnt = 7, 1234, 3000
    a = eval_configs(dp, srv, srv, n, rank_begin=rb, ncfg=cnt)
    cfg = np.array([_lib.colex_unrank(r, n, p.R) for r in range(rb, rb + cnt)], dtype=np.uint32)
    b = eval_configs(dp, srv, srv, n, configs=cfg)
    assert np.array_equal(a.vals, b.vals) and np.array_equal(a.leader, b.leader)


def test_unsorted_servers_and_members(gcp):
    """R13C13's server list is not in name order; members given out of order."""
    p, dp, o = gcp
    srv = p.idxs(GOLD["search"]["regions13"])
    rng = np.random.default_rng(5)
    for n in (3, 5, 6, 9):
        cfg = np.array([rng.permutation(len(srv))[:n] for _ in range(300)], dtype=np.uint32)
        _check_eval(o, dp, srv, srv, n, cfg)


def test_client_subsets_and_single_client(gcp):
    p, dp, o = gcp
    srv = np.arange(p.R, dtype=np.uint32)
    rng = np.random.default_rng(3)
    for nc in (1, 2, 7, 33):
        cli = rng.choice(p.R, nc, replace=nc > p.R).astype(np.uint32)
        cfg = np.array([rng.permutation(p.R)[:5] for _ in range(200)], dtype=np.uint32)
        _check_eval(o, dp, srv, cli, 5, cfg)


def test_aws_2021_all_leaders():
    """BASELINE config 3: AWS 2021_02_13 (R=5), FPaxos leader enumeration for every config."""
    p = Planet.from_dir(AWS_2021_DIR)
    dp = DevicePlanet(p)
    o = O.OraclePlanet.of(p)
    b = Bote(p)
    srv = np.arange(p.R, dtype=np.uint32)
    for n in (2, 3, 4, 5):
        cfg = np.array([_lib.colex_unrank(r, n, p.R) for r in range(_lib.binomial(p.R, n))], dtype=np.uint32)
        _check_eval(o, dp, srv, srv, n, cfg)
        for c in cfg:
            regs = [p.names[i] for i in c]
            for q in (2, 3):
                if q > n:
                    continue
                allst = b.all_leaders_stats(regs, p.names, q)
                for (lr, h), l in zip(allst, c):
                    assert list(h.iter_values()) == sorted(o.leader(int(l), c, srv, q).tolist())


def test_score_and_validity_vs_oracle(gcp):
    """Search::compute_score per config: bit-exact score and validity."""
    p, dp, o = gcp
    srv = np.arange(p.R, dtype=np.uint32)
    for params in ((30, 10, 0, 15), (110, 35, 0, 15), (0, 0, -1, 0), (20, 5, 1, 0)):
        rp = RankingParams.new(*params, 3, 13, FTMetric.F1F2)
        for n in (3, 5, 11, 13):
            total = _lib.binomial(p.R, n)
            ranks = np.random.default_rng(n).choice(total, min(total, 3000), replace=False)
            cfg = np.array([_lib.colex_unrank(int(x), n, p.R) for x in ranks], dtype=np.uint32)
            g = eval_configs(dp, srv, srv, n, configs=cfg, ranking=rp, values=False)
            sc, va = o.scores(srv[cfg], srv, [float(x) for x in params], 2)
            assert np.array_equal(g.valid.astype(bool), va.astype(bool))
            assert np.array_equal(g.score.view(np.uint64), sc.view(np.uint64))


# ---------------------------------------------------- Search end-to-end ---
def test_search_r13c13_golden():
    """search.rs:671-751 through the GPU path."""
    g = GOLD["search"]
    search = Search(3, 13, SearchInput.R13C13)
    params = RankingParams.new(110, 35, 0, 15, 3, 13, FTMetric.F1F2)
    score, css, _clients = search.sorted_evolving_configs(params)[0]
    assert score.round() == g["score"]
    sorted_config = []
    for cs in css:
        for region in cs.config:
            if region not in sorted_config:
                sorted_config.append(region)
        if len(cs.config) == 5:
            assert Search.stats_fmt(cs.stats, 5) == g["stats_fmt_n5"]
    assert [r.name for r in sorted_config] == g["sorted_config"]


# ---------------------------------------------------- sweep and top-K -----
def _oracle_sweep(o, srv, cli, n, rb, re, objectives, K, ranking, threads=16):
    rp = (ranking.min_mean_fpaxos_improv, ranking.min_mean_epaxos_improv, ranking.min_fairness_fpaxos_improv,
          ranking.min_mean_decrease)
    return o.sweep(srv, cli, n, rb, re, objectives, K, rp, ranking.ft_metric.value, threads)


@pytest.mark.parametrize("n,rb,re", [(3, 0, 1140), (5, 0, 15504), (7, 1000, 61000), (13, 0, 77520)])
def test_sweep_topk_gcp_vs_oracle(gcp, n, rb, re):
    p, dp, o = gcp
    srv = np.arange(p.R, dtype=np.uint32)
    rp = RankingParams.new(30, 10, 0, 15, 3, 13, FTMetric.F1F2)
    sw = Sweep(dp, srv, srv, n, DEFAULT_OBJECTIVES, K=100, ranking=rp, digest=True)
    sw.launch(rb, re)
    got = sw.result()
    tops, valid, digest = _oracle_sweep(o, srv, srv, n, rb, re, DEFAULT_OBJECTIVES, 100, rp)
    assert got.valid == valid
    assert got.digest == digest
    for a, b in zip(got.tops, tops):
        assert a == b


def test_sweep_synthetic_r64_n7_subrange_vs_oracle():
    """BASELINE config 4 workload on a bounded rank range, oracle-checked."""
    p = Planet.synthetic(64)
    dp = DevicePlanet(p)
    o = O.OraclePlanet.of(p)
    srv = np.arange(64, dtype=np.uint32)
    total = _lib.binomial(64, 7)
    for rb in (0, total // 2, total - 300_000):
        re = rb + 300_000
        sw = Sweep(dp, srv, srv, 7, DEFAULT_OBJECTIVES, K=100, ranking=DEFAULT_RANKING, digest=True)
        sw.launch(rb, re)
        got = sw.result()
        tops, valid, digest = _oracle_sweep(o, srv, srv, 7, rb, re, DEFAULT_OBJECTIVES, 100, DEFAULT_RANKING)
        assert (got.valid, got.digest) == (valid, digest)
        assert got.tops == [list(t) for t in tops]


def test_sweep_full_r64_n7_properties():
    """Full 621,216,192-config sweep: shard invariance (merged top-K, valid
    count and digest sum are independent of the split) and the reported top-K
    keys re-derived by the oracle for those configs."""
    p = Planet.synthetic(64)
    dp = DevicePlanet(p)
    o = O.OraclePlanet.of(p)
    srv = np.arange(64, dtype=np.uint32)
    sw = Sweep(dp, srv, srv, 7, DEFAULT_OBJECTIVES, K=100, ranking=DEFAULT_RANKING, digest=True)
    total = sw.total
    assert total == 621216192
    sw.launch(0, total)
    full = sw.result()
    import torch
    nb = sw.result_bytes()
    blocks = torch.empty(3 * nb, dtype=torch.uint8, device="cuda")
    cuts = [0, total // 3, 2 * total // 3, total]
    for i in range(3):
        sw.launch(cuts[i], cuts[i + 1])
        sw.result_device(blocks.data_ptr() + i * nb)
    out = torch.empty(nb, dtype=torch.uint8, device="cuda")
    sw.merge_device(blocks.data_ptr(), 3, out.data_ptr())
    torch.cuda.synchronize()
    merged = sw.parse_block(out.cpu().numpy())
    assert merged.tops == full.tops and merged.valid == full.valid and merged.digest == full.digest
    # every reported record is re-derived by the oracle (keys bit-exact)
    for oi, (kind, slot) in enumerate(DEFAULT_OBJECTIVES):
        recs = full.tops[oi][:10]
        for key, rank in recs:
            tops, _, _ = _oracle_sweep(o, srv, srv, 7, rank, rank + 1, [(kind, slot)], 1, DEFAULT_RANKING, 1)
            assert tops[0] == [(key, rank)]


def test_near_tie_replay_equidistant():
    """Equidistant planet: every FPaxos leader ties exactly -> device replay path."""
    regions, p = Planet.equidistant(10, 9)
    dp = DevicePlanet(p)
    o = O.OraclePlanet.of(p)
    srv = np.arange(p.R, dtype=np.uint32)
    for n in (3, 4, 7):
        cfg = np.array([_lib.colex_unrank(r, n, p.R) for r in range(_lib.binomial(p.R, n))], dtype=np.uint32)
        _check_eval(o, dp, srv, srv, n, cfg)


def test_zero_offdiagonal_planet():
    """Off-diagonal zero latencies: the colocated nearest server is not the client itself."""
    rng = np.random.default_rng(9)
    R = 12
    lat = rng.integers(0, 4, size=(R, R))
    np.fill_diagonal(lat, 0)
    p = Planet([f"z{i:02d}" for i in range(R)], lat)
    dp = DevicePlanet(p)
    o = O.OraclePlanet.of(p)
    srv = np.arange(R, dtype=np.uint32)
    for n in (2, 3, 5, 8, 12):
        total = _lib.binomial(R, n)
        cfg = np.array([_lib.colex_unrank(r, n, R) for r in range(min(total, 800))], dtype=np.uint32)
        _check_eval(o, dp, srv, srv, n, cfg)


def test_r128_n6_subrange_and_max_latency():
    p = Planet.synthetic(128)
    dp = DevicePlanet(p)
    o = O.OraclePlanet.of(p)
    srv = np.arange(128, dtype=np.uint32)
    rb = _lib.binomial(128, 6) - 50_000
    sw = Sweep(dp, srv, srv, 6, DEFAULT_OBJECTIVES, K=64, ranking=DEFAULT_RANKING, digest=True)
    sw.launch(rb, rb + 50_000)
    got = sw.result()
    tops, valid, digest = _oracle_sweep(o, srv, srv, 6, rb, rb + 50_000, DEFAULT_OBJECTIVES, 64, DEFAULT_RANKING)
    assert (got.valid, got.digest) == (valid, digest) and got.tops == [list(t) for t in tops]
    # extreme latencies
    lat = np.full((16, 16), 16383)
    np.fill_diagonal(lat, 0)
    lat[3, 5] = 1
    q = Planet([f"m{i:02d}" for i in range(16)], lat)
    qo = O.OraclePlanet.of(q)
    s16 = np.arange(16, dtype=np.uint32)
    cfg = np.array([_lib.colex_unrank(r, 9, 16) for r in range(0, _lib.binomial(16, 9), 7)], dtype=np.uint32)
    _check_eval(qo, DevicePlanet(q), s16, s16, 9, cfg)


# ------------------------------------------------ fast path vs generic ----
def _sweep(dp, srv, cli, n, rb, re, K=100, ranking=DEFAULT_RANKING, generic=False, kernel=None):
    """kernel: None (default choice), 'generic', 'fast' or 'group' (bote_sweep_create_ex)."""
    kernel = "generic" if generic else kernel
    if kernel == "group" and n < 4:
        kernel = "fast"
    sw = Sweep(dp, srv, cli, n, DEFAULT_OBJECTIVES, K=K, ranking=ranking, digest=True, kernel=kernel)
    if kernel:
        assert sw.kernel_path() == kernel
    sw.launch(rb, re)
    return sw.result()


def test_fast_path_equals_generic_path():
    p = Planet.synthetic(64)
    dp = DevicePlanet(p)
    srv = np.arange(64, dtype=np.uint32)
    for n, rb, re in ((7, 10_000_000, 12_000_000), (6, 0, 3_000_000), (4, 0, _lib.binomial(64, 4)),
                      (9, 123_456_789, 124_456_789)):
        b = _sweep(dp, srv, srv, n, rb, re, generic=True)
        for k in ("fast", "group"):
            a = _sweep(dp, srv, srv, n, rb, re, kernel=k)
            assert (a.valid, a.digest, a.tops) == (b.valid, b.digest, b.tops), k
    # a client subset (separate region-quad matrix) and a ragged client count
    g = Planet.new()
    gdp = DevicePlanet(g)
    gs = np.arange(g.R, dtype=np.uint32)
    for cli in (np.array([3, 1, 4, 15, 9, 2, 6], np.uint32), np.arange(0, 20, 2, dtype=np.uint32)):
        for n in (3, 5, 8):
            b = _sweep(gdp, gs, cli, n, 0, _lib.binomial(g.R, n), generic=True)
            for k in ("fast", "group"):
                a = _sweep(gdp, gs, cli, n, 0, _lib.binomial(g.R, n), kernel=k)
                assert (a.valid, a.digest, a.tops) == (b.valid, b.digest, b.tops), k


def test_group_kernel_custom_objectives():
    """Objective sets other than the default run the group kernel's generic
    key path (finish_config); it must equal the generic kernel."""
    p = Planet.synthetic(64)
    dp = DevicePlanet(p)
    srv = np.arange(64, dtype=np.uint32)
    objs = [(_lib.OBJ_COV, _lib.SLOT_AF2), (_lib.OBJ_MEAN, 5 + _lib.SLOT_FF2), (_lib.OBJ_SCORE, 0),
            (_lib.OBJ_COV, 5 + _lib.SLOT_E), (_lib.OBJ_MEAN, _lib.SLOT_AF1), (_lib.OBJ_COV, _lib.SLOT_FF1)]
    out = {}
    for k in ("generic", "group"):
        sw = Sweep(dp, srv, srv, 7, objs, K=50, ranking=DEFAULT_RANKING, digest=True, kernel=k)
        assert sw.kernel_path() == k
        sw.launch(200_000_000, 201_500_000)
        r = sw.result()
        out[k] = (r.valid, r.digest, r.tops)
    assert out["group"] == out["generic"]


def test_fast_path_deferral_equidistant():
    """Every FPaxos leader ties exactly: the fast kernel defers every config
    to the exact generic kernel; results still match the oracle."""
    regions, p = Planet.equidistant(10, 12)
    dp = DevicePlanet(p)
    o = O.OraclePlanet.of(p)
    srv = np.arange(p.R, dtype=np.uint32)
    rp = RankingParams.new(0, 0, 0, 0, 3, 13, FTMetric.F1F2)
    for n in (3, 5):
        total = _lib.binomial(p.R, n)
        tops, valid, digest = _oracle_sweep(o, srv, srv, n, 0, total, DEFAULT_OBJECTIVES, 100, rp)
        for k in ("fast", "group"):
            got = _sweep(dp, srv, srv, n, 0, total, ranking=rp, kernel=k)
            assert (got.valid, got.digest) == (valid, digest)
            assert got.tops == [list(t) for t in tops]


def test_fast_path_deferral_overflow():
    """More deferred configs than the queue holds: the range is recomputed on
    the generic path before results are returned."""
    regions, p = Planet.equidistant(7, 48)
    dp = DevicePlanet(p)
    o = O.OraclePlanet.of(p)
    srv = np.arange(p.R, dtype=np.uint32)
    total = _lib.binomial(p.R, 5)
    assert total > (1 << 20)
    tops, valid, digest = _oracle_sweep(o, srv, srv, 5, 0, total, DEFAULT_OBJECTIVES, 100, DEFAULT_RANKING)
    for k in ("fast", "group"):
        got = _sweep(dp, srv, srv, 5, 0, total, kernel=k)
        assert (got.valid, got.digest) == (valid, digest)
        assert got.tops == [list(t) for t in tops]


@pytest.mark.parametrize("world", [2, 8, 9])
def test_sharded_merge_tree_on_device(gcp, world):
    """bench.py's N>1 data path minus RCCL: `world` contiguous shards swept on
    the device, their result blocks concatenated in rank order (what
    all_gather_into_tensor yields) and merged by dist.merge_gathered (a tree
    beyond 8 shards) equal one unsharded sweep."""
    import torch

    from fantoch_amd.dist import merge_gathered, shard_range

    p, dp, _ = gcp
    srv = np.arange(p.R, dtype=np.uint32)
    sw = Sweep(dp, srv, srv, 7, DEFAULT_OBJECTIVES, K=100, ranking=DEFAULT_RANKING, digest=True)
    sw.launch(0, sw.total)
    full = sw.result()
    nb = sw.result_bytes()
    gathered = torch.empty(world * nb, dtype=torch.uint8, device="cuda")
    for r in range(world):
        b, e = shard_range(sw.total, world, r)
        sw.launch(b, e)
        sw.result_device(gathered.data_ptr() + r * nb)
    merged = merge_gathered(sw, gathered, world)
    assert merged.tops == full.tops and merged.valid == full.valid and merged.digest == full.digest


def test_checkpointed_sweep_resumes(gcp, tmp_path):
    """A chunked sweep interrupted after 3 chunks and resumed from its
    checkpoint equals the one-shot sweep; a checkpoint of another sweep is
    refused."""
    p, dp, _ = gcp
    srv = np.arange(p.R, dtype=np.uint32)
    sw = Sweep(dp, srv, srv, 7, DEFAULT_OBJECTIVES, K=100, ranking=DEFAULT_RANKING, digest=True)
    sw.launch(0, sw.total)
    full = sw.result()
    ck = str(tmp_path / "sweep.ckpt")
    assert sw.run_checkpointed(ck, chunk=9000, stop_after=3) is None
    assert os.path.exists(ck)
    res = sw.run_checkpointed(ck, chunk=9000)
    assert res.tops == full.tops and res.valid == full.valid and res.digest == full.digest
    # a finished checkpoint returns the result without sweeping again
    again = sw.run_checkpointed(ck, chunk=9000)
    assert again.tops == full.tops and again.digest == full.digest
    other = Sweep(dp, srv, srv, 5, DEFAULT_OBJECTIVES, K=100, ranking=DEFAULT_RANKING, digest=True)
    with pytest.raises(ValueError):
        other.run_checkpointed(ck)
    # same n, K, lists and objectives, but scored under other RankingParams:
    # its validity and score objective differ, so the checkpoint is refused
    rk = RankingParams.new(100, 35, 0, 15, 3, 13, FTMetric.F1F2)
    scored_other = Sweep(dp, srv, srv, 7, DEFAULT_OBJECTIVES, K=100, ranking=rk, digest=True)
    with pytest.raises(ValueError):
        scored_other.run_checkpointed(ck)
    # and without the digest
    nodig = Sweep(dp, srv, srv, 7, DEFAULT_OBJECTIVES, K=100, ranking=DEFAULT_RANKING, digest=False)
    with pytest.raises(ValueError):
        nodig.run_checkpointed(ck)


def test_search_r17cmaxn_client_sets(gcp):
    """search.rs:199-232 with many client sets (R17CMaxN: every max_n-subset of
    the 17 regions is a client set and its own server list); per-config stats
    against the oracle for a sample of the sets."""
    p, _, o = gcp
    s = Search(3, 5, SearchInput.R17CMaxN, planet=p)
    assert len(s.all_configs) == math.comb(17, 5)
    for ci in range(0, len(s.all_configs), 397):
        clients, configs = s.all_configs[ci]
        cli = p.idxs(clients)
        for n in (3, 5):
            d = configs[n]
            assert len(d["cfg"]) == math.comb(5, n)
            for i in range(len(d["cfg"])):
                ids = np.array([d["srv"][q] for q in d["cfg"][i]], dtype=np.uint32)
                vals, lead = o.compute_stats(ids.reshape(1, n), cli)
                st = s._stats(ci, n, i)
                for slot in range(10):
                    seg = (vals[0, slot * len(cli):(slot + 1) * len(cli)] if slot < 5
                           else vals[0, 5 * len(cli) + (slot - 5) * n:5 * len(cli) + (slot - 4) * n])
                    proto, f = SLOT_KEYS_T[slot % 5]
                    if f > min(n // 2, 2):
                        continue
                    from fantoch_amd.protocol import ClientPlacement
                    h = st.get(proto, f, ClientPlacement.Input if slot < 5 else ClientPlacement.Colocated)
                    assert list(h.iter_values()) == sorted(seg.tolist())


@pytest.mark.parametrize("n", [2, 4, 6, 7, 8, 9, 10, 11, 12])
def test_gcp_config2_full_sweep_digest(gcp, n):
    """BASELINE config 2 in full: every GCP R=20 config of size n (odd = the
    reference's n, even = extension) swept on the device; the digest covers
    every config's 10 slot moments and FPaxos leader, so equal digests, valid
    counts and top-K lists mean the whole sweep matches the oracle."""
    p, dp, o = gcp
    srv = np.arange(p.R, dtype=np.uint32)
    rp = RankingParams.new(30, 10, 0, 15, 3, 13, FTMetric.F1F2)
    sw = Sweep(dp, srv, srv, n, DEFAULT_OBJECTIVES, K=100, ranking=rp, digest=True)
    sw.launch(0, sw.total)
    got = sw.result()
    tops, valid, digest = _oracle_sweep(o, srv, srv, n, 0, sw.total, DEFAULT_OBJECTIVES, 100, rp)
    assert (got.valid, got.digest) == (valid, digest)
    assert got.tops == [list(t) for t in tops]


def test_sweep_full_r128_n6_properties():
    """BASELINE config 5 in full (5,423,611,200 configs): shard invariance of
    the merged result and the top records' keys re-derived by the oracle."""
    import torch

    from fantoch_amd.dist import merge_gathered, shard_range

    p = Planet.synthetic(128)
    dp = DevicePlanet(p)
    o = O.OraclePlanet.of(p)
    srv = np.arange(128, dtype=np.uint32)
    sw = Sweep(dp, srv, srv, 6, DEFAULT_OBJECTIVES, K=100, ranking=DEFAULT_RANKING, digest=True)
    assert sw.total == 5423611200
    sw.launch(0, sw.total)
    full = sw.result()
    nb = sw.result_bytes()
    gathered = torch.empty(3 * nb, dtype=torch.uint8, device="cuda")
    for r in range(3):
        b, e = shard_range(sw.total, 3, r)
        sw.launch(b, e)
        sw.result_device(gathered.data_ptr() + r * nb)
    merged = merge_gathered(sw, gathered, 3)
    assert merged.tops == full.tops and merged.valid == full.valid and merged.digest == full.digest
    for oi, (kind, slot) in enumerate(DEFAULT_OBJECTIVES):
        for key, rank in full.tops[oi][:5]:
            tops, _, _ = _oracle_sweep(o, srv, srv, 6, rank, rank + 1, [(kind, slot)], 1, DEFAULT_RANKING, 1)
            assert tops[0] == [(key, rank)]
