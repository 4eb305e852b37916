"""The extended key set in the CPU oracle (compute_stats_x, BASELINE config 5:
"Tempo f=1,2 + FPaxos all leaders"), against the oracle's reference-pinned
single calls: Tempo's tiny (2f) and write (f + 1) keys are Bote::leaderless
(lib.rs:38-59) at those quorum sizes (config.rs:317-329); the all-leader
moments are Bote::leader per leader (lib.rs:67-89, all_leaders_stats
lib.rs:129-150); fl1/fl2 are best_leader by Stats::Mean (lib.rs:99-121).
CPU only."""
import numpy as np
import pytest

import oracle as O
from fantoch_amd import _lib
from fantoch_amd.planet import Planet


def _mom(v):
    v = np.asarray(v, dtype=np.uint64)
    return int(v.sum()), int((v * v).sum())


@pytest.mark.parametrize("planet,n", [("gcp", 2), ("gcp", 3), ("gcp", 5), ("gcp", 7), ("gcp", 8), ("gcp", 13),
                                      ("syn64", 7), ("syn128", 6)])
def test_moments_x_equal_single_calls(planet, n):
    p = Planet.new() if planet == "gcp" else Planet.synthetic(64 if planet == "syn64" else 128)
    o = O.OraclePlanet.of(p)
    rng = np.random.default_rng(n)
    cfgs = np.array([rng.choice(p.R, n, replace=False) for _ in range(12)], dtype=np.uint32)
    cli = np.arange(p.R, dtype=np.uint32)
    s1, s2, a1, a2, lead = o.moments_x(cfgs, cli, threads=2)
    mf = min(n // 2, 2)
    vals, lead0 = o.compute_stats(cfgs, cli)
    nc = len(cli)
    for i, cfg in enumerate(cfgs):
        assert lead[i] == lead0[i]
        # the compute_stats slots are unchanged
        for s in range(10):
            seg = vals[i, s * nc:(s + 1) * nc] if s < 5 else vals[i, 5 * nc + (s - 5) * n:5 * nc + (s - 4) * n]
            if seg[0] == np.iinfo(np.uint64).max:
                assert s1[i, s] == np.iinfo(np.uint64).max
            else:
                assert (int(s1[i, s]), int(s2[i, s])) == _mom(seg)
        for f in range(1, 3):
            for pl, cl in ((0, cli), (1, cfg)):
                tt, tw = _lib.SLOT_TT1 + f - 1 + 4 * pl, _lib.SLOT_TW1 + f - 1 + 4 * pl
                if f > mf:
                    assert s1[i, tt] == s1[i, tw] == np.iinfo(np.uint64).max
                    continue
                assert (int(s1[i, tt]), int(s2[i, tt])) == _mom(o.leaderless(cfg, cl, 2 * f))
                assert (int(s1[i, tw]), int(s2[i, tw])) == _mom(o.leaderless(cfg, cl, f + 1))
            if f > mf:
                assert s1[i, _lib.SLOT_FL1 + f - 1] == np.iinfo(np.uint64).max
                continue
            per = [_mom(o.leader(int(l), cfg, cli, f + 1)) for l in cfg]
            assert [(int(a1[i, f - 1, k]), int(a2[i, f - 1, k])) for k in range(n)] == per
            best = o.best_leader(cfg, cli, f + 1, 0)  # Stats::Mean, first minimum
            assert (int(s1[i, _lib.SLOT_FL1 + f - 1]), int(s2[i, _lib.SLOT_FL1 + f - 1])) == per[best]


def test_sweep_x_keeps_base_results_and_changes_digest():
    """The extended key set leaves valid counts and the compute_stats objectives
    unchanged; its digest also folds the extended slots and every leader."""
    p = Planet.new()
    o = O.OraclePlanet.of(p)
    s = np.arange(p.R, dtype=np.uint32)
    objs = [(0, 0), (1, 0), (1, 1), (2, 0), (1, 4)]
    t0, v0, d0 = o.sweep(s, s, 5, 0, 15504, objs, 16, threads=4)
    t1, v1, d1 = o.sweep(s, s, 5, 0, 15504, objs + [(1, 10), (1, 13), (1, 18)], 16, threads=4, keys=1)
    assert v0 == v1 and t1[:5] == t0 and d0 != d1
    assert all(len(t) == 16 for t in t1)


def _digest_key(w):
    M = (1 << 64) - 1
    z = (0x9E3779B97F4A7C15 * (w + 1)) & M
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
    z ^= z >> 31
    return (z & 0xFFFFFFFF) | 0x00010001


def _digest(rank, lead, words):
    """DESIGN.md §7, written out: words = [(w, 32-bit value)]."""
    h = 0
    for w, x in words:
        k = _digest_key(w)
        h = (h + (x & 0xFFFF) * (k & 0xFFFF) + (x >> 16) * (k >> 16)) & 0xFFFFFFFF
    x = (h + (rank & 0xFFFFFFFF) * 0x9E3779B1 + (rank >> 32) * 0xEBCA77 + lead * 0xB2AE3D) & 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x85EBCA6B) & 0xFFFFFFFF
    x ^= x >> 13
    x = (x * 0xC2B2AE35) & 0xFFFFFFFF
    return x ^ (x >> 16)


@pytest.mark.parametrize("planet,n,keys", [("gcp", 3, 0), ("gcp", 5, 0), ("gcp", 5, 1), ("gcp", 2, 1),
                                           ("syn128", 6, 1), ("syn128", 6, 0)])
def test_sweep_digest_is_the_written_definition(planet, n, keys):
    """The oracle sweep's digest (the certificate every device sweep is checked
    against) equals DESIGN.md §7's formula applied to the oracle's own
    per-config moments: slot s's sum at word 2s and its folded sum of squares
    at 2s + 1, every leader of the extended key set at 40 + 2 (16 f + l)."""
    p = Planet.new() if planet == "gcp" else Planet.synthetic(128)
    o = O.OraclePlanet.of(p)
    s = np.arange(p.R, dtype=np.uint32)
    rb = 0 if planet == "gcp" else 2_711_805_600
    re = rb + min(600, _lib.binomial(p.R, n))
    _, _, dig = o.sweep(s, s, n, rb, re, [(1, 0)], 4, threads=2, keys=keys)
    cfgs = np.array([O.colex_unrank(r, n, p.R) for r in range(rb, re)], dtype=np.uint32)
    s1, s2, a1, a2, lead = o.moments_x(cfgs, s, threads=2)
    none = np.iinfo(np.uint64).max
    mf = min(n // 2, 2)
    want = 0
    for i, r in enumerate(range(rb, re)):
        words = []
        for sl in range(20 if keys else 10):
            if s1[i, sl] == none:
                continue
            q = int(s2[i, sl])
            words += [(2 * sl, int(s1[i, sl]) & 0xFFFFFFFF), (2 * sl + 1, (q ^ (q >> 32)) & 0xFFFFFFFF)]
        if keys:
            for f in range(mf):
                for l in range(n):
                    q = int(a2[i, f, l])
                    w = 40 + 2 * (16 * f + l)
                    words += [(w, int(a1[i, f, l]) & 0xFFFFFFFF), (w + 1, (q ^ (q >> 32)) & 0xFFFFFFFF)]
        want += _digest(r, int(lead[i]), words)
    assert dig == want % (1 << 64)


@pytest.mark.parametrize("keys", [0, 1])
def test_sweep_ranks_equals_sweep_on_a_range(keys):
    """oracle_sweep_ranks (the CPU baseline's seeded uniform sample) does the
    streaming sweep's per-config work: over an explicit list of a range's
    ranks, shuffled, it returns the range sweep's valid count, digest and top-K."""
    p = Planet.new()
    o = O.OraclePlanet.of(p)
    s = np.arange(p.R, dtype=np.uint32)
    objs = [(0, 0), (1, 0), (1, 1), (2, 0), (1, 4)] + ([(1, 10), (1, 13), (1, 18)] if keys else [])
    want = o.sweep(s, s, 5, 1000, 3000, objs, 16, threads=2, keys=keys)
    ranks = np.random.default_rng(7).permutation(np.arange(1000, 3000, dtype=np.uint64))
    got = o.sweep_ranks(s, s, 5, ranks, objs, 16, threads=3, keys=keys)
    assert got == want
    with pytest.raises(Exception):
        o.sweep_ranks(s, s, 5, np.array([15504], np.uint64), objs, 16)  # C(20, 5): out of range
