"""The `.data` cache format (search.rs:479-512): bincode 1.x of `Search`.

CPU: hand-derived known-answer bytes (bincode 1.x default options + serde
derive rules; no Rust-written `.data` ships with the reference, so the layout is
pinned by these bytes, not by a reference fixture), a round trip of oracle
histograms, and the error behaviour.  GPU: `Search(save_search=True)` writes the
file from device-computed histograms, which must equal the oracle's, and a
second `Search` loads it and reproduces the reference's golden ranking.
"""
import os
import struct

import numpy as np
import pytest

import oracle as O
from fantoch_amd import bincode
from fantoch_amd.planet import Planet

KEYS_N5 = ["af1", "ff1", "af2", "ff2", "e"]


def u64(x):
    return struct.pack("<Q", x)


def s(x):
    return u64(len(x)) + x.encode()


def test_histogram_bytes():
    # Histogram::from([10, 10, 20]) = BTreeMap {10: 2, 20: 1}
    got = bincode.encode_search([(["a"], {3: [(["c", "b", "a"], {"ff1": bincode.histogram_pairs([20, 10, 10])})]})])
    want = (u64(1)                                   # Vec<(Vec<Region>, Configs)> len
            + u64(1) + s("a")                        # clients
            + u64(1) + u64(3)                        # HashMap len, key n=3
            + u64(1)                                 # Vec<ConfigAndStats> len
            + u64(3) + s("a") + s("b") + s("c")      # BTreeSet<Region>: sorted
            + u64(1) + s("ff1")                      # ProtocolStats: 1 key
            + u64(2) + u64(10) + u64(2) + u64(20) + u64(1))
    assert got == want


def test_protocol_stats_key_order_is_byte_order():
    st = {k: bincode.histogram_pairs([1]) for k in ["ffC", "e", "af1C", "af1", "eC", "ff1"]}
    got = bincode.encode_search([([], {5: [(["x"], st)]})])
    rd = bincode._Reader(got)
    assert rd.u64() == 1 and rd.u64() == 0 and rd.u64() == 1 and rd.u64() == 5 and rd.u64() == 1
    assert rd.u64() == 1 and rd.str() == "x"
    keys = []
    for _ in range(rd.u64()):
        keys.append(rd.str())
        rd.histogram()
    assert keys == ["af1", "af1C", "e", "eC", "ff1", "ffC"]


def _oracle_all_configs(p, o, n, step=1):
    from itertools import combinations
    srv = np.arange(p.R, dtype=np.uint32)
    cfg = np.array(list(combinations(range(p.R), n))[::step], dtype=np.uint32)
    vals, _ = O.OraclePlanet.compute_stats(o, cfg, srv)
    return cfg, vals, oracle_stats(vals, n, p.R)


def oracle_stats(vals, n, nc):
    mf = min(n // 2, 2)
    out = []
    for row in vals:
        st = {}
        for slot in range(10):
            k = KEYS_N5[slot % 5]
            if k[0] != "e" and int(k[-1]) > mf:
                continue
            seg = row[slot * nc:(slot + 1) * nc] if slot < 5 else row[5 * nc + (slot - 5) * n:5 * nc + (slot - 4) * n]
            st[k + ("" if slot < 5 else "C")] = bincode.histogram_pairs(seg)
        out.append(st)
    return out


def test_round_trip_oracle_histograms():
    p = Planet.new()
    o = O.OraclePlanet.of(p)
    data = []
    for n in (3, 5):
        cfg, _, stats = _oracle_all_configs(p, o, n, step=7)
        data.append((n, [([p.names[i] for i in c], st) for c, st in zip(cfg, stats)]))
    ac = [(list(p.names), dict(data))]
    buf = bincode.encode_search(ac)
    back = bincode.read_search(buf)
    assert len(back) == 1 and back[0][0] == list(p.names)
    for n, lst in data:
        got = back[0][1][n]
        assert len(got) == len(lst)
        for (c0, s0), (c1, s1) in zip(lst, got):
            assert sorted(c0) == c1
            assert sorted(s0) == sorted(s1)
            for k in s0:
                assert np.array_equal(s0[k], s1[k])
    assert bincode.encode_search(back) == buf


def test_errors_truncated_and_trailing():
    buf = bincode.encode_search([(["a"], {3: [(["a", "b", "c"], {"e": bincode.histogram_pairs([1, 2])})]})])
    for cut in (1, 8, 9, len(buf) - 1):
        with pytest.raises(bincode.BincodeError):
            bincode.read_search(buf[:cut])
    with pytest.raises(bincode.BincodeError):
        bincode.read_search(buf + b"\0")
    # a length larger than the input is rejected before allocating
    with pytest.raises(bincode.BincodeError):
        bincode.read_search(u64(1 << 60))


def test_announced_length_must_match():
    class Short:
        def __len__(self):
            return 2

        def __iter__(self):
            yield ["a"], {}

    with pytest.raises(bincode.BincodeError):
        bincode.encode_search([([], {3: Short()})])


# ---------------------------------------------------------------- GPU -----
@pytest.mark.gpu
def test_search_save_and_load_data(tmp_path, monkeypatch):
    """search.rs:753-772 (`search_save`) through the GPU path, plus the file's
    histograms against the oracle and the golden ranking after a reload."""
    import json

    from fantoch_amd.bote import FTMetric, RankingParams, Search, SearchInput

    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_goldens.json")))["search"]
    monkeypatch.chdir(tmp_path)
    s1 = Search(3, 13, SearchInput.R13C13, save_search=True)
    fn = tmp_path / "3_13_R13C13.data"
    assert fn.exists()
    data = bincode.read_search(fn.read_bytes())
    p = s1.planet
    o = O.OraclePlanet.of(p)
    clients, configs = data[0]
    assert clients == [r.name for r in s1.all_configs[0][0]]
    cli = p.idxs(clients)
    assert sorted(configs) == [3, 5, 7, 9, 11, 13]
    for n, lst in configs.items():
        cfg_ids = np.array([p.idxs(names) for names, _ in lst], dtype=np.uint32)
        vals, _ = o.compute_stats(cfg_ids, cli)
        want = oracle_stats(vals, n, len(cli))
        for (names, st), w in zip(lst, want):
            assert sorted(st) == sorted(w)
            for k in w:
                assert np.array_equal(st[k], w[k]), (n, names, k)
    # reload: same means (bit-exact), COVs (1e-12), stats, and the golden ranking
    s2 = Search(3, 13, SearchInput.R13C13)
    for n in configs:
        a, b = s1.all_configs[0][1][n], s2.all_configs[0][1][n]
        assert np.array_equal(a["cfg"], b["cfg"])
        assert np.array_equal(a["mean"].view(np.uint64), b["mean"].view(np.uint64))
        assert np.array_equal(a["s1"], b["s1"])
        np.testing.assert_allclose(b["cov"], a["cov"], rtol=1e-12)
    params = RankingParams.new(110, 35, 0, 15, 3, 13, FTMetric.F1F2)
    score, css, _ = s2.sorted_evolving_configs(params)[0]
    assert score.round() == gold["score"]
    for cs in css:
        if len(cs.config) == 5:
            assert Search.stats_fmt(cs.stats, 5) == gold["stats_fmt_n5"]
    # re-saving the loaded search reproduces the file byte for byte
    s2.save_data(str(tmp_path / "again.data"))
    assert (tmp_path / "again.data").read_bytes() == fn.read_bytes()
