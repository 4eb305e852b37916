"""`Bote`, `Search` and the streaming GPU sweep.

Mirror of the `fantoch_bote` crate surface (reference `fantoch_bote/src/lib.rs`
and `search.rs`) on top of the C ABI in include/bote_hip.h.  Every latency,
quorum, leader choice, histogram moment, score and top-K selection is computed
by the gfx950 kernels in libbote_hip.so; this module marshals arguments, builds
the host-side `Histogram`/`ProtocolStats` result types and runs the ranking
chain of `Search::sorted_evolving_configs` over device-computed stats.
"""
from __future__ import annotations

import ctypes as C
import enum
import itertools
import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib, bincode
from ._lib import check, lib, ptr, u32
from .metrics import F64, Histogram, Stats
from .planet import Planet, Region
from .protocol import ClientPlacement, Protocol, ProtocolStats

SLOT_KEYS = [(Protocol.Atlas, 1), (Protocol.FPaxos, 1), (Protocol.Atlas, 2), (Protocol.FPaxos, 2),
             (Protocol.EPaxos, 0)]


def max_f(n: int) -> int:
    """search.rs:474-477"""
    return min(n // 2, 2)


class FTMetric(enum.Enum):
    """search.rs:652-666"""
    F1 = 1
    F1F2 = 2

    def fs(self, n: int) -> List[int]:
        return list(range(1, min(n // 2, self.value) + 1))


@dataclass
class RankingParams:
    """search.rs:617-649"""
    min_mean_fpaxos_improv: float
    min_mean_epaxos_improv: float
    min_fairness_fpaxos_improv: float
    min_mean_decrease: float
    min_n: int
    max_n: int
    ft_metric: FTMetric

    @classmethod
    def new(cls, min_mean_fpaxos_improv: int, min_mean_epaxos_improv: int, min_fairness_fpaxos_improv: int,
            min_mean_decrease: int, min_n: int, max_n: int, ft_metric: FTMetric) -> "RankingParams":
        return cls(float(min_mean_fpaxos_improv), float(min_mean_epaxos_improv), float(min_fairness_fpaxos_improv),
                   float(min_mean_decrease), min_n, max_n, ft_metric)


# --------------------------------------------------------------- planet ---
class DevicePlanet:
    """A `Planet` resident on one GPU (bote_planet_create)."""

    def __init__(self, planet: Planet, device: int = 0):
        self.planet = planet
        self.device = device
        h = C.c_void_p()
        check(lib().bote_planet_create(planet.lat, planet.R, device, C.byref(h)))
        self.h = h

    def __del__(self):
        try:
            if self.h:
                lib().bote_planet_destroy(self.h)
                self.h = None
        except Exception:
            pass


# ----------------------------------------------------------------- eval ---
@dataclass
class EvalResult:
    """Device outputs of `bote_eval` for a batch of configurations."""
    n: int
    nc: int
    vals: Optional[np.ndarray]   # (ncfg, 5*nc + 5*n) uint32
    leader: np.ndarray           # (ncfg,) position inside the config
    s1: np.ndarray               # (ncfg, 10) uint64
    s2: np.ndarray               # (ncfg, 10) uint64
    mean: np.ndarray             # (ncfg, 10) f64 (bit-exact Histogram::mean)
    cov: np.ndarray              # (ncfg, 10) f64
    score: Optional[np.ndarray]
    valid: Optional[np.ndarray]

    def slot_values(self, i: int, slot: int) -> np.ndarray:
        nc, n = self.nc, self.n
        row = self.vals[i]
        if slot < 5:
            return row[slot * nc:(slot + 1) * nc]
        return row[5 * nc + (slot - 5) * n:5 * nc + (slot - 4) * n]

    def protocol_stats(self, i: int) -> ProtocolStats:
        st = ProtocolStats.new()
        for slot in range(10):
            proto, f = SLOT_KEYS[slot % 5]
            if proto is not Protocol.EPaxos and f > max_f(self.n):
                continue
            placement = ClientPlacement.Input if slot < 5 else ClientPlacement.Colocated
            st.insert(proto, f, placement, Histogram.from_values(self.slot_values(i, slot).tolist()))
        return st


def eval_configs(dp: DevicePlanet, servers: Sequence[int], clients: Sequence[int], n: int,
                 configs: Optional[np.ndarray] = None, rank_begin: int = 0, ncfg: Optional[int] = None,
                 ranking: Optional[RankingParams] = None, values: bool = True) -> EvalResult:
    """`Search::compute_stats` over a batch (explicit position lists or colex ranks)."""
    srv, cli = u32(servers), u32(clients)
    if configs is not None:
        cfg = np.ascontiguousarray(np.asarray(configs, dtype=np.uint32).reshape(-1, n))
        ncfg = cfg.shape[0]
        cptr = ptr(cfg)
    else:
        cfg, cptr = None, None
        if ncfg is None:
            ncfg = _lib.binomial(len(srv), n) - rank_begin
    nc = len(cli)
    vals = np.zeros((ncfg, 5 * nc + 5 * n), np.uint32) if values else None
    lead = np.zeros(ncfg, np.uint32)
    s1 = np.zeros((ncfg, 10), np.uint64)
    s2 = np.zeros((ncfg, 10), np.uint64)
    mean = np.zeros((ncfg, 10), np.float64)
    cov = np.zeros((ncfg, 10), np.float64)
    score = np.zeros(ncfg, np.float64) if ranking else None
    valid = np.zeros(ncfg, np.uint8) if ranking else None
    rp = C.byref(_lib.ranking_params_c(ranking)) if ranking else None
    check(lib().bote_eval(dp.h, srv, len(srv), cli, nc, n, cptr, rank_begin, ncfg, rp, ptr(vals), ptr(lead),
                          ptr(s1), ptr(s2), ptr(mean), ptr(cov), ptr(score), ptr(valid)))
    return EvalResult(n, nc, vals, lead, s1, s2, mean, cov, score, valid)


@dataclass
class LeaderlessResult:
    """bote_eval_leaderless outputs: per config and quorum size."""
    n: int
    nc: int
    quorum_sizes: List[int]
    vals: Optional[np.ndarray]   # (ncfg, nq, nc + n) uint32: Input clients, then Colocated (config order)
    s1: np.ndarray               # (ncfg, nq, 2) uint64: [Input, Colocated]
    s2: np.ndarray               # (ncfg, nq, 2) uint64


def eval_leaderless(dp: DevicePlanet, servers: Sequence[int], clients: Sequence[int], n: int,
                    quorum_sizes: Sequence[int], configs: Optional[np.ndarray] = None, rank_begin: int = 0,
                    ncfg: Optional[int] = None, values: bool = True) -> LeaderlessResult:
    """`Bote::leaderless` (lib.rs:38-59) for a batch of configurations and up to
    8 quorum sizes at once (Tempo's fast/tiny/write quorums, config.rs:317-329)."""
    srv, cli, qs = u32(servers), u32(clients), u32(quorum_sizes)
    if configs is not None:
        cfg = np.ascontiguousarray(np.asarray(configs, dtype=np.uint32).reshape(-1, n))
        ncfg = cfg.shape[0]
        cptr = ptr(cfg)
    else:
        cfg, cptr = None, None
        if ncfg is None:
            ncfg = _lib.binomial(len(srv), n) - rank_begin
    nc, nq = len(cli), len(qs)
    vals = np.zeros((ncfg, nq, nc + n), np.uint32) if values else None
    s1 = np.zeros((ncfg, nq, 2), np.uint64)
    s2 = np.zeros((ncfg, nq, 2), np.uint64)
    check(lib().bote_eval_leaderless(dp.h, srv, len(srv), cli, nc, n, cptr, rank_begin, ncfg, qs, nq, ptr(vals),
                                     ptr(s1), ptr(s2)))
    return LeaderlessResult(n, nc, [int(q) for q in qs], vals, s1, s2)


@dataclass
class KeysResult:
    """bote_eval_keys outputs: exact moments of the extended key set."""
    n: int
    s1: np.ndarray       # (ncfg, 20) uint64; ~0 where a slot is absent
    s2: np.ndarray       # (ncfg, 20) uint64
    al_s1: np.ndarray    # (ncfg, 2, n) uint64: every leader's FPaxos sum, f = 1, 2, config order
    al_s2: np.ndarray
    leader: np.ndarray   # (ncfg,) the COV-best FPaxos leader (compute_stats)


def eval_keys(dp: DevicePlanet, servers: Sequence[int], clients: Sequence[int], n: int,
              configs: Optional[np.ndarray] = None, rank_begin: int = 0, ncfg: Optional[int] = None,
              keys: int = _lib.KEYS_TEMPO_ALL_LEADERS) -> KeysResult:
    """The extended key set per config (BASELINE config 5: Tempo tiny/write
    keys, config.rs:317-329, and FPaxos all leaders, lib.rs:129-150) as exact
    moments, from the device (bote_eval_keys)."""
    srv, cli = u32(servers), u32(clients)
    if configs is not None:
        cfg = np.ascontiguousarray(np.asarray(configs, dtype=np.uint32).reshape(-1, n))
        ncfg = cfg.shape[0]
        cptr = ptr(cfg)
    else:
        cfg, cptr = None, None
        if ncfg is None:
            ncfg = _lib.binomial(len(srv), n) - rank_begin
    ns_ = _lib.NSLOTS_X if keys else 10
    s1 = np.zeros((ncfg, ns_), np.uint64)
    s2 = np.zeros((ncfg, ns_), np.uint64)
    a1 = np.zeros((ncfg, 2, n), np.uint64)
    a2 = np.zeros((ncfg, 2, n), np.uint64)
    lead = np.zeros(ncfg, np.uint32)
    check(lib().bote_eval_keys(dp.h, srv, len(srv), cli, len(cli), n, cptr, rank_begin, ncfg, keys, ptr(lead),
                               ptr(s1), ptr(s2), ptr(a1) if keys else None, ptr(a2) if keys else None))
    return KeysResult(n, s1, s2, a1, a2, lead)


def tempo_quorums(n: int) -> List[Tuple[Protocol, int, int]]:
    """(protocol, f, quorum size) of Tempo's fast (non-tiny, tiny) and write
    quorums for f = 1..max_f(n) (config.rs:317-329; max_f: search.rs:474-477)."""
    out = []
    for f in range(1, max_f(n) + 1):
        for proto in (Protocol.Tempo, Protocol.TempoTiny, Protocol.TempoWrite):
            out.append((proto, f, proto.quorum_size(n, f)))
    return out


def tempo_stats(dp: DevicePlanet, servers: Sequence[int], clients: Sequence[int], n: int,
                configs: np.ndarray) -> List[ProtocolStats]:
    """Tempo keys (`tf{f}`, `ttf{f}`, `twf{f}` and their `C` variants) for each
    configuration, from the device (bote_eval_leaderless)."""
    tq = tempo_quorums(n)
    qs = sorted({q for _, _, q in tq})
    r = eval_leaderless(dp, servers, clients, n, qs, configs=configs)
    nc = len(u32(clients))
    out = []
    for i in range(r.vals.shape[0]):
        st = ProtocolStats.new()
        for proto, f, q in tq:
            row = r.vals[i, qs.index(q)]
            st.insert(proto, f, ClientPlacement.Input, Histogram.from_values(row[:nc].tolist()))
            st.insert(proto, f, ClientPlacement.Colocated, Histogram.from_values(row[nc:].tolist()))
        out.append(st)
    return out


# ----------------------------------------------------------------- Bote ---
class Bote:
    """lib.rs:16-186 — the analytic latency model over a device planet."""

    def __init__(self, planet: Optional[Planet] = None, device: int = 0):
        self.planet = planet if planet is not None else Planet.new()
        self.dp = DevicePlanet(self.planet, device)

    @classmethod
    def new(cls, device: int = 0) -> "Bote":
        return cls(Planet.new(), device)

    @classmethod
    def from_(cls, planet: Planet, device: int = 0) -> "Bote":
        return cls(planet, device)

    def _ids(self, regions) -> np.ndarray:
        return self.planet.idxs(regions)

    def quorum_latency(self, frm, regions: Sequence, quorum_size: int) -> int:
        """lib.rs:155-163"""
        out = np.zeros(1, np.uint64)
        fr = u32([self.planet.idx(frm)])
        regs = self._ids(regions)
        check(lib().bote_quorum_latencies(self.dp.h, fr, 1, regs, len(regs), quorum_size, out))
        return int(out[0])

    def leaderless(self, servers: Sequence, clients: Sequence, quorum_size: int) -> List[Tuple[Region, int]]:
        """lib.rs:38-59"""
        s, c = self._ids(servers), self._ids(clients)
        out = np.zeros(len(c), np.uint64)
        check(lib().bote_leaderless(self.dp.h, s, len(s), c, len(c), quorum_size, out))
        return [(Region(self.planet.names[i]), int(v)) for i, v in zip(c, out)]

    def leader(self, leader, servers: Sequence, clients: Sequence, quorum_size: int) -> List[Tuple[Region, int]]:
        """lib.rs:67-89"""
        s, c = self._ids(servers), self._ids(clients)
        out = np.zeros(len(c), np.uint64)
        check(lib().bote_leader(self.dp.h, self.planet.idx(leader), s, len(s), c, len(c), quorum_size, out))
        return [(Region(self.planet.names[i]), int(v)) for i, v in zip(c, out)]

    def all_leaders_stats(self, servers: Sequence, clients: Sequence, quorum_size: int) -> List[Tuple[Region, Histogram]]:
        """lib.rs:129-150"""
        s, c = self._ids(servers), self._ids(clients)
        out = np.zeros(len(s) * len(c), np.uint64)
        check(lib().bote_all_leaders(self.dp.h, s, len(s), c, len(c), quorum_size, out))
        out = out.reshape(len(s), len(c))
        return [(Region(self.planet.names[l]), Histogram.from_values(out[i].tolist())) for i, l in enumerate(s)]

    def best_leader(self, servers: Sequence, clients: Sequence, quorum_size: int,
                    stats_sort_by: Stats) -> Tuple[Region, Histogram]:
        """lib.rs:99-121"""
        s, c = self._ids(servers), self._ids(clients)
        pos = C.c_uint32()
        lat = np.zeros(max(len(c), 1), np.uint64)
        check(lib().bote_best_leader(self.dp.h, s, len(s), c, len(c), quorum_size, stats_sort_by.value,
                                     C.byref(pos), ptr(lat)))
        return Region(self.planet.names[s[pos.value]]), Histogram.from_values(lat[:len(c)].tolist())


# --------------------------------------------------------------- Search ---
class SearchInput(enum.Enum):
    """search.rs:516-611"""
    R13C13 = "R13C13"
    R17C17 = "R17C17"
    R20C20 = "R20C20"
    R17CMaxN = "R17CMaxN"

    def __str__(self):
        return self.value

    def get_inputs(self, max_n: int, planet: Planet) -> Tuple[Optional[List[Region]], List[List[Region]]]:
        regions13 = [Region(x) for x in (
            "asia-southeast1", "europe-west4", "southamerica-east1", "australia-southeast1", "europe-west2",
            "asia-south1", "us-east1", "asia-northeast1", "europe-west1", "asia-east1", "us-west1",
            "europe-west3", "us-central1")]
        regions17 = [Region(x) for x in (
            "asia-east1", "asia-northeast1", "asia-south1", "asia-southeast1", "australia-southeast1",
            "europe-north1", "europe-west1", "europe-west2", "europe-west3", "europe-west4",
            "northamerica-northeast1", "southamerica-east1", "us-central1", "us-east1", "us-east4", "us-west1",
            "us-west2")]
        all_regions = sorted(planet.regions())
        if self is SearchInput.R13C13:
            return regions13, [list(regions13)]
        if self is SearchInput.R17C17:
            return regions17, [list(regions17)]
        if self is SearchInput.R20C20:
            return all_regions, [list(all_regions)]
        return None, [list(c) for c in itertools.combinations(regions17, max_n)]


@dataclass
class ConfigAndStats:
    """(BTreeSet<Region>, ProtocolStats) of search.rs:24-25, with lazy stats."""
    config: List[Region]          # name order (BTreeSet iteration order)
    mask: int                     # bitmask of region ids
    _search: "Search"
    _key: Tuple[int, int, int]    # (client set index, n, config index)

    @property
    def stats(self) -> ProtocolStats:
        return self._search._stats(*self._key)

    def __iter__(self):
        yield self.config
        yield self.stats


def _slot_key(slot: int) -> str:
    proto, f = SLOT_KEYS[slot % 5]
    return ProtocolStats.key(proto, f, ClientPlacement.Input if slot < 5 else ClientPlacement.Colocated)


class _DeviceConfigStats:
    """The `Vec<(BTreeSet<Region>, ProtocolStats)>` of one n, produced lazily in
    device batches (bote_eval with per-client outputs) for the bincode writer."""

    def __init__(self, search: "Search", ci: int, n: int):
        self.s, self.ci, self.n = search, ci, n
        self.d = search.all_configs[ci][1][n]

    def __len__(self):
        return len(self.d["cfg"])

    def __iter__(self):
        d, n, names = self.d, self.n, self.s.planet.names
        slots = [s for s in range(10) if not (SLOT_KEYS[s % 5][0] is not Protocol.EPaxos and
                                                SLOT_KEYS[s % 5][1] > max_f(n))]
        for b in range(0, len(d["cfg"]), Search.BATCH):
            cfg = d["cfg"][b:b + Search.BATCH]
            r = eval_configs(self.s.dp, d["srv"], d["cli"], n, configs=cfg)
            for i in range(len(cfg)):
                stats = {_slot_key(s): bincode.histogram_pairs(r.slot_values(i, s)) for s in slots}
                yield [names[d["srv"][p]] for p in cfg[i]], stats


class Search:
    """search.rs:41-512 — exhaustive search, computed on the GPU."""

    BATCH = 1 << 18
    CHAIN_FETCH = 1 << 16  # chains fetched with the count in one device call (evolving_chain_arrays)

    def __init__(self, min_n: int, max_n: int, search_input: SearchInput, save_search: bool = False,
                 lat_dir: Optional[str] = None, device: int = 0, planet: Optional[Planet] = None):
        self.min_n, self.max_n, self.search_input = min_n, max_n, search_input
        self.planet = planet if planet is not None else (Planet.from_dir(lat_dir) if lat_dir else Planet.new())
        self.dp = DevicePlanet(self.planet, device)
        filename = self.filename(min_n, max_n, search_input)
        servers, all_clients = search_input.get_inputs(max_n, self.planet)
        self.all_configs: List[Tuple[List[Region], Dict[int, dict]]] = []
        self._file_stats: Dict[Tuple[int, int, int], dict] = {}
        loaded = self._load(filename) if os.path.exists(filename) else None
        if loaded is not None:
            self.all_configs = loaded
        else:
            for clients in all_clients:
                srv = servers if servers is not None else clients
                self.all_configs.append((clients, self._compute_configs(min_n, max_n, srv, clients)))
            if save_search:
                self._save(filename)
        self._stats_cache: Dict[Tuple[int, int, int], ProtocolStats] = {}

    @staticmethod
    def filename(min_n: int, max_n: int, search_input: SearchInput) -> str:
        """search.rs:479-485 — the reference's bincode cache name."""
        return f"{min_n}_{max_n}_{search_input}.data"

    # search.rs:234-260 — configs of each n in lexicographic order of positions.
    def _compute_configs(self, min_n: int, max_n: int, servers: Sequence[Region], clients: Sequence[Region]):
        srv_ids = self.planet.idxs(servers)
        cli_ids = self.planet.idxs(clients)
        out = {}
        for n in range(min_n, max_n + 1, 2):
            if n > len(srv_ids):
                out[n] = dict(cfg=np.zeros((0, n), np.uint32), mean=np.zeros((0, 10)), s1=np.zeros((0, 10), np.uint64),
                              srv=srv_ids, cli=cli_ids)
                continue
            cfg = np.array(list(itertools.combinations(range(len(srv_ids)), n)), dtype=np.uint32).reshape(-1, n)
            means, s1s, covs = [], [], []
            for b in range(0, len(cfg), self.BATCH):
                r = eval_configs(self.dp, srv_ids, cli_ids, n, configs=cfg[b:b + self.BATCH], values=False)
                means.append(r.mean)
                s1s.append(r.s1)
                covs.append(r.cov)
            out[n] = dict(cfg=cfg, mean=np.concatenate(means), s1=np.concatenate(s1s), cov=np.concatenate(covs),
                          srv=srv_ids, cli=cli_ids)
        return out

    def _save(self, filename: str):
        """search.rs:500-512: bincode `Search` (fantoch_amd/bincode.py), full per-config
        histograms from the device (bote_eval with per-client outputs)."""
        with open(filename, "wb") as w:
            bincode.write_search(w, [([r.name for r in clients], {n: _DeviceConfigStats(self, ci, n)
                                                                   for n in configs})
                                     for ci, (clients, configs) in enumerate(self.all_configs)])

    def save_data(self, filename: Optional[str] = None) -> str:
        """Write this search as the reference's `.data` file; returns its path."""
        filename = filename or self.filename(self.min_n, self.max_n, self.search_input)
        self._save(filename)
        return filename

    def _load(self, filename: str):
        """search.rs:487-498: read a bincode `Search` (written by the Rust crate or by
        `_save`).  Its histograms are kept as the configs' stats; per-key means,
        sums and COVs are derived from them (Histogram::mean / cov)."""
        with open(filename, "rb") as fh:
            data = bincode.read_search(fh.read())
        servers, _ = self.search_input.get_inputs(self.max_n, self.planet)
        out = []
        for ci, (client_names, configs) in enumerate(data):
            clients = [Region(x) for x in client_names]
            cli_ids = self.planet.idxs(clients)
            srv_ids = self.planet.idxs(servers if servers is not None else clients)
            pos_of = {int(r): p for p, r in enumerate(srv_ids)}
            name_id = {nm: i for i, nm in enumerate(self.planet.names)}
            for names, _ in (x for lst in configs.values() for x in lst):
                for x in names:
                    if x not in name_id or name_id[x] not in pos_of:
                        raise ValueError(f"{filename}: region {x!r} is not a server of this search's planet")
            per_n = {}
            for n, lst in configs.items():
                cfg = np.zeros((len(lst), n), np.uint32)
                # slots a config does not have (f=2 at n<4): sums all-ones, mean/COV NaN,
                # as bote_eval leaves them
                s1 = np.full((len(lst), 10), np.iinfo(np.uint64).max, np.uint64)
                mean = np.full((len(lst), 10), np.nan)
                cov = np.full((len(lst), 10), np.nan)
                for i, (names, stats) in enumerate(lst):
                    if len(names) != n:
                        raise ValueError(f"{filename}: config of size {len(names)} under n={n}")
                    # servers-list order = the order the reference's combination() yields
                    cfg[i] = sorted(pos_of[name_id[x]] for x in names)
                    self._file_stats[(ci, n, i)] = stats
                    for slot in range(10):
                        k = _slot_key(slot)
                        if k in stats:
                            h = Histogram({int(v): int(c) for v, c in stats[k]})
                            s1[i, slot] = sum(int(v) * int(c) for v, c in stats[k])
                            mean[i, slot] = h.mean().value()
                            cov[i, slot] = h.cov().value()
                per_n[n] = dict(cfg=cfg, mean=mean, s1=s1, cov=cov, srv=srv_ids, cli=cli_ids)
            out.append((clients, per_n))
        return out

    def _stats(self, ci: int, n: int, i: int) -> ProtocolStats:
        key = (ci, n, i)
        if key not in self._stats_cache and key in self._file_stats:
            st = ProtocolStats.new()
            st.map = {k: Histogram({int(v): int(c) for v, c in h}) for k, h in self._file_stats[key].items()}
            self._stats_cache[key] = st
        if key not in self._stats_cache:
            d = self.all_configs[ci][1][n]
            r = eval_configs(self.dp, d["srv"], d["cli"], n, configs=d["cfg"][i:i + 1])
            self._stats_cache[key] = r.protocol_stats(0)
        return self._stats_cache[key]

    def _config_set(self, ci: int, n: int, i: int) -> ConfigAndStats:
        d = self.all_configs[ci][1][n]
        ids = sorted(int(d["srv"][p]) for p in d["cfg"][i])
        mask = 0
        for r in ids:
            mask |= 1 << r
        return ConfigAndStats([Region(self.planet.names[r]) for r in ids], mask, self, (ci, n, i))

    @staticmethod
    def compute_stats(config: Sequence, all_clients: Sequence, bote: Bote, tempo: bool = False) -> ProtocolStats:
        """search.rs:262-319 for one configuration (config order = given order).
        tempo=True adds Tempo's keys (tempo_stats; BASELINE config 2)."""
        srv = bote.planet.idxs(config)
        cli = bote.planet.idxs(all_clients)
        n = len(srv)
        one = np.arange(n, dtype=np.uint32).reshape(1, n)
        st = eval_configs(bote.dp, srv, cli, n, configs=one).protocol_stats(0)
        if tempo:
            st.map.update(tempo_stats(bote.dp, srv, cli, n, one)[0].map)
        return st

    # ------------------------------------------------------------ ranking ---
    def _rank(self, configs: Dict[int, dict], p: RankingParams, ci: int):
        """search.rs:329-354: valid configs and their scores, per n, in enumeration order.
        Scores and validity come from the device (bote_eval with the ranking params);
        a search loaded from a .data file is ranked from the file's histograms only,
        as the reference ranks its stored ProtocolStats (compute_score_host)."""
        ranked = {}
        for n, d in configs.items():
            if not (p.min_n <= n <= p.max_n):
                continue
            cfg = d["cfg"]
            if len(cfg) == 0:
                ranked[n] = []
                continue
            if (ci, n, 0) in self._file_stats:
                out = []
                for i in range(len(cfg)):
                    ok, score = compute_score_host(n, self._stats(ci, n, i), p)
                    if ok:
                        out.append((score.value(), i))
                ranked[n] = out
                continue
            r = eval_configs(self.dp, d["srv"], d["cli"], n, configs=cfg, ranking=p, values=False)
            idx = np.nonzero(r.valid)[0]
            ranked[n] = [(float(r.score[i]), int(i)) for i in idx]
        return ranked

    def evolving_chain_arrays(self, p: RankingParams, limit: Optional[int] = None) -> List[dict]:
        """The device chain search (bote_evolving_chains) per client set, as
        arrays: {"ci", "total", "idx" (nout, 6) config indices per level (n = 3,
        5, .., 13) into all_configs[ci][1][n]["cfg"], "score" (nout,)}, each
        set's chains in the reference's order (score descending, equal scores
        in enumeration order).  `limit` caps the chains fetched per set."""
        assert p.min_n == 3 and p.max_n == 13
        u64p = C.POINTER(C.c_uint64)
        f64p = C.POINTER(C.c_double)
        out = []
        for ci, (clients, configs) in enumerate(self.all_configs):
            ranked = self._rank(configs, p, ci)
            counts = np.zeros(6, np.uint32)
            keep, arrs = [], []
            for lvl in range(6):
                n = 3 + 2 * lvl
                lst = ranked.get(n, [])
                idx = np.array([i for _, i in lst], dtype=np.int64)
                d = configs.get(n)
                if len(idx) and len(d["srv"]) > 64:
                    raise ValueError("chain search needs a server list of at most 64 regions")
                pos = d["cfg"][idx].astype(np.uint64) if len(idx) else np.zeros((0, n), np.uint64)
                mask = np.ascontiguousarray(np.bitwise_or.reduce(np.uint64(1) << pos, axis=1)
                                            if len(idx) else np.zeros(0, np.uint64), dtype=np.uint64)
                score = np.ascontiguousarray([sc for sc, _ in lst], dtype=np.float64)
                mean = np.ascontiguousarray(d["mean"][idx][:, [0, 2]] if len(idx) else np.zeros((0, 2)),
                                            dtype=np.float64)
                counts[lvl] = len(idx)
                keep.append(idx)
                arrs.append((mask, score, mean))
            ns = len(configs[3]["srv"]) if 3 in configs else 0
            if counts.min() == 0 or ns == 0:
                continue
            masks = (u64p * 6)(*[x[0].ctypes.data_as(u64p) for x in arrs])
            scores = (f64p * 6)(*[x[1].ctypes.data_as(f64p) for x in arrs])
            means = (f64p * 6)(*[x[2].ctypes.data_as(f64p) for x in arrs])
            total = C.c_uint64()
            # one device chain search per set: fetch up to `cap` chains with the
            # count; only a set with more chains than the first cap (no limit
            # given) runs the search again, sized exactly
            cap = limit if limit is not None else self.CHAIN_FETCH
            out_idx = np.zeros((cap, 6), np.uint32)
            out_sc = np.zeros(cap, np.float64)
            check(lib().bote_evolving_chains(self.dp.device, ns, counts, masks, scores, means,
                                             float(p.min_mean_decrease), int(p.ft_metric.value), cap,
                                             ptr(out_idx) if cap else None, ptr(out_sc) if cap else None,
                                             C.byref(total)))
            if limit is None and total.value > cap:
                cap = total.value
                out_idx = np.zeros((cap, 6), np.uint32)
                out_sc = np.zeros(cap, np.float64)
                check(lib().bote_evolving_chains(self.dp.device, ns, counts, masks, scores, means,
                                                 float(p.min_mean_decrease), int(p.ft_metric.value), cap,
                                                 ptr(out_idx), ptr(out_sc), C.byref(total)))
            nout = min(cap, total.value)
            out_idx, out_sc = out_idx[:nout], out_sc[:nout]
            idx = np.stack([keep[lvl][out_idx[:, lvl]] for lvl in range(6)], axis=1) if nout else \
                np.zeros((0, 6), np.int64)
            out.append({"ci": ci, "total": total.value, "idx": idx, "score": out_sc})
        return out

    def chains_digest(self, arrays: dict) -> int:
        """Order-dependent digest of one client set's chains (the oracle's
        oracle_search_chains digest): h = bits(score); h = mix64(h ^ mask_l)
        over the 6 configs' region-id bitmasks; sum over k of mix64(h + k)."""
        ci = arrays["ci"]
        configs = self.all_configs[ci][1]
        h = np.ascontiguousarray(arrays["score"], dtype=np.float64).view(np.uint64).copy()
        for lvl in range(6):
            d = configs[3 + 2 * lvl]
            regs = d["srv"][d["cfg"][arrays["idx"][:, lvl]]].astype(np.uint64)
            m = np.bitwise_or.reduce(np.uint64(1) << regs, axis=1) if len(regs) else np.zeros(0, np.uint64)
            h = _mix64(h ^ m)
        k = np.arange(len(h), dtype=np.uint64)
        return int(np.sum(_mix64(h + k), dtype=np.uint64))

    def sorted_evolving_configs(self, p: RankingParams, limit: Optional[int] = None):
        """search.rs:97-178: chains n = 3 -> 5 -> ... -> 13 of supersets, highest
        score first (equal scores: client-set order, then enumeration order).
        The superset/min_mean_decrease joins and the ordering run on the device
        (bote_evolving_chains); `limit` caps the chains returned per client set."""
        found = []  # (orderable key, client set, position, score, chain)
        for a in self.evolving_chain_arrays(p, limit):
            ci = a["ci"]
            clients = self.all_configs[ci][0]
            keys = ~(_orderable(a["score"]))
            for k in range(len(a["score"])):
                chain = [self._config_set(ci, 3 + 2 * lvl, int(a["idx"][k, lvl])) for lvl in range(6)]
                found.append((int(keys[k]), ci, k, F64(float(a["score"][k])), chain, clients))
        found.sort(key=lambda x: (x[0], x[1], x[2]))
        return [(sc, chain, clients) for _, _, _, sc, chain, clients in found]

    @staticmethod
    def stats_fmt(stats: ProtocolStats, n: int) -> str:
        """search.rs:180-197"""
        out = ""
        for placement in ClientPlacement.all():
            fmt = ""
            for f in range(1, max_f(n) + 1):
                fmt += f"{stats.fmt(Protocol.Atlas, f, placement)} {stats.fmt(Protocol.FPaxos, f, placement)} "
            out += f"{fmt}{stats.fmt(Protocol.EPaxos, 0, placement)} "
        return out


def _mix64(z: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser on uint64 arrays (wrapping)."""
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def _orderable(x: np.ndarray) -> np.ndarray:
    """F64 total order as uint64 keys (NaN greatest; -0.0 == 0.0)."""
    x = np.asarray(x, dtype=np.float64) + 0.0
    x = np.where(np.isnan(x), np.float64("nan"), x)
    b = x.view(np.uint64)
    return np.where(b >> np.uint64(63), ~b, b | np.uint64(0x8000000000000000))


def compute_score_host(n: int, stats: ProtocolStats, p: RankingParams) -> Tuple[bool, F64]:
    """search.rs:421-472 on host histograms (for searches loaded from a .data
    file, whose stats are the file's, not the device's): F64 arithmetic in the
    reference's order; `>=` is the derived PartialOrd (plain f64)."""
    valid = True
    score = F64.zero()
    inp = ClientPlacement.Input
    for f in p.ft_metric.fs(n):
        atlas = stats.get(Protocol.Atlas, f, inp)
        fpaxos = stats.get(Protocol.FPaxos, f, inp)
        fmi = fpaxos.mean_improv(atlas)
        ffi = fpaxos.cov_improv(atlas)
        valid = valid and fmi.ge(F64(p.min_mean_fpaxos_improv)) and ffi.ge(F64(p.min_fairness_fpaxos_improv))
        emi = stats.get(Protocol.EPaxos, 0, inp).mean_improv(atlas)
        if n in (11, 13):
            valid = valid and emi.ge(F64(p.min_mean_epaxos_improv))
        score = score + (fmi + F64(30.0) * emi)
    return valid, score


# ---------------------------------------------------------------- sweep ---
DEFAULT_OBJECTIVES = [(_lib.OBJ_SCORE, 0), (_lib.OBJ_MEAN, _lib.SLOT_AF1), (_lib.OBJ_MEAN, _lib.SLOT_FF1),
                      (_lib.OBJ_COV, _lib.SLOT_AF1), (_lib.OBJ_MEAN, _lib.SLOT_E)]
DEFAULT_RANKING = RankingParams.new(110, 35, 0, 15, 3, 13, FTMetric.F1F2)
# BASELINE config 5 (the extended key set): the default objectives, then the
# best Tempo tiny (f = 1) and write (f = 2) means and the best mean under
# FPaxos's mean-optimal leader (all leaders), Input
CONFIG5_OBJECTIVES = DEFAULT_OBJECTIVES + [(_lib.OBJ_MEAN, _lib.SLOT_TT1), (_lib.OBJ_MEAN, _lib.SLOT_TW2),
                                           (_lib.OBJ_MEAN, _lib.SLOT_FL1)]


@dataclass
class SweepResult:
    tops: List[List[Tuple[int, int]]]  # per objective: (key, rank) ascending
    valid: int
    digest: int


class Sweep:
    """Streaming exhaustive search with a device top-K (bote_sweep_*)."""

    def __init__(self, dp: DevicePlanet, servers: Sequence[int], clients: Sequence[int], n: int,
                 objectives=DEFAULT_OBJECTIVES, K: int = 100, ranking: Optional[RankingParams] = DEFAULT_RANKING,
                 digest: bool = False, kernel: Optional[str] = None, keys: int = _lib.KEYS_BASE):
        """kernel: None/'auto' (the library's choice), or force 'generic', 'fast'
        or 'group' (every path is exact; bote_sweep_create_keys).  keys: the
        key set (_lib.KEYS_BASE, or KEYS_TEMPO_ALL_LEADERS for BASELINE config 5)."""
        self.dp, self.n, self.K, self.keys = dp, n, K, keys
        self.servers, self.clients = u32(servers), u32(clients)
        self.objectives = list(objectives)
        self.ranking, self.digest = ranking, bool(digest)
        objs = (_lib.Objective * max(len(self.objectives), 1))(*[_lib.Objective(k, s) for k, s in self.objectives])
        rp = C.byref(_lib.ranking_params_c(ranking)) if ranking is not None else None
        h = C.c_void_p()
        check(lib().bote_sweep_create_keys(dp.h, self.servers, len(self.servers), self.clients, len(self.clients), n,
                                           objs, len(self.objectives), K, rp, 1 if digest else 0,
                                           _lib.KERNELS[kernel], keys, C.byref(h)))
        self.h = h
        self.total = _lib.binomial(len(self.servers), n)

    def __del__(self):
        try:
            if self.h:
                lib().bote_sweep_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def run_checkpointed(self, path: str, rank_begin: int = 0, rank_end: Optional[int] = None,
                         chunk: int = 1 << 28, stop_after: Optional[int] = None) -> Optional[SweepResult]:
        """Resumable sweep of [rank_begin, rank_end) in rank chunks (SURVEY.md §5:
        the reference only memoises a finished search, search.rs:55-57; a long
        sweep here checkpoints its running top-K instead).  After each chunk the
        running result block, merged on the device, and the next rank are
        written atomically to `path`; a later call with the same sweep and range
        resumes there.  `stop_after` ends the call after that many chunks and
        returns None (an interruption, for tests)."""
        import torch

        re = self.total if rank_end is None else rank_end
        if not 0 <= rank_begin <= re <= self.total or chunk < 1:
            raise ValueError("bad rank range or chunk")
        rk = self.ranking
        # ranking params as raw f64 bits, plus the digest flag: a checkpoint
        # scored under other thresholds (or without the digest) is refused
        rbits = (np.array([rk.min_mean_fpaxos_improv, rk.min_mean_epaxos_improv, rk.min_fairness_fpaxos_improv,
                           rk.min_mean_decrease], np.float64).view(np.uint64).tolist() + [rk.ft_metric.value]
                 if rk is not None else [0xFFFFFFFFFFFFFFFF] * 5)
        ident = np.concatenate([np.array([self.n, self.K, rank_begin, re, len(self.servers), len(self.clients),
                                          int(self.digest), int(self.keys)] + rbits, np.uint64),
                                self.servers.astype(np.uint64), self.clients.astype(np.uint64),
                                np.asarray(self.objectives, np.uint64).reshape(-1),
                                np.asarray(self.dp.planet.lat, np.uint64).reshape(-1)])
        dev = torch.device("cuda", self.dp.device)
        st = torch.cuda.current_stream(dev).cuda_stream
        nb = self.result_bytes()
        pair = torch.empty(2 * nb, dtype=torch.uint8, device=dev)
        out = torch.empty(nb, dtype=torch.uint8, device=dev)
        nxt, have = rank_begin, False
        if os.path.exists(path):
            z = np.load(path, allow_pickle=False)
            if not np.array_equal(z["ident"], ident):
                raise ValueError(f"checkpoint {path} belongs to a different sweep")
            nxt = int(z["next"])
            pair[:nb].copy_(torch.from_numpy(np.ascontiguousarray(z["block"])))
            have = True
        chunks = 0
        while nxt < re or not have:
            e = min(re, nxt + chunk)
            self.launch(nxt, e, st)
            if have:
                self.result_device(pair.data_ptr() + nb, st)
                self.merge_device(pair.data_ptr(), 2, out.data_ptr(), st)
                pair[:nb].copy_(out)
            else:
                self.result_device(pair.data_ptr(), st)
                have = True
            nxt = e
            blk = pair[:nb].cpu().numpy()
            tmp = path + ".tmp"
            with open(tmp, "wb") as fh:
                np.savez(fh, ident=ident, next=np.uint64(nxt), block=blk)
            os.replace(tmp, path)
            chunks += 1
            if stop_after is not None and chunks >= stop_after and nxt < re:
                return None
        return self.parse_block(pair[:nb].cpu().numpy())

    def launch(self, rank_begin: int = 0, rank_end: Optional[int] = None, stream: Optional[int] = None):
        re = self.total if rank_end is None else rank_end
        check(lib().bote_sweep_launch(self.h, rank_begin, re, C.c_void_p(stream) if stream else None))

    def result(self, stream: Optional[int] = None) -> SweepResult:
        no = len(self.objectives)
        recs = (_lib.TopKRecord * (no * self.K))()
        cnt = np.zeros(max(no, 1), np.uint32)
        valid, digest = C.c_uint64(), C.c_uint64()
        check(lib().bote_sweep_result(self.h, C.c_void_p(stream) if stream else None, recs, ptr(cnt),
                                      C.byref(valid), C.byref(digest)))
        tops = [[(recs[o * self.K + i].key, recs[o * self.K + i].rank) for i in range(cnt[o])] for o in range(no)]
        return SweepResult(tops, valid.value, digest.value)

    def result_bytes(self) -> int:
        return int(lib().bote_sweep_result_bytes(self.h))

    def result_device(self, dst_ptr: int, stream: Optional[int] = None):
        check(lib().bote_sweep_result_device(self.h, C.c_void_p(dst_ptr), C.c_void_p(stream) if stream else None))

    def merge_device(self, src_ptr: int, n_shards: int, dst_ptr: int, stream: Optional[int] = None):
        check(lib().bote_merge_device(self.h, C.c_void_p(src_ptr), n_shards, C.c_void_p(dst_ptr),
                                      C.c_void_p(stream) if stream else None))

    def parse_block(self, blk: np.ndarray) -> SweepResult:
        """Host view of a device result block (bote_sweep_result_device layout)."""
        no, K = len(self.objectives), self.K
        b = np.frombuffer(np.ascontiguousarray(blk), dtype=np.uint64)
        recs = b[:no * _lib.KP * 2].reshape(no, _lib.KP, 2)[:, :K]
        # each list ends at its first (all-ones, all-ones) padding record
        pad = (recs[:, :, 0] == np.uint64(0xFFFFFFFFFFFFFFFF)) & (recs[:, :, 1] == np.uint64(0xFFFFFFFFFFFFFFFF))
        ends = np.where(pad.any(axis=1), pad.argmax(axis=1), K)
        tops = [list(map(tuple, recs[o, :ends[o]].tolist())) for o in range(no)]
        return SweepResult(tops, int(b[no * _lib.KP * 2]), int(b[no * _lib.KP * 2 + 1]))

    def kernel_ms(self) -> float:
        v = C.c_float()
        check(lib().bote_sweep_last_kernel_ms(self.h, C.byref(v)))
        return v.value

    def timing_reset(self):
        check(lib().bote_sweep_timing_reset(self.h))

    def timing(self) -> Tuple[float, int]:
        """(total kernel ms, launches) since the last timing_reset."""
        ms, n = C.c_float(), C.c_uint32()
        check(lib().bote_sweep_timing(self.h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def deferred(self, stream: Optional[int] = None) -> int:
        """Configs the last launch deferred to the exact generic kernel."""
        v = C.c_uint64()
        check(lib().bote_sweep_deferred(self.h, C.c_void_p(stream) if stream else None, C.byref(v)))
        return v.value

    def is_fast(self) -> bool:
        """True when a fast-path kernel (packed or group) runs the sweep."""
        return self.kernel_path() != "generic"

    def kernel_path(self) -> str:
        """'generic' (bote_kernels.hip), 'fast' (bote_sweep.hip) or 'group' (bote_group.hip)."""
        v = C.c_int()
        check(lib().bote_sweep_is_fast(self.h, C.byref(v)))
        return ("generic", "fast", "group")[v.value]

    def split(self, rank_begin: int, rank_end: int, parts: int) -> List[int]:
        """Shard boundaries of equal estimated cost (bote_sweep_split):
        parts + 1 ascending ranks from rank_begin to rank_end."""
        cache = self.__dict__.setdefault("_splits", {})
        key = (rank_begin, rank_end, parts)
        if key not in cache:  # (a host walk of the groups, cached in the library too: ~15 ms at R=64 n=7)
            out = (C.c_uint64 * (parts + 1))()
            check(lib().bote_sweep_split(self.h, rank_begin, rank_end, parts, out))
            cache[key] = [int(x) for x in out]
        return list(cache[key])

    def geometry(self) -> Tuple[int, int, int]:
        g, b, l = C.c_uint32(), C.c_uint32(), C.c_uint32()
        check(lib().bote_sweep_grid(self.h, C.byref(g), C.byref(b), C.byref(l)))
        return g.value, b.value, l.value

    def config_of(self, rank: int) -> List[int]:
        pos = _lib.colex_unrank(rank, self.n, len(self.servers))
        return [int(self.servers[p]) for p in pos]


class MultiDeviceSearch:
    """bote_search_*: the sweep sharded over `planets` (one per shard; the same
    device may appear more than once), merged on planets[0]'s device, without
    torch.distributed.  All host work (shard bounds of equal estimated cost and
    every shard's work-chunk table, from one walk of the rank space) happens
    here, once; `launch` is device work only and can be repeated."""

    def __init__(self, planets: Sequence[DevicePlanet], servers: Sequence[int], clients: Sequence[int], n: int,
                 objectives=DEFAULT_OBJECTIVES, K: int = 100, ranking: Optional[RankingParams] = DEFAULT_RANKING,
                 digest: bool = True, rank_begin: int = 0, rank_end: Optional[int] = None,
                 keys: int = _lib.KEYS_BASE):
        srv, cli = u32(servers), u32(clients)
        self.objectives, self.K, self.n_shards = list(objectives), K, len(planets)
        no = len(self.objectives)
        objs = (_lib.Objective * max(no, 1))(*[_lib.Objective(k, s) for k, s in self.objectives])
        rp = C.byref(_lib.ranking_params_c(ranking)) if ranking is not None else None
        hs = (C.c_void_p * len(planets))(*[p.h.value for p in planets])
        self._planets = list(planets)  # the handle borrows them
        self.rank_begin = rank_begin
        self.rank_end = _lib.binomial(len(srv), n) if rank_end is None else rank_end
        h = C.c_void_p()
        check(lib().bote_search_create(hs, len(planets), srv, len(srv), cli, len(cli), n, rank_begin, self.rank_end,
                                       objs, no, K, rp, 1 if digest else 0, keys, C.byref(h)))
        self.h = h

    def __del__(self):
        try:
            if self.h:
                lib().bote_search_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def bounds(self) -> List[int]:
        out = (C.c_uint64 * (self.n_shards + 1))()
        check(lib().bote_search_bounds(self.h, out))
        return [int(x) for x in out]

    def launch(self):
        check(lib().bote_search_launch(self.h))

    def result(self) -> SweepResult:
        no, K = len(self.objectives), self.K
        recs = (_lib.TopKRecord * max(no * K, 1))()
        cnt = np.zeros(max(no, 1), np.uint32)
        valid, dig = C.c_uint64(), C.c_uint64()
        check(lib().bote_search_result(self.h, recs, ptr(cnt), C.byref(valid), C.byref(dig)))
        tops = [[(recs[o * K + i].key, recs[o * K + i].rank) for i in range(cnt[o])] for o in range(no)]
        return SweepResult(tops, valid.value, dig.value)


def search_topk(planets: Sequence[DevicePlanet], servers: Sequence[int], clients: Sequence[int], n: int,
                objectives=DEFAULT_OBJECTIVES, K: int = 100, ranking: Optional[RankingParams] = DEFAULT_RANKING,
                digest: bool = True, rank_begin: int = 0, rank_end: Optional[int] = None) -> SweepResult:
    """bote_search_topk: the sweep sharded over `planets` (one per shard; the
    same device may appear more than once) in ONE library call, merged on
    planets[0]'s device.  The multi-GPU search without torch.distributed."""
    srv, cli = u32(servers), u32(clients)
    objs_l = list(objectives)
    no = len(objs_l)
    objs = (_lib.Objective * max(no, 1))(*[_lib.Objective(k, s) for k, s in objs_l])
    rp = C.byref(_lib.ranking_params_c(ranking)) if ranking is not None else None
    hs = (C.c_void_p * len(planets))(*[p.h.value for p in planets])
    re = _lib.binomial(len(srv), n) if rank_end is None else rank_end
    recs = (_lib.TopKRecord * max(no * K, 1))()
    cnt = np.zeros(max(no, 1), np.uint32)
    valid, dig = C.c_uint64(), C.c_uint64()
    check(lib().bote_search_topk(hs, len(planets), srv, len(srv), cli, len(cli), n, rank_begin, re, objs, no, K, rp,
                                 1 if digest else 0, recs, ptr(cnt), C.byref(valid), C.byref(dig)))
    tops = [[(recs[o * K + i].key, recs[o * K + i].rank) for i in range(cnt[o])] for o in range(no)]
    return SweepResult(tops, valid.value, dig.value)
