"""TEST INFRASTRUCTURE — ctypes wrapper of the CPU oracle (bote_oracle.cpp).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  It restates the reference algorithm; see the header of
bote_oracle.cpp for the file:line map.  Parity: pinned against the reference's
own known-answer tests (tests/test_oracle.py).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import List, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

FPAXOS, EPAXOS, ATLAS = 0, 1, 2
OBJ_SCORE, OBJ_MEAN, OBJ_COV = 0, 1, 2
K_AF1, K_FF1, K_AF2, K_FF2, K_E = 0, 1, 2, 3, 4
SLOT_NAMES = ["af1", "ff1", "af2", "ff2", "e", "af1C", "ff1C", "af2C", "ff2C", "eC"]

u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")


def build(asan: bool = False) -> str:
    target = "build/liboracle_asan.so" if asan else "build/liboracle.so"
    subprocess.run(["make", "-s", "-C", _HERE, target], check=True)
    return os.path.join(_HERE, target)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "build", "liboracle.so")
        src = os.path.join(_HERE, "bote_oracle.cpp")
        if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
            build()
        L = C.CDLL(path)
        L.oracle_last_error.restype = C.c_char_p
        L.oracle_planet_new.restype = C.c_void_p
        L.oracle_planet_new.argtypes = [u16p, C.c_uint32, C.c_char_p]
        L.oracle_planet_free.argtypes = [C.c_void_p]
        L.oracle_planet_sorted.argtypes = [C.c_void_p, C.c_uint32, u32p, u64p]
        L.oracle_quorum_latency.argtypes = [C.c_void_p, C.c_uint32, u32p, C.c_uint32, C.c_uint32,
                                            C.POINTER(C.c_uint64)]
        L.oracle_leaderless.argtypes = [C.c_void_p, u32p, C.c_uint32, u32p, C.c_uint32, C.c_uint32, u64p]
        L.oracle_leader.argtypes = [C.c_void_p, C.c_uint32, u32p, C.c_uint32, u32p, C.c_uint32,
                                    C.c_uint32, u64p]
        L.oracle_best_leader.argtypes = [C.c_void_p, u32p, C.c_uint32, u32p, C.c_uint32, C.c_uint32,
                                         C.c_int, C.POINTER(C.c_uint32)]
        L.oracle_leaderless_batch.argtypes = [C.c_void_p, u32p, C.c_uint32, C.c_uint32, u32p, C.c_uint32, u32p,
                                              C.c_uint32, C.c_uint32, u64p]
        L.oracle_hist_stats.argtypes = [u64p, C.c_uint32, f64p]
        L.oracle_hist_percentile.argtypes = [u64p, C.c_uint32, C.c_double, C.POINTER(C.c_double)]
        L.oracle_hist_fmt.argtypes = [u64p, C.c_uint32, C.c_char_p, C.c_uint32]
        L.oracle_f64_round.argtypes = [C.c_double, C.c_char_p, C.c_uint32]
        L.oracle_f64_cmp.argtypes = [C.c_double, C.c_double]
        L.oracle_quorum_size.restype = C.c_uint32
        L.oracle_quorum_size.argtypes = [C.c_int, C.c_uint32, C.c_uint32]
        L.oracle_compute_stats.argtypes = [C.c_void_p, u32p, C.c_uint32, C.c_uint32, u32p, C.c_uint32,
                                           u64p, u32p]
        L.oracle_compute_stats_mt.argtypes = [C.c_void_p, u32p, C.c_uint32, C.c_uint32, u32p, C.c_uint32,
                                              u64p, u32p, C.c_uint32]
        L.oracle_scores.argtypes = [C.c_void_p, u32p, C.c_uint32, C.c_uint32, u32p, C.c_uint32, f64p, C.c_int,
                                    f64p, np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")]
        L.oracle_colex_unrank.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, u32p]
        L.oracle_sweep_x.argtypes = [C.c_void_p, u32p, C.c_uint32, u32p, C.c_uint32, C.c_uint32, C.c_uint64,
                                     C.c_uint64, u32p, C.c_uint32, C.c_uint32, f64p, C.c_int, C.c_uint32,
                                     C.c_uint32, u64p, u64p, u32p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.oracle_sweep_ranks.argtypes = [C.c_void_p, u32p, C.c_uint32, u32p, C.c_uint32, C.c_uint32, u64p,
                                         C.c_uint64, u32p, C.c_uint32, C.c_uint32, f64p, C.c_int, C.c_uint32,
                                         C.c_uint32, u64p, u64p, u32p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.oracle_moments_x.argtypes = [C.c_void_p, u32p, C.c_uint32, C.c_uint32, u32p, C.c_uint32, C.c_uint32,
                                       u64p, u64p, u64p, u64p, u32p]
        L.oracle_sweep.argtypes = [C.c_void_p, u32p, C.c_uint32, u32p, C.c_uint32, C.c_uint32,
                                   C.c_uint64, C.c_uint64, u32p, C.c_uint32, C.c_uint32, f64p, C.c_int,
                                   C.c_uint32, u64p, u64p, u32p, C.POINTER(C.c_uint64),
                                   C.POINTER(C.c_uint64)]
        L.oracle_search_best.argtypes = [C.c_void_p, u32p, C.c_uint32, u32p, C.c_uint32, f64p, C.c_int,
                                         C.POINTER(C.c_double), u32p, C.c_char_p, C.c_uint32,
                                         C.POINTER(C.c_uint64)]
        L.oracle_search_chains.argtypes = [C.c_void_p, u32p, C.c_uint32, u32p, C.c_uint32, f64p, C.c_int, C.c_uint32,
                                           f64p, u32p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        _LIB = L
    return _LIB


def _check(rc: int):
    if rc != 0:
        raise RuntimeError("oracle panic: " + lib().oracle_last_error().decode())


def _u32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint32))


class OraclePlanet:
    """Handle on an oracle planet built from a name-ordered u16 matrix."""

    def __init__(self, names: Sequence[str], lat: np.ndarray):
        self.names = list(names)
        self.R = len(self.names)
        blob = b"".join(n.encode() + b"\0" for n in self.names)
        self.h = lib().oracle_planet_new(np.ascontiguousarray(lat, dtype=np.uint16), self.R, blob)

    @classmethod
    def of(cls, planet) -> "OraclePlanet":
        return cls(planet.names, planet.lat)

    def __del__(self):
        try:
            if self.h:
                lib().oracle_planet_free(self.h)
        except Exception:
            pass

    def sorted(self, frm: int) -> List[Tuple[int, int]]:
        regs = np.zeros(self.R, np.uint32)
        lats = np.zeros(self.R, np.uint64)
        _check(lib().oracle_planet_sorted(self.h, frm, regs, lats))
        return [(int(l), int(r)) for l, r in zip(lats, regs)]

    def quorum_latency(self, frm: int, regions, q: int) -> int:
        out = C.c_uint64()
        r = _u32(regions)
        _check(lib().oracle_quorum_latency(self.h, frm, r, len(r), q, C.byref(out)))
        return out.value

    def leaderless(self, servers, clients, q: int) -> np.ndarray:
        s, c = _u32(servers), _u32(clients)
        out = np.zeros(len(c), np.uint64)
        _check(lib().oracle_leaderless(self.h, s, len(s), c, len(c), q, out))
        return out

    def leaderless_batch(self, configs: np.ndarray, clients, qs, threads: int = 1) -> np.ndarray:
        """Bote::leaderless for each config (rows of region ids) and quorum size:
        (ncfg, nq, nc + n) u64 — Input clients, then Colocated (config order)."""
        cfg = _u32(configs)
        ncfg, n = cfg.shape
        c, q = _u32(clients), _u32(qs)
        out = np.zeros((ncfg, len(q), len(c) + n), np.uint64)
        _check(lib().oracle_leaderless_batch(self.h, cfg.reshape(-1), ncfg, n, c, len(c), q, len(q), threads,
                                             out.reshape(-1)))
        return out

    def leader(self, leader: int, servers, clients, q: int) -> np.ndarray:
        s, c = _u32(servers), _u32(clients)
        out = np.zeros(len(c), np.uint64)
        _check(lib().oracle_leader(self.h, leader, s, len(s), c, len(c), q, out))
        return out

    def best_leader(self, servers, clients, q: int, stat: int) -> int:
        s, c = _u32(servers), _u32(clients)
        out = C.c_uint32()
        _check(lib().oracle_best_leader(self.h, s, len(s), c, len(c), q, stat, C.byref(out)))
        return out.value

    def compute_stats(self, configs: np.ndarray, clients, threads: int = 1) -> Tuple[np.ndarray, np.ndarray]:
        """configs: (ncfg, n) region ids. Returns (vals (ncfg, 5*nc+5*n) u64, leader_pos)."""
        cfg = _u32(configs)
        ncfg, n = cfg.shape
        c = _u32(clients)
        vals = np.zeros((ncfg, 5 * len(c) + 5 * n), np.uint64)
        lead = np.zeros(ncfg, np.uint32)
        _check(lib().oracle_compute_stats_mt(self.h, cfg.reshape(-1), ncfg, n, c, len(c),
                                             vals.reshape(-1), lead, threads))
        return vals, lead

    def scores(self, configs: np.ndarray, clients, rparams, ft_metric: int = 2):
        """compute_score per config: (score f64, valid u8)."""
        cfg = _u32(configs)
        ncfg, n = cfg.shape
        c = _u32(clients)
        sc = np.zeros(ncfg, np.float64)
        va = np.zeros(ncfg, np.uint8)
        _check(lib().oracle_scores(self.h, cfg.reshape(-1), ncfg, n, c, len(c),
                                   np.asarray(rparams, dtype=np.float64), ft_metric, sc, va))
        return sc, va

    def moments_x(self, configs: np.ndarray, clients, threads: int = 1):
        """compute_stats_x (the extended key set) per config: (s1, s2) of shape
        (ncfg, 20), all-leader (s1, s2) of shape (ncfg, 2, n), COV leaders."""
        cfg = np.ascontiguousarray(np.asarray(configs, dtype=np.uint32))
        ncfg, n = cfg.shape
        c = _u32(clients)
        s1 = np.zeros((ncfg, 20), np.uint64)
        s2 = np.zeros((ncfg, 20), np.uint64)
        a1 = np.zeros((ncfg, 2, n), np.uint64)
        a2 = np.zeros((ncfg, 2, n), np.uint64)
        lead = np.zeros(ncfg, np.uint32)
        _check(lib().oracle_moments_x(self.h, cfg.reshape(-1), ncfg, n, c, len(c), threads, s1.reshape(-1),
                                      s2.reshape(-1), a1.reshape(-1), a2.reshape(-1), lead))
        return s1, s2, a1, a2, lead

    def sweep(self, servers, clients, n: int, rb: int, re: int, objectives, K: int,
              rparams=(110.0, 35.0, 0.0, 15.0), ft_metric: int = 2, threads: int = 1, keys: int = 0):
        """Streaming sweep; keys=1 computes the extended key set (compute_stats_x)."""
        s, c = _u32(servers), _u32(clients)
        objs = _u32(np.asarray(objectives, dtype=np.uint32).reshape(-1))
        nobj = len(objs) // 2
        kv = np.zeros(nobj * K, np.uint64)
        ranks = np.zeros(nobj * K, np.uint64)
        cnt = np.zeros(nobj, np.uint32)
        valid, digest = C.c_uint64(), C.c_uint64()
        rp = np.asarray(rparams, dtype=np.float64)
        _check(lib().oracle_sweep_x(self.h, s, len(s), c, len(c), n, rb, re, objs, nobj, K, rp,
                                    ft_metric, keys, threads, kv, ranks, cnt, C.byref(valid),
                                    C.byref(digest)))
        tops = [list(zip(kv[o * K:o * K + cnt[o]].tolist(), ranks[o * K:o * K + cnt[o]].tolist()))
                for o in range(nobj)]
        return tops, valid.value, digest.value

    def sweep_ranks(self, servers, clients, n: int, ranks, objectives, K: int,
                    rparams=(110.0, 35.0, 0.0, 15.0), ft_metric: int = 2, threads: int = 1, keys: int = 0):
        """sweep over an explicit list of colex ranks (the CPU baseline's seeded
        uniform sample): the same per-config work as sweep()."""
        s, c = _u32(servers), _u32(clients)
        rk = np.ascontiguousarray(np.asarray(ranks, dtype=np.uint64))
        objs = _u32(np.asarray(objectives, dtype=np.uint32).reshape(-1))
        nobj = len(objs) // 2
        kv = np.zeros(nobj * K, np.uint64)
        out_r = np.zeros(nobj * K, np.uint64)
        cnt = np.zeros(nobj, np.uint32)
        valid, digest = C.c_uint64(), C.c_uint64()
        rp = np.asarray(rparams, dtype=np.float64)
        _check(lib().oracle_sweep_ranks(self.h, s, len(s), c, len(c), n, rk, len(rk), objs, nobj, K, rp, ft_metric,
                                        keys, threads, kv, out_r, cnt, C.byref(valid), C.byref(digest)))
        tops = [list(zip(kv[o * K:o * K + cnt[o]].tolist(), out_r[o * K:o * K + cnt[o]].tolist()))
                for o in range(nobj)]
        return tops, valid.value, digest.value

    def search_best(self, servers, clients, rparams=(110.0, 35.0, 0.0, 15.0), ft_metric: int = 2):
        s, c = _u32(servers), _u32(clients)
        score = C.c_double()
        chain = np.zeros(6 * 13, np.uint32)
        buf = C.create_string_buffer(1 << 16)
        nch = C.c_uint64()
        rp = np.asarray(rparams, dtype=np.float64)
        _check(lib().oracle_search_best(self.h, s, len(s), c, len(c), rp, ft_metric,
                                        C.byref(score), chain, buf, len(buf), C.byref(nch)))
        sets = [[int(x) for x in chain[i * 13:(i + 1) * 13] if x != 0xFFFFFFFF] for i in range(6)]
        return score.value, sets, buf.value.decode().split("\n")[:6], nch.value


    def search_chains(self, servers, clients, rparams=(110.0, 35.0, 0.0, 15.0), ft_metric: int = 2, K: int = 50):
        """The first K chains of sorted_evolving_configs (reference order), the total count
        and the order-dependent digest of all chains: ([(score, [[region ids by name] x 6])],
        nchains, digest)."""
        s, c = _u32(servers), _u32(clients)
        sc = np.zeros(max(K, 1), np.float64)
        ch = np.zeros(max(K, 1) * 6 * 13, np.uint32)
        nch, dig = C.c_uint64(), C.c_uint64()
        rp = np.asarray(rparams, dtype=np.float64)
        _check(lib().oracle_search_chains(self.h, s, len(s), c, len(c), rp, ft_metric, K, sc, ch, C.byref(nch),
                                          C.byref(dig)))
        out = []
        for k in range(min(K, nch.value)):
            sets = [[int(x) for x in ch[(k * 6 + i) * 13:(k * 6 + i + 1) * 13] if x != 0xFFFFFFFF] for i in range(6)]
            out.append((float(sc[k]), sets))
        return out, nch.value, dig.value


def hist_stats(values) -> np.ndarray:
    v = np.ascontiguousarray(np.asarray(values, dtype=np.uint64))
    out = np.zeros(6, np.float64)
    _check(lib().oracle_hist_stats(v, len(v), out))
    return out


def hist_percentile(values, p: float) -> float:
    v = np.ascontiguousarray(np.asarray(values, dtype=np.uint64))
    out = C.c_double()
    _check(lib().oracle_hist_percentile(v, len(v), p, C.byref(out)))
    return out.value


def hist_fmt(values) -> str:
    v = np.ascontiguousarray(np.asarray(values, dtype=np.uint64))
    buf = C.create_string_buffer(1024)
    _check(lib().oracle_hist_fmt(v, len(v), buf, len(buf)))
    return buf.value.decode()


def f64_round(x: float) -> str:
    buf = C.create_string_buffer(64)
    _check(lib().oracle_f64_round(x, buf, len(buf)))
    return buf.value.decode()


def f64_cmp(a: float, b: float) -> int:
    return lib().oracle_f64_cmp(a, b)


def quorum_size(proto: int, n: int, f: int) -> int:
    return lib().oracle_quorum_size(proto, n, f)


def colex_unrank(rank: int, n: int, ns: int) -> List[int]:
    out = np.zeros(n, np.uint32)
    lib().oracle_colex_unrank(rank, n, ns, out)
    return out.tolist()
