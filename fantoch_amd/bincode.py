"""bincode 1.x encoding of `fantoch_bote::Search` — the `.data` cache file.

The reference saves a finished search with `bincode::serialize_into` and loads
it with `bincode::deserialize_from` (`fantoch_bote/src/search.rs:487-512`), under
the name `{min_n}_{max_n}_{SearchInput}.data` (`search.rs:479-485`).  Writing the
same bytes lets an unchanged Rust consumer pick up a GPU-computed search through
`Search::get_saved_search`, and reading them lets this package reuse a search the
Rust crate saved.

bincode 1.x with its default options (what `bincode::serialize_into` uses) is:
little-endian, fixed-width integers, `usize` as u64, every sequence / map /
string prefixed by its length as u64, structs and tuples as their fields in
order with no tags, newtype structs as their inner value.  Applied to the
reference's types (`search.rs:24-44`, `protocol.rs:58-59`,
`fantoch/src/metrics/histogram.rs:14-18`, `fantoch/src/planet/region.rs:28-35`):

    Search       = AllConfigs                                   (one field)
    AllConfigs   = Vec<(Vec<Region>, Configs)>
    Configs      = HashMap<usize, Vec<(BTreeSet<Region>, ProtocolStats)>>
    ProtocolStats= BTreeMap<String, Histogram>                  (newtype)
    Histogram    = BTreeMap<u64, usize>                          (one field)
    Region       = str                                           (custom Serialize)

BTreeSet/BTreeMap iterate in key order (Region/String: byte order), so those
are written sorted.  HashMap iteration order is unspecified; we write ascending
n, and the reader accepts any order.  The byte layout follows the published
bincode 1.x format and serde's derive rules; no Rust-written `.data` file ships
with the reference, so it is pinned by hand-derived known-answer bytes in
tests/test_bincode.py, not by a reference fixture.

This module is host-side serialisation only; the histograms it writes come
from the device (`Search.save_data`).
"""
from __future__ import annotations

import io
import struct
from typing import BinaryIO, Dict, Iterable, List, Mapping, Sequence, Tuple

import numpy as np

# One histogram: (value, count) pairs, values strictly ascending.
HistPairs = np.ndarray                      # (k, 2) uint64
Stats = Dict[str, HistPairs]                # ProtocolStats
ConfigAndStats = Tuple[List[str], Stats]    # (BTreeSet<Region>, ProtocolStats)
AllConfigs = List[Tuple[List[str], Dict[int, List[ConfigAndStats]]]]

_U64 = struct.Struct("<Q")


class BincodeError(ValueError):
    """Malformed or truncated input (bincode's `Error`, which the reference `expect`s)."""


# ---------------------------------------------------------------- writer ---
def _u64(w: BinaryIO, x: int):
    w.write(_U64.pack(x))


def _str(w: BinaryIO, s: str):
    b = s.encode("utf-8")
    _u64(w, len(b))
    w.write(b)


def histogram_pairs(values) -> HistPairs:
    """`Histogram::from(values)` as sorted (value, count) pairs."""
    v, c = np.unique(np.asarray(values, dtype=np.uint64), return_counts=True)
    return np.stack([v, c.astype(np.uint64)], axis=1)


def write_histogram(w: BinaryIO, pairs: HistPairs):
    pairs = np.ascontiguousarray(np.asarray(pairs, dtype="<u8").reshape(-1, 2))
    _u64(w, pairs.shape[0])
    w.write(pairs.tobytes())


def write_protocol_stats(w: BinaryIO, stats: Mapping[str, HistPairs]):
    keys = sorted(stats, key=lambda k: k.encode("utf-8"))
    _u64(w, len(keys))
    for k in keys:
        _str(w, k)
        write_histogram(w, stats[k])


def write_region_set(w: BinaryIO, regions: Iterable[str]):
    names = sorted(set(regions), key=lambda s: s.encode("utf-8"))
    _u64(w, len(names))
    for r in names:
        _str(w, r)


def write_search(w: BinaryIO, all_configs: Sequence[Tuple[Sequence[str], Mapping[int, Sequence[ConfigAndStats]]]]):
    """`bincode::serialize_into(writer, &search)` (search.rs:500-512).

    `all_configs[i] = (clients in their Vec order, {n: [(config, stats), ...]})`.
    A value for `n` may be any sized sequence (e.g. a lazy batch producer with
    `__len__` and `__iter__`), so large searches stream to disk."""
    _u64(w, len(all_configs))
    for clients, configs in all_configs:
        _u64(w, len(clients))
        for r in clients:
            _str(w, r)
        _u64(w, len(configs))
        for n in sorted(configs):
            lst = configs[n]
            _u64(w, n)
            _u64(w, len(lst))
            written = 0
            for cfg, stats in lst:
                write_region_set(w, cfg)
                write_protocol_stats(w, stats)
                written += 1
            if written != len(lst):
                raise BincodeError(f"n={n}: announced {len(lst)} configs, produced {written}")


def encode_search(all_configs) -> bytes:
    buf = io.BytesIO()
    write_search(buf, all_configs)
    return buf.getvalue()


# ---------------------------------------------------------------- reader ---
class _Reader:
    def __init__(self, data):
        self.b = memoryview(data)
        self.o = 0

    def need(self, k: int):
        if self.o + k > len(self.b):
            raise BincodeError(f"truncated input: need {k} bytes at offset {self.o}, have {len(self.b) - self.o}")

    def u64(self) -> int:
        self.need(8)
        x = _U64.unpack_from(self.b, self.o)[0]
        self.o += 8
        return x

    def length(self, elem_bytes: int) -> int:
        k = self.u64()
        # a length can never exceed what is left (bincode's size check)
        if k * max(elem_bytes, 1) > len(self.b) - self.o:
            raise BincodeError(f"length {k} at offset {self.o - 8} exceeds the remaining input")
        return k

    def str(self) -> str:
        k = self.length(1)
        s = bytes(self.b[self.o:self.o + k])
        self.o += k
        try:
            return s.decode("utf-8")
        except UnicodeDecodeError as e:
            raise BincodeError(f"invalid utf-8 string at offset {self.o - k}") from e

    def histogram(self) -> HistPairs:
        k = self.length(16)
        a = np.frombuffer(self.b, dtype="<u8", count=2 * k, offset=self.o).reshape(k, 2).astype(np.uint64)
        self.o += 16 * k
        return a


def read_search(data) -> AllConfigs:
    """`bincode::deserialize_from` of a `Search` (search.rs:487-498)."""
    r = _Reader(data)
    out: AllConfigs = []
    for _ in range(r.length(16)):
        clients = [r.str() for _ in range(r.length(8))]
        configs: Dict[int, List[ConfigAndStats]] = {}
        for _ in range(r.length(16)):
            n = r.u64()
            lst: List[ConfigAndStats] = []
            for _ in range(r.length(16)):
                cfg = [r.str() for _ in range(r.length(8))]
                stats = {}
                for _ in range(r.length(16)):
                    k = r.str()
                    stats[k] = r.histogram()
                lst.append((cfg, stats))
            configs[n] = lst
        out.append((clients, configs))
    if r.o != len(r.b):
        raise BincodeError(f"{len(r.b) - r.o} trailing bytes after the Search value")
    return out
