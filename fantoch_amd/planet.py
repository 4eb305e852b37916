"""Latency planet: regions, `.dat` loading and the distance order.

Mirrors `fantoch::planet::{Planet, Region}` (reference
`fantoch/src/planet/mod.rs`, `dat.rs`, `region.rs`).

Layout decision (DESIGN.md "Data layout"): regions are held in *name order*, so
region index == rank of its name.  The reference sorts each distance row by the
tuple `(latency, Region)` (`planet/mod.rs:122-140`), so ties between equal
latencies go to the smaller name; with index == name rank the device kernels
reproduce that order by comparing `(latency, index)` as one packed integer.

The matrix is `lat[from, to]` (uint16, row = source), as `Planet::ping_latency`
(`planet/mod.rs:107-113`) and `Dat::latencies` (`dat.rs:33-54`) define it.
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

# planet/mod.rs:16
GCP_LAT_DIR = os.path.join(os.path.dirname(__file__), "data", "latency_gcp")
AWS_2020_DIR = os.path.join(os.path.dirname(__file__), "data", "latency_aws", "2020_06_05")
AWS_2021_DIR = os.path.join(os.path.dirname(__file__), "data", "latency_aws", "2021_02_13")

# planet/mod.rs:19
INTRA_REGION_LATENCY = 0

# Device kernels pack (latency << 4 | member) into 32 bits and sum squares of
# (latency + quorum latency) over up to 256 clients in 64 bits; 14 bits of
# latency keep every intermediate exact (DESIGN.md "Value ranges").
MAX_LATENCY = (1 << 14) - 1


class Region:
    """`fantoch::planet::Region` (`region.rs:4-18`): a named region, ordered by name."""

    __slots__ = ("name",)

    def __init__(self, name: str):
        self.name = str(name)

    def __eq__(self, other):
        return isinstance(other, Region) and self.name == other.name

    def __lt__(self, other):
        return self.name < other.name

    def __le__(self, other):
        return self.name <= other.name

    def __hash__(self):
        return hash(self.name)

    def __repr__(self):  # Debug prints the bare name (region.rs:21-25)
        return self.name

    __str__ = __repr__


def _as_name(r) -> str:
    return r.name if isinstance(r, Region) else str(r)


# ------------------------------------------------------------------ Dat -----
def dat_region(filename: str) -> Region:
    """`Dat::region` (`dat.rs:21-28`): the second-to-last '/' or '.' separated part."""
    parts = filename.replace(".", "/").split("/")
    return Region(parts[-2])


def dat_latency(line: str) -> Tuple[Region, int]:
    """`Dat::latency` (`dat.rs:58-75`): `min/avg/max/mdev:region` -> (region, floor(avg))."""
    parts = line.replace(":", "/").split("/")
    avg = float(parts[1])
    lat = int(avg)  # `as u64` truncates toward zero (and saturates at 0)
    if lat < 0:
        lat = 0
    return Region(parts[-1]), lat


def dat_latencies(filename: str) -> Dict[Region, int]:
    """`Dat::latencies` (`dat.rs:33-54`); intra-region latency is forced to 0."""
    this = dat_region(filename)
    out: Dict[Region, int] = {}
    with open(filename) as fh:
        for line in fh.read().splitlines():
            region, lat = dat_latency(line)
            out[region] = INTRA_REGION_LATENCY if region == this else lat
    return out


def all_dats(lat_dir: str) -> List[str]:
    """`Dat::all_dats` (`dat.rs:78-94`): every `*.dat` in `lat_dir`."""
    if not os.path.isdir(lat_dir):
        raise FileNotFoundError(f"read_dir {lat_dir!r} failed")
    return [os.path.join(lat_dir, f) for f in sorted(os.listdir(lat_dir)) if f.endswith(".dat")]


def write_dat(planet: "Planet", region, lat_dir: str) -> str:
    """Inverse of `Dat::latencies` for integral planets: one `min/avg/max/mdev:to`
    line per destination, ascending by (latency, name) like `ping_exp_gcp`'s `sort -n`."""
    os.makedirs(lat_dir, exist_ok=True)
    name = _as_name(region)
    path = os.path.join(lat_dir, name + ".dat")
    with open(path, "w") as fh:
        for lat, to in planet.sorted(name):
            v = float(lat)
            fh.write(f"{v:.3f}/{v:.3f}/{v:.3f}/0.000:{to.name}\n")
    return path


# --------------------------------------------------------------- Planet -----
class Planet:
    """`fantoch::planet::Planet` (`planet/mod.rs:21-28`)."""

    def __init__(self, names: Sequence[str], lat: np.ndarray):
        names = [str(n) for n in names]
        if list(names) != sorted(names) or len(set(names)) != len(names):
            raise ValueError("planet regions must be unique and given in name order")
        lat = np.asarray(lat)
        R = len(names)
        if lat.shape != (R, R):
            raise ValueError(f"latency matrix must be {R}x{R}, got {lat.shape}")
        if lat.min(initial=0) < 0 or lat.max(initial=0) > MAX_LATENCY:
            raise ValueError(f"latencies must lie in [0, {MAX_LATENCY}]")
        self.names: List[str] = names
        self.index: Dict[str, int] = {n: i for i, n in enumerate(names)}
        self.lat: np.ndarray = np.ascontiguousarray(lat, dtype=np.uint16)
        self._sorted_cache: Dict[int, List[Tuple[int, Region]]] = {}

    # planet/mod.rs:33-35
    @classmethod
    def new(cls) -> "Planet":
        return cls.from_dir(GCP_LAT_DIR)

    # planet/mod.rs:38-45
    @classmethod
    def from_dir(cls, lat_dir: str) -> "Planet":
        lats = {dat_region(f): dat_latencies(f) for f in all_dats(lat_dir)}
        return cls.from_latencies(lats)

    # `Planet::from` is a Rust constructor name; keep it for API parity.
    @classmethod
    def from_(cls, lat_dir: str) -> "Planet":
        return cls.from_dir(lat_dir)

    # planet/mod.rs:48-54
    @classmethod
    def from_latencies(cls, latencies: Dict) -> "Planet":
        names = sorted({_as_name(k) for k in latencies})
        idx = {n: i for i, n in enumerate(names)}
        R = len(names)
        lat = np.zeros((R, R), dtype=np.int64)
        seen = np.zeros((R, R), dtype=bool)
        for frm, row in latencies.items():
            i = idx[_as_name(frm)]
            for to, v in row.items():
                tn = _as_name(to)
                if tn not in idx:
                    raise ValueError(f"region {tn} has no .dat of its own")
                lat[i, idx[tn]] = int(v)
                seen[i, idx[tn]] = True
        if not seen.all():
            missing = [(names[i], names[j]) for i, j in zip(*np.where(~seen))][:4]
            raise ValueError(f"incomplete latency matrix, e.g. missing {missing}")
        return cls(names, lat)

    # planet/mod.rs:57-99
    @classmethod
    def equidistant(cls, planet_distance: int, region_number: int) -> Tuple[List[Region], "Planet"]:
        regions = [Region(f"r_{i}") for i in range(region_number)]
        lats = {a: {b: (INTRA_REGION_LATENCY if a == b else planet_distance) for b in regions}
                for a in regions}
        return regions, cls.from_latencies(lats)

    @classmethod
    def synthetic(cls, R: int, seed: Optional[int] = None) -> "Planet":
        """Synthetic planet of SURVEY.md §8d (extension, not in the reference).

        Names `r000..` (zero-padded so index order == name order).  splitmix64
        stream from `seed` (default 0x5EED0000 + R as written in hex digits, i.e.
        0x5EED0064 for R=64 and 0x5EED0128 for R=128):
          for i < j (row-major):  d = 5 + u % 346;  L[i,j] = L[j,i] = d
          for i != j (row-major): if u % 64 == 0: L[i,j] += 1 + (u >> 6) % 3
        Diagonal 0.  Equal latencies are frequent, which exercises the name
        tie-break.
        """
        if seed is None:
            seed = int(f"5EED{R:04d}", 16)
        names = [f"r{i:03d}" for i in range(R)]
        lat = np.zeros((R, R), dtype=np.int64)
        state = [seed & 0xFFFFFFFFFFFFFFFF]
        M = 0xFFFFFFFFFFFFFFFF

        def nxt() -> int:
            state[0] = (state[0] + 0x9E3779B97F4A7C15) & M
            z = state[0]
            z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
            z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
            return z ^ (z >> 31)

        for i in range(R):
            for j in range(i + 1, R):
                d = 5 + nxt() % 346
                lat[i, j] = d
                lat[j, i] = d
        for i in range(R):
            for j in range(R):
                if i == j:
                    continue
                u = nxt()
                if u % 64 == 0:
                    lat[i, j] += 1 + (u >> 6) % 3
        return cls(names, lat)

    # ------------------------------------------------------------ queries ---
    @property
    def R(self) -> int:
        return len(self.names)

    def regions(self) -> List[Region]:
        """planet/mod.rs:102-104 (returned in name order here)."""
        return [Region(n) for n in self.names]

    def idx(self, region) -> int:
        return self.index[_as_name(region)]

    def idxs(self, regions: Iterable) -> np.ndarray:
        return np.array([self.idx(r) for r in regions], dtype=np.uint32)

    def ping_latency(self, frm, to) -> Optional[int]:
        """planet/mod.rs:107-113."""
        a, b = self.index.get(_as_name(frm)), self.index.get(_as_name(to))
        if a is None or b is None:
            return None
        return int(self.lat[a, b])

    def sorted(self, frm) -> Optional[List[Tuple[int, Region]]]:
        """planet/mod.rs:117-119: `(latency, region)` ascending, ties by name."""
        i = self.index.get(_as_name(frm))
        if i is None:
            return None
        if i not in self._sorted_cache:
            row = self.lat[i].astype(np.int64)
            order = np.lexsort((np.arange(self.R), row))  # index == name rank
            self._sorted_cache[i] = [(int(row[j]), Region(self.names[j])) for j in order]
        return self._sorted_cache[i]

    def distance_matrix(self, regions: Sequence) -> str:
        """planet/mod.rs:144-177 (markdown table)."""
        out = "| |" + "".join(f" {_as_name(r)} |" for r in regions) + "\n"
        out += "|:---:|" + ":---:|" * len(regions) + "\n"
        for a in regions:
            out += f"| __{_as_name(a)}__ |"
            for b in regions:
                v = self.ping_latency(a, b)
                if v is None:
                    raise KeyError(f"no latency {a}->{b}")
                out += f" {v} |"
            out += "\n"
        return out

    def names_blob(self) -> bytes:
        return b"".join(n.encode() + b"\0" for n in self.names)

    def has_offdiag_zero(self) -> bool:
        off = self.lat.copy()
        np.fill_diagonal(off, 1)
        return bool((off == 0).any()) or bool(np.diag(self.lat).any())
