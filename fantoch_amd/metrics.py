"""Host-side metrics types: `F64`, `Stats`, `Histogram`.

Mirror of `fantoch::metrics` (reference `fantoch/src/metrics/float.rs` and
`histogram.rs`).  These are data types the search returns; their statistics
reproduce the reference's f64 arithmetic exactly (IEEE double, same operation
order).  The hot path never calls them: device kernels produce the per-client
latencies and exact moments these histograms are built from.
"""
from __future__ import annotations

import enum
import math
from typing import Dict, Iterable, Iterator, Optional


class Stats(enum.Enum):
    """histogram.rs:7-11"""
    Mean = 0
    COV = 1
    MDTM = 2


class F64:
    """float.rs:5-103 — f64 with a total order in which NaN is greatest."""

    __slots__ = ("v",)

    def __init__(self, x: float):
        self.v = float(x)

    @staticmethod
    def zero() -> "F64":
        return F64(0.0)

    @staticmethod
    def nan() -> "F64":
        return F64(float("nan"))

    def value(self) -> float:
        return self.v

    def round(self) -> str:
        """float.rs:22-24 — format!("{:.1}") (exact value, ties to even)."""
        if math.isnan(self.v):
            return "NaN"
        if math.isinf(self.v):
            return "inf" if self.v > 0 else "-inf"
        return format(self.v, ".1f")

    def cmp(self, other: "F64") -> int:
        a, b = self.v, other.v
        if a < b:
            return -1
        if a > b:
            return 1
        if a == b:
            return 0
        an, bn = math.isnan(a), math.isnan(b)
        if an and bn:
            return 0
        return 1 if an else -1

    def __add__(self, o):
        return F64(self.v + o.v)

    def __sub__(self, o):
        return F64(self.v - o.v)

    def __mul__(self, o):
        return F64(self.v * o.v)

    # Ord / PartialEq (float.rs:62-89)
    def __eq__(self, o):
        return isinstance(o, F64) and self.cmp(o) == 0

    def __lt__(self, o):
        return self.cmp(o) < 0

    def __le__(self, o):
        return self.cmp(o) <= 0

    def __gt__(self, o):
        return self.cmp(o) > 0

    def __ge__(self, o):
        return self.cmp(o) >= 0

    def __hash__(self):
        return hash("nan") if math.isnan(self.v) else hash(self.v)

    # PartialOrd derive (float.rs:5): plain f64 comparisons for `>=` on values
    def ge(self, o: "F64") -> bool:
        return self.v >= o.v

    def __repr__(self):
        return repr(self.v)


def rust_round(x: float) -> float:
    """f64::round: half away from zero (exact: the fractional part is exact)."""
    if math.isnan(x) or math.isinf(x):
        return x
    a = abs(x)
    r = math.floor(a)
    if a - r >= 0.5:
        r += 1.0
    return math.copysign(r, x)


def _display_round(x: float) -> str:
    """f64::round (half away from zero) then Rust's Display, padded `{:<5}`."""
    if math.isnan(x):
        s = "NaN"
    elif math.isinf(x):
        s = "inf" if x > 0 else "-inf"
    else:
        r = rust_round(x)
        s = "-0" if (r == 0 and math.copysign(1.0, r) < 0) else str(int(r))
    return s.ljust(5)


class Histogram:
    """histogram.rs:14-257 — exact multiset of u64 values (value -> count)."""

    __slots__ = ("values",)

    def __init__(self, values: Optional[Dict[int, int]] = None):
        self.values: Dict[int, int] = dict(sorted(values.items())) if values else {}

    @classmethod
    def new(cls) -> "Histogram":
        return cls()

    @classmethod
    def from_values(cls, values: Iterable[int]) -> "Histogram":
        d: Dict[int, int] = {}
        for v in values:
            v = int(v)
            d[v] = d.get(v, 0) + 1
        return cls(d)

    # Histogram::from
    from_ = from_values

    def count(self) -> int:
        return sum(self.values.values())

    def iter_values(self) -> Iterator[int]:
        for v, c in self.values.items():
            for _ in range(c):
                yield v

    def inner(self) -> Dict[int, int]:
        return self.values

    def increment(self, value: int):
        self.values[int(value)] = self.values.get(int(value), 0) + 1
        self.values = dict(sorted(self.values.items()))

    def merge(self, other: "Histogram"):
        for k, c in other.values.items():
            self.values[k] = self.values.get(k, 0) + c
        self.values = dict(sorted(self.values.items()))

    def _sum_and_count(self):
        s = 0
        c = 0
        for v, k in self.values.items():
            s += v * k
            c += k
        return s & 0xFFFFFFFFFFFFFFFF, c

    def _mean_and_count(self):
        s, c = self._sum_and_count()
        cf = float(c)
        return (float(s) / cf if cf != 0 else (float("nan") if s == 0 else math.copysign(float("inf"), s))), cf

    def _variance(self, mean: float, count: float) -> float:
        acc = 0.0
        for x, k in self.values.items():
            d = mean - float(x)
            acc = acc + (d * d) * float(k)
        denom = count - 1.0
        if denom == 0.0:
            return float("nan") if (acc == 0.0 or math.isnan(acc)) else math.copysign(float("inf"), acc)
        return acc / denom

    def mean(self) -> F64:
        return F64(self._mean_and_count()[0])

    def stddev(self) -> F64:
        m, c = self._mean_and_count()
        v = self._variance(m, c)
        return F64(math.sqrt(v) if v == v and v >= 0 else float("nan"))

    def cov(self) -> F64:
        m, c = self._mean_and_count()
        v = self._variance(m, c)
        sd = math.sqrt(v) if v == v and v >= 0 else float("nan")
        if m == 0.0 or math.isnan(m):
            return F64(float("nan") if (sd == 0.0 or math.isnan(sd) or math.isnan(m)) else math.copysign(float("inf"), sd))
        return F64(sd / m)

    def mdtm(self) -> F64:
        m, c = self._mean_and_count()
        acc = 0.0
        for x, k in self.values.items():
            acc = acc + abs(m - float(x)) * float(k)
        if c == 0.0:
            return F64(float("nan"))
        return F64(acc / c)

    def mean_improv(self, other: "Histogram") -> F64:
        return self.mean() - other.mean()

    def cov_improv(self, other: "Histogram") -> F64:
        return self.cov() - other.cov()

    def mdtm_improv(self, other: "Histogram") -> F64:
        return self.mdtm() - other.mdtm()

    def min(self) -> F64:
        return F64(float(next(iter(self.values)))) if self.values else F64.nan()

    def max(self) -> F64:
        return F64(float(next(reversed(self.values)))) if self.values else F64.nan()

    def percentile(self, percentile: float) -> F64:
        """histogram.rs:111-170"""
        assert 0.0 <= percentile <= 1.0
        if not self.values:
            return F64.zero()
        count = float(self.count())
        index = percentile * count
        index_rounded = rust_round(index)
        is_whole = abs(index - index_rounded) == 0.0
        idx = int(index_rounded)
        items = list(self.values.items())
        i = 0
        while True:
            if i >= len(items):
                raise RuntimeError("there should a next histogram value")
            value, cnt = items[i]
            if idx == cnt:
                left = float(value)
                right = float(items[i + 1][0]) if i + 1 < len(items) else None
                break
            if idx < cnt:
                left = float(value)
                right = left
                break
            idx -= cnt
            i += 1
        if is_whole:
            if right is None:
                raise RuntimeError("there should be a right value")
            return F64((left + right) / 2.0)
        return F64(left)

    def __eq__(self, o):
        return isinstance(o, Histogram) and self.values == o.values

    def __repr__(self):
        """histogram.rs:238-257 (Debug)."""
        if not self.values:
            return "(empty)"
        return ("avg={} std={} p95={} p99={} p99.9={} p99.99={} min={} max={}".format(
            _display_round(self.mean().value()), _display_round(self.stddev().value()),
            _display_round(self.percentile(0.95).value()), _display_round(self.percentile(0.99).value()),
            _display_round(self.percentile(0.999).value()), _display_round(self.percentile(0.9999).value()),
            _display_round(self.min().value()), _display_round(self.max().value())))
