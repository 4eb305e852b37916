"""`Protocol`, `ClientPlacement`, `ProtocolStats`.

Mirror of `fantoch_bote::protocol` (reference `fantoch_bote/src/protocol.rs`),
plus Tempo's fast-quorum sizes (`fantoch/src/config.rs:317-329`).
"""
from __future__ import annotations

import enum
from typing import Dict, Iterator

from .metrics import Histogram


class Protocol(enum.Enum):
    """protocol.rs:5-9 (+ Tempo, config.rs:317-329)."""
    FPaxos = 0
    EPaxos = 1
    Atlas = 2
    Tempo = 3        # fast quorum, non-tiny: n/2 + f
    TempoTiny = 4    # fast quorum, tiny: 2f
    TempoWrite = 5   # write quorum: f + 1

    def short_name(self) -> str:
        return {0: "f", 1: "e", 2: "a", 3: "t", 4: "tt", 5: "tw"}[self.value]

    def quorum_size(self, n: int, f: int) -> int:
        """protocol.rs:20-31; Tempo: config.rs:317-329 (fast and write quorums)."""
        if self is Protocol.FPaxos or self is Protocol.TempoWrite:
            return f + 1
        if self is Protocol.EPaxos:
            m = Protocol.minority(n)
            return m + (m + 1) // 2
        if self is Protocol.Atlas or self is Protocol.Tempo:
            return Protocol.minority(n) + f
        return 2 * f

    @staticmethod
    def minority(n: int) -> int:
        return n // 2


def tempo_quorum_sizes(n: int, f: int, tiny: bool):
    """config.rs:317-329: (fast quorum, write quorum, stability threshold)."""
    minority = n // 2
    fast, stab = (2 * f, n - f) if tiny else (minority + f, minority + 1)
    return fast, f + 1, stab


class ClientPlacement(enum.Enum):
    """protocol.rs:38-55"""
    Input = 0
    Colocated = 1

    def short_name(self) -> str:
        return "" if self is ClientPlacement.Input else "C"

    @staticmethod
    def all() -> Iterator["ClientPlacement"]:
        return iter([ClientPlacement.Input, ClientPlacement.Colocated])


class ProtocolStats:
    """protocol.rs:58-112 — mapping from protocol key to histogram."""

    def __init__(self):
        self.map: Dict[str, Histogram] = {}

    @staticmethod
    def new() -> "ProtocolStats":
        return ProtocolStats()

    @staticmethod
    def key(protocol: Protocol, f: int, placement: ClientPlacement) -> str:
        prefix = protocol.short_name() if protocol is Protocol.EPaxos else f"{protocol.short_name()}f{f}"
        return prefix + placement.short_name()

    def get(self, protocol: Protocol, f: int, placement: ClientPlacement) -> Histogram:
        k = self.key(protocol, f, placement)
        if k not in self.map:
            raise KeyError(f"stats with key {k} not found")
        return self.map[k]

    def insert(self, protocol: Protocol, f: int, placement: ClientPlacement, stats: Histogram):
        self.map[self.key(protocol, f, placement)] = stats

    def fmt(self, protocol: Protocol, f: int, placement: ClientPlacement) -> str:
        k = self.key(protocol, f, placement)
        return f"{k}={self.get(protocol, f, placement)!r}"

    def __eq__(self, o):
        return isinstance(o, ProtocolStats) and self.map == o.map

    def __repr__(self):
        return f"ProtocolStats({self.map!r})"
