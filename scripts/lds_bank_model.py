"""Where the R=64 n=7 sweep's LDS bank conflicts come from: a model of every
per-step LDS instruction of `sweep_group_kernel<7, ..., BN>` with the lanes'
real addresses, priced by the banking rules of MI355X_MICROARCH.md §LDS,
against the measured SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.

  python scripts/lds_bank_model.py [profiles/r06h_r64n7_profile.md] [--steps N]

A step is 64 colex-consecutive configs of one group (fixed positions
p3 < .. < p6, the lanes' (p0, p1, p2) the next 64 3-subsets of [0, p3) in
colex order, as the low table holds them); steps are drawn with probability
proportional to their share of the rank space.  SI: position = region.
Per instruction the LDS-array cycles are, per lane group, the largest number
of distinct dwords any bank holds (identical addresses broadcast); the
conflict cycles are those above one per group.  Lane groups and banks:
  ds_read_b32 / u16, ds_write_b32, ds_add_u32: {0-31}, {32-63}, bank (a/4) mod 32
  ds_read_b64: {0-31}, {32-63}, bank (a/4) mod 64 (two dwords per lane)
  ds_read_b128: {0-3,12-15,20-27}, {4-11,16-19,28-31}, {32-35,44-47,52-59},
                {36-43,48-51,60-63}, bank (a/4) mod 64 (four dwords per lane)
  ds_add_u64: four groups of 16 contiguous lanes, bank (a/4) mod 32
Addresses are relative to each table's base (a table starts 16-B aligned;
the bases only rotate the banks of all lanes together).
"""
import argparse
import os
import re
import sys
from collections import defaultdict
from math import comb

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R, N, NC = 64, 7, 64
NQ = NC // 4
CSTRIDE = 144  # bote_host.cpp quad_stride(16) = 18 quads of 8 B
G128 = [[0, 1, 2, 3, 12, 13, 14, 15] + list(range(20, 28)), [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
G128 = G128 + [[x + 32 for x in g] for g in G128]


def cycles(addrs, kind, active):
    """LDS-array cycles of one wave-instruction: (cycles, conflict-free cycles)."""
    if kind in ("b32", "u16", "w32", "add32"):
        groups, dwords, nb = [range(0, 32), range(32, 64)], 1, 32
    elif kind == "b64":
        groups, dwords, nb = [range(0, 32), range(32, 64)], 2, 64
    elif kind == "b128":
        groups, dwords, nb = G128, 4, 64
    elif kind == "add64":
        groups, dwords, nb = [range(i, i + 16) for i in range(0, 64, 16)], 2, 32
    else:
        raise ValueError(kind)
    tot = base = 0
    for g in groups:
        dw = set()
        for l in g:
            if active[l]:
                a = addrs[l] // 4
                dw.update(a + k for k in range(dwords))
        if not dw:
            continue
        per = defaultdict(int)
        for d in dw:
            per[d % nb] += 1
        tot += max(per.values())
        base += 1
    return tot, base


def step_lanes(rng, weights, groups):
    """One step: its group's fixed positions and the 64 lanes' (p0, p1, p2)."""
    gi = rng.choice(len(groups), p=weights)
    p3 = groups[gi]
    fixed = [p3] + sorted(rng.choice(np.arange(p3 + 1, R), size=N - 4, replace=False).tolist())
    n3 = comb(p3, 3)
    start = 64 * rng.integers(0, (n3 + 63) // 64)
    lanes = []
    # colex order of 3-subsets of [0, p3): p2 outermost, p0 innermost
    r = 0
    for p2 in range(2, p3):
        for p1 in range(1, p2):
            for p0 in range(p1):
                if start <= r < start + 64:
                    lanes.append((p0, p1, p2))
                r += 1
                if r >= start + 64:
                    break
            if r >= start + 64:
                break
        if r >= start + 64:
            break
    active = [True] * len(lanes) + [False] * (64 - len(lanes))
    lanes = lanes + [lanes[-1]] * (64 - len(lanes))
    return fixed, lanes, active


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("profile", nargs="?", default=os.path.join(ROOT, "profiles", "r06h_r64n7_profile.md"))
    ap.add_argument("--steps", type=int, default=3000)
    a = ap.parse_args()
    rng = np.random.default_rng(0x1D5)
    # steps per p3: C(R-1-p3, N-4) groups x ceil(C(p3, 3) / 64) steps
    groups = list(range(3, R - (N - 4)))
    w = np.array([comb(R - 1 - p3, N - 4) * ((comb(p3, 3) + 63) // 64) for p3 in groups], dtype=float)
    w /= w.sum()
    tot = defaultdict(lambda: [0, 0, 0])  # site -> [cycles, base, instructions]
    for _ in range(a.steps):
        fixed, lanes, act = step_lanes(rng, w, groups)
        pv = np.array(lanes)
        # the client line slot of each lane: index of its (p1, p2) among the step's pairs
        pairs = []
        for p0, p1, p2 in lanes:
            if (p1, p2) not in pairs:
                pairs.append((p1, p2))
        slot = [pairs.index((p1, p2)) for _, p1, p2 in lanes]
        leader = [[l[0], l[1], l[2]] + fixed for l in lanes]
        lead = [m[rng.integers(0, N)] for m in leader]  # (leader member: uniform, a model)

        def site(name, kind, addrs, times=1):
            c, b = cycles(addrs, kind, act)
            t = tot[name]
            t[0] += c * times
            t[1] += b * times
            t[2] += times

        M = lambda row, col: row * CSTRIDE + 2 * col  # u16 (row region, column region) of the matrix
        # client loop: member 0's CQT row and the lane's client line, 16 B (2 quads) per read
        for k in range(NQ // 2):
            site("client loop: member 0's CQT row (b128)", "b128", [p0 * CSTRIDE + 16 * k for p0 in pv[:, 0]])
            site("client loop: client line (b128)", "b128", [s * CSTRIDE + 16 * k for s in slot])
        site("client loop: bin adds (add32)", "add32", [256 * int(t) + 4 * l for l, t in enumerate(rng.integers(0, N, 64))], NC)
        site("epilogue: bin reads + re-zero (b32, w32)", "b32", [4 * l for l in range(64)], 2 * N)
        # Q phase
        for i in range(3):
            site("Q phase: position-table rows X0..X2 (b128)", "b128", [16 * p for p in pv[:, i]])
        for (r_, c_) in ((1, 0), (0, 1), (2, 0), (2, 1), (0, 2), (1, 2)):
            site("Q phase: variable-member distances (u16)", "u16", [M(p[r_], p[c_]) for p in pv])
        # per-position leader records of the 3 variable members
        for i in range(3):
            site("leader: per-position records lrec (b64)", "b64", [8 * p for p in pv[:, i]])
        # leader-dependent reads
        site("leader: cs2 / vcol32 (b64, b32)", "b64", [8 * p for p in lead])
        site("leader: cs2 / vcol32 (b64, b32)", "b32", [4 * p for p in lead])
        site("colocated: leader's table row (b64)", "b64", [16 * p + 8 for p in lead])
        for i in range(3):
            site("colocated: leader column, variable members (u16)", "u16", [M(lead[l], pv[l, i]) for l in range(64)])
        site("digest slot (add64)", "add64", [8 * l for l in range(64)])
    allc = sum(t[0] for t in tot.values())
    allb = sum(t[1] for t in tot.values())
    print("| LDS site (per step) | instructions | cycles | conflict cycles | share of conflicts |")
    print("|---|---|---|---|---|")
    for name, (c, b, n) in sorted(tot.items(), key=lambda x: -(x[1][0] - x[1][1])):
        print(f"| {name} | {n / a.steps:.0f} | {c / a.steps:.1f} | {(c - b) / a.steps:.1f} | "
              f"{(c - b) / max(1, allc - allb):.1%} |")
    print(f"\nModelled: {allc / a.steps:.0f} LDS-array cycles per step, {(allc - allb) / a.steps:.1f} of them "
          f"bank conflicts = {(allc - allb) / allc:.1%} (the sites above; the client lines' build and the "
          f"broadcast reads are left out).")
    if os.path.exists(a.profile):
        t = open(a.profile).read()
        m = re.findall(r"LDS bank-conflict cycles / LDS active cycles: ([0-9.]+)%", t)
        c = re.findall(r"\| SQ_LDS_IDX_ACTIVE \| ([0-9.e+]+) \|", t)
        if m:  # (the last section is the sweep launch; the first, the sample launches)
            print(f"Measured ({os.path.relpath(a.profile, ROOT)}, sweep launch): {m[-1]} % of LDS-array cycles, "
                  f"{float(c[-1]) / (comb(R, N) / 64 * 1.029):.0f} LDS-array cycles per wave-step "
                  f"(SQ_LDS_IDX_ACTIVE over 1.029 steps per 64 configs).")


if __name__ == "__main__":
    sys.exit(main())
