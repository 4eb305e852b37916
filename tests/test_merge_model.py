"""Model of the one-launch top-K merge and the bounded list dump (CPU).

The device path (DESIGN.md §4 "The list dump"): each group-kernel block keeps
the K least (key, rank) records of its configs; at its dump it publishes its
K-th key with an atomicMin (fantoch_amd/csrc/bote_group.hip, `a.kbound`) and
writes only the records whose key is at or below the least K-th key seen so
far, then a terminator; `merge_wide_kernel` (bote_kernels.hip) counts each
list's prefix at or below the final bound, gathers the prefixes in windows of
`room` records and keeps the K least with a sort per window.

This restates that procedure in plain Python with small sizes (ties in the
keys, blocks that finish in any order, windows smaller than the gathered
records) and checks it against the K least of all configs: the argument that
no record of the union's top-K is dropped is the thing under test.  The HIP
kernels themselves are checked on the GPU (tests/test_gpu_*.py, every
fixture's top-K).
"""
import random

import pytest

REC_MAX = (2**64 - 1, 2**64 - 1)


def block_lists(rng, n_blocks, per_block, K, key_range):
    lists = []
    rank = 0
    for _ in range(n_blocks):
        recs = []
        for _ in range(per_block):
            recs.append((rng.randrange(key_range), rank))
            rank += 1
        lists.append(sorted(recs)[:K])
    return lists


def dump(lists, K, order):
    """Each block in `order` publishes its K-th key, then writes its prefix."""
    bound = 2**64 - 1
    out = [None] * len(lists)
    for b in order:
        L = lists[b]
        if len(L) == K:
            bound = min(bound, L[K - 1][0])
        out[b] = [r for r in L if r[0] <= bound] + [REC_MAX]
    return out, bound


def wide_merge(dumped, K, bound, room):
    """merge_wide_kernel: prefix counts, exclusive scan, windows of `room`."""
    cnt = []
    for L in dumped:
        c = 0
        while c < K and L[c] != REC_MAX and L[c][0] <= bound:
            c += 1
        cnt.append(c)
    off, acc = [], 0
    for c in cnt:
        off.append(acc)
        acc += c
    total = acc
    have = []
    w0 = 0
    while w0 < total:
        nxt = total
        got = []
        for l, L in enumerate(dumped):
            if cnt[l] == 0 or off[l] < w0:
                continue
            if off[l] + cnt[l] - w0 <= room:
                got.extend(L[:cnt[l]])
            else:
                nxt = min(nxt, off[l])
        have = sorted(have + got)[:K]
        w0 = nxt
    return have + [REC_MAX] * (K - len(have))


@pytest.mark.parametrize("seed", range(12))
def test_bounded_dump_and_wide_merge_keep_the_k_least(seed):
    rng = random.Random(seed)
    K = rng.choice([1, 3, 10, 32])
    n_blocks = rng.choice([1, 5, 40, 130])
    per_block = rng.choice([0, 2, K, 3 * K])
    key_range = rng.choice([3, 50, 10**6])  # 3: heavy ties at the K-th key
    lists = block_lists(rng, n_blocks, per_block, K, key_range)
    order = list(range(n_blocks))
    rng.shuffle(order)
    dumped, bound = dump(lists, K, order)
    room = rng.choice([K + 1, 2 * K, 64, 4096 - K])
    room = max(room, K)  # (a list of K records always fits one window)
    got = wide_merge(dumped, K, bound, room)
    union = sorted(r for L in lists for r in L)[:K]
    assert got[:len(union)] == union
    assert all(r == REC_MAX for r in got[len(union):])


def test_bound_is_no_tighter_than_the_union_kth_key():
    rng = random.Random(7)
    K = 10
    lists = block_lists(rng, 50, 40, K, 20)
    _, bound = dump(lists, K, list(range(50)))
    union = sorted(r for L in lists for r in L)[:K]
    assert union[-1][0] <= bound


@pytest.mark.parametrize("seed", range(6))
def test_per_wave_sample_minima_bound_the_kth_key(seed):
    """The top-K seed (bote_capi.hip sample_seed, FastArgs::smin_wave): each
    wave's slot is the least key over the chunks it took, and the seed is the
    K-th least slot (all-ones when fewer than K slots hold a key).  K slots at
    or below the seed are K distinct configs of the range, so the seed is an
    upper bound on the range's K-th key."""
    rng = random.Random(100 + seed)
    K = rng.choice([1, 5, 100])
    waves = rng.choice([64, 300, 4096])
    chunks = [[rng.randrange(10**4) for _ in range(rng.randrange(0, 64))] for _ in range(waves * 8)]
    slots = [2**64 - 1] * waves
    order = list(range(len(chunks)))
    rng.shuffle(order)  # tickets: any wave may take any chunk
    for i, c in enumerate(order):
        w = i % waves
        if chunks[c]:
            slots[w] = min(slots[w], min(chunks[c]))
    # (seed_kernel: all-ones, no bound, with fewer than K slots)
    seed_key = sorted(slots)[K - 1] if waves >= K else 2**64 - 1
    every = sorted(k for ch in chunks for k in ch)
    if len(every) >= K and seed_key != 2**64 - 1:
        assert every[K - 1] <= seed_key
