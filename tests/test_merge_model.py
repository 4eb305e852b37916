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

Round 5 adds the heads' bound (BOTE_MERGE_HEADS): before counting, the merge
tightens the bound to a key t with at least K head records (the first
WIDE_HEAD of each list, their kept prefix) at or below it, found by a radix
select with 10-bit digits over (key - least head) that stops once the chosen
bin holds at most WIDE_SLACK heads beyond the K-th.  The kbound of round 4
alone left ~70 % of every list (the least of the blocks' K-th order
statistics is a loose bound when the blocks sample the same distribution);
`test_gathered_records_stay_near_k` models that realistic case and fails on a
loose bound.
"""
import random

import numpy as np
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


WIDE_HEAD, WIDE_SLACK, WIDE_RANK_MAX, WIDE_FEW = 2, 32, 1024, 64
ONES = 2**64 - 1


def wide_select(values, need, slack=WIDE_SLACK, stop_early=True, aux=None):
    """merge_wide_kernel's wide_select: a value x with at least `need` values
    <= x, by a radix select with 10-bit digits over (v - least) that stops
    once the chosen bin holds at most `slack` values beyond the need-th, or at
    the exact value.  Returns (x, left, inbin, exact, aux) or None (too few):
    a final bin of <= WIDE_FEW values is ranked by (value, aux) and `aux` is
    the selected item's aux word (None when the passes ended the select)."""
    if aux is None:
        aux = [0] * len(values)
    if len(values) < need or need == 0:
        return None
    mn, mx = min(values), max(values)
    if mn == mx:
        return mn, need, len(values), True, None
    s_hi = (mx - mn).bit_length()
    prefix = 0
    while True:
        s_lo = max(s_hi - 10, 0)
        w = s_hi - s_lo
        hist = [0] * 1024
        for v in values:
            v -= mn
            if s_hi >= 64 or (v >> s_hi) == prefix:
                hist[(v >> s_lo) & ((1 << w) - 1)] += 1
        before = 0
        for d, c in enumerate(hist):
            if before < need <= before + c:
                break
            before += c
        left, inbin = need - before, hist[d]
        prefix = (prefix << w) | d
        need = left
        s_hi = s_lo
        if s_hi == 0 or (stop_early and inbin - left <= slack):
            break
        if inbin <= WIDE_FEW:  # one wave finishes a small bin exactly, by (value, aux)
            few = sorted((v, a) for v, a in zip(values, aux) if ((v - mn) >> s_hi) == prefix)
            x, xa = few[left - 1]
            lt, le = sum(1 for v, _ in few if v < x), sum(1 for v, _ in few if v <= x)
            return x, left - lt, le - lt, True, xa
    x = (prefix << s_hi) | ((1 << s_hi) - 1)
    return min(ONES, mn + x), left, inbin, s_hi == 0, None


def head_bound(dumped, K, b0, H=WIDE_HEAD, slack=WIDE_SLACK):
    """merge_wide_kernel's bound record (bk, br): the K-th least head key
    (selected to the exact key), and when several heads tie at it, the
    matching rank among the tied heads (a rank bound that may stop within
    `slack` ranks), so (bk, br) is about the K-th least head record.  The heads are each list's kept prefix of its
    first min(H, K) records: before the first record that is padding, has a
    key of all ones or lies above b0 (the memory after a terminator is
    stale)."""
    heads = []
    for L in dumped:
        for r in L[:min(H, K)]:
            if r == REC_MAX or r[0] == ONES or r[0] > b0:
                break
            heads.append(r)
    ks = wide_select([k for k, _ in heads], K, slack, stop_early=False, aux=[rk for _, rk in heads])
    if ks is None:
        return ONES, ONES
    bk, left, inbin, exact, kaux = ks
    br = ONES
    if kaux is not None and inbin > 1:
        br = kaux  # (the small final bin ranked by (key, rank): the K-th head record)
    elif inbin > 1:
        rs = wide_select([rk for k, rk in heads if k == bk], left, slack)
        if rs is not None:
            br = rs[0]
    return bk, br


def keep(r, b0, bk, br):
    return r != REC_MAX and r[0] <= min(b0, bk) and (r[0] < bk or r[1] <= br)


def prefix_counts(dumped, K, b0, bk=ONES, br=ONES):
    cnt = []
    for L in dumped:
        c = 0
        while c < K and keep(L[c], b0, bk, br):
            c += 1
        cnt.append(c)
    return cnt


def wide_merge(dumped, K, bound, room, heads=True):
    """merge_wide_kernel: the heads' bound record, prefix counts, exclusive
    scan, then one pass ranked by counting or windows of `room`."""
    bk, br = head_bound(dumped, K, bound) if heads else (ONES, ONES)
    cnt = prefix_counts(dumped, K, bound, bk, br)
    off, acc = [], 0
    for c in cnt:
        off.append(acc)
        acc += c
    total = acc
    if total <= WIDE_RANK_MAX:  # one pass: each record's slot is its rank among the gathered
        got = [r for l, L in enumerate(dumped) for r in L[:cnt[l]]]
        out = [REC_MAX] * K
        for x in got:
            r = sum(1 for y in got if y < x)
            if r < K:
                out[r] = x
        return out
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
    union = sorted(r for L in lists for r in L)[:K]
    for heads in (True, False):
        got = wide_merge(dumped, K, bound, room, heads=heads)
        assert got[:len(union)] == union
        assert all(r == REC_MAX for r in got[len(union):])


def test_stale_records_after_a_terminator_are_not_heads():
    """A list shorter than WIDE_HEAD is followed in memory by a previous
    launch's records: they must not count towards the K heads."""
    K = 4
    stale = [(0, 1000 + i) for i in range(8)]  # small keys: would pull the bound down
    dumped = [[(50, 0), REC_MAX] + stale, [(60, 1), REC_MAX] + stale, [(70, 2), (71, 3), (72, 4), (73, 5)]]
    bk, br = head_bound(dumped, K, 2**64 - 1, H=4)
    assert bk >= 71  # the 4th least real head
    got = wide_merge(dumped, K, 2**64 - 1, 4096 - K)
    assert got == [(50, 0), (60, 1), (70, 2), (71, 3)]


@pytest.mark.parametrize("objective", ["mean", "cov"])
@pytest.mark.parametrize("blocks", [64, 512, 4096])
def test_gathered_records_stay_near_k(objective, blocks):
    """The realistic case: every block keeps the K least of a chunk drawn from
    the same distribution (ticket chunks spread each block over the whole
    range), as the R=64 n=7 sweep's 512 blocks do.  kbound alone gathers most
    of every list; with the heads' bound the merge gathers about K + K/8
    records, so it takes the one-pass rank path."""
    rng = np.random.default_rng(blocks)
    K, per_block = 100, 4000
    if objective == "mean":  # integer sums of latencies (S1), heavy ties
        keys = rng.normal(40000, 3000, size=(blocks, per_block)).astype(np.int64).clip(0)
    else:  # COV keys: bits of a positive f64, monotone in the value
        keys = rng.gamma(8.0, 0.02, size=(blocks, per_block)).astype(np.float64).view(np.int64)
    keys = np.sort(keys, axis=1)[:, :K]
    lists, rank = [], 0
    for b in range(blocks):
        lists.append([(int(k), rank + i) for i, k in enumerate(keys[b])])
        rank += per_block
    order = list(range(blocks))
    random.Random(blocks).shuffle(order)
    dumped, kb = dump(lists, K, order)
    loose = sum(prefix_counts(dumped, K, kb))
    bk, br = head_bound(dumped, K, kb)
    tight = sum(prefix_counts(dumped, K, kb, bk, br))
    assert tight >= K
    assert tight <= 2 * K, (tight, loose)
    assert tight <= WIDE_RANK_MAX
    if blocks >= 512:
        assert loose > 10 * K  # round 4's bound alone: most of every list
    got = wide_merge(dumped, K, kb, 4096 - K)
    union = sorted(r for L in lists for r in L)[:K]
    assert got == union


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


@pytest.mark.parametrize("blocks", [64, 544, 4096])
def test_heavy_ties_at_the_kth_key_are_bounded_by_rank(blocks):
    """FPaxos mean keys tie heavily (round 5, R=64 n=7 1/8 shard: over 100
    heads share the least key, and the key bound alone gathered 1,186
    records, past the one-pass limit).  The tied heads' rank bound keeps the
    gathered records near K."""
    rng = np.random.default_rng(7 + blocks)
    K, per_block = 100, 2000
    # ticket chunks spread every block over the whole rank space: the blocks'
    # ranks interleave (distinct across blocks)
    ranks = rng.permutation(blocks * per_block).reshape(blocks, per_block)
    lists = []
    for b in range(blocks):
        # a few distinct small keys, each shared by many configs of the block
        keys = rng.choice([1000, 1000, 1000, 1001, 1003, 1010], size=per_block)
        lists.append(sorted((int(k), int(r)) for k, r in zip(keys, ranks[b]))[:K])
    dumped, kb = dump(lists, K, list(range(blocks)))
    bk, br = head_bound(dumped, K, kb)
    keys_only = sum(prefix_counts(dumped, K, kb, bk, ONES))
    tight = sum(prefix_counts(dumped, K, kb, bk, br))
    assert K <= tight <= 2 * K + 64, (tight, keys_only)
    if blocks >= 544:
        assert keys_only > WIDE_RANK_MAX  # the key bound alone: every list's ties
    got = wide_merge(dumped, K, kb, 4096 - K)
    assert got == sorted(r for L in lists for r in L)[:K]


@pytest.mark.parametrize("seed", range(20))
def test_wide_select_finds_a_valid_bound(seed):
    """wide_select's value x has at least `need` values at or below it; with
    the early stop off it is exactly the need-th least value (any path: the
    radix passes, a one-wave finish of a small bin, a single distinct value)."""
    rng = random.Random(300 + seed)
    n = rng.choice([1, 5, 100, 2000])
    spread = rng.choice([1, 7, 1000, 2**40, 2**63])
    vals = [rng.randrange(spread) + rng.choice([0, 2**62]) for _ in range(n)]
    need = rng.randrange(1, n + 1)
    x, left, inbin, exact, _ = wide_select(vals, need, stop_early=False)
    srt = sorted(vals)
    assert x == srt[need - 1]
    assert exact and inbin == vals.count(x)
    assert sum(1 for v in vals if v < x) + left == need
    y = wide_select(vals, need)[0]
    assert sum(1 for v in vals if v <= y) >= need


@pytest.mark.parametrize("blocks", [1, 8, 32, 49])
def test_few_lists_fall_back_to_kbound(blocks):
    """with fewer than ceil(K / WIDE_HEAD) lists (a small grid, a
    small shard's launch) the heads hold fewer than K records, so the heads'
    bound never applies and the merge gathers every list's prefix at or below
    kbound alone.  Pinned here: no head bound, the gathered count is exactly
    the kbound prefix count, the path it takes (one pass up to WIDE_RANK_MAX
    records, windows beyond), and the K least of the union either way."""
    rng = np.random.default_rng(1000 + blocks)
    K, per_block = 100, 4000
    assert blocks * WIDE_HEAD < K
    keys = np.sort(rng.normal(40000, 3000, size=(blocks, per_block)).astype(np.int64).clip(0), axis=1)[:, :K]
    lists, rank = [], 0
    for b in range(blocks):
        lists.append([(int(k), rank + i) for i, k in enumerate(keys[b])])
        rank += per_block
    order = list(range(blocks))
    random.Random(blocks).shuffle(order)
    dumped, kb = dump(lists, K, order)
    assert head_bound(dumped, K, kb) == (ONES, ONES)  # fewer heads than K: no bound from them
    gathered = sum(prefix_counts(dumped, K, kb))
    assert gathered == sum(prefix_counts(dumped, K, kb, ONES, ONES))
    assert gathered <= blocks * K
    path = "one pass" if gathered <= WIDE_RANK_MAX else "windows"
    assert path == ("one pass" if blocks <= 8 else "windows"), (blocks, gathered)
    union = sorted(r for L in lists for r in L)[:K]
    for room in (K, 4096 - K):
        assert wide_merge(dumped, K, kb, room) == union
