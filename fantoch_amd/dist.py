"""Multi-GPU sharding of the sweep: one process per GPU, contiguous colex rank
shards, per-GPU top-K on the device, one all-gather of the fixed-size result
blocks (RCCL over xGMI with backend "nccl"; gloo on CPU for tests) and a
deterministic merge.  The merge order is by (key, rank), so the result does not
depend on the number of shards (tests/test_dist.py, tests/test_gpu_parity.py).

Reference: the only parallelism of the reference search is a rayon fork-join
over client sets (fantoch_bote/src/search.rs:209-231); the rank-space split is
this build's replacement.
"""
from __future__ import annotations

import os
from typing import Tuple


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous split of [0, total) into equal rank counts."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad shard {rank} of {world}")
    return total * rank // world, total * (rank + 1) // world


def shard_of(sweep, world: int, rank: int) -> Tuple[int, int]:
    """This rank's contiguous shard of [0, sweep.total).  Rank shares of equal
    size are not equal work on the group kernel (small groups cost more per
    config), so a sweep that offers `split` (bote_sweep_split) is cut into
    shards of equal estimated cost; anything else into equal rank counts."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad shard {rank} of {world}")
    split = getattr(sweep, "split", None)
    if world == 1:
        return 0, sweep.total
    if split is None:
        return shard_range(sweep.total, world, rank)
    b = split(0, sweep.total, world)
    return b[rank], b[rank + 1]


def _device_of(sweep, device):
    """The torch device of the sweep's planet (a Sweep), unless given."""
    import torch

    if device is not None:
        return torch.device(device)
    dp = getattr(sweep, "dp", None)
    return torch.device("cuda", dp.device) if dp is not None else torch.device("cuda")


def sharded_sweep(sweep, stream=None, group=None, device=None):
    """Run `sweep` (fantoch_amd.bote.Sweep) over this rank's shard and return
    the merged result of all ranks (every rank gets the same result).

    `sweep` provides launch(rb, re, stream), result_bytes(),
    result_device(ptr, stream), merge_device(src_ptr, n, dst_ptr, stream) and
    parse_block(np.ndarray); the blocks live on `device` (default: the GPU of
    the sweep's planet, whose current stream is used)."""
    return sharded_sweep_start(sweep, stream, group, device).result()


class PendingSweep:
    """A sharded sweep enqueued on the device (launch, all-gather, merge and
    the copy of the merged block to pinned host memory, all stream-ordered):
    result() waits for that copy only, so the host can enqueue the next sweep
    first and parse this one while the device runs it."""

    def __init__(self, sweep, host, event):
        self.sweep, self.host, self.event = sweep, host, event

    def result(self):
        if self.event is not None:
            self.event.synchronize()
        return self.sweep.parse_block(self.host.numpy())


def sharded_sweep_start(sweep, stream=None, group=None, device=None, host=None) -> PendingSweep:
    """Enqueue sharded_sweep without waiting for it.  `host`: a pinned uint8
    CPU tensor of sweep.result_bytes() to copy the merged block into (one per
    sweep in flight; allocated when None)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    b, e = shard_of(sweep, world, rank)
    device = _device_of(sweep, device)
    if device.type != "cuda":
        sweep.launch(b, e, stream)
        blk = torch.empty(sweep.result_bytes(), dtype=torch.uint8, device=device)
        sweep.result_device(blk.data_ptr(), stream)
        if world > 1:
            gathered = torch.empty(world * blk.numel(), dtype=torch.uint8, device=device)
            dist.all_gather_into_tensor(gathered, blk, group=group)
            blk = merge_gathered_device(sweep, gathered, world, stream, device)
        return PendingSweep(sweep, blk, None)
    # Every torch operation below runs with `stream` current: the caching
    # allocator then ties the block, the gather buffer and the merge
    # temporaries to that stream (no reuse while it may still read them), and
    # the collective is ordered after the sweep's writes on it.
    cur = torch.cuda.current_stream(device)
    if stream in (None, 0, cur.cuda_stream):
        st, stream = cur, cur.cuda_stream
    else:
        st = torch.cuda.ExternalStream(stream, device=device)
    with torch.cuda.stream(st):
        sweep.launch(b, e, stream)
        nbytes = sweep.result_bytes()
        if host is None:
            host = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        if world == 1:
            # one rank: the result block straight to pinned host memory
            sweep.result_device(host.data_ptr(), stream)
        else:
            blk = torch.empty(nbytes, dtype=torch.uint8, device=device)
            sweep.result_device(blk.data_ptr(), stream)
            if dist.get_backend(group) == "gloo":
                # gloo moves host memory: gather through the host (a rehearsal of
                # the N-rank path with several ranks on one GPU; RCCL gathers on the device)
                g = torch.empty(world * nbytes, dtype=torch.uint8)
                dist.all_gather_into_tensor(g, blk.cpu(), group=group)
                gathered = g.to(device, non_blocking=False)
            else:
                gathered = torch.empty(world * nbytes, dtype=torch.uint8, device=device)
                dist.all_gather_into_tensor(gathered, blk, group=group)
            blk = merge_gathered_device(sweep, gathered, world, stream, device)
            host.copy_(blk, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(st)
    return PendingSweep(sweep, host, ev)


def merge_gathered_device(sweep, gathered, world: int, stream=None, device=None):
    """Deterministic merge of `world` concatenated result blocks (the all-gather
    output, rank order) into one result block on the device (stream-ordered)."""
    import torch

    device = _device_of(sweep, device)
    nbytes = sweep.result_bytes()
    out = torch.empty(nbytes, dtype=torch.uint8, device=device)
    # merge_device takes at most 8 blocks per call: a tree for larger worlds
    src, n = gathered, world
    while n > 8:
        groups = (n + 7) // 8
        nxt = torch.empty(groups * nbytes, dtype=torch.uint8, device=device)
        for g in range(groups):
            k = min(8, n - 8 * g)
            sweep.merge_device(src.data_ptr() + 8 * g * nbytes, k, nxt.data_ptr() + g * nbytes, stream)
        src, n = nxt, groups
    sweep.merge_device(src.data_ptr(), n, out.data_ptr(), stream)
    return out


def merge_gathered(sweep, gathered, world: int, stream=None, device=None):
    """merge_gathered_device, then the merged result on the host."""
    return sweep.parse_block(merge_gathered_device(sweep, gathered, world, stream, device).cpu().numpy())


def world_census(device=None, group=None):
    """Every rank's (rank, local rank, device ordinal, device identity hash),
    all-gathered over the data-path backend: the evidence that the collective
    spans the ranks (and distinct GPUs) the bench line reports."""
    import hashlib

    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    ident = 0
    if dev.type == "cuda":
        props = torch.cuda.get_device_properties(dev)
        uid = str(getattr(props, "uuid", "")) + str(getattr(props, "pci_bus_id", "")) + props.name
        ident = int.from_bytes(hashlib.sha256(uid.encode()).digest()[:7], "little")
    mine = torch.tensor([rank, local, dev.index or 0, ident], dtype=torch.int64)
    if world == 1:
        rows = [mine.tolist()]
    else:
        on = dev if (dev.type == "cuda" and dist.get_backend(group) != "gloo") else torch.device("cpu")
        out = torch.empty(world * 4, dtype=torch.int64, device=on)
        dist.all_gather_into_tensor(out, mine.to(on), group=group)
        rows = out.view(world, 4).cpu().tolist()
    return {"ranks": sorted(r[0] for r in rows), "local_ranks": [r[1] for r in rows],
            "distinct_devices": len({(r[2], r[3]) for r in rows}),
            "backend": dist.get_backend(group) if dist.is_initialized() else None}
