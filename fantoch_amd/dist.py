"""Multi-GPU sharding of the sweep: one process per GPU, contiguous colex rank
shards, per-GPU top-K on the device, one all-gather of the fixed-size result
blocks (RCCL over xGMI with backend "nccl"; gloo on CPU for tests) and a
deterministic merge.  The merge order is by (key, rank), so the result does not
depend on the number of shards (tests/test_dist.py, tests/test_gpu_parity.py).
"""
from __future__ import annotations

from typing import Tuple


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced split of [0, total) (per-config cost is constant)."""
    return total * rank // world, total * (rank + 1) // world


def sharded_sweep(sweep, stream=None, group=None):
    """Run `sweep` (fantoch_amd.bote.Sweep) over this rank's shard and return
    the merged result of all ranks (every rank gets the same result)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    b, e = shard_range(sweep.total, world, rank)
    st = stream if stream is not None else torch.cuda.current_stream().cuda_stream
    sweep.launch(b, e, st)
    nbytes = sweep.result_bytes()
    blk = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    sweep.result_device(blk.data_ptr(), st)
    if world == 1:
        return sweep.parse_block(blk.cpu().numpy())
    gathered = torch.empty(world * nbytes, dtype=torch.uint8, device="cuda")
    dist.all_gather_into_tensor(gathered, blk, group=group)
    out = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    sweep.merge_device(gathered.data_ptr(), world, out.data_ptr(), st)
    return sweep.parse_block(out.cpu().numpy())
