"""Multi-rank orchestration of the sharded sweep (fantoch_amd/dist.py) under
gloo on CPU: world sizes 2, 3 and 9 (9 exercises the merge tree), each rank a
separate process sweeping its contiguous rank shard through the oracle-backed
stand-in (tests/oracle_sweep.py).  The merged top-K, valid count and digest
must equal one unsharded sweep and the committed oracle fixture
(tests/golden/topk.json, gcp_n5: the full C(20, 5) rank space).  The GPU path (device blocks, RCCL) runs the
same code with backend "nccl" in bench.py; tests/test_gpu_parity.py checks
its device merge against shard-count independence."""
import json
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, K = 5, 16


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup():
    for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import numpy as np

    import oracle as O
    from fantoch_amd.bote import DEFAULT_OBJECTIVES
    from fantoch_amd.planet import Planet
    from oracle_sweep import OracleSweep

    p = Planet.new()
    srv = np.arange(p.R, dtype=np.uint32)
    return OracleSweep(O.OraclePlanet.of(p), srv, srv, N, DEFAULT_OBJECTIVES, K)


def _worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fantoch_amd.dist import sharded_sweep
        sw = _setup()
        res = sharded_sweep(sw, stream=None, device="cpu")
        q.put((rank, res.tops, res.valid, res.digest))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 9])
def test_sharded_sweep_gloo_equals_unsharded(world):
    sw = _setup()
    sw.launch(0, sw.total)
    want = sw.parse_block(sw._blk)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "topk.json")))["cases"]["gcp_n5"]
    assert (int(fx["rank_begin"]), int(fx["rank_end"])) == (0, sw.total)
    for rank, tops, valid, digest in got:
        assert tops == want.tops, f"rank {rank}: merged top-K differs from the unsharded sweep"
        assert (valid, digest) == (want.valid, want.digest)
        assert (valid, digest) == (int(fx["valid"]), int(fx["digest"])), f"rank {rank}: differs from the fixture"
        for o, lst in enumerate(tops):
            assert len(lst) == K
            assert [(k, r) for k, r in lst] == [(int(k), r) for k, r in fx["tops"][o][:len(lst)]]


def test_shard_range_partition():
    from fantoch_amd.dist import shard_range
    for total in (0, 1, 7, 621216192, 5423611200):
        for world in (1, 2, 3, 8):
            rs = [shard_range(total, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
            assert max(e - b for b, e in rs) - min(e - b for b, e in rs) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def test_shard_of_uses_the_sweeps_split():
    """dist.shard_of: one shard is the whole range; a sweep offering `split`
    (bote_sweep_split: equal estimated cost) is cut there, anything else into
    equal rank counts."""
    from fantoch_amd.dist import shard_of

    class Plain:
        total = 100

    class Split(Plain):
        calls = 0

        def split(self, rb, re, parts):
            Split.calls += 1
            return [rb] + [rb + (re - rb) * (i * i) // (parts * parts) for i in range(1, parts)] + [re]

    assert shard_of(Plain(), 1, 0) == (0, 100)
    assert [shard_of(Plain(), 4, r) for r in range(4)] == [(0, 25), (25, 50), (50, 75), (75, 100)]
    assert shard_of(Split(), 1, 0) == (0, 100) and Split.calls == 0
    got = [shard_of(Split(), 4, r) for r in range(4)]
    assert got == [(0, 6), (6, 25), (25, 56), (56, 100)]
    with pytest.raises(ValueError):
        shard_of(Split(), 2, 2)
