"""One process per GPU without torchrun: start `nproc` ranks of one
torch.distributed world on this node (RANK, LOCAL_RANK, WORLD_SIZE,
MASTER_ADDR=127.0.0.1, MASTER_PORT in each child's environment) and wait for
them.  The launching process never touches HIP: the children are separate
programs (no fork of an initialised runtime, no exec of this process), and the
first rank to fail ends the others.

Reference: the reference search has no processes to launch (rayon threads,
fantoch_bote/src/search.rs:209-231); this is the launcher of its multi-GPU
replacement."""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_env(rank: int, world: int, port: int, base: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), GROUP_RANK="0", ROLE_RANK=str(rank))
    return env


def run_world(nproc: int, argv: Sequence[str], env: Optional[Dict[str, str]] = None, timeout: Optional[float] = None,
              port: Optional[int] = None) -> int:
    """Run `python argv...` as ranks 0..nproc-1 of one world and return 0 when
    every rank exits 0, else the first failing rank's exit code (the other
    ranks are terminated).  A rank killed by a signal returns 128 + signal."""
    if nproc < 1:
        raise ValueError("nproc must be >= 1")
    port = port or free_port()
    procs: List[subprocess.Popen] = []
    for r in range(nproc):
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=rank_env(r, nproc, port, env)))
    t0 = time.monotonic()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0] if bad[0] > 0 else 128 - bad[0]
                break
            if all(c == 0 for c in codes):
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                rc = 124
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc
