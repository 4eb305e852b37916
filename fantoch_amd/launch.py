"""One process per GPU without torchrun: start `nproc` ranks of one
torch.distributed world on this node (RANK, LOCAL_RANK, WORLD_SIZE,
MASTER_ADDR=127.0.0.1, MASTER_PORT in each child's environment) and wait for
them.  The launching process never touches HIP: the children are separate
programs (no fork of an initialised runtime, no exec of this process), the
GPUs are counted in a short-lived child process (count_gpus), and the first
rank seen to fail ends the others.  A rendezvous port taken by another
program between free_port() and the ranks' bind is retried on a new port
(a rank exits with PORT_IN_USE when its rendezvous cannot bind).

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

PORT_IN_USE = 98  # a rank's exit code when its rendezvous port is taken (EADDRINUSE)


def count_gpus() -> int:
    """Visible GPUs, counted in a child process so that this process never
    initialises HIP (on ROCm builds of torch without amdsmi, device_count()
    falls back to hipGetDeviceCount, which initialises the runtime)."""
    out = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                         capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        raise RuntimeError(f"counting GPUs failed: {out.stderr.strip()[-500:]}")
    return int(out.stdout.strip().splitlines()[-1])


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
              port: Optional[int] = None, port_retries: int = 3) -> int:
    """Run `python argv...` as ranks 0..nproc-1 of one world and return 0 when
    every rank exits 0, else the exit code of the first rank seen to fail (the
    other ranks are then terminated, so their codes would only mask the
    cause).  A rank killed by a signal returns 128 + signal.  A world whose
    first failure is PORT_IN_USE is started again on a new port (at most
    `port_retries` times; not when `port` is given)."""
    if nproc < 1:
        raise ValueError("nproc must be >= 1")
    for attempt in range(port_retries + 1):
        rc, who = _run_once(nproc, argv, env, timeout, port or free_port())
        if rc != PORT_IN_USE or port is not None or attempt == port_retries:
            break
        print(f"launch: rank {who}'s rendezvous port was taken; retrying on a new port", file=sys.stderr)
    if rc:
        print(f"launch: rank {who} failed first (exit code {rc})", file=sys.stderr)
    return rc


def _run_once(nproc, argv, env, timeout, port):
    procs: List[subprocess.Popen] = []
    for r in range(nproc):
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=rank_env(r, nproc, port, env)))
    t0 = time.monotonic()
    rc, who = 0, None
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                who, c = bad[0]
                rc = c if c > 0 else 128 - c
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
    return rc, who
