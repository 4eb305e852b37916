"""TEST INFRASTRUCTURE — pins a full-size sweep with the CPU oracle.

Runs the reference-faithful CPU restatement (oracle/bote_oracle.cpp,
`oracle_sweep` = search.rs:199-319 compute_stats + :421-472 compute_score per
config, streamed through a (key, rank) top-K) over EVERY colex rank of a
workload, in resumable chunks, and writes the result as a golden fixture:

  tests/golden/<name>_full.json = {valid, digest, tops[5][<=K] (key, rank), ...}

The GPU test `tests/test_gpu_parity.py::test_full_sweep_matches_oracle_fixture`
and bench.py's result check compare the device sweep against it.

  python scripts/oracle_full_sweep.py --workload r64n7 --threads 6

The per-chunk results go to oracle/build/<name>_chunks.jsonl (or --state), so a
killed run resumes where it stopped.  Ranges: --rank-begin/--rank-end restrict
the sweep (window fixtures, e.g. R=128 n=6).  Splitting one sweep over hosts:
--partial with --sweep-begin (a chunk-aligned rank inside the range) and
--time-limit sweeps chunks from there and only appends them to the state file;
concatenating the state files and re-running without --partial writes the
fixture (chunks already present are not recomputed).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
from fantoch_amd.planet import Planet  # noqa: E402

# the bench objectives / ranking (fantoch_amd/bote.py DEFAULT_OBJECTIVES, DEFAULT_RANKING)
OBJECTIVES = [(0, 0), (1, 0), (1, 1), (2, 0), (1, 4)]
RPARAMS = (110.0, 35.0, 0.0, 15.0)
FT_F1F2 = 2
WORKLOADS = {"r64n7": (64, 7), "r128n6": (128, 6)}


def binom(n, k):
    from math import comb
    return comb(n, k)


def merge_tops(parts, K):
    out = []
    for o in range(len(OBJECTIVES)):
        allrec = sorted({tuple(r) for p in parts for r in p[o]})
        out.append([list(r) for r in allrec[:K]])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="r64n7", choices=list(WORKLOADS))
    ap.add_argument("--threads", type=int, default=6)
    ap.add_argument("--chunk", type=int, default=1 << 22)
    ap.add_argument("--K", type=int, default=100)
    ap.add_argument("--rank-begin", type=int, default=0)
    ap.add_argument("--rank-end", type=int, default=None)
    ap.add_argument("--name", default=None)
    ap.add_argument("--state", default=None, help="chunk state file (default oracle/build/<name>_chunks.jsonl)")
    ap.add_argument("--partial", action="store_true", help="sweep chunks only; write no fixture")
    ap.add_argument("--sweep-begin", type=int, default=None, help="first chunk to sweep (chunk-aligned)")
    ap.add_argument("--sweep-end", type=int, default=None, help="stop before this rank (with --partial)")
    ap.add_argument("--time-limit", type=float, default=None, help="stop after this many seconds")
    ap.add_argument("--keys", type=int, default=0,
                    help="1: the extended key set (BOTE_KEYS_TEMPO_ALL_LEADERS) with CONFIG5_OBJECTIVES")
    args = ap.parse_args()

    global OBJECTIVES
    if args.keys:
        from fantoch_amd.bote import CONFIG5_OBJECTIVES
        OBJECTIVES = [tuple(o) for o in CONFIG5_OBJECTIVES]
    R, n = WORKLOADS[args.workload]
    planet = Planet.synthetic(R)
    total = binom(R, n)
    rb = args.rank_begin
    re = total if args.rank_end is None else args.rank_end
    name = args.name or (f"syn_{args.workload}_full" if (rb, re) == (0, total) else
                         f"syn_{args.workload}{'_x' if args.keys else ''}_{rb}_{re}")
    state = args.state or os.path.join(ROOT, "oracle", "build", f"{name}_chunks.jsonl")
    os.makedirs(os.path.dirname(state), exist_ok=True)
    done = {}
    if os.path.exists(state):
        for line in open(state):
            line = line.strip()
            if line:
                try:
                    d = json.loads(line)
                except ValueError:  # a line cut short by a killed run
                    continue
                done[d["begin"]] = d
    o = O.OraclePlanet.of(planet)
    srv = np.arange(R, dtype=np.uint32)
    t_start = time.time()
    swept = 0
    sb = rb if args.sweep_begin is None else args.sweep_begin
    assert (sb - rb) % args.chunk == 0, "--sweep-begin must be chunk-aligned"
    with open(state, "a") as fh:
        for b in range(sb, re if args.sweep_end is None else min(re, args.sweep_end), args.chunk):
            e = min(re, b + args.chunk)
            if b in done:
                continue
            if args.time_limit is not None and time.time() - t_start > args.time_limit:
                print(f"[{name}] time limit reached at rank {b}", flush=True)
                break
            t0 = time.time()
            tops, valid, digest = o.sweep(srv, srv, n, b, e, OBJECTIVES, args.K, RPARAMS, FT_F1F2, args.threads,
                                          keys=args.keys)
            d = {"begin": b, "end": e, "valid": valid, "digest": digest,
                 "tops": [[[int(k), int(r)] for k, r in t] for t in tops], "seconds": time.time() - t0}
            fh.write(json.dumps(d) + "\n")
            fh.flush()
            done[b] = d
            swept += e - b
            el = time.time() - t_start
            left = sum(min(re, x + args.chunk) - x for x in range(rb, re, args.chunk) if x not in done)
            print(f"[{name}] {e - rb}/{re - rb} ranks; {swept / el:.0f} configs/s; ~{left / max(swept / el, 1):.0f} s left",
                  flush=True)
    if args.partial:
        return
    parts = [done[b] for b in sorted(done) if rb <= b < re]
    covered = sum(p["end"] - p["begin"] for p in parts)
    assert covered == re - rb, (covered, re - rb)
    res = {
        "what": f"oracle (oracle/bote_oracle.cpp oracle_sweep) over colex ranks [{rb}, {re}) of the synthetic "
                f"R={R} planet (Planet.synthetic), n={n}, clients = all R regions + colocated",
        "generator": "scripts/oracle_full_sweep.py",
        "R": R, "n": n, "rank_begin": rb, "rank_end": re, "K": args.K, "keys": args.keys,
        "objectives": [list(o) for o in OBJECTIVES], "ranking": list(RPARAMS), "ft_metric": FT_F1F2,
        "valid": sum(p["valid"] for p in parts),
        "digest": sum(p["digest"] for p in parts) % (1 << 64),
        "tops": merge_tops([p["tops"] for p in parts], args.K),
        "cpu_seconds_wall": sum(p["seconds"] for p in parts), "threads": args.threads,
    }
    out = os.path.join(ROOT, "tests", "golden", f"{name}.json")
    with open(out, "w") as fh:
        json.dump(res, fh)
    print(f"wrote {out}: valid={res['valid']} digest={res['digest']}")


if __name__ == "__main__":
    main()
