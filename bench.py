"""Benchmark: BASELINE.json's metric — region configs evaluated/sec on the
synthetic 64-region planet, n=7, f=1,2 (621,216,192 configs per step).

A step = one full exhaustive sweep: every config gets compute_stats (all 10
histogram keys, FPaxos best-COV leader), compute_score validity, and enters the
device top-K (K=100 x 5 objectives); the per-GPU lists are merged on the device
(and all-gathered over RCCL when N > 1).  The rank space is split into N
contiguous shards, one per GPU, so total work per step is fixed (strong
scaling).  Inputs (the planet, the lists) are resident in HBM before timing.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload r64n7|r128n6|gcp]
  N>1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "region configs evaluated/sec (1/2/4/8 GPUs), synthetic 64-region planet n=7 f=1,2"
KERNEL_NAMES = {"group": "sweep_group_kernel<N> (bote_group.hip)", "fast": "sweep_fast_kernel<N> (bote_sweep.hip)",
                "generic": "eval_kernel<N,false> (bote_kernels.hip)"}
VALU_PEAK_TOPS = 78.6  # 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md chip table)


def work_per_config(n: int, C: int) -> int:
    """SURVEY.md §8d algorithmic int ops per config, W(n, C)."""
    mf = min(n // 2, 2)
    return n * n + (C + n) * n + (1 + mf) * (C + n) + 3 * n * C + mf * (C + n) + 2 * (2 * mf + 1) * (C + n)


def workloads():
    return {
        "r64n7": dict(R=64, n=7, desc="synthetic R=64 planet (splitmix64 seed 0x5EED0064), n=7, f=1,2, "
                                     "clients = all 64 regions + colocated"),
        "r128n6": dict(R=128, n=6, desc="synthetic R=128 planet (seed 0x5EED0128), n=6, f=1,2"),
        "gcp": dict(R=None, n=5, desc="GCP 20-region planet, n=5"),
    }


def cpu_baseline(planet, n, budget_s=12.0):
    """The reference-faithful CPU restatement (oracle/, 'port') timed on this
    host's cores over a bounded contiguous slice of the same rank space."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import oracle as O
    from fantoch_amd import _lib
    from fantoch_amd.bote import DEFAULT_OBJECTIVES

    o = O.OraclePlanet.of(planet)
    srv = np.arange(planet.R, dtype=np.uint32)
    total = _lib.binomial(planet.R, n)
    threads = max(1, min(16, os.cpu_count() or 1))
    rp = (110.0, 35.0, 0.0, 15.0)
    mid = total // 2
    # calibrate, then size the sample to ~budget_s of wall time
    cal = 2000 * threads
    t0 = time.perf_counter()
    o.sweep(srv, srv, n, mid, mid + cal, DEFAULT_OBJECTIVES, 100, rp, 2, threads)
    dt = max(time.perf_counter() - t0, 1e-6)
    count = int(max(cal, min(total - mid, cal * budget_s / dt)))
    t0 = time.perf_counter()
    o.sweep(srv, srv, n, mid, mid + count, DEFAULT_OBJECTIVES, 100, rp, 2, threads)
    dt = time.perf_counter() - t0
    return {"value": count / dt, "unit": "configs/s", "cores": threads, "kind": "port",
            "sample": f"{count} consecutive colex ranks from rank {mid} of {total}, full compute_stats + "
                      f"compute_score + top-K per config (oracle/bote_oracle.cpp, std::thread x {threads})",
            "seconds": round(dt, 3)}


def load_traffic(tag):
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(p):
        try:
            return json.load(open(p)).get(tag)
        except Exception:
            return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="r64n7", choices=list(workloads()))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from fantoch_amd import _lib
    from fantoch_amd.bote import DEFAULT_OBJECTIVES, DEFAULT_RANKING, DevicePlanet, Sweep
    from fantoch_amd.dist import shard_range, sharded_sweep
    from fantoch_amd.planet import Planet

    wl = workloads()[args.workload]
    planet = Planet.new() if wl["R"] is None else Planet.synthetic(wl["R"])
    n = wl["n"]
    dp = DevicePlanet(planet, local)
    srv = np.arange(planet.R, dtype=np.uint32)
    # digest=True: every config's 10 histogram moments and leader feed a
    # checksum, so none of compute_stats' work can be skipped.
    sweep = Sweep(dp, srv, srv, n, DEFAULT_OBJECTIVES, K=100, ranking=DEFAULT_RANKING, digest=True)
    total = sweep.total
    b, e = shard_range(total, world, rank)
    stream = torch.cuda.current_stream().cuda_stream

    def step():
        return sharded_sweep(sweep, stream)

    for _ in range(args.warmup):
        res = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    sweep.timing_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    kern_ms, launches = sweep.timing()
    tmax = torch.tensor([dt, kern_ms / max(launches, 1)], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dt, kavg_ms = float(tmax[0]), float(tmax[1])

    if rank == 0:
        W = work_per_config(n, planet.R)
        shard = e - b
        achieved = shard * W / (kavg_ms * 1e-3) / 1e12  # T int-ops/s, dominant kernel
        traffic = load_traffic(f"{args.workload}_n{world}")
        grid, block, lds = sweep.geometry()
        out = {
            "metric": METRIC if args.workload == "r64n7" else f"region configs evaluated/sec, {wl['desc']}",
            "value": total * args.steps / dt,
            "unit": "configs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic" if wl["R"] else "gcp",
            "config": {"workload": wl["desc"], "regions": planet.R, "n": n, "configs_per_step": total,
                       "keys": 10, "objectives": len(DEFAULT_OBJECTIVES), "K": 100,
                       "parallelism": f"rank-shard x{world}", "grid": grid, "block": block, "lds_bytes": lds,
                       "kernel_path": sweep.kernel_path()},
            "roofline": {"bound": "valu", "achieved": achieved, "peak": VALU_PEAK_TOPS, "unit": "Tops/s",
                         "frac": achieved / VALU_PEAK_TOPS, "traffic": traffic,
                         "work_per_config": W, "kernel_ms_avg": kavg_ms,
                         "kernel": KERNEL_NAMES[sweep.kernel_path()]},
            "result_check": {"valid": res.valid, "digest": res.digest,
                             "top_score_rank": res.tops[0][0][1] if res.tops[0] else None},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(planet, n)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
