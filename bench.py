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
       or python bench.py --gpus N, which starts the N ranks itself
       (fantoch_amd/launch.py; the launching process never touches the GPU).
The world size must equal --gpus (the run is refused otherwise), and n_gpus in
the line is the world that formed, with a census all-gathered over the
data-path backend as evidence (`world`).
BOTE_BENCH_REHEARSAL=1 (diagnostics only, never a bench line to quote): N
ranks share the visible GPUs round-robin and gather over gloo, to rehearse
the N-rank path on a 1-GPU box; the line is marked "rehearsal".
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


def work_per_config_group(n: int, C: int) -> int:
    """DESIGN.md §5 replacement W' (the `roofline.achieved` figure): the group
    algorithm's per-config ops with the work it shares counted once per group
    (amortised to ~0 per config) or once per sweep (column sums).
      3(n-1) + 3(n-3)   quorum rows: the 3 variable members' rows gathered, each
                        fixed member's sorted row gets 3 insertions
      4C + n            nearest server: per Input client the min over the 3
                        variable members and the group's nearest fixed member;
                        a colocated client is its own nearest server
      (1+mf)(C+n)       leaderless adds (af1, af2, e)
      3n                FPaxos leader choice (closed-form S, V per leader from
                        the sweep-wide column sums)
      4mf + n           FPaxos moments: closed form (Input), leader column (Colocated)
      2(1+mf)(C+n)      sum and sum of squares of the leaderless keys
    R=64 n=7: 968 ops (SURVEY's W counts 2,955: per-leader client loops and the
    all-member nearest-server scan that this algorithm never performs)."""
    mf = min(n // 2, 2)
    return 3 * (n - 1) + 3 * (n - 3) + 4 * C + n + (1 + mf) * (C + n) + 3 * n + 4 * mf + n + 2 * (1 + mf) * (C + n)


def work_per_config_keys(n: int, C: int) -> int:
    """W' of the extended key set (BASELINE config 5): W' plus,
    per Tempo quorum table the compute_stats keys lack (NX: 2 at n = 6, 7 --
    q = 2, 3), one add, one sum and one square per client (Input + colocated),
    and per leader and f the FPaxos moments from the column sums (3 ops) and
    the best-by-mean compare (1 op).  R=128 n=6: 1,780 + 804 + 48 = 2,632."""
    mf = min(n // 2, 2)
    m = n // 2
    base = {m + f for f in range(1, mf + 1)} | {m + (m + 1) // 2}
    ext = {2} | ({3, 4} if mf >= 2 else set())
    nx = len(ext - base)
    return work_per_config_group(n, C) + 3 * nx * (C + n) + 4 * mf * n


def workloads():
    return {
        "r64n7": dict(R=64, n=7, keys=0, desc="synthetic R=64 planet (splitmix64 seed 0x5EED0064), n=7, f=1,2, "
                                              "clients = all 64 regions + colocated"),
        "r128n6": dict(R=128, n=6, keys=1, desc="BASELINE config 5: synthetic R=128 planet (seed 0x5EED0128), n=6, "
                                                "f=1,2, compute_stats keys + Tempo tiny/write keys + FPaxos all "
                                                "leaders (BOTE_KEYS_TEMPO_ALL_LEADERS), 8 objectives"),
        "r128n6_base": dict(R=128, n=6, keys=0, desc="synthetic R=128 planet (seed 0x5EED0128), n=6, f=1,2, "
                                                     "the 10 compute_stats keys only"),
        "gcp": dict(R=None, n=None, keys=0, desc="GCP 20-region planet, every config of n=3..13 step 2 (main_gcp)"),
    }


def host_cpu_share() -> int:
    """CPUs this process may use: the affinity mask, capped by the job's CPU
    share when the launcher states one (OMP_NUM_THREADS; 16 per GPU on the
    GPU box, whose nproc shows every CPU of the machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    return max(1, n)


def cpu_baseline(planet, n, keys=0, objectives=None, budget_s=10.0, nsample=1_000_000, seed=0x5EED0001,
                 cap_s=60.0):
    """The reference-faithful CPU restatement (oracle/, 'port') timed on this
    host over a seeded uniform sample of the workload's rank space (BASELINE.md:
    "uniform sample of 10^6 ranks (fixed seed)"), with the workload's own key
    set and objectives (config 5: the extended keys, CONFIG5_OBJECTIVES):
      * all of this job's CPUs over the 10^6 sampled ranks (fewer only when the
        estimated time exceeds cap_s; the line then says how many);
      * one thread -- the reference's own parallelism for a single client set
        (search.rs:209-211: rayon only splits client sets) -- over a prefix of
        the same draw sized to about budget_s of work."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import oracle as O
    from fantoch_amd import _lib
    from fantoch_amd.bote import DEFAULT_OBJECTIVES

    objs = list(objectives or DEFAULT_OBJECTIVES)
    o = O.OraclePlanet.of(planet)
    srv = np.arange(planet.R, dtype=np.uint32)
    total = _lib.binomial(planet.R, n)
    rp = (110.0, 35.0, 0.0, 15.0)
    ranks = np.random.default_rng(seed).integers(0, total, size=nsample, dtype=np.uint64)

    def run(count, threads):
        t0 = time.perf_counter()
        o.sweep_ranks(srv, srv, n, ranks[:count], objs, 100, rp, 2, threads, keys)
        return time.perf_counter() - t0

    share = host_cpu_share()
    cal = 200
    rate1 = cal / max(run(cal, 1), 1e-6)
    c1 = int(max(cal, min(nsample, rate1 * budget_s)))
    d1 = run(c1, 1)
    if share > 1:
        calc = min(nsample, 200 * share)
        raten = calc / max(run(calc, share), 1e-6)
        cn = int(min(nsample, max(calc, raten * cap_s)))
        dn = run(cn, share)
    else:
        cn, dn = c1, d1
    key_set = "extended key set (Tempo tiny/write + FPaxos all leaders)" if keys else "the 10 compute_stats keys"
    return {"value": cn / dn, "unit": "configs/s", "cores": share, "kind": "port",
            "sample": f"{cn} colex ranks drawn uniformly from [0, {total}) (numpy default_rng({seed:#x})), "
                      f"{key_set}, {len(objs)} objectives, full compute_stats + compute_score + top-K per config "
                      f"(oracle/bote_oracle.cpp oracle_sweep_ranks, std::thread x {share})",
            "seconds": round(dn, 3), "nproc": os.cpu_count(), "cpu_share": share,
            "single_thread": {"value": c1 / d1, "unit": "configs/s", "cores": 1,
                              "sample": f"the first {c1} ranks of the same draw", "seconds": round(d1, 3)}}


GCP_NS = (3, 5, 7, 9, 11, 13)  # Search::compute_configs: n in (min_n..=max_n).step_by(2) (search.rs:241-246)


def cpu_baseline_gcp(planet, ns=GCP_NS):
    """SURVEY.md §8d for BASELINE configs 1 and 2: the reference-faithful CPU
    restatement (oracle/, 'port') over EVERY GCP config, in full: config 1
    (n = 3, 5) and config 2 (n = 3..13 step 2, the reference's own
    compute_configs), at 1 thread (the reference's parallelism for one client
    set, search.rs:209-211) and at this job's CPU share."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import oracle as O
    from fantoch_amd import _lib
    from fantoch_amd.bote import DEFAULT_OBJECTIVES

    o = O.OraclePlanet.of(planet)
    srv = np.arange(planet.R, dtype=np.uint32)
    share = host_cpu_share()

    def run(nset, threads):
        cfgs, t0 = 0, time.perf_counter()
        for n in nset:
            total = _lib.binomial(planet.R, n)
            o.sweep(srv, srv, n, 0, total, DEFAULT_OBJECTIVES, 100, (110.0, 35.0, 0.0, 15.0), 2, threads)
            cfgs += total
        dt = time.perf_counter() - t0
        return {"configs": cfgs, "seconds": round(dt, 3), "value": cfgs / dt, "threads": threads}

    c2_1, c2_n = run(ns, 1), run(ns, share)
    c1_1, c1_n = run((3, 5), 1), run((3, 5), share)
    return {"value": c2_n["value"], "unit": "configs/s", "cores": share, "kind": "port",
            "sample": f"every GCP config of n = {list(ns)} ({c2_n['configs']} configs), in full: compute_stats + "
                      f"compute_score + top-K per config (oracle/bote_oracle.cpp, std::thread x {share})",
            "nproc": os.cpu_count(), "cpu_share": share,
            "config2_single_thread": c2_1, "config2_all": c2_n, "config1_single_thread": c1_1, "config1_all": c1_n}


def main_gcp(args):
    """BASELINE configs 1-2 on one GPU: a step sweeps EVERY GCP config of
    n = 3..13 step 2 (507,604 configs; the reference's compute_configs) with
    compute_stats + compute_score + the device top-K, each n checked against
    its oracle fixture (tests/golden/topk.json).  Launch-bound: these are
    parity cases next to the CPU baseline, not the headline."""
    import numpy as np
    import torch

    from fantoch_amd import _lib
    from fantoch_amd.bote import DEFAULT_OBJECTIVES, DEFAULT_RANKING, DevicePlanet, Sweep
    from fantoch_amd.planet import Planet

    if int(os.environ.get("WORLD_SIZE", "1")) != 1 or args.gpus != 1:
        sys.exit("bench.py: --workload gcp runs on one GPU")
    torch.cuda.set_device(0)
    planet = Planet.new()
    dp = DevicePlanet(planet, 0)
    srv = np.arange(planet.R, dtype=np.uint32)
    sweeps = [Sweep(dp, srv, srv, n, DEFAULT_OBJECTIVES, K=100, ranking=DEFAULT_RANKING, digest=True) for n in GCP_NS]
    stream = torch.cuda.current_stream().cuda_stream
    total = sum(sw.total for sw in sweeps)
    # every sweep's result block goes to its own pinned buffer on the stream;
    # one synchronisation per step, then the host parses the six blocks
    hosts = [torch.empty(sw.result_bytes(), dtype=torch.uint8, pin_memory=True) for sw in sweeps]

    def step():
        for sw, h in zip(sweeps, hosts):
            sw.launch(0, sw.total, stream)
            sw.result_device(h.data_ptr(), stream)
        torch.cuda.current_stream().synchronize()
        return [sw.parse_block(h.numpy()) for sw, h in zip(sweeps, hosts)]

    for _ in range(args.warmup):
        res = step()
    torch.cuda.synchronize()
    for sw in sweeps:
        sw.timing_reset()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kern = sum(sw.timing()[0] for sw in sweeps) / max(args.steps, 1)
    fx = json.load(open(os.path.join(ROOT, "tests", "golden", "topk.json")))
    for n, r in zip(GCP_NS, res):
        c = fx["cases"][f"gcp_n{n}"]
        K = fx["K"]
        if (r.valid, str(r.digest)) != (c["valid"], c["digest"]) or \
                [[[str(k), rk] for k, rk in lst[:K]] for lst in r.tops] != c["tops"]:
            sys.exit(f"bench.py: GCP n={n} differs from the oracle fixture tests/golden/topk.json")
    W = sum(sw.total * work_per_config(sw.n, planet.R) for sw in sweeps)
    achieved = W / (kern * 1e-3) / 1e12
    out = {
        "metric": "region configs evaluated/sec, GCP 20-region planet, every config of n=3..13 step 2 (BASELINE "
                  "configs 1-2: the reference's compute_configs)",
        "value": total * args.steps / dt, "unit": "configs/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u32", "data": "gcp",
        "config": {"workload": "GCP R=20 (latency_gcp), n = 3,5,7,9,11,13, all configs, 10 keys, 5 objectives, K=100",
                   "configs_per_step": total, "kernel_paths": [sw.kernel_path() for sw in sweeps]},
        "roofline": {"bound": "launch", "achieved": achieved, "peak": VALU_PEAK_TOPS, "unit": "Tops/s",
                     "frac": achieved / VALU_PEAK_TOPS, "traffic": None, "work_per_config": "SURVEY W(n, 20)",
                     "kernel_ms_per_step": kern,
                     "note": "six sweeps of 1,140..167,960 configs: launch- and merge-bound, not a roofline case"},
        "result_check": {"fixture": "every n equal to tests/golden/topk.json (oracle, all ranks)",
                         "valid": [r.valid for r in res]},
    }
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_gcp(planet)
    print(json.dumps(out), flush=True)


def load_fixture(workload):
    """The full-sweep result the line is checked against, and its label:
    tests/golden/syn_<workload>_full.json (the oracle over every rank,
    scripts/oracle_full_sweep.py), else tests/golden/syn_<workload>_pin.json
    (a regression pin, NOT the oracle: config 5's 5.4e9 configs are beyond the
    oracle here; scripts/pin_r128n6.py: the group kernel equals the exact
    generic kernel at full size and the oracle re-derived every reported
    record), else (None, None)."""
    g = os.path.join(ROOT, "tests", "golden")
    p = os.path.join(g, f"syn_{workload}_full.json")
    if os.path.exists(p):
        fx = json.load(open(p))
        return fx, f"equal to tests/golden/syn_{workload}_full.json (oracle, all {fx['rank_end']} ranks)"
    p = os.path.join(g, f"syn_{workload}_pin.json")
    if os.path.exists(p):
        fx = json.load(open(p))
        return fx, (f"equal to tests/golden/syn_{workload}_pin.json: regression pin of all {fx['rank_end']} ranks "
                    "(group kernel == exact generic kernel at full size, every reported record re-derived by the "
                    "oracle; NOT an oracle sweep)")
    return None, None


def rederive_records(planet, n, keys, objectives, tops):
    """The checker half of the CPU leg (rank 0, after the timed region): every
    record the device reported is re-derived by the oracle -- compute_stats
    (+ the extended keys) and compute_score on those configs -- and, per
    objective, the oracle's ordered list over the reported configs must equal
    the device's list (keys bit-exact, (key, rank) order).  Returns a summary
    or exits non-zero."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import oracle as O
    from fantoch_amd.bote import DEFAULT_RANKING

    o = O.OraclePlanet.of(planet)
    srv = np.arange(planet.R, dtype=np.uint32)
    rp = (DEFAULT_RANKING.min_mean_fpaxos_improv, DEFAULT_RANKING.min_mean_epaxos_improv,
          DEFAULT_RANKING.min_fairness_fpaxos_improv, DEFAULT_RANKING.min_mean_decrease)
    nrec = 0
    for oi, obj in enumerate(objectives):
        recs = [(int(k), int(rk)) for k, rk in tops[oi]]
        t, _, _ = o.sweep_ranks(srv, srv, n, [rk for _, rk in recs], [obj], max(len(recs), 1), rp,
                                DEFAULT_RANKING.ft_metric.value, threads=host_cpu_share(), keys=keys)
        if [(int(k), int(rk)) for k, rk in t[0]] != recs:
            sys.exit(f"bench.py: objective {oi}'s reported records differ from the oracle's re-derivation")
        nrec += len(recs)
    return f"all {nrec} reported records ({len(objectives)} objectives) re-derived by the oracle: keys and order equal"


def lib_build():
    """Identity of the loaded product library: the first 16 hex digits of the
    sha256 of its file (fantoch_amd/lib/libbote_hip.so, or BOTE_LIB_PATH).
    Profile-derived figures (profiles/pmc.json, traffic.json) carry the build
    they were measured on, and the line quotes them only for the same build."""
    import hashlib

    from fantoch_amd import _lib

    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def load_pmc(tag):
    """Per-workload PMC figures committed under profiles/pmc.json
    (scripts/summarize_profile.py): VALU instructions per config-lane etc."""
    p = os.path.join(ROOT, "profiles", "pmc.json")
    if os.path.exists(p):
        try:
            return json.load(open(p)).get(tag)
        except Exception:
            return None
    return None


def load_traffic(tag):
    """HBM bytes per launch of the sweep kernel (profiles/traffic.json):
    {"bytes": B, "build": lib_build() of the profiled library, "source": ...}."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(p):
        try:
            t = json.load(open(p)).get(tag)
        except Exception:
            return None
        return t if isinstance(t, dict) else None
    return None


def profile_figures(pmc, traffic, build, shard, kavg_ms):
    """The line's profile-derived fields: VALU issue utilisation from the
    PMC instruction count and this run's kernel time, and the HBM traffic per
    launch -- each only when it was measured on this very build (ADVICE r04:
    a count from another build is not evidence for this one)."""
    valu, stale = None, []
    if pmc and pmc.get("valu_insts_per_config"):
        insts = pmc["valu_insts_per_config"] * shard / 64
        clk = pmc.get("clock_ghz", 2.4)
        same = pmc.get("build") == build
        valu = {"insts_per_config": pmc["valu_insts_per_config"], "clock_ghz": clk,
                # SQ_INSTS_VALU x 2 cycles (a wave64 VALU op issues over 2 cycles on a
                # SIMD-32) over SIMD-cycles of the live kernel time at the PMC run's clock
                "util": insts * 2 / (1024 * kavg_ms * 1e-3 * clk * 1e9) if same else None,
                "source": pmc.get("source"), "pmc_build": pmc.get("build"), "same_build": same}
        if not same:
            stale.append(f"valu_issue: profiles/pmc.json was measured on build {pmc.get('build')}, not {build}")
    tb = None
    if traffic:
        if traffic.get("build") == build:
            tb = traffic.get("bytes")
        else:
            stale.append(f"traffic: profiles/traffic.json was measured on build {traffic.get('build')}, not {build}")
    return valu, tb, stale


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="r64n7", choices=list(workloads()))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--skip-fixture-check", action="store_true",
                    help="diagnostics (A/B timing while a fixture is being re-pinned): no result check; the line "
                         "says so and is not a bench line to quote")
    args = ap.parse_args()
    # a timing-diagnostics environment must not produce a bench line
    for var in ("BOTE_ABLATE", "BOTE_SWEEP_KERNEL", "BOTE_FORCE_GENERIC", "BOTE_NO_DEF_OBJ", "BOTE_CHUNKS_PER_WAVE"):
        if os.environ.get(var):
            sys.exit(f"bench.py: refusing to run with {var} set (diagnostics only)")

    rehearsal = os.environ.get("BOTE_BENCH_REHEARSAL") == "1"
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # launcher: start the N ranks and exit with their status.  This
        # process never initialises HIP: the GPUs are counted in a child.
        from fantoch_amd.launch import count_gpus, run_world

        ndev = count_gpus()
        if ndev < args.gpus and not (rehearsal and ndev >= 1):
            sys.exit(f"bench.py: --gpus {args.gpus} but {ndev} GPU(s) visible; refusing to report "
                     f"{args.gpus} GPUs")

        sys.exit(run_world(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))

    if args.workload == "gcp":
        return main_gcp(args)

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: world size {world} (WORLD_SIZE) != --gpus {args.gpus}; refusing a mislabeled line")
    ndev = torch.cuda.device_count()
    if not rehearsal and local >= ndev:
        sys.exit(f"bench.py rank {rank}: LOCAL_RANK {local} but {ndev} GPU(s) visible")
    dev_index = local % max(ndev, 1) if rehearsal else local
    torch.cuda.set_device(dev_index)
    if world > 1:
        try:
            if rehearsal:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        except Exception as ex:  # (rank 0's store could not bind MASTER_PORT: the launcher retries)
            if "address already in use" in str(ex).lower() or "eaddrinuse" in str(ex).lower():
                from fantoch_amd.launch import PORT_IN_USE

                print(f"bench.py rank {rank}: {ex}", file=sys.stderr)
                sys.exit(PORT_IN_USE)
            raise

    from fantoch_amd import _lib
    from fantoch_amd.bote import CONFIG5_OBJECTIVES, DEFAULT_OBJECTIVES, DEFAULT_RANKING, DevicePlanet, Sweep
    from fantoch_amd.dist import shard_of, sharded_sweep_start, world_census
    from fantoch_amd.planet import Planet

    wl = workloads()[args.workload]
    planet = Planet.new() if wl["R"] is None else Planet.synthetic(wl["R"])
    n = wl["n"]
    dp = DevicePlanet(planet, dev_index)
    srv = np.arange(planet.R, dtype=np.uint32)
    # digest=True: every config's 10 histogram moments and leader feed a
    # checksum, so none of compute_stats' work can be skipped.
    objectives = CONFIG5_OBJECTIVES if wl["keys"] else DEFAULT_OBJECTIVES
    sweep = Sweep(dp, srv, srv, n, objectives, K=100, ranking=DEFAULT_RANKING, digest=True, keys=wl["keys"])
    total = sweep.total
    b, e = shard_of(sweep, world, rank)  # equal estimated cost (bote_sweep_split)
    stream = torch.cuda.current_stream().cuda_stream

    # Steps are pipelined: step i+1 is enqueued (launch, all-gather, merge,
    # copy of the merged block to pinned host memory) before the host parses
    # step i's result, so the device never waits for the host.  Every step's
    # full result is produced and parsed inside the timed region.
    hosts = [torch.empty(sweep.result_bytes(), dtype=torch.uint8, pin_memory=True) for _ in range(2)]

    def run(k):
        pend, res = None, None
        for i in range(k):
            nxt = sharded_sweep_start(sweep, stream, host=hosts[i % 2])
            if pend is not None:
                res = pend.result()
            pend = nxt
        return pend.result() if pend is not None else res

    res = run(args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    sweep.timing_reset()
    t0 = time.perf_counter()
    res = run(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    kern_ms, launches = sweep.timing()
    tmax = torch.tensor([dt, kern_ms / max(launches, 1)], dtype=torch.float64, device="cuda")
    if world > 1:
        if rehearsal:
            tcpu = tmax.cpu()
            dist.all_reduce(tcpu, op=dist.ReduceOp.MAX)
            tmax = tcpu
        else:
            dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dt, kavg_ms = float(tmax[0]), float(tmax[1])
    census = world_census()
    if census["ranks"] != list(range(world)):
        sys.exit(f"bench.py rank {rank}: the collective saw ranks {census['ranks']}, expected 0..{world - 1}")

    # the result must equal the oracle-pinned full sweep, or config 5's
    # regression pin (every rank holds the merged result)
    fx, label = (None, None) if args.skip_fixture_check else load_fixture(args.workload)
    check = "SKIPPED (--skip-fixture-check: diagnostics, not a bench line)" if args.skip_fixture_check else "no fixture"
    if fx is not None:
        assert (fx["rank_begin"], fx["rank_end"]) == (0, total)
        want = (int(fx["valid"]), int(fx["digest"]), [[(int(k), int(r)) for k, r in t] for t in fx["tops"]])
        got = (res.valid, res.digest, [[(int(k), int(r)) for k, r in t] for t in res.tops])
        if got != want:
            sys.exit(f"bench.py rank {rank}: result differs from {label.split(':')[0].replace('equal to ', '')} "
                     f"(valid {res.valid} vs {fx['valid']}, digest {res.digest} vs {fx['digest']})")
        check = label

    if rank == 0:
        W = work_per_config(n, planet.R)
        Wg = work_per_config_keys(n, planet.R) if wl["keys"] else work_per_config_group(n, planet.R)
        shard = e - b
        build = lib_build()
        grid, block, lds = sweep.geometry()
        valu, traffic, stale = profile_figures(load_pmc(f"{args.workload}_n1"),
                                               load_traffic(f"{args.workload}_n{world}"), build, e - b, kavg_ms)
        # achieved: the VALU lane-ops the sweep kernel issued per launch (the
        # same build's SQ_INSTS_VALU per 64 configs x 64 lanes x configs) over
        # its event-timed launch, against the lane-op peak: it cannot exceed
        # the peak, and it is null when the PMC figures are another build's.
        # W' (the algorithmic count of DESIGN.md §5) and SURVEY's W stay as
        # secondary fields: both count ops the packed instructions do several
        # at a time, so their fractions are not utilisations
        # (insts_per_config: wave-instructions per 64-config step = lane-ops per config)
        issued = valu["insts_per_config"] if valu and valu["same_build"] else None
        achieved = shard * issued / (kavg_ms * 1e-3) / 1e12 if issued else None
        out = {
            "metric": METRIC if args.workload == "r64n7" else f"region configs evaluated/sec, {wl['desc']}",
            "value": total * args.steps / dt,
            "unit": "configs/s",
            "n_gpus": world if not rehearsal else census["distinct_devices"],
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            # per-step time outside the sweep kernel: zeroing, sample launch,
            # seed, fix-up, merge, result copy (and the all-gather at N > 1)
            "step_overhead_ms": dt / args.steps * 1e3 - kavg_ms,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic" if wl["R"] else "gcp",
            "config": {"workload": wl["desc"], "regions": planet.R, "n": n, "configs_per_step": total,
                       "keys": 20 if wl["keys"] else 10, "key_set": wl["keys"], "objectives": len(objectives),
                       "K": 100,
                       "parallelism": f"rank-shard x{world}", "grid": grid, "block": block, "lds_bytes": lds,
                       "kernel_path": sweep.kernel_path(), "lib_build": build},
            "roofline": {"bound": "valu", "achieved": achieved, "peak": VALU_PEAK_TOPS, "unit": "Tops/s",
                         "frac": achieved / VALU_PEAK_TOPS if achieved else None, "traffic": traffic,
                         "work_per_config": issued,
                         "work_def": "issued VALU lane-ops per config: SQ_INSTS_VALU per 64-config wave step x 64 lanes / 64 "
                                     "(profiles/pmc.json, same build only; DESIGN.md §5)",
                         # (W' and SURVEY's W count algorithmic ops, several per packed
                         # instruction: reported as counts, never priced against the VALU peak)
                         "w_prime": {"per_config": Wg, "per_issued_lane_op": Wg / issued if issued else None,
                                     "def": "W' (DESIGN.md §5, bench.work_per_config_%s): algorithmic ops per config, "
                                            "several per packed instruction; a count, not a roofline" % (
                                                "keys" if wl["keys"] else "group")},
                         "survey_w": W,
                         "valu_issue": valu, "kernel_ms_avg": kavg_ms,
                         # VALU issue (SQ_INSTS_VALU x 2 cycles over SIMD-cycles at the PMC run's clock):
                         # frac above at the nominal 2.4 GHz
                         "util": valu["util"] if valu else None,
                         "stale": stale or None,
                         "util_def": "VALU issue: SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x kernel cycles), "
                                     "profiles/pmc.json",
                         "kernel": KERNEL_NAMES[sweep.kernel_path()]},
            "world": dict(census, size=world, shard=[b, e]),
            "result_check": {"valid": res.valid, "digest": res.digest, "deferred": sweep.deferred(stream),
                             "top_score_rank": res.tops[0][0][1] if res.tops[0] else None, "fixture": check},
        }
        if rehearsal:
            out["rehearsal"] = f"{world} ranks on {census['distinct_devices']} GPU(s) over gloo: not a bench line"
        if os.environ.get("BOTE_LIB_PATH"):
            out["config"]["lib_path"] = os.environ["BOTE_LIB_PATH"]  # an A/B build, not the product library
        if not args.no_cpu_baseline:  # (after the timed region; at N > 1 on rank 0 only)
            out["cpu_baseline"] = cpu_baseline(planet, n, wl["keys"], objectives)
            if fx is not None and "pin" in check:
                # a regression pin is not an oracle sweep: the oracle re-derives what it can, every reported record
                out["result_check"]["records"] = rederive_records(planet, n, wl["keys"], objectives, res.tops)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()  # (the other ranks wait for rank 0's CPU baseline)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
