"""Summarise a `STEPS=profile` run of scripts/gpu_job.sh (gpurun_out/<TAG>/trace, pmc1..4) into
profiles/<TAG>_profile.md and update profiles/traffic.json.

  python scripts/summarize_profile.py r04d/r64n7 [workload_tag]   (the profile step's output directory)

BOTE_PROFILE_SKIP=N (default: the bench line's own "warmup" count): the first
N sweep launches of each run are the bench's warm-up (the first one pays the clock ramp and the chunk-table
build: 14.85 ms vs 13.84-13.99 ms after it in r05u); they are left out of the
sweep launch's average duration and of the PMC per-dispatch averages (whose
instruction counts do not depend on it, but the clock estimate does).

Per kernel: calls and average duration (rocprofv3 --kernel-trace --stats), then
the per-dispatch PMC averages of each counter pass.  HBM traffic per launch of
the dominant kernel = FETCH_SIZE + WRITE_SIZE (rocprofv3 reports KiB).  The
gfx950 FETCH_SIZE halving applies to 16-B/lane streaming reads only; this
kernel's reads are a few KiB of staging loads, so the figure is used as is and
marked uncalibrated (MI355X_MICROARCH.md "HBM").
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = {"r64n7": 621216192, "r128n6": 5423611200}


def main():
    tag = sys.argv[1]
    wl = sys.argv[2] if len(sys.argv) > 2 else "r64n7_n1"
    src = os.path.join(ROOT, "gpurun_out", tag)
    out = []
    # the profiled library (bench.py's config.lib_build in the runs' own lines):
    # bench.py quotes pmc.json / traffic.json figures only for that build
    build, warmup = None, None
    for lg in ("trace.log", "pmc1.log"):
        p = os.path.join(src, lg)
        if os.path.exists(p):
            for line in open(p, errors="replace"):
                if line.startswith("{") and '"lib_build"' in line:
                    try:
                        d = json.loads(line)
                        build = d["config"]["lib_build"]
                        warmup = d.get("warmup")
                    except (ValueError, KeyError):
                        pass
        if build:
            break
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    rows = list(csv.DictReader(open(stats)))
    out.append(f"# rocprofv3 summary {tag} ({wl})\n")
    out.append(f"library build (sha256 prefix of libbote_hip.so, bench.py lib_build): `{build}`\n")
    out.append("## Kernel trace (`rocprofv3 --kernel-trace --stats`)\n")
    out.append("| kernel | calls | avg ms | min ms | max ms | % |")
    out.append("|---|---|---|---|---|---|")
    dominant = None
    for r in rows:
        name = r["Name"]
        out.append(f"| `{name[:70]}` | {r['Calls']} | {float(r['AverageNs']) / 1e6:.4f} | "
                   f"{float(r['MinNs']) / 1e6:.4f} | {float(r['MaxNs']) / 1e6:.4f} | {float(r['Percentage']):.2f} |")
        if dominant is None:
            dominant = name
    # The sweep kernel runs twice per step: a short sample launch (one step per
    # wave, the top-K seed) and the sweep proper.  Split its dispatches by
    # duration (a sample launch is < 1/4 of the longest) so that the averages
    # below describe the sweep launch alone.
    durs = collections.defaultdict(list)
    tr = os.path.join(src, "trace", "run_kernel_trace.csv")
    if os.path.exists(tr):
        for r in csv.DictReader(open(tr)):
            durs[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    skip = int(os.environ.get("BOTE_PROFILE_SKIP", warmup if warmup is not None else 1))
    main_avg = {}
    for name, ds in durs.items():
        cut = max(ds) / 4
        big, small = [d for d in ds if d >= cut], [d for d in ds if d < cut]
        steady = big[skip:] if len(big) > skip else big
        main_avg[name] = sum(steady) / len(steady)
        if small and "sweep" in name:
            out.append(f"\n`{name[:70]}`: {len(big)} sweep launches, avg **{main_avg[name] / 1e6:.4f} ms** over the "
                       f"{len(steady)} after the first {len(big) - len(steady)} (warm-up; all {len(big)}: "
                       f"{sum(big) / len(big) / 1e6:.4f} ms, each: {', '.join(f'{d / 1e6:.3f}' for d in big)}); "
                       f"{len(small)} sample launches (top-K seed), avg {sum(small) / len(small) / 1e6:.4f} ms")
    counters = collections.defaultdict(lambda: collections.defaultdict(float))
    ndisp = collections.defaultdict(set)
    i = 1
    while os.path.exists(os.path.join(src, f"pmc{i}", "run_counter_collection.csv")):
        rows_i = list(csv.DictReader(open(os.path.join(src, f"pmc{i}", "run_counter_collection.csv"))))
        longest = collections.defaultdict(int)
        for r in rows_i:
            longest[r["Kernel_Name"]] = max(longest[r["Kernel_Name"]],
                                            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        # the warm-up sweep launches (the first `skip` big dispatches of each kernel)
        firsts = collections.defaultdict(list)
        for r in rows_i:
            if int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) >= longest[r["Kernel_Name"]] / 4:
                firsts[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), r["Dispatch_Id"]))
        warm = set()
        for k, lst in firsts.items():
            ids = sorted(set(lst))
            if len(ids) > skip:
                warm |= {d for _, d in ids[:skip]}
        for r in rows_i:
            k = r["Kernel_Name"]
            if r["Dispatch_Id"] in warm:
                continue
            if int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) < longest[k] / 4:
                k = k + " [sample launch]"
            counters[k][r["Counter_Name"]] += float(r["Counter_Value"])
            ndisp[(k, i)].add(r["Dispatch_Id"])
            ndisp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
        i += 1
    out.append("\n## PMC per dispatch (separate `--pmc` passes, averaged over dispatches)\n")
    traffic = None
    pmc = {}
    for k, cs in counters.items():
        if "sweep" not in k and "eval_kernel" not in k:
            continue
        out.append(f"### `{k.replace(' [sample launch]', '')[:80]}`" +
                   (" — sample launches (top-K seed)" if k.endswith("[sample launch]") else "") + "\n")
        out.append("| counter | per dispatch |")
        out.append("|---|---|")
        per = {}
        for c, v in sorted(cs.items()):
            per[c] = v / max(len(ndisp[(k, c)]), 1)
            out.append(f"| {c} | {per[c]:.6g} |")
        if "SQ_WAVE_CYCLES" in per and "SQ_WAIT_ANY" in per:
            w = per["SQ_WAVE_CYCLES"]
            out.append(f"\nwave-cycle split: active {per.get('SQ_ACTIVE_INST_ANY', 0) / w:.1%}, "
                       f"wait (s_waitcnt/barrier) {per['SQ_WAIT_ANY'] / w:.1%}, "
                       f"issue-stall {per.get('SQ_WAIT_INST_ANY', 0) / w:.1%}")
        if "SQ_LDS_BANK_CONFLICT" in per and per.get("SQ_LDS_IDX_ACTIVE"):
            out.append(f"LDS bank-conflict cycles / LDS active cycles: "
                       f"{per['SQ_LDS_BANK_CONFLICT'] / per['SQ_LDS_IDX_ACTIVE']:.1%}")
        if k == dominant and "FETCH_SIZE" in per and "WRITE_SIZE" in per:
            traffic = (per["FETCH_SIZE"] + per["WRITE_SIZE"]) * 1024.0
            out.append(f"HBM traffic per launch (FETCH_SIZE + WRITE_SIZE, KiB -> bytes): {traffic:.4g} B")
        if k == dominant and "SQ_INSTS_VALU" in per:
            cfgs = CONFIGS.get(wl.split("_")[0])
            kns = main_avg.get(k) or next((float(r["AverageNs"]) for r in rows if r["Name"] == k), None)
            if cfgs and kns:
                lanes = cfgs / 64.0
                # GRBM_GUI_ACTIVE is summed over the 8 XCDs
                clk = per["GRBM_GUI_ACTIVE"] / kns / 8 if "GRBM_GUI_ACTIVE" in per else 2.4
                util = per["SQ_INSTS_VALU"] * 2 / (1024 * kns * clk)
                pmc[wl] = {"valu_insts_per_config": per["SQ_INSTS_VALU"] / lanes,
                           "lds_insts_per_config": per.get("SQ_INSTS_LDS", 0) / lanes,
                           "salu_insts_per_config": per.get("SQ_INSTS_SALU", 0) / lanes,
                           "clock_ghz": clk, "kernel_ns": kns, "valu_issue_util": util,
                           "source": f"profiles/{tag.replace('/', '_')}_profile.md", "build": build}
                out.append(f"VALU wave-instructions per config: {pmc[wl]['valu_insts_per_config']:.1f} "
                           f"(LDS {pmc[wl]['lds_insts_per_config']:.1f}, SALU {pmc[wl]['salu_insts_per_config']:.1f}); "
                           f"VALU issue utilisation (SQ_INSTS_VALU x 2 cyc / (1024 SIMD x cycles) at "
                           f"{clk:.2f} GHz): {util:.1%}")
        out.append("")
    open(os.path.join(ROOT, "profiles", f"{tag.replace('/', '_')}_profile.md"), "w").write("\n".join(out) + "\n")
    if pmc:
        p = os.path.join(ROOT, "profiles", "pmc.json")
        d = json.load(open(p)) if os.path.exists(p) else {}
        d.update(pmc)
        json.dump(d, open(p, "w"), indent=1, sort_keys=True)
    if traffic is not None:
        p = os.path.join(ROOT, "profiles", "traffic.json")
        d = json.load(open(p)) if os.path.exists(p) else {}
        d[wl] = {"bytes": traffic, "build": build, "source": f"profiles/{tag.replace('/', '_')}_profile.md"}
        json.dump(d, open(p, "w"), indent=1, sort_keys=True)
    print("\n".join(out))


if __name__ == "__main__":
    main()
