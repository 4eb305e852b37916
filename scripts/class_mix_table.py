"""Per-section VALU class mix of the bench group kernel, static and modelled
per 64-config step, reconciled against the measured SQ_INSTS_VALU.

  hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DBOTE_ISA_N7 -g \
      --offload-device-only -S -o kg.s fantoch_amd/csrc/bote_group.hip
  BOTE_PSTATS=<pathstats json> python scripts/class_mix_table.py kg.s ILi7ELb1ELb1ELb1ELb0ELb1E profiles/pmc.json \
      r64n7_n1 > profiles/<tag>_class_mix.md
  (optional 5th-7th arguments: R n trips -- the workload, and the client
  loop's unrolled-body trips per step: nq / (2 BIN_UB), two bodies per trip;
  default 64 7 2; the config-5 kernel, -DBOTE_ISA_N6: ... r128n6_n1 128 6 4)

Static: instructions per section (scripts/isa_lines.py markers).  Modelled
dynamic count per step: every basic block of a per-step section runs once per
step, except
  * blocks on the rare paths (f64 arithmetic: COV/mean decisions inside their
    ambiguity bands, the exact leader re-scan, the full score; the deferral
    queue; the block top-K merge under the LDS lock; the sample launch's
    per-chunk minima): 0;
  * the client loop's unrolled body (the lines variant, the block with the
    most v_dot2 or LDS adds and the fewest LDS reads): nq / U times, the
    blocks laid out after it (flush, exit) once; the other client-loop bodies
    (no-lines variant, remainder loops): 0;
  * the block top-K merge (wave_topk, inlined; found by its own source
    lines) and the sample launch's per-chunk minima (`if (a.smin)`): 0;
  * per-group sections (group precompute, next group): groups / steps;
  * per-wave and per-chunk setup: 0 (32 chunks per wave over ~2,370 steps).
Issue cost: fast class ~1.6 wave-instr per CU-clock, slow ~0.95
(profiles/r02_issue_rate_ops.json), so a slow op costs ~1.7 fast ones.
"""
import json
import os
import sys
from collections import Counter, defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from isa_lines import DEFAULT_SECTIONS, parse  # noqa: E402
from isa_mix import classify  # noqa: E402

RARE_MARK = ("v_div_", "global_atomic", "ds_cmpst", "ds_cmpswap", "s_sleep", "s_ff1", "v_rcp_f64", "v_sqrt_f64")
# f64 ARITHMETIC marks a rare path (the exact decisions inside the f64
# ambiguity bands); f64 <-> f32 conversions do not: every step converts the
# leader column's V (vcol) to f32 for the screens, and round 4's model, which
# zeroed every block with any f64 op, missed ~135 VALU per step in the leader
# choice block that holds that conversion
import re  # noqa: E402
RARE_F64 = re.compile(r"^v_(add|mul|fma|mad|ldexp|max|min|cmp[a-z_]*|frexp[a-z_]*|fract|trunc|floor)_f64")


def is_rare_op(o):
    return any(m in o for m in RARE_MARK) or bool(RARE_F64.match(o))
FAST_RATE, SLOW_RATE = 1.6, 0.95


# Rare regions: the body of an `if` that runs for a whole wavefront only when
# some lane takes it, weighted by its measured frequency per wave-step
# (scripts/pathstats.py, the -DBOTE_PATHSTATS build).  A region is the source
# lines from the marker line to its matching closing brace (the marker is the
# `if` line that follows the PSTAT site); a block is charged to the innermost
# region that holds most of its bote_group.hip lines.
RARE_REGIONS = [
    ("if (amb) {  // exact re-scan", "leader re-scan"),
    ("PSTAT(a, 3, amb);", "leader deferred"),
    ("mok = (mom_mean(mf) - mom_mean(ma)) >= a.p_fmean;", "f64 mean test f=1"),
    ("if (defer) {", "validity deferred"),
]
# (the f64 score and COV af1 key bodies hold f64 arithmetic, so their blocks
# are rare by their ops; as line regions they would also take in blocks the
# compiler sinks there, e.g. the digest, whose .loc lines say 1704)


def region_lines(src, marker):
    """(first, last) 1-based lines of the region a marker opens: a marker line
    with an opening brace runs to its matching brace; a PSTAT line, to the
    end of the `if` block on the next line; any other line is itself."""
    i = next(k for k, l in enumerate(src) if marker in l)
    if marker.startswith("PSTAT"):
        i += 1
    if "{" not in src[i]:
        return i + 1, i + 1
    depth = 0
    for k in range(i, len(src)):
        for ch in src[k]:  # (character by character: `} else {` closes the region)
            depth += 1 if ch == "{" else (-1 if ch == "}" else 0)
            if depth == 0 and ch == "}":
                return i + 1, k + 1
    return i + 1, len(src)


def main():
    from math import comb
    path, name = sys.argv[1], sys.argv[2]
    pmc = json.load(open(sys.argv[3])).get(sys.argv[4]) if len(sys.argv) > 4 else None
    # path frequencies per wave-step (BOTE_PSTATS=<pathstats json>): the rare
    # regions and the no-lines client loop are weighted by them; without it,
    # every rare region weighs 0 as before
    pst = json.load(open(os.environ["BOTE_PSTATS"]))["per_step"] if os.environ.get("BOTE_PSTATS") else {}
    R, n, trips = (int(x) for x in sys.argv[5:8]) if len(sys.argv) > 7 else (64, 7, 2)
    groups, steps = comb(R - 3, n - 3), comb(R, n) / 64.0  # groups: the fixed parts above position 3
    per_step_groups = groups / steps
    rows = parse(path, name, raw=True)
    secs = DEFAULT_SECTIONS
    src = open(__file__.rsplit("/", 2)[0] + "/fantoch_amd/csrc/bote_group.hip").read().split("\n")
    # the block top-K merge helper (inlined at its call site): rare after the seed
    wt0 = next(i + 1 for i, l in enumerate(src) if "void wave_topk(" in l)
    wt1 = next(i + 1 for i, l in enumerate(src) if i + 1 > wt0 and l.startswith("}"))
    # the sample launch's per-chunk minima (a.smin): not run by the sweep launch
    sm0 = next(i + 1 for i, l in enumerate(src) if "if (a.smin) {" in l or "if (LA(smin)) {" in l)
    sm1 = next(i + 1 for i, l in enumerate(src) if i + 1 > sm0 and "} else if (!ABLATE(a, 4)) {" in l)
    regions = [(region_lines(src, m), pst.get(name, 0.0)) for m, name in RARE_REGIONS]
    blk_src = defaultdict(Counter)  # bote_group.hip source lines per block
    blk_ops = defaultdict(list)
    blk_lines = defaultdict(Counter)
    merge_blk = set()
    own_line = defaultdict(bool)  # a block with instructions from bote_group.hip lines
    order = []
    blk_opl = defaultdict(list)
    hotl = Counter()
    for ln, b, op, raw_ln in rows:
        blk_opl[b].append((ln, op))
        if b not in blk_ops:
            order.append(b)
        blk_ops[b].append(op)
        own_line[b] |= raw_ln > 0
        if ln:  # (the kernel-body line: inlined helpers count at their call site)
            blk_src[b][ln] += 1
        if wt0 <= raw_ln <= wt1 or sm0 <= raw_ln < sm1:
            merge_blk.add(b)
        if ln:
            s = next((n for n, a, z in secs if a <= ln <= z), "other")
            blk_lines[b][s] += 1
    sec_of = {b: (blk_lines[b].most_common(1)[0][0] if blk_lines[b] else "other") for b in order}
    # the client loop's hot body (the lines variant: the block with the most
    # v_dot2 and the fewest LDS reads), and the run of client-loop blocks laid
    # out with it (its flush and exit); the other variants (no lines, the
    # remainder loops) do not run at R=64 n=7 (<= 16 pairs per step, nq % 4 == 0)
    loop_blocks = [b for b in order if sec_of[b].startswith("client loop")]
    dots = {b: sum(1 for o in blk_ops[b] if o.startswith("v_dot2") or o.startswith("ds_add")) for b in loop_blocks}
    adds = {b: sum(1 for o in blk_ops[b] if o.startswith("ds_add")) for b in loop_blocks}
    big = [b for b in loop_blocks if dots[b] >= 8]
    if any(adds[b] >= 8 for b in loop_blocks):
        # the member-binned loop (BIN kernels): its bodies are the blocks of
        # LDS adds (the epilogue after it has the most v_dot2 but runs once)
        big = [b for b in loop_blocks if adds[b] >= 8]
    hot = min(big, key=lambda b: sum(1 for o in blk_ops[b] if o.startswith("ds_"))) if big else None
    nolines = None
    # BIN with the flush-free loops (round 5): four bodies -- lines / no
    # lines, each with and without the flush.  The bench's one 32-bit sum
    # holds every client, so the flush-free bodies run: the lines body (4
    # quads, 16 LDS adds per iteration) and the no-lines body (2 quads, 8 adds)
    FLUSH_OPS = ("v_lshl_add_u64", "v_add_co_u32_e32", "v_addc_co_u32_e32", "v_cndmask_b32_e32", "v_cndmask_b32_e64")
    nf = [b for b in big if adds[b] >= 8 and not any(o in FLUSH_OPS for o in blk_ops[b])]
    if len(nf) >= 2:
        hot = max(nf, key=lambda b: adds[b])
        nolines = min(nf, key=lambda b: adds[b])
    run = set()
    if hot and any(adds[b] >= 8 for b in loop_blocks):
        # BIN: once per step, the blocks between the lines body and the next
        # loop body (its flush and exit), and the epilogue over the bins (the
        # client-loop block without LDS adds that has the most v_dot2)
        i = order.index(hot) + 1
        while i < len(order) and not (order[i] in big):
            if sec_of[order[i]].startswith("client loop") and adds[order[i]] == 0:
                run.add(order[i])
            i += 1
        tail = [b for b in loop_blocks if adds[b] == 0]
        if tail:
            run.add(max(tail, key=lambda b: sum(1 for o in blk_ops[b] if o.startswith("v_dot2"))))
    elif hot:
        i = order.index(hot)
        while i < len(order) and sec_of[order[i]].startswith("client loop"):
            run.add(order[i])
            i += 1
    static = defaultdict(Counter)
    dyn = defaultdict(Counter)
    for b in order:
        s = sec_of[b]
        c = Counter(classify(o) for o in blk_ops[b])
        static[s].update(c)
        # (top-K blocks made only of header code: the merge's inlined binary searches)
        rare = (b in merge_blk or any(is_rare_op(o) for o in blk_ops[b]) or
                (s.startswith("top-K") and not own_line[b]))
        # the innermost rare region holding most of the block's source lines
        reg = None
        if blk_src[b]:
            for (r0, r1), fr in regions:
                inside = sum(c for ln_, c in blk_src[b].items() if r0 <= ln_ <= r1)
                if inside * 2 > sum(blk_src[b].values()) and (reg is None or r1 - r0 < reg[0][1] - reg[0][0]):
                    reg = ((r0, r1), fr)
        if s.startswith("setup") or s == "other":
            w = 0.0
        elif pst and b in merge_blk and not (sm0 <= min(blk_src[b] or [0]) < sm1):
            w = pst.get("block top-K merge", 0.0)  # (wave_topk under the lock)
        elif pst and reg is not None:
            w = reg[1]
        elif rare:
            w = 0.0
        elif s in ("group precompute", "next group"):
            w = per_step_groups
        elif s.startswith("client loop"):
            # (the other variants' bodies and the remainder loops: 0)
            other_body = b != hot and (adds[b] > 0 or b in big)
            w = float(trips) if b == hot else (1.0 if b in run and not other_body else 0.0)
            if pst and b == hot:
                w *= 1.0 - pst.get("no client lines", 0.0)
            elif pst and b == nolines:
                # the no-lines body (2 quads per iteration: twice the lines
                # body's trips) on the steps with more pairs than line slots
                w = 2.0 * trips * pst.get("no client lines", 0.0)
        else:
            w = 1.0
        if os.environ.get("BOTE_MIX_BLOCKS") and w > 0:  # (diagnostics: the weighted blocks)
            print(f"# {b} {s!r} w={w:.3f} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())) +
                  f" lines={sorted(blk_src[b])[:3]}..{sorted(blk_src[b])[-1:]}", file=sys.stderr)
        for k, v in c.items():
            dyn[s][k] += w * v
        if w > 0 and os.environ.get("BOTE_MIX_LINE"):  # (diagnostics: one line's weighted instructions)
            sel = [o for ln_, o in blk_opl[b] if str(ln_) == os.environ["BOTE_MIX_LINE"]]
            if sel:
                print(f"# {b} w={w:.3f} " + " ".join(sel), file=sys.stderr)
        if w > 0:
            for (ln_, o) in blk_opl[b]:
                if classify(o) in ("valu_fast", "valu_slow", "spill_lane"):
                    hotl[ln_] += w
    if os.environ.get("BOTE_MIX_LINES"):  # (diagnostics: the heaviest source lines, VALU per step)
        for ln_, v in hotl.most_common(int(os.environ["BOTE_MIX_LINES"])):
            print(f"# {v:6.1f}  {ln_:5d}  {src[ln_ - 1].strip()[:110] if ln_ else '?'}", file=sys.stderr)
    print(f"# VALU class mix per section: `{name}`\n")
    print("Static instructions from the device assembly (`-g` line info, scripts/isa_lines.py sections);")
    print("modelled per 64-config step as described in scripts/class_mix_table.py.  Fast class")
    print(f"~{FAST_RATE} wave-instr/CU-clk, slow ~{SLOW_RATE} (profiles/r02_issue_rate_ops.json).\n")
    print("| section | static fast | static slow | per step fast | per step slow | per step spill-lane | "
          "issue cost (fast-op units) | share |")
    print("|---|---|---|---|---|---|---|---|")
    tot = Counter()
    costs = {}
    for s, _, _ in secs + [("other", 0, 0)]:
        d = dyn.get(s, Counter())
        costs[s] = d["valu_fast"] + d["valu_slow"] * FAST_RATE / SLOW_RATE + d["spill_lane"] * FAST_RATE / SLOW_RATE
    allc = sum(costs.values()) or 1.0
    for s, _, _ in secs + [("other", 0, 0)]:
        st, d = static.get(s, Counter()), dyn.get(s, Counter())
        if not st:
            continue
        tot.update(d)
        print(f"| {s} | {st['valu_fast']} | {st['valu_slow']} | {d['valu_fast']:.1f} | {d['valu_slow']:.1f} | "
              f"{d['spill_lane']:.1f} | {costs[s]:.0f} | {costs[s] / allc:.1%} |")
    model = tot["valu_fast"] + tot["valu_slow"] + tot["spill_lane"]
    print(f"| **total** | | | {tot['valu_fast']:.0f} | {tot['valu_slow']:.0f} | {tot['spill_lane']:.0f} | "
          f"{allc:.0f} | |\n")
    print(f"Modelled VALU instructions per step (fast + slow + spill-lane moves): **{model:.0f}**; "
          f"slow share {(tot['valu_slow'] + tot['spill_lane']) / model:.1%}; scratch accesses per step "
          f"{tot['scratch']:.2f}, LDS {tot['lds']:.0f}.")
    if pmc:
        meas = pmc["valu_insts_per_config"]
        # wavefront steps actually run per 64 configs: a group of C(p3, 3) configs takes ceil(/64) steps
        from math import ceil
        ns = R
        real = sum(comb(ns - 1 - p3, n - 4) * ceil(comb(p3, 3) / 64) for p3 in range(3, ns)) / (comb(ns, n) / 64)
        print(f"Measured SQ_INSTS_VALU per 64 configs ({pmc['source']}): **{meas:.0f}**.  Groups run "
              f"{real:.3f} steps per 64 configs (partial last steps), so the model accounts for "
              f"{model * real:.0f} = {model * real / meas:.0%} of it.  "
              + (f"Rare paths (f64 decisions inside their bands, leader re-scans, block top-K merges, the "
                 f"no-lines loop) are weighted by their measured frequency per wave-step "
                 f"({os.environ['BOTE_PSTATS']}); per-chunk setup counts 0."
                 if pst else
                 "The rest is the rare paths (f64 decisions inside their bands, leader re-scans, block top-K "
                 "merges), which run for a whole wavefront when any lane takes them, and per-chunk work."))
        ceil = 1.0 / (tot["valu_fast"] / model / FAST_RATE + (1 - tot["valu_fast"] / model) / SLOW_RATE) / 2.0
        print(f"Issue ceiling of this mix: {ceil:.1%} of the 2-cycle nominal rate; measured "
              f"{pmc['valu_issue_util']:.1%} ({pmc['valu_issue_util'] / ceil:.0%} of the ceiling).")
    print(f"\nClient-loop hot body: `{hot}` ({len(blk_ops[hot]) if hot else 0} instructions per unrolled iteration, "
          f"{trips} iterations per step).")


if __name__ == "__main__":
    main()
