"""Static instruction mix per source section of one kernel, from device
assembly built with -g (the .loc directives map every instruction to the
source line it came from; instructions inlined from headers are charged to
the bote_group.hip call site that is current when they appear).

  hipcc --offload-arch=gfx950 -O3 -g ... --offload-device-only -S -o kg.s bote_group.hip
  python scripts/isa_lines.py kg.s <kernel-substring> [SECTIONS.json]

Sections are (name, first line, last line) ranges of bote_group.hip; the
default set below follows the step loop of sweep_group_kernel.  Classes as in
scripts/isa_mix.py (measured issue rates, profiles/r02_issue_rate_ops.json).
"""
import json
import os
import re
import sys
from collections import Counter, defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from isa_mix import classify  # noqa: E402


# lines of bote_group.hip before the kernel body are helpers (inlined):
# charged, like header code, to the call site


def parse(path, name, raw=False):
    lines = open(path).read().split("\n")
    files = {}
    start = None
    for i, l in enumerate(lines):
        m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', l)
        if m:
            files[int(m.group(1))] = m.group(2)
        if start is None and l.startswith("_Z") and name in l and ":" in l:
            start = i
    if start is None:
        sys.exit(f"kernel {name} not found")
    cur_file, cur_line, main_line = 0, 0, 0
    out = []  # (main-file line, block label, op)
    block = "entry"
    sub = 0
    for l in lines[start + 1:]:
        s = l.strip()
        if s.startswith(".Lfunc_end"):
            break
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            cur_file, cur_line = int(m.group(1)), int(m.group(2))
            if files.get(cur_file, "").endswith("bote_group.hip") and cur_line >= BODY_FIRST:
                main_line = cur_line
            continue
        m = re.match(r"^(\.LBB\d+_\d+):", s)
        if m:
            block = m.group(1)
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        out.append((main_line, block, s.split()[0]) if not raw else
                   (main_line, block, s.split()[0], cur_line if files.get(cur_file, "").endswith("bote_group.hip") else 0))
        if s.startswith("s_cbranch"):
            # a conditional branch ends the basic block: the fall-through is a
            # block of its own (e.g. the code a divergent `if` runs only when
            # some lane takes it), even without a label
            sub += 1
            block = f"{block.split('+')[0]}+{sub}"
    obj = os.environ.get("BOTE_ISA_OBJ")
    if obj:
        # DWARF inline-tree attribution (scripts/isa_attrib.py): an inlined
        # helper's instructions go to their call line in the kernel body, not
        # to the body line the scheduler emitted last; the object's
        # instructions pair with this listing's by position
        from isa_attrib import attribute
        att = attribute(obj, name, BODY_FIRST, BODY_LAST)
        att = att[:len(out)]  # (the object may decode alignment padding after the kernel's last instruction)
        if len(att) != len(out) or any(a[1] != o[2] for a, o in zip(att, out)):
            sys.exit(f"{obj}: its {name} instructions differ from {path}'s (build both from one source)")
        out = [((a[2] or o[0]),) + tuple(o[1:]) for a, o in zip(att, out)]
    return out


# Sections start at marker text in bote_group.hip (so they follow edits)
MARKERS = [
    ("setup+chunks", "sweep_group_kernel(FastArgs a) {"),
    ("group precompute", "// ---------------- per-group, wave-uniform precompute"),
    ("step head (lowtab, keys init)", "while (left) {"),
    ("client lines build", "// ---- PERM: client lines."),
    ("step members (unpack)", "uint32_t pv[3], rv[3];"),
    # the member-binned client loop's one body (a lambda: its instructions
    # carry these lines wherever it runs, before the Q phase on the XK
    # kernels, after the leader choice on the R=64 kernel)
    ("client loop (binned body)", "// ---- BIN: the member-binned client loop, one body"),
    ("Q phase (rows, merges)", "// member m: 0..2 variable, 3.. fixed"),
    ("byte planes + colocated sums", "// ---- PERM: byte planes"),
    ("leader choice", "// ---- FPaxos leader (f = 1"),
    ("XK all leaders", "// ---- XK, before the client loop"),
    ("client loop (Input leaderless)", "// ---- Input leaderless: 3 lane columns"),
    ("FPaxos + colocated moments", "// ---- Input FPaxos from the leader column's sums"),
    ("validity", "// af1's exact V"),
    ("digest", "if ((SI || a.want_digest) && !ABLATE(a, 16))"),
    ("objective keys + score", "// ---- default objectives: 0 SCORE"),
    ("top-K screen + merge", "// ---- top-K: lock-free screen"),
    ("next group", "// (a sample chunk stops at its first group"),
    (None, "// ------------------------------------------------------------- launcher"),
]


def default_sections():
    src = open(__file__.rsplit("/", 2)[0] + "/fantoch_amd/csrc/bote_group.hip").read().split("\n")
    starts = []
    for name, text in MARKERS:
        ln = next(i + 1 for i, l in enumerate(src) if text in l)
        starts.append((name, ln))
    return [(n, a, starts[k + 1][1] - 1) for k, (n, a) in enumerate(starts[:-1])]


DEFAULT_SECTIONS = default_sections()
BODY_FIRST = DEFAULT_SECTIONS[0][1]
BODY_LAST = DEFAULT_SECTIONS[-1][2]


def main():
    path, name = sys.argv[1], sys.argv[2]
    secs = DEFAULT_SECTIONS if len(sys.argv) < 4 else [tuple(x) for x in json.load(open(sys.argv[3]))]
    rows = parse(path, name)
    per = defaultdict(Counter)
    for ln, _, op in rows:
        sec = next((s for s, a, b in secs if a <= ln <= b), "other")
        per[sec][classify(op)] += 1
    keys = ["valu_fast", "valu_slow", "salu", "lds", "vmem", "spill_lane", "scratch", "wait"]
    print(f"{'section':34s} " + " ".join(f"{k:>10s}" for k in keys))
    tot = Counter()
    for s, _, _ in secs + [("other", 0, 0)]:
        c = per.get(s)
        if not c:
            continue
        tot.update(c)
        print(f"{s:34s} " + " ".join(f"{c[k]:10d}" for k in keys))
    print(f"{'total':34s} " + " ".join(f"{tot[k]:10d}" for k in keys))


if __name__ == "__main__":
    main()


def blocks_listing(path, name, lo=563, hi=1330):
    """Per basic block, in layout order: the source-line span and class mix
    (blocks whose instructions come from lines [lo, hi] of bote_group.hip)."""
    rows = parse(path, name)
    order, per, span = [], defaultdict(Counter), {}
    for ln, b, op in rows:
        if b not in per:
            order.append(b)
        per[b][classify(op)] += 1
        if ln:
            a, z = span.get(b, (ln, ln))
            span[b] = (min(a, ln), max(z, ln))
    for b in order:
        a, z = span.get(b, (0, 0))
        if z < lo or a > hi:
            continue
        c = per[b]
        print(f"{b:>14s} lines {a:4d}-{z:4d} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
