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
import re
import sys
from collections import Counter, defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from isa_mix import classify  # noqa: E402


# lines of bote_group.hip before the kernel body are helpers (inlined):
# charged, like header code, to the call site
BODY_FIRST = 350


def parse(path, name):
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
        out.append((main_line, block, s.split()[0]))
    return out


DEFAULT_SECTIONS = [
    ("setup+chunks", 350, 491),
    ("group precompute", 492, 562),
    ("step head (lowtab, keys init)", 563, 587),
    ("client lines build", 588, 627),
    ("Q phase (rows, merges)", 628, 847),
    ("byte planes + colocated sums", 848, 869),
    ("leader choice", 870, 942),
    ("XK all leaders", 943, 992),
    ("client loop (Input leaderless)", 993, 1143),
    ("FPaxos + colocated moments", 1144, 1188),
    ("validity", 1189, 1237),
    ("digest", 1238, 1248),
    ("objective keys + score", 1249, 1315),
    ("top-K screen + merge", 1316, 1327),
    ("next group", 1328, 1400),
]


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
