"""Static instruction-class mix of one kernel from device assembly, per basic
block, with loop nesting from back-edges.  Classes follow the measured issue
rates (profiles/r02_issue_rate_ops.json): VALU "fast" (~1.6 wave-instr per
CU-clock: add/sub, and/or/xor, lshrrev, mul_f32, ...) and "slow" (~0.95:
min/max, lshlrev, bfe, perm, packed, dot2, 3-source, mul_u24, cvt, ...), plus
SALU, LDS, SMEM, VMEM, scratch and SGPR-spill lane moves.

  hipcc --offload-arch=gfx950 -O3 ... --offload-device-only -S -o k.s bote_group.hip
  python scripts/isa_mix.py k.s <kernel-substring> [--blocks]
"""
import re
import sys
from collections import Counter, defaultdict

FAST = re.compile(r"^v_(add|sub|subrev)_(u32|co_u32|nc_u32|f32|i32)|^v_(and|or|xor|not)_b32|^v_lshrrev_b32|"
                  r"^v_mul_f32|^v_mov_b32|^v_add_co_ci_u32|^v_sub_co_ci_u32|^v_cndmask_b32")
SLOW_HINT = re.compile(r"^v_(min|max|med3|lshlrev|ashrrev|bfe|bfi|perm|pk_|dot2|add3|lshl_add|lshl_or|and_or|or3|"
                       r"xad|mad|mul_u32|mul_lo|mul_hi|cvt|alignbit|alignbyte|sad|fma|cmp|cmpx|readfirstlane|"
                       r"rcp|sqrt|div|ldexp|frexp|fract|trunc|floor|ceil|rndne|bcnt|mbcnt|ffbh|ffbl|lshl|lshr|"
                       r"ashr|mul)")


def classify(op):
    if op.startswith("v_readlane") or op.startswith("v_writelane"):
        return "spill_lane"
    if op.startswith("scratch_") or op.startswith("buffer_") and "off" in op:
        return "scratch"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_"):
        return "vmem"
    if op.startswith("s_waitcnt") or op.startswith("s_nop") or op.startswith("s_barrier") or op.startswith("s_sleep"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        if FAST.match(op):
            return "valu_fast"
        return "valu_slow"
    return "other"


def parse(path, name):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if l.startswith("_Z") and name in l and l.rstrip().endswith(":") or (l.startswith("_Z") and name in l and ":" in l and "@" in l):
            start = i
            break
    if start is None:
        sys.exit(f"kernel {name} not found")
    blocks, order, cur = {}, [], "entry"
    blocks[cur] = []
    order.append(cur)
    for l in lines[start + 1:]:
        s = l.strip()
        if s.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+):", s)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            order.append(cur)
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        op = s.split()[0]
        blocks[cur].append((op, s))
    return blocks, order


def main():
    path, name = sys.argv[1], sys.argv[2]
    show_blocks = "--blocks" in sys.argv
    blocks, order = parse(path, name)
    idx = {b: i for i, b in enumerate(order)}
    # loops: a branch in block j to a block i <= j makes [i, j] a loop body
    loops = []
    for j, b in enumerate(order):
        for op, s in blocks[b]:
            if op.startswith("s_cbranch") or op == "s_branch":
                tgt = s.split()[-1]
                if tgt in idx and idx[tgt] <= j:
                    loops.append((idx[tgt], j))
    depth = [sum(1 for a, b in loops if a <= i <= b) for i in range(len(order))]
    tot = Counter()
    by_depth = defaultdict(Counter)
    for i, b in enumerate(order):
        c = Counter(classify(op) for op, _ in blocks[b])
        tot.update(c)
        by_depth[depth[i]].update(c)
        if show_blocks and (c["scratch"] or c["spill_lane"] or depth[i] >= 2):
            print(f"{b:>14} depth {depth[i]} n={len(blocks[b]):4d} " +
                  " ".join(f"{k}={v}" for k, v in sorted(c.items())))
    keys = ["valu_fast", "valu_slow", "salu", "lds", "smem", "vmem", "scratch", "spill_lane", "wait", "other"]
    print("depth  " + " ".join(f"{k:>10}" for k in keys))
    for d in sorted(by_depth):
        print(f"{d:5d}  " + " ".join(f"{by_depth[d][k]:10d}" for k in keys))
    print("total  " + " ".join(f"{tot[k]:10d}" for k in keys))
    print("loops:", sorted(set(loops))[:40])


if __name__ == "__main__":
    main()
