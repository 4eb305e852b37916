"""Source attribution of a kernel's instructions through the DWARF inline
tree, for scripts/isa_lines.py and class_mix_table.py.

The `.loc` directives of a -g assembly listing name the line an instruction
came from, but not where an inlined helper was called: the instructions of
merge_lists, digest_word, pk_min, ... carry the helper's own line, and the
listing's section tables charged them to whatever kernel-body line the
scheduler had emitted last (the R=64 Q phase showed up as
"leader choice").  The device object's DWARF has the inline tree
(DW_TAG_inlined_subroutine: address ranges and DW_AT_call_line), so here an
instruction is charged to
  * its own line, when that line lies in the kernel body of bote_group.hip;
  * else the call line of the innermost inlined call that contains its
    address and whose call site lies in the kernel body (a helper called
    from a lambda defined in the body is charged to the lambda's call of it,
    which is a body line).

  hipcc --offload-arch=gfx950 -O3 -g ... --offload-device-only -c -o k.o bote_group.hip
  python scripts/isa_attrib.py k.o <kernel-substring> BODY_FIRST BODY_LAST

The instruction order equals the `-S` listing's of the same source and flags,
so isa_lines.parse() pairs them by position (BOTE_ISA_OBJ=k.o).
"""
import os
import re
import subprocess
import sys

LLVM = "/opt/rocm/lib/llvm/bin"


def device_object(path):
    """The gfx950 code object of a (bundled) -c output."""
    out = path + ".gfx950"
    if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(path):
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={path}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={out}"], check=True)
    return out


def kernel_instructions(obj, name):
    """(address, mnemonic) of the kernel's instructions, in order."""
    txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", obj], check=True,
                         capture_output=True, text=True).stdout.split("\n")
    out, inside = [], False
    for l in txt:
        m = re.match(r"^([0-9a-f]+) <([^>]+)>:", l)
        if m:
            inside = name in m.group(2) and not m.group(2).endswith(".kd")
            continue
        if not inside:
            continue
        m = re.match(r"^\s+(\S+).*//\s*([0-9A-Fa-f]+):", l)  # (amdgcn: "  op operands  // ADDR: ENC")
        if m:
            out.append((int(m.group(2), 16), m.group(1)))
    return out


def line_table(obj):
    """address -> (file, line), from the DWARF line program (rows sorted by address)."""
    txt = subprocess.run([f"{LLVM}/llvm-dwarfdump", "--debug-line", obj], check=True, capture_output=True,
                         text=True).stdout.split("\n")
    files, rows = {}, []
    for l in txt:
        m = re.match(r"^file_names\[\s*(\d+)\]:", l)
        if m:
            cur = int(m.group(1))
            continue
        m = re.match(r'^\s+name: "([^"]+)"', l)
        if m and "cur" in dir():
            files[cur] = m.group(1)
            continue
        m = re.match(r"^0x([0-9a-f]+)\s+(\d+)\s+(\d+)\s+(\d+)", l)
        if m:
            rows.append((int(m.group(1), 16), int(m.group(4)), int(m.group(2))))
    return files, rows


def inline_tree(obj):
    """Every DW_TAG_inlined_subroutine: (ranges, call_file, call_line, depth)."""
    txt = subprocess.run([f"{LLVM}/llvm-dwarfdump", "--debug-info", obj], check=True, capture_output=True,
                         text=True).stdout.split("\n")
    out, cur = [], None
    for l in txt:
        m = re.match(r"^0x[0-9a-f]+:(\s+)(DW_TAG_\w+)", l)
        if m:
            if cur:
                out.append(cur)
            cur = {"depth": len(m.group(1)), "ranges": [], "file": None, "line": None} \
                if m.group(2) == "DW_TAG_inlined_subroutine" else None
            continue
        if cur is None:
            continue
        for a, b in re.findall(r"\[0x([0-9a-f]+), 0x([0-9a-f]+)\)", l):
            cur["ranges"].append((int(a, 16), int(b, 16)))
        m = re.search(r'DW_AT_call_file\s+\("([^"]+)"\)', l)
        if m:
            cur["file"] = m.group(1)
        m = re.search(r"DW_AT_call_line\s+\((\d+)\)", l)
        if m:
            cur["line"] = int(m.group(1))
        m = re.search(r"DW_AT_low_pc\s+\(0x([0-9a-f]+)\)", l)
        if m:
            cur["low"] = int(m.group(1), 16)
        m = re.search(r"DW_AT_high_pc\s+\(0x([0-9a-f]+)\)", l)
        if m and "low" in cur:
            cur["ranges"].append((cur["low"], int(m.group(1), 16)))
    if cur:
        out.append(cur)
    return out


def attribute(obj_path, name, body_first, body_last, main="bote_group.hip"):
    obj = device_object(obj_path)
    ins = kernel_instructions(obj, name)
    files, rows = line_table(obj)
    tree = [t for t in inline_tree(obj) if t["ranges"]]
    lo, hi = ins[0][0], ins[-1][0] + 1
    tree = [t for t in tree if any(a < hi and b > lo for a, b in t["ranges"])]
    rows = [r for r in rows if lo <= r[0] < hi + 64] or rows
    import bisect
    addrs = [r[0] for r in rows]

    def in_body(f, ln):
        return f is not None and f.endswith(main) and body_first <= ln <= body_last

    # one-line lambdas of the body (`auto s1_of = [&](int l) { ... };`): their
    # instructions are charged to the call, like a helper's (a lambda that
    # only a rare branch calls is then rare, not charged to its definition)
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fantoch_amd", "csrc",
                            main)).read().split("\n")
    one_line = {i + 1 for i, l in enumerate(src) if re.search(r"=\s*\[[&=]?\]\s*\(.*\{.*\};\s*(//.*)?$", l)}

    out = []
    for a, op in ins:
        i = bisect.bisect_right(addrs, a) - 1
        f, ln = (files.get(rows[i][1]), rows[i][2]) if i >= 0 else (None, 0)
        if in_body(f, ln) and ln not in one_line:
            out.append((a, op, ln))
            continue
        best, bd = 0, -1  # the innermost containing call whose site is in the body (and not a one-line lambda)
        for t in tree:
            if t["depth"] > bd and in_body(t["file"], t["line"]) and t["line"] not in one_line and \
                    any(x <= a < y for x, y in t["ranges"]):
                best, bd = t["line"], t["depth"]
        out.append((a, op, best or (ln if in_body(f, ln) else 0)))
    return out


if __name__ == "__main__":
    rows = attribute(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
    for a, op, ln in rows:
        print(f"{a:x} {ln} {op}")
