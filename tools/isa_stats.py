"""Register use / spills of the kernels in a gfx950 assembly listing, and an instruction histogram
of one kernel's body (diagnostic; the listing comes from
  hipcc <library CFLAGS> --cuda-device-only -S quantized_spectrum_cartography_amd/csrc/qsc_pass.hip -o pass.s)

  python tools/isa_stats.py pass.s [kernel-substring [line-range a:b]]
"""
import re
import sys
from collections import Counter


def kernels(lines):
    out = []
    cur = {}
    for l in lines:
        m = re.match(r"\s+\.name:\s+(\S+)", l)
        if m:
            cur = {"name": m.group(1)}
            out.append(cur)
        for key in ("vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                    "group_segment_fixed_size"):
            m = re.match(r"\s+\.%s:\s+(\d+)" % key, l)
            if m and cur:
                cur[key] = int(m.group(1))
    return out


def short(name):
    return name.replace("_ZN12_GLOBAL__N_1", "")[:48]


def body(lines, sub):
    for i, l in enumerate(lines):
        if re.match(r"^_Z\S*:", l) and sub in l.split(":")[0]:
            j = i
            while not lines[j].strip().startswith("s_endpgm"):
                j += 1
            return lines[i:j + 1]
    return []


def loops(b, min_len=60):
    """Backward branches (loops) of a kernel body with their instruction mix."""
    labels = {}
    for i, l in enumerate(b):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = i
    for i, l in enumerate(b):
        m = re.search(r"s_c?branch\w*\s+(\.LBB\S+)", l)
        if m and labels.get(m.group(1), i + 1) < i:
            ins = [x.split()[0] for x in b[labels[m.group(1)]:i]
                   if x.startswith("\t") and not x.strip().startswith((";", "."))]
            if len(ins) < min_len:
                continue
            c = Counter(ins)
            v = sum(n for op, n in c.items() if op.startswith("v_"))
            tr = sum(n for op, n in c.items() if re.match(r"v_(exp|log|rcp|sqrt|rsq)_f32", op))
            print("loop %5d-%5d  instrs %4d  valu %4d  trans %3d  ds %3d  vmem %3d  salu %3d  nop %3d" % (
                labels[m.group(1)], i, len(ins), v, tr,
                sum(n for op, n in c.items() if op.startswith("ds_")),
                sum(n for op, n in c.items() if op.startswith(("global_", "buffer_"))),
                sum(n for op, n in c.items() if op.startswith("s_") and op != "s_nop"), c["s_nop"]))


def main():
    lines = open(sys.argv[1]).read().split("\n")
    sub = sys.argv[2] if len(sys.argv) > 2 else None
    for k in kernels(lines):
        if sub is None or sub in k["name"]:
            print("%-50s vgpr %3s spill %s/%s" % (short(k["name"]), k.get("vgpr_count"),
                                                 k.get("vgpr_spill_count"), k.get("sgpr_spill_count")))
    if sub and len(sys.argv) == 4 and sys.argv[3] == "loops":
        loops(body(lines, sub))
    elif sub and len(sys.argv) > 3:
        b = body(lines, sub)
        a, z = (int(x) for x in sys.argv[3].split(":"))
        ops = Counter(l.split()[0] for l in b[a:z] if l.startswith("\t") and not l.strip().startswith((";", ".")))
        for op, n in ops.most_common(60):
            print("%6d %s" % (n, op))
        print("VALU", sum(n for op, n in ops.items() if op.startswith("v_")))


if __name__ == "__main__":
    main()
