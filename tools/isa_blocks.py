"""Per-basic-block instruction mix of one kernel in a hipcc --save-temps .s file (gfx950).

python tools/isa_blocks.py FILE.s KERNEL_SUBSTRING [--min N]
Prints, per block: label, source line, VALU / SALU / LDS / MFMA / VMEM counts and the block's loop annotation, so
the static cost of each region (group op, epilogue, setup) can be read off and multiplied by its dynamic count.
"""
import re
import sys


def kernel_lines(path, sub):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and sub in l)
    end = next((i for i in range(start + 1, len(lines)) if re.match(r"^_Z\S*:", lines[i])), len(lines))
    return lines[start:end]


def classify(op):
    if "mfma" in op:
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "vmem"
    return "other"


def blocks(lines):
    out, cur = [], None
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\d+_\d+):(.*)", l)
        if m:
            cur = {"label": m.group(1), "line": i + 1, "note": m.group(2).strip()[:60], "n": {}}
            out.append(cur)
            continue
        if cur is None:
            cur = {"label": "entry", "line": i + 1, "note": "", "n": {}}
            out.append(cur)
        t = l.strip().split()
        if not t or t[0].startswith((";", ".")):
            continue
        k = classify(t[0])
        cur["n"][k] = cur["n"].get(k, 0) + 1
    return out


def main():
    path, sub = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 0
    tot = {}
    for b in blocks(kernel_lines(path, sub)):
        n = b["n"]
        for k, v in n.items():
            tot[k] = tot.get(k, 0) + v
        if sum(n.values()) < mn:
            continue
        print(f"{b['label']:12s} L{b['line']:5d} valu {n.get('valu', 0):4d} salu {n.get('salu', 0):4d} "
              f"lds {n.get('lds', 0):3d} mfma {n.get('mfma', 0):3d} vmem {n.get('vmem', 0):3d}  {b['note']}")
    print("static totals:", tot)


if __name__ == "__main__":
    main()
