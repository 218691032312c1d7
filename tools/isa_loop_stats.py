"""Instruction mix of a kernel's basic blocks from a gfx950 asm listing
(hipcc --cuda-device-only -S): blocks over `--min` instructions get an opcode
histogram (diagnostic for the VALU count per bucket addition).
Usage: python tools/isa_loop_stats.py listing.s _ZN2pm12k_accumulateINS_8PallasFp [--min 500]"""
import collections
import re
import sys


def main():
    path, prefix = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 500
    s = open(path).read().split("\n")
    i = next(k for k, l in enumerate(s) if l.startswith(prefix) and ":" in l.split(";")[0])
    j = i
    while not s[j].startswith(".Lfunc_end"):
        j += 1
    blocks = [("entry", [])]
    for l in s[i:j]:
        if re.match(r"^\.LBB\d+_\d+:", l):
            blocks.append((l.split(":")[0], []))
            continue
        t = l.strip()
        if not t or t.startswith(";") or t.startswith(".") or t.endswith(":"):
            continue
        blocks[-1][1].append(t.split()[0])
    for name, ops in blocks:
        if len(ops) < mn:
            continue
        c = collections.Counter(ops)
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        mads = sum(v for k, v in c.items() if k.startswith("v_mad_u64") or k.startswith("v_mad_i64"))
        print(f"{name}: {len(ops)} instructions, {valu} VALU ({mads} 64-bit mads), s_nop {c.get('s_nop', 0)}")
        print("   ", c.most_common(24))
    for l in s[j:j + 800]:
        if any(k in l for k in (".vgpr_count", ".vgpr_spill_count", ".sgpr_spill_count")) and prefix[3:] in "".join(s[j:j + 800]):
            print(l.strip())


if __name__ == "__main__":
    main()
