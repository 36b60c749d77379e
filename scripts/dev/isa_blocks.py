#!/usr/bin/env python3
"""Instruction mix per basic block of one kernel in a hipcc -S listing (gfx950).

  hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I include --cuda-device-only \
      -S erp_match_eightpoint_test_amd/csrc/kernels.hip -o /tmp/kernels.s
  python scripts/dev/isa_blocks.py /tmp/kernels.s knn2_filter_kernelILi1 [--min 20] [--dump .LBB5_7]

VALU cycles use the issue costs measured on MI355X by scripts/dev/valu_rates.hip (cycles per
wave64 instruction per SIMD at >= 2 waves per SIMD): 2 for v_add/sub_u32, v_and/or_b32,
shifts by a constant, v_add/mul/fma_f32; 4 for the rest of the VALU (3-operand integer ops,
min/max, cvt, fp64, packed f32, compares).
"""
import collections
import re
import sys

FAST = {"v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32",
        "v_add_f32", "v_mul_f32", "v_fma_f32", "v_fmac_f32", "v_sub_f32", "v_mov_b32"}


def valu_cycles(op: str, line: str) -> int:
    base = op.split("_e32")[0].split("_e64")[0]
    if base in FAST:
        return 2
    if base in ("v_lshrrev_b32", "v_lshlrev_b32", "v_ashrrev_i32"):
        # shift by an inline constant measured at 2, by a VGPR at 4
        parts = line.split(",")
        return 2 if len(parts) > 1 and re.match(r"\s*-?\d+$", parts[1]) else 4
    return 4


def main():
    path, pat = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 20
    dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
    txt = open(path).read()
    m = re.search(r"^(_Z\S*%s\S*):" % re.escape(pat), txt, re.M)
    if not m:
        raise SystemExit(f"no kernel matching {pat}")
    i = m.start()
    j = txt.find(".Lfunc_end", i)
    print(m.group(1))
    blocks, cur = [], ("entry", [])
    for line in txt[i:j].splitlines():
        if re.match(r"^\.LBB\d+_\d+:", line):
            blocks.append(cur)
            cur = (line.split(":")[0], [])
            continue
        s = line.strip()
        if s and not s.startswith(";") and not s.startswith("."):
            cur[1].append(s)
    blocks.append(cur)
    for name, ins in blocks:
        if dump and name == dump:
            print("\n".join(ins))
        ops = [s.split()[0] for s in ins]
        c = collections.Counter(ops)
        valu = [(o, s) for o, s in zip(ops, ins) if o.startswith("v_") and "mfma" not in o]
        cyc = sum(valu_cycles(o, s) for o, s in valu)
        mf = sum(n for k, n in c.items() if "mfma" in k)
        ds = sum(n for k, n in c.items() if k.startswith("ds_"))
        gl = sum(n for k, n in c.items() if k.startswith(("global_", "buffer_")))
        if len(ins) >= mn:
            print(f"{name:12s} n={len(ins):4d} valu={len(valu):4d} valu_cyc={cyc:5d} mfma={mf:3d} "
                  f"ds={ds:3d} glb={gl:3d} top={c.most_common(8)}")


if __name__ == "__main__":
    main()
