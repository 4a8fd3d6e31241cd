#!/usr/bin/env python3
"""Algorithm-level VALU floor of the matrix-core Poseidon round (hash_rows_pm_kernel<0>), beside
the instruction-mix ceiling of tools/valu_mix.py.

The mix ceiling prices the kernel's OWN round-loop instructions, so it says how well that
instruction stream is scheduled, not how many instructions the arithmetic needs.  This floor
counts the minimum VALU operations of the algorithm the kernel implements -- per state element
and round: the Montgomery cube on 5 x 26-bit limbs (R' = 2^130), the fold of the 16 int32
digit columns the MFMA returns into limbs, and the byte packing of the cube as the next B
fragment -- each op priced at the measured chip-wide rate of its class (profiles/r01/madbench.txt),
with every non-arithmetic instruction (moves, selects, address arithmetic, waits) free:

  cube      square: 5 v_mad_u64_u32 squares + 10 cross products on doubled limbs (+4 shifts)
            multiply: 25 v_mad_u64_u32
            2 x REDC130: per digit (5): m = col & M26, col+1 += col >> 26 (64-bit shift + add),
            col+1 += m * 45*2^14, col+4 -= m * 2^24 (2 mads); bias: 3 64-bit adds; output: 4
            sequential carries (and, 64-bit shift, add)
  fold      5 neighbouring-digit pairs in 32 bits, 10 v_mad_i64_i32, 4 carries, the 2^128 fold
            (top * (2^26 - 1) + top * 737279 2^26: 2 mads, 2 shifts/ands, 2 adds)
  pack      4 words of 2 funnel shifts/ors, 4 xors, 1 shift (top)

    python tools/valu_floor.py > profiles/r03/valu_floor.json
"""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MADBENCH = os.path.join(ROOT, "profiles", "r01", "madbench.txt")
MIX = os.path.join(ROOT, "profiles", "r02", "valu_mix.json")


def rates():
    r = {}
    for line in open(MADBENCH):
        m = re.match(r"(\S+)\s+indep waves\s+8192:.*chip\s+([\d.]+) G wave-instr/s", line)
        if m:
            r[m.group(1)] = float(m.group(2))
    return r


def main():
    R = rates()
    mad, alu64, alu32 = R["v_mad_u64_u32"], R["v_lshl_add_u64"], R["v_add_u32"]
    redc = {"mad": 2 * 5, "alu64": 2 * 5 + 3 + 4 * 2, "alu32": 5 + 4}
    ops = {
        "cube_square": {"mad": 15, "alu32": 4},
        "cube_multiply": {"mad": 25},
        "cube_redc_x2": {k: 2 * v for k, v in redc.items()},
        "fold": {"mad": 10 + 2, "alu32": 5 + 4 + 4, "alu64": 4 + 2},
        "pack": {"alu32": 4 * 2 + 4 + 1},
    }
    tot = {"mad": 0, "alu64": 0, "alu32": 0}
    for v in ops.values():
        for k, n in v.items():
            tot[k] += n
    per_elem = sum(tot.values())
    # one wave-round = one round of 32 states = 12 x 32 / 64 = 6 element-rounds per lane
    ns = 6 * (tot["mad"] / mad + tot["alu64"] / alu64 + tot["alu32"] / alu32)
    floor_perms = 32 / 27 / (ns * 1e-9)
    mix = json.load(open(MIX))
    out = {
        "_note": "Minimum VALU of the round's arithmetic per state element (see the docstring), priced at the "
                 "chip-wide class rates of profiles/r01/madbench.txt; moves, selects and address arithmetic "
                 "counted free.  The MDS product itself runs on v_mfma_i32_32x32x32_i8 (42 per wave-round).",
        "ops_per_element_round": ops,
        "totals_per_element_round": tot,
        "valu_per_element_round": per_elem,
        "kernel_valu_per_element_round": round(mix["round_loop_valu"] / 6, 1),
        "floor_ns_per_wave_round_chip": round(ns, 4),
        "floor_perms_per_s": round(floor_perms),
        "mix_ceiling_perms_per_s": mix["peak_perms_per_s"],
        "class_rates_G_per_s": {"v_mad_u64_u32": mad, "v_lshl_add_u64": alu64, "v_add_u32": alu32},
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
