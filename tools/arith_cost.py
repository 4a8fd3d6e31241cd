#!/usr/bin/env python3
"""Costing of alternative arithmetics for the matrix-core Poseidon round (hash_rows_pm_kernel),
beside tools/valu_floor.py (VERDICT r3 "next" 4: cost at least one arithmetic that moves part
of the cube off the VALU; build it only if it beats the floor of 168 VALU per element-round).

Every option is priced per state element and round, per lane, at the measured chip-wide class
rates of profiles/r01/madbench.txt (8192 waves): a VALU instruction of class c costs 1/rate_c
chip-ns per wave-instruction.  MFMA work is priced as matrix-pipe cycles on one SIMD
(v_mfma_i32_32x32x32_i8: 32 cycles, the bf16 32x32x16 cycles, MI355X_MICROARCH.md constants)
and as issue time: round 2/3 measured that an MFMA burst holds the wave's VALU issue ~8 cycles
per MFMA.  One wave-round = 32 states x 12 elements = 6 element-rounds per lane.
Moves, selects and address arithmetic are free in every option (as in the floor).

  A  current: 5 x 26-bit limbs, Montgomery R' = 2^130 (two REDCs per cube), cube packed to 16
     offset bytes + top, MDS on 42 MFMAs per wave-round, digit-column fold on the VALU.
  B  x^2 as an int8 MFMA against a per-element Toeplitz fragment.  The MFMA's A operand may
     vary by row, but a per-state convolution needs an operand that varies with the state on
     both sides: with 4 states per 32x32 tile (block diagonal) each state's 8x8 block yields
     its 31 convolution columns (64 outputs, half redundant), at 1/4 of the tile useful; the
     Toeplitz rows (shifted digit copies, 256 bytes per state) are built by byte permutes.  The
     31 output columns then still need the carry + REDC the VALU does today.
  C  no final REDC: the unreduced x^2 * x (260 bits, 10 columns) carried into 33 offset bytes
     and fed to the MDS MFMA against digits of M * 2^(8j) / R' mod p for j < 33 (13 k-steps per
     tile instead of 7).  Saves one REDC130 but needs a 9-step column carry, twice the packing,
     and an unpaired digit-column fold (the column sums grow to 2^24).
  D  f64 FMA limbs: 6 x 24-bit limbs (products < 2^48, column sums of <= 6 exact in 53 bits),
     36 v_fma_f64 per product; the REDC steps also in f64 (floor / fma splitting per digit).
  E  24-bit integer products: 6 x 24-bit limbs, each 48-bit product as v_mad_u32_u24 (low 32)
     + v_mul_hi_u32_u24 (high 16) accumulated in 32-bit column pairs.
  F  4 x 32-bit words (p = 1 mod 2^32: REDC digit m = -t0 mod 2^32 with no multiply; cube packed
     into 16 bytes with no top byte after a conditional correction, so 6 k-steps per tile).  A
     32 x 32 product is 64 bits, so columns cannot stay lazy as with 26-bit limbs: every product
     enters its column through a 64-bit add (schoolbook rows: v_mad_u64_u32 + the running carry),
     and the REDC keeps signed 64-bit columns (per digit: negate, 64-bit add, 64-bit shift, 64-bit
     add, one v_mad_i64_i32 for m * 11520, 64-bit add of m at word i+4), then carries four words
     and folds the top bit.  Round 4 first priced these carries as 32-bit add-with-carry ops
     (1.109x, "build it"); counted with the 64-bit operations they need (v_lshl_add_u64 class,
     half the v_add_u32 rate, about the v_mad_u64_u32 rate) the option is slower than A.

    python tools/arith_cost.py > profiles/r04/arith_cost.json
"""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MADBENCH = os.path.join(ROOT, "profiles", "r01", "madbench.txt")
MFMA_CYC = 32          # v_mfma_i32_32x32x32_i8 on one SIMD (= bf16 32x32x16)
MFMA_ISSUE_CYC = 8     # VALU issue held per MFMA (measured round 2/3)
SIMDS = 1024
CLOCK_GHZ = 2.1        # under this load (2.1-2.3 GHz)


def rates():
    r = {}
    for line in open(MADBENCH):
        m = re.match(r"(\S+)\s+indep waves\s+8192:.*chip\s+([\d.]+) G wave-instr/s", line)
        if m:
            r[m.group(1)] = float(m.group(2))
    return r


CLASS = {"mad": "v_mad_u64_u32", "alu64": "v_lshl_add_u64", "alu32": "v_add_u32", "u24lo": "v_mad_u32_u24",
         "u24hi": "v_mul_hi_u32_u24", "fma64": "v_fma_f64"}


def redc130():
    # per digit (5): and, 64-bit shift, 64-bit add, 2 mads; bias 3 alu64; output carries
    # 4 x (and, 64-bit shift, add) -- the counts of tools/valu_floor.py
    return {"mad": 10, "alu64": 2 * 5 + 3 + 4 * 2, "alu32": 5 + 4}


def add(*ds):
    out = {}
    for d in ds:
        for k, v in d.items():
            out[k] = out.get(k, 0) + v
    return out


def options():
    fold = {"mad": 12, "alu32": 13, "alu64": 6}
    pack16 = {"alu32": 13}
    A = {"ops": add({"mad": 15, "alu32": 4}, {"mad": 25}, redc130(), redc130(), fold, pack16), "mfma_per_wave_round": 42}
    # B: per element, 2 states' worth of Toeplitz rows per lane (256 B per state over 64 lanes is
    # 4 B per lane per state; a tile holds 4 states and the wave's 32 states need 8 tiles per
    # element): byte permutes ~ 2 per 4 bytes built; the convolution's 31 columns arrive as int32
    # sums and still need the column carry (30 steps) and both REDCs' digit work for the multiply
    B_mfma = 8 * 12                # tiles per element x 12 elements per wave-round (32 states)
    B = {"ops": add({"alu32": 8 * 2 * 4 // 2}, {"alu64": 30, "alu32": 30}, {"mad": 25}, redc130(), redc130(), fold,
                    pack16),
         "mfma_per_wave_round": 42 + B_mfma}
    # C: carry 10 columns into 26-bit limbs (9 x (and, 64-bit shift+add)), pack 33 bytes (~2x pack)
    # the digit-column sums then run over 12 x 33 bytes: |Y_c| < 2^24, so two neighbouring
    # digits no longer pair in 32 bits and the fold takes 16 mads instead of 10
    C = {"ops": add({"mad": 15, "alu32": 4}, {"mad": 25}, redc130(), {"alu64": 9, "alu32": 9}, fold, {"mad": 6},
                    {"alu32": 26}),
         "mfma_per_wave_round": 6 * 13}
    # D: 36 fma per product, 21 for the square (symmetric), REDC in f64: per 24-bit digit (6):
    # floor-split (2 fma), m*p contributions (3 fma), carry (2 fma) ~ 7
    D = {"ops": add({"fma64": 21}, {"fma64": 36}, {"fma64": 2 * 6 * 7}, fold, pack16, {"alu32": 12}),
         "mfma_per_wave_round": 42}
    # E: 2 instructions per 24x24 product (36 / 21 products), column pairs carried (12 alu32 per
    # product set), REDC as A but on 6 digits
    E = {"ops": add({"u24lo": 21, "u24hi": 21}, {"u24lo": 36, "u24hi": 36}, {"alu32": 2 * 24},
                    {"u24lo": 2 * 12, "u24hi": 2 * 12, "alu32": 2 * 20}, fold, pack16),
         "mfma_per_wave_round": 42}
    # F: square 10 products (mad + 64-bit accumulate each), cross terms doubled (7 64-bit
    # shifts), diagonal carried in (8 alu32); REDC: 4 x (1 alu32 + 4 alu64 + 1 mad) + 4 word
    # carries (8 alu64) + top fold (6 alu32); multiply 16 products (mad + 64-bit accumulate);
    # second REDC as the first; fold of the digit columns into 4 words: 8 mads (digit pairs), 4
    # carries (8 alu64), top fold 8 alu32; pack 4 xors
    redc32 = {"mad": 4, "alu64": 16 + 8, "alu32": 4 + 6}
    F = {"ops": add({"mad": 10, "alu64": 10 + 7, "alu32": 8}, redc32, {"mad": 16, "alu64": 16}, redc32,
                    {"mad": 8, "alu64": 8, "alu32": 8}, {"alu32": 4}),
         "mfma_per_wave_round": 36}
    return {"A_current_26bit_montgomery": A, "B_toeplitz_mfma_square": B, "C_unreduced_cube_into_mds_mfma": C,
            "D_f64_fma_limbs": D, "E_u24_products": E, "F_32bit_words": F}


def main():
    R = rates()
    out = {"_note": __doc__.split("\n\n")[0].replace("\n", " "), "class_rates_G_per_s": {c: R[CLASS[c]] for c in CLASS},
           "options": {}}
    base = None
    for name, o in options().items():
        ops = o["ops"]
        valu_ns = 6 * sum(n / R[CLASS[c]] for c, n in ops.items())   # chip-ns per wave-round
        valu_cyc = valu_ns * 1e-9 * SIMDS * CLOCK_GHZ * 1e9          # SIMD cycles per wave-round
        mf = o["mfma_per_wave_round"]
        mfma_pipe = mf * MFMA_CYC
        issue = valu_cyc + mf * MFMA_ISSUE_CYC
        bound = max(issue, mfma_pipe)
        perms = 32 / 27 / (bound / (SIMDS * CLOCK_GHZ * 1e9))
        if base is None:
            base = bound
        out["options"][name] = {"valu_ops_per_element_round": ops, "valu_instr_per_element_round": sum(ops.values()),
                                "mfma_per_wave_round": mf, "valu_issue_cycles_per_wave_round": round(issue),
                                "mfma_pipe_cycles_per_wave_round": mfma_pipe, "bound": "valu-issue" if issue >= mfma_pipe
                                else "mfma-pipe", "perms_per_s_M": round(perms / 1e6, 1),
                                "relative_to_current": round(base / bound, 3)}
    best = max(out["options"].items(), key=lambda kv: kv[1]["relative_to_current"])
    gain = best[1]["relative_to_current"]
    fewer = [k for k, v in out["options"].items() if v["valu_instr_per_element_round"] < 168 and not k.startswith("A_")]
    out["valu_count_below_floor"] = fewer
    out["verdict"] = (f"best: {best[0]} at {gain}x the current arithmetic; "
                      + ("none of the alternatives beats the current one: not built" if best[0].startswith("A_") else
                         "within the model's error (< 5%), and it needs more MFMAs per round and nearly twice the LDS "
                         "operand traffic (13 A fragments per tile instead of 7) with ~24 more live VGPRs in a kernel "
                         "already at ~206: not built" if gain < 1.05
                         else "build it"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
