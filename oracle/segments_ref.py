"""ORACLE — test infrastructure only (tests/ may import it; the product never does).

Python restatement of how the reference cuts one program trace into step segments:
  segment_planner.rs:93-276   WinterfellSegmentPlanner::plan_segments
  segment_planner.rs:283-334  compute_segment_features_for_levels / compute_segment_feature_mask
  vm/trace/mod.rs             slice_trace_segment_with_layout (SegmentLayout::from_full_columns:
                              the segment's columns picked out of the full layout by name)
  prove.rs:1057-1134          prove_segment (effective mask, layout, boundaries)
  prove.rs:1197-1287          compute_segment_boundary_bytes
  prove.rs:292-423,1289-1392  build_air_pi_for_trace (VM output, usage mask)
  utils.rs:312-339            vm_state_hash_row_with_layout
Operates on the C oracle's full traces (oracle_lib.build_trace) and ops given as
(kind name, fields) via zkl_op records; checked against zkl_slice_segment in
tests/test_segments.py.
"""
import ctypes as C

FM_POSEIDON, FM_VM, FM_VM_EXPECT, FM_SPONGE, FM_MERKLE, FM_RAM = 1, 2, 16, 32, 64, 128
SPONGE_KINDS = {18, 19}        # ZKL_OP_SABSORBN, ZKL_OP_SSQUEEZE
MERKLE_KINDS = {20, 21, 22}    # ZKL_OP_MERKLE_FIRST / _STEP / _LAST
RAM_KINDS = {16, 17}           # ZKL_OP_LOAD, ZKL_OP_STORE


def column_names(ram: bool, merkle: bool):
    """Columns::width order (vm/layout.rs:183-313) as names; optional RAM / Merkle blocks."""
    names = [f"lane{i}" for i in range(12)] + ["g_map", "g_final"] + [f"g_r{j}" for j in range(27)] + ["mask"]
    names += [f"r{i}" for i in range(8)] + [f"op{k}" for k in range(17)]
    for grp in ("dst0", "a", "b", "c", "dst1"):
        names += [f"sel_{grp}{i}" for i in range(8)]
    names += [f"sel_s_bit{i}" for i in range(30)] + [f"sel_s_active{i}" for i in range(10)] + ["imm", "eq_inv"]
    if ram:
        names += ["ram_sorted", "ram_s_addr", "ram_s_clk", "ram_s_val", "ram_s_is_write", "ram_s_last_write",
                  "ram_gp_unsorted", "ram_gp_sorted"]
    if merkle:
        names += ["merkle_g", "merkle_dir", "merkle_sib", "merkle_acc", "merkle_first", "merkle_last", "merkle_leaf"]
    names += ["pi_prog", "pc"] + [f"rom_op{k}" for k in range(17)] + ["pose_active"]
    names += [f"gadget{i}" for i in range(32)] + ["rom_s0", "rom_s1", "rom_s2"]
    return names


def plan_segments(n_ops: int, max_rows: int):
    levels = 1
    while levels < n_ops:
        levels *= 2
    if levels * 32 <= max_rows:
        return [(0, levels * 32)]
    per = max(max_rows // 32, 1)
    out, lvl = [], 0
    while lvl < levels:
        end = min(levels, lvl + per)
        out.append((lvl * 32, end * 32))
        lvl = end
    return out


def features(kinds):
    return (any(k in SPONGE_KINDS for k in kinds), any(k in RAM_KINDS for k in kinds),
            any(k in MERKLE_KINDS for k in kinds))


def segment_mask(base: int, kinds):
    sp, rm, mk = features(kinds)
    m = 0
    if base & FM_VM:
        m |= FM_VM
    if base & FM_VM_EXPECT:
        m |= FM_VM_EXPECT
    if base & FM_RAM and rm:
        m |= FM_RAM
    if base & FM_MERKLE and mk:
        m |= FM_MERKLE
    if base & FM_SPONGE and sp:
        m |= FM_SPONGE
    if base & FM_POSEIDON and (sp or mk):
        m |= FM_POSEIDON
    return m if (m != 0 and m != base) else base


def _get(t, n, col, row):
    e = t[col * n + row]
    return e.lo | (e.hi << 64)


def slice_segment(oracle, full, n_full, kinds, pi_full, r0, r1):
    """Returns (trace as F128 array, AirPublicInputs, width, state_in, state_out)."""
    import pyref
    sp, rm, mk = features(kinds)
    full_names = column_names(rm, mk)
    idx = {nm: i for i, nm in enumerate(full_names)}
    lvl0, lvl1 = r0 // 32, min(r1 // 32, len(kinds))
    eff = segment_mask(pi_full.feature_mask, kinds[lvl0:lvl1])
    seg_names = column_names(bool(eff & FM_RAM), bool(eff & FM_MERKLE))
    m = r1 - r0
    t = (oracle.F128 * (len(seg_names) * m))()
    for c, nm in enumerate(seg_names):
        src = idx[nm] * n_full + r0
        C.memmove(C.byref(t, c * m * 16), C.byref(full, src * 16), m * 16)
    pi = oracle.AirPublicInputs()
    C.memmove(C.byref(pi), C.byref(pi_full), C.sizeof(pi))
    pi.segment_feature_mask = eff

    def put(f, v):
        f.lo, f.hi = v & (2**64 - 1), v >> 64

    put(pi.pc_init, _get(full, n_full, idx["pc"], r0))
    for nm, row, f in (("ram_gp_unsorted", r0, pi.ram_gp_unsorted_in), ("ram_gp_unsorted", r1 - 1, pi.ram_gp_unsorted_out),
                       ("ram_gp_sorted", r0, pi.ram_gp_sorted_in), ("ram_gp_sorted", r1 - 1, pi.ram_gp_sorted_out)):
        put(f, _get(full, n_full, idx[nm], row) if nm in idx else 0)
    for i in range(3):
        put(pi.rom_s_in[i], _get(full, n_full, idx[f"rom_s{i}"], r0))
        put(pi.rom_s_out[i], _get(full, n_full, idx[f"rom_s{i}"], r1 - 32 + 28))
    sidx = {nm: i for i, nm in enumerate(seg_names)}
    g = lambda nm, row: _get(t, m, sidx[nm], row)  # noqa: E731
    # vm_output_from_trace_with_layout: last final row with a dst0 selector
    pi.vm_out_reg, pi.vm_out_row = 0, 29
    for lvl in range(m // 32 - 1, -1, -1):
        rf = lvl * 32 + 28
        hit = [i for i in range(8) if g(f"sel_dst0{i}", rf) == 1]
        if hit:
            pi.vm_out_reg, pi.vm_out_row = hit[0], rf + 1
            break
    mask = bits = 0
    ram_seg = "ram_sorted" in sidx
    for r in range(m):
        fin = r % 32 == 28
        op = lambda k: g(f"op{k}", r) != 0  # noqa: E731
        if fin and (op(9) or op(7)):
            mask |= 1
        for bit, k in ((1, 10), (2, 11), (3, 12), (4, 14), (5, 13), (6, 6)):
            if fin and op(k):
                mask |= 1 << bit
        if op(8):
            mask |= 1 << 7
        if ram_seg and r + 1 < m and g("ram_sorted", r) and g("ram_sorted", r + 1) and \
                g("ram_s_addr", r) == g("ram_s_addr", r + 1):
            mask |= 1 << 8
            for i in range(32):
                if g(f"gadget{i}", r):
                    bits |= 1 << i
    pi.vm_usage_mask, pi.ram_delta_clk_bits = mask, bits

    def state(row):
        return pyref.blake3(b"zkl/vm/state-v1" + b"".join(g(f"r{i}", row).to_bytes(16, "little") for i in range(8)))

    return t, pi, len(seg_names), state(0), state(m - 1)
