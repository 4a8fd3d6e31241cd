"""§8(f)3 — the per-segment trace builder (zkl_program_new / zkl_build_segment_trace): every
segment of a program written from one pass over the ops, without the full trace, equal bit for
bit to prove_segment's input side over the full trace (build_full_trace + slice_trace_segment_
with_layout + compute_segment_boundary_bytes, vm/trace/mod.rs:316-524, prove.rs:1057-1287) --
zkl_slice_segment(zkl_build_trace(..)) -- and to the oracle twin orc_build_segment_trace, which
streams every level through a 32-row scratch.

Programs: the reference's real examples rollup-bench (RAM, sponge; its sorted RAM table crosses
segment cuts) and fib-2pow16-log-n, each at the plans 1024 (rollup's 64 segments, configs[3]),
4096 (the CLI default) and 65536; the multi-segment cases of tests/test_segments.py (sponge,
Merkle path, RAM, every ALU op); and windows that do not start on a checkpoint.
"""
import json
import os
import sys

import pytest

import zkl_hip

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
G = json.load(open(os.path.join(ROOT, "tests", "golden", "programs.json")))


def _prog(name):
    g = G[name]
    ops = [zkl_hip.op(k, **f) for k, f in g["ops"]]
    ma = [(tg, bytes.fromhex(b)) for tg, b in g["cli"]["main_args"]]
    return ops, bytes.fromhex(g["program_id"]), g["cli"]["secret_u64"], ma


def _check_windows(ops, pid, secret, ma, windows, oracle=None):
    t, pi, w, n = zkl_hip.build_trace(ops, pid, secret_args=secret, main_args=ma)
    P = zkl_hip.Program(ops, pid, secret_args=secret, main_args=ma)
    assert (P.width, P.n_rows) == (w, n)
    arr = (zkl_hip.ZklOp * len(ops))(*ops)
    va = zkl_hip._vm_args(ma) if ma else None
    for a, b in windows:
        st, spi, sw, sin, sout = zkl_hip.slice_segment(t, w, n, ops, pi, a, b)
        qt, qpi, qw, qin, qout = P.segment(a, b)
        assert qw == sw and bytes(qt) == bytes(st), f"[{a},{b}) trace"
        assert bytes(qpi) == bytes(spi), f"[{a},{b}) public inputs"
        assert (qin, qout) == (sin, sout), f"[{a},{b}) state hashes"
        if oracle is not None:
            rc, ot, opi, ow, oin, oout = oracle.build_segment_trace(arr, pid, a, b, secret_args=secret, main_args=va)
            assert rc == 0 and ow == sw and bytes(ot) == bytes(st) and bytes(opi) == bytes(spi), f"[{a},{b}) oracle"
            assert (oin, oout) == (sin, sout)


@pytest.mark.parametrize("name", sorted(G))
@pytest.mark.parametrize("max_rows", [1 << 10, 1 << 12, 1 << 16])
def test_real_program_segments_equal_full_trace_slices(oracle, name, max_rows):
    ops, pid, secret, ma = _prog(name)
    plan = zkl_hip.plan_segments(len(ops), max_rows)
    _check_windows(ops, pid, secret, ma, plan, oracle if max_rows != 1 << 16 else None)


def test_rollup_64_segment_plan_crosses_the_ram_table():
    """At --max-segment-rows 1024 rollup-bench is 64 segments: the RAM-using ones are 212 wide,
    the last ones 204 (no RAM or sponge op), and the sorted RAM table -- three events per level
    in the pad rows, from level 0 on -- runs through the first segments (ram_gp_sorted grows
    across their cuts)."""
    ops, pid, secret, ma = _prog("rollup-bench")
    plan = zkl_hip.plan_segments(len(ops), 1 << 10)
    assert len(plan) == 64 and all(b - a == 1024 for a, b in plan)
    P = zkl_hip.Program(ops, pid, secret_args=secret, main_args=ma)
    widths = [P.segment_width(a, b) for a, b in plan]
    assert widths[0] == 212 and widths[-1] == 204 and set(widths) == {204, 212}
    n_events = sum(k in ("Load", "Store") for k, _ in G["rollup-bench"]["ops"])
    table_segments = -(-n_events // 96)  # 3 events per 32-row level, 32 levels per segment
    fe = lambda f: f.lo | (f.hi << 64)  # noqa: E731
    for i, (a, b) in enumerate(plan[:table_segments + 1]):
        _, pi, w, _, _ = P.segment(a, b)
        grows = fe(pi.ram_gp_sorted_in) != fe(pi.ram_gp_sorted_out)
        assert grows == (i < table_segments), i


@pytest.mark.parametrize("name", sorted(G))
def test_windows_off_checkpoints(oracle, name):
    """Windows that start between the builder's 32-level checkpoints, windows of one level and
    the last level."""
    ops, pid, secret, ma = _prog(name)
    P = zkl_hip.Program(ops, pid, secret_args=secret, main_args=ma)
    n = P.n_rows
    windows = [(32 * 33, 32 * 34), (32 * 70, 32 * 72), (32 * 5, 32 * 9), (32 * 100, 32 * 164), (n - 32, n),
               (0, 32), (32 * 31, 32 * 32)]
    _check_windows(ops, pid, secret, ma, windows, oracle)


@pytest.mark.parametrize("prog", ["multiseg", "ram", "alu"])
def test_segment_programs_of_test_segments(oracle, prog):
    from test_segments import PID, PROGRAMS
    fn, max_rows = PROGRAMS[prog]
    ops = fn()
    plan = zkl_hip.plan_segments(len(ops), max_rows)
    _check_windows(ops, PID, [], [], plan, oracle)


def test_rejections():
    ops, pid, secret, ma = _prog("fib-2pow16-log-n")
    P = zkl_hip.Program(ops, pid)
    n = P.n_rows
    for a, b in [(0, 48), (16, 48), (0, 96), (1024, 1024), (0, 2 * n), (n - 32, n + 32)]:
        with pytest.raises(zkl_hip.ZklError):
            P.segment(a, b)
    with pytest.raises(zkl_hip.ZklError):
        zkl_hip.Program([zkl_hip.op("SAbsorbN", regs=[0] * 10), zkl_hip.op("SAbsorbN", regs=[1]),
                         zkl_hip.op("End")], pid)  # push_absorb: more than 10 pending (vm.rs:925-935)


def test_rollup_1024_sorted_ram_chain_breaks_where_the_table_is_cut():
    """Why the 64-segment plan's valid-mode aggregation is refused (tests/golden/programs.json
    "rejected"): compute_segment_boundary_bytes takes ram_gp_sorted at a segment's
    first and last rows (prove.rs:1224-1227) and the aggregation chains out(i) -> in(i+1)
    (agg/trace.rs:515-521).  The sorted grand product counts a sorted row on the row after it, so
    where the cut falls inside the sorted table (the last row of a level is a sorted row) in(i+1)
    exceeds out(i) by exactly that row's compression; below the table the chain holds."""
    import oracle_lib
    ops, pid, secret, ma = _prog("rollup-bench")
    P = zkl_hip.Program(ops, pid, secret_args=secret, main_args=ma)
    plan = zkl_hip.plan_segments(len(ops), 1 << 10)
    n_events = sum(k in ("Load", "Store") for k, _ in G["rollup-bench"]["ops"])
    fe = lambda f: f.lo | (f.hi << 64)  # noqa: E731
    breaks = []
    for i in range(len(plan) - 1):
        _, a, _, _, _ = P.segment(*plan[i])
        _, b, _, _, _ = P.segment(*plan[i + 1])
        diff = oracle_lib.fe_sub(fe(b.ram_gp_sorted_in), fe(a.ram_gp_sorted_out))
        assert (fe(b.ram_gp_unsorted_in), fe(b.rom_s_in[0])) == (fe(a.ram_gp_unsorted_out), fe(a.rom_s_out[0]))
        if diff:
            breaks.append(i)
    # cuts after segment i lie inside the table while event 3 * 32 * (i + 1) - 1 exists
    assert breaks == [i for i in range(len(plan) - 1) if 96 * (i + 1) <= n_events]
    assert breaks  # the published 16 x 4096 plan keeps the table inside segment 0; this one does not
