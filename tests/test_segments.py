"""§8(f)3 — a compiled program proved as step segments: the planner's cut
(zkl_plan_segments, segment_planner.rs:93-276) and prove_segment's per-segment trace and public
inputs (zkl_slice_segment, prove.rs:1057-1287), against the Python restatement
oracle/segments_ref.py over the C oracle's full trace, then the zl1 steps of all segments
aggregated (zkl_agg_prove vs oracle/agg_ref.py), as `zk-lisp prove` does for a program longer
than one segment.  The program of agg_multiseg.rs:70-121 (arithmetic, a sponge, a two-step
Merkle path, a run of Consts, max_rows 2^10) is the reference's own multi-segment case.
"""
import ctypes as C
import os
import sys

import pytest

import zkl_hip
from zkl_hip import op

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import segments_ref  # noqa: E402

PID = bytes(range(3, 35))


def multiseg_ops():
    ops = [op("Const", dst=0, imm=7), op("Const", dst=1, imm=9), op("Add", dst=2, a=0, b=1),
           op("SAbsorbN", regs=[0, 1, 2]), op("SSqueeze", dst=3),
           op("Const", dst=4, imm=1), op("Const", dst=5, imm=0), op("Const", dst=6, imm=2),
           op("MerkleStepFirst", leaf_reg=4, dir_reg=5, sib_reg=6),
           op("Const", dst=5, imm=1), op("Const", dst=6, imm=3), op("MerkleStepLast", dir_reg=5, sib_reg=6)]
    ops += [op("Const", dst=0, imm=1) for _ in range((1 << 10) // 32 + 1)]
    ops.append(op("End"))
    return ops


def ram_ops():
    ops = []
    for k in range(6):
        ops += [op("Const", dst=7, imm=k % 3), op("Const", dst=0, imm=10 + k), op("Store", addr=7, src=0),
                op("Load", dst=1, addr=7), op("Add", dst=2, a=1, b=2)]
    ops += [op("Mul", dst=3, a=2, b=2) for _ in range(20)]
    ops += [op("Load", dst=4, addr=7), op("End")]
    return ops


def alu_ops():
    from test_trace_builder import ALU_OPS
    return ALU_OPS


PROGRAMS = {"multiseg": (multiseg_ops, 1 << 10), "ram": (ram_ops, 1 << 9), "alu": (alu_ops, 64)}


def _segments(oracle, ops, max_rows):
    """(product segments, oracle segments): each a list of (trace, pi, width, state_in, state_out)."""
    t, pi, w, n = zkl_hip.build_trace(ops, PID)
    arr = (zkl_hip.ZklOp * len(ops))(*ops)
    rc, ot, opi, ow, on = oracle.build_trace(arr, PID)
    assert rc == 0 and bytes(ot) == bytes(t)
    plan = zkl_hip.plan_segments(len(ops), max_rows)
    assert plan == segments_ref.plan_segments(len(ops), max_rows)
    kinds = [o.kind for o in ops]
    got = [zkl_hip.slice_segment(t, w, n, ops, pi, a, b) for a, b in plan]
    want = [segments_ref.slice_segment(oracle, ot, on, kinds, opi, a, b) for a, b in plan]
    return plan, got, want


@pytest.mark.parametrize("n_ops,max_rows", [(1, 4096), (46, 1 << 10), (46, 1 << 12), (100, 256), (513, 1 << 12),
                                            (3000, 1 << 12), (8, 32)])
def test_plan_segments(n_ops, max_rows):
    assert zkl_hip.plan_segments(n_ops, max_rows) == segments_ref.plan_segments(n_ops, max_rows)


@pytest.mark.parametrize("prog", sorted(PROGRAMS))
def test_slices_match_oracle_and_satisfy_air(oracle, prog):
    fn, max_rows = PROGRAMS[prog]
    plan, got, want = _segments(oracle, fn(), max_rows)
    assert len(plan) > 1
    for (a, b), g, wnt in zip(plan, got, want):
        t, pi, w, sin, sout = g
        ot, opi, ow, osin, osout = wnt
        assert w == ow and bytes(t) == bytes(ot), f"segment [{a},{b}) trace"
        assert bytes(pi) == bytes(opi), f"segment [{a},{b}) public inputs"
        assert (sin, sout) == (osin, osout)
        assert oracle.check_trace(t, pi, w, b - a) == (0, 0, 0), f"segment [{a},{b}) violates the AIR"
    # the chains the aggregation checks: ROM lane 0 carries across every cut; the VM state hash
    # across cuts into program levels (levels past the last op hold zero registers, as
    # build_empty_trace leaves them, so a cut into the padding breaks the VM chain there, as in
    # the reference)
    n_ops = len(fn())
    for (a, b), g0, g1 in zip(plan[1:], got, got[1:]):
        assert (g0[1].rom_s_out[0].lo, g0[1].rom_s_out[0].hi) == (g1[1].rom_s_in[0].lo, g1[1].rom_s_in[0].hi)
        if a // 32 < n_ops:
            assert g0[4] == g1[3]


def test_multiseg_segment_layouts(oracle):
    """Segment 0 carries the sponge and the Merkle path (its own mask, width 211); segment 1
    only Consts and padding (FM_VM, width 204); pc_init = the first level of each."""
    plan, got, _ = _segments(oracle, multiseg_ops(), 1 << 10)
    assert plan == [(0, 1024), (1024, 2048)]
    (t0, p0, w0, _, _), (t1, p1, w1, _, _) = got
    base = zkl_hip.FM_VM | zkl_hip.FM_SPONGE | zkl_hip.FM_POSEIDON | zkl_hip.FM_MERKLE
    assert p0.feature_mask == p1.feature_mask == base
    assert p0.segment_feature_mask == base and w0 == 211
    assert p1.segment_feature_mask == zkl_hip.FM_VM and w1 == 204
    assert (p0.pc_init.lo, p1.pc_init.lo) == (0, 32)


def _steps(oracle, got, queries=8, grind=4, prover=None, verify=False):
    steps = []
    for i, (t, pi, w, sin, sout) in enumerate(got):
        n = len(t) // w
        opts = oracle.default_options(w, n, queries=queries, grind=grind)
        opi = oracle.AirPublicInputs()
        C.memmove(C.byref(opi), C.byref(pi), C.sizeof(opi))
        proof = prover(t, w, n, pi, opts) if prover else oracle.prove(t, w, n, opi, opts)
        if verify:  # the product verifier (verify_proof, prove.rs:802-941) on the segment's own inputs
            zkl_hip.verify_segment(proof, pi, zkl_hip.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_]))
        info = zkl_hip.step_info_for(pi, i, len(got), sin, sout)
        steps.append(zkl_hip.step_proof_encode(pi, info, proof))
    return steps


def test_multiseg_program_aggregates(oracle):
    """Both segments proved (oracle prover) and verified by the product verifier, wrapped as zl1
    steps with their real state hashes, aggregated: the library's ZKLRC1 artifact equals
    agg_ref's and verifies.  Segment 1's step carries the program's feature mask while its trace
    has the VM-only layout; the child replay rebuilds the AIR from the program's mask as
    agg/fs.rs:38-80 does (the composition width is what it needs)."""
    import agg_ref
    _, got, _ = _segments(oracle, multiseg_ops(), 1 << 10)
    steps = _steps(oracle, got, verify=True)
    art, dg = zkl_hip.agg_prove(steps, queries=64, blowup=16, grind=8)
    want_art, want_dg, _ = agg_ref.agg_prove(oracle, steps, queries=64, blowup=16, grind=8)
    assert (art, dg) == (want_art, want_dg)
    zkl_hip.agg_verify(art)
    d = zkl_hip.parse_agg_artifact(art)
    assert d["children_count"] == 2 and d["vm_state_initial"] == got[0][3] and d["vm_state_final"] == got[1][4]


def test_slice_rejections():
    ops = multiseg_ops()
    t, pi, w, n = zkl_hip.build_trace(ops, PID)
    for a, b in [(0, 48), (16, 48), (0, 96), (1024, 1024), (0, 4096)]:
        with pytest.raises(zkl_hip.ZklError):
            zkl_hip.slice_segment(t, w, n, ops, pi, a, b)


@pytest.mark.gpu
def test_multiseg_segments_prove_on_gpu(oracle, gpu_ctx):
    """The segments proved on the GPU equal the oracle's proofs; their aggregation equals the
    artifact built from the oracle's."""
    _, got, _ = _segments(oracle, multiseg_ops(), 1 << 10)

    def gpu(t, w, n, pi, opts):
        zo = zkl_hip.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_])
        return gpu_ctx.prove_segment(t, w, n, pi, zo)

    steps_gpu = _steps(oracle, got, queries=32, grind=8, prover=gpu)
    steps_orc = _steps(oracle, got, queries=32, grind=8)
    assert steps_gpu == steps_orc
    art, _ = zkl_hip.agg_prove(steps_gpu, queries=64, blowup=16, grind=8)
    zkl_hip.agg_verify(art)
