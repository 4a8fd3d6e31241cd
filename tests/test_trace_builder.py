"""§8(f)3 — the op-list trace builder (zkl_build_trace, host) against its oracle twin
(orc_build_trace) and the reference's own trace-builder unit tests.

Each program is a builder::Op list (zk-lisp-compiler/src/builder.rs:25-158).  Checks per
program: the product's trace and AIR public inputs equal the oracle's bit for bit, and the
oracle's ZkLispAir restatement accepts the trace (every transition constraint and assertion,
tests/test_oracle_air.py), so the witness columns each op writes (vm.rs:199-842) are the ones
the AIR constrains.  The programs of vm.rs:953-1110 (alu_const_add, alu_eq_and_select,
sponge_absorb_squeeze_simple, program_commit_bound_at_level0) keep their reference assertions.
"""
import pytest

import zkl_hip
from zkl_hip import op

PID = bytes(range(1, 33))
P = 2**128 - 45 * 2**40 + 1
STEPS = 32
MAP, FINAL = 0, 28


def _build_both(oracle, ops, **kw):
    got = zkl_hip.build_trace(ops, PID, **kw)
    arr = (zkl_hip.ZklOp * len(ops))(*ops)
    margs = kw.get("main_args", ())
    ma = zkl_hip._vm_args(list(margs)) if margs else None
    rc, t, pi, w, n = oracle.build_trace(arr, PID, secret_args=kw.get("secret_args", ()), main_args=ma,
                                         rom0=kw.get("rom0", 0))
    assert rc == 0
    return got, (t, pi, w, n)


def _same(got, want):
    t, pi, w, n = got
    ot, opi, ow, on = want
    assert (w, n) == (ow, on)
    assert bytes(t) == bytes(ot), "trace differs from the oracle"
    assert bytes(pi) == bytes(opi), "public inputs differ from the oracle"


R_START = 12 + 2 + 27 + 1          # lanes, g_map, g_final, 27 round gates, mask
OP_START = R_START + 8


def _reg(t, n, i, row):
    e = t[(R_START + i) * n + row]
    return e.lo | (e.hi << 64)


def _opbit(t, n, k, row):
    e = t[(OP_START + k) * n + row]
    return e.lo | (e.hi << 64)


def _check(oracle, ops, **kw):
    got, want = _build_both(oracle, ops, **kw)
    _same(got, want)
    t, pi, w, n = got
    assert oracle.check_trace(t, pi, w, n) == (0, 0, 0)
    return t, pi, w, n


def test_alu_const_add(oracle):
    """vm.rs:953-996 alu_const_add."""
    t, pi, w, n = _check(oracle, [op("Const", dst=0, imm=7), op("Const", dst=1, imm=9),
                                  op("Add", dst=2, a=0, b=1), op("End")])
    assert n == 4 * STEPS and w == 204
    assert _opbit(t, n, 0, MAP) == 1 and _reg(t, n, 0, FINAL + 1) == 7
    assert _opbit(t, n, 0, STEPS + MAP) == 1 and _reg(t, n, 1, STEPS + FINAL + 1) == 9
    assert _opbit(t, n, 2, 2 * STEPS + MAP) == 1 and _reg(t, n, 2, 2 * STEPS + FINAL + 1) == 16


def test_alu_eq_and_select(oracle):
    """vm.rs:998-1040 alu_eq_and_select: 5 ops -> 8 levels; r2 = (r0 == r1), r3 = select."""
    t, pi, w, n = _check(oracle, [op("Const", dst=0, imm=5), op("Const", dst=1, imm=5),
                                  op("Eq", dst=2, a=0, b=1), op("Select", dst=3, c=2, a=0, b=1), op("End")])
    assert n == 8 * STEPS
    assert _opbit(t, n, 6, 2 * STEPS + MAP) == 1 and _reg(t, n, 2, 2 * STEPS + FINAL + 1) == 1
    assert _opbit(t, n, 7, 3 * STEPS + MAP) == 1 and _reg(t, n, 3, 3 * STEPS + FINAL + 1) == 5
    # levels past the program: schedule gates and pc only, registers zero
    assert all(_reg(t, n, i, 6 * STEPS + 3) == 0 for i in range(8))
    assert pi.vm_usage_mask & 1 and pi.vm_usage_mask & (1 << 6)


def test_sponge_absorb_squeeze_simple(oracle):
    """vm.rs:1042-1072: SSqueeze writes poseidon_hash_two_lanes(program, r0, r1) to r3."""
    import pyref
    t, pi, w, n = _check(oracle, [op("Const", dst=0, imm=1), op("Const", dst=1, imm=2),
                                  op("SAbsorbN", regs=[0, 1]), op("SSqueeze", dst=3), op("End")])
    s = pyref.suite(PID)
    st = [1, 2] + [0] * 8 + list(s[0])
    want = pyref.permute(st, s)[0]
    assert _opbit(t, n, 8, 3 * STEPS + FINAL) == 1
    assert _reg(t, n, 3, 3 * STEPS + FINAL + 1) == want
    assert pi.feature_mask == zkl_hip.FM_VM | zkl_hip.FM_SPONGE | zkl_hip.FM_POSEIDON


def test_program_commit_bound_at_level0(oracle):
    """vm.rs:1074-1090: pi_prog at row 0 = be_from_le8(commitment) — the AIR asserts it (the
    oracle check passes) and a different commitment breaks that assertion."""
    t, pi, w, n = _check(oracle, [op("Const", dst=0, imm=1), op("End")])
    assert n == 2 * STEPS
    assert bytes(pi.program_commitment) == PID
    t2, pi2, _, _ = zkl_hip.build_trace([op("Const", dst=0, imm=1), op("End")], PID, program_commitment=bytes(32 * [7]))
    assert oracle.check_trace(t2, pi2, w, n)[0] != 0


def test_sponge_overflow_errors(oracle):
    """sponge.rs:195-222: 12 pending absorbs exceed the rate -> build error."""
    ops = [op("Const", dst=r, imm=r + 1) for r in range(8)]
    ops += [op("SAbsorbN", regs=[2 * i % 8, (2 * i + 1) % 8]) for i in range(6)]
    ops += [op("SSqueeze", dst=0), op("End")]
    with pytest.raises(zkl_hip.ZklError):
        zkl_hip.build_trace(ops, PID)
    arr = (zkl_hip.ZklOp * len(ops))(*ops)
    assert oracle.build_trace(arr, PID)[0] != 0


def test_sponge_multiple_absorbs_then_squeeze(oracle):
    """sponge.rs:115-190: absorbs across three levels, one squeeze of 10 lanes."""
    ops = [op("Const", dst=r, imm=r + 1) for r in range(8)]
    ops += [op("Const", dst=0, imm=9), op("Const", dst=1, imm=10), op("SAbsorbN", regs=[0, 1]),
            op("SAbsorbN", regs=[2, 3, 4]), op("SAbsorbN", regs=[5, 6, 7, 0, 1]), op("SSqueeze", dst=0), op("End")]
    _check(oracle, ops)


def test_sponge_all_lanes(oracle):
    """sponge.rs:370-406: 8 rounds of 10-lane absorbs with rotating registers."""
    ops = [op("Const", dst=r, imm=r + 1) for r in range(8)]
    for k in range(8):
        ops += [op("SAbsorbN", regs=[(k + i) % 8 for i in range(10)]), op("SSqueeze", dst=k % 8)]
    ops.append(op("End"))
    _check(oracle, ops)


def test_multiseg_program(oracle):
    """agg_multiseg.rs:70-121: arithmetic, a sponge, a two-step Merkle path and a run of
    Consts; merkle_root = the accumulator after MerkleStepLast."""
    ops = [op("Const", dst=0, imm=7), op("Const", dst=1, imm=9), op("Add", dst=2, a=0, b=1),
           op("SAbsorbN", regs=[0, 1, 2]), op("SSqueeze", dst=3),
           op("Const", dst=4, imm=1), op("Const", dst=5, imm=0), op("Const", dst=6, imm=2),
           op("MerkleStepFirst", leaf_reg=4, dir_reg=5, sib_reg=6),
           op("Const", dst=5, imm=1), op("Const", dst=6, imm=3), op("MerkleStepLast", dir_reg=5, sib_reg=6)]
    ops += [op("Const", dst=0, imm=1)] * ((1 << 10) // 32 + 1)
    ops.append(op("End"))
    t, pi, w, n = _check(oracle, ops)
    assert n == 64 * STEPS
    assert pi.feature_mask & zkl_hip.FM_MERKLE and any(pi.merkle_root)


ALU_OPS = [
    op("Const", dst=0, imm=0xFFFF_FFFF_FFFF_FFF1), op("Const", dst=1, imm=12345), op("Neg", dst=2, a=1),
    op("Sub", dst=3, a=1, b=0), op("Mul", dst=4, a=0, b=0), op("Mov", dst=5, src=4),
    op("DivMod", dst_q=6, dst_r=7, a=0, b=1),
    op("MulWide", dst_hi=2, dst_lo=3, a=0, b=1),
    op("DivMod128", a_hi=1, a_lo=0, b=6, dst_q=4, dst_r=5),
    op("Const", dst=6, imm=1), op("AssertBit", dst=7, r=6), op("Assert", dst=5, c=6),
    op("Const", dst=1, imm=200), op("AssertRange", dst=2, r=1, bits=8),
    op("Const", dst=1, imm=0xDEAD_BEEF), op("AssertRange", dst=2, r=1, bits=32),
    op("Const", dst=3, imm=0x1234_5678_9ABC_DEF0), op("AssertRangeLo", dst=4, r=3), op("AssertRangeHi", dst=4, r=3),
    op("Eq", dst=5, a=0, b=1), op("Select", dst=6, c=5, a=0, b=1), op("Neg", dst=0, a=0),
    op("Eq", dst=2, a=0, b=0), op("End"),
]


def test_full_alu_program(oracle):
    """Every ALU op of vm.rs:199-564 on values near 2^64: product == oracle and the AIR's ALU /
    range / division constraints hold."""
    t, pi, w, n = _check(oracle, ALU_OPS)
    # usage mask bits: select/assert, assert_bit, range, divmod, mulwide, div128, eq
    assert pi.vm_usage_mask & 0x7F == 0x7F


@pytest.mark.parametrize("div", ["DivMod", "DivMod128"])
def test_zero_divisor(oracle, div):
    """A zero divisor: the builder writes q = 0, r = a mod 2^64 and eq_inv = 0 (vm.rs:455-470,
    520-545) — both builders agree — and the AIR's b * inv_b = 1 constraint (alu.rs:292, 313)
    rejects the trace, as the reference's prover would."""
    d = (op("DivMod", dst_q=2, dst_r=3, a=1, b=7) if div == "DivMod"
         else op("DivMod128", a_hi=0, a_lo=1, b=7, dst_q=2, dst_r=3))
    ops = [op("Const", dst=1, imm=77), op("Const", dst=7, imm=0), d, op("End")]
    got, want = _build_both(oracle, ops)
    _same(got, want)
    t, pi, w, n = got
    assert _reg(t, n, 2, 2 * STEPS + FINAL + 1) == 0 and _reg(t, n, 3, 2 * STEPS + FINAL + 1) == 77
    rc, row, _ = oracle.check_trace(t, pi, w, n)
    assert rc == 1 and row == 2 * STEPS + FINAL


def test_ram_program(oracle):
    """Load / Store (vm.rs:803-842) with repeated addresses and a read of an unwritten address."""
    ops = [op("Const", dst=7, imm=3), op("Const", dst=0, imm=11), op("Store", addr=7, src=0),
           op("Load", dst=1, addr=7), op("Const", dst=6, imm=5), op("Load", dst=2, addr=6),
           op("Add", dst=3, a=1, b=1), op("Store", addr=7, src=3), op("Store", addr=6, src=1),
           op("Load", dst=4, addr=7), op("Load", dst=5, addr=6), op("End")]
    t, pi, w, n = _check(oracle, ops)
    assert pi.feature_mask & zkl_hip.FM_RAM and pi.vm_usage_mask & (1 << 8)
    assert _reg(t, n, 2, 5 * STEPS + FINAL + 1) == 0        # unwritten address reads 0
    assert _reg(t, n, 4, 9 * STEPS + FINAL + 1) == 22


def test_args_seed_registers(oracle):
    """vm.rs:64-104: secret args fill r0.., main-arg slots the tail registers (a Bytes32 takes
    two slots) and become the AIR's main_slots."""
    b32 = bytes(range(100, 132))
    ops = [op("Add", dst=0, a=0, b=1), op("Mul", dst=1, a=5, b=6), op("End")]
    t, pi, w, n = _check(oracle, ops, secret_args=(3, 4, 99, 98, 97, 96), main_args=[5, (2, b32)])
    assert pi.n_main_slots == 3
    assert [_reg(t, n, i, 0) for i in range(5)] == [3, 4, 99, 98, 97]    # the sixth secret arg is dropped
    assert _reg(t, n, 5, 0) == 5
    assert _reg(t, n, 6, 0) == int.from_bytes(b32[:16], "little") % P


def test_rom_chain_input(oracle):
    """ROM lane 0 entering the first level (the aggregation's accumulator chain)."""
    t, pi, w, n = _check(oracle, [op("Const", dst=0, imm=1), op("End")], rom0=123456789)
    assert (pi.rom_s_in[0].lo | (pi.rom_s_in[0].hi << 64)) == 123456789


@pytest.mark.parametrize("prog", ["alu", "sponge", "ram", "multiseg"])
def test_rom_acc_from_program(oracle, prog):
    """romacc.rs:22-80, from the ops alone, equals the accumulator the oracle's trace ends on
    (rom.rs:29-108 over the built map rows) — the identity the verifier relies on."""
    ops = {
        "alu": ALU_OPS,
        "sponge": [op("Const", dst=0, imm=1), op("SAbsorbN", regs=[0, 0]), op("SSqueeze", dst=3), op("End")],
        "ram": [op("Const", dst=7, imm=3), op("Store", addr=7, src=0), op("Load", dst=1, addr=7), op("End")],
        "multiseg": [op("Const", dst=4, imm=1), op("Const", dst=5, imm=0), op("Const", dst=6, imm=2),
                     op("MerkleStepFirst", leaf_reg=4, dir_reg=5, sib_reg=6), op("MerkleStep", dir_reg=5, sib_reg=6),
                     op("MerkleStepLast", dir_reg=5, sib_reg=6), op("End")],
    }[prog]
    arr = (zkl_hip.ZklOp * len(ops))(*ops)
    rc, t, pi, w, n = oracle.build_trace(arr, PID)
    assert rc == 0
    assert zkl_hip.rom_acc_from_program(ops, PID) == [e.lo | (e.hi << 64) for e in pi.rom_acc]


def _hello_zk():
    """examples/hello-zk.zlisp lowered by hand (not the compiler's exact output): main(pub_x,
    pub_y) with s = secret-arg 0 asserts pub_y == pub_x + s and returns 1.  main args take the
    tail registers r6, r7; the secret arg r0."""
    return [op("Add", dst=1, a=6, b=0), op("Eq", dst=2, a=7, b=1), op("Assert", dst=3, c=2),
            op("Const", dst=0, imm=1), op("End")]


def test_hello_zk_program(oracle):
    t, pi, w, n = _check(oracle, _hello_zk(), secret_args=(5,), main_args=[37, 42])
    assert _reg(t, n, 0, 3 * STEPS + FINAL + 1) == 1
    assert pi.n_main_slots == 2 and pi.vm_usage_mask & 1
    # a wrong secret: the Assert level's c == 1 constraint fails
    t2, pi2, _, _ = zkl_hip.build_trace(_hello_zk(), PID, secret_args=(6,), main_args=[37, 42])
    rc, row, _ = oracle.check_trace(t2, pi2, w, n)
    assert rc == 1 and row == 2 * STEPS + FINAL


def test_invalid_programs():
    with pytest.raises(ValueError):
        op("Add", dst=0, a=1)
    with pytest.raises(zkl_hip.ZklError):
        zkl_hip.build_trace([op("Mov", dst=9, src=0), op("End")], PID)
    with pytest.raises(zkl_hip.ZklError):
        zkl_hip.build_trace([op("End")], PID, main_args=[(2, bytes(32))] * 5)
    # 32-byte ids are checked before the C side reads them
    with pytest.raises(ValueError):
        zkl_hip.build_trace([op("End")], PID[:31])
    with pytest.raises(ValueError):
        zkl_hip.Program([op("End")], PID, program_commitment=b"short")
    with pytest.raises(ValueError):
        zkl_hip.rom_acc_from_program([op("End")], b"")
    with pytest.raises(ValueError):
        zkl_hip.children_root(bytes(32), [bytes(32)], [bytes(31)])


@pytest.mark.gpu
@pytest.mark.parametrize("prog", ["alu", "hello"])
def test_op_list_proof_parity(oracle, gpu_ctx, prog):
    """Op-list programs proved on the GPU: bytes equal the oracle's proof and the host verifier
    accepts them."""
    if prog == "alu":
        t, pi, w, n = zkl_hip.build_trace(ALU_OPS, PID)
    else:
        t, pi, w, n = zkl_hip.build_trace(_hello_zk(), PID, secret_args=(5,), main_args=[37, 42])
    opts = zkl_hip.proof_options(w, n, queries=32, grind=8)
    got = gpu_ctx.prove_segment(t, w, n, pi, opts)
    want = oracle.prove(t, w, n, pi, oracle.ProofOptions(*[getattr(opts, f) for f, _ in opts._fields_]))
    assert got == want
    zkl_hip.verify_segment(got, pi, opts)
