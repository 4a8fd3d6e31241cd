"""ORACLE (test infrastructure, not product): a Python restatement of the zk-lisp compiler's
front end for the forms the reference's examples use (hello-zk, rollup-bench,
fib-2pow16-log-n), so the op list the prover is fed for a real `.zlisp` program is the one
`compile_entry` emits, derived by code rather than by hand.

Follows zk-lisp-compiler/src:
  * lex / parse                lib.rs:259-491
  * compile_str / compile_entry lib.rs:113-256 (main's arity, (main ARGS...) lowered after the
                               top-level forms, result moved to r0, End; program_id = BLAKE3(src))
  * LowerCtx                   lower/ctx.rs:38-145 (free list 0..7, alloc pops the end = the
                               highest free register, free pushes back; emit_mov elides dst == src)
  * lower_top / lower_expr     lower/mod.rs:126-246
  * def (function and `(def NAME INT)` constant)  lower/mod.rs:248-308
  * let / begin / block / call lower/mod.rs:310-391, 553-631, 738-752, 835-852
  * lower_bin (Sethi-Ullman order, Imm folding, dst reuse)  lower/mod.rs:393-551, 889-1026
  * secret-arg                 lower/mod.rs:754-782
  * typed-fn / typed-let       lower/mod.rs:784-833, 1049-1103 (schema only: no ops)
  * loop / recur               lower/iter.rs:14-244 (flat unroll to :max; recur arguments are
                               evaluated in order and each rebinds its variable before the next
                               is lowered; the last iteration runs the prefix only)
  * if / when / = / neg / select  lower/operators.rs:15-145, 238-282
  * assert / assert-bit / assert-range  lower/assert.rs:15-138
  * safe-add / safe-sub / safe-mul, assert_range_bits_for_reg  lower/alu.rs:15-142, 617-642
  * load / store               lower/store.rs:15-67
  * hash2                      lower/hash.rs:15-49 (SAbsorbN of two registers + SSqueeze)
  * ProgramBuilder::push       builder.rs:188-310 (a Mov onto itself is dropped; one op per level)
Forms the reference has but no example uses (merkle-verify, load-ca/store-ca, push/pop, divmod,
mulwide, muldiv, in-set, bit?, hex-to-bytes32, deftype) raise NotImplementedError: this is not a
compiler, only the subset the examples need.
"""

NR = 8

UNRESTATED = {"merkle-verify", "load-ca", "store-ca", "push", "pop", "push*", "pop*", "divmod-q",
              "divmod-r", "mulwide-hi", "mulwide-lo", "muldiv", "in-set", "bit?", "hex-to-bytes32",
              "deftype"}


class Sym(str):
    pass


class LowerError(ValueError):
    pass


def lex(src):
    """lib.rs:259-438 (parens, quote, ';' comments, decimal u64, symbols, strings)."""
    out, i = [], 0
    start = set("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ_+-*=<>:")
    cont = start | set("0123456789/:?")
    while i < len(src):
        ch = src[i]
        if ch in "()'":
            out.append(ch)
            i += 1
        elif ch == ";":
            while i < len(src) and src[i] != "\n":
                i += 1
        elif ch in " \n\r\t":
            i += 1
        elif ch.isdigit():
            j = i
            while j < len(src) and src[j].isdigit():
                j += 1
            v = int(src[i:j])
            if v >= 1 << 64:
                raise LowerError(f"lex: invalid char {ch!r} at {j}")
            out.append(v)
            i = j
        elif ch in start:
            j = i
            while j < len(src) and src[j] in cont:
                j += 1
            out.append(Sym(src[i:j]))
            i = j
        elif ch == '"':
            raise NotImplementedError("string literals")
        else:
            raise LowerError(f"lex: invalid char {ch!r} at {i}")
    return out


def parse(toks):
    """lib.rs:441-491: forms*; 'X -> (quote X)."""
    pos = 0

    def one():
        nonlocal pos
        if pos >= len(toks):
            raise LowerError("parse: unexpected EOF")
        t = toks[pos]
        pos += 1
        if t == "(":
            items = []
            while True:
                if pos >= len(toks):
                    raise LowerError("parse: unexpected EOF")
                if toks[pos] == ")":
                    break
                items.append(one())
            pos += 1
            return items
        if t == "'":
            return [Sym("quote"), one()]
        if t == ")":
            raise LowerError("parse: unmatched ')'")
        return t

    forms = []
    while pos < len(toks):
        forms.append(one())
    return forms


class Ctx:
    """LowerCtx (ctx.rs:23-145) + the ProgramBuilder state lowering touches (ops, blocks)."""

    def __init__(self):
        self.free = list(range(NR))
        self.vars = {}
        self.funs = {}
        self.const_ints = {}
        self.schemas = {}
        self.call_stack = []
        self.ops = []
        self.blocks = []

    def alloc(self):
        if not self.free:
            raise LowerError("lower: regs exhausted (need 1, have 0)")
        return self.free.pop()

    def free_reg(self, r):
        self.free.append(r)

    def push(self, kind, **f):
        if kind == "Mov" and f["dst"] == f["src"]:
            return
        self.ops.append((kind, f))

    def emit_mov(self, dst, src):
        if dst != src:
            self.push("Mov", dst=dst, src=src)

    def level(self):
        return len(self.ops)

    def push_block(self, start, end):
        if end > start:
            self.blocks.append((start, end - start))


# RVal: ("own", r) | ("bor", r) | ("imm", v)
def into_owned(cx, v):
    if v[0] == "own":
        return v
    dst = cx.alloc()
    if v[0] == "bor":
        cx.emit_mov(dst, v[1])
    else:
        cx.push("Const", dst=dst, imm=v[1])
    return ("own", dst)


def materialize_imm(cx, v):
    """store.rs:43-51 / hash.rs:23-34: only immediates get a register; borrowed stay borrowed."""
    return into_owned(cx, v) if v[0] == "imm" else v


def free_if_owned(cx, v):
    if v[0] == "own":
        cx.free_reg(v[1])


def binding_val(b):
    return ("imm", b[1]) if b[0] == "imm" else ("bor", b[1])


def bind_of(v):
    return ("imm", v[1]) if v[0] == "imm" else ("reg", v[1])


def implicit_begin(forms):
    return forms[0] if len(forms) == 1 else [Sym("begin")] + list(forms)


def is_pure_arith(a):
    if isinstance(a, (int, Sym)):
        return True
    if isinstance(a, list) and a and isinstance(a[0], Sym):
        if a[0] in ("+", "-", "*", "neg", "=", "select", "if", "let"):
            return all(is_pure_arith(x) for x in a[1:])
    return False


def su_number(a):
    if not isinstance(a, list) or not a:
        return 1
    if not isinstance(a[0], Sym) or len(a) < 3:
        return 1
    sl, sr = su_number(a[1]), su_number(a[2])
    if a[0] in ("+", "-", "*"):
        return sl + 1 if sl == sr else max(sl, sr)
    return 1


def ast_size(a):
    return 1 + sum(ast_size(x) for x in a) if isinstance(a, list) else 1


def contains_symbol(a, name):
    if isinstance(a, Sym):
        return a == name
    if isinstance(a, list):
        return any(contains_symbol(x, name) for x in a)
    return False


def balance_chain(op, items):
    flat = []

    def flatten(nodes):
        for n in nodes:
            if isinstance(n, list) and n and n[0] == op and len(n) >= 3:
                flatten(n[1:])
            else:
                flat.append(n)

    def build(v):
        if len(v) == 1:
            return v[0]
        mid = len(v) // 2
        return [Sym(op), build(v[:mid]), build(v[mid:])]

    flatten(items)
    return build(flat)


def lower_bin(cx, rest, op):
    if len(rest) != 2:
        raise LowerError("lower: invalid form 'bin'")
    both_pure = is_pure_arith(rest[0]) and is_pure_arith(rest[1])
    su_l, su_r = su_number(rest[0]), su_number(rest[1])
    if not both_pure:
        left_first = True
    elif su_l != su_r:
        left_first = su_l > su_r
    else:
        left_first = ast_size(rest[0]) >= ast_size(rest[1])
    if left_first:
        av, bv = lower_expr(cx, rest[0]), lower_expr(cx, rest[1])
    else:
        av, bv = lower_expr(cx, rest[1]), lower_expr(cx, rest[0])
    ai, bi = (av, bv) if left_first else (bv, av)
    if ai[0] == "imm" and bi[0] == "imm":  # constant folding when the result fits u64
        x, y = ai[1], bi[1]
        r = {"Add": x + y, "Sub": x - y if x >= y else None, "Mul": x * y}[op]
        if r is not None and r < 1 << 64:
            return ("imm", r)
    av, bv = into_owned(cx, av), into_owned(cx, bv)
    a_val, b_val = (av, bv) if left_first else (bv, av)
    if op in ("Add", "Mul"):
        if a_val[0] == "own":
            dst, reused = a_val[1], True
        elif b_val[0] == "own":
            dst, reused = b_val[1], True
        else:
            dst, reused = cx.alloc(), False
    else:
        dst, reused = (a_val[1], True) if a_val[0] == "own" else (cx.alloc(), False)
    a_r, b_r = a_val[1], b_val[1]
    cx.push(op, dst=dst, a=a_r, b=b_r)
    if reused:
        free_if_owned(cx, b_val if dst == a_r else a_val)
    else:
        free_if_owned(cx, a_val)
        free_if_owned(cx, b_val)
    return ("own", dst)


def _rebind_and_lower(cx, names_vals, body):
    """The binding / cleanup discipline shared by let (mod.rs:321-390) and calls (:583-625):
    each value mapped as Imm or Reg; afterwards names are restored to their prior binding, and an
    owned register without a prior binding is freed unless it carries the result."""
    res = lower_expr(cx, body)
    res_reg = res[1] if res[0] != "imm" else None
    for name, prior, v in reversed(names_vals):
        cx.vars.pop(name, None)
        if prior is not None:
            cx.vars[name] = prior
        elif v[0] == "own" and res_reg != v[1]:
            cx.free_reg(v[1])
    return res


def lower_let(cx, rest):
    if not rest or not isinstance(rest[0], list):
        raise LowerError("lower: invalid form 'let: binds'")
    saved = []
    for kv in rest[0]:
        if not isinstance(kv, list) or len(kv) != 2 or not isinstance(kv[0], Sym):
            raise LowerError("lower: invalid form 'let: pair'")
        name = kv[0]
        v = lower_expr(cx, kv[1])
        saved.append((name, cx.vars.get(name), v))
        cx.vars[name] = bind_of(v)
    if len(rest) < 2:
        raise LowerError("lower: invalid form 'let: body'")
    return _rebind_and_lower(cx, saved, implicit_begin(rest[1:]))


def lower_call(cx, name, args):
    if name not in cx.funs:
        raise LowerError(f"lower: unknown symbol '{name}'")
    params, body = cx.funs[name]
    if name in cx.call_stack:
        raise LowerError(f"lower: recursion detected in call '{name}'")
    cx.call_stack.append(name)
    if len(params) != len(args):
        raise LowerError(f"lower: invalid form 'call: {name} expects {len(params)} args'")
    argv = [lower_expr(cx, a) for a in args]
    saved = []
    for p, v in zip(params, argv):
        saved.append((p, cx.vars.get(p), v))
        cx.vars[p] = bind_of(v)
    res = _rebind_and_lower(cx, saved, body)
    cx.call_stack.pop()
    return res


def lower_begin(cx, rest):
    if not rest:
        raise LowerError("lower: invalid form 'begin'")
    for it in rest[:-1]:
        free_if_owned(cx, lower_expr(cx, it))
    return lower_expr(cx, rest[-1])


def lower_block(cx, rest):
    """mod.rs:835-852: begin + a block record of the levels it covered (planner metadata)."""
    if not rest:
        raise LowerError("lower: invalid form 'block'")
    l0 = cx.level()
    res = lower_begin(cx, rest)
    cx.push_block(l0, cx.level())
    return res


def lower_loop(cx, rest):
    """iter.rs:14-244."""
    if len(rest) < 3:
        raise LowerError("lower: invalid form 'loop'")
    if not isinstance(rest[0], Sym) or rest[0] != ":max":
        raise LowerError("lower: invalid form 'loop: expected :max keyword'")
    mx = rest[1]
    if isinstance(mx, int):
        max_n = mx
    elif isinstance(mx, Sym):
        b = cx.vars.get(mx)
        if b is not None and b[0] == "imm":
            max_n = b[1]
        elif mx in cx.const_ints:
            max_n = cx.const_ints[mx]
        else:
            raise LowerError("lower: invalid form 'loop: :max must be integer literal or constant'")
    else:
        raise LowerError("lower: invalid form 'loop: :max must be integer literal or constant'")
    if max_n == 0:
        raise LowerError("lower: invalid form 'loop: :max must be >= 1'")
    if not isinstance(rest[2], list):
        raise LowerError("lower: invalid form 'loop: expected binding list'")
    if not rest[2]:
        raise LowerError("lower: invalid form 'loop: empty binding list'")
    names, inits = [], []
    for kv in rest[2]:
        if not isinstance(kv, list) or len(kv) != 2:
            raise LowerError("lower: invalid form 'loop: binding pair'")
        if not isinstance(kv[0], Sym):
            raise LowerError("lower: invalid form 'loop: binding name'")
        names.append(kv[0])
        inits.append(kv[1])
    if len(rest) < 4:
        raise LowerError("lower: invalid form 'loop: missing body'")
    body = rest[3:]
    last = body[-1]
    recur_args = None
    if isinstance(last, list) and last and last[0] == "recur":
        recur_args = last[1:]
        if len(recur_args) != len(names):
            raise LowerError("lower: invalid form 'recur: arity must match loop bindings'")
        for f in body[:-1]:
            if contains_symbol(f, "recur"):
                raise LowerError("lower: invalid form 'recur: only allowed in tail position of loop body'")
    if recur_args is None:
        expanded = [Sym("block"), [Sym("let"), [[n, i] for n, i in zip(names, inits)], implicit_begin(body)]]
        return lower_expr(cx, expanded)
    prefix = body[:-1]
    l0 = cx.level()
    states = []  # [name, prior, reg]
    for name, init in zip(names, inits):
        r = into_owned(cx, lower_expr(cx, init))[1]
        prior = cx.vars.get(name)
        cx.vars[name] = ("reg", r)
        states.append([name, prior, r])
    result = None
    for it in range(max_n):
        last_val = None
        for idx, form in enumerate(prefix):
            v = lower_expr(cx, form)
            if idx + 1 < len(prefix):
                free_if_owned(cx, v)
            else:
                last_val = v
        if last_val is None:
            last_val = ("imm", 0)
        if it + 1 == max_n:
            result = last_val
            break
        free_if_owned(cx, last_val)
        for idx, expr in enumerate(recur_args):
            new_r = into_owned(cx, lower_expr(cx, expr))[1]
            st = states[idx]
            old_r = st[2]
            cx.vars[st[0]] = ("reg", new_r)
            st[2] = new_r
            if old_r != new_r:
                cx.free_reg(old_r)
    res = result if result is not None else ("imm", 0)
    res_reg = res[1] if res[0] != "imm" else None
    for name, prior, reg in reversed(states):
        cx.vars.pop(name, None)
        if prior is not None:
            cx.vars[name] = prior
        elif reg != res_reg:
            cx.free_reg(reg)
    cx.push_block(l0, cx.level())
    return res


def lower_select_like(cx, rest, what):
    """operators.rs:15-54 (if) and 238-282 (select): all three operands lowered first, an
    immediate 0/1 condition picks one; otherwise Select into a fresh register."""
    if len(rest) != 3:
        raise LowerError(f"lower: invalid form '{what}'")
    c, t, e = lower_expr(cx, rest[0]), lower_expr(cx, rest[1]), lower_expr(cx, rest[2])
    if c[0] == "imm":
        if c[1] == 0:
            free_if_owned(cx, t)
            return e
        if c[1] == 1:
            free_if_owned(cx, e)
            return t
        raise LowerError(f"lower: invalid form '{what}: cond must be boolean (0/1)'")
    c, t, e = into_owned(cx, c), into_owned(cx, t), into_owned(cx, e)
    dst = cx.alloc()
    cx.push("Select", dst=dst, c=c[1], a=t[1], b=e[1])
    free_if_owned(cx, c)
    free_if_owned(cx, t)
    free_if_owned(cx, e)
    return ("own", dst)


def range_assert(cx, r, bits):
    """alu.rs:617-642 assert_range_bits_for_reg."""
    dst = cx.alloc()
    if bits == 32:
        cx.push("AssertRange", dst=dst, r=r, bits=32)
    else:
        cx.push("AssertRangeLo", dst=dst, r=r)
        cx.push("AssertRangeHi", dst=dst, r=r)
    cx.free_reg(dst)


def lower_safe(cx, rest, what):
    """alu.rs:15-142: fold immediates when the result stays in u64; otherwise range-check both
    operands, compute into the left operand's register, range-check the result."""
    if len(rest) != 2:
        raise LowerError(f"lower: invalid form '{what}'")
    av, bv = lower_expr(cx, rest[0]), lower_expr(cx, rest[1])
    if av[0] == "imm" and bv[0] == "imm":
        x, y = av[1], bv[1]
        r = {"safe-add": x + y, "safe-sub": x - y if x >= y else None, "safe-mul": x * y}[what]
        if r is not None and 0 <= r < 1 << 64:
            return ("imm", r)
    a, b = into_owned(cx, av), into_owned(cx, bv)
    in_bits = 32 if what == "safe-mul" else 64
    range_assert(cx, a[1], in_bits)
    range_assert(cx, b[1], in_bits)
    dst = a[1]
    cx.push({"safe-add": "Add", "safe-sub": "Sub", "safe-mul": "Mul"}[what], dst=dst, a=a[1], b=b[1])
    range_assert(cx, dst, 64)
    free_if_owned(cx, b)
    return ("own", dst)


def lower_expr(cx, a):
    if isinstance(a, int) and not isinstance(a, bool):
        return ("imm", a)
    if isinstance(a, Sym):
        if a not in cx.vars:
            raise LowerError(f"lower: unknown symbol '{a}'")
        return binding_val(cx.vars[a])
    if not isinstance(a, list) or not a or not isinstance(a[0], Sym):
        raise LowerError("lower: invalid form 'expr'")
    h, rest = a[0], a[1:]
    if h in ("+", "*"):
        if len(rest) != 2:
            return lower_expr(cx, balance_chain(h, rest))
        return lower_bin(cx, rest, "Add" if h == "+" else "Mul")
    if h == "-":
        return lower_bin(cx, rest, "Sub")
    if h == "=":
        if len(rest) != 2:
            raise LowerError("lower: invalid form '='")
        x, y = lower_expr(cx, rest[0]), lower_expr(cx, rest[1])
        if x[0] == "imm" and y[0] == "imm":
            return ("imm", 1 if x[1] == y[1] else 0)
        x, y = into_owned(cx, x), into_owned(cx, y)
        dst = cx.alloc()
        cx.push("Eq", dst=dst, a=x[1], b=y[1])
        free_if_owned(cx, x)
        free_if_owned(cx, y)
        return ("own", dst)
    if h in ("if", "select"):
        return lower_select_like(cx, rest, h)
    if h == "when":
        if len(rest) < 2:
            raise LowerError("lower: invalid form 'when: expected cond and body'")
        return lower_expr(cx, [Sym("if"), rest[0], implicit_begin(rest[1:]), 0])
    if h == "neg":
        if len(rest) != 1:
            raise LowerError("lower: invalid form 'neg'")
        x = lower_expr(cx, rest[0])
        if x[0] == "imm" and x[1] == 0:
            return ("imm", 0)
        x = into_owned(cx, x)
        cx.push("Neg", dst=x[1], a=x[1])
        return x
    if h == "assert":
        if len(rest) != 1:
            raise LowerError("lower: invalid form 'assert'")
        c = lower_expr(cx, rest[0])
        if c[0] == "imm":
            if c[1] == 1:
                return ("imm", 1)
            raise LowerError("lower: invalid form 'assert: constant false'")
        c = into_owned(cx, c)
        dst = cx.alloc()
        cx.push("Assert", dst=dst, c=c[1])
        free_if_owned(cx, c)
        return ("own", dst)
    if h == "assert-bit":
        if len(rest) != 1:
            raise LowerError("lower: invalid form 'assert-bit'")
        x = lower_expr(cx, rest[0])
        if x[0] == "imm":
            if x[1] in (0, 1):
                return ("imm", 1)
            raise LowerError("lower: invalid form 'assert-bit: constant not a bit'")
        x = into_owned(cx, x)
        dst = cx.alloc()
        cx.push("AssertBit", dst=dst, r=x[1])
        free_if_owned(cx, x)
        return ("own", dst)
    if h == "assert-range":
        if len(rest) != 2:
            raise LowerError("lower: invalid form 'assert-range'")
        bits = rest[1]
        if not isinstance(bits, int):
            raise LowerError("lower: invalid form 'assert-range: bits must be integer'")
        x = lower_expr(cx, rest[0])
        if bits not in (32, 64):
            raise LowerError("lower: invalid form 'assert-range: bits must be 32 or 64'")
        if x[0] == "imm":
            if bits == 64 or x[1] < 1 << 32:
                return ("imm", 1)
            raise LowerError("lower: invalid form 'assert-range: constant out of range'")
        x = into_owned(cx, x)
        dst = cx.alloc()
        if bits == 32:
            cx.push("AssertRange", dst=dst, r=x[1], bits=32)
        else:
            cx.push("AssertRangeLo", dst=dst, r=x[1])
            cx.push("AssertRangeHi", dst=dst, r=x[1])
        free_if_owned(cx, x)
        return ("own", dst)
    if h in ("safe-add", "safe-sub", "safe-mul"):
        return lower_safe(cx, rest, h)
    if h == "load":
        if len(rest) != 1:
            raise LowerError("lower: invalid form 'load'")
        addr = into_owned(cx, lower_expr(cx, rest[0]))
        dst = cx.alloc()
        cx.push("Load", dst=dst, addr=addr[1])
        free_if_owned(cx, addr)
        return ("own", dst)
    if h == "store":
        if len(rest) != 2:
            raise LowerError("lower: invalid form 'store'")
        av, vv = lower_expr(cx, rest[0]), lower_expr(cx, rest[1])
        av, vv = materialize_imm(cx, av), materialize_imm(cx, vv)
        cx.push("Store", addr=av[1], src=vv[1])
        free_if_owned(cx, av)
        free_if_owned(cx, vv)
        return ("imm", 0)
    if h == "hash2":
        if len(rest) != 2:
            raise LowerError("lower: invalid form 'hash2'")
        x, y = lower_expr(cx, rest[0]), lower_expr(cx, rest[1])
        x, y = materialize_imm(cx, x), materialize_imm(cx, y)
        cx.push("SAbsorbN", regs=[x[1], y[1]])
        dst = cx.alloc()
        cx.push("SSqueeze", dst=dst)
        free_if_owned(cx, x)
        free_if_owned(cx, y)
        return ("own", dst)
    if h == "let":
        return lower_let(cx, rest)
    if h == "begin":
        return lower_begin(cx, rest)
    if h == "block":
        return lower_block(cx, rest)
    if h == "loop":
        return lower_loop(cx, rest)
    if h == "recur":
        raise LowerError("lower: invalid form 'recur outside loop'")
    if h == "typed-let":
        return ("imm", 0)
    if h == "secret-arg":
        if len(rest) != 1:
            raise LowerError("lower: invalid form 'secret-arg'")
        idx = rest[0]
        if not isinstance(idx, int):
            raise LowerError("lower: invalid form 'secret-arg: index must be integer literal'")
        if idx >= NR:
            raise LowerError("lower: invalid form 'secret-arg: index out of range for register file'")
        return ("bor", idx)
    if h in UNRESTATED:
        raise NotImplementedError(f"form {h!r} is outside the restated subset")
    return lower_call(cx, h, rest)


def lower_top(cx, f):
    if isinstance(f, list) and f and f[0] == "def":
        rest = f[1:]
        if not rest:
            raise LowerError("lower: invalid form 'def'")
        head = rest[0]
        if len(rest) < 2:
            raise LowerError("lower: invalid form 'def: body'")
        body = implicit_begin(rest[1:])
        if isinstance(head, list) and head:
            if not isinstance(head[0], Sym) or not all(isinstance(p, Sym) for p in head[1:]):
                raise LowerError("lower: invalid form 'def: name'")
            cx.funs[head[0]] = ([p for p in head[1:]], body)
        elif isinstance(head, Sym):
            if isinstance(body, int):  # (def NAME INT): compile-time constant + global binding
                cx.const_ints[head] = body
                cx.vars[head] = ("imm", body)
            cx.funs[head] = ([], body)
        else:
            raise LowerError("lower: invalid form 'def'")
    elif isinstance(f, list) and f and f[0] == "typed-fn":
        if len(f) != 5:
            raise LowerError("lower: invalid form 'typed-fn'")
        name, args, arrow, ret = f[1:]
        if arrow != "->":
            raise LowerError("lower: invalid form 'typed-fn: expected '->''")
        roles = []
        for spec in args:  # parse_arg_spec: bare type = Const, (role type)
            roles.append(("const", spec) if isinstance(spec, Sym) else (spec[0], spec[1]))
        cx.schemas[name] = (roles, ret)
    elif isinstance(f, list) and f and f[0] == "typed-let":
        pass
    elif isinstance(f, list) and f and f[0] == "deftype":
        raise NotImplementedError("deftype is outside the restated subset")
    else:
        free_if_owned(cx, lower_expr(cx, f))


def _finish(cx):
    if not cx.blocks and cx.ops:  # builder.rs:454-466: at least one block
        cx.blocks.append((0, len(cx.ops)))


def compile_str(src):
    """lib.rs:113-151.  Returns (ops, schemas, blocks)."""
    cx = Ctx()
    for f in parse(lex(src)):
        lower_top(cx, f)
    cx.push("End")
    _finish(cx)
    return cx.ops, cx.schemas, cx.blocks


def compile_entry(src, args, with_blocks=False):
    """lib.rs:155-256.  Returns (ops as [(kind, fields)], main schema or None)[, blocks]."""
    forms = parse(lex(src))
    arity = None
    for f in forms:
        if isinstance(f, list) and f and f[0] == "def" and len(f) > 1 and isinstance(f[1], list) \
                and f[1] and f[1][0] == "main":
            arity = len(f[1]) - 1
    if arity is None:
        raise LowerError("lower: invalid form 'main: not found'")
    if arity != len(args):
        raise LowerError(f"lower: invalid form 'main expects {arity} args (got {len(args)})'")
    cx = Ctx()
    for f in forms:
        lower_top(cx, f)
    res = into_owned(cx, lower_expr(cx, [Sym("main")] + [int(a) for a in args]))
    if res[1] != 0:
        cx.emit_mov(0, res[1])
    cx.push("End")
    _finish(cx)
    if with_blocks:
        return cx.ops, cx.schemas.get("main"), cx.blocks
    return cx.ops, cx.schemas.get("main")
