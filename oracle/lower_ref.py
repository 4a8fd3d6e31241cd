"""ORACLE (test infrastructure, not product): a Python restatement of the zk-lisp compiler's
front end for the forms examples/hello-zk.zlisp uses, so the op list the prover is fed for
BASELINE configs[0] is the one `compile_entry` emits, derived by code rather than by hand.

Follows zk-lisp-compiler/src:
  * lex / parse                lib.rs:259-491
  * compile_entry              lib.rs:155-256 (main's arity, (main ARGS...) lowered after the
                               top-level forms, result moved to r0, End; program_id = BLAKE3(src))
  * LowerCtx                   lower/ctx.rs:38-145 (free list 0..7, alloc pops the end = the
                               highest free register, free pushes back; emit_mov elides dst == src)
  * lower_top / lower_expr     lower/mod.rs:126-246
  * def / let / begin / call   lower/mod.rs:248-391, 553-631, 738-752
  * lower_bin (Sethi-Ullman order, Imm folding, dst reuse)  lower/mod.rs:393-551, 889-1026
  * secret-arg                 lower/mod.rs:754-782
  * typed-fn                   lower/mod.rs:784-825, 1049-1103 (schema only: no ops)
  * =                          lower/operators.rs:78-105
  * assert                     lower/assert.rs:15-40
  * ProgramBuilder::push       builder.rs:188-200 (a Mov onto itself is dropped)
Any other form raises NotImplementedError: this is not a compiler, only the subset needed.
"""

NR = 8


class Sym(str):
    pass


def lex(src):
    """lib.rs:259-430 (parens, quote, ';' comments, decimal u64, symbols, strings)."""
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
                raise ValueError("lex: integer out of u64 range")
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
            raise ValueError(f"lex: invalid char {ch!r} at {i}")
    return out


def parse(toks):
    """lib.rs:441-491: forms*; 'X -> (quote X)."""
    pos = 0

    def one():
        nonlocal pos
        t = toks[pos]
        pos += 1
        if t == "(":
            items = []
            while toks[pos] != ")":
                items.append(one())
            pos += 1
            return items
        if t == "'":
            return [Sym("quote"), one()]
        if t == ")":
            raise ValueError("parse: unmatched ')'")
        return t

    forms = []
    while pos < len(toks):
        forms.append(one())
    return forms


class Ctx:
    def __init__(self):
        self.free = list(range(NR))
        self.vars = {}
        self.funs = {}
        self.schemas = {}
        self.call_stack = []
        self.ops = []

    def alloc(self):
        if not self.free:
            raise ValueError("lower: regs exhausted")
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


def free_if_owned(cx, v):
    if v[0] == "own":
        cx.free_reg(v[1])


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
        raise ValueError("bin")
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


def lower_let(cx, rest):
    saved = []
    for kv in rest[0]:
        name = kv[0]
        v = lower_expr(cx, kv[1])
        saved.append((name, cx.vars.get(name), v))
        cx.vars[name] = ("imm", v[1]) if v[0] == "imm" else ("reg", v[1])
    res = lower_expr(cx, implicit_begin(rest[1:]))
    res_reg = res[1] if res[0] != "imm" else None
    for name, prior, v in reversed(saved):
        cx.vars.pop(name, None)
        if prior is not None:
            cx.vars[name] = prior
        elif v[0] == "own" and res_reg != v[1]:
            cx.free_reg(v[1])
    return res


def lower_call(cx, name, args):
    if name not in cx.funs:
        raise ValueError(f"lower: unknown symbol {name!r}")
    params, body = cx.funs[name]
    if name in cx.call_stack:
        raise ValueError("lower: recursion")
    cx.call_stack.append(name)
    if len(params) != len(args):
        raise ValueError("call: arity")
    argv = [lower_expr(cx, a) for a in args]
    saved = []
    for p, v in zip(params, argv):
        saved.append((p, cx.vars.get(p), v))
        cx.vars[p] = ("imm", v[1]) if v[0] == "imm" else ("reg", v[1])
    res = lower_expr(cx, body)
    res_reg = res[1] if res[0] != "imm" else None
    for p, prior, v in reversed(saved):
        cx.vars.pop(p, None)
        if prior is not None:
            cx.vars[p] = prior
        elif v[0] == "own" and res_reg != v[1]:
            cx.free_reg(v[1])
    cx.call_stack.pop()
    return res


def lower_expr(cx, a):
    if isinstance(a, int) and not isinstance(a, bool):
        return ("imm", a)
    if isinstance(a, Sym):
        if a not in cx.vars:
            raise ValueError(f"lower: unknown symbol {a!r}")
        b = cx.vars[a]
        return ("imm", b[1]) if b[0] == "imm" else ("bor", b[1])
    if not isinstance(a, list) or not a or not isinstance(a[0], Sym):
        raise ValueError("expr")
    h, rest = a[0], a[1:]
    if h in ("+", "*"):
        if len(rest) != 2:
            return lower_expr(cx, balance_chain(h, rest))
        return lower_bin(cx, rest, "Add" if h == "+" else "Mul")
    if h == "-":
        return lower_bin(cx, rest, "Sub")
    if h == "=":
        x, y = lower_expr(cx, rest[0]), lower_expr(cx, rest[1])
        if x[0] == "imm" and y[0] == "imm":
            return ("imm", 1 if x[1] == y[1] else 0)
        x, y = into_owned(cx, x), into_owned(cx, y)
        dst = cx.alloc()
        cx.push("Eq", dst=dst, a=x[1], b=y[1])
        free_if_owned(cx, x)
        free_if_owned(cx, y)
        return ("own", dst)
    if h == "assert":
        c = lower_expr(cx, rest[0])
        if c[0] == "imm":
            if c[1] == 1:
                return ("imm", 1)
            raise ValueError("assert: constant false")
        c = into_owned(cx, c)
        dst = cx.alloc()
        cx.push("Assert", dst=dst, c=c[1])
        free_if_owned(cx, c)
        return ("own", dst)
    if h == "let":
        return lower_let(cx, rest)
    if h == "begin":
        for it in rest[:-1]:
            free_if_owned(cx, lower_expr(cx, it))
        return lower_expr(cx, rest[-1])
    if h == "secret-arg":
        idx = rest[0]
        if not isinstance(idx, int) or idx >= NR:
            raise ValueError("secret-arg: index")
        return ("bor", idx)
    if h in cx.funs:
        return lower_call(cx, h, rest)
    raise NotImplementedError(f"form {h!r} is outside the restated subset")


def lower_top(cx, f):
    if isinstance(f, list) and f and f[0] == "def":
        head = f[1]
        if not isinstance(head, list):
            raise NotImplementedError("(def NAME ...)")
        cx.funs[head[0]] = ([p for p in head[1:]], implicit_begin(f[2:]))
    elif isinstance(f, list) and f and f[0] == "typed-fn":
        name, args, arrow, ret = f[1:]
        if arrow != "->":
            raise ValueError("typed-fn: expected '->'")
        roles = []
        for spec in args:  # parse_arg_spec: bare type = Const, (role type)
            roles.append(("const", spec) if isinstance(spec, Sym) else (spec[0], spec[1]))
        cx.schemas[name] = (roles, ret)
    else:
        free_if_owned(cx, lower_expr(cx, f))


def compile_entry(src, args):
    """lib.rs:155-256.  Returns (ops as [(kind, fields)], main schema or None)."""
    forms = parse(lex(src))
    arity = None
    for f in forms:
        if isinstance(f, list) and f and f[0] == "def" and isinstance(f[1], list) and f[1] and f[1][0] == "main":
            arity = len(f[1]) - 1
    if arity is None:
        raise ValueError("main: not found")
    if arity != len(args):
        raise ValueError(f"main expects {arity} args (got {len(args)})")
    cx = Ctx()
    for f in forms:
        lower_top(cx, f)
    res = into_owned(cx, lower_expr(cx, [Sym("main")] + [int(a) for a in args]))
    if res[1] != 0:
        cx.emit_mov(0, res[1])
    cx.push("End")
    return cx.ops, cx.schemas.get("main")
