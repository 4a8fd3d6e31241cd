"""Pure-Python restatement (test infrastructure) used to pin the C oracle on small inputs.

BLAKE3 per the published spec; Poseidon suite derivation and PoseidonHasher per
zk-lisp-proof-winterfell/src/poseidon/mod.rs:56-217,421-440 and hasher.rs:57-231;
byte folding per utils.rs:33-74,346-381.  Big-int arithmetic mod p, so it is independent
of the C oracle's limb code.
"""
P = 2**128 - 45 * 2**40 + 1
M32 = 0xFFFFFFFF
IV = [0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A, 0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19]
PERM = [2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8]


def _rotr(x, n):
    return ((x >> n) | (x << (32 - n))) & M32


def _g(s, a, b, c, d, x, y):
    s[a] = (s[a] + s[b] + x) & M32
    s[d] = _rotr(s[d] ^ s[a], 16)
    s[c] = (s[c] + s[d]) & M32
    s[b] = _rotr(s[b] ^ s[c], 12)
    s[a] = (s[a] + s[b] + y) & M32
    s[d] = _rotr(s[d] ^ s[a], 8)
    s[c] = (s[c] + s[d]) & M32
    s[b] = _rotr(s[b] ^ s[c], 7)


def _compress(cv, block, ctr, blen, flags):
    s = list(cv) + IV[:4] + [ctr & M32, (ctr >> 32) & M32, blen, flags]
    m = list(block)
    for r in range(7):
        _g(s, 0, 4, 8, 12, m[0], m[1]); _g(s, 1, 5, 9, 13, m[2], m[3])
        _g(s, 2, 6, 10, 14, m[4], m[5]); _g(s, 3, 7, 11, 15, m[6], m[7])
        _g(s, 0, 5, 10, 15, m[8], m[9]); _g(s, 1, 6, 11, 12, m[10], m[11])
        _g(s, 2, 7, 8, 13, m[12], m[13]); _g(s, 3, 4, 9, 14, m[14], m[15])
        m = [m[PERM[i]] for i in range(16)]
    return [s[i] ^ s[i + 8] for i in range(8)]


def _words(b):
    b = b + bytes(64 - len(b))
    return [int.from_bytes(b[4 * i:4 * i + 4], "little") for i in range(16)]


def _chunk(data, idx, root):
    cv = list(IV)
    blocks = [data[i:i + 64] for i in range(0, len(data), 64)] or [b""]
    for bi, blk in enumerate(blocks):
        flags = (1 if bi == 0 else 0) | (2 if bi == len(blocks) - 1 else 0)
        if bi == len(blocks) - 1:
            return (cv, _words(blk), idx, len(blk), flags)
        cv = _compress(cv, _words(blk), idx, 64, flags)


def blake3(data: bytes) -> bytes:
    chunks = [data[i:i + 1024] for i in range(0, len(data), 1024)] or [b""]
    stack = []
    for ci, ch in enumerate(chunks[:-1]):
        cv = _compress(*_chunk(ch, ci, False))
        tot = ci + 1
        while tot & 1 == 0:
            cv = _compress(IV, stack.pop() + cv, 0, 64, 4)
            tot >>= 1
        stack.append(cv)
    node = _chunk(chunks[-1], len(chunks) - 1, False)
    while stack:
        cv = _compress(*node)
        node = (IV, stack.pop() + cv, 0, 64, 4)
    out = _compress(node[0], node[1], node[2], node[3], node[4] | 8)
    return b"".join(w.to_bytes(4, "little") for w in out)


def ro(domain: str, *parts: bytes) -> int:
    return int.from_bytes(blake3(domain.encode() + b"".join(parts))[:16], "little") % P


def fold32(b: bytes) -> int:
    return (int.from_bytes(b[:16], "little") % P + (int.from_bytes(b[16:32], "little") % P) * 2**64) % P


def suite(sid: bytes, rounds=27):
    dom = [ro("zkl/poseidon2/dom/c0", sid), ro("zkl/poseidon2/dom/c1", sid)]

    def pts(d, n):
        out, ctr = [], 0
        while len(out) < n:
            c = ro(d, sid, bytes([len(out)]), ctr.to_bytes(4, "little"))
            if c != 0 and c not in out:
                out.append(c)
            else:
                ctr += 1
        return out
    x = pts("zkl/poseidon2/mds/x", 12)
    y = pts("zkl/poseidon2/mds/y", 12)
    assert all((a + b) % P for a in x for b in y)
    mds = [[pow((x[i] + y[j]) % P, P - 2, P) for j in range(12)] for i in range(12)]
    rc = [[ro("zkl/poseidon2/rc", sid, bytes([r]), bytes([l])) for l in range(12)] for r in range(rounds)]
    return dom, mds, rc


_HS = None


def hasher_suite():
    global _HS
    if _HS is None:
        _HS = suite(bytes(32))
    return _HS


def permute(st, s=None):
    dom, mds, rc = s or hasher_suite()
    st = list(st)
    for r in range(len(rc)):
        c = [pow(v, 3, P) for v in st]
        st = [(sum(mds[i][k] * c[k] for k in range(12)) + rc[r][i]) % P for i in range(12)]
    return st


def sponge(domain: str, data: bytes) -> int:
    s = hasher_suite()
    st = [0] * 12
    st[10], st[11] = s[0]
    d = domain.encode()[:32]
    msgs = [fold32(d + bytes(32 - len(d)))]
    for i in range(0, len(data), 32):
        ch = data[i:i + 32]
        msgs.append(fold32(ch + bytes(32 - len(ch))))
    lane = 0
    for m in msgs:
        st[lane] = (st[lane] + m) % P
        lane += 1
        if lane == 10:
            st = permute(st, s)
            lane = 0
    if lane:
        st = permute(st, s)
    return st[0]


def digest(x):
    return x.to_bytes(16, "little") + bytes(16)


def hash_elements(elems):
    return sponge("winter/hash/elements", b"".join(e.to_bytes(16, "little") for e in elems))


def merge(a, b):
    return sponge("zkl/winter/hash/merge", digest(a) + digest(b))


def merge_many(ds):
    return sponge("zkl/winter/hash/merge_many", b"".join(digest(d) for d in ds)) if ds else 0


def merge_with_int(s, v):
    return sponge("zkl/winter/hash/merge_with_int", digest(s) + v.to_bytes(8, "little"))


def hash_bytes(b):
    return sponge("zkl/winter/hash/bytes", b)
