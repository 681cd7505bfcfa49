#!/usr/bin/env python3
"""Generate csrc/fec_bitslice.inc: the bit-sliced RS encode networks of the fixed shapes.

Multiplying a byte by a constant c of GF(2^8) is a GF(2)-linear map on its 8 bits (an 8x8 bit
matrix). klauspost's encode (reed_solomon.go:51; parity[i] = sum_j M[k+i][j] * data[j], M =
vandermonde(n, k) * inv(top k x k), field 0x11D) is therefore one (8m x 8k) bit matrix applied to
every byte column. Held as bit planes (plane b of a shard = bit b of 32 of its bytes, one dword),
the whole parity computation is a fixed XOR network over planes: no tables, no lookups, and the
network is known at compile time, so common sub-sums can be shared (greedy pair extraction,
Paar's heuristic). Inputs stream in groups of G shards: within a group the 8G planes are combined,
and every output plane folds its group terms into its accumulator with three-input XORs.

The network is emitted as straight-line device code, one function per group of shards
(`bs_grp<k, m, group>`), which rs_encode_bits_kernel (fec_encode.hip) calls between the loads of
the next group. schedule() returns the same network as data
so the CPU tests can run it against the oracle (tests/test_bitslice.py).

usage: python 0xfec_amd/gen_bitslice.py            (rewrites 0xfec_amd/csrc/fec_bitslice.inc)
       python 0xfec_amd/gen_bitslice.py --check    (exit 1 if the file is stale)
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "csrc", "fec_bitslice.inc")
SHAPES = ((8, 4, 4), (16, 8, 4), (20, 10, 4))   # (k, m, group size G)

# ---------------------------------------------------------------- GF(2^8), poly 0x11D, generator 2
_EXP = [0] * 512
_LOG = [0] * 256
_v = 1
for _i in range(255):
    _EXP[_i] = _v
    _LOG[_v] = _i
    _v <<= 1
    if _v & 0x100:
        _v ^= 0x11D
for _i in range(255, 512):
    _EXP[_i] = _EXP[_i - 255]


def gmul(a, b):
    return 0 if a == 0 or b == 0 else _EXP[_LOG[a] + _LOG[b]]


def gpow(a, e):
    if e == 0:
        return 1
    return 0 if a == 0 else _EXP[(_LOG[a] * e) % 255]


def ginv(a):
    return _EXP[255 - _LOG[a]]


def _invert(m):
    n = len(m)
    a = [row[:] + [1 if i == j else 0 for j in range(n)] for i, row in enumerate(m)]
    for c in range(n):
        p = next(r for r in range(c, n) if a[r][c])
        a[c], a[p] = a[p], a[c]
        iv = ginv(a[c][c])
        a[c] = [gmul(iv, x) for x in a[c]]
        for r in range(n):
            if r != c and a[r][c]:
                f = a[r][c]
                a[r] = [x ^ gmul(f, y) for x, y in zip(a[r], a[c])]
    return [row[n:] for row in a]


def parity_rows(k, m):
    """klauspost v1.12.4 buildMatrix: vandermonde(n, k) (V[r][c] = r^c) times the inverse of its
    top k x k square; rows k..n-1."""
    n = k + m
    v = [[gpow(r, c) for c in range(k)] for r in range(n)]
    top = _invert(v[:k])
    return [[_dot(v[r], [top[i][c] for i in range(k)]) for c in range(k)] for r in range(k, n)]


def _dot(x, y):
    s = 0
    for a, b in zip(x, y):
        s ^= gmul(a, b)
    return s


def bit_matrix(k, m):
    """rows[8r + b] = the set of input planes 8j + i whose XOR is bit plane b of parity r."""
    rows = parity_rows(k, m)
    out = []
    for r in range(m):
        for b in range(8):
            s = set()
            for j in range(k):
                for i in range(8):
                    if (gmul(rows[r][j], 1 << i) >> b) & 1:
                        s.add(8 * j + i)
            out.append(s)
    return out


# ---------------------------------------------------------------- schedule
def _paar(rows, first_var):
    """Greedy pair extraction: repeatedly name the pair of variables shared by the most rows.
    Returns the new variables as (var, a, b) and the rows rewritten over all variables."""
    rows = [set(r) for r in rows]
    nxt = first_var
    pairs = []
    while True:
        cnt = {}
        for r in rows:
            lst = sorted(r)
            for x in range(len(lst)):
                for y in range(x + 1, len(lst)):
                    key = (lst[x], lst[y])
                    cnt[key] = cnt.get(key, 0) + 1
        if not cnt:
            break
        (a, b), n = max(cnt.items(), key=lambda t: (t[1], -t[0][0], -t[0][1]))
        if n < 2:
            break
        pairs.append((nxt, a, b))
        for r in rows:
            if a in r and b in r:
                r -= {a, b}
                r.add(nxt)
        nxt += 1
    return pairs, rows


def schedule(k, m, g, temp_base=None):
    """The network as ops over variables: 0..8k-1 are the input planes (8j + i); temporaries
    follow (from temp_base). Ops: ("t", v, a, b, group)  v = a ^ b;  ("acc", r, terms, group)
    y[r] ^= XOR(terms) (the first acc of a row assigns). Rows r = 8 * parity + bit."""
    full = bit_matrix(k, m)
    ops = []
    nxt = 8 * k if temp_base is None else temp_base
    for gi, s0 in enumerate(range(0, k, g)):
        cols = set(range(8 * s0, 8 * min(k, s0 + g)))
        sub = [sorted(r & cols) for r in full]
        pairs, rows = _paar(sub, nxt)
        nxt += len(pairs)
        ops += [("t", v, a, b, gi) for v, a, b in pairs]
        ops += [("acc", r, sorted(t), gi) for r, t in enumerate(rows) if t]
    return ops


def run_schedule(ops, planes, nrows):
    """Evaluate a schedule on integer planes (numpy arrays or ints); returns the nrows outputs."""
    var = dict(enumerate(planes))
    y = [None] * nrows
    for op in ops:
        if op[0] == "t":
            var[op[1]] = var[op[2]] ^ var[op[3]]
        else:
            acc = y[op[1]]
            for t in op[2]:
                acc = var[t] if acc is None else acc ^ var[t]
            y[op[1]] = acc
    return y


def op_count(ops):
    """VALU ops of the emitted code: one per pair, three-input XOR folds for the row terms."""
    n, seen = 0, set()
    for op in ops:
        if op[0] == "t":
            n += 1
        else:
            t = len(op[2]) - (0 if op[1] in seen else 1)
            n += (t + 1) // 2
            seen.add(op[1])
    return n


# ---------------------------------------------------------------- emit
def _name(v, g):
    return "x[%d][%d]" % (v // 8 % g, v % 8) if v < 8 * 256 else "t%d" % (v - 8 * 256)


def emit_fn(k, m, g):
    """One device function per group of g shards: bs_grp<k, m, group>(x, y), x the group's planes."""
    ops = schedule(k, m, g, temp_base=8 * 256)
    out = ["// RS(%d,%d): %d input planes -> %d parity planes, groups of %d shards, %d VALU ops per"
           % (k, k + m, 8 * k, 8 * m, g, op_count(ops)),
           "// 32-byte column (a dense bit matrix has %d ones)." % sum(len(r) for r in bit_matrix(k, m))]
    out += ["template <>", "struct BsShape<%d, %d> {" % (k, m), "    static constexpr int G = %d;" % g, "};"]
    seen = set()
    for gi in range((k + g - 1) // g):
        lines = ["template <>",
                 "__device__ __forceinline__ void bs_grp<%d, %d, %d>(const uint32_t (&x)[%d][8], uint32_t (&y)[%d][8]) {"
                 % (k, m, gi, g, m)]
        for op in ops:
            if op[-1] != gi:
                continue
            if op[0] == "t":
                lines.append("    const uint32_t %s = %s ^ %s;" % (_name(op[1], g), _name(op[2], g), _name(op[3], g)))
                continue
            r, terms = op[1], [_name(t, g) for t in op[2]]
            dst = "y[%d][%d]" % (r // 8, r % 8)
            if r in seen:
                acc = dst
            else:
                acc, terms = terms[0], terms[1:]
                seen.add(r)
            while len(terms) >= 2:
                acc = "xor3(%s, %s, %s)" % (acc, terms[0], terms[1])
                terms = terms[2:]
            if terms:
                acc = "(%s ^ %s)" % (acc, terms[0])
            lines.append("    %s = %s;" % (dst, acc))
        lines.append("}")
        out += lines
    return "\n".join(out) + "\n"


def render():
    head = ("// fec_bitslice.inc — GENERATED by 0xfec_amd/gen_bitslice.py; do not edit.\n"
            "// Bit-sliced XOR networks of klauspost's systematic RS parity rows (reed_solomon.go:51\n"
            "// Encode), included by fec_encode.hip. bs_grp<k, m, group>: x[j][b] = bit plane b of data shard\n"
            "// group * G + j; y[r][b] = bit plane b of parity shard r.\n\n")
    return head + "\n".join(emit_fn(k, m, g) for k, m, g in SHAPES)


def main():
    text = render()
    if "--check" in sys.argv:
        cur = open(OUT).read() if os.path.exists(OUT) else ""
        if cur != text:
            print("stale:", OUT)
            sys.exit(1)
        print("up to date:", OUT)
        return
    with open(OUT, "w") as f:
        f.write(text)
    for k, m, g in SHAPES:
        print("RS(%d,%d): %d ops" % (k, k + m, op_count(schedule(k, m, g))))


if __name__ == "__main__":
    main()
