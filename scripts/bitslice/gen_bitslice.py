#!/usr/bin/env python3
"""Generate scripts/bitslice/hb_bs_gen.hpp: the bitsliced AES S-box and
MixColumns as 3-input v_bitop3_b32 networks for gfx950.

Both circuits start from 2-input gate netlists:
  * S-box: the Boyar-Peralta circuit (tower-field inversion; 34 AND, 94
    XOR/XNOR), with the round key folded into its inputs (W_i = U_i ^ K_i:
    the key planes are all-zero / all-one masks, one per input bit);
  * MixColumns: out_r = xtime(a_r ^ a_(r+1)) ^ a_(r+1) ^ (a_(r+2) ^ a_(r+3))
    per bit.
A 3-feasible-cut technology mapper (area flow + exact-area refinement, the
FPGA LUT-mapping recipe) covers each netlist with 3-input LUTs; every LUT
becomes one v_bitop3_b32 whose 8-bit truth table is computed here by
simulation (src0 = 0xf0, src1 = 0xcc, src2 = 0xaa convention), 2-input LUTs
one v_xor/v_and/v_or form.  Every generated function is checked here against
the AES S-box (all 256 inputs x 2 key bits) and the GF(2^8) MixColumns.

Bit order: plane i of a byte is bit 7 - i (i = 0 is the most significant bit).
Usage: python scripts/bitslice/gen_bitslice.py  (rewrites the header in place).
"""
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "hb_bs_gen.hpp")

# ---------------------------------------------------------------- netlists
BP = """
T1 = U0 ^ U3
T2 = U0 ^ U5
T3 = U0 ^ U6
T4 = U3 ^ U5
T5 = U4 ^ U6
T6 = T1 ^ T5
T7 = U1 ^ U2
T8 = U7 ^ T6
T9 = U7 ^ T7
T10 = T6 ^ T7
T11 = U1 ^ U5
T12 = U2 ^ U5
T13 = T3 ^ T4
T14 = T6 ^ T11
T15 = T5 ^ T11
T16 = T5 ^ T12
T17 = T9 ^ T16
T18 = U3 ^ U7
T19 = T7 ^ T18
T20 = T1 ^ T19
T21 = U6 ^ U7
T22 = T7 ^ T21
T23 = T2 ^ T22
T24 = T2 ^ T10
T25 = T20 ^ T17
T26 = T3 ^ T16
T27 = T1 ^ T12
M1 = T13 & T6
M2 = T23 & T8
M3 = T14 ^ M1
M4 = T19 & U7
M5 = M4 ^ M1
M6 = T3 & T16
M7 = T22 & T9
M8 = T26 ^ M6
M9 = T20 & T17
M10 = M9 ^ M6
M11 = T1 & T15
M12 = T4 & T27
M13 = M12 ^ M11
M14 = T2 & T10
M15 = M14 ^ M11
M16 = M3 ^ M2
M17 = M5 ^ T24
M18 = M8 ^ M7
M19 = M10 ^ M15
M20 = M16 ^ M13
M21 = M17 ^ M15
M22 = M18 ^ M13
M23 = M19 ^ T25
M24 = M22 ^ M23
M25 = M22 & M20
M26 = M21 ^ M25
M27 = M20 ^ M21
M28 = M23 ^ M25
M29 = M28 & M27
M30 = M26 & M24
M31 = M20 & M23
M32 = M27 & M31
M33 = M27 ^ M25
M34 = M21 & M22
M35 = M24 & M34
M36 = M24 ^ M25
M37 = M21 ^ M29
M38 = M32 ^ M33
M39 = M23 ^ M30
M40 = M35 ^ M36
M41 = M38 ^ M40
M42 = M37 ^ M39
M43 = M37 ^ M38
M44 = M39 ^ M40
M45 = M42 ^ M41
M46 = M44 & T6
M47 = M40 & T8
M48 = M39 & U7
M49 = M43 & T16
M50 = M38 & T9
M51 = M37 & T17
M52 = M42 & T15
M53 = M45 & T27
M54 = M41 & T10
M55 = M44 & T13
M56 = M40 & T23
M57 = M39 & T19
M58 = M43 & T3
M59 = M38 & T22
M60 = M37 & T20
M61 = M42 & T1
M62 = M45 & T4
M63 = M41 & T2
L0 = M61 ^ M62
L1 = M50 ^ M56
L2 = M46 ^ M48
L3 = M47 ^ M55
L4 = M54 ^ M58
L5 = M49 ^ M61
L6 = M62 ^ L5
L7 = M46 ^ L3
L8 = M51 ^ M59
L9 = M52 ^ M53
L10 = M53 ^ L4
L11 = M60 ^ L2
L12 = M48 ^ M51
L13 = M50 ^ L0
L14 = M52 ^ M61
L15 = M55 ^ L1
L16 = M56 ^ L0
L17 = M57 ^ L1
L18 = M58 ^ L8
L19 = M63 ^ L4
L20 = L0 ^ L1
L21 = L1 ^ L7
L22 = L3 ^ L12
L23 = L18 ^ L2
L24 = L15 ^ L9
L25 = L6 ^ L10
L26 = L7 ^ L9
L27 = L8 ^ L10
L28 = L11 ^ L14
L29 = L11 ^ L17
Y0 = L6 ^ L24
Y1 = L16 ~ L26
Y2 = L19 ~ L28
Y3 = L6 ^ L21
Y4 = L20 ^ L22
Y5 = L25 ^ L29
Y6 = L13 ~ L27
Y7 = L6 ~ L23
"""


def sbox_netlist(keyed):
    lines = []
    if keyed:
        for i in range(8):
            lines.append(f"W{i} = U{i} ^ K{i}")
    for ln in BP.strip().split("\n"):
        if keyed:
            import re
            ln = re.sub(r"\bU(\d)\b", r"W\1", ln)
        lines.append(ln)
    return lines, [f"Y{i}" for i in range(8)]


def mixcol_netlist():
    # xtime(p) in MSB-first planes: [p1, p2, p3, p4^p0, p5^p0, p6, p7^p0, p0]
    xt = {0: [1], 1: [2], 2: [3], 3: [4, 0], 4: [5, 0], 5: [6], 6: [7, 0], 7: [0]}
    lines, outs = [], []
    for r in range(4):
        for i in range(8):
            lines.append(f"P{r}_{i} = A{r}_{i} ^ A{(r + 1) % 4}_{i}")
    for r in range(4):
        for i in range(8):
            terms = [f"P{r}_{s}" for s in xt[i]] + [f"A{(r + 1) % 4}_{i}", f"P{(r + 2) % 4}_{i}"]
            cur = terms[0]
            for k, t in enumerate(terms[1:]):
                name = f"O{r}_{i}" if k == len(terms) - 2 else f"X{r}_{i}_{k}"
                lines.append(f"{name} = {cur} ^ {t}")
                cur = name
            outs.append(f"O{r}_{i}")
    return lines, outs


# ---------------------------------------------------------------- mapper
def parse(lines):
    gates, order = {}, []
    for ln in lines:
        lhs, rhs = [s.strip() for s in ln.split("=")]
        a, op, b = rhs.split()
        gates[lhs] = (op, a, b)
        order.append(lhs)
    return gates, order


def lut_map(lines, outputs, iters=30, seed=0):
    gates, order = parse(lines)
    inputs = sorted({x for g in gates.values() for x in g[1:] if x not in gates})
    cuts = {x: [frozenset([x])] for x in inputs}
    for n in order:
        _, a, b = gates[n]
        cs = sorted({ca | cb for ca in cuts[a] for cb in cuts[b] if len(ca | cb) <= 3}, key=lambda c: (len(c), sorted(c)))
        keep = []
        for c in cs:
            if not any(k <= c for k in keep):
                keep.append(c)
        cuts[n] = keep + [frozenset([n])]
    fan = {n: 0 for n in list(gates) + inputs}
    for n in order:
        for x in gates[n][1:]:
            fan[x] += 1
    for o in outputs:
        fan[o] += 1
    af, best = {x: 0.0 for x in inputs}, {}
    for n in order:
        bc, bv = None, 1e9
        for c in cuts[n][:-1]:
            v = 1 + sum(af[x] / max(fan[x], 1) for x in c)
            if v < bv:
                bv, bc = v, c
        af[n], best[n] = bv, bc

    def cover():
        seen, stack = {}, list(outputs)
        while stack:
            n = stack.pop()
            if n in seen or n in inputs:
                continue
            seen[n] = best[n]
            stack.extend(best[n])
        return seen

    rng = random.Random(seed)
    cur = len(cover())
    for _ in range(iters):
        changed = False
        nodes = list(order)
        rng.shuffle(nodes)
        for n in nodes:
            if n not in cover():
                continue
            keep, kv = best[n], cur
            for c in cuts[n][:-1]:
                best[n] = c
                v = len(cover())
                if v < kv:
                    keep, kv = c, v
            if keep != best[n] or kv < cur:
                changed = changed or kv < cur
            best[n] = keep
            cur = kv
        if not changed:
            break
    return gates, order, inputs, cover()


def evaluate(gates, order, env):
    val = dict(env)
    full = (1 << 256) - 1
    for n in order:
        op, a, b = gates[n]
        x, y = val[a], val[b]
        val[n] = x ^ y if op == "^" else (x & y if op == "&" else full ^ x ^ y)
    return val


def lut_table(gates, order, node, leaves):
    """Truth table of `node` over its leaves: bit k = f(leaf0 = k>>2 & 1, ...)
    (v_bitop3_b32: src0 pattern 0xf0, src1 0xcc, src2 0xaa)."""
    pats = [0xF0, 0xCC, 0xAA]
    env = {}
    # simulate the cone with 8-bit patterns; any signal outside the cone is 0
    cone = set()
    stack = [node]
    while stack:
        n = stack.pop()
        if n in cone or n in leaves:
            continue
        cone.add(n)
        if n in gates:
            stack.extend(gates[n][1:])
    for i, l in enumerate(leaves):
        env[l] = pats[i]
    for n in order:
        if n not in cone:
            continue
        op, a, b = gates[n]
        x, y = env.get(a, 0), env.get(b, 0)
        env[n] = (x ^ y if op == "^" else (x & y if op == "&" else 0xFF ^ x ^ y)) & 0xFF
    return env[node]


def emit(fname, args, gates, order, luts, inmap, outmap, doc):
    """C++ body: each LUT -> one op.  inmap: netlist input -> C++ expr;
    outmap: netlist output -> C++ lvalue."""
    body = []
    names = {x: e for x, e in inmap.items()}
    nops = 0
    for n in order:
        if n not in luts:
            continue
        leaves = sorted(luts[n], key=lambda x: order.index(x) if x in gates else -1 - sorted(inmap).index(x))
        tt = lut_table(gates, order, n, leaves)
        ops = [names[l] for l in leaves]
        var = "t_" + n
        if len(leaves) == 3:
            expr = f"bs3<0x{tt:02x}>({ops[0]}, {ops[1]}, {ops[2]})"
        elif len(leaves) == 2:
            a, b = ops
            # 2-input: truth table over (a, b) = bits of tt at c = 0 / 1 duplicates
            t2 = {0x3c: f"{a} ^ {b}", 0xc3: f"~({a} ^ {b})", 0x30: f"{a} & ~{b}", 0xc0: f"{a} & {b}",
                  0x0c: f"~{a} & {b}", 0xfc: f"{a} | {b}", 0xf3: f"{a} | ~{b}", 0xcf: f"~{a} | {b}",
                  0x3f: f"~({a} & {b})", 0x03: f"~({a} | {b})"}
            # with pattern f0 (a) / cc (b), the table has c-independent pairs
            expr = t2.get(tt)
            if expr is None:
                expr = f"bs3<0x{tt:02x}>({a}, {b}, {b})"
        elif len(leaves) == 1:
            a = ops[0]
            expr = a if tt == 0xF0 else f"~{a}"
        else:
            raise ValueError(n)
        body.append(f"    const V {var} = {expr};")
        names[n] = var
        nops += 1
    for o, lv in outmap.items():
        body.append(f"    {lv} = {names[o]};")
    return (f"// {doc}\n// {nops} bitwise ops (generated).\n"
            f"template <class V>\nHB_HD void {fname}({args}) {{\n" + "\n".join(body) + "\n}\n"), nops


# ---------------------------------------------------------------- checks
def aes_sbox():
    def xt(x):
        return ((x << 1) ^ (0x1B if x & 0x80 else 0)) & 0xFF

    def mul(a, b):
        r = 0
        while b:
            if b & 1:
                r ^= a
            a = xt(a)
            b >>= 1
        return r
    sb = []
    for x in range(256):
        inv = 0 if x == 0 else next(y for y in range(1, 256) if mul(x, y) == 1)
        s, r = inv, inv
        for _ in range(4):
            r = ((r << 1) | (r >> 7)) & 0xFF
            s ^= r
        sb.append(s ^ 0x63)
    return sb, xt


def check_sbox(gates, order, ev=None):
    ev = ev or (lambda env: evaluate(gates, order, env))
    sb, _ = aes_sbox()
    for kbyte in (0x00, 0xFF, 0x5A, 0xC3):
        env = {}
        for i in range(8):
            env[f"U{i}"] = sum(((x >> (7 - i)) & 1) << x for x in range(256))
            env[f"K{i}"] = ((1 << 256) - 1) if (kbyte >> (7 - i)) & 1 else 0
        val = ev(env)
        for x in range(256):
            y = sum(((val[f"Y{i}"] >> x) & 1) << (7 - i) for i in range(8))
            assert y == sb[x ^ kbyte], (hex(x), hex(kbyte))


def check_mixcol(gates, order, ev=None):
    ev = ev or (lambda env: evaluate(gates, order, env))
    _, xt = aes_sbox()
    rng = random.Random(1)
    cols = [[rng.randrange(256) for _ in range(4)] for _ in range(256)]
    env = {}
    for r in range(4):
        for i in range(8):
            env[f"A{r}_{i}"] = sum(((c[r] >> (7 - i)) & 1) << n for n, c in enumerate(cols))
    val = ev(env)
    for n, c in enumerate(cols):
        for r in range(4):
            want = xt(c[r]) ^ xt(c[(r + 1) % 4]) ^ c[(r + 1) % 4] ^ c[(r + 2) % 4] ^ c[(r + 3) % 4]
            got = sum(((val[f"O{r}_{i}"] >> n) & 1) << (7 - i) for i in range(8))
            assert got == want


def lut_netlist(gates, order, luts, inputs):
    """The mapped network as a gate list of (name, tt, leaves), so the checks
    run on exactly what emit() writes."""
    out = []
    for n in order:
        if n in luts:
            leaves = sorted(luts[n], key=lambda x: order.index(x) if x in gates else -1 - sorted(inputs).index(x))
            out.append((n, lut_table(gates, order, n, leaves), leaves))
    return out


def eval_luts(net, env):
    full = (1 << 256) - 1
    val = dict(env)
    for n, tt, leaves in net:
        xs = [val[l] for l in leaves] + [0] * (3 - len(leaves))
        if len(leaves) == 2:
            xs[2] = xs[1]
        r = 0
        for k in range(8):
            if (tt >> k) & 1:
                a = xs[0] if k & 4 else full ^ xs[0]
                b = xs[1] if k & 2 else full ^ xs[1]
                c = xs[2] if k & 1 else full ^ xs[2]
                r |= a & b & c
        val[n] = r
    return val


def main():
    sl, so = sbox_netlist(keyed=True)
    sg, sord, sin, sl_luts = lut_map(sl, so)
    check_sbox(sg, sord)
    snet = lut_netlist(sg, sord, sl_luts, sin)
    check_sbox(None, None, lambda env: eval_luts(snet, env))
    ml, mo = mixcol_netlist()
    mg, mord, min_, ml_luts = lut_map(ml, mo)
    check_mixcol(mg, mord)
    mnet = lut_netlist(mg, mord, ml_luts, min_)
    check_mixcol(None, None, lambda env: eval_luts(mnet, env))
    s_in = {f"U{i}": f"u[{i}]" for i in range(8)}
    s_in.update({f"K{i}": f"k[{i}]" for i in range(8)})
    s_src, s_ops = emit("bs_sbox", "const V *u, const V *k, V *y", sg, sord, sl_luts, s_in,
                        {f"Y{i}": f"y[{i}]" for i in range(8)},
                        "y = AES S-box(u ^ k), 8 bit planes each, plane 0 = most significant bit")
    m_in = {f"A{r}_{i}": f"a[{r}][{i}]" for r in range(4) for i in range(8)}
    m_src, m_ops = emit("bs_mixcol", "const V (*a)[8], V (*o)[8]", mg, mord, ml_luts, m_in,
                        {f"O{r}_{i}": f"o[{r}][{i}]" for r in range(4) for i in range(8)},
                        "o = MixColumns(a) of one column: a[r] = row r, 8 bit planes each")
    hdr = f"""// hb_bs_gen.hpp -- GENERATED by scripts/bitslice/gen_bitslice.py; do not edit.
// Bitsliced AES S-box ({s_ops} ops, Boyar-Peralta circuit with the round key
// folded into its inputs) and MixColumns ({m_ops} ops), mapped onto 3-input
// v_bitop3_b32 LUTs.  Checked by the generator against the AES S-box for all
// 256 inputs under 4 key bytes and against GF(2^8) MixColumns; end to end on
// the GPU by ubench_bs.hip (CFB-8 against the host AES).
#pragma once

{s_src}
{m_src}"""
    with open(OUT, "w") as f:
        f.write(hdr)
    print(f"wrote {OUT}: sbox {s_ops} ops, mixcolumns {m_ops} ops")


if __name__ == "__main__":
    main()
