#!/usr/bin/env python3
"""Generates tools/aes_bitsliced.inc: a fully unrolled bitsliced
AES-128 encryption for 32 blocks per lane (one u32 per state bit) under the
fixed PRG keys of dpf/dpf.go:23-24.  Used by tools/aes_variants.hip to
compare the bitsliced back end with the LDS T-table one on MI355X.

State word index = 32*c + 8*r + b  (column c, row r, bit b; b = 0 is the
LSB of the byte), each u32 holding that bit of 32 independent blocks.
  SubBytes   : Boyar-Peralta depth-16 circuit (tools/sbox_circuit.py)
  ShiftRows  : renaming (no instructions)
  MixColumns : xtime on bit-planes
  AddRoundKey: compile-time key -> polarity flips
The whole round is built as a netlist of 2-input gates, then mapped onto
3-input cones (greedy LUT mapping), each emitted as one v_bitop3_b32 with
its truth table (src0 = 0xF0, src1 = 0xCC, src2 = 0xAA).
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
from sbox_circuit import parse  # noqa: E402

KEY_L = bytes([36, 156, 50, 234, 92, 230, 49, 9, 174, 170, 205, 160, 98, 236, 29, 243])
KEY_R = bytes([209, 12, 199, 173, 29, 74, 44, 128, 194, 224, 14, 44, 2, 201, 110, 28])


def sbox():
    def xt(a):
        return ((a << 1) ^ (0x1b if a & 0x80 else 0)) & 0xff
    exp, log = [0] * 256, [0] * 256
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x ^= xt(x)
    s = []
    for a in range(256):
        inv = exp[(255 - log[a]) % 255] if a else 0
        r, acc = inv, inv
        for _ in range(4):
            r = ((r << 1) | (r >> 7)) & 0xff
            acc ^= r
        s.append(acc ^ 0x63)
    return s


def expand(key):
    S = sbox()
    rcon = [1, 2, 4, 8, 16, 32, 64, 128, 0x1b, 0x36]
    w = [list(key[4 * i:4 * i + 4]) for i in range(4)]
    for i in range(4, 44):
        t = list(w[i - 1])
        if i % 4 == 0:
            t = [S[t[1]] ^ rcon[i // 4 - 1], S[t[2]], S[t[3]], S[t[0]]]
        w.append([w[i - 4][j] ^ t[j] for j in range(4)])
    return [bytes(sum((w[4 * r + c] for c in range(4)), [])) for r in range(11)]


def idx(c, r, b):
    return 32 * c + 8 * r + b


class Net:
    """2-input gate netlist: ops XOR, AND, NOT; leaves are named inputs."""

    def __init__(self):
        self.nodes = []          # (op, a, b) ; a/b are node ids or ('in', name)
        self.names = {}

    def leaf(self, name):
        if name not in self.names:
            self.nodes.append(("in", name, None))
            self.names[name] = len(self.nodes) - 1
        return self.names[name]

    def op(self, o, a, b=None):
        self.nodes.append((o, a, b))
        return len(self.nodes) - 1


def round_netlist(rk, last):
    """One AES round (SubBytes, ShiftRows, [MixColumns], AddRoundKey) as a
    netlist over inputs s0..s127; returns (net, outputs[128])."""
    net = Net()
    gates = parse()
    sub = {}
    for c in range(4):
        for r in range(4):
            v = {f"U{i}": net.leaf(f"s[{idx(c, r, 7 - i)}]") for i in range(8)}
            for dst, a, op, b in gates:
                if op == "+":
                    v[dst] = net.op("xor", v[a], v[b])
                elif op == "x":
                    v[dst] = net.op("and", v[a], v[b])
                else:
                    v[dst] = net.op("not", net.op("xor", v[a], v[b]))
            for i in range(8):
                sub[(c, r, 7 - i)] = v[f"S{i}"]

    def sr(c, r, b):   # ShiftRows: new column c, row r comes from column c + r
        return sub[((c + r) % 4, r, b)]

    outs = [None] * 128
    for c in range(4):
        if last:
            for r in range(4):
                for b in range(8):
                    o = sr(c, r, b)
                    if (rk[4 * c + r] >> b) & 1:
                        o = net.op("not", o)
                    outs[idx(c, r, b)] = o
            continue
        a = {(r, b): sr(c, r, b) for r in range(4) for b in range(8)}
        d = {(r, b): net.op("xor", a[(r, b)], a[((r + 1) % 4, b)]) for r in range(4) for b in range(8)}
        for r in range(4):
            r1, r2, r3 = (r + 1) % 4, (r + 2) % 4, (r + 3) % 4
            for b in range(8):
                # out_r = xtime(a_r ^ a_r1) ^ a_r1 ^ a_r2 ^ a_r3
                x = net.op("xor", a[(r2, b)], a[(r3, b)])
                x = net.op("xor", x, a[(r1, b)])
                x = net.op("xor", x, d[(r, 7)] if b == 0 else d[(r, b - 1)])
                if b in (1, 3, 4):
                    x = net.op("xor", x, d[(r, 7)])
                if (rk[4 * c + r] >> b) & 1:
                    x = net.op("not", x)
                outs[idx(c, r, b)] = x
    return net, outs


def lut_map(net, outs, k=3):
    """Greedy K-input cone mapping.  Returns emit list of (node, leaves, func)."""
    fanout = [0] * len(net.nodes)
    for o, a, b in net.nodes:
        if o == "in":
            continue
        fanout[a] += 1
        if b is not None:
            fanout[b] += 1
    for o in outs:
        fanout[o] += 1
    cut = {}
    for i, (o, a, b) in enumerate(net.nodes):
        if o == "in":
            cut[i] = {i}
            continue
        fins = [a] if b is None else [a, b]
        leaves = set(fins)
        # absorb single-fanout internal fanins while the cut stays <= k
        changed = True
        while changed:
            changed = False
            for f in sorted(leaves, key=lambda x: -len(cut.get(x, {x}))):
                if net.nodes[f][0] == "in" or fanout[f] != 1:
                    continue
                cand = (leaves - {f}) | cut[f]
                if len(cand) <= k:
                    leaves = cand
                    changed = True
                    break
        cut[i] = leaves
    # Nodes to emit: outputs and every node used as a leaf by an emitted node.
    need = set(outs)
    emit = []
    order = []
    stack = list(outs)
    seen = set()
    while stack:
        n = stack.pop()
        if n in seen or net.nodes[n][0] == "in":
            continue
        seen.add(n)
        order.append(n)
        for l in cut[n]:
            stack.append(l)
    order.sort()
    for n in order:
        emit.append((n, sorted(cut[n])))
    return emit, cut


def cone_func(net, n, leaves):
    masks = [0xF0, 0xCC, 0xAA]
    val = {l: masks[i] for i, l in enumerate(leaves)}

    def ev(x):
        if x in val:
            return val[x]
        o, a, b = net.nodes[x]
        if o == "xor":
            v = ev(a) ^ ev(b)
        elif o == "and":
            v = ev(a) & ev(b)
        elif o == "not":
            v = ~ev(a) & 0xFF
        else:
            raise ValueError(o)
        val[x] = v
        return v
    return ev(n)


def emit_round(L, rk, last, rnd):
    net, outs = round_netlist(rk, last)
    emit, _ = lut_map(net, outs)
    L.append(f"    {{  // round {rnd}: {len(emit)} v_bitop3")
    name = {}
    for i, (o, a, b) in enumerate(net.nodes):
        if o == "in":
            name[i] = a
    for n, leaves in emit:
        f = cone_func(net, n, leaves)
        args = [name[l] for l in leaves]
        while len(args) < 3:
            args.append(args[0])
        L.append(f"        const uint32_t v{n} = __builtin_amdgcn_bitop3_b32({args[0]}, {args[1]}, {args[2]}, 0x{f:02x});")
        name[n] = f"v{n}"
    for i in range(128):
        L.append(f"        t[{i}] = {name[outs[i]]};")
    L.append("        for (int i = 0; i < 128; ++i) s[i] = t[i];")
    L.append("    }")
    return len(emit)


def emit(keyname, key, out):
    rks = expand(key)
    L = []
    L.append(f"// AES-128 under the fixed PRG key {keyname} (dpf/dpf.go:23-24), 32 blocks per")
    L.append("// lane in bit-plane form s[32*c + 8*r + b].  Generated by tools/gen_bitsliced.py.")
    L.append(f"__device__ __forceinline__ void aes_bs_{keyname}(uint32_t* s) {{")
    L.append("    uint32_t t[128];")
    for c in range(4):
        for r in range(4):
            for b in range(8):
                if (rks[0][4 * c + r] >> b) & 1:
                    L.append(f"    s[{idx(c, r, b)}] = ~s[{idx(c, r, b)}];")
    total = 0
    for rnd in range(1, 11):
        total += emit_round(L, rks[rnd], rnd == 10, rnd)
    L.append("}")
    out.extend(L)
    return total


def main():
    out = ["// aes_bitsliced.inc — generated by tools/gen_bitsliced.py; do not edit.", "#pragma once", ""]
    nl = emit("L", KEY_L, out)
    out.append("")
    nr = emit("R", KEY_R, out)
    dst = os.path.join(HERE, "aes_bitsliced.inc")
    with open(dst, "w") as f:
        f.write("\n".join(out) + "\n")
    print(f"wrote {dst}: {nl} / {nr} bitop3 per 32-block encryption "
          f"({nl / 32:.1f} per block)")


if __name__ == "__main__":
    main()


def selftest(nblocks=32, seed=1):
    """Evaluate the mapped cones on random blocks and compare with a plain AES."""
    import random
    rnd_ = random.Random(seed)
    S = sbox()

    def xt(a):
        return ((a << 1) ^ (0x1b if a & 0x80 else 0)) & 0xff

    def aes(rks, blk):
        s = [blk[i] ^ rks[0][i] for i in range(16)]
        for r in range(1, 11):
            s = [S[x] for x in s]
            t = [s[4 * ((c + rr) % 4) + rr] for c in range(4) for rr in range(4)]
            if r < 10:
                u = []
                for c in range(4):
                    a0, a1, a2, a3 = t[4 * c:4 * c + 4]
                    al = a0 ^ a1 ^ a2 ^ a3
                    u += [a0 ^ al ^ xt(a0 ^ a1), a1 ^ al ^ xt(a1 ^ a2), a2 ^ al ^ xt(a2 ^ a3), a3 ^ al ^ xt(a3 ^ a0)]
                t = u
            s = [t[i] ^ rks[r][i] for i in range(16)]
        return bytes(s)

    for key in (KEY_L, KEY_R):
        rks = expand(key)
        blocks = [bytes(rnd_.getrandbits(8) for _ in range(16)) for _ in range(nblocks)]
        planes = [0] * 128
        for j, blk in enumerate(blocks):
            for c in range(4):
                for r in range(4):
                    for b in range(8):
                        if (blk[4 * c + r] >> b) & 1:
                            planes[idx(c, r, b)] |= 1 << j
        full = (1 << nblocks) - 1
        for i in range(128):
            if (rks[0][(i // 32) * 4 + (i % 32) // 8] >> (i % 8)) & 1:
                planes[i] ^= full
        for rnd in range(1, 11):
            net, outs = round_netlist(rks[rnd], rnd == 10)
            emit_l, _ = lut_map(net, outs)
            val = {}
            for i, (o, a, b) in enumerate(net.nodes):
                if o == "in":
                    val[i] = planes[int(a[2:-1])]
            for n, leaves in emit_l:
                f = cone_func(net, n, leaves)
                xs = [val[l] for l in leaves] + [val[leaves[0]]] * (3 - len(leaves))
                r_ = 0
                for bit in range(8):
                    if (f >> bit) & 1:
                        m0 = xs[0] if bit & 4 else ~xs[0]
                        m1 = xs[1] if bit & 2 else ~xs[1]
                        m2 = xs[2] if bit & 1 else ~xs[2]
                        r_ |= m0 & m1 & m2
                val[n] = r_ & full
            planes = [val[o] for o in outs]
        for j, blk in enumerate(blocks):
            got = bytearray(16)
            for i in range(128):
                if (planes[i] >> j) & 1:
                    got[(i // 32) * 4 + (i % 32) // 8] |= 1 << (i % 8)
            assert bytes(got) == aes(rks, blk), "bitsliced netlist mismatch"
    print("selftest ok: mapped netlist == AES-128 on", nblocks, "blocks, both keys")


if __name__ == "__main__" and "--selftest" in sys.argv:
    selftest()
