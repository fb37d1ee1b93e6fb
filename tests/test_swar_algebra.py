"""CPU check of the SWAR identities the bitmap kernel (k_bits in hq_kernels.hip) relies on: four
groups per 32-bit word, byte-wise popcount / compare, v_perm_b32 byte lookup for (1 << n) - 1.
The formulas are restated here in Python and compared against the per-group scalar rule on
random words, including invalid n and ragged tails. (The kernel itself is checked against the
oracle on the GPU; this pins the algebra on hosts without one.)"""
import random

M = 0xFFFFFFFF
B80, B01 = 0x80808080, 0x01010101


def popc_bytes(x):
    x = (x - ((x >> 1) & 0x55555555)) & M
    x = ((x & 0x33333333) + ((x >> 2) & 0x33333333)) & M
    return (x + (x >> 4)) & 0x0F0F0F0F


def ge(a, b):
    return (((a | B80) - b) & M) & B80


def pack4(f):
    return ((((f >> 7) & B01) * 0x01020408) & M) >> 24


def pack4x2(f):
    return ((((f >> 7) & B01) * 0x01041040) & M) >> 24


def valid(n):
    lo, hi = n & 0x0F0F0F0F, (n >> 4) & 0x0F0F0F0F
    return ((lo + 0x7F7F7F7F) & ~(lo + 0x77777777) & ~(hi + 0x7F7F7F7F)) & B80


def v_perm_b32(s0, s1, sel):
    v = (s0 << 32) | s1
    out = 0
    for i in range(4):
        s = (sel >> (8 * i)) & 0xFF
        b = (v >> (8 * s)) & 0xFF if s < 8 else (0 if s < 13 else 0xFF)
        out |= b << (8 * i)
    return out


def mask_n(n):
    return v_perm_b32(0x7F3F1F0F, 0x07030100, n | ((((n >> 3) & B01) * 0x0D) & M))


def scalar(n, a, g, r, ac, slot):
    bad = not 1 <= n <= 8
    mask = 0 if bad else (1 << n) - 1
    q = n // 2 + 1
    conf = (not bad) and bin(a & mask).count("1") + 1 >= q
    gm, rm = g & mask, r & mask & ~(g & mask)
    o = 1
    if not bad:
        o = 2 if bin(gm).count("1") >= q else (0 if bin(rm).count("1") >= q else 1)
    selfok = (not bad) and slot < n
    hq = selfok and bin((ac | (1 << slot)) & mask).count("1") >= q
    return conf, o, bad, hq, not selfok


def test_swar_matches_scalar_rule():
    rnd = random.Random(1)
    word = lambda v: sum(x << (8 * i) for i, x in enumerate(v))
    for _ in range(20000):
        ns = [rnd.choice([0, 9, 15, 16, 128, 255]) if rnd.random() < 0.3 else rnd.randint(1, 8)
              for _ in range(4)]
        av, gv, rv, acv = ([rnd.randint(0, 255) for _ in range(4)] for _ in range(4))
        slot, left = rnd.randint(0, 7), rnd.randint(1, 4)
        n, a, g, r, ac = word(ns), word(av), word(gv), word(rv), word(acv)
        inr = B80 if left >= 4 else B80 >> (8 * (4 - left))
        ok = valid(n) & inr
        mask = mask_n(n)
        q = (((n >> 1) & 0x7F7F7F7F) + B01) & M
        conf = pack4(ge(popc_bytes(a & mask), (q - B01) & M) & ok)
        gm = g & mask
        rm = r & mask & ~gm & M
        lead = ge(popc_bytes(gm), q) & ok
        foll = ge(popc_bytes(rm), q) & ok & ~lead & M
        outc = pack4x2(inr & ~lead & ~foll & M) | (pack4x2(lead) << 1)
        selfok = ge(n, ((slot + 1) * B01) & M) & ok
        hq = pack4(ge(popc_bytes((ac | (B01 << slot)) & mask), q) & selfok)
        fb_rv, fb_cq = pack4(~ok & inr & M), pack4(~selfok & inr & M)
        for k in range(4):
            got = ((conf >> k) & 1, (outc >> (2 * k)) & 3, (fb_rv >> k) & 1, (hq >> k) & 1,
                   (fb_cq >> k) & 1)
            if k < left:
                c, o, b, h, bq = scalar(ns[k], av[k], gv[k], rv[k], acv[k], slot)
                assert got == (int(c), o, int(b), int(h), int(bq)), (ns, k)
            else:
                assert got == (0, 0, 0, 0, 0)
