#!/usr/bin/env python3
"""Generate halo2-aggregation_amd/csrc/fp29_asm.hpp: per-field radix-2^29
Montgomery multiply / square with one inline-asm statement per product column.

Why: the compiler pads every inline-asm statement that writes an SGPR (the
dead carry-out of v_mad_u64_u32) with an `s_nop 0`, and, left to plain C, it
adds m and m << 22 (Pasta's power-of-two limbs) as 64-bit shift-adds of
{m, 0} pairs that each need a v_mov.  Here statement k holds the carry of
column k-1 (acc += m_{k-1} p_0; acc >>= 29) and every multiply-add of column
k: operand products, and the reduction's m_i p_j for all non-zero limbs p_j.
The two VALU ops that need acc's low word (m_k = acc (-p^-1) mod 2^29, or the
output limb) stay in C between statements.  Same arithmetic and result as
f29_mul_g / f29_sqr_g in fp29.hpp (see the bound comments there).

Subtractive form (Pasta, p = 1 mod 2^29): with m_k = acc mod 2^29 (no
negation), T - M p vanishes mod 2^29 column by column, so m_k p_0 = m_k
needs no multiply-add at all: the carry is acc >> 29, arithmetic (the
columns are signed 64-bit: the reduction terms m_i p_j enter as
v_mad_i64_i32 with -p_j).  Adding p R (p_j into column 9 + j) keeps the
result (T - M p) / R + p in (T / R, T / R + p], the range of the additive
form.  Per column: one AND instead of SUB + AND + a multiply-add, i.e. 18
instructions less per product; p R costs 3 adds (limbs paired into 64-bit
constants, pr_add).

Usage: python tools/gen_fp29_asm.py > halo2-aggregation_amd/csrc/fp29_asm.hpp
"""
import re

FIELDS = {
    "PallasFp": 0x40000000000000000000000000000000224698fc094cf91b992d30ed00000001,
    "VestaFp": 0x40000000000000000000000000000000224698fc0994a8dd8c46eb2100000001,
    "Bn254Fq": 21888242871839275222246405745257275088696311157297823662689037894645226208583,
    "Bn254Fr": 21888242871839275222246405745257275088548364400416034343698204186575808495617,
}
M29 = (1 << 29) - 1


def limbs(p):
    return [(p >> (29 * i)) & M29 for i in range(9)]


def const(ins, v):
    """Multiplier operand for a constant: inline constant when it is one."""
    if v <= 64:
        return str(v)
    return opnd(ins, "s", "%du" % v)


def nconst(ins, v):
    """Multiplier operand for the constant -v (v > 0) as a signed 32-bit value."""
    if v <= 16:
        return "-%d" % v
    return opnd(ins, "s", "%du" % ((-v) & 0xFFFFFFFF))


def pr_add(body, ins, k, P, kp):
    """+ kp p R at output column k (9 <= k <= 17): p_j goes into column 9 + j.
    Two limbs per 64-bit add (v_lshl_add_u64 of an SGPR-pair constant): column
    9 + 2i takes kp (p_2i + p_2i+1 2^29), the carry moves p_2i+1 into column
    10 + 2i (round 2 spent one multiply-add by 1 per limb)."""
    j = k - 9
    if j % 2:
        return
    v = kp * P[j] + (kp * P[j + 1] << 29 if j + 1 < 9 else 0)
    if not v:
        return
    if v < 1 << 32:
        body.append("v_mad_u64_u32 %%0, %%1, 1, %s, %%0" % const(ins, v))
    else:
        body.append("v_lshl_add_u64 %%0, %s, 0, %%0" % opnd(ins, "s", "%dull" % v))


def opnd(ins, c, e):
    for n, (c2, e2) in enumerate(ins):
        if (c2, e2) == (c, e):
            return "%%%d" % (n + 2)
    ins.append((c, e))
    return "%%%d" % (len(ins) + 1)


def statement(k, sq, P, sa=False, kp=None):
    """asm text and input list of statement k (acc is %0, the carry sink %1).
    sa: the operand a has signed limbs (two's complement, |a_i| < 2^29): its
    products are v_mad_i64_i32 and the columns signed (arithmetic carries);
    kp: the multiple of p R added to the result (default: 1 subtractive, 0
    additive)."""
    ins, body = [], []
    sub = P[0] == 1
    if kp is None:
        kp = 1 if sub else 0

    def mad(x, y):
        body.append("v_mad_u64_u32 %%0, %%1, %s, %s, %%0" % (x, y))

    def omad(x, y):  # operand product: signed when a is
        body.append("v_mad_%s %%0, %%1, %s, %s, %%0" % ("i64_i32" if sa else "u64_u32", x, y))

    if k >= 10:
        # dummy input: orders the C extraction of the previous output limb
        # before this statement (else the compiler copies acc with v_mov_b64)
        opnd(ins, "v", "r.l[%d]" % (k - 10))
    if k > 0:
        if not sub and k - 1 < 9:
            mad(opnd(ins, "v", "m[%d]" % (k - 1)), const(ins, P[0]))
        body.append("v_ashrrev_i64 %0, 29, %0" if sub or sa else "v_lshrrev_b64 %0, 29, %0")
        if kp and k >= 9:
            pr_add(body, ins, k, P, kp)  # + kp p R
    if k < 17:
        if not sq:
            for i in range(9):
                j = k - i
                if 0 <= j < 9:
                    omad(opnd(ins, "v", "a.l[%d]" % i), opnd(ins, "v", "b.l[%d]" % j))
        else:
            for i in range(9):
                j = k - i
                if i < j < 9:
                    omad(opnd(ins, "v", "d[%d]" % i), opnd(ins, "v", "a.l[%d]" % j))
            if k % 2 == 0 and k // 2 < 9:
                x = opnd(ins, "v", "a.l[%d]" % (k // 2))
                omad(x, x)
        for i in range(9):
            j = k - i
            if i < k and 1 <= j < 9 and P[j] != 0:
                if sub:
                    body.append("v_mad_i64_i32 %%0, %%1, %s, %s, %%0" % (opnd(ins, "v", "m[%d]" % i),
                                                                         nconst(ins, P[j])))
                else:
                    mad(opnd(ins, "v", "m[%d]" % i), const(ins, P[j]))
    return body, ins


def statement2(k, P, neg=False, sb=False):
    """f29_mul2_a, column k: statement A = carry-in + the a b terms, statement B
    = the u v terms + the reduction terms (one statement would exceed the
    inline-asm operand limit).

    neg (f29_mul2n_a): the u v terms are subtracted -- multiply-adds of u_i
    by the negated limbs nv_j (signed: v_mad_i64_i32), so the columns are
    signed (arithmetic carries) in both reduction forms, and the result gets
    p R more than the plain form (2 p R subtractive, p R additive) to stay
    positive: a b - u v > -R p / 16 for the operand bounds the curve
    routines use (u v < 6 p^2 < R p / 16)."""
    insA, bodyA, insB, bodyB = [], [], [], []
    sub = P[0] == 1
    signed = sub or neg or sb
    kp = (2 if sub else 1) if neg else (1 if sub else 0)  # multiple of p R added

    def mad(body, x, y):
        body.append("v_mad_u64_u32 %%0, %%1, %s, %s, %%0" % (x, y))

    if k >= 10:
        opnd(insA, "v", "r.l[%d]" % (k - 10))
    if k > 0:
        if not sub and k - 1 < 9:
            mad(bodyA, opnd(insA, "v", "m[%d]" % (k - 1)), const(insA, P[0]))
        bodyA.append("v_ashrrev_i64 %0, 29, %0" if signed else "v_lshrrev_b64 %0, 29, %0")
        if kp and k >= 9:
            pr_add(bodyA, insA, k, P, kp)
    if k < 17:
        for i in range(9):
            j = k - i
            if 0 <= j < 9:
                if sb:  # b signed (f29_mul2n_sb_a)
                    bodyA.append("v_mad_i64_i32 %%0, %%1, %s, %s, %%0" % (opnd(insA, "v", "a.l[%d]" % i),
                                                                          opnd(insA, "v", "b.l[%d]" % j)))
                else:
                    mad(bodyA, opnd(insA, "v", "a.l[%d]" % i), opnd(insA, "v", "b.l[%d]" % j))
                if neg:
                    bodyB.append("v_mad_i64_i32 %%0, %%1, %s, %s, %%0" % (opnd(insB, "v", "u.l[%d]" % i),
                                                                          opnd(insB, "v", "nv[%d]" % j)))
                else:
                    mad(bodyB, opnd(insB, "v", "u.l[%d]" % i), opnd(insB, "v", "v.l[%d]" % j))
        for i in range(9):
            j = k - i
            if i < k and 1 <= j < 9 and P[j] != 0:
                if sub:
                    bodyB.append("v_mad_i64_i32 %%0, %%1, %s, %s, %%0" % (opnd(insB, "v", "m[%d]" % i),
                                                                          nconst(insB, P[j])))
                else:
                    mad(bodyB, opnd(insB, "v", "m[%d]" % i), const(insB, P[j]))
    return [(bodyA, insA), (bodyB, insB)]


def asm_stmt(body, ins, first):
    """One inline-asm statement.  The product's first multiply-add starts the
    accumulator from the inline constant 0 (acc an early-clobber output), so
    no v_mov_b64 zeroes it."""
    if first:
        assert body[0].endswith(", %0")
        body = [body[0][:-len("%0")] + "0"] + body[1:]
    return '  asm("%s"\n      : "%s"(acc), "=&s"(c)\n      : %s);' % (
        "\\n\\t".join(body), "=&v" if first else "+v", ", ".join('"%s"(%s)' % ce for ce in ins))


def gen_fn2(field, neg=False, sb=False):
    """(a b + u v) 2^-261 mod p with ONE Montgomery reduction (sum of products);
    neg: (a b - u v) 2^-261 (f29_mul2n_a); sb: b with signed limbs
    (f29_mul2n_sb_a, neg only)."""
    p = FIELDS[field]
    P = limbs(p)
    inv = (-pow(p, -1, 1 << 29)) % (1 << 29)
    sub = P[0] == 1
    kp = (2 if sub else 1) if neg else (1 if sub else 0)
    name = "f29_mul2n_sb_a" if sb else "f29_mul2n_a" if neg else "f29_mul2_a"
    L = []
    L.append("template <>\n__device__ __forceinline__ F29<%s> %s<%s>(const F29<%s>& a, const F29<%s>& b, "
             "const F29<%s>& u, const F29<%s>& v) {" % (field, name, field, field, field, field, field))
    L.append("  F29<%s> r;\n  uint32_t m[9];\n  uint64_t acc, c;" % field)
    if neg:
        L.append("  uint32_t nv[9];\n#pragma unroll\n  for (int i = 0; i < 9; i++) nv[i] = 0u - v.l[i];")
    first = True
    for k in range(17):
        for body, ins in statement2(k, P, neg, sb):
            if not body:
                continue
            L.append(asm_stmt(body, ins, first))
            first = False
        if k < 9:
            if P[0] == 1:
                L.append("  m[%d] = (uint32_t)acc & kM29;" % k)
            elif inv == M29:
                L.append("  m[%d] = (0u - (uint32_t)acc) & kM29;" % k)
            else:
                L.append("  m[%d] = ((uint32_t)acc * %du) & kM29;" % (k, inv))
        else:
            L.append("  r.l[%d] = (uint32_t)acc & kM29;" % (k - 9))
    if kp:
        L.append("  r.l[8] = (uint32_t)((int64_t)acc >> 29) + %du;\n  (void)c;\n  return r;\n}\n" % (kp * P[8]))
    else:
        L.append("  r.l[8] = (uint32_t)(acc >> 29);\n  (void)c;\n  return r;\n}\n")
    return "\n".join(L)


def gen_fn(name, field, sq, sa=False):
    """sa: a with signed limbs; the product then gets p R more (subtractive 2,
    additive 1) unless it is a square (never negative)."""
    p = FIELDS[field]
    P = limbs(p)
    inv = (-pow(p, -1, 1 << 29)) % (1 << 29)
    sub = P[0] == 1
    kp = (1 if sub else 0) + (1 if sa and not sq else 0)
    L = []
    args = "const F29<%s>& a" % field + ("" if sq else ", const F29<%s>& b" % field)
    L.append("template <>\n__device__ __forceinline__ F29<%s> %s<%s>(%s) {" % (field, name, field, args))
    L.append("  F29<%s> r;\n  uint32_t m[9];\n  uint64_t acc, c;" % field)
    if sq:
        L.append("  uint32_t d[8];\n#pragma unroll\n  for (int i = 0; i < 8; i++) d[i] = a.l[i] << 1;")
    for k in range(17):
        body, ins = statement(k, sq, P, sa, kp)
        L.append(asm_stmt(body, ins, k == 0))
        if k < 9:
            if P[0] == 1:
                L.append("  m[%d] = (uint32_t)acc & kM29;" % k)
            elif inv == M29:
                L.append("  m[%d] = (0u - (uint32_t)acc) & kM29;" % k)
            else:
                L.append("  m[%d] = ((uint32_t)acc * %du) & kM29;" % (k, inv))
        else:
            L.append("  r.l[%d] = (uint32_t)acc & kM29;" % (k - 9))
    if sub or sa:
        L.append("  r.l[8] = (uint32_t)((int64_t)acc >> 29) + %du;\n  (void)c;\n  return r;\n}\n" % (kp * P[8]))
    else:
        L.append("  r.l[8] = (uint32_t)(acc >> 29);\n  (void)c;\n  return r;\n}\n")
    return "\n".join(L)


def main():
    doc = "\n".join("// " + l if l else "//" for l in __doc__.strip().split("\n"))
    out = [doc, "//", "// GENERATED by tools/gen_fp29_asm.py -- do not edit.", "#pragma once", '#include "fp29.hpp"', "",
           "namespace pm {", "",
           "template <class P>\n__device__ F29<P> f29_mul_a(const F29<P>& a, const F29<P>& b);",
           "template <class P>\n__device__ F29<P> f29_sqr_a(const F29<P>& a);",
           "template <class P>\n__device__ F29<P> f29_mul2_a(const F29<P>& a, const F29<P>& b, const F29<P>& u, "
           "const F29<P>& v);",
           "template <class P>\n__device__ F29<P> f29_mul2n_a(const F29<P>& a, const F29<P>& b, const F29<P>& u, "
           "const F29<P>& v);",
           "template <class P>\n__device__ F29<P> f29_mul_sa_a(const F29<P>& a, const F29<P>& b);",
           "template <class P>\n__device__ F29<P> f29_sqr_sa_a(const F29<P>& a);",
           "template <class P>\n__device__ F29<P> f29_mul2n_sb_a(const F29<P>& a, const F29<P>& b, const F29<P>& u, "
           "const F29<P>& v);", ""]
    for f in FIELDS:
        out.append(gen_fn("f29_mul_a", f, False))
        out.append(gen_fn("f29_sqr_a", f, True))
        out.append(gen_fn2(f))
        out.append(gen_fn2(f, neg=True))
    for f in ("PallasFp", "VestaFp", "Bn254Fq"):  # the MSM base fields (k_accumulate)
        out.append(gen_fn("f29_mul_sa_a", f, False, sa=True))
        out.append(gen_fn("f29_sqr_sa_a", f, True, sa=True))
        out.append(gen_fn2(f, neg=True, sb=True))
    out.append("}  // namespace pm")
    print("\n".join(out))


if __name__ == "__main__":
    main()
