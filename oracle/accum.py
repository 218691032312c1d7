"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the multiopen accumulator.

This is the Python big-integer restatement used as the *checker* for the HIP
accumulator kernels (SURVEY.md §8 rows a-3 … a-9).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it; the product library never does.

What it restates, in the native (out-of-circuit) meaning of the reference's
in-circuit gadgets (``main_gate.mul/add`` = field ops in C::ScalarExt,
``ecc_chip.mul_var/add`` = the group law of C):

  * ``eval_expr``              src/verifier.rs:58-151 (compute_expr)
  * ``scalar_block``           src/verifier.rs:512-652 (x^n, l_0 / l_last /
                               l_blind, expression order gates → permutation →
                               lookups, vanishing.verify)
  * ``permutation_expressions`` src/permutation.rs:190-324
  * ``lookup_expressions``     src/lookup.rs:173-311 (compress_expressions in
                               theta, Horner from zero)
  * ``vanishing_verify``       src/vanishing.rs:136-201 (h_eval Horner in y,
                               divided by x^n - 1; H = sum h_i (x^n)^i)
  * ``build_queries``          src/verifier.rs:654-715 + permutation.rs:332-358,
                               lookup.rs:314-347, vanishing.rs:206-220
  * ``construct_intermediate_sets`` src/multiopen.rs:19-45 (BTreeMap order)
  * ``calc_witness``           src/multiopen.rs:271-509 (Horner in v inside a
                               rotation set, Horner in u across sets,
                               e = [-eval_multi] g1)

PARITY STATUS: parity unpinned by the reference -- it holds no test vectors for
this path (``src/lib.rs:43-44``).  Pinned instead by two independent
restatements that must agree on every proof: ``accumulate`` (literal Horner /
group-law walk of the reference code) and ``accumulate_msm`` (closed-form
coefficients, one MSM per output), plus the field constants checked in
``tests/test_accum_oracle.py`` (roots of unity and DELTA equal the published
pasta_curves / halo2curves constants).

Layout of one proof's inputs (transcript read order of verifier.rs):
  points : instance commitments, advice commitments, per lookup (A', S'),
           permutation product commitments Z_p (one per chunk), per lookup Z,
           vanishing random commitment r, quotient pieces h_0..h_{d-1},
           multiopen witnesses W_0..W_{S-1} (one per rotation set, ascending)
  scalars: instance evals, advice evals, fixed evals, r(x), sigma evals,
           per permutation set (Z_p(x), Z_p(wx), [Z_p(w^last x) unless last]),
           per lookup (Z(x), Z(wx), A'(x), A'(w^-1 x), S'(x))
  challenges: theta, beta, gamma, y, x, v, u
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import pasta as P

# ------------------------------------------------------------------ constants
# 2-adic roots of unity and DELTA = GENERATOR^(2^S) of the scalar fields
# (pasta_curves: GENERATOR 5, S 32; halo2curves/pairing_bn256 Fr: GENERATOR 7,
# S 28).  tests/test_accum_oracle.py re-derives them and checks the published
# ROOT_OF_UNITY / DELTA constants.
FIELD_TWO_ADIC = {
    # scalar modulus: (generator, S)
    P.VESTA_P: (5, 32),   # Pallas scalar field (= Vesta base)
    P.PALLAS_P: (5, 32),  # Vesta scalar field (= Pallas base)
    P.BN254_R: (7, 28),
}


def two_adic(r):
    g, s = FIELD_TWO_ADIC[r]
    t = (r - 1) >> s
    return pow(g, t, r), pow(g, 1 << s, r), s


def domain_omega(r, k):
    """halo2 EvaluationDomain::new: omega = ROOT_OF_UNITY squared S-k times."""
    root, _, s = two_adic(r)
    assert k <= s
    return pow(root, 1 << (s - k), r)


def field_delta(r):
    return two_adic(r)[1]


# ---------------------------------------------------------------- expressions
# halo2 plonk::Expression restated as tuples:
#   ("const", c) ("fixed", q) ("advice", q) ("instance", q)
#   ("neg", e) ("sum", a, b) ("prod", a, b) ("scaled", e, c)
def Const(c):
    return ("const", c)


def Fixed(q):
    return ("fixed", q)


def Advice(q):
    return ("advice", q)


def Instance(q):
    return ("instance", q)


def Neg(e):
    return ("neg", e)


def Sum(a, b):
    return ("sum", a, b)


def Prod(a, b):
    return ("prod", a, b)


def Scaled(e, c):
    return ("scaled", e, c)


def eval_expr(r, e, adv, fixed, inst):
    """compute_expr, src/verifier.rs:58-151 (native field meaning)."""
    op = e[0]
    if op == "const":
        return e[1] % r
    if op == "fixed":
        return fixed[e[1]]
    if op == "advice":
        return adv[e[1]]
    if op == "instance":
        return inst[e[1]]
    if op == "neg":
        return (-eval_expr(r, e[1], adv, fixed, inst)) % r
    if op == "sum":
        return (eval_expr(r, e[1], adv, fixed, inst) + eval_expr(r, e[2], adv, fixed, inst)) % r
    if op == "prod":
        return eval_expr(r, e[1], adv, fixed, inst) * eval_expr(r, e[2], adv, fixed, inst) % r
    if op == "scaled":
        return eval_expr(r, e[1], adv, fixed, inst) * (e[2] % r) % r
    raise ValueError(op)


# ------------------------------------------------------------------- shape
KIND_ADVICE, KIND_FIXED, KIND_INSTANCE = 0, 1, 2


@dataclass
class ProofShape:
    """Everything of the VerifyingKey / ConstraintSystem the accumulator reads
    (src/verifier.rs:227-285)."""
    log_n: int
    blinding_factors: int
    num_instance_columns: int
    num_advice_columns: int
    num_fixed_columns: int
    num_lookups: int
    perm_chunk_len: int            # cs.degree() - 2 (verifier.rs:236)
    quotient_degree: int           # vk.domain.get_quotient_poly_degree()
    instance_queries: List[Tuple[int, int]]   # (column, rotation)
    advice_queries: List[Tuple[int, int]]
    fixed_queries: List[Tuple[int, int]]
    perm_columns: List[Tuple[int, int]]       # (kind, query index), verifier.rs:255
    gates: list
    lookup_inputs: list            # flattened over all lookups (verifier.rs:244-251)
    lookup_tables: list
    omega: int
    delta: int
    fixed_commitments: list = field(default_factory=list)   # VK points
    sigma_commitments: list = field(default_factory=list)

    @property
    def n_perm_sets(self):
        return (len(self.perm_columns) + self.perm_chunk_len - 1) // self.perm_chunk_len

    # per-proof point layout
    def point_offsets(self):
        o = {}
        k = 0
        for name, cnt in (("inst", self.num_instance_columns), ("adv", self.num_advice_columns),
                          ("lk_perm", 2 * self.num_lookups), ("perm_z", self.n_perm_sets),
                          ("lk_z", self.num_lookups), ("rand", 1), ("h", self.quotient_degree)):
            o[name] = (k, cnt)
            k += cnt
        o["W"] = (k, self.num_sets())
        return o

    def points_per_proof(self):
        return sum(self.point_offsets()[k][1] for k in self.point_offsets())

    def scalar_offsets(self):
        o = {}
        k = 0
        nps = self.n_perm_sets
        for name, cnt in (("inst", len(self.instance_queries)), ("adv", len(self.advice_queries)),
                          ("fixed", len(self.fixed_queries)), ("rand", 1), ("sigma", len(self.perm_columns)),
                          ("perm", 3 * nps - 1 if nps else 0), ("lk", 5 * self.num_lookups)):
            o[name] = (k, cnt)
            k += cnt
        return o

    def scalars_per_proof(self):
        return sum(v[1] for v in self.scalar_offsets().values())

    def rotations(self):
        rots = set()
        for _, rot in self.instance_queries + self.advice_queries + self.fixed_queries:
            rots.add(rot)
        if self.n_perm_sets:
            rots |= {0, 1}
            if self.n_perm_sets > 1:
                rots.add(-(self.blinding_factors + 1))
        if self.num_lookups:
            rots |= {0, -1, 1}
        if self.perm_columns:
            rots.add(0)
        rots.add(0)  # vanishing
        return sorted(rots)

    def num_sets(self):
        return len(self.rotations())


def simple_example_shape(curve, log_n):
    """Synthetic shape of the reference's inner circuit
    (examples/simple-example.rs:99-159, 331-344):
    advice 2, instance 1, fixed 4 (constant, u8 table, s_mul, s_lookup),
    gate s_mul*(a0*a1 - a0(next)), lookup s_lookup*a0 in table,
    permutation over (instance, constant, a0, a1), degree 5 -> chunk 3,
    blinding factors 5, quotient pieces 4.  Degree rules are halo2's [3P,
    estimate]; the kernels take the shape as data, not these numbers."""
    r = curve.r
    inst_q = [(0, 0)]
    adv_q = [(0, 0), (1, 0), (0, 1)]
    fixed_q = [(0, 0), (1, 0), (2, 0), (3, 0)]  # constant, table, s_mul, s_lookup
    gate = Prod(Fixed(2), Sum(Prod(Advice(0), Advice(1)), Neg(Advice(2))))
    lk_in = [Prod(Fixed(3), Advice(0))]
    lk_tab = [Fixed(1)]
    perm_cols = [(KIND_INSTANCE, 0), (KIND_FIXED, 0), (KIND_ADVICE, 0), (KIND_ADVICE, 1)]
    return ProofShape(log_n=log_n, blinding_factors=5, num_instance_columns=1, num_advice_columns=2,
                      num_fixed_columns=4, num_lookups=1, perm_chunk_len=3, quotient_degree=4,
                      instance_queries=inst_q, advice_queries=adv_q, fixed_queries=fixed_q,
                      perm_columns=perm_cols, gates=[gate], lookup_inputs=lk_in, lookup_tables=lk_tab,
                      omega=domain_omega(r, log_n), delta=field_delta(r))


# -------------------------------------------------------------- proof parse
@dataclass
class Proof:
    points: list      # affine (x, y) tuples or None, shape.points_per_proof()
    scalars: list     # ints mod r, shape.scalars_per_proof()
    challenges: list  # theta, beta, gamma, y, x, v, u


def _split(shape, pf):
    po, so = shape.point_offsets(), shape.scalar_offsets()

    def pts(name):
        a, n = po[name]
        return pf.points[a:a + n]

    def scs(name):
        a, n = so[name]
        return pf.scalars[a:a + n]

    lk_perm = pts("lk_perm")
    lk_ev = scs("lk")
    perm_ev = scs("perm")
    sets = []
    k = 0
    zps = pts("perm_z")
    for i in range(shape.n_perm_sets):
        zp, zpn = perm_ev[k], perm_ev[k + 1]
        k += 2
        last = None
        if i + 1 < shape.n_perm_sets:
            last = perm_ev[k]
            k += 1
        sets.append(dict(comm=zps[i], eval=zp, next=zpn, last=last))
    lookups = []
    for i in range(shape.num_lookups):
        z, zw, a, ap, s = lk_ev[5 * i:5 * i + 5]
        lookups.append(dict(a_comm=lk_perm[2 * i], s_comm=lk_perm[2 * i + 1], z_comm=pts("lk_z")[i],
                            z=z, z_w=zw, a=a, a_prev=ap, s=s))
    return dict(inst=pts("inst"), adv=pts("adv"), rand=pts("rand")[0], h=pts("h"), W=pts("W"),
                inst_ev=scs("inst"), adv_ev=scs("adv"), fixed_ev=scs("fixed"), rand_ev=scs("rand")[0],
                sigma_ev=scs("sigma"), perm_sets=sets, lookups=lookups)


# ---------------------------------------------------------- scalar block
def lagrange_evals(r, shape, x, xn):
    """verifier.rs:553-591 -> (l_0, l_last, l_blind)."""
    n = 1 << shape.log_n
    omega_inv = pow(shape.omega, -1, r)
    w = 1
    ls = []
    for _ in range(2 + shape.blinding_factors):
        num = w * (xn - 1) % r
        den = (x - w) % r * n % r
        ls.append(num * pow(den, -1, r) % r)
        w = w * omega_inv % r
    ls.reverse()
    l_last = ls[0]
    l_blind = 0
    for i in range(1, 1 + shape.blinding_factors):
        l_blind = (l_blind + ls[i]) % r
    l_0 = ls[1 + shape.blinding_factors]
    return l_0, l_last, l_blind


def permutation_expressions(r, shape, d, l_0, l_last, l_blind, beta, gamma, x):
    """permutation.rs:190-324."""
    sets = d["perm_sets"]
    exprs = [l_0 * (1 - sets[0]["eval"]) % r]
    zl = sets[-1]["eval"]
    exprs.append(l_last * (zl * zl - zl) % r)
    for i in range(1, len(sets)):
        exprs.append(l_0 * (sets[i]["eval"] - sets[i - 1]["last"]) % r)
    deltas = []
    acc = 1
    for _ in range(len(shape.perm_columns)):
        deltas.append(acc)
        acc = acc * shape.delta % r
    src = {KIND_ADVICE: d["adv_ev"], KIND_FIXED: d["fixed_ev"], KIND_INSTANCE: d["inst_ev"]}
    cl = shape.perm_chunk_len
    for ci, st in enumerate(sets):
        cols = shape.perm_columns[ci * cl:(ci + 1) * cl]
        sig = d["sigma_ev"][ci * cl:(ci + 1) * cl]
        left = st["next"]
        for (kind, q), s in zip(cols, sig):
            left = left * ((beta * s + src[kind][q]) % r + gamma) % r
        right = st["eval"]
        for i, (kind, q) in enumerate(cols):
            t = beta * deltas[cl * ci + i] % r * x % r
            right = right * ((t + src[kind][q]) % r + gamma) % r
        exprs.append((left - right) * (1 - (l_last + l_blind)) % r)
    return exprs


def lookup_expressions(r, shape, lk, d, l_0, l_last, l_blind, theta, beta, gamma):
    """lookup.rs:173-311 (compress over the flattened expression lists)."""
    def compress(exprs):
        acc = 0
        for e in exprs:
            acc = (acc * theta + eval_expr(r, e, d["adv_ev"], d["fixed_ev"], d["inst_ev"])) % r
        return acc

    e1 = l_0 * (1 - lk["z"]) % r
    e2 = l_last * (lk["z"] * lk["z"] - lk["z"]) % r
    omb = (1 - (l_last + l_blind)) % r
    left = (lk["a"] + beta) * (lk["s"] + gamma) % r * lk["z_w"] % r
    right = (compress(shape.lookup_inputs) + beta) * (compress(shape.lookup_tables) + gamma) % r * lk["z"] % r
    e3 = omb * (left - right) % r
    aps = (lk["a"] - lk["s"]) % r
    e4 = l_0 * aps % r
    e5 = omb * (aps * (lk["a"] - lk["a_prev"]) % r) % r
    return [e1, e2, e3, e4, e5]


STATUS_DENOM_ZERO = 4  # PM_ACCUM_DENOM_ZERO


def proof_status(curve, shape, ch):
    """Status bit of the scalar block: a zero denominator, i.e. x^n = 1 or
    x = omega^-i for i < bf + 2 (both mean x is an n-th root of unity), where
    the reference's main_gate.div fails (vanishing.rs:175, verifier.rs:580)."""
    r = curve.r
    x = ch[4] % r
    xn = x
    for _ in range(shape.log_n):
        xn = xn * xn % r
    if xn == 1:
        return STATUS_DENOM_ZERO
    omega_inv = pow(shape.omega, -1, r)
    w = 1
    for _ in range(2 + shape.blinding_factors):
        if x == w:
            return STATUS_DENOM_ZERO
        w = w * omega_inv % r
    return 0


def scalar_block(curve, shape, d, ch):
    """verifier.rs:512-652 -> (expressions, xn, h_eval)."""
    r = curve.r
    theta, beta, gamma, y, x, v, u = ch
    xn = x
    for _ in range(shape.log_n):
        xn = xn * xn % r
    l_0, l_last, l_blind = lagrange_evals(r, shape, x, xn)
    exprs = [eval_expr(r, g, d["adv_ev"], d["fixed_ev"], d["inst_ev"]) for g in shape.gates]
    exprs += permutation_expressions(r, shape, d, l_0, l_last, l_blind, beta, gamma, x)
    for lk in d["lookups"]:
        exprs += lookup_expressions(r, shape, lk, d, l_0, l_last, l_blind, theta, beta, gamma)
    # vanishing.rs:145-175
    h = exprs[0]
    for e in exprs[1:]:
        h = (e + h * y) % r
    h_eval = h * pow((xn - 1) % r, -1, r) % r
    return exprs, xn, h_eval


# ----------------------------------------------------------------- queries
H_POINT = "H"  # the vanishing commitment H = sum h_i xn^i (vanishing.rs:178-188)


def build_queries(shape, d, h_eval):
    """verifier.rs:654-715: list of (point ref, rotation, eval).  Point refs are
    ("proof", index) / ("fixed", column) / ("sigma", k) / H_POINT so the two
    restatements (and the GPU plan) share them."""
    po = shape.point_offsets()
    q = []
    for i, (col, rot) in enumerate(shape.instance_queries):
        q.append((("proof", po["inst"][0] + col), rot, d["inst_ev"][i]))
    for i, (col, rot) in enumerate(shape.advice_queries):
        q.append((("proof", po["adv"][0] + col), rot, d["adv_ev"][i]))
    # permutation.rs:332-358
    last_rot = -(shape.blinding_factors + 1)
    for i, st in enumerate(d["perm_sets"]):
        ref = ("proof", po["perm_z"][0] + i)
        q.append((ref, 0, st["eval"]))
        q.append((ref, 1, st["next"]))
    for i in range(len(d["perm_sets"]) - 2, -1, -1):
        q.append((("proof", po["perm_z"][0] + i), last_rot, d["perm_sets"][i]["last"]))
    # lookup.rs:314-347
    for i, lk in enumerate(d["lookups"]):
        zr = ("proof", po["lk_z"][0] + i)
        ar = ("proof", po["lk_perm"][0] + 2 * i)
        sr = ("proof", po["lk_perm"][0] + 2 * i + 1)
        q += [(zr, 0, lk["z"]), (ar, 0, lk["a"]), (sr, 0, lk["s"]), (ar, -1, lk["a_prev"]), (zr, 1, lk["z_w"])]
    for i, (col, rot) in enumerate(shape.fixed_queries):
        q.append((("fixed", col), rot, d["fixed_ev"][i]))
    for k, ev in enumerate(d["sigma_ev"]):
        q.append((("sigma", k), 0, ev))
    # vanishing.rs:206-220
    q.append((H_POINT, 0, h_eval))
    q.append((("proof", po["rand"][0]), 0, d["rand_ev"]))
    return q


def construct_intermediate_sets(queries):
    """multiopen.rs:19-45: group by rotation, ascending (BTreeMap), keeping the
    query order inside each set."""
    by = {}
    for qu in queries:
        by.setdefault(qu[1], []).append(qu)
    return [(rot, by[rot]) for rot in sorted(by)]


# ----------------------------------------------------------- accumulators
def _resolve(curve, shape, pf, ref, H):
    if ref == H_POINT:
        return H
    kind, i = ref
    if kind == "proof":
        return pf.points[i]
    if kind == "fixed":
        return shape.fixed_commitments[i]
    return shape.sigma_commitments[i]


def vanishing_H(curve, d, xn):
    """vanishing.rs:178-188."""
    r = curve.r
    Hp = curve.jac(d["h"][0])
    xp = xn
    for hc in d["h"][1:]:
        Hp = curve.jadd(Hp, curve.jac(curve.mul(xp, hc)))
        xp = xp * xn % r
    return curve.jaffine(Hp)


def accumulate(curve, shape, pf, g1=None):
    """Literal restatement: scalar block, queries, calc_witness (Horner walk).
    Returns (w, zw, f, e, h_eval) with affine points (None = identity)."""
    r = curve.r
    g1 = g1 or curve.gen
    d = _split(shape, pf)
    theta, beta, gamma, y, x, v, u = pf.challenges
    _, xn, h_eval = scalar_block(curve, shape, d, pf.challenges)
    H = vanishing_H(curve, d, xn)
    sets = construct_intermediate_sets(build_queries(shape, d, h_eval))
    assert len(sets) == len(d["W"]), (len(sets), len(d["W"]))
    omega_inv = pow(shape.omega, -1, r)

    def madd(Pa, Qa):
        return curve.jaffine(curve.jadd(curve.jac(Pa), curve.jac(Qa)))

    Ws, ZWs, Fs = [], [], []
    eval_multi = 0
    for j, (rot, qs) in enumerate(sets):
        omega_eval = pow(shape.omega, rot, r) if rot >= 0 else pow(omega_inv, -rot, r)
        z = omega_eval * x % r
        wi = d["W"][j]
        Ws.append(wi)
        ZWs.append(curve.mul(z, wi))
        eval_multi = eval_multi * u % r
        cb = _resolve(curve, shape, pf, qs[0][0], H)
        eb = qs[0][2]
        for ref, _, ev in qs[1:]:
            cb = curve.mul(v, cb)
            eb = eb * v % r
            cb = madd(cb, _resolve(curve, shape, pf, ref, H))
            eb = (eb + ev) % r
        Fs.append(cb)
        eval_multi = (eval_multi + eb) % r

    def horner(pts):
        acc = pts[0]
        for p_ in pts[1:]:
            acc = madd(curve.mul(u, acc), p_)
        return acc

    w, zw, f = horner(Ws), horner(ZWs), horner(Fs)
    e = curve.mul((-eval_multi) % r, g1)
    return w, zw, f, e, h_eval


def accumulate_msm(curve, shape, pf, g1=None):
    """Closed form of the same accumulator: per-point coefficients
    (u^{S-1-j} v^{m_j-1-i}, H expanded as sum h_i xn^i) and one MSM per output."""
    r = curve.r
    g1 = g1 or curve.gen
    d = _split(shape, pf)
    theta, beta, gamma, y, x, v, u = pf.challenges
    _, xn, h_eval = scalar_block(curve, shape, d, pf.challenges)
    sets = construct_intermediate_sets(build_queries(shape, d, h_eval))
    S = len(sets)
    coef = {}
    ev = 0
    wco, zco = [], []
    for j, (rot, qs) in enumerate(sets):
        uj = pow(u, S - 1 - j, r)
        m = len(qs)
        for i, (ref, _, e_) in enumerate(qs):
            c = uj * pow(v, m - 1 - i, r) % r
            ev = (ev + c * e_) % r
            coef[ref] = (coef.get(ref, 0) + c) % r
        wco.append(uj)
        z = pow(shape.omega, rot, r) * x % r if rot >= 0 else pow(pow(shape.omega, -1, r), -rot, r) * x % r
        zco.append(uj * z % r)
    terms = []
    for ref, c in coef.items():
        if ref == H_POINT:
            xp = 1
            for hc in d["h"]:
                terms.append((c * xp % r, hc))
                xp = xp * xn % r
        else:
            terms.append((c, _resolve(curve, shape, pf, ref, None)))
    f = curve.msm_naive([c for c, _ in terms], [p_ for _, p_ in terms])
    w = curve.msm_naive(wco, d["W"])
    zw = curve.msm_naive(zco, d["W"])
    e = curve.mul((-ev) % r, g1)
    return w, zw, f, e, h_eval


# ------------------------------------------------------- synthetic proofs
def synth_point(curve, seed, i):
    return curve.mul(P.synth_base_dlog(curve, seed, i), curve.gen)


def synth_vk_points(curve, shape, seed=0x7EC):
    shape.fixed_commitments = [synth_point(curve, seed, i) for i in range(shape.num_fixed_columns)]
    shape.sigma_commitments = [synth_point(curve, seed, 1000 + i) for i in range(len(shape.perm_columns))]
    return shape


def synth_proof(curve, shape, seed, b):
    """Shape-conformant random proof b: points [a]G, scalars / challenges
    uniform in [0, r)."""
    r = curve.r
    npts, nsc = shape.points_per_proof(), shape.scalars_per_proof()
    base = b * 4096
    pts = [synth_point(curve, seed, base + i) for i in range(npts)]
    scs = [P.synth_scalar(seed ^ 0x5CA1A, base + i, r) for i in range(nsc)]
    ch = [P.synth_scalar(seed ^ 0xC4A1, base + i, r) for i in range(7)]
    return Proof(points=pts, scalars=scs, challenges=ch)


# ----------------------------------------------------------- limb packing
def pack_proofs(curve, shape, proofs):
    """-> (points (B, npts, 8) u64, scalars (B, nsc, 4) u64, challenges
    (B, 7, 4) u64), Montgomery limbs like the Rust in-memory types."""
    import numpy as np
    r = curve.r
    pts = np.array([[P.point_to_limbs(curve, q) for q in pf.points] for pf in proofs], dtype=np.uint64)
    scs = np.array([[P.to_limbs(s * P.R_MONT % r) for s in pf.scalars] for pf in proofs],
                   dtype=np.uint64).reshape(len(proofs), shape.scalars_per_proof(), 4)
    chs = np.array([[P.to_limbs(s * P.R_MONT % r) for s in pf.challenges] for pf in proofs], dtype=np.uint64)
    return pts.reshape(len(proofs), shape.points_per_proof(), 8), scs, chs


def pack_result(curve, res):
    import numpy as np
    w, zw, f, e, h = res
    quad = np.array([P.point_to_limbs(curve, q) for q in (w, zw, f, e)], dtype=np.uint64)
    return quad, np.array(P.to_limbs(h * P.R_MONT % curve.r), dtype=np.uint64)


def to_limbs_mont(curve_r, v):
    return P.to_limbs(v * P.R_MONT % curve_r)


def rich_shape(curve, log_n):
    """A second, deliberately irregular synthetic shape that exercises every
    code path of the accumulator: 2 instance / 3 advice / 3 fixed columns,
    rotations -2..2, constants and Scaled nodes, 2 lookups (flattened
    expression lists, lookup.rs:214-243), 7 permutation columns in chunks of
    3 (3 permutation sets), 3 blinding factors, 3 quotient pieces."""
    r = curve.r
    inst_q = [(0, 0), (1, 0), (1, -2)]
    adv_q = [(0, 0), (1, 0), (2, 0), (0, 1), (2, -1), (1, 2)]
    fixed_q = [(0, 0), (1, 0), (2, 1)]
    gates = [
        Prod(Fixed(0), Sum(Prod(Advice(0), Advice(1)), Neg(Advice(3)))),
        Sum(Scaled(Prod(Advice(2), Instance(2)), 7), Neg(Const(r - 3))),
        Prod(Sum(Fixed(2), Const(5)), Sum(Advice(4), Neg(Scaled(Advice(5), 11)))),
    ]
    lk_in = [Prod(Fixed(1), Advice(0)), Sum(Advice(2), Instance(0))]
    lk_tab = [Fixed(1), Scaled(Fixed(2), 3)]
    perm_cols = [(KIND_INSTANCE, 0), (KIND_INSTANCE, 1), (KIND_FIXED, 0), (KIND_ADVICE, 0), (KIND_ADVICE, 1),
                 (KIND_ADVICE, 2), (KIND_FIXED, 1)]
    return ProofShape(log_n=log_n, blinding_factors=3, num_instance_columns=2, num_advice_columns=3,
                      num_fixed_columns=3, num_lookups=2, perm_chunk_len=3, quotient_degree=3,
                      instance_queries=inst_q, advice_queries=adv_q, fixed_queries=fixed_q,
                      perm_columns=perm_cols, gates=gates, lookup_inputs=lk_in, lookup_tables=lk_tab,
                      omega=domain_omega(r, log_n), delta=field_delta(r))
