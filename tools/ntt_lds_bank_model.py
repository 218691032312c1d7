"""Bank model of the NTT LDS access patterns (csrc/ntt_kernels.hpp: the
fused load of ntt_load_first, the radix-4 rounds of lds_ntt4, the fused or
plain store) for candidate XOR swizzles: conflict degree per wave
instruction, 64 banks of 4 B, summed over the (logL, logC, lanes-walk-m)
shapes of the 2^20 / 2^22 two-pass and 2^23-2^25 three-pass forms.  Picked
lds_swz = x2,5,6.  Usage: python tools/ntt_lds_bank_model.py"""
def brev(x, bits): return int(format(x, f'0{bits}b')[::-1], 2) if bits else 0
def waves(total):
    for w0 in range(0, total, 64):
        yield range(w0, min(total, w0 + 64))
def patterns(logL, logC, kfast, fuse_last=True):
    L, C = 1 << logL, 1 << logC
    plane = L * C; pats = []
    # fused load
    if logL & 1:
        nm = L >> 1; t0 = 1
        for w in waves(plane >> 1):
            cols = [[], []]
            for b in w:
                m, c = (b & (nm - 1), b >> (logL - 1)) if kfast else (b >> logC, b & (C - 1))
                pos = brev(m, logL)
                for q in range(2): cols[q].append(((pos + q) << logC) | c)
            pats += [('ld', x) for x in cols]
    else:
        nm = L >> 2; t0 = 2
        for w in waves(plane >> 2):
            cols = [[], [], [], []]
            for b in w:
                m, c = (b & (nm - 1), b >> (logL - 2)) if kfast else (b >> logC, b & (C - 1))
                pos = brev(m, logL)
                for q in range(4): cols[q].append(((pos + q) << logC) | c)
            pats += [('ld', x) for x in cols]
    t = t0
    fuse = fuse_last and logL - 2 >= t0 and logL >= 3
    while t + 1 < logL and not (fuse and t == logL - 2):
        h = 1 << t
        for w in waves(plane >> 2):
            cols = [[], [], [], []]
            for b in w:
                c, bb = b & (C - 1), b >> logC
                lo = bb & (h - 1); j = ((bb >> t) << (t + 2)) | lo
                for q in range(4): cols[q].append(((j + q * h) << logC) | c)
            pats += [('r4', x) for x in cols] * 2  # read + write
        t += 2
    if fuse:
        h = L >> 2
        for w in waves(plane >> 2):
            cols = [[], [], [], []]
            for b in w:
                c, j = b & (C - 1), b >> logC
                for q in range(4): cols[q].append(((j + q * h) << logC) | c)
            pats += [('st', x) for x in cols]
    else:
        for w in waves(plane): pats.append(('st', list(w)))
    return pats
def cost(pats, f, NB=64):
    tot = {}
    for kind, idx in pats:
        banks = {}
        for a in set(f(i) for i in idx): banks.setdefault(a % NB, set()).add(a)
        tot[kind] = tot.get(kind, 0) + max([len(v) for v in banks.values()] or [0])
    return tot
cfgs = [(10, 1, False), (10, 1, True), (11, 0, False), (11, 0, True), (9, 2, False), (8, 2, False), (8, 2, True), (7, 2, True)]
allp = {c: patterns(*c) for c in cfgs}
cands = {'none': lambda i: i, 'x2,8': lambda i: i ^ (((i >> 2) ^ (i >> 8)) & 63)}
for s1 in range(1, 9):
    cands[f'x{s1}'] = (lambda s1: lambda i: i ^ ((i >> s1) & 63))(s1)
    for s2 in range(s1 + 1, 12):
        cands[f'x{s1},{s2}'] = (lambda s1, s2: lambda i: i ^ (((i >> s1) ^ (i >> s2)) & 63))(s1, s2)
        for s3 in range(s2 + 1, 12):
            cands[f'x{s1},{s2},{s3}'] = (lambda s1, s2, s3: lambda i: i ^ (((i >> s1) ^ (i >> s2) ^ (i >> s3)) & 63))(s1, s2, s3)
res = sorted((sum(sum(cost(allp[c], f).values()) for c in cfgs), n) for n, f in cands.items())
print(res[:6]); print([r for r in res if r[1] in ('none', 'x2,8')])
for n in (res[0][1], 'x2,8'):
    for c in cfgs: print(n, c, cost(allp[c], cands[n]))
