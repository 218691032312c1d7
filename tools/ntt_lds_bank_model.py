"""Bank model of the NTT LDS access patterns (csrc/ntt_kernels.hpp: load
phase, radix-2 / radix-4 rounds, store phase) for candidate index swizzles:
conflict degree per wave instruction, 64 banks of 4 B.  Picked lds_swz
(x2,8).  Usage: python tools/ntt_lds_bank_model.py"""
import itertools
def brev(x, bits): return int(format(x, f'0{bits}b')[::-1], 2) if bits else 0
def patterns(logL, logC, T=256):
    plane = 1 << (logL + logC); cmask = (1 << logC) - 1
    pats = []
    # load phase (cols-like): e -> brev(i1) << logC | c
    for m in range(0, plane, T):
        for w in range(0, T, 64):
            idx = []
            for lane in range(64):
                e = m + w + lane
                if e >= plane: continue
                i1, c = e >> logC, e & cmask
                idx.append((brev(i1, logL) << logC) | c)
            pats.append(('ld', idx))
    # rows-like load: r = e >> logL, i2 = e & (L-1): idx = brev(i2) << logR | r
    for m in range(0, plane, T):
        for w in range(0, T, 64):
            idx = []
            for lane in range(64):
                e = m + w + lane
                r, i2 = e >> logL, e & ((1 << logL) - 1)
                idx.append((brev(i2, logL) << logC) | r)
            pats.append(('ldrow', idx))
    t = 0
    if logL & 1:
        for m in range(0, plane >> 1, T):
            for w in range(0, T, 64):
                ia=[];ib=[]
                for lane in range(64):
                    b = m + w + lane
                    if b >= plane >> 1: continue
                    c, j = b & cmask, (b >> logC) << 1
                    ia.append((j << logC) | c); ib.append(((j + 1) << logC) | c)
                pats += [('r2', ia), ('r2', ib)]
        t = 1
    while t + 1 < logL:
        h = 1 << t
        for m in range(0, plane >> 2, T):
            for w in range(0, T, 64):
                cols = [[], [], [], []]
                for lane in range(64):
                    b = m + w + lane
                    if b >= plane >> 2: continue
                    c, bb = b & cmask, b >> logC
                    lo = bb & (h - 1); j = ((bb >> t) << (t + 2)) | lo
                    for q in range(4): cols[q].append(((j + q * h) << logC) | c)
                pats += [('r4', x) for x in cols]
        t += 2
    # store phase contiguous
    for m in range(0, plane, T):
        for w in range(0, T, 64):
            pats.append(('st', [m + w + l for l in range(64) if m + w + l < plane]))
    return pats
def cost(pats, f, NB=64):
    tot = {}
    for kind, idx in pats:
        phys = [f(i) for i in idx]
        banks = {}
        for a in set(phys): banks.setdefault(a % NB, set()).add(a)
        deg = max([len(v) for v in banks.values()] or [0])
        tot[kind] = tot.get(kind, 0) + deg
    return tot
fs = {'none': lambda i: i, 'pad>>6': lambda i: i + (i >> 6), 'pad>>5': lambda i: i + (i >> 5), 'pad>>4': lambda i: i + (i >> 4),
      'pad>>3': lambda i: i + (i >> 3), 'xor': lambda i: i ^ ((i >> 6) & 63)}
for cfg in [(10, 1), (9, 2), (11, 0), (8, 2), (10, 0)]:
    pats = patterns(*cfg)
    for name, f in fs.items():
        c = cost(pats, f)
        print(cfg, name, c, sum(c.values()))
print('---- search')
cfgs = [(10, 1), (9, 2), (11, 0), (8, 2), (10, 0), (7, 0), (12, 0)]
allp = {cfg: patterns(*cfg) for cfg in cfgs}
cands = {}
for s1 in range(2, 9):
    cands[f'x{s1}'] = (lambda s1: lambda i: i ^ ((i >> s1) & 63))(s1)
    for s2 in range(s1 + 1, 11):
        cands[f'x{s1},{s2}'] = (lambda s1, s2: lambda i: i ^ (((i >> s1) ^ (i >> s2)) & 63))(s1, s2)
res = []
for name, f in cands.items():
    tot = sum(sum(cost(allp[c], f).values()) for c in cfgs)
    res.append((tot, name))
res.sort()
print(res[:8], 'none', sum(sum(cost(allp[c], lambda i: i).values()) for c in cfgs), 'x6', [r for r in res if r[1]=='x6'])
best = res[0][1]
for c in cfgs: print(c, best, cost(allp[c], cands[best]))
