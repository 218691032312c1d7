"""Host-logic model of the HIP MSM pipeline (test helper).

Mirrors halo2-aggregation_amd/csrc/{capi.hip:make_plan, msm_kernels.hpp} step
by step, but over the additive group Z_r (a point is replaced by its discrete
log, point addition by integer addition mod r).  It lets the CPU test-suite
check the design's algebra -- signed digits, counting sort, slice ownership +
chain folds, segment / bit-decomposed bucket reduction and the window Horner --
independently of any curve arithmetic.
"""
from __future__ import annotations

import math


def bit_length(v):
    return int(v).bit_length()


def make_plan(n, c_override=0, chunk_override=0):
    lg = bit_length(max(n, 1)) - 1
    c = c_override if c_override > 0 else max(4, min(16, lg - 2 if lg >= 14 else lg - 4))
    c = max(4, min(20, c))
    W = (256 + c - 1) // c
    base, extra = 256 // W, 256 % W
    cmax = base + (1 if extra else 0)
    K = 1 << (cmax - 1)
    L1 = min(4, K)
    NB = ((K + 1 + L1 - 1) // L1) * L1
    M1 = K // L1  # segments cover slots [0, K); bucket K is a host term of its own
    NB2 = bit_length(M1 - 1)
    work = n * W  # one window group (capi.hip make_plan)
    target = 256 * 1024
    chunk = max(16, (work + target - 1) // target)
    if chunk_override:
        chunk = chunk_override
    nthreads = (work + chunk - 1) // chunk
    widths = [base + (1 if w < extra else 0) for w in range(W)]
    return dict(c=c, W=W, widths=widths, K=K, L1=L1, log2L1=L1.bit_length() - 1, NB=NB, M1=M1, NB2=NB2, chunk=chunk,
                nthreads=nthreads, cmax=cmax)


def window_widths(W):
    base, extra = 256 // W, 256 % W
    return [base + (1 if w < extra else 0) for w in range(W)]


def digits(s, W):
    """k_digits: signed digits of canonical scalar s over the W balanced
    windows (WinGeom) -> list of (|d|, neg)."""
    out = []
    carry = 0
    off = 0
    for w, c in enumerate(window_widths(W)):
        raw = (s >> off) & ((1 << c) - 1)
        off += c
        d = raw + carry
        neg = 0
        if w != W - 1 and d > (1 << (c - 1)):
            d = (1 << c) - d
            neg, carry = 1, 1
        else:
            carry = 0
        out.append((d, neg))
    return out


K_TJOBS = 2  # msm_kernels.hpp kTJobs


def msm_model(scalars, dlogs, r, c_override=0, chunk_override=0):
    n = len(scalars)
    if n == 0:
        return 0
    pl = make_plan(n, c_override, chunk_override)
    c, W, NB, L1, M1, NB2 = pl["c"], pl["W"], pl["NB"], pl["L1"], pl["M1"], pl["NB2"]
    TOT = W * NB + 1
    counts = [0] * TOT
    dig = [digits(s, W) for s in scalars]
    for i in range(n):
        for w, (d, _) in enumerate(dig[i]):
            assert d <= pl["K"]
            if d:
                counts[w * NB + d] += 1
    offsets, run = [], 0
    for x in counts:
        offsets.append(run)
        run += x
    cursor = list(offsets)
    total = offsets[-1]
    sorted_ = [None] * total
    for w in range(W):  # scatter (any order inside a bucket is valid)
        for i in range(n):
            d, neg = dig[i][w]
            if d:
                sorted_[cursor[w * NB + d]] = (i, neg)
                cursor[w * NB + d] += 1
    nslots = TOT - 1

    def find_bucket(lo, hi, pos):
        while hi - lo > 1:
            mid = (lo + hi) // 2
            if offsets[mid] <= pos:
                lo = mid
            else:
                hi = mid
        return lo

    buckets = [0] * nslots
    chunk = pl["chunk"]
    s1 = W * NB
    head = [0] * pl["nthreads"]
    for t in range(pl["nthreads"]):  # k_accumulate (one launch over every window)
        start = t * chunk
        if start >= total:
            continue
        end = min(start + chunk, total)
        gb = find_bucket(0, s1, start)
        bend = offsets[gb + 1]
        owned = offsets[gb] == start
        acc = 0
        for p in range(start, end):
            if p == bend:
                if owned:
                    buckets[gb] = acc
                else:
                    head[t] = acc
                acc = 0
                gb += 1
                while offsets[gb + 1] <= p:
                    gb += 1
                bend = offsets[gb + 1]
                owned = True
            i, neg = sorted_[p]
            acc = (acc + (-dlogs[i] if neg else dlogs[i])) % r
        if owned:
            buckets[gb] = acc
        else:
            head[t] = acc

    def folded(slot):  # k_bucket_seg_q: the bucket plus its slice-boundary chain
        bs, be = offsets[slot], offsets[slot + 1]
        if bs == be:
            return 0
        tf, tl = bs // chunk, min((be - 1) // chunk, pl["nthreads"] - 1)
        return (buckets[slot] + sum(head[tf + 1:tl + 1])) % r  # serial or wave-wide: same sum

    S = [0] * (W * M1)
    T = [0] * (W * M1)
    for w in range(W):  # k_bucket_seg_q: S = B0 + .. + B3, T = B1 + 2 B2 + 3 B3
        for j in range(M1):
            Bq = [folded(w * NB + j * L1 + q) for q in range(L1)]
            S[w * M1 + j] = sum(Bq) % r
            T[w * M1 + j] = sum(q * Bq[q] for q in range(L1)) % r
    widths = pl["widths"]
    at = {}
    for w in range(W):  # k_bucket_bits -> host Horner over absolute bit positions
        G = [sum(S[w * M1 + j] for j in range(M1) if (j >> b) & 1) % r for b in range(NB2)]
        per = (M1 + K_TJOBS - 1) // K_TJOBS
        Tp = [sum(T[w * M1 + j0:w * M1 + min(M1, j0 + per)]) % r for j0 in range(0, K_TJOBS * per, per)]
        bK = folded(w * NB + M1 * L1)  # the top bucket K (segment 0's slot-0 lane)
        o = sum(widths[:w])
        for b in range(NB2):
            at.setdefault(o + b + pl["log2L1"], []).append(G[b])
        at.setdefault(o, []).extend(Tp)
        at.setdefault(o + pl["cmax"] - 1, []).append(bK)
    acc = 0
    for q in range(max(at), -1, -1):
        acc = 2 * acc % r
        for v in at.get(q, []):
            acc = (acc + v) % r
    return acc


def halo2_window(n):
    """halo2 multiexp_serial window width (for documentation / comparison)."""
    return 1 if n < 4 else (3 if n < 32 else int(math.ceil(math.log(n))))


def sort_model(dig, n, W, K, cmax, NB, sort_b=2048):
    """Two-level LDS bucket sort (k_sort_hist / k_scan / k_sort_coarse /
    k_sort_fine) -> (offsets, sorted entries as (i, neg))."""
    FB = max(0, cmax - 1 - 8)
    NCB = (K >> FB) + 1
    nblk = (n + sort_b - 1) // sort_b
    bh = [0] * (W * NCB * nblk + 1)
    for blk in range(nblk):
        for i in range(blk * sort_b, min(n, (blk + 1) * sort_b)):
            for w in range(W):
                d, _ = dig[i][w]
                if d:
                    bh[(w * NCB + (d >> FB)) * nblk + blk] += 1
    bofs, run = [], 0
    for x in bh:
        bofs.append(run)
        run += x
    total = bofs[-1]
    mid = [None] * total
    for blk in range(nblk):
        for w in range(W):
            cur = {}
            for i in range(blk * sort_b, min(n, (blk + 1) * sort_b)):
                d, neg = dig[i][w]
                if d:
                    cb = d >> FB
                    k = cur.get(cb, 0)
                    mid[bofs[(w * NCB + cb) * nblk + blk] + k] = (d, i, neg)
                    cur[cb] = k + 1
    offsets = [None] * (W * NB + 1)
    sorted_ = [None] * total
    nf = 1 << FB
    for seg in range(W * NCB):
        w, cb = divmod(seg, NCB)
        s0, s1 = bofs[seg * nblk], bofs[(seg + 1) * nblk]
        hist = [0] * nf
        for e in range(s0, s1):
            hist[mid[e][0] & (nf - 1)] += 1
        run = s0
        cursor = []
        for k in range(nf):
            slot = (cb << FB) + k
            if slot < NB:
                offsets[w * NB + slot] = run
            cursor.append(run)
            run += hist[k]
        if cb == NCB - 1:
            for slot in range(NCB << FB, NB):
                offsets[w * NB + slot] = s1
            if w == W - 1:
                offsets[W * NB] = s1
        for e in range(s0, s1):
            d, i, neg = mid[e]
            f = d & (nf - 1)
            sorted_[cursor[f]] = (i, neg)
            cursor[f] += 1
    return offsets, sorted_
