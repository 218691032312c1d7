"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the NTT (pm_fft*).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it.

Restates halo2's ``serial_fft`` / ``best_fft`` [3P: halo2 arithmetic.rs,
branch kzg-agg2, not vendored]: bit-reverse the input in place, then radix-2
decimation-in-time butterflies with w_m = omega^(n / 2m), the twiddle advanced
by repeated multiplication (w *= w_m), exactly as the published source walks
it.  ``ifft`` is EvaluationDomain::ifft: best_fft with omega^-1, then every
element times the divisor 1/n.  The result is exact field arithmetic, so the
GPU's four-step factorisation must agree bit for bit.

PARITY STATUS: the reference holds no FFT vectors; the restatement is pinned
by the DFT definition itself (``dft`` below, O(n^2)), by the convolution
theorem and by the inverse round trip (tests/test_ntt_oracle.py).
"""
from __future__ import annotations


def bitreverse(x, bits):
    r = 0
    for _ in range(bits):
        r = (r << 1) | (x & 1)
        x >>= 1
    return r


def serial_fft(a, omega, log_n, r):
    """In place; a is a list of ints mod r (halo2 serial_fft)."""
    n = len(a)
    assert n == 1 << log_n
    for k in range(n):
        rk = bitreverse(k, log_n)
        if k < rk:
            a[k], a[rk] = a[rk], a[k]
    m = 1
    for _ in range(log_n):
        w_m = pow(omega, n // (2 * m), r)
        k = 0
        while k < n:
            w = 1
            for j in range(m):
                t = a[k + j + m] * w % r
                a[k + j + m] = (a[k + j] - t) % r
                a[k + j] = (a[k + j] + t) % r
                w = w * w_m % r
            k += 2 * m
        m *= 2
    return a


def ifft(a, omega, log_n, r):
    """EvaluationDomain::ifft: best_fft(omega^-1) then * n^-1."""
    serial_fft(a, pow(omega, -1, r), log_n, r)
    d = pow(1 << log_n, -1, r)
    for i in range(len(a)):
        a[i] = a[i] * d % r
    return a


def dft(a, omega, r):
    """O(n^2) definition: A_k = sum_j a_j omega^(jk)."""
    n = len(a)
    return [sum(a[j] * pow(omega, j * k % n, r) for j in range(n)) % r for k in range(n)]


def eval_at(a, omega, k, r):
    """One output A_k = sum_j a_j omega^(jk) in O(n) (Horner in omega^k)."""
    x = pow(omega, k, r)
    acc = 0
    for c in reversed(a):
        acc = (acc * x + c) % r
    return acc
