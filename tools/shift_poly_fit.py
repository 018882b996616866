"""Minimax-style (weighted least squares on Chebyshev nodes, mpmath) fits of sin(d) and
cos(d) - 1 on |d| <= D for the short shift polynomials of geodesic.hip (sincos_shift).
Usage: python tools/shift_poly_fit.py 0.0625  -> coefficients (double) and max abs error."""
import mpmath as mp
mp.mp.dps = 50
D = mp.mpf('0.0625')   # fit interval |delta| <= D (slightly above the 0.05 used, margin)
import sys
if len(sys.argv) > 1: D = mp.mpf(sys.argv[1])
N = 400
# Chebyshev points in delta over (0, D]
pts = [D * (1 + mp.cos(mp.pi * (2*k+1) / (2*N))) / 2 for k in range(N)]
pts = [p for p in pts if p > D*mp.mpf('1e-6')]
def lsq(rows, rhs, w):
    A = mp.matrix([[r*wi for r in row] for row, wi in zip(rows, w)])
    b = mp.matrix([v*wi for v, wi in zip(rhs, w)])
    return mp.lu_solve(A.T*A, A.T*b)
def fit_sin(n):
    # sin d = d + d^3 * (S1 + S2 z + ... ), minimise abs error; weight d^3
    rows = [[p**(2*j) for j in range(n)] for p in pts]
    rhs = [(mp.sin(p) - p) / p**3 for p in pts]
    w = [p**3 for p in pts]
    return lsq(rows, rhs, w)
def fit_cos(n):
    # cos d - 1 = -z/2 + z^2 (C1 + C2 z + ...); weight d^4
    rows = [[p**(2*j) for j in range(n)] for p in pts]
    rhs = [(mp.cos(p) - 1 + p**2/2) / p**4 for p in pts]
    w = [p**4 for p in pts]
    return lsq(rows, rhs, w)
for n in (2, 3):
    S = fit_sin(n); C = fit_cos(n)
    Sd = [float(x) for x in S]; Cd = [float(x) for x in C]
    # max abs error with double coefficients (exact arithmetic)
    es = ec = 0
    for k in range(2001):
        d = D * k / 2000
        z = d*d
        ps = sum(mp.mpf(Sd[j]) * z**j for j in range(n))
        pc = sum(mp.mpf(Cd[j]) * z**j for j in range(n))
        es = max(es, abs(d + d**3*ps - mp.sin(d)))
        ec = max(ec, abs(-z/2 + z*z*pc - (mp.cos(d)-1)))
    print(n, 'sin', [repr(x) for x in Sd], mp.nstr(es, 3))
    print(n, 'cos', [repr(x) for x in Cd], mp.nstr(ec, 3))
