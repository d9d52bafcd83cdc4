"""Minimax kernel polynomials of include/eslam_detmath.h (sin, cos, exp, log kernels).

Provenance: a Remez exchange in mpmath at 60 digits on the reduced ranges the header uses,
coefficients then rounded to double; the printed error is that of the rounded polynomial
(exact arithmetic), the Horner rounding comes on top.  Re-run to regenerate:
    python tools/gen_minimax.py

  sin  sin(r) = r - r z P(z),            P(z) = (1 - sin(sqrt z)/sqrt z) / z,   z = r^2 <= (pi/4)^2
  cos  cos(r) = 1 + z (-1/2 + z P(z)),   P(z) = (cos(sqrt z) - 1 + z/2) / z^2
  exp  e^r = 1 + r (1 + r (1/2 + r P(r))), P(r) = (e^r - 1 - r - r^2/2) / r^3, |r| <= ln2/2
  log  log(1+f) = f - s (f - z P(z)),    P(z) = 2 (atanh(sqrt z)/sqrt z - 1) / z,
       s = f / (2 + f), z = s^2 <= ((sqrt2 - 1)/(sqrt2 + 1))^2
"""
import mpmath as mp

mp.mp.dps = 60


def p_sin(z):
    if z == 0:
        return mp.mpf(1) / 6
    r = mp.sqrt(z)
    return (1 - mp.sin(r) / r) / z


def p_cos(z):
    if z == 0:
        return mp.mpf(1) / 24
    r = mp.sqrt(z)
    return (mp.cos(r) - 1 + z / 2) / (z * z)


def p_exp(r):
    if r == 0:
        return mp.mpf(1) / 6
    return (mp.exp(r) - 1 - r - r * r / 2) / (r ** 3)


def p_log(z):
    if z == 0:
        return mp.mpf(2) / 3
    s = mp.sqrt(z)
    return 2 * (mp.atanh(s) / s - 1) / z


def peval(c, x):                       # c: lowest degree first
    p = mp.mpf(0)
    for a in reversed(c):
        p = p * x + a
    return p


def remez(f, a, b, deg, iters=30, grid=4000, w=lambda x: 1):
    """minimise max |w(x) (f(x) - p(x))| over [a, b]"""
    a, b = mp.mpf(a), mp.mpf(b)
    n = deg + 2
    xs = [(a + b) / 2 - (b - a) / 2 * mp.cos(mp.pi * i / (n - 1)) for i in range(n)]
    samples = [a + (b - a) * i / grid for i in range(grid + 1)]
    c = None
    for _ in range(iters):
        A = mp.matrix(n, n)
        rhs = mp.matrix(n, 1)
        for i, x in enumerate(xs):
            for j in range(deg + 1):
                A[i, j] = x ** j
            A[i, deg + 1] = (-1) ** i / w(x)
            rhs[i] = f(x)
        sol = mp.lu_solve(A, rhs)
        c = [sol[j] for j in range(deg + 1)]
        err = [w(x) * (f(x) - peval(c, x)) for x in samples]
        # alternating extrema: local maxima of |err| with sign changes between them
        ext = [0]
        for i in range(1, grid):
            if abs(err[i]) >= abs(err[i - 1]) and abs(err[i]) >= abs(err[i + 1]):
                ext.append(i)
        ext.append(grid)
        merged = []
        for i in ext:
            if merged and mp.sign(err[i]) == mp.sign(err[merged[-1]]):
                if abs(err[i]) > abs(err[merged[-1]]):
                    merged[-1] = i
            else:
                merged.append(i)
        while len(merged) > n:        # drop the smaller end
            if abs(err[merged[0]]) < abs(err[merged[-1]]):
                merged.pop(0)
            else:
                merged.pop()
        if len(merged) < n:
            break
        xs = [samples[i] for i in merged]
    return c


def report(name, f, a, b, deg, scale=lambda x: 1):
    c = remez(f, a, b, deg, w=lambda x: scale(x) + mp.mpf('1e-40'))
    cd = [float(v) for v in c]
    xs = [mp.mpf(a) + (mp.mpf(b) - a) * i / 20000 for i in range(20001)]
    worst = max(abs((f(x) - peval([mp.mpf(v) for v in cd], x)) * scale(x)) for x in xs)
    print(f"/* {name}: degree {deg}, max |error x scale| of the rounded polynomial {mp.nstr(worst, 3)} */")
    print(", ".join(repr(v) for v in reversed(cd)))   # highest degree first (DM_POLY order)
    return cd


if __name__ == "__main__":
    zs = (mp.pi / 4) ** 2
    # scale: the polynomial error's contribution relative to the function value
    report("sin P(z)", p_sin, 0, zs, 5, scale=lambda z: z)
    report("cos P(z)", p_cos, 0, zs, 5, scale=lambda z: z * z / mp.cos(mp.sqrt(z)))
    h = mp.log(2) / 2 + mp.mpf("1e-6")
    report("exp P(r)", p_exp, -h, h, 9, scale=lambda r: abs(r) ** 3 / mp.exp(r))
    sm = (mp.sqrt(2) - 1) / (mp.sqrt(2) + 1)
    report("log P(z)", p_log, 0, sm * sm, 6, scale=lambda z: z * mp.sqrt(z) / (2 * mp.atanh(mp.sqrt(z)) + mp.mpf("1e-300")))
