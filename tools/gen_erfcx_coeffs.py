"""Generate the piecewise polynomial coefficients of erfcx(t) = exp(t^2) erfc(t), t >= 0,
used by include/eslam_detmath.h (dm_erfcx_pos).

Provenance: Chebyshev-economised least-max fits computed with mpmath at 60 digits
(mpmath.chebyfit), then rounded to double.  Re-run to regenerate:
    python tools/gen_erfcx_coeffs.py > /tmp/coeffs.txt
"""
import mpmath as mp

mp.mp.dps = 60


def erfcx(t):
    return mp.exp(t * t) * mp.erfc(t)


# intervals on t: polynomial in u = (t - mid) / half, u in [-1, 1]
INTERVALS = [(0.0, 0.5, 18), (0.5, 1.5, 20), (1.5, 3.0, 20), (3.0, 5.0, 20)]
TAIL_TMIN = 5.0
TAIL_DEG = 14


def fit(a, b, deg):
    mid = mp.mpf(a + b) / 2
    half = mp.mpf(b - a) / 2
    f = lambda u: erfcx(mid + half * u)
    poly, err = mp.chebyfit(f, [-1, 1], deg + 1, error=True)
    rel = err / f(1)
    return [float(c) for c in poly], float(rel), float(mid), float(half)


def fit_tail(deg):
    # t >= TAIL_TMIN: erfcx(t) = q(w) / (t sqrt(pi)),  w = 1/t^2 in (0, 1/TAIL_TMIN^2]
    def q(w):
        if w == 0:
            return mp.mpf(1)
        t = 1 / mp.sqrt(w)
        return erfcx(t) * t * mp.sqrt(mp.pi)
    wmax = 1 / mp.mpf(TAIL_TMIN) ** 2
    poly, err = mp.chebyfit(lambda u: q(wmax * (u + 1) / 2), [-1, 1], deg + 1, error=True)
    return [float(c) for c in poly], float(err), float(wmax)


if __name__ == "__main__":
    for (a, b, deg) in INTERVALS:
        poly, rel, mid, half = fit(a, b, deg)
        print(f"/* t in [{a}, {b}): mid {mid!r} half {half!r} deg {deg} max rel fit err {rel:.2e} */")
        print("{" + ", ".join(repr(c) for c in poly) + "},")
    poly, err, wmax = fit_tail(TAIL_DEG)
    print(f"/* tail: q(w), w = 1/t^2, u = 2 w / wmax - 1, wmax {wmax!r}, err {err:.2e} */")
    print("{" + ", ".join(repr(c) for c in poly) + "},")
