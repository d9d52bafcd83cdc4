"""include/eslam_detmath.h (host build via the oracle) against independent references:
mpmath (60 digits) for the transcendentals, published Philox4x32-10 known-answer vectors,
a direct minstd recurrence, and Python's exact integers for the fixed-point helpers."""
import ctypes as C
import math
import struct
from fractions import Fraction

import mpmath as mp
import numpy as np
import pytest

mp.mp.dps = 40


def ulp_err(got, want):
    want = float(want)
    if want == 0.0:
        return abs(got)
    return abs(got - want) / math.ulp(abs(want))


@pytest.fixture(scope="module")
def dm(oracle):
    return oracle.dm


def _rng():
    return np.random.default_rng(12345)


def test_exp(dm):
    xs = np.concatenate([_rng().uniform(-700, 700, 2000), _rng().uniform(-1, 1, 2000), [0.0, 1.0, -1.0, 709.7, -744.0]])
    worst = max(ulp_err(dm(0, float(x)), mp.exp(mp.mpf(float(x)))) for x in xs if x > -708)
    assert worst <= 2.0
    assert dm(0, 710.0) == math.inf
    assert dm(0, -746.0) == 0.0
    assert math.isnan(dm(0, float("nan")))
    # gradual underflow is rounded once
    for x in (-709.0, -720.0, -740.0, -745.0):
        assert dm(0, x) == pytest.approx(float(mp.exp(x)), rel=1e-12 if x > -735 else 1e-3)


def test_log(dm):
    xs = np.concatenate([np.exp(_rng().uniform(-700, 700, 2000)), _rng().uniform(0.5, 2, 2000), [1.0, 2.0, 5e-324, 1e-310]])
    worst = max(ulp_err(dm(1, float(x)), mp.log(mp.mpf(float(x)))) for x in xs)
    assert worst <= 2.0
    assert dm(1, 0.0) == -math.inf
    assert math.isnan(dm(1, -1.0))


@pytest.mark.parametrize("fn,ref", [(2, mp.sin), (3, mp.cos)])
def test_sincos(dm, fn, ref):
    xs = np.concatenate([_rng().uniform(-10, 10, 3000), _rng().uniform(-2000, 2000, 1000), [0.0, math.pi, math.pi / 2]])
    worst_abs = max(abs(dm(fn, float(x)) - float(ref(mp.mpf(float(x))))) for x in xs)
    assert worst_abs <= 4.5e-16


@pytest.mark.parametrize("fn,ref", [(13, mp.sin), (14, mp.cos)])
def test_sincos2pi(dm, fn, ref):
    """sin/cos(2 pi u) of the Box-Muller angle, u = (a + 1/2) 2^-32 (dm_box_muller32)."""
    a = _rng().integers(0, 2 ** 32, 4000, dtype=np.uint64)
    us = np.concatenate([(a.astype(np.float64) + 0.5) * 2.0 ** -32, [0.125, 0.25, 0.5, 0.75, 0.999]])
    worst_abs = max(abs(dm(fn, float(u)) - float(ref(2 * mp.pi * mp.mpf(float(u))))) for u in us)
    assert worst_abs <= 4.5e-16


def test_box_muller32_moments(oracle):
    """Normals of the 32-bit Box-Muller draw layout: mean 0, variance 1, symmetric."""
    z = []
    for g in range(20000):
        out = (C.c_uint32 * 4)()
        oracle.lib().or_dm_philox(42, 1, 0, g, 0, out)
        u1 = (out[0] + 0.5) * 2.0 ** -32
        u2 = (out[1] + 0.5) * 2.0 ** -32
        r = math.sqrt(-2.0 * math.log(u1))
        z.append(r * math.cos(2 * math.pi * u2))
    z = np.array(z)
    assert abs(z.mean()) < 0.03 and abs(z.var() - 1.0) < 0.04 and abs(np.mean(z ** 3)) < 0.08


def test_erfc(dm):
    xs = np.concatenate([_rng().uniform(-6, 27, 4000), _rng().uniform(-0.5, 0.5, 1000), [0.0, 0.5, 1.5, 3.0, 5.0, 26.5]])
    for x in xs:
        want = mp.erfc(mp.mpf(float(x)))
        got = dm(4, float(x))
        assert abs(got - float(want)) <= 2e-15 * abs(float(want)) + 1e-300, x


def test_normal_pdf_cdf_ratio(dm):
    """boost::math pdf(N(0,s),z)/cdf(N(0,s),z) (src/ContactModel.cpp:104-115)."""
    r = _rng()
    for _ in range(3000):
        s = float(10 ** r.uniform(-3, 3))
        z = float(r.uniform(-9, 9) * s)
        zz, ss = mp.mpf(z), mp.mpf(s)
        pdf = mp.exp(-zz * zz / (2 * ss * ss)) / (ss * mp.sqrt(2 * mp.pi))
        cdf = mp.erfc(-zz / (ss * mp.sqrt(2))) / 2
        want = float(pdf / cdf)
        assert dm(7, z, s) == pytest.approx(want, rel=5e-15)


def test_pow(dm):
    r = _rng()
    for _ in range(2000):
        x = float(r.uniform(0, 1.5))
        for k in (0, 1, 2, 3, 4):
            assert dm(8, x, float(k)) == float(mp.power(mp.mpf(x), k))   # correctly rounded
        y = 1.0 / int(r.integers(1, 9))
        assert dm(8, x, y) == pytest.approx(float(mp.power(mp.mpf(x), y)), rel=4e-16)
    # size_t wrap of 4 - cpoints.size() (src/PoseEstimator.cpp:336)
    big = float(2 ** 64 - 1)
    assert dm(8, 0.9, big) == 0.0 and dm(8, 1.0, big) == 1.0 and dm(8, 1.1, big) == math.inf
    assert dm(8, 0.81, 0.5) == math.sqrt(0.81)


def test_weighting_function(dm):
    # src/PoseEstimator.cpp:114-128 with alpha 0, gamma 0
    assert dm(12, -0.1, 0.9) == 1.0
    assert dm(12, 0.0, 0.9) == 1.0
    assert dm(12, 0.45, 0.9) == pytest.approx(0.5)
    assert dm(12, 0.9, 0.9) == 0.0
    assert dm(12, float("nan"), 0.9) == 0.0


def test_philox_kat(oracle):
    """Random123 known-answer vectors for philox4x32_10."""
    L = oracle.lib()
    cases = [
        ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
        ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
        ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
         (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
    ]
    for ctr, key, want in cases:
        out = (C.c_uint32 * 4)()
        L.or_dm_philox_raw((C.c_uint32 * 4)(*ctr), key[0], key[1], out)
        assert tuple(out) == want


def test_minstd_jump(oracle):
    L = oracle.lib()
    x = 42
    seq = []
    for _ in range(5000):
        x = x * 48271 % 2147483647
        seq.append(x)
    for n in (1, 2, 17, 999, 5000):
        assert L.or_dm_minstd_jump(42, n) == seq[n - 1]
    # the 10000th value of minstd_rand seeded with 1 is 399268537 (C++11 [rand.predef])
    assert L.or_dm_minstd_jump(1, 10000) == 399268537


def test_fixed_point_roundtrip(oracle):
    L = oracle.lib()
    r = _rng()
    for _ in range(300):
        vals = [float(v) for v in 10 ** r.uniform(-30, 0, int(r.integers(1, 50)))]
        scale = 112
        limbs = [0, 0, 0, 0]
        exact = 0
        for v in vals:
            out = (C.c_uint32 * 4)()
            L.or_dm_fx128(v, scale, out)
            t = sum(int(out[j]) << (32 * j) for j in range(4))
            assert t == int(Fraction(v) * 2 ** scale)        # truncation
            exact += t
            for j in range(4):
                limbs[j] += int(out[j])
        got = L.or_dm_limbs_to_double((C.c_uint64 * 4)(*limbs), scale)
        assert got == float(Fraction(exact, 2 ** scale))      # correctly rounded


def test_fx61(dm):
    def fx(v):
        return struct.unpack("<Q", struct.pack("<d", dm(9, v)))[0]
    assert fx(0.0) == 0 and fx(-1.0) == 0 and fx(float("nan")) == 0
    assert fx(1.0) == 2 ** 61
    assert fx(0.5) == 2 ** 60
    assert fx(1e-300) == 0
    v = 0.123456789
    assert fx(v) == int(Fraction(v) * 2 ** 61)
    assert fx(3.0) == 2 ** 62 - 1


def _check_div_bin(tmp_path_factory):
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path_factory.mktemp("checkdiv") / "check_div")
    subprocess.run(["gcc", "-O2", "-std=c11", "-mfma", "-ffp-contract=off", "-I" + os.path.join(root, "include"),
                    os.path.join(root, "tests", "c", "check_div.c"), "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("mode,arg", [("uniform", "61"), ("draws", "2000000")])
def test_div_recip_equals_division(tmp_path_factory, mode, arg):
    """dm_div_recip (the device's division-free a/b for per-step constant b) equals IEEE a/b.
    The uniform mode also ran with stride 1 (all 2^31 - 1 minstd states, 0 mismatches) and the
    draws mode with 5e8 cases; here a sample keeps the suite fast."""
    import subprocess
    out = subprocess.run([_check_div_bin(tmp_path_factory), mode, arg], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert " 0 mismatches" in out.stdout


def test_log_bm(dm):
    """the Box-Muller log (dm_log_bm: 128-interval table + log1p series) against mpmath over
    the uniform words' range, both ends and the interval boundaries included"""
    a = _rng().integers(0, 2 ** 32, 6000, dtype=np.uint64)
    us = list((a.astype(np.float64) + 0.5) * 2.0 ** -32)
    us += [2.0 ** -33, (2.0 ** 32 - 0.5) * 2.0 ** -32, 0.5, 0.75, 0.99609375, 1.0 - 2.0 ** -40]
    us += [0.75 + i / 256 for i in range(64)] + [0.5 * (1 + i / 128) for i in range(64)]
    worst = max(ulp_err(dm(15, float(u)), mp.log(mp.mpf(float(u)))) for u in us)
    assert worst <= 2.0


@pytest.mark.parametrize("fn,ref", [(16, mp.sin), (17, mp.cos)])
def test_sincos2pi32(dm, fn, ref):
    """sin/cos of the Box-Muller angle 2 pi (b + 1/2) 2^-32 from the 32-bit word (dm_sincos2pi32:
    256-entry table + Taylor series + angle sums) against mpmath"""
    b = list(_rng().integers(0, 2 ** 32, 6000, dtype=np.uint64)) + [0, 2 ** 32 - 1, 2 ** 30, 2 ** 31, 3 * 2 ** 30, 2 ** 24 - 1]
    worst_abs = max(abs(dm(fn, float(x)) - float(ref(2 * mp.pi * (mp.mpf(int(x)) + mp.mpf(0.5)) / 2 ** 32))) for x in b)
    assert worst_abs <= 3.5e-16


@pytest.mark.parametrize("fn,ref", [(26, mp.sin), (27, mp.cos)])
def test_sincos2pi32f(dm, fn, ref):
    """the fp32 Box-Muller angle (dm_sincos2pi32f: fp32 table + Taylor series + angle sums)
    against mpmath: within 1.5 fp32 ulps of 1 (the values lie in [-1, 1])"""
    b = list(_rng().integers(0, 2 ** 32, 6000, dtype=np.uint64)) + [0, 2 ** 32 - 1, 2 ** 30, 2 ** 31, 3 * 2 ** 30, 2 ** 24 - 1]
    worst_abs = max(abs(dm(fn, float(x)) - float(ref(2 * mp.pi * (mp.mpf(int(x)) + mp.mpf(0.5)) / 2 ** 32))) for x in b)
    assert worst_abs <= 1.5 * 2.0 ** -24


def test_box_muller32_normals(dm):
    """the contract's Box-Muller pair from two words against the same formula in mpmath: the
    fp32 radius and angle (dm_box_muller32) keep each normal within 2^-22 of the radius"""
    rng = _rng()
    for a, b in zip(rng.integers(0, 2 ** 32, 2000), rng.integers(0, 2 ** 32, 2000)):
        u = (mp.mpf(int(a)) + mp.mpf(0.5)) / 2 ** 32
        t = 2 * mp.pi * (mp.mpf(int(b)) + mp.mpf(0.5)) / 2 ** 32
        r = mp.sqrt(-2 * mp.log(u))
        for fn, want in ((18, r * mp.cos(t)), (19, r * mp.sin(t))):
            got = dm(fn, float(a), float(b))
            assert abs(got - float(want)) <= 2.0 ** -22 * max(1.0, float(r)), (a, b, fn)
