"""The kernels' shared-divisor quotients (rtpb_math.h make_rcp / div1 / div1_as / div3 / div3_norm) and square root
(tsqrt) are bit-identical to IEEE division and sqrt (NumPy's a / b, np.sqrt) on the GPU -- including the sign of zero -- on adversarial operands:
random bit patterns over the whole double range, operands straddling the fast-path range limits,
denormals, 0 / inf / NaN combinations, and realistic normalisation inputs (vector components over
their norm).  The end-to-end bit-exact traces (test_gpu_parity.py) cover the same code in context."""
import numpy as np
import pytest

import native_harness

pytestmark = pytest.mark.gpu


def _same(got, exp):
    """bitwise equal where exp is not NaN; NaN exactly where exp is NaN"""
    nan = np.isnan(exp)
    assert np.array_equal(np.isnan(got), nan)
    g, e = got[~nan].view(np.uint64), exp[~nan].view(np.uint64)
    bad = np.flatnonzero(g != e)
    assert bad.size == 0, f"{bad.size} mismatches, first: got {got[~nan][bad[:4]]} expected {exp[~nan][bad[:4]]}"


def _check(a, a2, a3, b, kill):
    out = native_harness.fastdiv_check(a, a2, a3, b, kill)
    with np.errstate(all="ignore"):
        _same(out[1], a / b)             # the device's own division is IEEE
        _same(out[0], a / b)             # div1
        _same(out[2], a / b)             # div3
        _same(out[3], a2 / b)
        _same(out[4], a3 / b)
        bb = np.where(kill.astype(bool), np.nan, b)
        _same(out[5], a / bb)            # div1_as
        _same(out[6], np.sqrt(b))        # tsqrt
        _same(out[7], np.sqrt(a))
        _same(out[8], a / b)             # div1 with the host's reciprocal (descriptor rR / rf)
        nrm = np.sqrt(a * a + a2 * a2 + a3 * a3)   # div3_norm: the vector over its own norm
        _same(out[19], a / nrm)
        _same(out[20], a2 / nrm)
        _same(out[21], a3 / nrm)
        # the sphere's root choice and Snell's np.sign(v) * root against the reference's own chains
        root = np.sqrt(np.abs(b))
        t1, t2 = 0.5 * (-a + root), 0.5 * (-a - root)          # RT:1497-1505 (oracle sphere_hit)
        t1 = np.where(t1 < 0, np.inf, t1)
        t2 = np.where(t2 < 0, np.inf, t2)
        t = np.minimum(t1, t2)
        _same(out[26], np.where(t == np.inf, np.nan, t))
        _same(out[38], np.sqrt(1.0 - a * a))                    # tsqrt_1m: Snell's / PerfectLens' sqrt(1 - m m)
        _same(out[27], np.sign(a) * root)                       # RT:1217
        # unit_or_zero (RT:1203-1209): NumPy's v / |v| with NaN components -> 0, through the combined norm
        # test (norm2_fast) or the full sequences
        nrm2 = np.sqrt(a * a + a2 * a2 + a3 * a3)
        for k, comp in enumerate((a, a2, a3)):
            exp = comp / nrm2
            _same(out[28 + k], np.where(np.isnan(exp), 0.0, exp))
            _same(out[35 + k], np.where(np.isnan(exp), 0.0, exp))    # unit_near1_or_zero: the same values
        _same(out[31], nrm2 * (2 * np.pi) / b)     # a norm's range needs no numerator test (RT:297 order)
        # the axial sphere normal (p - c) / R: no div_fixup for a finite nonzero R in the divisor range; its
        # numerators are finite and at most 2^513 wherever the row survives the on-surface test
        mb = np.abs(b)
        in_b = (mb >= 2.0 ** -120) & (mb < 2.0 ** 120)
        for k, comp in enumerate((a, a2, a3)):
            sel = in_b & np.isfinite(comp) & (np.abs(comp) <= 2.0 ** 513)
            _same(out[32 + k][sel], (comp / b)[sel])
        # GuardDefer: no fallback branch; where the flag is clear the value is the exact one, and the
        # flag is set only where an operand left the shortcut's exact range (the flagged rays are re-traced)
        for val, flag, exp in ((out[9], out[10], a / b), (out[11], out[14], a / b), (out[12], out[14], a2 / b),
                               (out[13], out[14], a3 / b), (out[15], out[16], np.sqrt(b)),
                               (out[17], out[18], a / bb), (out[22], out[25], a / nrm),
                               (out[23], out[25], a2 / nrm), (out[24], out[25], a3 / nrm)):
            ok = flag == 0
            _same(val[ok], exp[ok])
        return out


def _rand_bits(rng, n):
    return rng.integers(0, 2**64, size=n, dtype=np.uint64, endpoint=False).view(np.float64)


def _pow2_band(rng, n, lo, hi):
    """signed values m * 2^k, m in [1, 2), k uniform in [lo, hi] (denormals where k < -1022)"""
    k = rng.integers(lo, hi + 1, size=n)
    m = 1.0 + rng.random(n)
    s = np.where(rng.random(n) < 0.5, -1.0, 1.0)
    with np.errstate(over="ignore", under="ignore"):
        return s * np.ldexp(m, k)


def test_fastdiv_random_bit_patterns():
    rng = np.random.default_rng(1)
    n = 1 << 21
    a, a2, a3, b = (_rand_bits(rng, n) for _ in range(4))
    _check(a, a2, a3, b, rng.random(n) < 0.1)


def test_fastdiv_range_edges():
    rng = np.random.default_rng(2)
    n = 1 << 21
    bands_a = [(-1074, -1020), (-975, -960), (-806, -794), (-770, -764), (-10, 10), (594, 606), (760, 780), (1010, 1023)]
    bands_b = [(-1074, -1020), (-126, -114), (-10, 10), (114, 126), (1010, 1023)]
    a = np.concatenate([_pow2_band(rng, n // len(bands_a) + 1, lo, hi) for lo, hi in bands_a])[:n]
    b = np.concatenate([_pow2_band(rng, n // len(bands_b) + 1, lo, hi) for lo, hi in bands_b])[:n]
    rng.shuffle(a)
    rng.shuffle(b)
    a2, a3 = rng.permutation(a), rng.permutation(a)
    _check(a, a2, a3, b, rng.random(n) < 0.1)


def test_fastdiv_specials():
    vals = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, -1.0, 3.0, 5e-324, -5e-324, 2.2250738585072014e-308,
                     1.7976931348623157e308, -1.7976931348623157e308, 2.0 ** (-800), 2.0 ** 600, 2.0 ** (-120), 2.0 ** 120,
                     2.0 ** (-801), 2.0 ** 601, 2.0 ** (-121), 2.0 ** 121, 1e-12, 25.4, -100.0, 2.0 ** (-767),
                     np.nextafter(2.0 ** (-767), 0), np.nextafter(2.0 ** (-767), 1)])
    a, b = np.meshgrid(vals, vals)
    a, b = a.ravel(), b.ravel()
    a2, a3 = np.roll(a, 1), np.roll(a, 2)
    kill = (np.arange(a.size) % 3 == 0)
    _check(a, a2, a3, b, kill)


def test_deferred_guards_flag_only_out_of_range_operands():
    """Ordinary operands (the magnitudes a trace produces, zeros and infinities included) are never
    flagged by the GuardDefer forms (the shortcuts' exact ranges cover them: a deferred-guard kernel would re-trace
    only pathological rays)."""
    rng = np.random.default_rng(11)
    n = 200_000
    a = _pow2_band(rng, n, -300, 300)
    b = _pow2_band(rng, n, -100, 100)
    a[::97] = 0.0
    b[::89] = 0.0
    a[::101] = np.inf
    b[::103] = np.inf
    kill = np.zeros(n, dtype=np.uint8)
    out = _check(a, a * 0.5, -a, b, kill)
    for f in (10, 14, 16, 18):          # (25: div3_norm divides by the norm of (a, a / 2, -a), up to 2^300)
        assert not out[f].any(), (f, int(out[f].sum()))


def test_fastdiv_normalisation_inputs():
    """what the kernels divide: vector components by their norm (tiny and zero components included),
    positions by radii, phases by wavelengths"""
    rng = np.random.default_rng(3)
    n = 1 << 21
    scale = 10.0 ** rng.uniform(-300, 300, size=(3, n))
    v = rng.standard_normal((3, n)) * scale
    v[0, ::7] = 0.0
    v[1, ::5] = -0.0
    v[2, ::11] = 1e-310
    with np.errstate(all="ignore"):
        nrm = np.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
    _check(v[0], v[1], v[2], nrm, rng.random(n) < 0.05)
    a = rng.uniform(-30, 30, n) * 10.0 ** rng.uniform(-16, 3, n)
    b = rng.choice([-1.0, 1.0], n) * 10.0 ** rng.uniform(-4, 4, n)
    _check(a, np.roll(a, 1), np.roll(a, 2), b, rng.random(n) < 0.05)


def test_fused_norm_test_range_edges():
    """unit_or_zero's combined test (norm2_fast: 2^-240 <= |v|^2 < 2^238 or NaN) straddled: vectors whose norm
    squared lies just inside and outside both limits, with tiny, zero, huge, infinite and NaN companions --
    bit for bit equal to NumPy's v / |v| with NaN -> 0."""
    rng = np.random.default_rng(17)
    n = 1 << 18
    edge = np.where(rng.random(n) < 0.5, 2.0 ** -120, 2.0 ** 119) * (1.0 + rng.uniform(-1e-3, 1e-3, n))
    edge *= np.where(rng.random(n) < 0.5, 1.0, 1.0 + np.ldexp(rng.integers(-4, 5, n).astype(float), -52))
    a = edge * rng.choice([-1.0, 1.0], n)
    a2 = np.where(rng.random(n) < 0.3, 0.0, a * rng.uniform(-1e-9, 1e-9, n))
    a3 = np.where(rng.random(n) < 0.3, -0.0, np.ldexp(rng.uniform(0.5, 1.0, n), rng.integers(-1074, 600, n)))
    a3[::97] = np.inf
    a2[::89] = np.nan
    kill = np.zeros(n, dtype=np.uint8)
    _check(a, a2, a3, np.abs(a) + 1.0, kill)


def test_near_unit_normalisation():
    """unit_near1_or_zero (Snell's second tangent vector, RT:1207-1209): vectors whose norm squared lies within a few
    ulps to 2^-31 of 1 -- where the square root and the reciprocal come from the bit pattern of the norm squared --
    and just outside that window, with zero, tiny (below 2^-799), negative-zero and NaN components: NumPy's
    v / |v| with NaN -> 0, bit for bit."""
    rng = np.random.default_rng(23)
    n = 1 << 20
    v = rng.standard_normal((3, n))
    v /= np.sqrt((v * v).sum(0))                                  # unit vectors, |v|^2 = 1 +- a few ulps
    scale = np.ones(n)
    k = rng.integers(0, 4, n)
    scale[k == 1] = 1 + rng.uniform(-2.0 ** -32, 2.0 ** -32, (k == 1).sum())     # inside the window
    scale[k == 2] = 1 + rng.choice([-1, 1], (k == 2).sum()) * 2.0 ** -31.5 * (1 + rng.random((k == 2).sum()))  # edge
    scale[k == 3] = 1 + rng.uniform(-1e-3, 1e-3, (k == 3).sum())  # outside: the fallback
    v *= scale
    v[0, ::7] = 0.0
    v[1, ::11] = -0.0
    v[2, ::13] = 1e-300                                           # tiny: the quotients' slow path
    v[0, ::17] = -np.sqrt(1 - v[1, ::17] ** 2)                    # meridional rays: one exact zero, |v| ~ 1
    v[2, ::17] = 0.0
    v[:, ::101] = 0.0                                             # normal incidence: 0 / 0 -> 0
    v[1, ::103] = np.nan
    kill = np.zeros(n, dtype=np.uint8)
    _check(v[0], v[1], v[2], np.ones(n), kill)
