"""The kernel's per-ray arithmetic (rtpb_math.h, instantiated on the host by a test-only harness)
reproduces the reference's golden histories BIT FOR BIT, through the product's own lowering
(ray_trace_pb_amd._engine.lower).  Runs without a GPU."""
import ctypes

import numpy as np
import pytest

import ray_trace_pb_amd.materials as mat
import ray_trace_pb_amd.raytrace as rt
from ray_trace_pb_amd import _capi as C
from ray_trace_pb_amd import _engine as E
from native_harness import harness, harness_trace
from parity import same_bits, CASES, load_case
from serialize import system_from_json
import json


def lowered_case(name):
    d = np.load(f"{__import__('parity').GOLDEN}/{name}.npz")
    system, m0, m1 = system_from_json(rt, mat, str(d["system_json"]))
    rays = d["rays_in"]
    low = E.lower(system.surfaces, [m0] + list(system.materials) + [m1],
                  lambda: np.unique(rays[:, 7]), C.RTPB_F64)
    return low, rays, d["history"]


@pytest.mark.parametrize("name", CASES)
def test_kernel_math_bitwise_vs_reference(name):
    low, rays, ref = lowered_case(name)
    got = harness_trace(low, rays)
    assert same_bits(got, ref)


def _up(x):
    return np.nextafter(x, np.inf)


def _down(x):
    return np.nextafter(x, -np.inf)


@pytest.mark.parametrize("ap", [25.4, 1e6, 12.7, 0.0, 1e-300, 3.0, 7.25, np.inf, -1.0, np.nan, 2.0 ** 0.5])
def test_aperture_threshold_is_exact(ap):
    """s <= ap_sq  <=>  sqrt(s) <= ap for every double s >= 0 (checked at and around the bound)."""
    out = np.zeros(3)
    harness().harness_bounds(ap, 1.0, 1e-12, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    T = out[0]
    if np.isnan(ap) or ap < 0:
        assert T == -np.inf
        return
    if np.isinf(ap):
        assert T == np.inf
        return
    assert np.sqrt(T) <= ap and not np.sqrt(_up(T)) <= ap
    for s in (ap * ap, _up(ap * ap), _down(ap * ap), T, _down(T)):
        if s >= 0:                      # sums of squares are never negative
            assert (np.sqrt(s) <= ap) == (s <= T)


@pytest.mark.parametrize("A", [30.0, 25.0, 1e6, 50.0, 1e-13, 0.0, 65.8, 280.6, np.inf, 3.5e4])
def test_sphere_shell_bounds_are_exact(A):
    """shell_lo <= s <= shell_hi  <=>  |sqrt(s) - A| < 1e-12 (the R=1e6 quirk included: only the
    squares whose root rounds to A itself are on the surface)."""
    tol = 1e-12
    out = np.zeros(3)
    harness().harness_bounds(1.0, A, tol, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    lo, hi = out[1], out[2]
    P = lambda s: abs(np.sqrt(s) - A) < tol  # noqa: E731
    if np.isinf(A):
        assert lo > hi
        return
    assert P(lo) and P(hi)
    assert not P(_up(hi))
    if lo > 0:
        assert not P(_down(lo))
    rng = np.random.default_rng(0)
    for s in np.concatenate((np.linspace(lo, hi, 50), [A * A, _up(A * A), _down(A * A)],
                             A * A * (1 + rng.normal(scale=1e-13, size=200)))):
        if s >= 0:
            assert P(s) == (lo <= s <= hi)


def test_near_unit_sqrt_and_reciprocal_bit_formulas():
    """rtpb_math.h unit_near1_or_zero: for v = 1 + d ulps (d = bits(v) - bits(1), |d| <= 2^22, i.e. |v - 1| <= 2^-31
    and beyond), RN(sqrt(v)) = bits(1) + (d >> 1) and RN(1 / RN(sqrt(v))) = bits(1) - 2m (m = d >> 1 >= 0) or
    bits(1) + ceil(-m / 2) (m < 0), and d is the low word of v read as a signed 32-bit integer -- exhaustively,
    against NumPy's correctly rounded sqrt and division."""
    b1 = np.float64(1.0).view(np.int64)
    d = np.arange(-(1 << 22), (1 << 22) + 1, dtype=np.int64)
    v = (b1 + d).view(np.float64)
    m = d >> 1
    s = (b1 + m).view(np.float64)
    assert np.array_equal(np.sqrt(v).view(np.int64), s.view(np.int64))
    y = np.where(m >= 0, b1 - 2 * m, b1 + ((1 - m) >> 1)).view(np.float64)
    assert np.array_equal((1.0 / s).view(np.int64), y.view(np.int64))
    lo = (v.view(np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.uint32).view(np.int32)
    assert np.array_equal(lo.astype(np.int64), d)
    # the kernel's branch-free select for the reciprocal's offset, written in d
    d32 = d.astype(np.int32)
    neg = d32 >> 31
    t = (neg & ((3 - d32) >> 2)) | (~neg & -(d32 & ~1))
    assert np.array_equal(t.astype(np.int64), np.where(m >= 0, -2 * m, (1 - m) >> 1))
    # the window test |v - 1| <= 2^-31 keeps d inside the checked range
    inside = np.abs(v - 1.0) <= 2.0 ** -31
    assert np.abs(d[inside]).max() <= 1 << 22


@pytest.mark.parametrize("name", ["c5_odt", "c3_relay", "stress", "fuzz_03", "fuzz_23"])
def test_sweep_pair_step_equals_two_steps(name):
    """The spot sweep's shared first surface (surface_step_pair: one intersection, normal, tests and tangent basis,
    two refractions) gives each wavelength's ray bit for bit what its own surface_step gives (positions and
    directions, NaN pattern included), for every refracting Flat / Sphere surface of the system, on the golden
    rays and on rays with zero, tiny, infinite and NaN components."""
    import json
    import systems
    lib = harness()
    fn = lib.harness_pair_vs_steps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_double, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    spec, rays, _ = load_case(name)
    system, m0, m1 = system_from_json(rt, mat, json.dumps(spec))
    rays = np.concatenate([rays, systems.stress_rays(256, seed=11)], axis=0)
    low = E.lower(system.surfaces, [m0] + list(system.materials) + [m1], lambda: np.unique(rays[:, 7]), C.RTPB_F64)
    tried = 0
    for k in range(low.nsurf):
        if low.surfaces[k].kind not in (C.RTPB_FLAT, C.RTPB_SPHERE) or not isinstance(
                system.surfaces[k], rt.RefractingSurface):
            continue
        x = np.ascontiguousarray(rays, dtype=np.float64)
        out = np.empty((x.shape[0], 4, 6))
        assert fn(ctypes.byref(low.surfaces[k]), 1.0 / 1.5, 1.0 / 1.52, x.ctypes.data, x.shape[0], out.ctypes.data) == 0
        assert same_bits(out[:, 0], out[:, 2]) and same_bits(out[:, 1], out[:, 3]), (name, k)
        tried += 1
    assert tried > 0


@pytest.mark.parametrize("name", ["c5_odt", "c3_relay", "c2_achromat", "stress", "fuzz_03", "fuzz_23"])
def test_positions_only_step_matches_the_full_step(name):
    """The spot sweep's positions-only steps (kPosOnly: a kAxial sphere's backward or infinite root kills the row
    instead of becoming a NaN t, no TIR position fill, the front-side test joined to the final kill) leave every live
    row of the full step bit for bit (positions and directions) and a NaN direction on every other row -- the
    final-position semantics the sweep's reduction applies.  Rays: the golden bundle, the same rays reversed (both
    roots behind them), started from inside the spheres' balls and beyond the system, and adversarial components."""
    import json
    import systems
    lib = harness()
    fn = lib.harness_pos_vs_full
    fn.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    spec, rays, _ = load_case(name)
    system, m0, m1 = system_from_json(rt, mat, json.dumps(spec))
    back = rays.copy()
    back[:, 3:6] *= -1
    deep = rays.copy()
    deep[:, 2] += np.linspace(0.0, 3000.0, rays.shape[0])           # from the front of the system to far beyond it
    rays = np.concatenate([rays, back, deep, systems.stress_rays(256, seed=5)], axis=0)
    low = E.lower(system.surfaces, [m0] + list(system.materials) + [m1], lambda: np.unique(rays[:, 7]), C.RTPB_F64)
    tried = killed = 0
    for k in range(low.nsurf):
        if low.surfaces[k].kind not in (C.RTPB_FLAT, C.RTPB_SPHERE) or not isinstance(
                system.surfaces[k], rt.RefractingSurface):
            continue
        x = np.ascontiguousarray(rays, dtype=np.float64)
        out = np.empty((x.shape[0], 2, 6))
        assert fn(ctypes.byref(low.surfaces[k]), 1.0 / 1.5, x.ctypes.data, x.shape[0], out.ctypes.data) == 0
        live = ~np.isnan(out[:, 1, 3])
        assert same_bits(out[live, 0], out[live, 1]), (name, k)
        assert np.isnan(out[~live, 0, 3]).all(), (name, k)
        tried += 1
        killed += int((~live).sum())
    assert tried > 0 and killed > 0


def test_sweep_fan_index_division_is_exact():
    """rtpb_spot_sweep divides the fan index j by n_thetas as (j * mul) >> shift (rtpb_math.h sweep_divisor):
    exact for every j < 2^31 -- checked at the quotient boundaries (multiples of d and their neighbours), near 2^31
    and on random indices for divisors from 1 to 2^31 - 1; no multiplier for group sizes of 2^31 or more."""
    lib = harness()
    fn = lib.harness_sweep_divisor
    fn.restype = None
    fn.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int32)]
    rng = np.random.default_rng(5)
    divisors = [1, 2, 3, 7, 64, 255, 256, 257, 3162, 3163, 10001, 46341, 65537, 1 << 20, (1 << 20) + 1,
                (1 << 30) - 1, 1 << 30, (1 << 31) - 1] + rng.integers(1, 1 << 31, 64).tolist()
    mul, shift = ctypes.c_uint32(), ctypes.c_int32()
    for d in divisors:
        fn(d, (1 << 31) - 1, ctypes.byref(mul), ctypes.byref(shift))
        assert mul.value != 0, d
        k = np.arange(0, min(4096, ((1 << 31) - 1) // d + 1), dtype=np.uint64)
        j = np.concatenate([k * np.uint64(d), k * np.uint64(d) + np.uint64(d - 1), k * np.uint64(d) - np.uint64(1),
                            np.arange((1 << 31) - 4096, 1 << 31, dtype=np.uint64),
                            rng.integers(0, 1 << 31, 20000).astype(np.uint64)])
        j = j[j < (1 << 31)]
        q = (j * np.uint64(mul.value)) >> np.uint64(shift.value)
        assert np.array_equal(q, j // np.uint64(d)), d
    fn(3163, 1 << 31, ctypes.byref(mul), ctypes.byref(shift))
    assert mul.value == 0                         # the kernel then divides in 64 bits
