// rtpb_math.h -- per-ray arithmetic of the sequential ray trace, shared by the gfx950 kernel
// (rtpb_trace.hip and the other kernels) and the CPU test harness (tests/native/math_harness.cpp).
//
// Every function restates one piece of the reference (QI2lab/ray_trace_pb @ 2024_10_08,
// src/raytrace/raytrace.py = RT, src/raytrace/materials.py = MAT) for ONE ray, with the operations
// in exactly the order NumPy evaluates the reference's vector expressions (left-to-right products,
// norm = sqrt((a*a + b*b) + c*c), np.cross component formulas).  Compiled with -ffp-contract=off and
// without fast-math, the f64 instantiation is IEEE-identical to the reference.
//
// Descriptors arrive by value (the kernel loads them with scalar loads from the constant address
// space, so they live in SGPRs); per-ray state lives in VGPRs.
#pragma once

#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <limits>
#include <type_traits>

#include "rtpb.h"

#if defined(__HIPCC__)
#define RTPB_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#define RTPB_HD inline
#endif

namespace rtpb {

// internal surface / material kinds (public ones from rtpb.h + host-detected specialisations)
enum SurfKind : int32_t { FLAT = 0, SPHERE = 1, PLANE_MIRROR = 2, PERFECT_LENS = 3 };
enum MatKind : int32_t { CONSTANT = 0, SELLMEIER = 1, POLY6 = 2, TABLE = 3,
                         VACUUM = 4 /* SELLMEIER with all-zero coefficients (MAT:54-56) */ };

template <typename T>
struct DevSurface {
    int32_t kind;
    int32_t rcp_ok;   // bit 0: rR, bit 1: rf usable by the shared-divisor quotients (host_rcp_ok); bit 2: nr
                      // valid; bit 3: rn2 valid and usable by the quotients; bits 4 / 5: bits 2 / 3 for a
                      // boundary with a Vacuum side, valid where the wavelength squared is finite and nonzero;
                      // bit 6: axial geometry (kAxial, see axdot)
    T c[3];      // center
    T nrm[3];    // plane normal (flat / mirror / lens)
    T ax[3];     // input_axis
    T R;         // signed radius
    T R2;        // radius**2 as evaluated by the host
    T absR;      // abs(radius)
    T ap;        // aperture_rad
    T f;         // focal length
    T sin_a;     // sin(alpha)
    T tol;       // on-surface tolerance
    // exact squared-distance thresholds of the on-surface tests (see lower_surface): the tests
    // compare sums of squares with these instead of taking their square roots
    T ap_sq;     // sqrt(s) <= ap           <=>  s <= ap_sq
    T shell_lo;  // |sqrt(s) - |R|| < tol   <=>  shell_lo <= s <= shell_hi
    T shell_hi;
    // correctly rounded reciprocals of the surface's uniform divisors, computed on the host (the same y a
    // per-lane make_rcp would refine, without its 5 VALU per lane per surface): 1 / radius, 1 / focal_len
    T rR;
    T rf;
    // PerfectLens: normal * focal_len, the host-side product of F = C - n f n1 and B = C + n f n2 (RT:1682-1687
    // evaluate `normal * self.focal_len` before the per-ray index)
    T nf[3];
    // both adjacent media Constant or Vacuum (rcp_ok bit 2, or bit 4 with a Vacuum side): n1 and n2 are the
    // same for every ray (Vacuum: 1, MAT:54-56), so the Snell ratio n1 / n2 (RT:1213) and 1 / n2
    // (PerfectLens sin_t2, RT:1749) are computed once on the host (IEEE division: the same correctly
    // rounded values the per-lane divisions give)
    T nr;
    T rn2;
    // PerfectLens between uniform media (rcp_ok bit kLensUni; kLensUniVac: valid where Vacuum's n is 1): the focal
    // points F = C - (n f) n1 and B = C + (n f) n2 (RT:1682-1687), n1 f (RT:1755) and the phase term
    // n1 n1 f + n2 n2 f (RT:1776-1777), evaluated on the host in the kernel's order
    T lF[3];
    T lB[3];
    T ln1f;
    T lph;
};

template <typename T>
struct DevMaterial {
    int32_t kind;
    int32_t table_off;   // TABLE: offset (in pairs) into the plan's table array
    int32_t table_len;
    int32_t pad;
    T c[6];
};

template <typename T>
struct Ray {
    T x, y, z, dx, dy, dz, ph, wl;
};

template <typename T> RTPB_HD T qnan() { return T(__builtin_nan("")); }
template <> RTPB_HD float qnan<float>() { return __builtin_nanf(""); }

template <typename T> RTPB_HD bool is_nan(T v) { return v != v; }

// Device fast paths of the f64 division and square root that are bit-identical to the compiler's own
// expansions (see "shared-divisor quotients" below and tsqrt); host builds (the CPU harness) use the
// plain operators.
#if defined(__HIP_DEVICE_COMPILE__)
#define RTPB_FASTDIV 1
#define RTPB_FASTSQRT 1
#endif

#if defined(__HIP_DEVICE_COMPILE__)
// A class-test mask as a scalar register: v_cmp_class_f64 then takes it as an SGPR operand (VOP3) instead of
// a VGPR the compiler rematerialises with a v_mov (one VALU per test) when registers are tight.
__device__ __forceinline__ int class_mask(int k) {
    int r;
    asm("s_mov_b32 %0, %1" : "=s"(r) : "i"(k));
    return r;
}
#endif

// Guard policies of the exact fast paths below.  Each shortcut is exact only inside a range of its
// operands; outside it the operation must take the compiler's full sequence.
//   GuardBranch: a per-operation branch to the full sequence -- what every shipped kernel uses.
//   GuardDefer:  no branch -- the operation only records that a lane left the range (g->bad) and a caller would
//                re-trace such rays with GuardBranch.  Measured slower in every kernel (DESIGN.md §5, round 3:
//                the re-trace path raises register use, and the flags cost more VALU than the branches' exec
//                updates); kept for tests/native/fastdiv_check.hip, which checks that the flags are raised
//                exactly where a shortcut leaves its exact range (tests/test_gpu_fastdiv.py).
struct GuardBranch { static constexpr bool kDefer = false; };
struct GuardDefer { static constexpr bool kDefer = true; bool bad = false; };

// gfx950 has no f64 sqrt instruction: the compiler emits (i) x < 2^-767 ? x * 2^256 : x, (ii) rsq + two
// Goldschmidt/Newton rounds (mul, mul, 7 fma), (iii) the inverse rescale, and (iv) a select that returns
// x itself for +-0 and +inf -- 18 instructions.  For 2^-767 <= x < inf, for x < 0 and for NaN, steps (i),
// (iii) and (iv) are identities (a negative or NaN x gives NaN either way), so the device path runs step
// (ii) alone -- the identical instructions, hence identical bits -- and hands the remaining inputs
// (+-0, denormals, tiny normals, +inf) to the full expansion.
#if defined(RTPB_FASTSQRT)
// step (ii) alone: RN(sqrt(v)) for 2^-767 <= v < inf, NaN for v < 0 and v NaN
__device__ __forceinline__ double sqrt_core(double v) {
    const double y = __builtin_amdgcn_rsq(v);
    const double s0 = v * y;
    const double h0 = y * 0.5;
    const double r0 = __builtin_fma(-h0, s0, 0.5);
    const double s1 = __builtin_fma(s0, r0, s0);
    const double d0 = __builtin_fma(-s1, s1, v);
    const double h1 = __builtin_fma(h0, r0, h0);
    const double s2 = __builtin_fma(d0, h1, s1);
    const double d1 = __builtin_fma(-s2, s2, v);
    return __builtin_fma(d1, h1, s2);
}
#endif

template <typename T, class G = GuardBranch>
RTPB_HD T tsqrt(T v, G* g = nullptr) {
    if constexpr (sizeof(T) != 8) {
        return sqrtf(v);
    } else {
#if defined(RTPB_FASTSQRT)
    double s3 = sqrt_core(v);
    // the set -- +-0, +denormals, +normals below 2^-767, +inf -- as one class test and one 32-bit
    // compare of the high word (negative values and NaN have it at or above 0x10000000 unsigned)
    // (bitwise |: both tests are one VALU each; a short-circuit || puts the core under a branch of its own)
    const bool special = __builtin_amdgcn_class(v, class_mask(0x2E0));
    const bool slow = special | (static_cast<uint32_t>(__double2hiint(v)) < 0x10000000u);
    if constexpr (G::kDefer) {
        // +-0 and +inf (normal incidence gives sqrt(0) on every axial ray) are their own square roots:
        // a select, so only 0 < v < 2^-767 is left to the re-trace
        if (v == 0.0 || v == __builtin_inf()) s3 = v;
        g->bad = g->bad || (v > 0.0 && v < 0x1p-767);
    } else {
        if (__builtin_expect(slow, 0)) s3 = sqrt(v);
    }
    return s3;
#else
    (void)g;
    return sqrt(v);
#endif
    }
}

// sqrt(1 - m m) (Snell's tangential root RT:1217, PerfectLens cos_t2 RT:1763): the argument w = RN(1 - RN(m m)) is
// NaN, negative, +0 or at least 2^-53 -- RN(m m) < 1 is a multiple of 2^-53 where it is at least 1/2 (so 1 - it is
// exact), and w > 1/2 elsewhere -- so +0 (|m| = 1) is the only argument the square-root core cannot take: one
// compare instead of tsqrt's class and range tests
template <typename T, class G = GuardBranch>
RTPB_HD T tsqrt_1m(T w, G* g = nullptr) {
#if defined(RTPB_FASTSQRT)
    if constexpr (sizeof(T) == 8 && !G::kDefer) {
        T s = sqrt_core(w);
        if (__builtin_expect(w == T(0), 0)) s = sqrt(w);
        return s;
    }
#endif
    return tsqrt<T>(w, g);
}

// numpy.abs: |v| with +0 for -0 -- the sign-bit clear (one VALU, or a free operand modifier in a compare)
template <typename T> RTPB_HD T tabs(T v) { return std::fabs(v); }

template <typename T> RTPB_HD T tpow(T b, T e);
template <> RTPB_HD double tpow<double>(double b, double e) { return pow(b, e); }
template <> RTPB_HD float tpow<float>(float b, float e) { return powf(b, e); }

template <typename T> struct Const {
    static constexpr double pi = 3.141592653589793;        // numpy.pi
    static constexpr double two_pi = 6.283185307179586;    // 2 * numpy.pi (exact doubling)
};

template <typename T>
RTPB_HD void kill(Ray<T>& r) {
    const T n = qnan<T>();
    r.x = n; r.y = n; r.z = n; r.dx = n; r.dy = n; r.dz = n; r.ph = n; r.wl = n;
}

// Per-lane row kill (backward rays, misses, apertures, NA clips); the compiler already branches around the
// NaN fill (an if-converting variant with a volatile asm barrier measured no faster)
template <typename T>
RTPB_HD void kill_if(bool c, Ray<T>& r) {
    if (c) kill(r);
}

// Selects a value by a wave-uniform descriptor bit as a real (scalar) branch: the empty volatile asm in the
// (cheap) uniform side keeps the compiler from folding the diamond into a select that computes the per-lane
// side on every path; the per-lane side keeps its normal scheduling.
#if defined(__HIP_DEVICE_COMPILE__)
#define RTPB_NO_SPECULATE() asm volatile("")
#else
#define RTPB_NO_SPECULATE() ((void)0)
#endif

// 0 <= v < inf, -0 included (v a zero, positive denormal or positive normal number)
template <typename T>
RTPB_HD bool nonneg_finite(T v) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (sizeof(T) == 8) return __builtin_amdgcn_class(v, class_mask(0x1E0));  // -0 | +0 | +denorm | +normal
#endif
    return v >= T(0) && v < T(1) / T(0);
}

// numpy.sign: -1, 0, +1, NaN
template <typename T>
RTPB_HD T np_sign(T v) {
    return v > T(0) ? T(1) : (v < T(0) ? T(-1) : (v == T(0) ? T(0) : v));
}

// ------------------------------------------------------------------ axial geometry
// Most surfaces of real systems sit on the z axis: normal and input axis exactly (+0, +0, 1), center
// (+0, +0, cz) (lower_surface sets kAxial then).  Their products with the 0 and 1 components are exact, so
//   v - (+0) == v,   v * 1 == v,   RN(RN(a * 0) + b) == fma(a, 0, b)
// bit for bit -- zero signs, infinities and NaN included (an fma rounds once, and a product that is exact
// leaves nothing to round) -- and the reference's expressions shrink without changing a result:
//   ((x - 0) * 0 + (y - 0) * 0) + (z - cz) * 1  ==  fma(y, 0, x * 0) + (z - cz)      (5 -> 3 float64 ops)
// The specialised surface steps (surface_step<..., GEO = kGeoAxial>) use only these identities.
//
// A surface TILTED in the x-z plane (the OPM's remote-focus optics, RT:1306-1347 / RT:1558-1801 with a normal
// (-sin t, 0, cos t)) has normal, input axis and center with y components exactly +0: the same identities remove
// every product with those zeros (kPlaneXZ, GEO = kGeoXZ) -- a dot product with the normal becomes
// fma(vy, 0, vx nx) + vz nz (5 -> 4 float64 operations), a cross product with it loses two of its six products, and
// y - (+0) = y.
constexpr int32_t kAxial = 64;
// rcp_ok bit 7: a PerfectLens with 2^-80 <= |focal_len| < 2^120, so -|r1| / f is inside the shortcut range
constexpr int32_t kLensQ1 = 128;
// rcp_ok bits 8 / 9: a PerfectLens between uniform media whose focal points and constants come from the descriptor
// (lF, lB, ln1f, lph); bit 9 = the same next to a Vacuum, valid when every ray of the wave has an ordinary
// wavelength (the trace kernel turns it into bit 8).  On a kAxial lens the host sets them only when F and B lie on
// the axis bit for bit (x, y = +0), so the focal-plane propagation takes the axial form too.
constexpr int32_t kLensUni = 256;
constexpr int32_t kLensUniVac = 512;
// rcp_ok bits 10 / 11: the radius is positive / negative, finite and in the shortcut divisor range (a sphere normal's
// quotients then need no div_fixup, fastdiv_q_nofix)
constexpr int32_t kRPos = 1024;
constexpr int32_t kRNeg = 2048;
// rcp_ok bit 12: the x-z-plane geometry (flats and PerfectLens steps; set only where kAxial is not)
constexpr int32_t kPlaneXZ = 4096;

// geometry forms of the surface steps (template parameter GEO)
constexpr int kGeoGeneral = 0;     // any normal, input axis and center
constexpr int kGeoAxial = 1;       // kAxial: normal and input axis (+0, +0, 1), center (+0, +0, cz)
constexpr int kGeoXZ = 2;          // kPlaneXZ: normal, input axis and center with y == +0

RTPB_HD double tfma(double a, double b, double c) { return __builtin_fma(a, b, c); }

// +0 as an operand the compiler cannot see is zero: fma(-a, 0, b) with a visible zero is rewritten to
// fma(a, -0, b), and -0 is no inline constant of gfx950, so the product needs the two-address fmac with a
// literal (plus a register copy wherever b stays live).  With the zero in a scalar register the negation stays a
// source modifier of one three-address v_fma_f64.  Same operation, same bits.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ double zero_s() {
    double z;
    asm("s_mov_b64 %0, 0" : "=s"(z));
    return z;
}
#else
inline double zero_s() { return 0.0; }
#endif

// v . n for a surface vector n; kGeoAxial: n == (+0, +0, 1); kGeoXZ: ny == +0
template <int GEO, typename T>
RTPB_HD T axdot(T vx, T vy, T vz, T nx, T ny, T nz) {
    if constexpr (GEO == kGeoAxial) {
        (void)nx; (void)ny; (void)nz;
        return tfma(vy, T(0), vx * T(0)) + vz;
    } else if constexpr (GEO == kGeoXZ) {
        (void)ny;
        return tfma(vy, T(0), vx * nx) + vz * nz;
    } else {
        return vx * nx + vy * ny + vz * nz;
    }
}

// v - c for the x component of a surface center; kGeoAxial: c == +0
template <int GEO, typename T>
RTPB_HD T axsub_x(T v, T c) {
    if constexpr (GEO == kGeoAxial) {
        (void)c;
        return v;
    } else {
        return v - c;
    }
}

// v - c for the y component of a surface center; kGeoAxial, kGeoXZ: c == +0
template <int GEO, typename T>
RTPB_HD T axsub_y(T v, T c) {
    if constexpr (GEO != kGeoGeneral) {
        (void)c;
        return v;
    } else {
        return v - c;
    }
}

// ------------------------------------------------------------------ shared-divisor quotients
// Several quotients a_i / b with ONE divisor (a vector normalised by its norm, a normal divided by the
// radius, phases divided by the wavelength).  gfx950 has no f64 divide instruction; the compiler expands
// every `a / b` into div_scale(b), rcp, four Newton FMAs (all on b only), div_scale(a), mul, fma,
// div_fmas, div_fixup.  Rcp holds the b-only part (y = the same Newton-refined reciprocal, same
// instructions) so each further quotient costs mul + fma + fma + div_fixup -- the compiler's own
// sequence minus the scaling steps, which are identities when
//   * b is 0, inf or NaN, or 2^-120 <= |b| <= 2^120, and
//   * a is 0, inf or NaN, or 2^-800 <= |a| <= 2^600
// (div_scale rescales only for |b| near the overflow/denormal range, a quotient in the denormal range,
// an exponent gap >= 768 or |a| < 2^-969; div_fixup turns 0, inf and NaN operands into the IEEE result
// on its own).  A lane outside those ranges takes the plain division, so every quotient is bit-identical
// to `a / b`, i.e. correctly rounded.  Host builds (the CPU harness) always divide.
template <typename T>
struct Rcp {
    T b;
    T y;
    bool ok;   // b in the range above (device); host: unused
    T k;       // make_wl_rcp only: 2 pi / b (the PerfectLens wave number, RT:1773)
};

#if defined(RTPB_FASTDIV)
// The range tests read the frexp exponent e (|x| = m 2^e, 0.5 <= m < 1; v_frexp_exp_i32_f64 gives e = 0 for
// +-0, +-inf and NaN, which are in range either way, and e <= -1021 for denormals, which are not).
__device__ __forceinline__ bool fastdiv_den_ok(double b) {
    // 2^-120 <= |b| < 2^120 <=> -119 <= e <= 120; or b = 0, inf, NaN (e = 0)
    return static_cast<uint32_t>(__builtin_amdgcn_frexp_exp(b) + 119) <= 239u;
}
__device__ __forceinline__ bool fastdiv_num_ok(double a) {
    // 2^-800 <= |a| < 2^600 <=> -799 <= e <= 600 (a subset of the exact range); or a = 0, inf, NaN (e = 0)
    return static_cast<uint32_t>(__builtin_amdgcn_frexp_exp(a) + 799) <= 1399u;
}
__device__ __forceinline__ double fastdiv_q(double a, double b, double y) {
    const double q0 = a * y;
    const double e = __builtin_fma(-b, q0, a);
    return __builtin_amdgcn_div_fixup(__builtin_fma(e, y, q0), b, a);
}
// The same quotient without div_fixup, for a divisor of known sign (SIGN = +1: b > 0, -1: b < 0) in the shortcut
// range and a FINITE numerator in range (NaN is fine too: it propagates).  For such operands div_fixup only
// re-applies sign(a) ^ sign(b) to |q| (the special-value cases -- b = 0 / inf / NaN, a = inf, quotient
// under/overflow -- cannot occur), and q already carries that sign unless a = +-0.  For a zero numerator the
// residual is an exact +0, so the sign of the correction's zero product decides: with the residual taken as
// -(a - b q0) = fma(b, q0, -a) and subtracted, the product -0 * y is -0 for y > 0; with a - b q0 added, +0 * y
// is -0 for y < 0 -- either way q0 (which has the right sign) survives the final addition.  Non-zero results
// are RN(q0 + (a - b q0) y), the fixup sequence's value bit for bit.
template <int SIGN>
__device__ __forceinline__ double fastdiv_q_nofix(double a, double b, double y) {
    static_assert(SIGN == 1 || SIGN == -1, "divisor sign");
    const double q0 = a * y;
    if constexpr (SIGN > 0) {
        const double e = __builtin_fma(b, q0, -a);
        return __builtin_fma(-e, y, q0);
    } else {
        const double e = __builtin_fma(-b, q0, a);
        return __builtin_fma(e, y, q0);
    }
}
#endif

// Rcp of a divisor whose reciprocal y = RN(1/b) the host computed: quotients through it are still correctly
// rounded (Markstein: q0 = RN(a y) is within 1 ulp of a/b, r = fma(-b, q0, a) is exact, RN(q0 + r y) =
// RN(a/b) when y = RN(1/b)); tests/test_gpu_fastdiv.py checks it on the same adversarial operands
template <typename T>
RTPB_HD Rcp<T> host_rcp(T b, T y, bool ok) {
    return Rcp<T>{b, y, ok, T(0)};
}

// host: the range test of fastdiv_den_ok, exactly (2^-120 <= |b| < 2^120, or 0, inf, NaN)
inline bool host_rcp_ok(double b) {
    const double m = std::fabs(b);
    return (m >= 0x1p-120 && m < 0x1p120) || b == 0.0 || std::isinf(b) || std::isnan(b);
}

template <typename T>
RTPB_HD Rcp<T> make_rcp(T b) {
#if defined(RTPB_FASTDIV)
    if constexpr (sizeof(T) == 8) {
        const double y0 = __builtin_amdgcn_rcp(b);
        const double y1 = __builtin_fma(y0, __builtin_fma(-b, y0, 1.0), y0);
        const double y2 = __builtin_fma(y1, __builtin_fma(-b, y1, 1.0), y1);
        return Rcp<T>{b, y2, fastdiv_den_ok(b), T(0)};
    }
#endif
    return Rcp<T>{b, T(0), true, T(0)};
}

#if defined(RTPB_FASTDIV) && defined(RTPB_FASTSQRT)
// Norms of 3-vectors, fused: for v = (x x + y y) + z z in [2^-240, 2^238), sqrt(v) takes the fast core
// (v >= 2^-767, finite) and nrm = RN(sqrt(v)) lies in [2^-120, 2^119], inside the shared-divisor range of
// fastdiv_den_ok -- so ONE test on v (its high word: the bounds have zero low words) replaces the square
// root's class / high-word test and the divisor's frexp test.  NaN v also takes the fast path (the core,
// the reciprocal and the quotients all give NaN, as the full sequences do).
__device__ __forceinline__ bool norm2_in_range(double v) {
    const uint32_t hi = static_cast<uint32_t>(__double2hiint(v));
    return hi - 0x30F00000u < 0x4ED00000u - 0x30F00000u;
}
__device__ __forceinline__ bool norm2_fast(double v) { return norm2_in_range(v) | (v != v); }

// make_rcp for a divisor known to be in range (or NaN): the same instructions without the test
__device__ __forceinline__ Rcp<double> make_rcp_in_range(double b) {
    const double y0 = __builtin_amdgcn_rcp(b);
    const double y1 = __builtin_fma(y0, __builtin_fma(-b, y0, 1.0), y0);
    const double y2 = __builtin_fma(y1, __builtin_fma(-b, y1, 1.0), y1);
    return Rcp<double>{b, y2, true, 0.0};
}
#define RTPB_FASTNORM 1
#endif

// a / r.b
// NUM_IN_RANGE: the caller guarantees the numerator is 0, inf, NaN or 2^-800 <= |a| <= 2^600 (see
// norm_quotient_bound), so only the divisor's range is tested
template <typename T, class G = GuardBranch, bool NUM_IN_RANGE = false>
RTPB_HD T div1(T a, const Rcp<T>& r, G* g = nullptr) {
#if defined(RTPB_FASTDIV)
    if constexpr (sizeof(T) == 8) {
        T q = fastdiv_q(a, r.b, r.y);
        const bool num_ok = NUM_IN_RANGE || fastdiv_num_ok(a);
        const bool slow = !(r.ok & num_ok);     // bitwise: no short-circuit branch around the fast path
        if constexpr (G::kDefer) {
            g->bad = g->bad || slow;
        } else {
            if (__builtin_expect(slow, 0)) q = a / r.b;
        }
        return q;
    }
#endif
    (void)g;
    return a / r.b;
}

// a / b where r = make_rcp(b0) and b is b0 or NaN (a wavelength after its row was killed): a NaN b gives
// NaN either way (div_fixup / the division), so y of b0 serves every value b can take
template <typename T, class G = GuardBranch, bool NUM_IN_RANGE = false>
RTPB_HD T div1_as(T a, T b, const Rcp<T>& r, G* g = nullptr) {
#if defined(RTPB_FASTDIV)
    if constexpr (sizeof(T) == 8) {
        T q = fastdiv_q(a, b, r.y);
        const bool num_ok = NUM_IN_RANGE || fastdiv_num_ok(a);
        const bool slow = !(r.ok & num_ok);     // bitwise: no short-circuit branch around the fast path
        if constexpr (G::kDefer) {
            g->bad = g->bad || slow;
        } else {
            if (__builtin_expect(slow, 0)) q = a / b;
        }
        return q;
    }
#endif
    (void)g;
    return a / b;
}

// Numerators bounded by construction.  A Euclidean norm RN(sqrt(v)), v a sum of squares, is 0, +inf, NaN or
// between sqrt(2^-1074) = 2^-537 and sqrt(DBL_MAX) < 2^512; its product with 2 pi (the phase updates'
// distance terms, RT:297 / RT:1512) lies in [2^-535, 2^515], and its quotient by a focal length with
// 2^-80 <= |f| < 2^120 (PerfectLens sin_t2, RT:1749) in [2^-657, 2^592] -- all inside the exact range of the
// shortcut quotients (2^-800 <= |a| <= 2^600), so those divisions test the divisor only (NUM_IN_RANGE).

// The per-ray divisor of every phase update (the wavelength) with 2 pi / wl once per ray
template <typename T, class G = GuardBranch>
RTPB_HD Rcp<T> make_wl_rcp(T wl, G* g = nullptr) {
    Rcp<T> r = make_rcp(wl);
    r.k = div1(T(Const<T>::two_pi), r, g);
    return r;
}

// (x, y, z) / r.b, one guard for the three quotients
template <typename T, class G = GuardBranch>
RTPB_HD void div3(T& x, T& y, T& z, const Rcp<T>& r, G* g = nullptr) {
#if defined(RTPB_FASTDIV)
    if constexpr (sizeof(T) == 8) {
        const T qx = fastdiv_q(x, r.b, r.y), qy = fastdiv_q(y, r.b, r.y), qz = fastdiv_q(z, r.b, r.y);
        const bool ox = fastdiv_num_ok(x), oy = fastdiv_num_ok(y), oz = fastdiv_num_ok(z);
        const bool slow = !(r.ok & ox & oy & oz);
        if constexpr (G::kDefer) {
            g->bad = g->bad || slow;
        } else {
            if (__builtin_expect(slow, 0)) {
                x = x / r.b; y = y / r.b; z = z / r.b;
                return;
            }
        }
        x = qx; y = qy; z = qz;
        return;
    }
#endif
    (void)g;
    x = x / r.b; y = y / r.b; z = z / r.b;
}

// (x, y, z) / r.b where r.b = RN(sqrt((x x + y y) + z z)), the vector's own norm.  Each |component| is at
// most the norm (up to rounding) when the norm is finite, so with r.ok the numerators need only the lower
// bound of the exact range (frexp exponent >= -799; 0, inf and NaN give 0): one min3 for the three instead
// of three two-sided tests.  A norm of 0, inf or NaN is in r.ok's range and div_fixup returns the IEEE
// quotient for those divisors whatever the numerator.
// SIGN = +1 / -1: the divisor is known positive / negative and the numerators finite wherever the result matters
// (fastdiv_q_nofix: no div_fixup); 0: any divisor and numerator (div_fixup).
// (Round 5 tried min(|x|, |y|, |z|) >= 2^-800 as the numerator test -- two v_min_f64 + a compare instead of three
// frexp + min3 + compare: fewer instructions, but C4 +7 %, C3 +3 % and the C5 sweep +1 % slower, profiles/r05/f.)
template <typename T, class G = GuardBranch, int SIGN = 0>
RTPB_HD void div3_norm(T& x, T& y, T& z, const Rcp<T>& r, G* g = nullptr) {
#if defined(RTPB_FASTDIV)
    if constexpr (sizeof(T) == 8) {
        auto q = [&](T a) { if constexpr (SIGN == 0) return fastdiv_q(a, r.b, r.y); else return fastdiv_q_nofix<SIGN>(a, r.b, r.y); };
        const T qx = q(x), qy = q(y), qz = q(z);
        const int e = std::min(std::min(__builtin_amdgcn_frexp_exp(x), __builtin_amdgcn_frexp_exp(y)),
                               __builtin_amdgcn_frexp_exp(z));
        const bool slow = !(r.ok & (e >= -799));
        if constexpr (G::kDefer) {
            g->bad = g->bad || slow;
        } else {
            if (__builtin_expect(slow, 0)) {
                x = x / r.b; y = y / r.b; z = z / r.b;
                return;
            }
        }
        x = qx; y = qy; z = qz;
        return;
    }
#endif
    (void)g;
    x = x / r.b; y = y / r.b; z = z / r.b;
}

// Round-up multiplier for unsigned division by d of every x < 2^31 (Granlund-Montgomery): l = ceil(log2 d),
// m = ceil(2^(31+l) / d) < 2^32, x / d = (x m) >> (31 + l) -- with e = m d - 2^(31+l) in [0, d) the product
// overshoots x / d by x e / (d 2^(31+l)) < 2^-l <= 1 / d, less than the gap to the next integer.
inline void sweep_divisor(int64_t d, int64_t gsize, uint32_t& mul, int32_t& shift) {
    mul = 0;
    shift = 0;
    if (d <= 0 || d > 0x7fffffff || gsize > 0x7fffffff) return;
    int l = 0;
    while ((int64_t(1) << l) < d) ++l;
    const uint64_t p = uint64_t(1) << (31 + l);
    const uint64_t m = (p + uint64_t(d) - 1) / uint64_t(d);
    if (m >> 32) return;
    mul = static_cast<uint32_t>(m);
    shift = 31 + l;
}

// ------------------------------------------------------------------ Material.n (MAT:39-144)
// WITH_POLY6 = false compiles the RTPB_POLY6 case out (its pow() calls dominate the kernel's register
// budget); WITH_TABLE = false compiles the TABLE case out.  Either is only valid for plans without such
// materials (rtpb_plan::feat).
template <typename T, bool WITH_POLY6 = true, bool WITH_TABLE = true, typename TablePtr, class G = GuardBranch>
RTPB_HD T material_n(const DevMaterial<T>& m, T wl, TablePtr table, G* g = nullptr) {
    switch (m.kind) {
    case CONSTANT:
        return m.c[0];                                               // MAT:72-79
    case VACUUM: {
        // (0*w2)/(w2-0) summed thrice + 1: exactly 1 unless w2 is 0, inf or NaN (then NaN)
        const T w2 = wl * wl;
        return (w2 != T(0) && w2 - w2 == T(0)) ? T(1) : qnan<T>();
    }
    case SELLMEIER: {                                                // MAT:48-51
        const T w2 = wl * wl;
        const T acc = m.c[0] * w2 / (w2 - m.c[3]) + m.c[1] * w2 / (w2 - m.c[4]) + m.c[2] * w2 / (w2 - m.c[5]);
        return tsqrt<T>(acc + T(1), g);
    }
    case POLY6: {                                                    // MAT:137-144 (Ebaf11)
        if constexpr (!WITH_POLY6) {
            return qnan<T>();
        } else {
            const T w2 = wl * wl;
            const T n2 = m.c[0] + m.c[1] * w2 + m.c[2] * tpow<T>(wl, T(-2)) + m.c[3] * tpow<T>(wl, T(-4)) +
                         m.c[4] * tpow<T>(wl, T(-6)) + m.c[5] * tpow<T>(wl, T(-8));
            return tsqrt<T>(n2, g);
        }
    }
    default: {                                                       // TABLE: host-evaluated n(lambda)
        if constexpr (!WITH_TABLE) return qnan<T>();
        // (wavelength, n) pairs sorted by wavelength, NaN keys last (sort_table): binary search for
        // the exact wavelength; NaN compares false, so NaN keys behave as +inf in the search.
        const int len = m.table_len, off = m.table_off;
        if (is_nan(wl)) {
            const bool has = len > 0 && is_nan(T(table[2 * (off + len - 1)]));
            return has ? T(table[2 * (off + len - 1) + 1]) : qnan<T>();
        }
        int lo = 0, hi = len;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (T(table[2 * (off + mid)]) < wl) lo = mid + 1;
            else hi = mid;
        }
        return (lo < len && T(table[2 * (off + lo)]) == wl) ? T(table[2 * (off + lo) + 1]) : qnan<T>();
    }
    }
}

// Whether wl is a key of TABLE material m (the same search and matching rule as material_n's TABLE case:
// NaN finds a NaN key).  A ray whose wavelength is no key would get n = NaN from the table.
template <typename T, typename TablePtr>
RTPB_HD bool table_has_key(const DevMaterial<T>& m, T wl, TablePtr table) {
    const int len = m.table_len, off = m.table_off;
    if (is_nan(wl)) return len > 0 && is_nan(T(table[2 * (off + len - 1)]));
    int lo = 0, hi = len;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (T(table[2 * (off + mid)]) < wl) lo = mid + 1;
        else hi = mid;
    }
    return lo < len && T(table[2 * (off + lo)]) == wl;
}

// ------------------------------------------------------------------ propagate_ray2plane (RT:241-306)
// Returns the ray moved onto the plane {(p - c).nrm = 0}; phase += |d t| sign(t) 2pi/wl n.
// iden: optional make_rcp of the denominator d.nrm, shared by several planes with the same normal.
// GN: the normal's geometry form, GC: the center's (axdot / axsub_x / axsub_y).
template <int GN = kGeoGeneral, int GC = kGeoGeneral, typename T, class G = GuardBranch>
RTPB_HD Ray<T> to_plane(const Ray<T>& r, T nx, T ny, T nz, T cx, T cy, T cz, T n, bool exclude_backward,
                        const Rcp<T>& iwl, T* t_out = nullptr, const Rcp<T>* iden = nullptr, G* g = nullptr) {
    const T num = -axdot<GN>(axsub_x<GC>(r.x, cx), axsub_y<GC>(r.y, cy), r.z - cz, nx, ny, nz);
    const T den = axdot<GN>(r.dx, r.dy, r.dz, nx, ny, nz);
    const T t = iden ? div1_as(num, den, *iden, g) : num / den;
    const T s = t < T(0) ? T(-1) : T(1);
    const T vx = r.dx * t, vy = r.dy * t, vz = r.dz * t;
    Ray<T> o;
    o.x = r.x + vx;
    o.y = r.y + vy;
    o.z = r.z + vz;
    o.dx = r.dx; o.dy = r.dy; o.dz = r.dz;
    const T dist = tsqrt<T>(vx * vx + vy * vy + vz * vz, g);
    // dist * s * 2 * pi (RT:297): s = +-1 is a sign, and 2 * pi is exact, so ((d s) 2) pi == (+-d) (2 pi)
    // bit for bit -- the two real products are the same number (overflow to inf included)
    o.ph = r.ph + div1_as<T, G, true>((s < T(0) ? -dist : dist) * T(Const<T>::two_pi), r.wl, iwl, g) * n;
    o.wl = r.wl;
    kill_if(exclude_backward && s == T(-1), o);
    if (t_out) *t_out = t;
    return o;
}

// ------------------------------------------------------------------ SphericalSurface.get_intersect (RT:1479-1516)
// The intersection parameter from B and root = sqrt(B^2 - 4C): t1 = (-B + root) / 2, t2 = (-B - root) / 2,
// negative roots -> inf, then numpy's min over (t1, t2) -- NaN-propagating, and the SECOND operand on a tie
// (min(+0, -0) is -0) -- and inf -> NaN (RT:1497-1505).  root is >= +0 or NaN (B^2 - 4C is never -0), so
// where both roots are numbers t2 <= t1, and t2 is NaN only with t1 NaN or +inf.  Hence: t2 when t2 >= 0,
// else t1, and NaN unless the choice is in [0, inf) -- the same value, zero signs included
// (tests/test_gpu_fastdiv.py checks it against the reference's chain on adversarial B, root).
// One product: with u2 = -B - root, 0.5 u2 >= 0 exactly when u2 >= -2^-1074 (half the smallest denormal rounds to
// -0, to even; NaN fails both), so the halving can follow the choice.
//
// FWD (the positions-only steps of kAxial spheres, whose finite shell_hi bounds every on-sphere point): no NaN for a
// root outside [0, inf) -- *fwd reports whether the chosen root is forward, u1 >= -2^-1074 (u1 >= u2: a forward u2 is
// chosen whenever there is one; NaN fails), and the caller folds it into the row's final kill.  A backward root gives
// a point ON the sphere (killed through *fwd), an infinite one a point off every finite shell (killed by the
// on-surface test) -- the row ends all NaN as with the reference's NaN t, and no stored value reads the position.
template <bool FWD = false, typename T>
RTPB_HD T sphere_root(T B, T root, bool* fwd = nullptr) {
    const T u1 = -B + root;
    const T u2 = -B - root;
    T t = T(0.5) * (u2 >= -std::numeric_limits<T>::denorm_min() ? u2 : u1);
    if constexpr (FWD) {
        *fwd = u1 >= -std::numeric_limits<T>::denorm_min();
        return t;
    }
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (sizeof(T) == 8) {
        // the NaN's high word from a scalar register (a VOP2 select's first operand), not a VGPR constant
        if (!nonneg_finite(t)) t = __hiloint2double(class_mask(0x7FF80000), 0);
        return t;
    }
#endif
    if (!nonneg_finite(t)) t = qnan<T>();
    return t;
}

// sqrt(B^2 - 4C) of the sphere's quadratic (RT:1503).  FWD (positions-only axial steps, see sphere_root): the
// argument is never -0 (B B >= +0), and of the arguments the square-root core cannot take only +0 and
// 0 < v < 2^-767 need the full sequence -- for +inf the core's NaN instead of +inf kills the row exactly as the
// reference's t = inf -> NaN does (sphere_root<true> reports no forward root) -- so ONE unsigned compare of the bit
// pattern guards the core (negative and NaN arguments give NaN either way).
template <bool FWD, typename T, class G>
RTPB_HD T disc_root(T v, G* g) {
#if defined(RTPB_FASTSQRT)
    if constexpr (FWD && sizeof(T) == 8 && !G::kDefer) {
        T root = sqrt_core(v);
        if (__builtin_expect(__builtin_bit_cast(uint64_t, v) < 0x1000000000000000ull, 0)) root = sqrt(v);  // v < 2^-767
        return root;
    }
#endif
    return tsqrt<T>(v, g);
}

// rxy (AX only): x x + y y of the ray's position, as on_sphere computed it at the previous axial surface (the
// same expression for a center on the axis) -- or nullptr.  fwd: FWD roots (sphere_root<true>), else nullptr.
template <bool AX = false, typename T, class G = GuardBranch>
RTPB_HD Ray<T> sphere_hit(const Ray<T>& r, const DevSurface<T>& s, T n, const Rcp<T>& iwl, G* g = nullptr,
                          const T* rxy = nullptr, bool* fwd = nullptr) {
    constexpr int GEO = AX ? kGeoAxial : kGeoGeneral;
    const T ox = axsub_x<GEO>(r.x, s.c[0]), oy = axsub_y<GEO>(r.y, s.c[1]), oz = r.z - s.c[2];
    const T B = T(2) * (r.dx * ox + r.dy * oy + r.dz * oz);
    const T C = ((AX && rxy) ? *rxy : ox * ox + oy * oy) + oz * oz - s.R2;
    T t;
    if (AX && fwd) t = sphere_root<true>(B, disc_root<true>(B * B - T(4) * C, g), fwd);
    else t = sphere_root(B, tsqrt<T>(B * B - T(4) * C, g));
    Ray<T> o;
    o.x = r.x + r.dx * t;
    o.y = r.y + r.dy * t;
    o.z = r.z + r.dz * t;
    o.dx = r.dx; o.dy = r.dy; o.dz = r.dz;
    const T sx = o.x - r.x, sy = o.y - r.y, sz = o.z - r.z;
    const T dist = tsqrt<T>(sx * sx + sy * sy + sz * sz, g);
    o.ph = r.ph + div1_as<T, G, true>(dist * T(Const<T>::two_pi), r.wl, iwl, g) * n;  // == (d 2) pi, see to_plane
    o.wl = r.wl;
    return o;
}

// 0 < v < inf (v a positive normal or denormal number)
template <typename T>
RTPB_HD bool positive_finite(T v) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (sizeof(T) == 8) return __builtin_amdgcn_class(v, class_mask(0x180));  // +denormal | +normal
#endif
    return v > T(0) && v < T(1) / T(0);
}

// v / |v| with NaN components replaced by 0 (RT:1203-1209)
// Device: a norm squared in [2^-240, 2^238) takes one range test (norm2_in_range) instead of the square
// root's, the divisor's and the class test of the NaN fix-ups -- the norm is then positive and finite, so no
// quotient can be NaN.  The rest (0, tiny, huge, infinite and NaN norms: normal incidence, dead rows) takes
// the full sequences and fix-ups below.
template <typename T, class G = GuardBranch>
RTPB_HD void unit_or_zero(T& x, T& y, T& z, G* g = nullptr) {
#if defined(RTPB_FASTNORM)
    if constexpr (sizeof(T) == 8 && !G::kDefer) {
        const T v = x * x + y * y + z * z;
        if (__builtin_expect(norm2_in_range(v), 1)) {
            // positive norm, finite components: the quotients need no div_fixup
            div3_norm<T, G, 1>(x, y, z, make_rcp_in_range(sqrt_core(v)), g);
        } else {
            // the compiler's correctly rounded sqrt and divisions (one straight sequence: compact code for the
            // rare lanes), then the reference's NaN -> 0
            const T nrm = sqrt(v);
            x = x / nrm; y = y / nrm; z = z / nrm;
            if (is_nan(x)) x = T(0);
            if (is_nan(y)) y = T(0);
            if (is_nan(z)) z = T(0);
        }
        return;
    }
#endif
    const T nrm = tsqrt<T>(x * x + y * y + z * z, g);
    div3_norm(x, y, z, make_rcp(nrm), g);
    // A NaN quotient needs a zero, infinite or NaN norm: when 0 < |v| < inf every component is finite and
    // every quotient a number, so one class test skips the three per-component fix-ups (normal incidence,
    // dead rows and garbage input take them)
    if (__builtin_expect(!positive_finite(nrm), 0)) {
        if (is_nan(x)) x = T(0);
        if (is_nan(y)) y = T(0);
        if (is_nan(z)) z = T(0);
    }
}

// (mask & a) | (~mask & b) as one v_bfi_b32 (LLVM turns the sign-splat form into a compare and a select)
RTPB_HD int32_t bit_select(int32_t mask, int32_t a, int32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
    int32_t r;
    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(mask), "v"(a), "v"(b));
    return r;
#else
    return (mask & a) | (~mask & b);
#endif
}

// a * B for |a| < 2^23 and a small constant B (v_mul_i32_i24 with an inline constant: one VALU where the compiler,
// not knowing the range, emits two)
template <int B>
RTPB_HD int32_t mul_i24(int32_t a) {
    static_assert(B >= -16 && B <= 64, "inline constant");
#if defined(__HIP_DEVICE_COMPILE__)
    int32_t r;
    asm("v_mul_i32_i24 %0, %1, %2" : "=v"(r) : "v"(a), "i"(B));
    return r;
#else
    return a * B;
#endif
}

// A nearly unit vector over its norm, NaN components replaced by 0: nc = N x nb (RT:1207-1209), with N a unit normal
// and nb a unit tangent, has |nc|^2 = |N|^2 |nb|^2 - (N . nb)^2 within a few ulps of 1 on every live row away from
// normal incidence.  For |v - 1| <= 2^-31 the square root and the reciprocal the quotients need are read off the
// bit pattern of v: with d = bits(v) - bits(1) (there the low word of v as a signed 32-bit integer) and m = d >> 1,
//   RN(sqrt(v)) = bits(1) + m,   RN(1 / RN(sqrt(v))) = bits(1) - 2m (m >= 0) or bits(1) + ceil(-m / 2) (m < 0)
// as bit patterns (sqrt(1 + k 2^-52) = 1 + k 2^-53 - k^2 2^-107 ..., just below a midpoint for odd k; below 1 the
// steps are 2^-53; checked exhaustively for |d| <= 2^22 against NumPy in tests/test_math_harness.py), and
// Markstein's correction with the correctly rounded reciprocal yields correctly rounded quotients -- the bits of
// the compiler's sequences, which also round correctly.  ~11 integer operations replace two transcendental-seeded
// sequences (rsq + 9, rcp + 4); other v take unit_or_zero.
template <typename T, class G = GuardBranch>
RTPB_HD void unit_near1_or_zero(T& x, T& y, T& z, G* g = nullptr) {
#if defined(RTPB_FASTNORM)
    if constexpr (sizeof(T) == 8 && !G::kDefer) {
        const T v = x * x + y * y + z * z;
        if (__builtin_expect(tabs<T>(v - T(1)) <= T(0x1p-31), 1)) {      // v - 1 is exact (Sterbenz); NaN fails
            const int32_t d = __double2loint(v);
            const int32_t neg = d >> 31;                                // -1 where v < 1
            const int32_t m = d >> 1;
            // the reciprocal's offset, m >= 0 ? -2m : ceil(-m / 2) = (1 - m) >> 1, as a bit select; -2m as one 24-bit
            // multiply (|m| <= 2^21 inside the window)
            const int32_t t = bit_select(neg, (1 - m) >> 1, mul_i24<-2>(m));
            const double s = __hiloint2double(__double2hiint(v), m);    // hi(v) = 0x3FF00000 + neg here
            const double yr = __hiloint2double(0x3FF00000 + (t >> 31), t);
            div3_norm<T, G, 1>(x, y, z, Rcp<T>{s, yr, true, T(0)}, g);   // components at most ~1: no fixup
            return;
        }
    }
#endif
    unit_or_zero(x, y, z, g);
}

// basis (normal, nb, nc): nb = d x N / |.|, nc = N x nb / |.|  (RT:1203-1209 / RT:1271-1277)
// kGeoAxial: N == (+0, +0, 1), so each cross-product component has at most one inexact product (axdot);
// kGeoXZ: Ny == +0, the x and z components lose a product each: RN(p - RN(a 0)) == fma(-a, 0, p)
template <int GEO = kGeoGeneral, typename T, class G = GuardBranch>
RTPB_HD void tangent_basis(const Ray<T>& ri, T Nx, T Ny, T Nz, T& cx, T& cy, T& cz, G* g = nullptr) {
    T bx, by, bz;
    if constexpr (GEO == kGeoAxial) {
        bx = tfma(-ri.dz, zero_s(), ri.dy);               // dy * 1 - dz * 0
        by = tfma(ri.dz, T(0), -ri.dx);                   // dz * 0 - dx * 1
        bz = tfma(-ri.dy, T(0), ri.dx * T(0));            // dx * 0 - dy * 0
    } else if constexpr (GEO == kGeoXZ) {
        bx = tfma(-ri.dz, T(0), ri.dy * Nz);              // dy Nz - dz * 0
        by = ri.dz * Nx - ri.dx * Nz;
        bz = tfma(ri.dx, T(0), -(ri.dy * Nx));            // dx * 0 - dy Nx
    } else {
        bx = ri.dy * Nz - ri.dz * Ny;
        by = ri.dz * Nx - ri.dx * Nz;
        bz = ri.dx * Ny - ri.dy * Nx;
    }
    unit_or_zero(bx, by, bz, g);
    if constexpr (GEO == kGeoAxial) {
        cx = tfma(bz, T(0), -by);                         // 0 * bz - 1 * by
        cy = tfma(-bz, zero_s(), bx);                     // 1 * bx - 0 * bz
        cz = tfma(-bx, T(0), by * T(0));                  // 0 * by - 0 * bx
    } else if constexpr (GEO == kGeoXZ) {
        cx = tfma(bz, T(0), -(Nz * by));                  // 0 * bz - Nz by
        cy = Nz * bx - Nx * bz;
        cz = tfma(-bx, T(0), Nx * by);                    // Nx by - 0 * bx
    } else {
        cx = Ny * bz - Nz * by;
        cy = Nz * bx - Nx * bz;
        cz = Nx * by - Ny * bx;
    }
    unit_near1_or_zero(cx, cy, cz, g);
}

// np.sign(v) * root for root >= +0 or NaN (RT:1217; 1 - m^2 is never -0): for v < 0 or v > 0 the product is
// root carrying v's sign (one bit operation); v = +-0 and NaN keep the product itself
template <typename T>
RTPB_HD T signed_root(T v, T root) {
    T r = std::copysign(root, v);
    if (__builtin_expect(!(v < T(0) || v > T(0)), 0)) r = np_sign<T>(v) * root;
    return r;
}

// Snell refraction of the intersected ray (RT:1197-1221)
// ratio: n1 / n2, computed by the caller (per lane, or once on the host for uniform media)
// AX: N == (+0, +0, 1) (axdot)
// TIR_FILL = false (the spot sweep's final-position semantics, kPosOnly): the position is left as it is where the
// direction is NaN -- the next surface's intersection turns it into NaN, and the sweep applies the rule to the
// final plane itself
// The ratio-independent part of snell (RT:1203-1217): the unit tangent c of the incidence plane, c . d and N . d.
// A spot sweep that traces one geometric ray at two wavelengths through a surface shares it (surface_step_pair).
template <typename T>
struct SnellBasis {
    T cx, cy, cz, cd, nd;
};

template <int GEO = kGeoGeneral, typename T, class G = GuardBranch>
RTPB_HD SnellBasis<T> snell_basis(const Ray<T>& ri, T Nx, T Ny, T Nz, G* g = nullptr) {
    SnellBasis<T> b;
    tangent_basis<GEO>(ri, Nx, Ny, Nz, b.cx, b.cy, b.cz, g);
    b.cd = b.cx * ri.dx + b.cy * ri.dy + b.cz * ri.dz;
    b.nd = axdot<GEO>(ri.dx, ri.dy, ri.dz, Nx, Ny, Nz);
    return b;
}

// The refracted ray from the basis and the Snell ratio n1 / n2
template <int GEO = kGeoGeneral, bool TIR_FILL = true, typename T, class G = GuardBranch>
RTPB_HD Ray<T> snell_apply(const Ray<T>& ri, T Nx, T Ny, T Nz, const SnellBasis<T>& b, T ratio, G* g = nullptr) {
    const T mag = ratio * b.cd;
    const T tang = signed_root(b.nd, tsqrt_1m<T>(T(1) - mag * mag, g));
    Ray<T> o;
    if constexpr (GEO == kGeoAxial) {
        o.dx = tfma(tang, T(0), mag * b.cx);
        o.dy = tfma(tang, T(0), mag * b.cy);
        o.dz = mag * b.cz + tang;
    } else if constexpr (GEO == kGeoXZ) {
        o.dx = mag * b.cx + tang * Nx;
        o.dy = tfma(tang, T(0), mag * b.cy);              // mag cy + tang * 0
        o.dz = mag * b.cz + tang * Nz;
    } else {
        o.dx = mag * b.cx + tang * Nx;
        o.dy = mag * b.cy + tang * Ny;
        o.dz = mag * b.cz + tang * Nz;
    }
    o.x = ri.x; o.y = ri.y; o.z = ri.z;
    o.ph = ri.ph;
    o.wl = ri.wl;
    if constexpr (TIR_FILL) {
        if (__builtin_expect(is_nan(o.dx), 0)) {   // TIR (and dead rows): position NaN only (RT:1221)
            o.x = qnan<T>(); o.y = qnan<T>(); o.z = qnan<T>();
        }
    }
    return o;
}

template <int GEO = kGeoGeneral, bool TIR_FILL = true, typename T, class G = GuardBranch>
RTPB_HD Ray<T> snell(const Ray<T>& ri, T Nx, T Ny, T Nz, T ratio, G* g = nullptr) {
    return snell_apply<GEO, TIR_FILL>(ri, Nx, Ny, Nz, snell_basis<GEO>(ri, Nx, Ny, Nz, g), ratio, g);
}

// law of reflection (RT:1267-1289)
template <typename T, class G = GuardBranch>
RTPB_HD Ray<T> reflect(const Ray<T>& ri, T Nx, T Ny, T Nz, G* g = nullptr) {
    T cx, cy, cz;
    tangent_basis(ri, Nx, Ny, Nz, cx, cy, cz, g);
    const T mag_na = -(Nx * ri.dx + Ny * ri.dy + Nz * ri.dz);
    const T mag_nc = cx * ri.dx + cy * ri.dy + cz * ri.dz;
    Ray<T> o;
    o.dx = mag_na * Nx + mag_nc * cx;
    o.dy = mag_na * Ny + mag_nc * cy;
    o.dz = mag_na * Nz + mag_nc * cz;
    o.x = ri.x; o.y = ri.y; o.z = ri.z;
    o.ph = ri.ph;
    o.wl = ri.wl;
    if (__builtin_expect(is_nan(o.dx), 0)) {       // position NaN where the direction is (RT:1289)
        o.x = qnan<T>(); o.y = qnan<T>(); o.z = qnan<T>();
    }
    return o;
}

// FlatSurface / PlaneMirror .is_pt_on_surface (RT:1339-1347, RT:1405-1412)
template <int GEO = kGeoGeneral, typename T>
RTPB_HD bool on_flat(const Ray<T>& p, const DevSurface<T>& s) {
    const T rx = axsub_x<GEO>(p.x, s.c[0]), ry = axsub_y<GEO>(p.y, s.c[1]), rz = p.z - s.c[2];
    const T h = axdot<GEO>(rx, ry, rz, s.nrm[0], s.nrm[1], s.nrm[2]);
    return tabs<T>(h) < s.tol && rx * rx + ry * ry + rz * rz <= s.ap_sq;      // norm(p - c) <= aperture
}

// SphericalSurface.is_pt_on_surface (RT:1518-1535): aperture about the ORIGIN-through input axis
// AX: axis (+0, +0, 1), center (+0, +0, cz) and a finite shell_hi.  Where `on` holds, d2 <= shell_hi < inf
// makes p finite; then a = p.z up to a zero sign, q = (p.x -+ 0, p.y -+ 0, +-0), and the aperture sum
// (qx qx + qy qy) + qz qz is exactly p.x p.x + p.y p.y -- the first partial sum of d2.
template <bool AX = false, typename T>
RTPB_HD bool on_sphere(const Ray<T>& p, const DevSurface<T>& s, T* rxy_out = nullptr) {
    constexpr int GEO = AX ? kGeoAxial : kGeoGeneral;
    const T rx = axsub_x<GEO>(p.x, s.c[0]), ry = axsub_y<GEO>(p.y, s.c[1]), rz = p.z - s.c[2];
    const T rxy = rx * rx + ry * ry;
    if (rxy_out) *rxy_out = rxy;
    const T d2 = rxy + rz * rz;
    const bool on = d2 >= s.shell_lo && d2 <= s.shell_hi;                      // |norm(p - c) - |R|| < tol
    if constexpr (AX) {
        return on && rxy <= s.ap_sq;
    } else {
        const T a = p.x * s.ax[0] + p.y * s.ax[1] + p.z * s.ax[2];
        const T qx = p.x - a * s.ax[0], qy = p.y - a * s.ax[1], qz = p.z - a * s.ax[2];
        return on && qx * qx + qy * qy + qz * qz <= s.ap_sq;                    // norm(ortho) <= aperture
    }
}

// ------------------------------------------------------------------ PerfectLens (RT:1558-1801)
// The "at" plane (the lens plane, RT:1790-1793) is emitted first: it depends on r only.
// UNI: the media on both sides are uniform (Constant, or Vacuum with an ordinary wavelength on every lane of the
// wave): F, B, n1 f and n1 n1 f + n2 n2 f come from the descriptor, computed on the host by the same operations.
template <typename T, int GEO, bool UNI, typename EmitAt, class G>
RTPB_HD void lens_step(const DevSurface<T>& s, const Ray<T>& r, T n1, T n2, const Rcp<T>& iwl, EmitAt&& emit_at,
                       Ray<T>& after, G* g) {
    const T f = s.f;
    const T nx = s.nrm[0], ny = s.nrm[1], nz = s.nrm[2];
    // the "before" plane and the front focal plane share the normal, so d.n divides both (one Rcp)
    const Rcp<T> iden = make_rcp(axdot<GEO>(r.dx, r.dy, r.dz, nx, ny, nz));
    emit_at(to_plane<GEO, GEO>(r, nx, ny, nz, s.c[0], s.c[1], s.c[2], n1, false, iwl, static_cast<T*>(nullptr), &iden,
                               g));   // RT:1790-1793
    T Fx, Fy, Fz, Bx, By, Bz;
    if constexpr (UNI) {
        Fx = s.lF[0]; Fy = s.lF[1]; Fz = s.lF[2];
        Bx = s.lB[0]; By = s.lB[1]; Bz = s.lB[2];
    } else {
        Fx = s.c[0] - s.nf[0] * n1; Fy = s.c[1] - s.nf[1] * n1; Fz = s.c[2] - s.nf[2] * n1;
        Bx = s.c[0] + s.nf[0] * n2; By = s.c[1] + s.nf[1] * n2; Bz = s.c[2] + s.nf[2] * n2;
    }
    // axial (x-z plane) and uniform: the host checked F = (+0, +0, Fz) (Fy = +0), so the front focal plane has the
    // surface's center form too
    constexpr int GF = UNI ? GEO : kGeoGeneral;
    const Ray<T> rf = to_plane<GEO, GF>(r, nx, ny, nz, Fx, Fy, Fz, n1, false, iwl, static_cast<T*>(nullptr), &iden, g);
    const T dn = axdot<GEO>(rf.dx, rf.dy, rf.dz, nx, ny, nz);
    T spx, spy, spz;
    if constexpr (GEO == kGeoAxial) {
        spx = tfma(-dn, zero_s(), rf.dx);             // dx - dn * 0
        spy = tfma(-dn, zero_s(), rf.dy);
        spz = rf.dz - dn;                             // dz - dn * 1
    } else if constexpr (GEO == kGeoXZ) {
        spx = rf.dx - dn * nx;
        spy = tfma(-dn, zero_s(), rf.dy);             // dy - dn * 0
        spz = rf.dz - dn * nz;
    } else {
        spx = rf.dx - dn * nx; spy = rf.dy - dn * ny; spz = rf.dz - dn * nz;
    }
    // |s1_perp| and |r1| (RT:1704-1728): a norm squared in range takes the combined test (norm2_fast), the
    // rest the full tests -- bit-identical either way, NaN included
    const T spv = spx * spx + spy * spy + spz * spz;
    const T r1x = axsub_x<GF>(rf.x, Fx), r1y = axsub_y<GF>(rf.y, Fy), r1z = rf.z - Fz;
    const T r1v = r1x * r1x + r1y * r1y + r1z * r1z;
    T ux = r1x, uy = r1y, uz = r1z;
    T r1n;
#if defined(RTPB_FASTNORM)
    if constexpr (sizeof(T) == 8 && !G::kDefer) {
        if (__builtin_expect(norm2_fast(spv), 1)) {
            const T spn = sqrt_core(spv);
            if (spn > T(1e-12)) div3_norm<T, G, 1>(spx, spy, spz, make_rcp_in_range(spn), g);   // |s| <= norm
        } else {
            const T spn = sqrt(spv);                              // the compiler's full sequences
            if (spn > T(1e-12)) {
                spx = spx / spn; spy = spy / spn; spz = spz / spn;
            }
        }
        if (__builtin_expect(norm2_fast(r1v), 1)) {
            r1n = sqrt_core(r1v);
            div3_norm<T, G, 1>(ux, uy, uz, make_rcp_in_range(r1n), g);   // r1n >= 2^-120 (or NaN: NaN out)
        } else {
            r1n = sqrt(r1v);
            if (r1n != T(0)) {
                ux = ux / r1n; uy = uy / r1n; uz = uz / r1n;
            }
        }
    } else
#endif
    {
        const T spn = tsqrt<T>(spv, g);
        if (spn > T(1e-12)) div3_norm(spx, spy, spz, make_rcp(spn), g);
        r1n = tsqrt<T>(r1v, g);
        if (r1n != T(0)) div3_norm(ux, uy, uz, make_rcp(r1n), g);
    }
    const T sin_t1 = spx * rf.dx + spy * rf.dy + spz * rf.dz;
    Ray<T> o;
    const T h = (UNI ? s.ln1f : n1 * f) * sin_t1;                  // (n1 f) sin_t1, RT:1755
    o.x = h * spx + Bx;
    o.y = h * spy + By;
    o.z = h * spz + Bz;
    // -r1n is a norm (bounded, see NUM_IN_RANGE); with 2^-80 <= |f| < 2^120 (host bit kLensQ1) so is q1 =
    // -r1n / f: 2^-657 <= |q1| <= 2^592, or 0, inf, NaN
    const T q1 = div1<T, G, true>(-r1n, host_rcp(f, s.rf, (s.rcp_ok & 2) != 0), g);
    T sin_t2;
    if (s.rcp_ok & 8) {
        RTPB_NO_SPECULATE();
        if (s.rcp_ok & kLensQ1) sin_t2 = div1<T, G, true>(q1, host_rcp(n2, s.rn2, true), g);
        else sin_t2 = div1(q1, host_rcp(n2, s.rn2, true), g);
    } else {
        sin_t2 = q1 / n2;
    }
    const T cos_t2 = tsqrt_1m<T>(T(1) - sin_t2 * sin_t2, g);
    if constexpr (GEO == kGeoAxial) {
        o.dx = tfma(cos_t2, T(0), sin_t2 * ux);
        o.dy = tfma(cos_t2, T(0), sin_t2 * uy);
        o.dz = sin_t2 * uz + cos_t2;
    } else if constexpr (GEO == kGeoXZ) {
        o.dx = sin_t2 * ux + cos_t2 * nx;
        o.dy = tfma(cos_t2, T(0), sin_t2 * uy);       // sin_t2 uy + cos_t2 * 0
        o.dz = sin_t2 * uz + cos_t2 * nz;
    } else {
        o.dx = sin_t2 * ux + cos_t2 * nx;
        o.dy = sin_t2 * uy + cos_t2 * ny;
        o.dz = sin_t2 * uz + cos_t2 * nz;
    }
    o.wl = r.wl;
    kill_if(tabs<T>(sin_t1) > s.sin_a || tabs<T>(sin_t2) > s.sin_a, o);
    const T pw = r1x * rf.dx + r1y * rf.dy + r1z * rf.dz;
    // 2 pi / wl (RT:1773): the ray's wavelength is wl0 or NaN, and where it is NaN rf.ph is NaN already
    const T k = iwl.k;
    o.ph = rf.ph - k * n1 * pw + k * (UNI ? s.lph : n1 * n1 * f + n2 * n2 * f);
    after = to_plane<GEO, GEO>(o, nx, ny, nz, s.c[0], s.c[1], s.c[2], n2, false, iwl, static_cast<T*>(nullptr),
                               static_cast<const Rcp<T>*>(nullptr), g);
}

// The front-side test d . input_axis < 0 (RT:1187-1192).  POS_ONLY (the sweep's final-position semantics) on an
// axial surface: the sum is fma(dy, 0, dx 0) + dz, i.e. +-0 + dz, or NaN where dx or dy is infinite or NaN, so it
// is negative exactly when dz < 0 except on rows whose dx or dy is infinite or NaN -- and those get a NaN
// intersection and are killed by the on-surface test either way (only their unstored at-plane differs): dz < 0
// alone.  (A class-test form of the exact test -- dz < 0 with dx, dy finite -- measured no cheaper in the history
// kernels: the compiler then keeps register copies for the kill.)
template <int GEO, bool POS_ONLY, typename T>
RTPB_HD bool front_side_fails(const Ray<T>& r, const DevSurface<T>& s) {
    if constexpr (GEO == kGeoAxial && POS_ONLY) {
        (void)s;
        return r.dz < T(0);
    } else {
        return axdot<GEO>(r.dx, r.dy, r.dz, s.ax[0], s.ax[1], s.ax[2]) < T(0);
    }
}

// The intersection and the surface normal there (RefractingSurface / ReflectingSurface.propagate RT:1181-1186 with
// get_intersect / get_normal of FlatSurface RT:1323-1337, PlaneMirror RT:1398-1403, SphericalSurface RT:1467-1516)
// fwd (positions-only steps): for a kAxial sphere the forward-root flag (sphere_root<true>), for a flat whether the
// plane lies ahead (t >= 0 or NaN; the row is then not killed here), both for the row's final kill; other spheres
// leave it as it is
template <typename T, int KIND, int GEO, class G>
RTPB_HD void hit_and_normal(const DevSurface<T>& s, const Ray<T>& r, T n1, const Rcp<T>& iwl, G* g, T* rxy, Ray<T>& ri,
                            T& Nx, T& Ny, T& Nz, bool* fwd = nullptr) {
    if constexpr (KIND == SPHERE) {
        static_assert(GEO != kGeoXZ, "x-z plane steps: flats and PerfectLens only");
        constexpr bool AX = GEO == kGeoAxial;
        ri = sphere_hit<AX>(r, s, n1, iwl, g, static_cast<const T*>(rxy), AX ? fwd : nullptr);
        Nx = axsub_x<GEO>(ri.x, s.c[0]);                               // (p - c) / R, RT:1476
        Ny = axsub_y<GEO>(ri.y, s.c[1]);
        Nz = ri.z - s.c[2];
        if constexpr (AX) {
            // kAxial spheres have a finite shell_hi: where the on-surface test passes (the only rays whose
            // normal reaches a stored value) each |p - c| component is below sqrt(shell_hi) < 2^513, so the
            // numerators need only the lower bound of the exact range (div3_norm's single min3 test)
            // a finite nonzero radius in the shortcut range (host bits kRPos / kRNeg): no div_fixup -- the
            // numerators of every row that survives the on-surface test are finite (above)
            const Rcp<T> iR = host_rcp(s.R, s.rR, (s.rcp_ok & 1) != 0);
            if (s.rcp_ok & kRPos) {
                RTPB_NO_SPECULATE();
                div3_norm<T, G, 1>(Nx, Ny, Nz, iR, g);
            } else if (s.rcp_ok & kRNeg) {
                RTPB_NO_SPECULATE();
                div3_norm<T, G, -1>(Nx, Ny, Nz, iR, g);
            } else {
                div3_norm(Nx, Ny, Nz, iR, g);
            }
        } else {
            div3(Nx, Ny, Nz, host_rcp(s.R, s.rR, (s.rcp_ok & 1) != 0), g);
        }
    } else {                                                           // FLAT, PLANE_MIRROR
        Nx = s.nrm[0]; Ny = s.nrm[1]; Nz = s.nrm[2];
        if (fwd) {
            // positions-only steps: the backward-propagation exclusion reported (*fwd = t >= 0 or NaN) instead of
            // applied -- the caller folds it into the row's final kill (the sweep's flats: 5-7 VALU fewer per ray)
            T t;
            ri = to_plane<GEO, GEO>(r, Nx, Ny, Nz, s.c[0], s.c[1], s.c[2], n1, false, iwl, &t,
                                    static_cast<const Rcp<T>*>(nullptr), g);    // RT:1331-1337, 1398-1403
            *fwd = !(t < T(0));
        } else {
            ri = to_plane<GEO, GEO>(r, Nx, Ny, Nz, s.c[0], s.c[1], s.c[2], n1, true, iwl, static_cast<T*>(nullptr),
                                    static_cast<const Rcp<T>*>(nullptr), g);
        }
    }
}

// ------------------------------------------------------------------ one surface: (at, after)
// Refracting surfaces RT:1160-1234, reflecting RT:1238-1303, PerfectLens RT:1601-1801.
// One surface of a known kind (KIND = PERFECT_LENS, SPHERE, FLAT or PLANE_MIRROR).  The "at" plane is
// handed to emit_at as soon as it is final, so the kernel can stage it to LDS before the rest of the
// surface is computed (the PerfectLens path computes it first: it depends on r only).
// GEO: kGeoAxial for kAxial geometry (not for PLANE_MIRROR), kGeoXZ for kPlaneXZ (FLAT, PERFECT_LENS only).
// MODE kPosOnly: the spot sweep's final-position semantics (snell's TIR fill left to the next surface, see snell; the
// front-side test folded into the final kill; no "at" plane: emit_at is not called).
// rxy (kAxial spheres in kPosOnly runs): in: x x + y y of r (on_sphere's value at the previous axial surface); out:
// the same of the intersection point, for the next one.
constexpr int kPosOnly = 1;
// MODE kUniMedia: the caller guarantees rcp_ok bit 2 (the Snell ratio n1 / n2 of uniform media in the descriptor,
// e.g. the spot sweep, whose host evaluates every medium at the group's one wavelength): no per-lane division path,
// and the ratio stays a scalar operand
constexpr int kUniMedia = 2;
// MODE kNoAt: the caller stores no "at" plane (the final-plane kernels: emit_at does nothing) but keeps the full
// semantics of `after`: the front-side test and a flat's backward exclusion join the final kill of `after` instead of
// filling the intersection with NaN first -- `after` is all NaN either way (the reference refracts the NaN
// intersection into an all-NaN ray), one fill instead of three and no copy of the incoming direction
constexpr int kNoAt = 4;
template <typename T, int KIND, int GEO = kGeoGeneral, int MODE = 0, typename EmitAt, class G = GuardBranch>
RTPB_HD void surface_step(const DevSurface<T>& s, const Ray<T>& r, T n1, T n2, const Rcp<T>& iwl, EmitAt&& emit_at,
                          Ray<T>& after, G* g = nullptr, T* rxy = nullptr) {
    constexpr bool kTirFill = (MODE & kPosOnly) == 0;
    constexpr bool AX = GEO == kGeoAxial;
    if constexpr (KIND == PERFECT_LENS) {
        // uniform media: the instantiation with the focal points and constants in scalar registers (a wave-uniform
        // branch between two whole steps: merged values would cost vector registers on both paths)
        if (s.rcp_ok & kLensUni) {
            RTPB_NO_SPECULATE();
            lens_step<T, GEO, true>(s, r, n1, n2, iwl, emit_at, after, g);
        } else {
            lens_step<T, GEO, false>(s, r, n1, n2, iwl, emit_at, after, g);
        }
    } else {
        T Nx, Ny, Nz;
        Ray<T> ri;
        bool fwd = true;
        // positions only: a flat's backward exclusion joins the row's final kill (fwd), as a kAxial sphere's root
        // test does; the history steps apply it to the intersection inside to_plane (there the kill's condition is
        // the sign test the phase needs anyway: measured 2 VALU cheaper than a separate flag)
        constexpr bool kFold = (MODE & kPosOnly) != 0 || ((MODE & kNoAt) != 0 && KIND == FLAT);
        hit_and_normal<T, KIND, GEO>(s, r, n1, iwl, g, rxy, ri, Nx, Ny, Nz, kFold ? &fwd : nullptr);
        if constexpr (KIND == PLANE_MIRROR) {
            emit_at(ri);
            after = reflect(ri, Nx, Ny, Nz, g);
            kill_if(!on_flat(ri, s), after);
        } else {
            // front-side test against input_axis uses the INCOMING ray's direction (RT:1187-1192)
            bool ok;
            if constexpr ((MODE & kPosOnly) != 0) {
                // positions only: the failure joins the on-surface kill of `after` below instead of filling ri with
                // NaN first (6 register fills issued on every path) -- `after` is all NaN either way, and so is every
                // later position of the row (its next intersection reads a NaN direction); emit_at is not called
                ok = !front_side_fails<GEO, true>(r, s) && fwd;
            } else if constexpr ((MODE & kNoAt) != 0) {
                ok = !front_side_fails<GEO, false>(r, s) && fwd;           // joins the final kill (kNoAt)
            } else {
                kill_if(front_side_fails<GEO, false>(r, s), ri);
                emit_at(ri);
                ok = true;
            }
            T ratio;
            if constexpr ((MODE & kUniMedia) != 0) {
                ratio = s.nr;
            } else if (s.rcp_ok & 4) {
                RTPB_NO_SPECULATE();
                ratio = s.nr;
            } else {
                ratio = n1 / n2;
            }
            // the Snell normal of a flat is its own normal (its geometry form); a sphere's is per ray (general)
            after = snell<KIND == FLAT ? GEO : kGeoGeneral, kTirFill>(ri, Nx, Ny, Nz, ratio, g);
            if constexpr (KIND == SPHERE) ok = on_sphere<AX>(ri, s, rxy) && ok;    // (rxy is written either way)
            else ok = on_flat<GEO>(ri, s) && ok;
            kill_if(!ok, after);
        }
    }
}

// One refracting Flat / Sphere surface for ONE geometric ray at two wavelengths (two Snell ratios): the spot sweep
// traces a fan at several wavelengths from the same field point, and at the first surface every ray is the same
// for all of them -- the intersection, the normal, the front-side and on-surface tests and the tangent basis
// (snell_basis) are computed once, the refraction (snell_apply) per ratio.  kPosOnly semantics only: the phase of
// `after_b` is r's (the sweep reads positions); wl_b is the second ray's wavelength.
template <typename T, int KIND, int GEO, int MODE, class G = GuardBranch>
RTPB_HD void surface_step_pair(const DevSurface<T>& s, const Ray<T>& r, T n1, const Rcp<T>& iwl, T ratio_a, T ratio_b,
                               T wl_b, Ray<T>& after_a, Ray<T>& after_b, G* g = nullptr, T* rxy = nullptr) {
    static_assert((MODE & kPosOnly) != 0 && (KIND == SPHERE || KIND == FLAT), "refracting surfaces, positions only");
    T Nx, Ny, Nz;
    Ray<T> ri;
    bool fwd = true;
    hit_and_normal<T, KIND, GEO>(s, r, n1, iwl, g, rxy, ri, Nx, Ny, Nz, &fwd);
    const bool front_ok = !front_side_fails<GEO, true>(r, s) && fwd;     // joins the final kill, as in surface_step
    constexpr int kBasis = KIND == FLAT ? GEO : kGeoGeneral;
    const SnellBasis<T> b = snell_basis<kBasis>(ri, Nx, Ny, Nz, g);
    after_a = snell_apply<kBasis, false>(ri, Nx, Ny, Nz, b, ratio_a, g);
    after_b = snell_apply<kBasis, false>(ri, Nx, Ny, Nz, b, ratio_b, g);
    after_b.wl = wl_b;
    bool ok;
    if constexpr (KIND == SPHERE) ok = on_sphere<GEO == kGeoAxial>(ri, s, rxy) && front_ok;
    else ok = on_flat<GEO>(ri, s) && front_ok;
    kill_if(!ok, after_a);
    kill_if(!ok, after_b);
}

// The geometry form of a surface's steps from its flags (kAxial, kPlaneXZ; a mirror and any sphere not kAxial run
// the general form)
RTPB_HD int surface_geo(int kind, int32_t rcp_ok) {
    if (kind == PLANE_MIRROR) return kGeoGeneral;
    if (rcp_ok & kAxial) return kGeoAxial;
    return (kind != SPHERE && (rcp_ok & kPlaneXZ)) ? kGeoXZ : kGeoGeneral;
}

// The surface forms a kernel variant compiles (rtpb_plan::feat bit 32): every form, or only PerfectLens and Flat
// steps in the kAxial / kPlaneXZ forms (C4's OPM and the other PerfectLens relays: 4 arms instead of 9 -- fewer
// values to merge after the switch, measured 292.8 -> 272.1 VALU per ray-surface on C4, profiles/r06/x)
constexpr int kKindsAll = 0;
constexpr int kKindsLensFlat = 1;

// Any surface: a wave-uniform switch on the kind and the geometry form: calls
// step(integral_constant<int, KIND>, integral_constant<int, GEO>).  WITH_LENS = false compiles the
// PerfectLens case out (lower register pressure -> 5 waves/SIMD instead of 4); only valid for plans
// without PerfectLens surfaces (rtpb_plan::feat).  KINDS = kKindsLensFlat: only valid for plans whose feat has bit 32.
template <bool WITH_LENS, int KINDS = kKindsAll, typename T, typename Step>
RTPB_HD void dispatch_kind(const DevSurface<T>& s, Step&& step) {
    using std::integral_constant;
    const int kind = s.kind;
    const int geo = surface_geo(kind, s.rcp_ok);
    if constexpr (KINDS == kKindsLensFlat) {
        static_assert(WITH_LENS, "the lens-and-flat variant carries the PerfectLens code");
        if (kind == PERFECT_LENS) {
            if (geo == kGeoAxial) step(integral_constant<int, PERFECT_LENS>(), integral_constant<int, kGeoAxial>());
            else step(integral_constant<int, PERFECT_LENS>(), integral_constant<int, kGeoXZ>());
        } else if (geo == kGeoAxial) {
            step(integral_constant<int, FLAT>(), integral_constant<int, kGeoAxial>());
        } else {
            step(integral_constant<int, FLAT>(), integral_constant<int, kGeoXZ>());
        }
        return;
    }
    if (WITH_LENS && kind == PERFECT_LENS) {
        if constexpr (WITH_LENS) {
            if (geo == kGeoAxial) step(integral_constant<int, PERFECT_LENS>(), integral_constant<int, kGeoAxial>());
            else if (geo == kGeoXZ) step(integral_constant<int, PERFECT_LENS>(), integral_constant<int, kGeoXZ>());
            else step(integral_constant<int, PERFECT_LENS>(), integral_constant<int, kGeoGeneral>());
        }
    } else if (kind == SPHERE) {
        if (geo == kGeoAxial) step(integral_constant<int, SPHERE>(), integral_constant<int, kGeoAxial>());
        else step(integral_constant<int, SPHERE>(), integral_constant<int, kGeoGeneral>());
    } else if (kind == PLANE_MIRROR) {
        step(integral_constant<int, PLANE_MIRROR>(), integral_constant<int, kGeoGeneral>());
    } else if (geo == kGeoAxial) {
        step(integral_constant<int, FLAT>(), integral_constant<int, kGeoAxial>());
    } else if (geo == kGeoXZ) {
        step(integral_constant<int, FLAT>(), integral_constant<int, kGeoXZ>());
    } else {
        step(integral_constant<int, FLAT>(), integral_constant<int, kGeoGeneral>());
    }
}

// The (kind, geometry form) pair of dispatch_kind as one integer, and the dispatch on it: a loop can run a whole RUN
// of consecutive surfaces of one code inside one instantiation of the step (no per-surface join of the kind
// branches, so the ray's registers carry over from surface to surface without copies)
template <typename T>
RTPB_HD int surface_code(int kind, int32_t rcp_ok) {
    return 3 * kind + surface_geo(kind, rcp_ok);
}

template <bool WITH_LENS, typename Step>
RTPB_HD void dispatch_code(int code, Step&& step) {
    using std::integral_constant;
    switch (code) {
    case 3 * PERFECT_LENS + kGeoAxial:
        if constexpr (WITH_LENS) { step(integral_constant<int, PERFECT_LENS>(), integral_constant<int, kGeoAxial>()); break; }
        [[fallthrough]];
    case 3 * FLAT + kGeoAxial:
        step(integral_constant<int, FLAT>(), integral_constant<int, kGeoAxial>());
        break;
    case 3 * PERFECT_LENS + kGeoXZ:
        if constexpr (WITH_LENS) { step(integral_constant<int, PERFECT_LENS>(), integral_constant<int, kGeoXZ>()); break; }
        [[fallthrough]];
    case 3 * FLAT + kGeoXZ:
        step(integral_constant<int, FLAT>(), integral_constant<int, kGeoXZ>());
        break;
    case 3 * SPHERE + kGeoAxial:
        step(integral_constant<int, SPHERE>(), integral_constant<int, kGeoAxial>());
        break;
    case 3 * SPHERE:
        step(integral_constant<int, SPHERE>(), integral_constant<int, kGeoGeneral>());
        break;
    case 3 * PLANE_MIRROR:
        step(integral_constant<int, PLANE_MIRROR>(), integral_constant<int, kGeoGeneral>());
        break;
    case 3 * PERFECT_LENS:
        if constexpr (WITH_LENS) { step(integral_constant<int, PERFECT_LENS>(), integral_constant<int, kGeoGeneral>()); break; }
        [[fallthrough]];
    default:
        step(integral_constant<int, FLAT>(), integral_constant<int, kGeoGeneral>());
        break;
    }
}

// MODE: 0 (both planes of the surface) or kNoAt (final-plane kernels: no "at" plane); KINDS: dispatch_kind's
template <typename T, bool WITH_LENS = true, int MODE = 0, int KINDS = kKindsAll, typename EmitAt, class G = GuardBranch>
RTPB_HD void propagate_surface_emit(const DevSurface<T>& s, const Ray<T>& r, T n1, T n2, const Rcp<T>& iwl,
                                    EmitAt&& emit_at, Ray<T>& after, G* g = nullptr) {
    dispatch_kind<WITH_LENS, KINDS>(s, [&](auto kind, auto geo) {
        surface_step<T, decltype(kind)::value, decltype(geo)::value, MODE>(s, r, n1, n2, iwl, emit_at, after, g);
    });
}

template <typename T, bool WITH_LENS = true>
RTPB_HD void propagate_surface(const DevSurface<T>& s, const Ray<T>& r, T n1, T n2, Ray<T>& at, Ray<T>& after) {
    propagate_surface_emit<T, WITH_LENS>(s, r, n1, n2, make_wl_rcp(r.wl), [&](const Ray<T>& v) { at = v; }, after);
}

// ------------------------------------------------------------------ host: descriptor lowering
// Exact replacement of the on-surface square roots.  s -> RN(sqrt(s)) is monotone, so for every
// double s >= 0 (and NaN, for which both sides are false):
//   RN(sqrt(s)) <= ap                 <=>  s <= ap_sq            (ap_sq = largest such s)
//   |RN(RN(sqrt(s)) - A)| < tol       <=>  shell_lo <= s <= shell_hi
// (the second set is an interval because q -> RN(q - A) is monotone too).  The bounds are found by
// bisection over the ordered bit patterns of non-negative doubles with the host's correctly
// rounded sqrt, i.e. with the very predicates the reference evaluates (RT:1343-1346, RT:1528-1533).
// Host-only (plan build / CPU harness).
namespace host {
inline uint64_t bits(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
inline double from_bits(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }

// largest s in [lo, hi] with pred(s), given pred(lo) and !pred(hi) and pred true..false on [lo, hi]
template <class P> double last_true(P pred, double lo, double hi) {
    uint64_t a = bits(lo), b = bits(hi);
    while (b - a > 1) {
        const uint64_t m = a + (b - a) / 2;
        if (pred(from_bits(m))) a = m; else b = m;
    }
    return from_bits(a);
}

inline double sqrt_le_bound(double ap) {
    auto P = [ap](double s) { return std::sqrt(s) <= ap; };
    if (!P(0.0)) return -HUGE_VAL;
    if (P(HUGE_VAL)) return HUGE_VAL;
    return last_true(P, 0.0, HUGE_VAL);
}

inline void shell_bounds(double A, double tol, double& lo, double& hi) {
    auto P = [A, tol](double s) { return std::fabs(std::sqrt(s) - A) < tol; };
    const double s0 = A * A;
    if (!(s0 >= 0.0) || !P(s0)) { lo = HUGE_VAL; hi = -HUGE_VAL; return; }       // empty
    if (P(0.0)) lo = 0.0;
    else lo = from_bits(bits(last_true([&](double s) { return !P(s); }, 0.0, s0)) + 1);
    hi = P(HUGE_VAL) ? HUGE_VAL : last_true(P, s0, HUGE_VAL);
}
}  // namespace host

// Order (wavelength, n) pairs by wavelength with NaN keys last, as material_n's search expects.
inline void sort_table(double* pairs, int64_t n) {
    struct P { double k, v; };
    P* p = reinterpret_cast<P*>(pairs);
    std::sort(p, p + n, [](const P& a, const P& b) {
        const bool an = a.k != a.k, bn = b.k != b.k;
        if (an || bn) return !an && bn;
        return a.k < b.k;
    });
}

inline DevSurface<double> lower_surface(const rtpb_surface& s) {
    DevSurface<double> d{};
    d.kind = s.kind;
    for (int j = 0; j < 3; ++j) {
        d.c[j] = s.center[j];
        d.nrm[j] = s.normal[j];
        d.ax[j] = s.input_axis[j];
    }
    d.R = s.radius;
    d.R2 = s.radius_sq;
    d.absR = std::fabs(s.radius);
    d.ap = s.aperture;
    d.f = s.focal_len;
    d.sin_a = s.sin_alpha;
    d.tol = s.on_tol;
    d.ap_sq = host::sqrt_le_bound(s.aperture);
    host::shell_bounds(d.absR, s.on_tol, d.shell_lo, d.shell_hi);
    d.rR = 1.0 / s.radius;                       // IEEE division: RN(1/R) (inf for R = 0)
    d.rf = 1.0 / s.focal_len;
    d.rcp_ok = (host_rcp_ok(s.radius) ? 1 : 0) | (host_rcp_ok(s.focal_len) ? 2 : 0);
    if (host_rcp_ok(s.radius) && std::isfinite(s.radius) && s.radius != 0.0) d.rcp_ok |= s.radius > 0.0 ? kRPos : kRNeg;
    for (int j = 0; j < 3; ++j) d.nf[j] = s.normal[j] * s.focal_len;     // RT:1682-1687 `normal * focal_len`
    // kAxial: the exact +0 / 1 components the specialised steps rely on (bit patterns: -0 does not qualify)
    auto is_p0 = [](double v) { return host::bits(v) == 0; };
    auto z_axis = [&](const double* v) { return is_p0(v[0]) && is_p0(v[1]) && v[2] == 1.0; };
    const bool on_axis = is_p0(s.center[0]) && is_p0(s.center[1]);
    bool axial = false;
    if (d.kind == FLAT) axial = on_axis && z_axis(s.normal) && z_axis(s.input_axis);
    else if (d.kind == SPHERE) axial = on_axis && z_axis(s.input_axis) && d.shell_hi < HUGE_VAL;
    else if (d.kind == PERFECT_LENS) axial = on_axis && z_axis(s.normal);
    if (axial) {
        d.rcp_ok |= kAxial;
    } else {
        // x-z plane geometry: every vector and point the step reads has an exact +0 y component (a flat's input axis
        // drives its front-side test; a PerfectLens has none)
        const bool y0 = is_p0(s.center[1]) && is_p0(s.normal[1]);
        if ((d.kind == FLAT && y0 && is_p0(s.input_axis[1])) || (d.kind == PERFECT_LENS && y0)) d.rcp_ok |= kPlaneXZ;
    }
    if (d.kind == PERFECT_LENS && std::fabs(s.focal_len) >= 0x1p-80 && std::fabs(s.focal_len) < 0x1p120)
        d.rcp_ok |= kLensQ1;
    d.nr = 0.0;
    d.rn2 = 0.0;
    return d;
}

// The media on either side (the plan's device materials m1 = before, m2 = after): uniform when both are
// Constant (MAT:72-79: n does not depend on the wavelength, NaN included).
inline void lower_surface_media(DevSurface<double>& d, const DevMaterial<double>& m1, const DevMaterial<double>& m2) {
    // Constant: c0 for every ray; Vacuum: 1 for every ray whose wavelength squared is finite and nonzero
    auto uniform_n = [](const DevMaterial<double>& m, double& n) {
        if (m.kind == CONSTANT) { n = m.c[0]; return true; }
        if (m.kind == VACUUM) { n = 1.0; return true; }
        return false;
    };
    double n1, n2;
    if (uniform_n(m1, n1) && uniform_n(m2, n2)) {
        d.nr = n1 / n2;
        d.rn2 = 1.0 / n2;
        const int bits = 4 | (host_rcp_ok(n2) ? 8 : 0);
        // next to a Vacuum the values hold only for ordinary wavelengths: bits 4 / 8 moved to 16 / 32, which
        // the trace kernel turns into 4 / 8 when every ray of the wave has one
        d.rcp_ok |= (m1.kind == VACUUM || m2.kind == VACUUM) ? bits << 2 : bits;
        if (d.kind == PERFECT_LENS && std::isfinite(n1) && std::isfinite(n2)) {
            // the per-ray expressions of lens_step<..., false> with these n1, n2
            for (int j = 0; j < 3; ++j) {
                d.lF[j] = d.c[j] - d.nf[j] * n1;
                d.lB[j] = d.c[j] + d.nf[j] * n2;
            }
            d.ln1f = n1 * d.f;
            d.lph = n1 * n1 * d.f + n2 * n2 * d.f;
            auto is_p0 = [](double v) { return host::bits(v) == 0; };
            // the focal planes take the step's center form (lens_step: GF), so F and B must have its zeros
            const bool in_xz = is_p0(d.lF[1]) && is_p0(d.lB[1]);
            const bool on_axis = in_xz && is_p0(d.lF[0]) && is_p0(d.lB[0]);
            if ((d.rcp_ok & kAxial) ? on_axis : (d.rcp_ok & kPlaneXZ) ? in_xz : true)
                d.rcp_ok |= (m1.kind == VACUUM || m2.kind == VACUUM) ? kLensUniVac : kLensUni;
        }
    }
}

}  // namespace rtpb
