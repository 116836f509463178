// fastdiv_check.hip -- TEST INFRASTRUCTURE ONLY: runs the shared-divisor quotient helpers of
// ray_trace_pb_amd/csrc/rtpb_math.h (make_rcp / div1 / div1_as / div3 / div3_norm), its square root (tsqrt) and
// the sphere-root choice and Snell sign (sphere_root / signed_root) on the GPU over caller-supplied
// operand pairs, next to the compiler's own `a / b`, so tests/test_gpu_fastdiv.py can check that every
// quotient is bit-identical to the IEEE division (NumPy's a / b) on adversarial inputs.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -I include \
//         -o tests/native/_build/libfastdiv_check.so tests/native/fastdiv_check.hip
#include <hip/hip_runtime.h>

#include "../../ray_trace_pb_amd/csrc/rtpb_math.h"

using namespace rtpb;

namespace {

constexpr int kOut = 39;

// out: [0] div1(a, rcp(b)), [1] a / b, [2..4] div3((a, a2, a3), rcp(b)) -> x, y, z,
//      [5] div1_as(a, bb, rcp(b)) (bb = b, or NaN where kill[i]), [6] tsqrt(b), [7] tsqrt(a),
//      [8] div1(a, host_rcp(b, yh)) with yh = the host's RN(1 / b) (the descriptors' rR / rf),
//      then the GuardDefer forms (no fallback branch; a flag instead): [9] div1, [10] its flag,
//      [11..13] div3, [14] its flag, [15] tsqrt(b), [16] its flag, [17] div1_as, [18] its flag,
//      [19..21] div3_norm((a, a2, a3), rcp(their norm)), [22..24] its GuardDefer form, [25] that flag,
//      [26] sphere_root(B = a, root = tsqrt(|b|)), [27] signed_root(a, tsqrt(|b|)),
//      [28..30] unit_or_zero(a, a2, a3) (the combined norm test, NaN components of the quotient replaced by 0),
//      [31] the phase term |(a, a2, a3)| * 2 pi / b with the numerator's range implied (div1_as NUM_IN_RANGE),
//      [32..34] div3_norm((a, a2, a3), host_rcp(b, yh)) in the axial sphere normal's form: without div_fixup
//      (SIGN = +1 / -1) where b is finite, nonzero and in the divisor range, with it elsewhere,
//      [35..37] unit_near1_or_zero(a, a2, a3) (square root and reciprocal from the bit pattern of a norm squared
//      within 2^-31 of 1, unit_or_zero elsewhere),
//      [38] tsqrt_1m(1 - RN(a a))
__global__ void check_kernel(const double* a, const double* a2, const double* a3, const double* b,
                             const double* yh, const unsigned char* kill, int64_t n, double* out) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double ai = a[i], bi = b[i];
    const Rcp<double> r = make_rcp(bi);
    out[i] = div1(ai, r);
    out[n + i] = ai / bi;
    double x = ai, y = a2[i], z = a3[i];
    div3(x, y, z, r);
    out[2 * n + i] = x;
    out[3 * n + i] = y;
    out[4 * n + i] = z;
    const double bb = kill[i] ? __builtin_nan("") : bi;
    out[5 * n + i] = div1_as(ai, bb, r);
    out[6 * n + i] = tsqrt<double>(bi);
    out[7 * n + i] = tsqrt<double>(ai);
    const double mb = fabs(bi);          // host_rcp_ok (rtpb_math.h), the flag lower_surface stores
    const bool ok = (mb >= 0x1p-120 && mb < 0x1p120) || bi == 0.0 || isinf(bi) || isnan(bi);
    out[8 * n + i] = div1(ai, host_rcp(bi, yh[i], ok));
    GuardDefer g1, g2, g3, g4;
    out[9 * n + i] = div1(ai, r, &g1);
    out[10 * n + i] = g1.bad ? 1.0 : 0.0;
    double dx = ai, dy = a2[i], dz = a3[i];
    div3(dx, dy, dz, r, &g2);
    out[11 * n + i] = dx;
    out[12 * n + i] = dy;
    out[13 * n + i] = dz;
    out[14 * n + i] = g2.bad ? 1.0 : 0.0;
    out[15 * n + i] = tsqrt<double>(bi, &g3);
    out[16 * n + i] = g3.bad ? 1.0 : 0.0;
    out[17 * n + i] = div1_as(ai, bb, r, &g4);
    out[18 * n + i] = g4.bad ? 1.0 : 0.0;
    double ux = ai, uy = a2[i], uz = a3[i];
    const Rcp<double> rn = make_rcp(tsqrt<double>(ux * ux + uy * uy + uz * uz));
    div3_norm(ux, uy, uz, rn);
    out[19 * n + i] = ux;
    out[20 * n + i] = uy;
    out[21 * n + i] = uz;
    GuardDefer g5;
    double vx = ai, vy = a2[i], vz = a3[i];
    div3_norm(vx, vy, vz, rn, &g5);
    out[22 * n + i] = vx;
    out[23 * n + i] = vy;
    out[24 * n + i] = vz;
    out[25 * n + i] = g5.bad ? 1.0 : 0.0;
    const double rt = tsqrt<double>(fabs(bi));          // >= +0, +inf or NaN, as sqrt(B^2 - 4C) / sqrt(1 - m^2)
    out[26 * n + i] = sphere_root(ai, rt);
    out[27 * n + i] = signed_root(ai, rt);
    double fx = ai, fy = a2[i], fz = a3[i];
    unit_or_zero(fx, fy, fz);
    out[28 * n + i] = fx;
    out[29 * n + i] = fy;
    out[30 * n + i] = fz;
    const double dist = tsqrt<double>(ai * ai + a2[i] * a2[i] + a3[i] * a3[i]);
    out[31 * n + i] = div1_as<double, GuardBranch, true>(dist * Const<double>::two_pi, bi, r);
    double sx = ai, sy = a2[i], sz = a3[i];
    const Rcp<double> hr = host_rcp(bi, yh[i], ok);
    if (ok && bi > 0.0 && !isinf(bi)) div3_norm<double, GuardBranch, 1>(sx, sy, sz, hr);
    else if (ok && bi < 0.0 && !isinf(bi)) div3_norm<double, GuardBranch, -1>(sx, sy, sz, hr);
    else div3_norm(sx, sy, sz, hr);
    out[32 * n + i] = sx;
    out[33 * n + i] = sy;
    out[34 * n + i] = sz;
    double ex = ai, ey = a2[i], ez = a3[i];
    unit_near1_or_zero(ex, ey, ez);
    out[35 * n + i] = ex;
    out[36 * n + i] = ey;
    out[37 * n + i] = ez;
    out[38 * n + i] = tsqrt_1m<double>(1.0 - ai * ai);
}

}  // namespace

extern "C" int fastdiv_check(const double* a, const double* a2, const double* a3, const double* b,
                             const double* yh, const unsigned char* kill, int64_t n, double* out) {
    const size_t bytes = static_cast<size_t>(n) * sizeof(double);
    const double* src[5] = {a, a2, a3, b, yh};
    double* dev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    double* dout = nullptr;
    unsigned char* dk = nullptr;
    hipError_t e = hipSuccess;
    for (int k = 0; k < 5 && e == hipSuccess; ++k) {
        e = hipMalloc(&dev[k], bytes);
        if (e == hipSuccess) e = hipMemcpy(dev[k], src[k], bytes, hipMemcpyHostToDevice);
    }
    if (e == hipSuccess) e = hipMalloc(&dk, static_cast<size_t>(n));
    if (e == hipSuccess) e = hipMemcpy(dk, kill, static_cast<size_t>(n), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&dout, kOut * bytes);
    if (e == hipSuccess) {
        check_kernel<<<static_cast<unsigned>((n + 255) / 256), 256>>>(dev[0], dev[1], dev[2], dev[3], dev[4], dk, n,
                                                                      dout);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(out, dout, kOut * bytes, hipMemcpyDeviceToHost);
    for (double* p : dev) (void)hipFree(p);
    (void)hipFree(dk);
    (void)hipFree(dout);
    return e == hipSuccess ? 0 : -static_cast<int>(e);
}
