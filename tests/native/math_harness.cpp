// CPU harness for the kernel arithmetic -- TEST INFRASTRUCTURE ONLY (never shipped, never on the
// product path).  It instantiates ray_trace_pb_amd/csrc/rtpb_math.h -- the exact per-ray code the
// gfx950 kernel runs -- on the host, so tests/test_math_harness.py can check that arithmetic
// against the reference's golden vectors in a container without a GPU.  Built by that test with
//   g++ -O2 -std=c++17 -ffp-contract=off -fPIC -shared
#include <cmath>
#include <cstdint>
#include <vector>

#include "rtpb.h"
#include "../../ray_trace_pb_amd/csrc/rtpb_math.h"

using namespace rtpb;

// TS = storage type of the ray buffers; arithmetic is float64 like the kernel
template <typename TS>
static int harness_trace(const rtpb_surface* surfaces, int32_t nsurf, const rtpb_material* materials, const TS* in,
                         int64_t n, TS* out) {
    using T = double;
    std::vector<DevSurface<T>> S(nsurf);
    for (int k = 0; k < nsurf; ++k) S[k] = lower_surface(surfaces[k]);
    std::vector<DevMaterial<T>> M(nsurf + 1);
    std::vector<T> table;
    for (int k = 0; k <= nsurf; ++k) {
        const rtpb_material& m = materials[k];
        DevMaterial<T>& d = M[k];
        d.kind = m.kind;
        bool zero = m.kind == RTPB_SELLMEIER;
        for (int j = 0; j < 6; ++j) { d.c[j] = T(m.c[j]); zero = zero && m.c[j] == 0.0; }
        if (zero) d.kind = VACUUM;
        d.table_off = static_cast<int32_t>(table.size() / 2);
        d.table_len = m.kind == RTPB_TABLE ? m.table_len : 0;
        if (m.kind == RTPB_TABLE) {
            for (int j = 0; j < 2 * m.table_len; ++j) table.push_back(T(m.table[j]));
            sort_table(table.data() + table.size() - 2 * m.table_len, m.table_len);
        }
    }
    for (int k = 0; k < nsurf; ++k) lower_surface_media(S[k], M[k], M[k + 1]);
    const int64_t P = 2 * nsurf + 1;
    for (int64_t i = 0; i < n; ++i) {
        const TS* a = in + 8 * i;
        Ray<T> r{a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7]};
        auto put = [&](int64_t p, const Ray<T>& q) {
            TS* o = out + (p * n + i) * 8;
            o[0] = TS(q.x); o[1] = TS(q.y); o[2] = TS(q.z); o[3] = TS(q.dx); o[4] = TS(q.dy); o[5] = TS(q.dz);
            o[6] = TS(q.ph); o[7] = TS(q.wl);
        };
        put(0, r);
        const T wl0 = r.wl;
        // the trace kernel's per-wave Vacuum test for a one-ray wave: an ordinary wavelength turns the Vacuum-side
        // uniform-media bits into the plain ones (rtpb_trace_kernel.h, vac_one)
        const T w2 = wl0 * wl0;
        const bool vac_one = w2 != T(0) && w2 - w2 == T(0);
        T n_cur = material_n<T>(M[0], wl0, table.data());
        for (int s = 0; s < nsurf; ++s) {
            const T n_next = material_n<T>(M[s + 1], wl0, table.data());
            Ray<T> at, after;
            DevSurface<T> d = S[s];
            if ((d.rcp_ok & 16) && vac_one) d.rcp_ok |= 4 | ((d.rcp_ok & 32) ? 8 : 0);
            if ((d.rcp_ok & kLensUniVac) && vac_one) d.rcp_ok |= kLensUni;
            propagate_surface<T>(d, r, n_cur, n_next, at, after);
            put(2 * s + 1, at);
            put(2 * s + 2, after);
            r = after;
            n_cur = n_next;
        }
    }
    (void)P;
    return 0;
}

extern "C" int harness_trace_f64(const rtpb_surface* s, int32_t ns, const rtpb_material* m, const double* in,
                                 int64_t n, double* out) {
    return harness_trace<double>(s, ns, m, in, n, out);
}

extern "C" int harness_trace_f32(const rtpb_surface* s, int32_t ns, const rtpb_material* m, const float* in,
                                 int64_t n, float* out) {
    return harness_trace<float>(s, ns, m, in, n, out);
}

// on-surface thresholds of lower_surface (rtpb_math.h): out = {ap_sq, shell_lo, shell_hi}
extern "C" void harness_bounds(double aperture, double abs_radius, double tol, double* out) {
    out[0] = host::sqrt_le_bound(aperture);
    host::shell_bounds(abs_radius, tol, out[1], out[2]);
}

// rcp_ok flags lower_surface (rtpb_math.h) gives a surface (kAxial = 64: the axial-geometry steps)
extern "C" int harness_surface_flags(const rtpb_surface* s) { return lower_surface(*s).rcp_ok; }

// The spot sweep's shared first surface (surface_step_pair, rtpb_math.h) against two separate steps, on the host:
// n rays through surface s at Snell ratios ra and rb (uniform media), kPosOnly semantics.  out: [n][4][6] -- the
// pair's two rays, then the two separate steps' rays (x, y, z, dx, dy, dz each).
template <int K, int AX>
static void pair_vs_steps(const DevSurface<double>& base, double ra, double rb, const double* in, int64_t n,
                          double* out) {
    constexpr int kMode = kPosOnly | kUniMedia;
    DevSurface<double> da = base, db = base;
    da.nr = ra;
    db.nr = rb;
    da.rcp_ok |= 4;
    db.rcp_ok |= 4;
    for (int64_t i = 0; i < n; ++i) {
        const double* a = in + 8 * i;
        const Ray<double> r{a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7]};
        const Rcp<double> iwl = make_wl_rcp(r.wl);
        Ray<double> res[4];
        double rxy[3] = {r.x * r.x + r.y * r.y, r.x * r.x + r.y * r.y, r.x * r.x + r.y * r.y};
        const bool carry = K == SPHERE && AX == kGeoAxial;
        surface_step_pair<double, K, AX, kMode>(da, r, 1.0, iwl, ra, rb, r.wl, res[0], res[1],
                                                static_cast<GuardBranch*>(nullptr), carry ? &rxy[0] : nullptr);
        auto none = [](const Ray<double>&) {};
        surface_step<double, K, AX, kMode>(da, r, 1.0, 1.0, iwl, none, res[2], static_cast<GuardBranch*>(nullptr),
                                           carry ? &rxy[1] : nullptr);
        surface_step<double, K, AX, kMode>(db, r, 1.0, 1.0, iwl, none, res[3], static_cast<GuardBranch*>(nullptr),
                                           carry ? &rxy[2] : nullptr);
        for (int k = 0; k < 4; ++k) {
            double* o = out + (i * 4 + k) * 6;
            o[0] = res[k].x; o[1] = res[k].y; o[2] = res[k].z; o[3] = res[k].dx; o[4] = res[k].dy; o[5] = res[k].dz;
        }
    }
}

extern "C" int harness_pair_vs_steps(const rtpb_surface* s, double ra, double rb, const double* in, int64_t n,
                                     double* out) {
    const DevSurface<double> d = lower_surface(*s);
    const bool ax = (d.rcp_ok & kAxial) != 0;
    if (d.kind == SPHERE) {
        if (ax) pair_vs_steps<SPHERE, kGeoAxial>(d, ra, rb, in, n, out);
        else pair_vs_steps<SPHERE, kGeoGeneral>(d, ra, rb, in, n, out);
    } else if (d.kind == FLAT) {
        if (ax) pair_vs_steps<FLAT, kGeoAxial>(d, ra, rb, in, n, out);
        else if (d.rcp_ok & kPlaneXZ) pair_vs_steps<FLAT, kGeoXZ>(d, ra, rb, in, n, out);
        else pair_vs_steps<FLAT, kGeoGeneral>(d, ra, rb, in, n, out);
    } else {
        return -1;
    }
    return 0;
}

// A positions-only step (the spot sweep's kPosOnly | kUniMedia semantics: forward-root kill of kAxial spheres, no TIR
// position fill, front-side test folded into the final kill) against the full step of the history kernels, on the
// host: n rays through surface s at the uniform Snell ratio `ratio`.  out: [n][2][6] -- the positions-only ray, then
// the full step's "after" ray (x, y, z, dx, dy, dz each).
template <int K, int AX>
static void pos_vs_full(DevSurface<double> d, double ratio, const double* in, int64_t n, double* out) {
    d.nr = ratio;
    d.rcp_ok |= 4;
    for (int64_t i = 0; i < n; ++i) {
        const double* a = in + 8 * i;
        const Ray<double> r{a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7]};
        const Rcp<double> iwl = make_wl_rcp(r.wl);
        auto none = [](const Ray<double>&) {};
        Ray<double> res[2];
        double rxy = r.x * r.x + r.y * r.y;
        constexpr bool carry = K == SPHERE && AX == kGeoAxial;
        surface_step<double, K, AX, kPosOnly | kUniMedia>(d, r, 1.0, 1.0, iwl, none, res[0],
                                                           static_cast<GuardBranch*>(nullptr), carry ? &rxy : nullptr);
        surface_step<double, K, AX, 0>(d, r, 1.0, 1.0, iwl, none, res[1]);
        for (int k = 0; k < 2; ++k) {
            double* o = out + (i * 2 + k) * 6;
            o[0] = res[k].x; o[1] = res[k].y; o[2] = res[k].z; o[3] = res[k].dx; o[4] = res[k].dy; o[5] = res[k].dz;
        }
    }
}

extern "C" int harness_pos_vs_full(const rtpb_surface* s, double ratio, const double* in, int64_t n, double* out) {
    const DevSurface<double> d = lower_surface(*s);
    const bool ax = (d.rcp_ok & kAxial) != 0;
    if (d.kind == SPHERE) {
        if (ax) pos_vs_full<SPHERE, kGeoAxial>(d, ratio, in, n, out);
        else pos_vs_full<SPHERE, kGeoGeneral>(d, ratio, in, n, out);
    } else if (d.kind == FLAT) {
        if (ax) pos_vs_full<FLAT, kGeoAxial>(d, ratio, in, n, out);
        else if (d.rcp_ok & kPlaneXZ) pos_vs_full<FLAT, kGeoXZ>(d, ratio, in, n, out);
        else pos_vs_full<FLAT, kGeoGeneral>(d, ratio, in, n, out);
    } else {
        return -1;
    }
    return 0;
}

// the sweep's fan-index division (rtpb_spot_sweep): multiplier and shift for divisor d and group size g
extern "C" void harness_sweep_divisor(int64_t d, int64_t g, uint32_t* mul, int32_t* shift) {
    sweep_divisor(d, g, *mul, *shift);
}
