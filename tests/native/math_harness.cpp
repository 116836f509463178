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
