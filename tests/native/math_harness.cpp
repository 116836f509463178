// CPU harness for the kernel arithmetic -- TEST INFRASTRUCTURE ONLY (never shipped, never on the
// product path).  It instantiates ray_trace_pb_amd/csrc/rtpb_math.h -- the exact per-ray code the
// gfx950 kernel runs -- on the host, so tests/test_math_harness.py can check that arithmetic
// against the reference's golden vectors in a container without a GPU.  Built by that test with
//   g++ -O2 -std=c++17 -ffp-contract=off -fPIC -shared
#include <cmath>
#include <cstdint>
#include <vector>

#include "../../include/rtpb.h"
#include "../../ray_trace_pb_amd/csrc/rtpb_math.h"

using namespace rtpb;

extern "C" int harness_trace_f64(const rtpb_surface* surfaces, int32_t nsurf, const rtpb_material* materials,
                                 const double* in, int64_t n, double* out) {
    std::vector<DevSurface<double>> S(nsurf);
    for (int k = 0; k < nsurf; ++k) {
        const rtpb_surface& s = surfaces[k];
        DevSurface<double>& d = S[k];
        d.kind = s.kind;
        for (int j = 0; j < 3; ++j) { d.c[j] = s.center[j]; d.nrm[j] = s.normal[j]; d.ax[j] = s.input_axis[j]; }
        d.R = s.radius; d.R2 = s.radius_sq; d.absR = std::fabs(s.radius); d.ap = s.aperture;
        d.f = s.focal_len; d.sin_a = s.sin_alpha; d.tol = s.on_tol;
    }
    std::vector<DevMaterial<double>> M(nsurf + 1);
    std::vector<double> table;
    for (int k = 0; k <= nsurf; ++k) {
        const rtpb_material& m = materials[k];
        DevMaterial<double>& d = M[k];
        d.kind = m.kind;
        bool zero = m.kind == RTPB_SELLMEIER;
        for (int j = 0; j < 6; ++j) { d.c[j] = m.c[j]; zero = zero && m.c[j] == 0.0; }
        if (zero) d.kind = VACUUM;
        d.table_off = static_cast<int32_t>(table.size() / 2);
        d.table_len = m.kind == RTPB_TABLE ? m.table_len : 0;
        if (m.kind == RTPB_TABLE) table.insert(table.end(), m.table, m.table + 2 * m.table_len);
    }
    const int64_t P = 2 * nsurf + 1;
    for (int64_t i = 0; i < n; ++i) {
        const double* a = in + 8 * i;
        Ray<double> r{a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7]};
        auto put = [&](int64_t p, const Ray<double>& q) {
            double* o = out + (p * n + i) * 8;
            o[0] = q.x; o[1] = q.y; o[2] = q.z; o[3] = q.dx; o[4] = q.dy; o[5] = q.dz; o[6] = q.ph; o[7] = q.wl;
        };
        put(0, r);
        const double wl0 = r.wl;
        double n_cur = material_n<double>(M[0], wl0, table.data());
        for (int s = 0; s < nsurf; ++s) {
            const double n_next = material_n<double>(M[s + 1], wl0, table.data());
            Ray<double> at, after;
            propagate_surface<double>(S[s], r, n_cur, n_next, at, after);
            put(2 * s + 1, at);
            put(2 * s + 2, after);
            r = after;
            n_cur = n_next;
        }
    }
    (void)P;
    return 0;
}
