// rtpb_generators.hip -- get_ray_fan (RT:45-96) and get_collimated_rays (RT:99-161) written straight
// into device memory.
#include "rtpb_internal.h"

using namespace rtpbi;

namespace {

// Device ray generators.  Every angle the reference feeds to np.cos / np.sin takes only n_thetas (or
// n_disps) + nphis distinct values, so a first tiny kernel evaluates (cos, sin) once per distinct
// angle -- with the same expressions, hence the same bits -- and the generator proper is pure table
// lookups + a few multiply-adds, written through the wave's LDS tile so every store instruction
// writes 1 KiB contiguous (like the trace kernel's planes).
struct TrigArgs {
    double2* __restrict__ tab;          // [n_a] (cos, sin) of the linspace angles, then [n_b] of the phis
    int64_t n_a, n_b;
    double start, stop, step;           // numpy.linspace(start, stop, n_a)
    double phi_start;
    int32_t want_a;                     // 0: the linspace values are not angles (collimated offsets)
};

__global__ __launch_bounds__(kBlock) void trig_table_kernel(TrigArgs a) {
    const int64_t j = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (j < a.n_a) {
        if (a.want_a) {
            // numpy.linspace: start + k*step, endpoint forced to stop (num > 1)
            const double tt = (a.n_a > 1 && j == a.n_a - 1) ? a.stop : double(j) * a.step + a.start;
            a.tab[j] = make_double2(cos(tt), sin(tt));
        }
    } else if (j < a.n_a + a.n_b) {
        const int64_t ip = j - a.n_a;
        const double pp = double(ip) * 2.0 * Const<double>::pi / double(a.n_b) + a.phi_start;
        a.tab[j] = make_double2(cos(pp), sin(pp));
    }
}

// get_ray_fan (RT:45-96) on the device: ray k = iphi * n_thetas + itheta.
template <typename T>
struct FanArgs {
    T* __restrict__ out;
    const double2* __restrict__ tab;    // trig_table_kernel output
    int64_t n_thetas, nphis;
    double pt[3], c[3], ex[3], ey[3];
    double wl;
    const double* __restrict__ wls;     // per-ray wavelengths (device, ray-index order) or NULL: `wl` for all
};

template <typename T>
__global__ __launch_bounds__(kTraceBlock) void ray_fan_kernel(FanArgs<T> a) {
    __shared__ uint4 tile[kTileBytes / 16];
    const int lane = threadIdx.x & 63;
    const int64_t k = static_cast<int64_t>(blockIdx.x) * kTraceBlock + threadIdx.x;
    const int64_t total = a.n_thetas * a.nphis;
    const int64_t ray0 = k - lane;
    if (ray0 >= total) return;                           // wave-uniform exit
    if (k < total) {
        const int64_t it = k % a.n_thetas, ip = k / a.n_thetas;
        const double2 t = a.tab[it], ph = a.tab[a.n_thetas + ip];
        const double ct = t.x, st = t.y, cp = ph.x, sp = ph.y;
        Ray<double> r;
        r.x = a.pt[0]; r.y = a.pt[1]; r.z = a.pt[2];
        r.dx = a.c[0] * ct + a.ex[0] * cp * st + a.ey[0] * sp * st;
        r.dy = a.c[1] * ct + a.ex[1] * cp * st + a.ey[1] * sp * st;
        r.dz = a.c[2] * ct + a.ex[2] * cp * st + a.ey[2] * sp * st;
        r.ph = 0.0;
        r.wl = a.wls ? a.wls[k] : a.wl;                  // rays[:, 7] = wavelengths (RT:94)
        tile_write<T>(tile, lane, r);
    }
    lds_wait();
    tile_flush<T, true>(tile, a.out, ray0, total, lane);
}

// get_collimated_rays (RT:99-161) on the device: ray k = idisp * nphis + iphi, position
// pt + n1 * (off cos phi) + n2 * (off sin phi), direction = normal.
struct CollArgs {
    void* __restrict__ out;
    const double2* __restrict__ tab;    // trig_table_kernel output ([n_disps] unused, then nphis)
    int64_t n_disps, nphis;
    double pt[3], n1[3], n2[3], nrm[3];
    double start, stop, step, wl;
    const double* __restrict__ wls;     // per-ray wavelengths (device, ray-index order) or NULL: `wl` for all
    int32_t use_offsets;                // 1: offset of idisp = tab[idisp].x (the caller's np.linspace)
};

template <typename T>
__global__ __launch_bounds__(kTraceBlock) void collimated_kernel(CollArgs a) {
    __shared__ uint4 tile[kTileBytes / 16];
    const int lane = threadIdx.x & 63;
    const int64_t k = static_cast<int64_t>(blockIdx.x) * kTraceBlock + threadIdx.x;
    const int64_t total = a.n_disps * a.nphis;
    const int64_t ray0 = k - lane;
    if (ray0 >= total) return;                           // wave-uniform exit
    if (k < total) {
        const int64_t id = k / a.nphis, ip = k % a.nphis;
        const double oo = a.use_offsets ? a.tab[id].x
                          : (a.n_disps > 1 && id == a.n_disps - 1) ? a.stop : double(id) * a.step + a.start;
        const double2 ph = a.tab[a.n_disps + ip];
        const double oc = oo * ph.x, os = oo * ph.y;
        Ray<double> r;
        r.x = a.pt[0] + a.n1[0] * oc + a.n2[0] * os;
        r.y = a.pt[1] + a.n1[1] * oc + a.n2[1] * os;
        r.z = a.pt[2] + a.n1[2] * oc + a.n2[2] * os;
        r.dx = a.nrm[0]; r.dy = a.nrm[1]; r.dz = a.nrm[2];
        r.ph = 0.0;
        r.wl = a.wls ? a.wls[k] : a.wl;                  // rays[:, 7] = wavelengths (RT:159)
        tile_write<T>(tile, lane, r);
    }
    lds_wait();
    tile_flush<T, true>(tile, static_cast<T*>(a.out), ray0, total, lane);
}


// Generator tables on the device: (cos, sin) pairs [n_a] then [n_b].  With host tables (the caller's
// own np.cos / np.sin / np.linspace values) they are copied; otherwise trig_table_kernel evaluates
// them with the device's libm (within an ulp of the host's).
int gen_tables(double2** tab, int64_t n_a, int64_t n_b, const double* host_a, const double* host_b, int a_pairs,
               const TrigArgs& ta, hipStream_t st) {
    const size_t bytes = size_t(n_a + n_b) * sizeof(double2);
    HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(tab), bytes, st));
    if (host_a || host_b) {
        PinnedStaging& g_pinned = pinned_staging();
        int rc = g_pinned.reserve(bytes);
        if (rc) return rc;
        double2* h = reinterpret_cast<double2*>(g_pinned.buf);
        for (int64_t j = 0; j < n_a; ++j)
            h[j] = a_pairs ? make_double2(host_a[2 * j], host_a[2 * j + 1]) : make_double2(host_a[j], 0.0);
        for (int64_t j = 0; j < n_b; ++j) h[n_a + j] = make_double2(host_b[2 * j], host_b[2 * j + 1]);
        return g_pinned.upload(*tab, bytes, st);
    }
    TrigArgs a = ta;
    a.tab = *tab;
    hipLaunchKernelGGL(trig_table_kernel, dim3(static_cast<unsigned>((n_a + n_b + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, st, a);
    HIP_TRY(hipGetLastError());
    return RTPB_OK;
}

int fan_impl(int32_t device, int32_t dtype, void* rays_out, const double pt[3], double theta_max, int64_t n_thetas,
             int64_t nphis, const double c[3], const double* ex_in, const double* ey_in, const double* theta_cs,
             const double* phi_cs, double wavelength, const double* wls, void* stream) {
    int rc = check_device(device);
    if (rc) return rc;
    if (reinterpret_cast<uintptr_t>(wls) % 8) return fail(RTPB_E_INVALID, "wavelengths must be 8-byte aligned");
    if (n_thetas <= 0 || nphis <= 0 || !rays_out || !pt || !c) return fail(RTPB_E_INVALID, "bad ray-fan arguments");
    if ((theta_cs == nullptr) != (phi_cs == nullptr)) return fail(RTPB_E_INVALID, "pass both trig tables or neither");
    if (reinterpret_cast<uintptr_t>(rays_out) % 16) return fail(RTPB_E_INVALID, "rays_out must be 16-byte aligned");
    if (dtype != RTPB_F64 && dtype != RTPB_F32) return fail(RTPB_E_INVALID, "bad dtype");
    double ex[3], ey[3];
    if (ex_in && ey_in) {
        for (int j = 0; j < 3; ++j) { ex[j] = ex_in[j]; ey[j] = ey_in[j]; }
    } else {
        // enx = cross((0,1,0), c) / |.|; eny = cross(c, enx)   (RT:79-81)
        ex[0] = 1.0 * c[2] - 0.0 * c[1]; ex[1] = 0.0 * c[0] - 0.0 * c[2]; ex[2] = 0.0 * c[1] - 1.0 * c[0];
        const double en = std::sqrt(ex[0] * ex[0] + ex[1] * ex[1] + ex[2] * ex[2]);
        for (double& v : ex) v = v / en;
        ey[0] = c[1] * ex[2] - c[2] * ex[1]; ey[1] = c[2] * ex[0] - c[0] * ex[2]; ey[2] = c[0] * ex[1] - c[1] * ex[0];
    }
    DeviceGuard g(device);
    const int64_t total = n_thetas * nphis;
    hipStream_t st = static_cast<hipStream_t>(stream);
    TrigArgs ta{};
    ta.n_a = n_thetas;
    ta.n_b = nphis;
    ta.start = -theta_max;
    ta.stop = theta_max;
    ta.step = n_thetas > 1 ? (theta_max - (-theta_max)) / double(n_thetas - 1) : 0.0;
    ta.phi_start = 0.0;
    ta.want_a = 1;
    double2* tab = nullptr;
    rc = gen_tables(&tab, n_thetas, nphis, theta_cs, phi_cs, 1, ta, st);
    if (rc) return rc;
    const unsigned blocks = static_cast<unsigned>((total + kTraceBlock - 1) / kTraceBlock);
    auto go = [&](auto tag) {
        using T = decltype(tag);
        FanArgs<T> a{};
        a.out = static_cast<T*>(rays_out);
        a.tab = tab;
        a.n_thetas = n_thetas;
        a.nphis = nphis;
        for (int j = 0; j < 3; ++j) {
            a.pt[j] = pt[j]; a.c[j] = c[j]; a.ex[j] = ex[j]; a.ey[j] = ey[j];
        }
        a.wl = wavelength;
        a.wls = wls;
        hipLaunchKernelGGL(ray_fan_kernel<T>, dim3(blocks), dim3(kTraceBlock), 0, st, a);
    };
    if (dtype == RTPB_F64) go(double{});
    else go(float{});
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipFreeAsync(tab, st));
    return RTPB_OK;
}

int collimated_impl(int32_t device, int32_t dtype, void* rays_out, const double pt[3], double displacement_max,
                    int64_t n_disps, int64_t nphis, double phi_start, const double nv[3], const double* n1_in,
                    const double* n2_in, const double* offsets, const double* phi_cs, double wavelength,
                    const double* wls, void* stream) {
    int rc = check_device(device);
    if (rc) return rc;
    if (reinterpret_cast<uintptr_t>(wls) % 8) return fail(RTPB_E_INVALID, "wavelengths must be 8-byte aligned");
    if (n_disps <= 0 || nphis <= 0 || !rays_out || !pt || !nv)
        return fail(RTPB_E_INVALID, "bad collimated-ray arguments");
    if ((offsets == nullptr) != (phi_cs == nullptr)) return fail(RTPB_E_INVALID, "pass both tables or neither");
    if (reinterpret_cast<uintptr_t>(rays_out) % 16) return fail(RTPB_E_INVALID, "rays_out must be 16-byte aligned");
    if (dtype != RTPB_F64 && dtype != RTPB_F32) return fail(RTPB_E_INVALID, "bad dtype");
    CollArgs a{};
    a.out = rays_out;
    a.n_disps = n_disps;
    a.nphis = nphis;
    double n1[3], n2[3];
    if (n1_in && n2_in) {
        for (int j = 0; j < 3; ++j) { n1[j] = n1_in[j]; n2[j] = n2_in[j]; }
    } else {
        // n1 = (0,1,0) x normal, or normal x (1,0,0) when that vanishes; n2 = normal x n1 (RT:135-144)
        n1[0] = 1.0 * nv[2] - 0.0 * nv[1]; n1[1] = 0.0 * nv[0] - 0.0 * nv[2]; n1[2] = 0.0 * nv[1] - 1.0 * nv[0];
        if (std::sqrt(n1[0] * n1[0] + n1[1] * n1[1] + n1[2] * n1[2]) == 0.0) {
            n1[0] = nv[1] * 0.0 - nv[2] * 0.0;
            n1[1] = nv[2] * 1.0 - nv[0] * 0.0;
            n1[2] = nv[0] * 0.0 - nv[1] * 1.0;
        }
        const double l1 = std::sqrt(n1[0] * n1[0] + n1[1] * n1[1] + n1[2] * n1[2]);
        for (double& v : n1) v = v / l1;
        n2[0] = nv[1] * n1[2] - nv[2] * n1[1]; n2[1] = nv[2] * n1[0] - nv[0] * n1[2];
        n2[2] = nv[0] * n1[1] - nv[1] * n1[0];
        const double l2 = std::sqrt(n2[0] * n2[0] + n2[1] * n2[1] + n2[2] * n2[2]);
        for (double& v : n2) v = v / l2;
    }
    for (int j = 0; j < 3; ++j) {
        a.pt[j] = pt[j]; a.n1[j] = n1[j]; a.n2[j] = n2[j]; a.nrm[j] = nv[j];
    }
    a.start = -displacement_max;
    a.stop = displacement_max;
    a.step = n_disps > 1 ? (displacement_max - (-displacement_max)) / double(n_disps - 1) : 0.0;
    a.use_offsets = offsets != nullptr;
    a.wl = wavelength;
    a.wls = wls;
    DeviceGuard g(device);
    hipStream_t st = static_cast<hipStream_t>(stream);
    TrigArgs ta{};
    ta.n_a = n_disps;
    ta.n_b = nphis;
    ta.phi_start = phi_start;
    ta.want_a = 0;
    double2* tab = nullptr;
    rc = gen_tables(&tab, n_disps, nphis, offsets, phi_cs, 0, ta, st);
    if (rc) return rc;
    a.tab = tab;
    const unsigned blocks = static_cast<unsigned>((n_disps * nphis + kTraceBlock - 1) / kTraceBlock);
    if (dtype == RTPB_F64) hipLaunchKernelGGL(collimated_kernel<double>, dim3(blocks), dim3(kTraceBlock), 0, st, a);
    else hipLaunchKernelGGL(collimated_kernel<float>, dim3(blocks), dim3(kTraceBlock), 0, st, a);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipFreeAsync(tab, st));
    return RTPB_OK;
}

}  // namespace

extern "C" {

int rtpb_ray_fan(int32_t device, int32_t dtype, void* rays_out, const double pt[3], double theta_max,
                 int64_t n_thetas, int64_t nphis, const double center_ray[3], double wavelength, void* stream) {
    return fan_impl(device, dtype, rays_out, pt, theta_max, n_thetas, nphis, center_ray, nullptr, nullptr, nullptr,
                    nullptr, wavelength, nullptr, stream);
}

int rtpb_ray_fan_tables(int32_t device, int32_t dtype, void* rays_out, const double pt[3], int64_t n_thetas,
                        int64_t nphis, const double center_ray[3], const double ex[3], const double ey[3],
                        const double* theta_cos_sin, const double* phi_cos_sin, double wavelength, void* stream) {
    if (!ex || !ey || !theta_cos_sin || !phi_cos_sin) return fail(RTPB_E_INVALID, "NULL table argument");
    return fan_impl(device, dtype, rays_out, pt, 0.0, n_thetas, nphis, center_ray, ex, ey, theta_cos_sin, phi_cos_sin,
                    wavelength, nullptr, stream);
}

int rtpb_ray_fan_tables_wl(int32_t device, int32_t dtype, void* rays_out, const double pt[3], int64_t n_thetas,
                           int64_t nphis, const double center_ray[3], const double ex[3], const double ey[3],
                           const double* theta_cos_sin, const double* phi_cos_sin, const double* wavelengths,
                           void* stream) {
    if (!ex || !ey || !theta_cos_sin || !phi_cos_sin || !wavelengths)
        return fail(RTPB_E_INVALID, "NULL table or wavelength argument");
    return fan_impl(device, dtype, rays_out, pt, 0.0, n_thetas, nphis, center_ray, ex, ey, theta_cos_sin, phi_cos_sin,
                    0.0, wavelengths, stream);
}

int rtpb_collimated_rays(int32_t device, int32_t dtype, void* rays_out, const double pt[3], double displacement_max,
                         int64_t n_disps, int64_t nphis, double phi_start, const double normal[3], double wavelength,
                         void* stream) {
    return collimated_impl(device, dtype, rays_out, pt, displacement_max, n_disps, nphis, phi_start, normal, nullptr,
                           nullptr, nullptr, nullptr, wavelength, nullptr, stream);
}

int rtpb_collimated_rays_tables(int32_t device, int32_t dtype, void* rays_out, const double pt[3], int64_t n_disps,
                                int64_t nphis, const double normal[3], const double n1[3], const double n2[3],
                                const double* offsets, const double* phi_cos_sin, double wavelength, void* stream) {
    if (!n1 || !n2 || !offsets || !phi_cos_sin) return fail(RTPB_E_INVALID, "NULL table argument");
    return collimated_impl(device, dtype, rays_out, pt, 0.0, n_disps, nphis, 0.0, normal, n1, n2, offsets, phi_cos_sin,
                           wavelength, nullptr, stream);
}

int rtpb_collimated_rays_tables_wl(int32_t device, int32_t dtype, void* rays_out, const double pt[3],
                                   int64_t n_disps, int64_t nphis, const double normal[3], const double n1[3],
                                   const double n2[3], const double* offsets, const double* phi_cos_sin,
                                   const double* wavelengths, void* stream) {
    if (!n1 || !n2 || !offsets || !phi_cos_sin || !wavelengths)
        return fail(RTPB_E_INVALID, "NULL table or wavelength argument");
    return collimated_impl(device, dtype, rays_out, pt, 0.0, n_disps, nphis, 0.0, normal, n1, n2, offsets, phi_cos_sin,
                           0.0, wavelengths, stream);
}

}  // extern "C"
