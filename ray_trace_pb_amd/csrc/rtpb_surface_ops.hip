// rtpb_surface_ops.hip -- single-surface operations outside the fused trace: propagate_ray2plane
// (RT:241-306) and the front-side / Snell / reflection kernels that complete RefractingSurface and
// ReflectingSurface.propagate (RT:1160-1303) around a user subclass's own geometry hooks.
#include "rtpb_internal.h"

using namespace rtpbi;

namespace {

// propagate_ray2plane (RT:241-306) as a standalone operation: per-ray or broadcast plane normal/center,
// material n(lambda) from a lowered descriptor, optional exclusion of backward propagation; also
// returns the propagation parameter t.
struct PlaneArgs {
    const void* __restrict__ in;
    void* __restrict__ out;
    double* __restrict__ ts;
    const double* __restrict__ nrm;   // 3 or 3*n doubles
    const double* __restrict__ ctr;
    const DevMaterial<double>* __restrict__ mat;
    const double* __restrict__ table;
    int64_t n;
    int32_t nrm_per_ray, ctr_per_ray, exclude;
};

template <typename TS>
__global__ __launch_bounds__(kTraceBlock) void plane_kernel(PlaneArgs a) {
    __shared__ uint4 tile[kTileBytes / 16];
    const int lane = threadIdx.x & 63;
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kTraceBlock + threadIdx.x;
    const int64_t ray0 = i - lane;
    if (ray0 >= a.n) return;                             // wave-uniform exit
    if (i < a.n) {
        const Ray<double> r = load_ray<TS, RTPB_AOS>(static_cast<const TS*>(a.in), i, 0);
        const double* nv = a.nrm + (a.nrm_per_ray ? 3 * i : 0);
        const double* cv = a.ctr + (a.ctr_per_ray ? 3 * i : 0);
        DevMaterial<double> m = *a.mat;
        const double n = material_n<double>(m, r.wl, a.table);
        double t;
        const Ray<double> o = to_plane(r, nv[0], nv[1], nv[2], cv[0], cv[1], cv[2], n, a.exclude != 0,
                                                  make_rcp(r.wl), &t);
        tile_write<TS>(tile, lane, o);
        if (a.ts) a.ts[i] = t;
    }
    lds_wait();
    tile_flush<TS, true>(tile, static_cast<TS*>(a.out), ray0, a.n, lane);
}

// RefractingSurface / ReflectingSurface.propagate around a user Surface subclass's own geometry
// hooks (RT:1160-1234, RT:1238-1303): the caller evaluates get_intersect / get_normal /
// is_pt_on_surface; these kernels do the front-side test and the Snell / reflection step.
struct HookArgs {
    const void* __restrict__ rays;      // previous plane (N x 8)
    const void* __restrict__ hits;      // get_intersect result (N x 8)
    const void* __restrict__ normals;   // get_normal result (N x 3)
    const uint8_t* __restrict__ on;     // is_pt_on_surface result (N), NULL = all on
    void* __restrict__ out;
    const DevSurface<double>* __restrict__ surf;
    const DevMaterial<double>* __restrict__ mats;
    const double* __restrict__ table;
    int64_t n;
    int32_t mode;
};

template <typename TS>
__global__ __launch_bounds__(kTraceBlock) void front_side_kernel(HookArgs a) {
    __shared__ uint4 tile[kTileBytes / 16];
    const int lane = threadIdx.x & 63;
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kTraceBlock + threadIdx.x;
    const int64_t ray0 = i - lane;
    if (ray0 >= a.n) return;                             // wave-uniform exit
    if (i < a.n) {
        const DevSurface<double> s = load_surface<double>((cptr<DevSurface<double>>)(a.surf));
        const Ray<double> r = load_ray<TS, RTPB_AOS>(static_cast<const TS*>(a.rays), i, 0);
        Ray<double> h = load_ray<TS, RTPB_AOS>(static_cast<const TS*>(a.hits), i, 0);
        if (r.dx * s.ax[0] + r.dy * s.ax[1] + r.dz * s.ax[2] < 0.0) kill(h);  // RT:1184-1192
        tile_write<TS>(tile, lane, h);
    }
    lds_wait();
    tile_flush<TS, true>(tile, static_cast<TS*>(a.out), ray0, a.n, lane);   // hits_out may alias hits
}

template <typename TS>
__global__ __launch_bounds__(kTraceBlock) void interact_kernel(HookArgs a) {
    __shared__ uint4 tile[kTileBytes / 16];
    const int lane = threadIdx.x & 63;
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kTraceBlock + threadIdx.x;
    const int64_t ray0 = i - lane;
    if (ray0 >= a.n) return;                             // wave-uniform exit
    if (i < a.n) {
        const Ray<double> h = load_ray<TS, RTPB_AOS>(static_cast<const TS*>(a.hits), i, 0);
        const TS* nv = static_cast<const TS*>(a.normals) + 3 * i;
        const double Nx = nv[0], Ny = nv[1], Nz = nv[2];
        Ray<double> o;
        if (a.mode == RTPB_REFLECT) {
            o = reflect<double>(h, Nx, Ny, Nz);                                      // RT:1266-1289
        } else {
            const cptr<DevMaterial<double>> mp = (cptr<DevMaterial<double>>)(a.mats);
            const double n1 = material_n<double>(load_material<double>(mp), h.wl, a.table);
            const double n2 = material_n<double>(load_material<double>(mp + 1), h.wl, a.table);
            o = snell(h, Nx, Ny, Nz, n1 / n2);                              // RT:1194-1221
        }
        if (a.on && !a.on[i]) kill(o);                                               // RT:1225-1226, 1293-1294
        tile_write<TS>(tile, lane, o);
    }
    lds_wait();
    tile_flush<TS, true>(tile, static_cast<TS*>(a.out), ray0, a.n, lane);
}

}  // namespace

extern "C" {

int rtpb_propagate_plane(int32_t device, int32_t dtype, const void* rays_in, int64_t n_rays, const double* normal,
                         int32_t normal_per_ray, const double* center, int32_t center_per_ray,
                         const rtpb_material* material, int32_t exclude_backward, void* rays_out, double* ts_out,
                         void* workspace, int64_t workspace_bytes, void* stream) {
    int rc = check_device(device);
    if (rc) return rc;
    if (dtype != RTPB_F64 && dtype != RTPB_F32) return fail(RTPB_E_INVALID, "bad dtype");
    if (n_rays < 0 || !material || !normal || !center) return fail(RTPB_E_INVALID, "bad propagate-plane arguments");
    if (n_rays == 0) return RTPB_OK;
    if (!rays_in || !rays_out) return fail(RTPB_E_INVALID, "NULL ray buffer");
    if ((reinterpret_cast<uintptr_t>(rays_in) | reinterpret_cast<uintptr_t>(rays_out)) % 16)
        return fail(RTPB_E_INVALID, "ray buffers must be 16-byte aligned");
    if (material->kind < RTPB_CONSTANT || material->kind > RTPB_TABLE) return fail(RTPB_E_INVALID, "bad material kind");
    const int64_t ntab = material->kind == RTPB_TABLE ? material->table_len : 0;
    if (material->kind == RTPB_TABLE && (ntab <= 0 || !material->table))
        return fail(RTPB_E_INVALID, "empty material table");
    // workspace (device): [DevMaterial<double>][table pairs], staged with one async H2D copy
    const size_t need = align256(sizeof(DevMaterial<double>)) + size_t(2 * std::max<int64_t>(ntab, 1)) * sizeof(double);
    if (!workspace || workspace_bytes < static_cast<int64_t>(need))
        return fail(RTPB_E_INVALID, "workspace too small (need " + std::to_string(need) + " bytes)");
    std::vector<unsigned char> host(need, 0);
    DevMaterial<double> dm{};
    dm.kind = material->kind;
    bool zero = material->kind == RTPB_SELLMEIER;
    for (int j = 0; j < 6; ++j) {
        dm.c[j] = material->c[j];
        zero = zero && material->c[j] == 0.0;
    }
    if (zero) dm.kind = VACUUM;
    dm.table_off = 0;
    dm.table_len = static_cast<int32_t>(ntab);
    std::memcpy(host.data(), &dm, sizeof(dm));
    if (ntab) {
        double* t = reinterpret_cast<double*>(host.data() + align256(sizeof(dm)));
        std::memcpy(t, material->table, size_t(2 * ntab) * sizeof(double));
        sort_table(t, ntab);
    }
    DeviceGuard g(device);
    hipStream_t st = static_cast<hipStream_t>(stream);
    HIP_TRY(hipMemcpyAsync(workspace, host.data(), need, hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));      // `host` is a pageable temporary
    PlaneArgs a{};
    a.in = rays_in;
    a.out = rays_out;
    a.ts = ts_out;
    a.nrm = normal;
    a.ctr = center;
    a.mat = reinterpret_cast<const DevMaterial<double>*>(workspace);
    a.table = reinterpret_cast<const double*>(static_cast<char*>(workspace) + align256(sizeof(dm)));
    a.n = n_rays;
    a.nrm_per_ray = normal_per_ray;
    a.ctr_per_ray = center_per_ray;
    a.exclude = exclude_backward;
    const unsigned blocks = static_cast<unsigned>((n_rays + kTraceBlock - 1) / kTraceBlock);
    if (dtype == RTPB_F64) hipLaunchKernelGGL(plane_kernel<double>, dim3(blocks), dim3(kTraceBlock), 0, st, a);
    else hipLaunchKernelGGL(plane_kernel<float>, dim3(blocks), dim3(kTraceBlock), 0, st, a);
    HIP_TRY(hipGetLastError());
    return RTPB_OK;
}

namespace {
int hook_launch(const rtpb_plan* plan_c, int32_t device, bool interact, int32_t mode, const void* rays,
                const void* hits, const void* normals, const uint8_t* on, int64_t n, void* out, void* stream) {
    auto* plan = const_cast<rtpb_plan*>(plan_c);
    if (!plan) return fail(RTPB_E_INVALID, "plan is NULL");
    int rc = check_device(device);
    if (rc) return rc;
    if (plan->nsurf < 1 || plan->mats.size() < 2)
        return fail(RTPB_E_INVALID, "surface-hook plans need one surface and two materials");
    if (mode != RTPB_REFRACT && mode != RTPB_REFLECT) return fail(RTPB_E_INVALID, "bad mode");
    if (n < 0) return fail(RTPB_E_INVALID, "n < 0");
    if (n == 0) return RTPB_OK;
    if (!hits || !out || (interact ? !normals : !rays)) return fail(RTPB_E_INVALID, "NULL ray buffer");
    if ((reinterpret_cast<uintptr_t>(hits) | reinterpret_cast<uintptr_t>(out) |
         reinterpret_cast<uintptr_t>(interact ? nullptr : rays)) % 16)
        return fail(RTPB_E_INVALID, "ray buffers must be 16-byte aligned");
    DeviceGuard g(device);
    void* blob = nullptr;
    rc = plan_device_blob(plan, device, &blob);
    if (rc) return rc;
    HookArgs a{};
    a.rays = rays;
    a.hits = hits;
    a.normals = normals;
    a.on = on;
    a.out = out;
    a.surf = static_cast<const DevSurface<double>*>(blob);
    a.mats = reinterpret_cast<const DevMaterial<double>*>(static_cast<char*>(blob) + plan->off_mats);
    a.table = reinterpret_cast<const double*>(static_cast<char*>(blob) + plan->off_table);
    a.n = n;
    a.mode = mode;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const unsigned blocks = static_cast<unsigned>((n + kTraceBlock - 1) / kTraceBlock);
    const bool f64 = plan->dtype == RTPB_F64;
    if (interact) {
        if (f64) hipLaunchKernelGGL(interact_kernel<double>, dim3(blocks), dim3(kTraceBlock), 0, st, a);
        else hipLaunchKernelGGL(interact_kernel<float>, dim3(blocks), dim3(kTraceBlock), 0, st, a);
    } else {
        if (f64) hipLaunchKernelGGL(front_side_kernel<double>, dim3(blocks), dim3(kTraceBlock), 0, st, a);
        else hipLaunchKernelGGL(front_side_kernel<float>, dim3(blocks), dim3(kTraceBlock), 0, st, a);
    }
    HIP_TRY(hipGetLastError());
    return RTPB_OK;
}
}  // namespace

int rtpb_front_side(const rtpb_plan* plan, int32_t device, const void* rays, const void* hits, int64_t n,
                    void* hits_out, void* stream) {
    return hook_launch(plan, device, false, RTPB_REFRACT, rays, hits, nullptr, nullptr, n, hits_out, stream);
}

int rtpb_interact(const rtpb_plan* plan, int32_t device, int32_t mode, const void* hits, const void* normals,
                  const uint8_t* on_surface, int64_t n, void* out, void* stream) {
    return hook_launch(plan, device, true, mode, nullptr, hits, normals, on_surface, n, out, stream);
}

}  // extern "C"
