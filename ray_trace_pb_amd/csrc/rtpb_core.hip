// rtpb_core.hip -- errors, plans and device queries of the C ABI (include/rtpb.h).
//
// A plan is the reference's System plus its initial/final materials (RT:641-661) lowered to POD
// descriptors (rtpb_surface / rtpb_material); on first use per device it is uploaded as one immutable
// blob [surfaces][materials][(wavelength, n) tables] that every kernel reads through scalar loads.
#include "rtpb_internal.h"

namespace rtpbi {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

PinnedStaging& pinned_staging() {
    thread_local PinnedStaging sg;
    return sg;
}

// Blob layout: [S surfaces][S+1 materials][table pairs], each part 256-byte aligned.  Computed once at
// plan creation, so launches on any device read the offsets without synchronisation.
template <typename T>
void blob_layout(rtpb_plan& p) {
    p.off_mats = align256(p.surf.size() * sizeof(DevSurface<T>));
    p.off_table = p.off_mats + align256(p.mats.size() * sizeof(DevMaterial<T>));
    p.off_itab = p.off_table + align256(std::max<size_t>(p.table.size(), 2) * sizeof(T));
    p.blob_bytes = p.off_itab + align256(std::max<size_t>(p.itab.size(), 2) * sizeof(T));
}

// The device material descriptor of plan material k (zero-coefficient Sellmeier = VACUUM, as the
// kernels see it).
DevMaterial<double> device_material(const rtpb_plan& p, size_t k) {
    const rtpb_material& m = p.mats[k];
    DevMaterial<double> d{};
    d.kind = m.kind;
    bool zero = m.kind == RTPB_SELLMEIER;
    for (int j = 0; j < 6; ++j) {
        d.c[j] = m.c[j];
        zero = zero && m.c[j] == 0.0;
    }
    if (zero) d.kind = VACUUM;
    d.table_off = p.table_off[k];
    d.table_len = m.kind == RTPB_TABLE ? m.table_len : 0;
    return d;
}

// Indexed materials (kLdsIndexedDoubles): when every TABLE material shares one strictly increasing key
// set (NaN last allowed) and there is no POLY6 material, tabulate every material at those keys --
// TABLE materials by their own values, the others with material_n itself (host build of the kernel's
// function, -ffp-contract=off: the same IEEE operations, hence the same bits) -- and every surface's Snell
// ratio n_s / n_s+1 at those keys.
void build_indexed(rtpb_plan& p) {
    if (p.table.empty() || (p.feat & 2)) return;
    const size_t M = p.mats.size();
    int first = -1;
    for (size_t k = 0; k < M; ++k)
        if (p.mats[k].kind == RTPB_TABLE) { first = static_cast<int>(k); break; }
    if (first < 0) return;
    const int K = p.mats[first].table_len;
    const size_t S = p.surf.size();
    if (K <= 0 || static_cast<size_t>(K) * (M + 1 + S) > static_cast<size_t>(kLdsIndexedDoubles)) return;
    const double* keys0 = p.table.data() + 2 * static_cast<size_t>(p.table_off[first]);
    for (int j = 0; j < K; ++j) {
        const double kj = keys0[2 * j];
        if (kj != kj && j != K - 1) return;                               // NaN only as the last key
        if (j > 0 && kj == kj && !(keys0[2 * (j - 1)] < kj)) return;       // strictly increasing
    }
    for (size_t k = 0; k < M; ++k) {                                      // one key set for every table
        if (p.mats[k].kind != RTPB_TABLE) continue;
        if (p.mats[k].table_len != K) return;
        const double* kk = p.table.data() + 2 * static_cast<size_t>(p.table_off[k]);
        for (int j = 0; j < K; ++j) {
            const double a = kk[2 * j], b = keys0[2 * j];
            if (a != a ? b == b : std::memcmp(&a, &b, sizeof(double)) != 0) return;
        }
    }
    std::vector<double> it(static_cast<size_t>(K) * (M + 1 + S));
    for (int j = 0; j < K; ++j) it[j] = keys0[2 * j];
    for (size_t k = 0; k < M; ++k) {
        const double* kk = p.table.data() + 2 * static_cast<size_t>(p.table_off[k]);
        const DevMaterial<double> d = device_material(p, k);
        for (int j = 0; j < K; ++j)
            it[K * (k + 1) + j] = p.mats[k].kind == RTPB_TABLE ? kk[2 * j + 1]
                                                               : material_n<double, false, false>(d, keys0[2 * j], static_cast<const double*>(nullptr));
    }
    // the Snell ratio n_s / n_s+1 of every surface at every key (IEEE division: the per-lane quotient)
    for (size_t s = 0; s < S; ++s)
        for (int j = 0; j < K; ++j) it[K * (M + 1 + s) + j] = it[K * (s + 1) + j] / it[K * (s + 2) + j];
    p.itab.swap(it);
    p.nkeys = K;
    p.feat = (p.feat & ~(4 | 8)) | 16;
}

template <typename T>
std::vector<unsigned char> build_blob(const rtpb_plan& p) {
    const size_t S = p.surf.size(), M = p.mats.size(), off_mats = p.off_mats, off_table = p.off_table;
    std::vector<unsigned char> blob(p.blob_bytes, 0);
    auto* ds = reinterpret_cast<DevSurface<T>*>(blob.data());
    for (size_t k = 0; k < S; ++k) {
        DevSurface<double> d = lower_surface(p.surf[k]);
        lower_surface_media(d, device_material(p, k), device_material(p, k + 1));
        DevSurface<T>& o = ds[k];
        o.kind = d.kind;
        for (int j = 0; j < 3; ++j) {
            o.c[j] = T(d.c[j]);
            o.nrm[j] = T(d.nrm[j]);
            o.ax[j] = T(d.ax[j]);
        }
        o.R = T(d.R); o.R2 = T(d.R2); o.absR = T(d.absR); o.ap = T(d.ap); o.f = T(d.f); o.sin_a = T(d.sin_a);
        o.tol = T(d.tol); o.ap_sq = T(d.ap_sq); o.shell_lo = T(d.shell_lo); o.shell_hi = T(d.shell_hi);
        o.rR = T(d.rR); o.rf = T(d.rf); o.rcp_ok = d.rcp_ok;
        for (int j = 0; j < 3; ++j) o.nf[j] = T(d.nf[j]);
        o.nr = T(d.nr); o.rn2 = T(d.rn2);
        for (int j = 0; j < 3; ++j) {
            o.lF[j] = T(d.lF[j]);
            o.lB[j] = T(d.lB[j]);
        }
        o.ln1f = T(d.ln1f); o.lph = T(d.lph);
    }
    auto* dm = reinterpret_cast<DevMaterial<T>*>(blob.data() + off_mats);
    for (size_t k = 0; k < M; ++k) dm[k] = device_material(p, k);
    auto* tb = reinterpret_cast<T*>(blob.data() + off_table);
    for (size_t k = 0; k < p.table.size(); ++k) tb[k] = T(p.table[k]);
    auto* it = reinterpret_cast<T*>(blob.data() + p.off_itab);
    for (size_t k = 0; k < p.itab.size(); ++k) it[k] = T(p.itab[k]);
    return blob;
}

int plan_device_blob(rtpb_plan* p, int dev, void** out) {
    std::lock_guard<std::mutex> lk(p->mu);
    if (!p->blob[dev]) {
        std::vector<unsigned char> host = build_blob<double>(*p);
        DeviceGuard g(dev);
        void* d = nullptr;
        HIP_TRY(hipMalloc(&d, host.size()));
        hipError_t e = hipMemcpy(d, host.data(), host.size(), hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            (void)hipFree(d);
            return fail(RTPB_E_HIP, std::string("hipMemcpy(plan): ") + hipGetErrorString(e));
        }
        p->blob[dev] = d;
    }
    *out = p->blob[dev];
    return RTPB_OK;
}

int check_device(int dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(RTPB_E_NODEV, "no GPU device visible");
    if (dev < 0 || dev >= n || dev >= kMaxDevices)
        return fail(RTPB_E_NODEV, "device index " + std::to_string(dev) + " out of range");
    return RTPB_OK;
}

}  // namespace rtpbi

using namespace rtpbi;

extern "C" {

int rtpb_abi_version(void) { return RTPB_ABI_VERSION; }

const char* rtpb_last_error(void) { return g_last_error.c_str(); }

int rtpb_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int rtpb_plan_create(const rtpb_surface* surfaces, int32_t nsurf, const rtpb_material* materials, int32_t nmat,
                     int32_t dtype, rtpb_plan** plan_out) {
    if (!plan_out) return fail(RTPB_E_INVALID, "plan_out is NULL");
    *plan_out = nullptr;
    if (nsurf < 0 || (nsurf > 0 && !surfaces)) return fail(RTPB_E_INVALID, "bad surfaces array");
    if (nsurf > RTPB_MAX_SURFACES)
        return fail(RTPB_E_LIMIT, "more than RTPB_MAX_SURFACES (" + std::to_string(RTPB_MAX_SURFACES) + ") surfaces");
    if (nmat != nsurf + 1 || !materials)
        return fail(RTPB_E_INVALID, "length of materials should be len(surfaces) + 1");
    if (dtype != RTPB_F64 && dtype != RTPB_F32) return fail(RTPB_E_INVALID, "dtype must be RTPB_F64 or RTPB_F32");
    auto* p = new (std::nothrow) rtpb_plan();
    if (!p) return fail(RTPB_E_INVALID, "out of host memory");
    p->dtype = dtype;
    p->nsurf = nsurf;
    for (int k = 0; k < nsurf; ++k) {
        if (surfaces[k].kind < RTPB_FLAT || surfaces[k].kind > RTPB_PERFECT_LENS) {
            delete p;
            return fail(RTPB_E_INVALID, "surface " + std::to_string(k) + ": unknown kind");
        }
        p->surf.push_back(surfaces[k]);
        if (surfaces[k].kind == RTPB_PERFECT_LENS) p->feat |= 1;
    }
    for (int k = 0; k < nmat; ++k) {
        rtpb_material m = materials[k];
        if (m.kind < RTPB_CONSTANT || m.kind > RTPB_TABLE) {
            delete p;
            return fail(RTPB_E_INVALID, "material " + std::to_string(k) + ": unknown kind");
        }
        p->table_off.push_back(static_cast<int32_t>(p->table.size() / 2));
        if (m.kind == RTPB_POLY6) p->feat |= 3;
        if (m.kind == RTPB_TABLE) {
            if (m.table_len <= 0 || !m.table) {
                delete p;
                return fail(RTPB_E_INVALID, "material " + std::to_string(k) + ": empty table");
            }
            if (p->table.size() / 2 + m.table_len > RTPB_MAX_TABLE) {
                delete p;
                return fail(RTPB_E_LIMIT, "more than RTPB_MAX_TABLE wavelength table entries");
            }
            p->table.insert(p->table.end(), m.table, m.table + 2 * m.table_len);
            sort_table(p->table.data() + p->table.size() - 2 * m.table_len, m.table_len);
        }
        m.table = nullptr;
        p->mats.push_back(m);
    }
    if (!p->table.empty()) p->feat |= (p->table.size() / 2 <= static_cast<size_t>(kLdsTablePairs)) ? 4 : 8;
    if (g_indexed_materials.load()) build_indexed(*p);
    if (p->feat == 1) {
        // PerfectLens code and plain media: the lens-and-flat variant when every surface takes one of its 4 forms
        bool lens_flat = true;
        for (const rtpb_surface& s : p->surf) {
            const DevSurface<double> d = lower_surface(s);
            lens_flat = lens_flat && (d.kind == FLAT || d.kind == PERFECT_LENS) &&
                        surface_geo(d.kind, d.rcp_ok) != kGeoGeneral;
        }
        if (lens_flat) p->feat |= 32;
    }
    blob_layout<double>(*p);
    *plan_out = p;
    return RTPB_OK;
}

int rtpb_plan_destroy(rtpb_plan* plan) {
    if (!plan) return RTPB_OK;
    for (int d = 0; d < kMaxDevices; ++d) {
        if (plan->blob[d]) {
            DeviceGuard g(d);
            (void)hipFree(plan->blob[d]);
        }
    }
    delete plan;
    return RTPB_OK;
}

}  // extern "C"
