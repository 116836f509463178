// rtpb_trace.hip -- host side of the hot path: rtpb_trace / rtpb_trace_host (the C ABI replacing
// System.ray_trace's surface loop RT:658-659), the pinned host-buffer pipeline, tuning knobs and launch
// timing.  The kernel itself is rtpb_trace_kernel.h, instantiated per (input, storage) type pair in
// rtpb_trace_<tin>_<ts>.hip.

#include "rtpb_internal.h"

using namespace rtpbi;

namespace rtpbi {
// tuning knobs (rtpb_set_tuning); process-wide, read by launch_trace
std::atomic<int> g_aos_staging{1};
std::atomic<int> g_nt_stores{1};
std::atomic<int> g_stage_input{0};
std::atomic<int> g_host_chunk_mib{128};
std::atomic<int> g_indexed_materials{1};          // read at plan creation (rtpb_plan_create)
}  // namespace rtpbi

namespace {

int popcount128(uint64_t lo, uint64_t hi) { return __builtin_popcountll(lo) + __builtin_popcountll(hi); }

// ---------------------------------------------------------------------------------- timing
struct TimingState {
    bool on = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
};
thread_local TimingState g_timing;


int trace_impl(rtpb_plan* plan, int dev, const void* in, int in_dtype, int64_t n, int il, int64_t in_fs, void* out,
               int ol, int64_t out_ps, int64_t out_fs, uint64_t lo, uint64_t hi, hipStream_t st,
               int32_t* miss = nullptr) {
    void* blob = nullptr;
    int rc = plan_device_blob(plan, dev, &blob);
    if (rc) return rc;
    if (n == 0) return RTPB_OK;
    auto run = [&](auto tin, auto tag) -> hipError_t {
        using TIN = decltype(tin);
        using TS = decltype(tag);
        TraceArgs<TIN, TS> a{};
        a.in = static_cast<const TIN*>(in);
        a.out = static_cast<TS*>(out);
        a.surf = reinterpret_cast<const DevSurface<double>*>(blob);
        a.mats = reinterpret_cast<const DevMaterial<double>*>(static_cast<char*>(blob) + plan->off_mats);
        a.table = reinterpret_cast<const double*>(static_cast<char*>(blob) + plan->off_table);
        a.itab = reinterpret_cast<const double*>(static_cast<char*>(blob) + plan->off_itab);
        a.miss = miss;
        a.n = n;
        a.in_fs = in_fs;
        a.out_ps = out_ps;
        a.out_fs = out_fs;
        a.mask_lo = lo;
        a.mask_hi = hi;
        a.nsurf = plan->nsurf;
        a.ntable = static_cast<int32_t>(plan->table.size() / 2);
        a.nkeys = plan->nkeys;
        return launch_trace<TIN, TS>(a, il, ol, plan->feat, st);
    };
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (g_timing.on) {
        if (!g_timing.pool.empty()) {
            std::tie(e0, e1) = g_timing.pool.back();
            g_timing.pool.pop_back();
        } else {
            HIP_TRY(hipEventCreate(&e0));
            HIP_TRY(hipEventCreate(&e1));
        }
        HIP_TRY(hipEventRecord(e0, st));
    }
    hipError_t e;
    if (plan->dtype == RTPB_F64) e = in_dtype == RTPB_F64 ? run(double{}, double{}) : run(float{}, double{});
    else e = in_dtype == RTPB_F64 ? run(double{}, float{}) : run(float{}, float{});
    if (e != hipSuccess) return fail(RTPB_E_HIP, std::string("trace kernel launch: ") + hipGetErrorString(e));
    if (g_timing.on) {
        HIP_TRY(hipEventRecord(e1, st));
        g_timing.pending.emplace_back(e0, e1);
    }
    return RTPB_OK;
}

// ---------------------------------------------------------------------------------- host pipeline
// NumPy-in / NumPy-out path.  Pageable host memory caps PCIe copies at ~11 GB/s, so each device keeps a
// cached set of pinned staging buffers and runs a two-deep pipeline over ray chunks:
//   CPU: input chunk k -> pinned_in[k%2];  GPU stream: H2D(k) -> trace(k) -> D2H(k) into pinned_out[k%2]
//   CPU (overlapping GPU chunk k): scatter pinned_out[(k-1)%2] into every output plane, multi-threaded.
struct HostStage {
    std::mutex mu;                 // one rtpb_trace_host call per device at a time
    hipStream_t st = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    void* pin_in[2] = {nullptr, nullptr};
    void* pin_out[2] = {nullptr, nullptr};
    void* d_in[2] = {nullptr, nullptr};
    void* d_out[2] = {nullptr, nullptr};
    size_t in_bytes = 0, out_bytes = 0;
};
HostStage g_stage[kMaxDevices];

int stage_reserve(HostStage& hs, size_t in_bytes, size_t out_bytes) {
    if (!hs.st) {
        HIP_TRY(hipStreamCreateWithFlags(&hs.st, hipStreamNonBlocking));
        for (auto& e : hs.ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    if (in_bytes > hs.in_bytes || out_bytes > hs.out_bytes) {
        for (int k = 0; k < 2; ++k) {
            if (hs.pin_in[k]) (void)hipHostFree(hs.pin_in[k]);
            if (hs.pin_out[k]) (void)hipHostFree(hs.pin_out[k]);
            if (hs.d_in[k]) (void)hipFree(hs.d_in[k]);
            if (hs.d_out[k]) (void)hipFree(hs.d_out[k]);
            hs.pin_in[k] = hs.pin_out[k] = hs.d_in[k] = hs.d_out[k] = nullptr;
        }
        hs.in_bytes = hs.out_bytes = 0;
        for (int k = 0; k < 2; ++k) {
            HIP_TRY(hipHostMalloc(&hs.pin_in[k], in_bytes, hipHostMallocDefault));
            HIP_TRY(hipHostMalloc(&hs.pin_out[k], out_bytes, hipHostMallocDefault));
            HIP_TRY(hipMalloc(&hs.d_in[k], in_bytes));
            HIP_TRY(hipMalloc(&hs.d_out[k], out_bytes));
        }
        hs.in_bytes = in_bytes;
        hs.out_bytes = out_bytes;
    }
    return RTPB_OK;
}

// parallel memcpy of `count` equally sized pieces (piece i: dst_i <- src_i) over T threads
void parallel_scatter(char* out, const char* staged, int nslots, int64_t slot_stride_bytes, int64_t piece_bytes,
                      int T) {
    const int64_t total = piece_bytes * nslots;
    // a thread per >= 8 MiB: spawning threads costs ~10-20 us each, a small scatter is one memcpy
    T = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(T, total >> 23)));
    const int64_t per = (total + T - 1) / T;
    auto job = [&](int t) {
        int64_t lo = t * per, hi = std::min<int64_t>(total, lo + per);
        while (lo < hi) {
            const int64_t s = lo / piece_bytes, off = lo % piece_bytes;
            const int64_t len = std::min<int64_t>(hi - lo, piece_bytes - off);
            std::memcpy(out + s * slot_stride_bytes + off, staged + s * piece_bytes + off, static_cast<size_t>(len));
            lo += len;
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(job, t);
    job(0);
    for (auto& x : th) x.join();
}

bool is_pinned_host(const void* p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeHost;
}

// rec_in / rec: bytes per input record (in_dtype) / per output record (the plan's storage type)
int host_shard_pipeline(rtpb_plan* plan, int dev, const char* in, int in_dtype, char* out, int64_t n_rays, int64_t a,
                        int64_t b, size_t rec_in, size_t rec, int nslots, uint64_t lo, uint64_t hi, int T) {
    HostStage& hs = g_stage[dev];
    std::lock_guard<std::mutex> lk(hs.mu);
    DeviceGuard guard(dev);
    // an early error return must not leave copies into the caller's buffers (or into staging buffers a
    // later call may free) in flight: drain the stream first
#define HIP_TRY_SYNC(expr)                                                                     \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) {                                                                \
            (void)hipStreamSynchronize(hs.st);                                                 \
            return fail(RTPB_E_HIP, std::string(#expr ": ") + hipGetErrorString(e_));          \
        }                                                                                      \
    } while (0)
    // pinned (page-locked, e.g. torch pin_memory) output: DMA every plane slice straight into place
    const bool direct = is_pinned_host(out) && is_pinned_host(out + (int64_t(nslots) * n_rays * rec - 1));
    // ~128 MiB of output per chunk (at least 64k rays), two chunks in flight
    // chunk: ~g_host_chunk_mib of input + output per chunk (at least 64k rays), two chunks in flight
    const int64_t target = int64_t(g_host_chunk_mib.load()) << 20;
    const int64_t chunk = std::min<int64_t>(b - a, std::max<int64_t>(1 << 16, target / int64_t(nslots * rec + rec_in)));
    int rc = stage_reserve(hs, chunk * rec_in, chunk * rec * nslots);
    if (rc) return rc;
    const int64_t nchunks = (b - a + chunk - 1) / chunk;
    auto scatter = [&](int64_t k) -> int {
        const int buf = static_cast<int>(k & 1);
        HIP_TRY(hipEventSynchronize(hs.ev[buf]));
        if (direct) return RTPB_OK;
        const int64_t c0 = a + k * chunk, m = std::min<int64_t>(chunk, b - c0);
        parallel_scatter(out + c0 * rec, static_cast<const char*>(hs.pin_out[buf]), nslots,
                         static_cast<int64_t>(n_rays * rec), static_cast<int64_t>(m * rec), T);
        return RTPB_OK;
    };
    for (int64_t k = 0; k < nchunks; ++k) {
        const int buf = static_cast<int>(k & 1);
        const int64_t c0 = a + k * chunk, m = std::min<int64_t>(chunk, b - c0);
        // pin_in[buf] / pin_out[buf] were last used by chunk k-2, whose event was waited in scatter(k-2)
        parallel_scatter(static_cast<char*>(hs.pin_in[buf]), in + c0 * rec_in, 1, 0, static_cast<int64_t>(m * rec_in), T);
        HIP_TRY_SYNC(hipMemcpyAsync(hs.d_in[buf], hs.pin_in[buf], m * rec_in, hipMemcpyHostToDevice, hs.st));
        rc = trace_impl(plan, dev, hs.d_in[buf], in_dtype, m, RTPB_AOS, 0, hs.d_out[buf], RTPB_AOS, m * 8, 0, lo, hi,
                        hs.st);
        if (rc) {
            (void)hipStreamSynchronize(hs.st);
            return rc;
        }
        if (direct)
            HIP_TRY_SYNC(hipMemcpy2DAsync(out + c0 * rec, n_rays * rec, hs.d_out[buf], m * rec, m * rec, nslots,
                                          hipMemcpyDeviceToHost, hs.st));
        else
            HIP_TRY_SYNC(hipMemcpyAsync(hs.pin_out[buf], hs.d_out[buf], m * rec * nslots, hipMemcpyDeviceToHost, hs.st));
        HIP_TRY_SYNC(hipEventRecord(hs.ev[buf], hs.st));
        if (k >= 1) {
            rc = scatter(k - 1);
            if (rc) {
                (void)hipStreamSynchronize(hs.st);
                return rc;
            }
        }
    }
    return scatter(nchunks - 1);
#undef HIP_TRY_SYNC
}

}  // namespace

extern "C" {

int rtpb_shutdown(void) {
    rtpb_oneshot_clear();                          // the one-shot entry points' cached plans (rtpb_oneshot.hip)
    (void)rtpb_buffer_trim();                      // pooled history buffers (rtpb_buffers.hip)
    for (int d = 0; d < kMaxDevices; ++d) {
        HostStage& hs = g_stage[d];
        std::lock_guard<std::mutex> lk(hs.mu);
        if (!hs.st) continue;
        DeviceGuard g(d);
        (void)hipStreamSynchronize(hs.st);
        for (int k = 0; k < 2; ++k) {
            if (hs.pin_in[k]) (void)hipHostFree(hs.pin_in[k]);
            if (hs.pin_out[k]) (void)hipHostFree(hs.pin_out[k]);
            if (hs.d_in[k]) (void)hipFree(hs.d_in[k]);
            if (hs.d_out[k]) (void)hipFree(hs.d_out[k]);
            hs.pin_in[k] = hs.pin_out[k] = hs.d_in[k] = hs.d_out[k] = nullptr;
            (void)hipEventDestroy(hs.ev[k]);
            hs.ev[k] = nullptr;
        }
        (void)hipStreamDestroy(hs.st);
        hs.st = nullptr;
        hs.in_bytes = hs.out_bytes = 0;
    }
    return RTPB_OK;
}

int rtpb_trace(const rtpb_plan* plan_c, int32_t device, const void* rays_in, int32_t in_dtype, int64_t n_rays,
               int32_t in_layout, int64_t in_field_stride, void* out, int32_t out_layout, int64_t out_plane_stride,
               int64_t out_field_stride, uint64_t plane_mask_lo, uint64_t plane_mask_hi, void* stream) {
    return rtpb_trace_checked(plan_c, device, rays_in, in_dtype, n_rays, in_layout, in_field_stride, out, out_layout,
                              out_plane_stride, out_field_stride, plane_mask_lo, plane_mask_hi, stream, nullptr);
}

static_assert(sizeof(rtpb_trace_call) == 5 * 8 + 6 * 8 + 4 * 4, "rtpb_trace_call: no padding (bindings mirror it)");

int rtpb_trace_packed(const rtpb_trace_call* c) {
    if (!c) return fail(RTPB_E_INVALID, "call is NULL");
    return rtpb_trace_checked(c->plan, c->device, c->rays_in, c->in_dtype, c->n_rays, c->in_layout, c->in_field_stride,
                              c->out, c->out_layout, c->out_plane_stride, c->out_field_stride, c->plane_mask_lo,
                              c->plane_mask_hi, c->stream, c->table_miss);
}

int rtpb_trace_checked(const rtpb_plan* plan_c, int32_t device, const void* rays_in, int32_t in_dtype,
                       int64_t n_rays, int32_t in_layout, int64_t in_field_stride, void* out, int32_t out_layout,
                       int64_t out_plane_stride, int64_t out_field_stride, uint64_t plane_mask_lo,
                       uint64_t plane_mask_hi, void* stream, int32_t* table_miss) {
    auto* plan = const_cast<rtpb_plan*>(plan_c);
    if (!plan) return fail(RTPB_E_INVALID, "plan is NULL");
    int rc = check_device(device);
    if (rc) return rc;
    if (n_rays < 0) return fail(RTPB_E_INVALID, "n_rays < 0");
    const int nplanes = 2 * plan->nsurf + 1;
    if (nplanes < 128 && ((nplanes >= 64 ? (plane_mask_hi >> (nplanes - 64)) : (plane_mask_hi | (plane_mask_lo >> nplanes))) != 0))
        return fail(RTPB_E_INVALID, "plane mask selects planes beyond 2*nsurf");
    const int nslots = popcount128(plane_mask_lo, plane_mask_hi);
    if (in_layout != RTPB_AOS && in_layout != RTPB_SOA) return fail(RTPB_E_INVALID, "bad in_layout");
    if (out_layout != RTPB_AOS && out_layout != RTPB_SOA) return fail(RTPB_E_INVALID, "bad out_layout");
    if (in_dtype != RTPB_F64 && in_dtype != RTPB_F32) return fail(RTPB_E_INVALID, "bad in_dtype");
    if (in_dtype != plan->dtype && in_layout != RTPB_AOS)
        return fail(RTPB_E_INVALID, "SOA input must have the plan's storage type");
    if (n_rays > 0 && !rays_in) return fail(RTPB_E_INVALID, "rays_in is NULL");
    if (n_rays > 0 && nslots > 0 && !out) return fail(RTPB_E_INVALID, "out is NULL");
    const size_t w = plan->dtype == RTPB_F64 ? 8 : 4;
    if (in_layout == RTPB_AOS && (reinterpret_cast<uintptr_t>(rays_in) % 16))
        return fail(RTPB_E_INVALID, "AOS rays_in must be 16-byte aligned");
    if (out_layout == RTPB_AOS && nslots > 0 &&
        ((reinterpret_cast<uintptr_t>(out) % 16) || ((out_plane_stride * w) % 16)))
        return fail(RTPB_E_INVALID, "AOS out and its plane stride must be 16-byte aligned");
    if (nslots > 1 && out_plane_stride < 8 * n_rays) return fail(RTPB_E_INVALID, "out_plane_stride < 8*n_rays");
    if (in_layout == RTPB_SOA && in_field_stride < n_rays) return fail(RTPB_E_INVALID, "in_field_stride < n_rays");
    if (out_layout == RTPB_SOA && out_field_stride < n_rays) return fail(RTPB_E_INVALID, "out_field_stride < n_rays");
    DeviceGuard g(device);
    return trace_impl(plan, device, rays_in, in_dtype, n_rays, in_layout, in_field_stride, out, out_layout,
                      out_plane_stride, out_field_stride, plane_mask_lo, plane_mask_hi, static_cast<hipStream_t>(stream),
                      table_miss);
}

int rtpb_trace_host(const rtpb_plan* plan_c, const void* rays_in, int32_t in_dtype, int64_t n_rays, void* out,
                    uint64_t plane_mask_lo, uint64_t plane_mask_hi, const int32_t* devices, int32_t n_devices) {
    auto* plan = const_cast<rtpb_plan*>(plan_c);
    if (!plan) return fail(RTPB_E_INVALID, "plan is NULL");
    if (n_rays < 0) return fail(RTPB_E_INVALID, "n_rays < 0");
    if (in_dtype != RTPB_F64 && in_dtype != RTPB_F32) return fail(RTPB_E_INVALID, "bad in_dtype");
    std::vector<int> devs;
    if (!devices || n_devices <= 0) devs.push_back(0);
    else devs.assign(devices, devices + n_devices);
    for (int d : devs) {
        int rc = check_device(d);
        if (rc) return rc;
    }
    const int nslots = popcount128(plane_mask_lo, plane_mask_hi);
    if (n_rays == 0 || nslots == 0) return RTPB_OK;
    if (!rays_in || !out) return fail(RTPB_E_INVALID, "NULL host buffer");
    const size_t rec = 8 * (plan->dtype == RTPB_F64 ? 8 : 4);
    const size_t rec_in = 8 * (in_dtype == RTPB_F64 ? 8 : 4);
    const int G = static_cast<int>(devs.size());
    // host threads that scatter staged chunks into the caller's array, per device
    const unsigned hw = std::max(2u, std::thread::hardware_concurrency());
    const int copy_threads = static_cast<int>(std::max(2u, std::min(16u, hw / static_cast<unsigned>(G))));
    std::vector<int> rcs(G, RTPB_OK);
    std::vector<std::string> errs(G);
    auto worker = [&](int g) {
        const int dev = devs[g];
        const int64_t a = n_rays * g / G, b = n_rays * (g + 1) / G;
        if (b <= a) return;
        rcs[g] = host_shard_pipeline(plan, dev, static_cast<const char*>(rays_in), in_dtype, static_cast<char*>(out),
                                     n_rays, a, b, rec_in, rec, nslots, plane_mask_lo, plane_mask_hi, copy_threads);
        if (rcs[g]) errs[g] = g_last_error;
    };
    if (G == 1) {
        worker(0);
    } else {
        std::vector<std::thread> th;
        for (int g = 0; g < G; ++g) th.emplace_back(worker, g);
        for (auto& t : th) t.join();
    }
    for (int g = 0; g < G; ++g)
        if (rcs[g]) return fail(rcs[g], "device " + std::to_string(devs[g]) + ": " + errs[g]);
    return RTPB_OK;
}

int rtpb_set_tuning(const char* key, int64_t value) {
    if (!key) return fail(RTPB_E_INVALID, "key is NULL");
    if (std::strcmp(key, "aos_staging") == 0) {
        if (value < 0 || value > 2) return fail(RTPB_E_INVALID, "aos_staging must be 0, 1 or 2");
        g_aos_staging.store(static_cast<int>(value));
        return RTPB_OK;
    }
    if (std::strcmp(key, "nt_stores") == 0) {
        g_nt_stores.store(value != 0);
        return RTPB_OK;
    }
    if (std::strcmp(key, "stage_input") == 0) {
        g_stage_input.store(value != 0);
        return RTPB_OK;
    }
    if (std::strcmp(key, "host_chunk_mib") == 0) {
        if (value < 1 || value > 4096) return fail(RTPB_E_INVALID, "host_chunk_mib must be in [1, 4096]");
        g_host_chunk_mib.store(static_cast<int>(value));
        return RTPB_OK;
    }
    if (std::strcmp(key, "indexed_materials") == 0) {
        g_indexed_materials.store(value != 0);
        return RTPB_OK;
    }
    if (std::strcmp(key, "buffer_pool_buffers") == 0) return set_buffer_pool_keep(value);
    if (std::strcmp(key, "buffer_dead_va_limit") == 0) return set_buffer_dead_va_limit(value);
    return fail(RTPB_E_INVALID, std::string("unknown tuning key ") + key);
}

int rtpb_timing_enable(int32_t on) {
    g_timing.on = on != 0;
    return RTPB_OK;
}

int rtpb_timing_collect(double* total_ms, int64_t* launches) {
    double tot = 0.0;
    int64_t cnt = 0;
    for (auto& pr : g_timing.pending) {
        HIP_TRY(hipEventSynchronize(pr.second));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, pr.first, pr.second));
        tot += ms;
        ++cnt;
        g_timing.pool.push_back(pr);
    }
    g_timing.pending.clear();
    if (total_ms) *total_ms = tot;
    if (launches) *launches = cnt;
    return RTPB_OK;
}

}  // extern "C"
