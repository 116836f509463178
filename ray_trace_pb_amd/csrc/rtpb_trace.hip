// rtpb_trace.hip -- the hot path: one fused HIP kernel traces every ray through every surface of a
// plan (replacing System.ray_trace's surface loop RT:658-659 and the per-surface NumPy ufunc chains of
// RT:1160-1801), plus the host-buffer pipeline, tuning knobs and launch timing of the C ABI.
// Hot path: ONE kernel launch traces every ray through every surface of the system (replacing the
// Python surface loop RT:658-659 and the per-surface NumPy ufunc chains of RT:1160-1801).  One lane
// owns one ray for the whole system:
//   * the ray record (8 values) is read once from HBM (AOS: 16-byte vector loads; SOA: coalesced
//     per-field loads) and kept in VGPRs;
//   * surface and material descriptors are wave-uniform -- they are read through constant-address-
//     space pointers with uniform indices, i.e. scalar loads (s_load) into SGPRs, once per wave;
//   * n(lambda) of every material is evaluated once per ray (the reference re-evaluates it 3-4x per
//     surface, MAT:39-51 via RT:297/1213/1512) and carried across the surface loop;
//   * every requested history plane is written exactly once, at its final location -- no
//     O(S^2 N) re-copying of the history (RT:1229-1232);
//   * per-ray failures are NaN selects, never divergent early exits, so a wave stays converged.
// The surface loop is wave-uniform (same system for every lane), so its `kind` switches never diverge.
//
// Precision: arithmetic is ALWAYS float64 in registers (the reference's numerics); the storage type TS
// of the ray buffers is float64 or float32.  float32 storage halves the HBM bytes (the bound) while the
// values stay the correctly rounded float64 results: a float32 trace equals the float64 reference on the
// float32-rounded input, rounded once on store.
//
// Memory roofline: per ray the kernel moves 8w bytes in and 8w bytes per stored plane out
// (w = sizeof(TS)); see DESIGN.md for the algorithmic-byte accounting used by bench.py.

#include "rtpb_internal.h"

using namespace rtpbi;

namespace {

// Workgroup size per variant: the LDS-staged AoS kernels run one wave per workgroup (see kTraceBlock);
// the direct-store variants (SoA output, unstaged AoS) keep four-wave workgroups, which measured faster
// for their strided stores (C5 SoA: 0.53 vs 0.69 ms).
constexpr int trace_block(int out_layout, int store) {
    return (out_layout == RTPB_AOS && (store & 1)) ? kTraceBlock : 256;
}

// The fused multi-surface trace: one lane = one ray through all surfaces (float64 arithmetic, TS
// storage).  STORE: bit 0 = LDS-staged AOS stores (OUT_LAYOUT == AOS only), bit 1 = non-temporal global
// stores for the staged tiles, bit 2 = LDS-staged AOS input loads, bit 3 = final plane only.
// FEAT: bit 0 = PerfectLens code, bit 1 = RTPB_POLY6 code compiled in, bit 2 = TABLE materials looked up
// in an LDS copy of the plan's table (dynamic LDS, copied at launch), bit 3 = TABLE materials looked up
// in global memory.  Leaving out what a plan does not use lowers register pressure (f64 staged: 92 VGPRs
// without the PerfectLens code, 100 with both), 10-15 % faster when compute-bound, and without a global
// table lookup the surface loop never waits on the vmcnt counter, which on gfx950 would also wait for
// every history store in flight (see kLdsTablePairs).  rtpb_plan::feat picks the variant.
template <typename TS, int IN_LAYOUT, int OUT_LAYOUT, int STORE, int WPE, int FEAT>
__global__ __launch_bounds__(trace_block(OUT_LAYOUT, STORE)) __attribute__((amdgpu_waves_per_eu(WPE, 8)))
void trace_kernel(TraceArgs<TS> a) {
    constexpr int kB = trace_block(OUT_LAYOUT, STORE);
    using T = double;
    constexpr bool kStaged = (STORE & 1) && OUT_LAYOUT == RTPB_AOS;
    constexpr bool kNT = (STORE & 2) != 0;
    // STORE bit 3: only the final plane is stored (planes='final'): no per-surface store logic, one
    // LDS tile, fewer live registers (the C5 / spot-diagram and focus-finding mode)
    constexpr bool kFinal = (STORE & 8) != 0;
    constexpr bool kLens = (FEAT & 1) != 0, kPoly = (FEAT & 2) != 0;
    constexpr bool kTabLds = (FEAT & 12) == 4, kTabGlobal = (FEAT & 8) != 0;
    extern __shared__ double lds_table[];                // FEAT bit 2: the plan's (wavelength, n) pairs
    if constexpr (kTabLds) {
        // before any wave can leave: the unstaged variants run four-wave workgroups and need the barrier
        for (int k = threadIdx.x; k < 2 * a.ntable; k += kB) lds_table[k] = a.table[k];
        if constexpr (kB > 64) __syncthreads();
    }
    // per wave: "at" and "after" tiles of 64 records (4 KiB f64, 2 KiB f32: the LDS budget allows 5 f64 /
    // 10 f32 waves per SIMD in the all-planes mode, so registers set the f32 occupancy)
    __shared__ uint4 tiles[kB / 64][kFinal ? 1 : 2][kTileBytes / 16 * sizeof(TS) / 8];
    const int lane = threadIdx.x & 63;
    // one block of kB rays (the whole kernel, or one step of the persistent experiment's loop)
    auto body = [&](const int64_t blk) {
#if defined(RTPB_EXP_XCD_REMAP)             // experiment only: each XCD takes a contiguous range of ray blocks
    // workgroups are dispatched round-robin over the 8 XCDs: block b runs on XCD b % 8
    const uint32_t nb = gridDim.x, per = nb / 8, xcd = blockIdx.x % 8, k = blockIdx.x / 8;
    const uint32_t bid = blockIdx.x < per * 8 ? xcd * per + k : blockIdx.x;
    const int64_t i = static_cast<int64_t>(bid) * kB + threadIdx.x;
#elif defined(RTPB_EXP_SCATTER)           // experiment only: ray blocks visited in a scattered order
    // block b -> (b * RTPB_EXP_SCATTER) mod nb, a bijection when nb is not a multiple of the prime
    const int64_t nb = gridDim.x;
    const int64_t bs = (nb % RTPB_EXP_SCATTER) ? (blk * RTPB_EXP_SCATTER) % nb : blk;
    const int64_t i = bs * kB + threadIdx.x;
#else
    const int64_t i = blk * kB + threadIdx.x;
#endif
    const int64_t ray0 = i - lane;                       // first ray of this wave
    if (ray0 >= a.n) return;                             // wave-uniform exit
#if defined(RTPB_EXP_STAGGER)              // experiment only: desynchronise the first round of waves
    // consecutive workgroups go to different XCDs, so the delay step uses blockIdx / 8 (varies inside
    // an XCD); 0..7 steps of s_sleep(RTPB_EXP_STAGGER) (64 cycles per unit)
    if (blockIdx.x < 8192)
        for (unsigned k = 0; k < ((blockIdx.x >> 3) & 7u); ++k) __builtin_amdgcn_s_sleep(RTPB_EXP_STAGGER);
#endif
    const bool valid = i < a.n;
    uint4* tile_a = tiles[threadIdx.x >> 6][0];
    uint4* tile_b = tiles[threadIdx.x >> 6][kFinal ? 0 : 1];
    Ray<T> r;
#if defined(RTPB_EXP_NO_INPUT)             // experiment only: no input reads (write-only memory path)
    {
        const T v = T(i);
        r.x = v; r.y = v; r.z = v; r.dx = v; r.dy = v; r.dz = v; r.ph = v; r.wl = T(0.5);
    }
#else
    if constexpr (kStaged && IN_LAYOUT == RTPB_AOS && (STORE & 4)) r = tile_load<TS>(tile_b, a.in, ray0, a.n, lane);
    else r = load_ray<TS, IN_LAYOUT>(a.in, valid ? i : a.n - 1, a.in_fs);
#endif
    const T wl0 = r.wl;
    const Rcp<T> iwl = make_rcp(wl0);                    // shared divisor of every phase update
    TS* __restrict__ out = a.out;
    const cptr<DevSurface<T>> surf = (cptr<DevSurface<T>>)(a.surf);
    const cptr<DevMaterial<T>> mats = (cptr<DevMaterial<T>>)(a.mats);
    const cptr<T> table = (cptr<T>)(a.table);
    auto mat_n = [&](cptr<DevMaterial<T>> mp) -> T {
        if constexpr (kTabLds) return material_n<T, kPoly, true>(load_material<T>(mp), wl0, lds_table);
        else return material_n<T, kPoly, kTabGlobal>(load_material<T>(mp), wl0, table);
    };
    if constexpr (kFinal) {
        T n_cur = mat_n(mats);
        for (int s = 0; s < a.nsurf; ++s) {
            const T n_next = mat_n(mats + s + 1);
            Ray<T> after;
            propagate_surface_emit<T, kLens>(load_surface<T>(surf + s), r, n_cur, n_next, iwl,
                                                         [](const Ray<T>&) {}, after);
            r = after;
            n_cur = n_next;
        }
        if constexpr (kStaged) {
            tile_write<TS>(tile_b, lane, r);
            lds_wait();
            tile_flush<TS, kNT>(tile_b, out, ray0, a.n, lane);
        } else if (valid) {
            store_ray<TS, OUT_LAYOUT>(out, i, a.out_fs, r);
        }
        return;
    }
    int64_t slot_off = 0;
    if (a.mask_lo & 1ull) {
        if constexpr (kStaged) {
            tile_write<TS>(tile_a, lane, r);
            lds_wait();
            tile_flush<TS, kNT>(tile_a, out, ray0, a.n, lane);
        } else if (valid) {
            store_ray<TS, OUT_LAYOUT>(out, i, a.out_fs, r);
        }
        slot_off += a.out_ps;
    }
    T n_cur = mat_n(mats);
    for (int s = 0; s < a.nsurf; ++s) {
        const T n_next = mat_n(mats + s + 1);
        const int p = 2 * s + 1;
        const bool st_at = plane_bit(a.mask_lo, a.mask_hi, p);          // wave-uniform
        const bool st_after = plane_bit(a.mask_lo, a.mask_hi, p + 1);
        const int64_t off_at = slot_off;
        slot_off += st_at ? a.out_ps : 0;
        const int64_t off_after = slot_off;
        slot_off += st_after ? a.out_ps : 0;
        // the "at" plane goes to its LDS tile (or straight out) as soon as it is final
        auto emit_at = [&](const Ray<T>& at) {
            if constexpr (kStaged) {
                if (st_at) tile_write<TS>(tile_a, lane, at);
            } else {
                if (valid && st_at) store_ray<TS, OUT_LAYOUT>(out + off_at, i, a.out_fs, at);
            }
        };
        Ray<T> after;
#if defined(RTPB_EXP_NO_COMPUTE)           // experiment only: the kernel's pure memory path
        after = r;
        after.ph = r.ph + n_next + n_cur;
        emit_at(r);
#else
        propagate_surface_emit<T, kLens>(load_surface<T>(surf + s), r, n_cur, n_next, iwl, emit_at, after);
#endif
        if constexpr (kStaged) {
            // both planes of the surface share one LDS round trip
            if (st_after) tile_write<TS>(tile_b, lane, after);
            if (st_at || st_after) lds_wait();
            if (st_at) tile_flush<TS, kNT>(tile_a, out + off_at, ray0, a.n, lane);
            if (st_after) tile_flush<TS, kNT>(tile_b, out + off_after, ray0, a.n, lane);
        } else if (valid) {
            if (st_after) store_ray<TS, OUT_LAYOUT>(out + off_after, i, a.out_fs, after);
        }
        r = after;
        n_cur = n_next;
    }
    };
#if defined(RTPB_EXP_PERSIST)              // experiment only: persistent grid, block-stride loop
    for (int64_t blk = blockIdx.x; blk * kB < a.n; blk += gridDim.x) body(blk);
#else
    body(static_cast<int64_t>(blockIdx.x));
#endif
}


int popcount128(uint64_t lo, uint64_t hi) { return __builtin_popcountll(lo) + __builtin_popcountll(hi); }

// ---------------------------------------------------------------------------------- timing
struct TimingState {
    bool on = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
};
thread_local TimingState g_timing;

// tuning knobs (rtpb_set_tuning); process-wide
std::atomic<int> g_aos_staging{1};
std::atomic<int> g_nt_stores{1};
std::atomic<int> g_waves_per_eu{0};
std::atomic<int> g_stage_input{0};
std::atomic<int> g_host_chunk_mib{128};

template <typename T, int IL, int OL, int ST, int W, int FEAT>
hipError_t launch_w(const TraceArgs<T>& a, hipStream_t st) {
    constexpr int kB = trace_block(OL, ST);
    const int64_t blocks = (a.n + kB - 1) / kB;
    const size_t lds = (FEAT & 12) == 4 ? static_cast<size_t>(a.ntable) * 2 * sizeof(double) : 0;
#if defined(RTPB_EXP_PERSIST)
    static int resident = 0;                     // experiment: one wave slot per workgroup of the grid
    if (!resident) {
        int per_cu = 0, dev = 0, cus = 0;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, trace_kernel<T, IL, OL, ST, W, FEAT>, kB, lds);
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        resident = per_cu * cus * RTPB_EXP_PERSIST;
    }
    const int64_t grid = blocks < resident ? blocks : resident;
#else
    const int64_t grid = blocks;
#endif
    hipLaunchKernelGGL((trace_kernel<T, IL, OL, ST, W, FEAT>), dim3(static_cast<unsigned>(grid)), dim3(kB), lds,
                       st, a);
    return hipGetLastError();
}

template <typename T, int IL, int OL, int ST>
hipError_t launch_one(const TraceArgs<T>& a, int feat, hipStream_t st) {
    if constexpr (IL == RTPB_AOS && OL == RTPB_AOS && ST == 3) {       // occupancy experiments (tuning)
        const int w = g_waves_per_eu.load();
        if (w == 5) return launch_w<T, IL, OL, ST, 5, 15>(a, st);
    }
#if defined(RTPB_EXP_WPE)                  // experiment only: minimum waves per SIMD for every variant
    constexpr int kW = RTPB_EXP_WPE;
#else
    constexpr int kW = 1;
#endif
    switch (feat) {
    case 0: return launch_w<T, IL, OL, ST, kW, 0>(a, st);
    case 1: return launch_w<T, IL, OL, ST, kW, 1>(a, st);
    case 4: return launch_w<T, IL, OL, ST, kW, 4>(a, st);
    case 5: return launch_w<T, IL, OL, ST, kW, 5>(a, st);
    default: return launch_w<T, IL, OL, ST, kW, 15>(a, st);    // POLY6 or a large table: everything in
    }
}

template <typename T>
hipError_t launch_trace(const TraceArgs<T>& a, int il, int ol, int feat, hipStream_t st) {
    const bool staged = g_aos_staging.load() != 0;
    const bool nt = g_nt_stores.load() != 0;
    const int last = 2 * a.nsurf;                       // planes='final': only the last plane stored
    const bool final_only = a.nsurf > 0 && (last < 64 ? (a.mask_lo == (1ull << last) && a.mask_hi == 0)
                                                      : (a.mask_lo == 0 && a.mask_hi == (1ull << (last - 64))));
    if (final_only && ol == RTPB_AOS && il == RTPB_AOS && staged && nt && !g_stage_input.load() &&
        g_waves_per_eu.load() == 0)
        return launch_one<T, RTPB_AOS, RTPB_AOS, 11>(a, feat, st);
    if (ol == RTPB_AOS) {
        if (!staged)
            return il == RTPB_AOS ? launch_one<T, RTPB_AOS, RTPB_AOS, 0>(a, feat, st) : launch_one<T, RTPB_SOA, RTPB_AOS, 0>(a, feat, st);
        if (nt && il == RTPB_AOS && g_stage_input.load()) return launch_one<T, RTPB_AOS, RTPB_AOS, 7>(a, feat, st);
        if (nt)
            return il == RTPB_AOS ? launch_one<T, RTPB_AOS, RTPB_AOS, 3>(a, feat, st) : launch_one<T, RTPB_SOA, RTPB_AOS, 3>(a, feat, st);
        return il == RTPB_AOS ? launch_one<T, RTPB_AOS, RTPB_AOS, 1>(a, feat, st) : launch_one<T, RTPB_SOA, RTPB_AOS, 1>(a, feat, st);
    }
    if (il == RTPB_AOS) return launch_one<T, RTPB_AOS, RTPB_SOA, 0>(a, feat, st);
    return launch_one<T, RTPB_SOA, RTPB_SOA, 0>(a, feat, st);
}

int trace_impl(rtpb_plan* plan, int dev, const void* in, int64_t n, int il, int64_t in_fs, void* out, int ol,
               int64_t out_ps, int64_t out_fs, uint64_t lo, uint64_t hi, hipStream_t st) {
    void* blob = nullptr;
    int rc = plan_device_blob(plan, dev, &blob);
    if (rc) return rc;
    if (n == 0) return RTPB_OK;
    auto run = [&](auto tag) -> hipError_t {
        using TS = decltype(tag);
        TraceArgs<TS> a{};
        a.in = static_cast<const TS*>(in);
        a.out = static_cast<TS*>(out);
        a.surf = reinterpret_cast<const DevSurface<double>*>(blob);
        a.mats = reinterpret_cast<const DevMaterial<double>*>(static_cast<char*>(blob) + plan->off_mats);
        a.table = reinterpret_cast<const double*>(static_cast<char*>(blob) + plan->off_table);
        a.n = n;
        a.in_fs = in_fs;
        a.out_ps = out_ps;
        a.out_fs = out_fs;
        a.mask_lo = lo;
        a.mask_hi = hi;
        a.nsurf = plan->nsurf;
        a.ntable = static_cast<int32_t>(plan->table.size() / 2);
        return launch_trace<TS>(a, il, ol, plan->feat, st);
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
    hipError_t e = plan->dtype == RTPB_F64 ? run(double{}) : run(float{});
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

int host_shard_pipeline(rtpb_plan* plan, int dev, const char* in, char* out, int64_t n_rays, int64_t a, int64_t b,
                        size_t rec, int nslots, uint64_t lo, uint64_t hi, int T) {
    HostStage& hs = g_stage[dev];
    std::lock_guard<std::mutex> lk(hs.mu);
    DeviceGuard guard(dev);
    // pinned (page-locked, e.g. torch pin_memory) output: DMA every plane slice straight into place
    const bool direct = is_pinned_host(out) && is_pinned_host(out + (int64_t(nslots) * n_rays * rec - 1));
    // ~128 MiB of output per chunk (at least 64k rays), two chunks in flight
    // chunk: ~g_host_chunk_mib of input + output per chunk (at least 64k rays), two chunks in flight
    const int64_t target = int64_t(g_host_chunk_mib.load()) << 20;
    const int64_t chunk = std::min<int64_t>(b - a, std::max<int64_t>(1 << 16, target / int64_t((nslots + 1) * rec)));
    int rc = stage_reserve(hs, chunk * rec, chunk * rec * nslots);
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
        parallel_scatter(static_cast<char*>(hs.pin_in[buf]), in + c0 * rec, 1, 0, static_cast<int64_t>(m * rec), T);
        HIP_TRY(hipMemcpyAsync(hs.d_in[buf], hs.pin_in[buf], m * rec, hipMemcpyHostToDevice, hs.st));
        rc = trace_impl(plan, dev, hs.d_in[buf], m, RTPB_AOS, 0, hs.d_out[buf], RTPB_AOS, m * 8, 0, lo, hi, hs.st);
        if (rc) return rc;
        if (direct)
            HIP_TRY(hipMemcpy2DAsync(out + c0 * rec, n_rays * rec, hs.d_out[buf], m * rec, m * rec, nslots,
                                     hipMemcpyDeviceToHost, hs.st));
        else
            HIP_TRY(hipMemcpyAsync(hs.pin_out[buf], hs.d_out[buf], m * rec * nslots, hipMemcpyDeviceToHost, hs.st));
        HIP_TRY(hipEventRecord(hs.ev[buf], hs.st));
        if (k >= 1) {
            rc = scatter(k - 1);
            if (rc) return rc;
        }
    }
    return scatter(nchunks - 1);
}

}  // namespace

extern "C" {

int rtpb_shutdown(void) {
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

int rtpb_trace(const rtpb_plan* plan_c, int32_t device, const void* rays_in, int64_t n_rays, int32_t in_layout,
               int64_t in_field_stride, void* out, int32_t out_layout, int64_t out_plane_stride,
               int64_t out_field_stride, uint64_t plane_mask_lo, uint64_t plane_mask_hi, void* stream) {
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
    return trace_impl(plan, device, rays_in, n_rays, in_layout, in_field_stride, out, out_layout, out_plane_stride,
                      out_field_stride, plane_mask_lo, plane_mask_hi, static_cast<hipStream_t>(stream));
}

int rtpb_trace_host(const rtpb_plan* plan_c, const void* rays_in, int64_t n_rays, void* out, uint64_t plane_mask_lo,
                    uint64_t plane_mask_hi, const int32_t* devices, int32_t n_devices) {
    auto* plan = const_cast<rtpb_plan*>(plan_c);
    if (!plan) return fail(RTPB_E_INVALID, "plan is NULL");
    if (n_rays < 0) return fail(RTPB_E_INVALID, "n_rays < 0");
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
    const size_t w = plan->dtype == RTPB_F64 ? 8 : 4;
    const size_t rec = 8 * w;
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
        rcs[g] = host_shard_pipeline(plan, dev, static_cast<const char*>(rays_in), static_cast<char*>(out), n_rays, a,
                                     b, rec, nslots, plane_mask_lo, plane_mask_hi, copy_threads);
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
        g_aos_staging.store(value != 0);
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
    if (std::strcmp(key, "waves_per_eu") == 0) {
        if (value != 0 && value != 5) return fail(RTPB_E_INVALID, "waves_per_eu must be 0 or 5");
        g_waves_per_eu.store(static_cast<int>(value));
        return RTPB_OK;
    }
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
