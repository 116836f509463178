// rtpb_internal.h -- internals shared by the translation units of librtpb.so (not part of the ABI):
// launch constants, error plumbing, the plan object, descriptor access through the constant address
// space, ray record loads/stores and the per-wave LDS tiles that turn 64-byte AoS records into 1 KiB
// contiguous stores.  The public interface is include/rtpb.h; the per-ray arithmetic is rtpb_math.h.
//
// Translation units:
//   rtpb_core.hip          errors, plans (lowering to device blobs), device queries
//   rtpb_trace.hip         the fused trace kernel, rtpb_trace / rtpb_trace_host, tuning and timing
//   rtpb_generators.hip    device ray fans and collimated bundles (RT:45-161)
//   rtpb_analysis.hip      intersect_rays, spot statistics, the fused spot sweep, grid interpolation
//   rtpb_surface_ops.hip   propagate_ray2plane and the user-geometry hook kernels
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rtpb.h"
#include "rtpb_math.h"

namespace rtpbi {

using namespace rtpb;

constexpr int kBlock = 256;               // auxiliary kernels
// The trace kernel runs one wave per workgroup: a workgroup's LDS tile and wave slot are released the
// moment its wave finishes, so the dispatcher refills CUs wave by wave instead of waiting for the
// slowest of four (-6 % kernel time on C2 f64 full history vs 256-thread workgroups, same occupancy).
constexpr int kTraceBlock = 64;
constexpr int kMaxDevices = 64;

// Thread-local message of the last failure (rtpb_last_error) and the helper every entry point uses.
extern thread_local std::string g_last_error;
int fail(int code, const std::string& msg);

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(RTPB_E_HIP, std::string(#expr ": ") + hipGetErrorString(e_));          \
    } while (0)

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// ---------------------------------------------------------------------------------- kernel args
// TIN: element type of the input rays, TS: storage type of the output planes (the plan's dtype).  They
// differ when float64 rays are stored as float32 history (or float32 rays as float64): the input is read
// as given, so no value is rounded before the float64 arithmetic.
template <typename TIN, typename TS>
struct TraceArgs {
    const TIN* __restrict__ in;
    TS* __restrict__ out;
    const DevSurface<double>* __restrict__ surf;
    const DevMaterial<double>* __restrict__ mats;
    const double* __restrict__ table;
    const double* __restrict__ itab;   // indexed materials: [nkeys keys][(nsurf+1) x nkeys n][nsurf x nkeys ratios]
    int32_t* miss;        // rtpb_trace_checked: set to 1 when a ray's wavelength is no TABLE key (or NULL)
    int64_t n;
    int64_t in_fs;        // SOA input field stride
    int64_t out_ps;       // output plane (slot) stride
    int64_t out_fs;       // SOA output field stride
    uint64_t mask_lo;
    uint64_t mask_hi;
    int32_t nsurf;
    int32_t ntable;       // (wavelength, n) pairs in `table`
    int32_t nkeys;        // keys of `itab` (feat bit 16)
};

// The trace kernel's launcher for one (input, storage) type pair: picks the kernel variant for the
// layouts, the tuning knobs and the plan's features (rtpb_trace_kernel.h).  The plan-feature variants come in two
// groups compiled in separate translation units (rtpb_trace_<tin>_<ts>.hip: group 0, ..._g1.hip: group 1), so the
// eight largest compiles of the library run in parallel.
// group 0: feat 0, 1, 4, 5 (constant / Sellmeier / LDS-table media, with or without PerfectLens code) and 33 (feat 1
// with only PerfectLens and Flat surfaces in the kAxial / kPlaneXZ forms); group 1: feat 16, 17 (indexed materials)
// and 15 (everything)
constexpr int trace_feat_group(int feat) {
    return (feat == 0 || feat == 1 || feat == 4 || feat == 5 || feat == 33) ? 0 : 1;
}
template <typename TIN, typename TS, int GROUP>
hipError_t launch_trace_group(const TraceArgs<TIN, TS>& a, int il, int ol, int feat, hipStream_t st);
#define RTPB_TRACE_GROUP_EXTERN(TI, TS)                                                                             \
    extern template hipError_t launch_trace_group<TI, TS, 0>(const TraceArgs<TI, TS>&, int, int, int, hipStream_t); \
    extern template hipError_t launch_trace_group<TI, TS, 1>(const TraceArgs<TI, TS>&, int, int, int, hipStream_t);
RTPB_TRACE_GROUP_EXTERN(double, double)
RTPB_TRACE_GROUP_EXTERN(float, float)
RTPB_TRACE_GROUP_EXTERN(double, float)
RTPB_TRACE_GROUP_EXTERN(float, double)
#undef RTPB_TRACE_GROUP_EXTERN
template <typename TIN, typename TS>
inline hipError_t launch_trace(const TraceArgs<TIN, TS>& a, int il, int ol, int feat, hipStream_t st) {
    return trace_feat_group(feat) == 0 ? launch_trace_group<TIN, TS, 0>(a, il, ol, feat, st)
                                       : launch_trace_group<TIN, TS, 1>(a, il, ol, feat, st);
}
// tuning knobs (rtpb_set_tuning, defined in rtpb_trace.hip)
extern std::atomic<int> g_aos_staging, g_nt_stores, g_stage_input, g_host_chunk_mib, g_indexed_materials;
int set_buffer_pool_keep(int64_t k);              // rtpb_buffers.hip: rtpb_set_tuning("buffer_pool_buffers")
int set_buffer_dead_va_limit(int64_t bytes);     // rtpb_buffers.hip: rtpb_set_tuning("buffer_dead_va_limit")

// Descriptors are read-only for the whole launch: read them through the constant address space so
// the uniform-index loads become scalar loads (s_load_*) into SGPRs instead of per-lane vector loads.
template <typename T> using cptr = const __attribute__((address_space(4))) T*;

template <typename T>
__device__ __forceinline__ DevSurface<T> load_surface(cptr<DevSurface<T>> p) {
    DevSurface<T> d;
    d.kind = p->kind;
    d.rcp_ok = p->rcp_ok;
    for (int j = 0; j < 3; ++j) {
        d.c[j] = p->c[j];
        d.nrm[j] = p->nrm[j];
        d.ax[j] = p->ax[j];
    }
    d.R = p->R; d.R2 = p->R2; d.absR = p->absR; d.ap = p->ap; d.f = p->f; d.sin_a = p->sin_a; d.tol = p->tol;
    d.ap_sq = p->ap_sq; d.shell_lo = p->shell_lo; d.shell_hi = p->shell_hi;
    d.rR = p->rR; d.rf = p->rf;
    d.nf[0] = p->nf[0]; d.nf[1] = p->nf[1]; d.nf[2] = p->nf[2];
    d.nr = p->nr; d.rn2 = p->rn2;
    for (int j = 0; j < 3; ++j) {
        d.lF[j] = p->lF[j];
        d.lB[j] = p->lB[j];
    }
    d.ln1f = p->ln1f; d.lph = p->lph;
    return d;
}

template <typename T>
__device__ __forceinline__ DevMaterial<T> load_material(cptr<DevMaterial<T>> p) {
    DevMaterial<T> d;
    d.kind = p->kind;
    d.table_off = p->table_off;
    d.table_len = p->table_len;
    d.pad = 0;
    for (int j = 0; j < 6; ++j) d.c[j] = p->c[j];
    return d;
}

template <typename TS, int LAYOUT>
__device__ __forceinline__ Ray<double> load_ray(const TS* __restrict__ in, int64_t i, int64_t fs) {
    Ray<double> r;
    if constexpr (LAYOUT == RTPB_AOS) {
        if constexpr (sizeof(TS) == 8) {
            const double2* p = reinterpret_cast<const double2*>(in + i * 8);
            const double2 a = p[0], b = p[1], c = p[2], d = p[3];
            r.x = a.x; r.y = a.y; r.z = b.x; r.dx = b.y; r.dy = c.x; r.dz = c.y; r.ph = d.x; r.wl = d.y;
        } else {
            const float4* p = reinterpret_cast<const float4*>(in + i * 8);
            const float4 a = p[0], b = p[1];
            r.x = a.x; r.y = a.y; r.z = a.z; r.dx = a.w; r.dy = b.x; r.dz = b.y; r.ph = b.z; r.wl = b.w;
        }
    } else {
        r.x = in[i]; r.y = in[fs + i]; r.z = in[2 * fs + i]; r.dx = in[3 * fs + i];
        r.dy = in[4 * fs + i]; r.dz = in[5 * fs + i]; r.ph = in[6 * fs + i]; r.wl = in[7 * fs + i];
#if defined(__HIP_DEVICE_COMPILE__)
        // Codegen workaround (ROCm 7.2 LLVM, float64 SoA-input kernels): with the eight fields defined by
        // separate 64-bit loads, the greedy allocator splits the (ph, wl) 128-bit tuple that feeds the
        // ds_write_b128 of the staged record and the rewriter marks the split copy's source undef, so the
        // phase after the first surface was lost (-0.0).  Defining the four pairs as whole 128-bit values,
        // as the AoS loads do, avoids it.  tests/test_codegen_guard.py scans every kernel's assembly for
        // the signature (a 64-bit KILL of another register pair).
        typedef double v2d __attribute__((ext_vector_type(2)));
        v2d a = {r.x, r.y}, b = {r.z, r.dx}, c = {r.dy, r.dz}, d = {r.ph, r.wl};
        asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
        r.x = a.x; r.y = a.y; r.z = b.x; r.dx = b.y; r.dy = c.x; r.dz = c.y; r.ph = d.x; r.wl = d.y;
#endif
    }
    return r;
}

template <typename TS, int LAYOUT>
__device__ __forceinline__ void store_ray(TS* __restrict__ out, int64_t i, int64_t fs, const Ray<double>& r) {
    if constexpr (LAYOUT == RTPB_AOS) {
        if constexpr (sizeof(TS) == 8) {
            double2* p = reinterpret_cast<double2*>(out + i * 8);
            p[0] = make_double2(r.x, r.y);
            p[1] = make_double2(r.z, r.dx);
            p[2] = make_double2(r.dy, r.dz);
            p[3] = make_double2(r.ph, r.wl);
        } else {
            float4* p = reinterpret_cast<float4*>(out + i * 8);
            p[0] = make_float4(float(r.x), float(r.y), float(r.z), float(r.dx));
            p[1] = make_float4(float(r.dy), float(r.dz), float(r.ph), float(r.wl));
        }
    } else {
        out[i] = TS(r.x); out[fs + i] = TS(r.y); out[2 * fs + i] = TS(r.z); out[3 * fs + i] = TS(r.dx);
        out[4 * fs + i] = TS(r.dy); out[5 * fs + i] = TS(r.dz); out[6 * fs + i] = TS(r.ph); out[7 * fs + i] = TS(r.wl);
    }
}

__device__ __forceinline__ bool plane_bit(uint64_t lo, uint64_t hi, int p) {
    return p < 64 ? ((lo >> p) & 1ull) : ((hi >> (p - 64)) & 1ull);
}

// ---------------------------------------------------------------------------------- AOS plane stores
// A ray record is 8*sizeof(TS) = 64 B (f64) or 32 B (f32).  Stored directly, lane l writes its record
// with 16-byte stores at a 64/32-byte lane stride: every store instruction touches 4 KiB of address
// space at 25/50 % density and the history write (11 of 12 bytes moved) runs at ~3.4 TB/s.  Staged,
// each wave first drops its 64 records into a private LDS tile, then lane l stores 16-byte chunks
// l, l+64, ... of the wave's contiguous 4/2 KiB block: every global store instruction writes 1 KiB
// contiguous.  The tile is XOR-swizzled so the b128 writes and reads are bank-conflict free:
//   f64: chunk p of ray L lives at slot 4L + (p ^ ((L >> 1) & 3));  f32: 2L + (p ^ ((L >> 2) & 1)).
// Only the owning wave touches its tile and LDS executes one wave's DS operations in order, so no
// workgroup barrier is needed -- just the lgkmcnt waits (asm, with a memory clobber so the compiler
// cannot move the tile accesses across them).
// Plans whose TABLE materials hold at most this many (wavelength, n) pairs in total get kernels that copy
// the table into LDS at launch (rtpb_plan::feat bit 4), so the per-surface lookups are LDS reads.  A
// global-memory lookup inside the surface loop costs far more than its latency: gfx950 counts loads and
// stores in one in-order counter (vmcnt), so waiting for a table load also waits for every history
// store the wave has in flight.
constexpr int kLdsTablePairs = 256;
// Indexed materials (rtpb_plan::feat bit 16): when every TABLE material of a plan is tabulated at the
// same wavelengths (the bundle's distinct wavelengths, as the Python layer lowers them) and no POLY6
// material is present, the plan also carries n of EVERY material at those K keys, evaluated on the host
// with the kernel's own material_n (so the values are the ones the kernel would compute).  The kernel
// then finds each ray's key index once and reads n(material, key) from LDS at every surface, instead of
// re-evaluating Sellmeier dispersion (three divisions and a square root) and searching tables per
// surface, and each surface's Snell ratio n1 / n2 instead of dividing.  Layout: [K keys][(S+1) x K
// values][S x K ratios]; at most this many doubles.
constexpr int kLdsIndexedDoubles = 512;

// Index of wavelength wl among the K sorted keys (NaN last, as sort_table orders them; NaN wl finds a NaN
// key), or -1.  Same matching rule as material_n's TABLE search, so indexed and searched lookups agree.
__device__ __forceinline__ int key_index(const double* keys, int K, double wl) {
    if (wl != wl) return (K > 0 && keys[K - 1] != keys[K - 1]) ? K - 1 : -1;
    int lo = 0, hi = K;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (keys[mid] < wl) lo = mid + 1;
        else hi = mid;
    }
    return (lo < K && keys[lo] == wl) ? lo : -1;
}

constexpr int kTileBytes = 64 * 64;    // 64 records of <= 64 B

typedef double v2d __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));

// Stage one record into the wave's tile (XOR-swizzled slots)
template <typename TS>
__device__ __forceinline__ void tile_write(uint4* __restrict__ tile, int lane, const Ray<double>& r) {
    if constexpr (sizeof(TS) == 8) {
        const int sw = (lane >> 1) & 3;
        double2* t = reinterpret_cast<double2*>(tile);
        t[4 * lane + (0 ^ sw)] = make_double2(r.x, r.y);
        t[4 * lane + (1 ^ sw)] = make_double2(r.z, r.dx);
        t[4 * lane + (2 ^ sw)] = make_double2(r.dy, r.dz);
        t[4 * lane + (3 ^ sw)] = make_double2(r.ph, r.wl);
    } else {
        const int sw = (lane >> 2) & 1;
        float4* t = reinterpret_cast<float4*>(tile);
        t[2 * lane + (0 ^ sw)] = make_float4(float(r.x), float(r.y), float(r.z), float(r.dx));
        t[2 * lane + (1 ^ sw)] = make_float4(float(r.dy), float(r.dz), float(r.ph), float(r.wl));
    }
}

// A wave-uniform 64-bit value the divergence analysis cannot prove uniform (e.g. derived from threadIdx.x
// & ~63): moved to SGPRs so the address arithmetic that uses it is scalar.
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
    return (static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32))) << 32) |
           static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v)));
}

// Write the wave's staged block (64 records) to `plane` lane-contiguously: 1 KiB per store instruction.
// Callers wait for the tile writes first (lgkmcnt(0)); the compiler waits for the tile reads before the
// global stores that consume them, and a wave's DS operations execute in order, so the next tile_write
// cannot overtake these reads.
// The stores are raw buffer stores through a per-wave resource (SGPRs): base = the block's first record,
// num_records = the block's bytes, so the address is lane*16 + an immediate and the bounds check of the
// buffer unit drops the tail of the last block -- no 64-bit VALU address arithmetic and no exec-mask
// branches per plane.  (ray0 and the plane pointer are wave-uniform; readfirstlane tells the compiler.)
template <typename TS, bool NT>
__device__ __forceinline__ void tile_flush(const uint4* __restrict__ tile, TS* __restrict__ plane, int64_t ray0,
                                           int64_t n, int lane) {
    constexpr int kRec = 8 * sizeof(TS);
    // gfx950 cache policy nt + sc1 (streaming, system scope): 0.5 % faster than nt alone on C2-C4 in
    // interleaved A/B (profiles/r02/experiments/ab_aux*.log); without nt the C3 history is 26 % slower
    constexpr int kAux = NT ? (2 | 16) : 0;
    const int64_t left = n - ray0;
    const int nbytes = static_cast<int>((left < 64 ? left : 64) * kRec);
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(uniform_u64(reinterpret_cast<uint64_t>(plane + ray0 * 8))), static_cast<short>(0),
        __builtin_amdgcn_readfirstlane(nbytes), 0x00020000);
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const v4u* t = reinterpret_cast<const v4u*>(tile);
    if constexpr (sizeof(TS) == 8) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = lane + 64 * j, rr = c >> 2, pp = c & 3;
            __builtin_amdgcn_raw_buffer_store_b128(t[4 * rr + (pp ^ ((rr >> 1) & 3))], rsrc, c * 16, 0, kAux);
        }
    } else {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int c = lane + 64 * j, rr = c >> 1, pp = c & 1;
            __builtin_amdgcn_raw_buffer_store_b128(t[2 * rr + (pp ^ ((rr >> 2) & 1))], rsrc, c * 16, 0, kAux);
        }
    }
}

__device__ __forceinline__ void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Register-exchange flush of float32 records (no LDS): the same 1 KiB-contiguous stores as tile_flush, with
// the transpose done by one DPP swap between neighbouring lanes.  It needs the exchange lane mapping:
// lane 2m traces ray m of the wave's block and lane 2m+1 ray 32+m (xchg_ray).  A record is two 16-byte
// chunks (lo = x y z dx, hi = dy dz ph wl); store 0 writes chunks 0..63 (rays 0..31), store 1 chunks
// 64..127 (rays 32..63), so lane 2m stores its own lo and its partner's lo, lane 2m+1 its partner's hi and
// its own hi: each lane sends one half (even: hi, odd: lo) and receives the other's.
__device__ __forceinline__ int xchg_ray(int lane) { return (lane & 1) ? 32 + (lane >> 1) : (lane >> 1); }

template <bool NT>
__device__ __forceinline__ void xchg_flush(float* __restrict__ plane, int64_t ray0, int64_t n, int lane,
                                           const Ray<double>& r) {
    constexpr int kAux = NT ? (2 | 16) : 0;            // nt + sc1, as tile_flush
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const float lo[4] = {float(r.x), float(r.y), float(r.z), float(r.dx)};
    const float hi[4] = {float(r.dy), float(r.dz), float(r.ph), float(r.wl)};
    const bool odd = (lane & 1) != 0;
    v4u s0, s1;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int send = __float_as_int(odd ? lo[k] : hi[k]);
        const unsigned recv = static_cast<unsigned>(__builtin_amdgcn_mov_dpp(send, 0xB1, 0xF, 0xF, false));  // lane ^ 1
        s0[k] = odd ? recv : __float_as_uint(lo[k]);
        s1[k] = odd ? __float_as_uint(hi[k]) : recv;
    }
    const int64_t left = n - ray0;
    const int nbytes = static_cast<int>((left < 64 ? left : 64) * 32);
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(uniform_u64(reinterpret_cast<uint64_t>(plane + ray0 * 8))), static_cast<short>(0),
        __builtin_amdgcn_readfirstlane(nbytes), 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(s0, rsrc, lane * 16, 0, kAux);
    __builtin_amdgcn_raw_buffer_store_b128(s1, rsrc, 1024 + lane * 16, 0, kAux);
}

// Inverse of tile_flush for the input: lane l loads 16-byte chunks l, l+64, ... of the wave's contiguous
// record block (1 KiB per load instruction) into the tile, then reads back its own record.
template <typename TS>
__device__ __forceinline__ Ray<double> tile_load(uint4* __restrict__ tile, const TS* __restrict__ in, int64_t ray0,
                                                 int64_t n, int lane) {
    Ray<double> r;
    if constexpr (sizeof(TS) == 8) {
        double2* t = reinterpret_cast<double2*>(tile);
        const double2* g = reinterpret_cast<const double2*>(in + ray0 * 8);
        const int64_t nchunks = (n - ray0 < 64 ? n - ray0 : 64) * 4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = lane + 64 * j, rr = c >> 2, pp = c & 3;
            const double2 v = g[c < nchunks ? c : nchunks - 4 + pp];      // tail lanes re-read the last ray
            t[4 * rr + (pp ^ ((rr >> 1) & 3))] = v;
        }
        lds_wait();
        const int sw = (lane >> 1) & 3;
        const double2 a = t[4 * lane + (0 ^ sw)], b = t[4 * lane + (1 ^ sw)], c = t[4 * lane + (2 ^ sw)],
                      d = t[4 * lane + (3 ^ sw)];
        r.x = a.x; r.y = a.y; r.z = b.x; r.dx = b.y; r.dy = c.x; r.dz = c.y; r.ph = d.x; r.wl = d.y;
    } else {
        float4* t = reinterpret_cast<float4*>(tile);
        const float4* g = reinterpret_cast<const float4*>(in + ray0 * 8);
        const int64_t nchunks = (n - ray0 < 64 ? n - ray0 : 64) * 2;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int c = lane + 64 * j, rr = c >> 1, pp = c & 1;
            const float4 v = g[c < nchunks ? c : nchunks - 2 + pp];
            t[2 * rr + (pp ^ ((rr >> 2) & 1))] = v;
        }
        lds_wait();
        const int sw = (lane >> 2) & 1;
        const float4 a = t[2 * lane + (0 ^ sw)], b = t[2 * lane + (1 ^ sw)];
        r.x = a.x; r.y = a.y; r.z = a.z; r.dx = a.w; r.dy = b.x; r.dz = b.y; r.ph = b.z; r.wl = b.w;
    }
    return r;
}

inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Per-thread pinned staging buffer for small host->device uploads (tables, per-group parameters): the
// caller fills it, then upload() copies it to `dev` on `st`.  It is reused once its previous copy has
// completed, so uploads never synchronise the stream.
struct PinnedStaging {
    double* buf = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;

    int reserve(size_t bytes) {
        if (done) HIP_TRY(hipEventSynchronize(done));
        if (!done) HIP_TRY(hipEventCreateWithFlags(&done, hipEventDisableTiming));
        if (cap < bytes) {
            if (buf) HIP_TRY(hipHostFree(buf));
            buf = nullptr;
            cap = 0;
            HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&buf), bytes, hipHostMallocDefault));
            cap = bytes;
        }
        return RTPB_OK;
    }
    int upload(void* dev, size_t bytes, hipStream_t st) {
        HIP_TRY(hipMemcpyAsync(dev, buf, bytes, hipMemcpyHostToDevice, st));
        HIP_TRY(hipEventRecord(done, st));
        return RTPB_OK;
    }
};
PinnedStaging& pinned_staging();     // this thread's buffer

}  // namespace rtpbi

// ---------------------------------------------------------------------------------- plans
struct rtpb_plan {
    int32_t dtype = RTPB_F64;
    int32_t nsurf = 0;
    std::vector<rtpb_surface> surf;
    std::vector<rtpb_material> mats;    // table pointers cleared; see table_off/table_len
    std::vector<int32_t> table_off;
    std::vector<double> table;          // (wavelength, n) pairs of every TABLE material
    // kernel features needed: 1 = PerfectLens, 2 = POLY6 material, 4 = TABLE materials whose table fits
    // the kernel's LDS copy (kLdsTablePairs), 8 = TABLE materials read from global memory, 16 = indexed
    // materials (replaces 4 / 8; see kLdsIndexedDoubles), 32 = with 1 and nothing else: every surface a PerfectLens
    // or a Flat in the kAxial / kPlaneXZ form (dispatch_kind's kKindsLensFlat)
    int feat = 0;
    std::vector<double> itab;           // indexed materials: [nkeys keys][(nsurf+1) x nkeys n][nsurf x nkeys ratios]
    int32_t nkeys = 0;
    std::mutex mu;
    void* blob[rtpbi::kMaxDevices] = {};
    size_t off_mats = 0, off_table = 0, off_itab = 0, blob_bytes = 0;   // blob layout, fixed at plan creation
};

namespace rtpbi {
// Device copy of a plan's descriptors (created on first use per device, then immutable).
int plan_device_blob(rtpb_plan* p, int dev, void** out);
// The device material descriptor of plan material k, as the kernels see it (zero Sellmeier = VACUUM).
DevMaterial<double> device_material(const rtpb_plan& p, size_t k);
// RTPB_OK, or RTPB_E_NODEV with the message set.
int check_device(int dev);
}  // namespace rtpbi
