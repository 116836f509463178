// rtpb_device.hip -- gfx950 kernels and the C ABI (include/rtpb.h) of the sequential ray tracer.
//
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

using namespace rtpb;

namespace {

constexpr int kBlock = 256;               // auxiliary kernels
// The trace kernel runs one wave per workgroup: a workgroup's LDS tile and wave slot are released the
// moment its wave finishes, so the dispatcher refills CUs wave by wave instead of waiting for the
// slowest of four (-6 % kernel time on C2 f64 full history vs 256-thread workgroups, same occupancy).
#if defined(RTPB_EXP_TRACE_BLOCK)          // experiment builds only (tools/ab_libs.py)
constexpr int kTraceBlock = RTPB_EXP_TRACE_BLOCK;
#else
constexpr int kTraceBlock = 64;
#endif
constexpr int kMaxDevices = 64;

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

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
template <typename TS>
struct TraceArgs {
    const TS* __restrict__ in;
    TS* __restrict__ out;
    const DevSurface<double>* __restrict__ surf;
    const DevMaterial<double>* __restrict__ mats;
    const double* __restrict__ table;
    int64_t n;
    int64_t in_fs;        // SOA input field stride
    int64_t out_ps;       // output plane (slot) stride
    int64_t out_fs;       // SOA output field stride
    uint64_t mask_lo;
    uint64_t mask_hi;
    int32_t nsurf;
};

// Descriptors are read-only for the whole launch: read them through the constant address space so
// the uniform-index loads become scalar loads (s_load_*) into SGPRs instead of per-lane vector loads.
template <typename T> using cptr = const __attribute__((address_space(4))) T*;

template <typename T>
__device__ __forceinline__ DevSurface<T> load_surface(cptr<DevSurface<T>> p) {
    DevSurface<T> d;
    d.kind = p->kind;
    d.pad = 0;
    for (int j = 0; j < 3; ++j) {
        d.c[j] = p->c[j];
        d.nrm[j] = p->nrm[j];
        d.ax[j] = p->ax[j];
    }
    d.R = p->R; d.R2 = p->R2; d.absR = p->absR; d.ap = p->ap; d.f = p->f; d.sin_a = p->sin_a; d.tol = p->tol;
    d.ap_sq = p->ap_sq; d.shell_lo = p->shell_lo; d.shell_hi = p->shell_hi;
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
constexpr int kTileBytes = 64 * 64;    // 64 records of <= 64 B

typedef double v2d __attribute__((ext_vector_type(2)));
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void gstore(double2* p, const double2& v, bool nt) {
    if (nt) __builtin_nontemporal_store(v2d{v.x, v.y}, reinterpret_cast<v2d*>(p));
    else *p = v;
}
__device__ __forceinline__ void gstore(float4* p, const float4& v, bool nt) {
    if (nt) __builtin_nontemporal_store(v4f{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f*>(p));
    else *p = v;
}

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

// Write the wave's staged block (64 records) to `plane` lane-contiguously: 1 KiB per store instruction.
// Callers wait for the tile writes first (lgkmcnt(0)); the compiler waits for the tile reads before the
// global stores that consume them, and a wave's DS operations execute in order, so the next tile_write
// cannot overtake these reads.
template <typename TS, bool NT>
__device__ __forceinline__ void tile_flush(const uint4* __restrict__ tile, TS* __restrict__ plane, int64_t ray0,
                                           int64_t n, int lane) {
    if constexpr (sizeof(TS) == 8) {
        const double2* t = reinterpret_cast<const double2*>(tile);
        const int64_t nchunks = (n - ray0 < 64 ? n - ray0 : 64) * 4;
        double2* g = reinterpret_cast<double2*>(plane + ray0 * 8);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = lane + 64 * j, rr = c >> 2, pp = c & 3;
            const double2 v = t[4 * rr + (pp ^ ((rr >> 1) & 3))];
            if (c < nchunks) gstore(g + c, v, NT);
        }
    } else {
        const float4* t = reinterpret_cast<const float4*>(tile);
        const int64_t nchunks = (n - ray0 < 64 ? n - ray0 : 64) * 2;
        float4* g = reinterpret_cast<float4*>(plane + ray0 * 8);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int c = lane + 64 * j, rr = c >> 1, pp = c & 1;
            const float4 v = t[2 * rr + (pp ^ ((rr >> 2) & 1))];
            if (c < nchunks) gstore(g + c, v, NT);
        }
    }
}

__device__ __forceinline__ void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

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

// The fused multi-surface trace: one lane = one ray through all surfaces (float64 arithmetic,
// TS storage).  STORE: bit 0 = LDS-staged AOS stores (OUT_LAYOUT == AOS only), bit 1 = non-temporal
// global stores for the staged tiles.
// Workgroup size per variant: the LDS-staged AoS kernels run one wave per workgroup (see kTraceBlock);
// the direct-store variants (SoA output, unstaged AoS) keep four-wave workgroups, which measured faster
// for their strided stores (C5 SoA: 0.53 vs 0.69 ms).
constexpr int trace_block(int out_layout, int store) {
    return (out_layout == RTPB_AOS && (store & 1)) ? kTraceBlock : 256;
}

// FEAT: bit 0 = PerfectLens code, bit 1 = RTPB_POLY6 code compiled in.  Leaving out what a plan does
// not use lowers register pressure (f64 staged: 92 VGPRs without both -> 5 waves/SIMD; 118 with both
// -> 4), 10-15 % faster when compute-bound.  rtpb_plan::feat picks the variant.
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
    __shared__ uint4 tiles[kB / 64][kFinal ? 1 : 2][kTileBytes / 16];  // per wave: "at" and "after" tiles
    const int lane = threadIdx.x & 63;
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kB + threadIdx.x;
    const int64_t ray0 = i - lane;                       // first ray of this wave
    if (ray0 >= a.n) return;                             // wave-uniform exit
#if defined(RTPB_EXP_STAGGER)              // experiment only: desynchronise the first round of waves
    if (blockIdx.x < RTPB_EXP_STAGGER)
        for (unsigned k = 0; k < (blockIdx.x & 7u); ++k) __builtin_amdgcn_s_sleep(20);
#endif
    const bool valid = i < a.n;
    uint4* tile_a = tiles[threadIdx.x >> 6][0];
    uint4* tile_b = tiles[threadIdx.x >> 6][kFinal ? 0 : 1];
    Ray<T> r;
    if constexpr (kStaged && IN_LAYOUT == RTPB_AOS && (STORE & 4)) r = tile_load<TS>(tile_b, a.in, ray0, a.n, lane);
    else r = load_ray<TS, IN_LAYOUT>(a.in, valid ? i : a.n - 1, a.in_fs);
    const T wl0 = r.wl;
    TS* __restrict__ out = a.out;
    const cptr<DevSurface<T>> surf = (cptr<DevSurface<T>>)(a.surf);
    const cptr<DevMaterial<T>> mats = (cptr<DevMaterial<T>>)(a.mats);
    const cptr<T> table = (cptr<T>)(a.table);
    if constexpr (kFinal) {
        T n_cur = material_n<T, (FEAT & 2) != 0>(load_material<T>(mats), wl0, table);
        for (int s = 0; s < a.nsurf; ++s) {
            const T n_next = material_n<T, (FEAT & 2) != 0>(load_material<T>(mats + s + 1), wl0, table);
            Ray<T> after;
            propagate_surface_emit<T, (FEAT & 1) != 0>(load_surface<T>(surf + s), r, n_cur, n_next,
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
    T n_cur = material_n<T, (FEAT & 2) != 0>(load_material<T>(mats), wl0, table);
    for (int s = 0; s < a.nsurf; ++s) {
        const T n_next = material_n<T, (FEAT & 2) != 0>(load_material<T>(mats + s + 1), wl0, table);
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
        propagate_surface_emit<T, (FEAT & 1) != 0>(load_surface<T>(surf + s), r, n_cur, n_next, emit_at, after);
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
}

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
        r.wl = a.wl;
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
        r.wl = a.wl;
        tile_write<T>(tile, lane, r);
    }
    lds_wait();
    tile_flush<T, true>(tile, static_cast<T*>(a.out), ray0, total, lane);
}

// intersect_rays (RT:164-238): closest-approach solve from the first non-singular 2x2 sub-system,
// verified to 1e-12.  NaN determinants count as "non-zero" exactly like numpy's truthiness.
struct IsectArgs {
    const void* __restrict__ r1;
    const void* __restrict__ r2;
    void* __restrict__ out;
    int64_t n, n1, n2;
};

template <typename T>
__global__ __launch_bounds__(kBlock) void intersect_kernel(IsectArgs a) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (i >= a.n) return;
    const T* p = static_cast<const T*>(a.r1) + (a.n1 == 1 ? 0 : i) * 8;
    const T* q = static_cast<const T*>(a.r2) + (a.n2 == 1 ? 0 : i) * 8;
    const double x1 = p[0], y1 = p[1], z1 = p[2], dx1 = p[3], dy1 = p[4], dz1 = p[5];
    const double x2 = q[0], y2 = q[1], z2 = q[2], dx2 = q[3], dy2 = q[4], dz2 = q[5];
    const double nan = qnan<double>();
    const double det_xz = dx2 * dz1 - dz2 * dx1, det_xy = dx2 * dy1 - dy2 * dx1, det_yz = dz2 * dy1 - dy2 * dz1;
    double s = nan;
    if (det_xz != 0.0) s = ((z2 - z1) * dx1 - (x2 - x1) * dz1) / det_xz;
    else if (det_xy != 0.0) s = ((y2 - y1) * dx1 - (x2 - x1) * dy1) / det_xy;
    else if (det_yz != 0.0) s = ((y2 - y1) * dz1 - (z2 - z1) * dy1) / det_yz;
    double t;
    if (dz1 != 0.0) t = (z2 + s * dz2 - z1) / dz1;
    else if (dy1 != 0.0) t = (y2 + s * dy2 - y1) / dy1;
    else t = (x2 + s * dx2 - x1) / dx1;
    double o[3] = {x1 + t * dx1, y1 + t * dy1, z1 + t * dz1};
    const double e[3] = {o[0] - (x2 + s * dx2), o[1] - (y2 + s * dy2), o[2] - (z2 + s * dz2)};
    // numpy.max over the 3 |differences| propagates NaN, and NaN > 1e-12 is false
    double m = tabs(e[0]);
    for (int k = 1; k < 3; ++k) {
        const double v = tabs(e[k]);
        if (is_nan(m)) break;
        if (is_nan(v) || v > m) m = v;
    }
    if (m > 1e-12) o[0] = o[1] = o[2] = nan;
    T* out = static_cast<T*>(a.out) + i * 3;
    out[0] = T(o[0]); out[1] = T(o[1]); out[2] = T(o[2]);
}

// Spot statistics of one history plane, per contiguous group of `gsize` rays (per
// (field, wavelength) spot diagrams).  Rays whose x or y is not finite are skipped.  Deterministic:
// pass 1 reduces each 256-ray tile of a group in a fixed tree order into partials[group][tile];
// pass 2 sums a group's partials in a fixed order.  Stats: n, Sx, Sy, Sz, Sxx, Syy, Sxy.
constexpr int kStats = 7;
struct SpotArgs {
    const void* __restrict__ plane;
    double* __restrict__ partials;
    double* __restrict__ stats;
    int64_t gsize, ngroups, tiles;
};

template <typename T>
__global__ __launch_bounds__(kBlock) void spot_partial_kernel(SpotArgs a) {
    __shared__ double red[kStats][kBlock];
    const int64_t g = blockIdx.y, tile = blockIdx.x;
    const int64_t j = tile * kBlock + threadIdx.x;
    double v[kStats] = {0, 0, 0, 0, 0, 0, 0};
    if (j < a.gsize) {
        const T* r = static_cast<const T*>(a.plane) + (g * a.gsize + j) * 8;
        const double x = r[0], y = r[1], z = r[2];
        if (x - x == 0.0 && y - y == 0.0) {
            v[0] = 1.0; v[1] = x; v[2] = y; v[3] = z; v[4] = x * x; v[5] = y * y; v[6] = x * y;
        }
    }
    for (int k = 0; k < kStats; ++k) red[k][threadIdx.x] = v[k];
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w)
            for (int k = 0; k < kStats; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x < kStats) a.partials[(g * a.tiles + tile) * kStats + threadIdx.x] = red[threadIdx.x][0];
}

__global__ __launch_bounds__(kBlock) void spot_final_kernel(SpotArgs a) {
    __shared__ double red[kStats][kBlock];
    const int64_t g = blockIdx.x;
    double v[kStats] = {0, 0, 0, 0, 0, 0, 0};
    for (int64_t t = threadIdx.x; t < a.tiles; t += kBlock)
        for (int k = 0; k < kStats; ++k) v[k] += a.partials[(g * a.tiles + t) * kStats + k];
    for (int k = 0; k < kStats; ++k) red[k][threadIdx.x] = v[k];
    __syncthreads();
    for (int w = kBlock / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w)
            for (int k = 0; k < kStats; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x < kStats) a.stats[g * kStats + threadIdx.x] = red[threadIdx.x][0];
}

// Spot-diagram sweep, fused (C5).  Group g is the fan get_ray_fan(pt_g, ..., wl_g)
// (RT:45-96, same per-ray arithmetic as ray_fan_kernel, angles from the caller's tables); each ray is
// generated in registers, traced through the plan keeping only its final state, and reduced into the
// same 256-ray tile partials as spot_partial_kernel.  spot_final_kernel then produces statistics
// bit-identical to generating, tracing (planes='final') and reducing separately -- without the
// 3 x 64 B per ray of HBM traffic and the launches in between.
struct SweepArgs {
    const DevSurface<double>* __restrict__ surf;
    const DevMaterial<double>* __restrict__ mats;
    const double* __restrict__ table;
    const double2* __restrict__ tab;    // (cos, sin): thetas [n_thetas], then phis [nphis]
    const double* __restrict__ grp;     // per group: x, y, z, wavelength
    double* __restrict__ partials;
    int64_t n_thetas, nphis, gsize, tiles;
    double c[3], ex[3], ey[3];
    int32_t nsurf;
};

template <typename TS>
__device__ __forceinline__ double stored(double v) { return static_cast<double>(static_cast<TS>(v)); }

// Two rays per lane: block b covers tiles 2b and 2b+1 of its group; both rays go through each surface
// in one straight-line region (propagate_surface_pair) so two independent dependency chains
// interleave (-6 % vs one ray per lane); each tile is reduced separately, with the same tree as
// spot_partial_kernel.
template <typename TS, int FEAT>
__global__ __launch_bounds__(kBlock) void sweep_kernel(SweepArgs a) {
    __shared__ double red[kStats][kBlock];
    const int64_t g = blockIdx.y;
    const int64_t tileA = 2 * int64_t(blockIdx.x), tileB = tileA + 1;
    const int64_t jA = tileA * kBlock + threadIdx.x, jB = tileB * kBlock + threadIdx.x;
    const bool okA = jA < a.gsize, okB = jB < a.gsize;
    const double* gp = a.grp + 4 * g;
    auto gen = [&](int64_t j) {
        const int64_t jj = j < a.gsize ? j : 0;
        const int64_t it = jj % a.n_thetas, ip = jj / a.n_thetas;
        const double2 t = a.tab[it], ph = a.tab[a.n_thetas + ip];
        const double ct = t.x, st = t.y, cp = ph.x, sp = ph.y;
        Ray<double> r;
        r.x = stored<TS>(gp[0]); r.y = stored<TS>(gp[1]); r.z = stored<TS>(gp[2]);
        r.dx = stored<TS>(a.c[0] * ct + a.ex[0] * cp * st + a.ey[0] * sp * st);
        r.dy = stored<TS>(a.c[1] * ct + a.ex[1] * cp * st + a.ey[1] * sp * st);
        r.dz = stored<TS>(a.c[2] * ct + a.ex[2] * cp * st + a.ey[2] * sp * st);
        r.ph = 0.0;
        r.wl = stored<TS>(gp[3]);
        return r;
    };
    Ray<double> rA = gen(jA), rB = gen(jB);
    const cptr<DevSurface<double>> surf = (cptr<DevSurface<double>>)(a.surf);
    const cptr<DevMaterial<double>> mats = (cptr<DevMaterial<double>>)(a.mats);
    const cptr<double> table = (cptr<double>)(a.table);
    const double wl0 = rA.wl;                          // one wavelength per group
    double n_cur = material_n<double, (FEAT & 2) != 0>(load_material<double>(mats), wl0, table);
    for (int s = 0; s < a.nsurf; ++s) {
        const double n_next = material_n<double, (FEAT & 2) != 0>(load_material<double>(mats + s + 1), wl0, table);
        const DevSurface<double> sd = load_surface<double>(surf + s);
        Ray<double> aA, aB;
        propagate_surface_pair<double, (FEAT & 1) != 0>(sd, rA, rB, n_cur, n_next, aA, aB);
        rA = aA;
        rB = aB;
        n_cur = n_next;
    }
    auto reduce = [&](const Ray<double>& r, bool ok, int64_t tile) {
        double v[kStats] = {0, 0, 0, 0, 0, 0, 0};
        if (ok) {
            const double x = stored<TS>(r.x), y = stored<TS>(r.y), z = stored<TS>(r.z);
            if (x - x == 0.0 && y - y == 0.0) {
                v[0] = 1.0; v[1] = x; v[2] = y; v[3] = z; v[4] = x * x; v[5] = y * y; v[6] = x * y;
            }
        }
        for (int k = 0; k < kStats; ++k) red[k][threadIdx.x] = v[k];
        __syncthreads();
        for (int w = kBlock / 2; w > 0; w >>= 1) {
            if (threadIdx.x < w)
                for (int k = 0; k < kStats; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x < kStats && tile < a.tiles)
            a.partials[(g * a.tiles + tile) * kStats + threadIdx.x] = red[threadIdx.x][0];
        __syncthreads();
    };
    reduce(rA, okA, tileA);
    reduce(rB, okB, tileB);
}

// griddata(method='linear') on a regular grid + the pupil field of the PSF script (rtpb_grid_interpolate).
__global__ __launch_bounds__(kBlock) void grid_interp_kernel(rtpb_triangulation t, const double* __restrict__ xs,
                                                             int64_t nx, const double* __restrict__ ys, int64_t ny,
                                                             double radius, double* __restrict__ phase_out,
                                                             double* __restrict__ field_out) {
    const int64_t k = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (k >= nx * ny) return;
    const int64_t iy = k / nx, ix = k % nx;
    const double x = xs[ix], y = ys[iy];
    constexpr double eps = 100.0 * 2.220446049250313e-16;      // scipy qhull: 100 * DBL_EPSILON
    double phase = __builtin_nan("");
    const double fx = (x - t.x0) / t.cell_w, fy = (y - t.y0) / t.cell_h;
    if (fx >= 0.0 && fy >= 0.0 && fx < double(t.cells_x) && fy < double(t.cells_y)) {
        const int64_t cell = int64_t(fy) * t.cells_x + int64_t(fx);
        for (int32_t q = t.cell_start[cell]; q < t.cell_start[cell + 1]; ++q) {
            const int32_t s = t.cell_tris[q];
            const double* T = t.transform + 6 * int64_t(s);
            // scipy/spatial/_qhull.pyx _barycentric_inside / _barycentric_coordinates (ndim = 2)
            double c0 = 0.0;
            c0 += T[0] * (x - T[4]);
            c0 += T[1] * (y - T[5]);
            double c1 = 0.0;
            c1 += T[2] * (x - T[4]);
            c1 += T[3] * (y - T[5]);
            const double c2 = (1.0 - c0) - c1;
            if (!(-eps <= c0 && c0 <= 1.0 + eps) || !(-eps <= c1 && c1 <= 1.0 + eps) ||
                !(-eps <= c2 && c2 <= 1.0 + eps))
                continue;
            // scipy/interpolate/_interpnd.pyx LinearNDInterpolator._do_evaluate
            const int32_t* v = t.simplices + 3 * int64_t(s);
            double o = 0.0;
            o = o + c0 * t.values[v[0]];
            o = o + c1 * t.values[v[1]];
            o = o + c2 * t.values[v[2]];
            phase = o;
            break;
        }
    }
    if (phase_out) phase_out[k] = phase;
    if (field_out) {
        const bool off = sqrt(x * x + y * y) > radius || phase != phase;
        field_out[2 * k] = off ? 0.0 : cos(phase);
        field_out[2 * k + 1] = off ? 0.0 : sin(phase);
    }
}

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
        const Ray<double> o = to_plane<double>(r, nv[0], nv[1], nv[2], cv[0], cv[1], cv[2], n, a.exclude != 0, &t);
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
            o = snell<double>(h, Nx, Ny, Nz, n1, n2);                               // RT:1194-1221
        }
        if (a.on && !a.on[i]) kill(o);                                               // RT:1225-1226, 1293-1294
        tile_write<TS>(tile, lane, o);
    }
    lds_wait();
    tile_flush<TS, true>(tile, static_cast<TS*>(a.out), ray0, a.n, lane);
}

}  // namespace

// ---------------------------------------------------------------------------------- plans
struct rtpb_plan {
    int32_t dtype = RTPB_F64;
    int32_t nsurf = 0;
    std::vector<rtpb_surface> surf;
    std::vector<rtpb_material> mats;    // table pointers cleared; see table_off/table_len
    std::vector<int32_t> table_off;
    std::vector<double> table;          // (wavelength, n) pairs of every TABLE material
    int feat = 0;                       // kernel features needed: 1 = PerfectLens, 2 = POLY6 material
    std::mutex mu;
    void* blob[kMaxDevices] = {};
    size_t off_mats = 0, off_table = 0, blob_bytes = 0;   // blob layout, fixed at plan creation
};

namespace {

size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

// Blob layout: [S surfaces][S+1 materials][table pairs], each part 256-byte aligned.  Computed once at
// plan creation, so launches on any device read the offsets without synchronisation.
template <typename T>
void blob_layout(rtpb_plan& p) {
    p.off_mats = align256(p.surf.size() * sizeof(DevSurface<T>));
    p.off_table = p.off_mats + align256(p.mats.size() * sizeof(DevMaterial<T>));
    p.blob_bytes = p.off_table + align256(std::max<size_t>(p.table.size(), 2) * sizeof(T));
}

template <typename T>
std::vector<unsigned char> build_blob(const rtpb_plan& p) {
    const size_t S = p.surf.size(), M = p.mats.size(), off_mats = p.off_mats, off_table = p.off_table;
    std::vector<unsigned char> blob(p.blob_bytes, 0);
    auto* ds = reinterpret_cast<DevSurface<T>*>(blob.data());
    for (size_t k = 0; k < S; ++k) {
        const DevSurface<double> d = lower_surface(p.surf[k]);
        DevSurface<T>& o = ds[k];
        o.kind = d.kind;
        for (int j = 0; j < 3; ++j) {
            o.c[j] = T(d.c[j]);
            o.nrm[j] = T(d.nrm[j]);
            o.ax[j] = T(d.ax[j]);
        }
        o.R = T(d.R); o.R2 = T(d.R2); o.absR = T(d.absR); o.ap = T(d.ap); o.f = T(d.f); o.sin_a = T(d.sin_a);
        o.tol = T(d.tol); o.ap_sq = T(d.ap_sq); o.shell_lo = T(d.shell_lo); o.shell_hi = T(d.shell_hi);
    }
    auto* dm = reinterpret_cast<DevMaterial<T>*>(blob.data() + off_mats);
    for (size_t k = 0; k < M; ++k) {
        const rtpb_material& m = p.mats[k];
        DevMaterial<T> d{};
        d.kind = m.kind;
        bool zero = m.kind == RTPB_SELLMEIER;
        for (int j = 0; j < 6; ++j) {
            d.c[j] = T(m.c[j]);
            zero = zero && m.c[j] == 0.0;
        }
        if (zero) d.kind = VACUUM;
        d.table_off = p.table_off[k];
        d.table_len = m.kind == RTPB_TABLE ? m.table_len : 0;
        dm[k] = d;
    }
    auto* tb = reinterpret_cast<T*>(blob.data() + off_table);
    for (size_t k = 0; k < p.table.size(); ++k) tb[k] = T(p.table[k]);
    return blob;
}

// Device copy of the plan's descriptors (created on first use per device, then immutable).
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

template <typename T, int IL, int OL, int ST, int W, int FEAT>
hipError_t launch_w(const TraceArgs<T>& a, hipStream_t st) {
    constexpr int kB = trace_block(OL, ST);
    const int64_t blocks = (a.n + kB - 1) / kB;
    hipLaunchKernelGGL((trace_kernel<T, IL, OL, ST, W, FEAT>), dim3(static_cast<unsigned>(blocks)), dim3(kB), 0, st,
                       a);
    return hipGetLastError();
}

template <typename T, int IL, int OL, int ST>
hipError_t launch_one(const TraceArgs<T>& a, int feat, hipStream_t st) {
    if constexpr (IL == RTPB_AOS && OL == RTPB_AOS && ST == 3) {       // occupancy experiments (tuning)
        const int w = g_waves_per_eu.load();
        if (w == 5) return launch_w<T, IL, OL, ST, 5, 3>(a, st);
    }
    if (feat == 0) return launch_w<T, IL, OL, ST, 1, 0>(a, st);
    if (feat == 1) return launch_w<T, IL, OL, ST, 1, 1>(a, st);
    return launch_w<T, IL, OL, ST, 1, 3>(a, st);
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
    const int64_t chunk = std::min<int64_t>(b - a, std::max<int64_t>(1 << 16, (int64_t(128) << 20) / int64_t(nslots * rec)));
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
        std::memcpy(hs.pin_in[buf], in + c0 * rec, static_cast<size_t>(m * rec));
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

// ================================================================================== C ABI
extern "C" {

int rtpb_abi_version(void) { return RTPB_ABI_VERSION; }

const char* rtpb_last_error(void) { return g_last_error.c_str(); }

int rtpb_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

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

namespace {
// Generator tables on the device: (cos, sin) pairs [n_a] then [n_b].  With host tables (the caller's
// own np.cos / np.sin / np.linspace values) they are copied; otherwise trig_table_kernel evaluates
// them with the device's libm (within an ulp of the host's).
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
thread_local PinnedStaging g_pinned;

int gen_tables(double2** tab, int64_t n_a, int64_t n_b, const double* host_a, const double* host_b, int a_pairs,
               const TrigArgs& ta, hipStream_t st) {
    const size_t bytes = size_t(n_a + n_b) * sizeof(double2);
    HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(tab), bytes, st));
    if (host_a || host_b) {
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
             const double* phi_cs, double wavelength, void* stream) {
    int rc = check_device(device);
    if (rc) return rc;
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
                    void* stream) {
    int rc = check_device(device);
    if (rc) return rc;
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

int rtpb_ray_fan(int32_t device, int32_t dtype, void* rays_out, const double pt[3], double theta_max,
                 int64_t n_thetas, int64_t nphis, const double center_ray[3], double wavelength, void* stream) {
    return fan_impl(device, dtype, rays_out, pt, theta_max, n_thetas, nphis, center_ray, nullptr, nullptr, nullptr,
                    nullptr, wavelength, stream);
}

int rtpb_ray_fan_tables(int32_t device, int32_t dtype, void* rays_out, const double pt[3], int64_t n_thetas,
                        int64_t nphis, const double center_ray[3], const double ex[3], const double ey[3],
                        const double* theta_cos_sin, const double* phi_cos_sin, double wavelength, void* stream) {
    if (!ex || !ey || !theta_cos_sin || !phi_cos_sin) return fail(RTPB_E_INVALID, "NULL table argument");
    return fan_impl(device, dtype, rays_out, pt, 0.0, n_thetas, nphis, center_ray, ex, ey, theta_cos_sin, phi_cos_sin,
                    wavelength, stream);
}

int rtpb_collimated_rays(int32_t device, int32_t dtype, void* rays_out, const double pt[3], double displacement_max,
                         int64_t n_disps, int64_t nphis, double phi_start, const double normal[3], double wavelength,
                         void* stream) {
    return collimated_impl(device, dtype, rays_out, pt, displacement_max, n_disps, nphis, phi_start, normal, nullptr,
                           nullptr, nullptr, nullptr, wavelength, stream);
}

int rtpb_collimated_rays_tables(int32_t device, int32_t dtype, void* rays_out, const double pt[3], int64_t n_disps,
                                int64_t nphis, const double normal[3], const double n1[3], const double n2[3],
                                const double* offsets, const double* phi_cos_sin, double wavelength, void* stream) {
    if (!n1 || !n2 || !offsets || !phi_cos_sin) return fail(RTPB_E_INVALID, "NULL table argument");
    return collimated_impl(device, dtype, rays_out, pt, 0.0, n_disps, nphis, 0.0, normal, n1, n2, offsets, phi_cos_sin,
                           wavelength, stream);
}

int rtpb_intersect_rays(int32_t device, int32_t dtype, const void* ray1, int64_t n1, const void* ray2, int64_t n2,
                        void* pts_out, void* stream) {
    int rc = check_device(device);
    if (rc) return rc;
    if (dtype != RTPB_F64 && dtype != RTPB_F32) return fail(RTPB_E_INVALID, "bad dtype");
    if (n1 < 0 || n2 < 0 || (n1 != n2 && n1 != 1 && n2 != 1))
        return fail(RTPB_E_INVALID, "ray1 and ray2 must be the same length");
    const int64_t n = std::max(n1, n2);
    if (n == 0) return RTPB_OK;
    if (!ray1 || !ray2 || !pts_out) return fail(RTPB_E_INVALID, "NULL pointer");
    IsectArgs a{ray1, ray2, pts_out, n, n1, n2};
    DeviceGuard g(device);
    const unsigned blocks = static_cast<unsigned>((n + kBlock - 1) / kBlock);
    if (dtype == RTPB_F64)
        hipLaunchKernelGGL(intersect_kernel<double>, dim3(blocks), dim3(kBlock), 0, static_cast<hipStream_t>(stream), a);
    else
        hipLaunchKernelGGL(intersect_kernel<float>, dim3(blocks), dim3(kBlock), 0, static_cast<hipStream_t>(stream), a);
    HIP_TRY(hipGetLastError());
    return RTPB_OK;
}

int rtpb_spot_stats(int32_t device, int32_t dtype, const void* plane, int64_t group_size, int64_t n_groups,
                    double* workspace, int64_t workspace_len, double* stats_out, void* stream) {
    int rc = check_device(device);
    if (rc) return rc;
    if (dtype != RTPB_F64 && dtype != RTPB_F32) return fail(RTPB_E_INVALID, "bad dtype");
    if (group_size <= 0 || n_groups <= 0 || !plane || !stats_out || !workspace)
        return fail(RTPB_E_INVALID, "bad spot-stats arguments");
    const int64_t tiles = (group_size + kBlock - 1) / kBlock;
    if (workspace_len < n_groups * tiles * kStats)
        return fail(RTPB_E_INVALID, "workspace too small: need n_groups * ceil(group_size/256) * 7 doubles");
    if (tiles > 65535 * 16384ll || n_groups > 65535) return fail(RTPB_E_LIMIT, "too many groups");
    SpotArgs a{plane, workspace, stats_out, group_size, n_groups, tiles};
    DeviceGuard g(device);
    hipStream_t st = static_cast<hipStream_t>(stream);
    dim3 grid(static_cast<unsigned>(tiles), static_cast<unsigned>(n_groups));
    if (dtype == RTPB_F64) hipLaunchKernelGGL(spot_partial_kernel<double>, grid, dim3(kBlock), 0, st, a);
    else hipLaunchKernelGGL(spot_partial_kernel<float>, grid, dim3(kBlock), 0, st, a);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(spot_final_kernel, dim3(static_cast<unsigned>(n_groups)), dim3(kBlock), 0, st, a);
    HIP_TRY(hipGetLastError());
    return RTPB_OK;
}

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

int rtpb_spot_sweep(const rtpb_plan* plan_c, int32_t device, int64_t n_groups, const double* group_params,
                    int64_t n_thetas, int64_t nphis, const double center_ray[3], const double ex[3],
                    const double ey[3], const double* theta_cos_sin, const double* phi_cos_sin, double* workspace,
                    int64_t workspace_len, double* stats_out, void* stream) {
    auto* plan = const_cast<rtpb_plan*>(plan_c);
    if (!plan) return fail(RTPB_E_INVALID, "plan is NULL");
    int rc = check_device(device);
    if (rc) return rc;
    if (n_groups <= 0 || n_thetas <= 0 || nphis <= 0 || !group_params || !center_ray || !ex || !ey ||
        !theta_cos_sin || !phi_cos_sin || !workspace || !stats_out)
        return fail(RTPB_E_INVALID, "bad spot-sweep arguments");
    const int64_t gsize = n_thetas * nphis;
    const int64_t tiles = (gsize + kBlock - 1) / kBlock;
    if (workspace_len < n_groups * tiles * kStats)
        return fail(RTPB_E_INVALID, "workspace too small: need n_groups * ceil(n_thetas*nphis/256) * 7 doubles");
    if (tiles > 0x7fffffffll || n_groups > 65535) return fail(RTPB_E_LIMIT, "too many groups or rays per group");
    DeviceGuard g(device);
    void* blob = nullptr;
    rc = plan_device_blob(plan, device, &blob);
    if (rc) return rc;
    hipStream_t st = static_cast<hipStream_t>(stream);
    // one upload: trig tables then the per-group parameters
    const size_t ntab = size_t(n_thetas + nphis), bytes = ntab * sizeof(double2) + size_t(4 * n_groups) * sizeof(double);
    void* dbuf = nullptr;
    HIP_TRY(hipMallocAsync(&dbuf, bytes, st));
    rc = g_pinned.reserve(bytes);
    if (rc) return rc;
    std::memcpy(g_pinned.buf, theta_cos_sin, size_t(2 * n_thetas) * sizeof(double));
    std::memcpy(g_pinned.buf + 2 * n_thetas, phi_cos_sin, size_t(2 * nphis) * sizeof(double));
    std::memcpy(g_pinned.buf + 2 * ntab, group_params, size_t(4 * n_groups) * sizeof(double));
    rc = g_pinned.upload(dbuf, bytes, st);
    if (rc) return rc;
    SweepArgs a{};
    a.surf = static_cast<const DevSurface<double>*>(blob);
    a.mats = reinterpret_cast<const DevMaterial<double>*>(static_cast<char*>(blob) + plan->off_mats);
    a.table = reinterpret_cast<const double*>(static_cast<char*>(blob) + plan->off_table);
    a.tab = static_cast<const double2*>(dbuf);
    a.grp = reinterpret_cast<const double*>(static_cast<char*>(dbuf) + ntab * sizeof(double2));
    a.partials = workspace;
    a.n_thetas = n_thetas;
    a.nphis = nphis;
    a.gsize = gsize;
    a.tiles = tiles;
    for (int j = 0; j < 3; ++j) {
        a.c[j] = center_ray[j]; a.ex[j] = ex[j]; a.ey[j] = ey[j];
    }
    a.nsurf = plan->nsurf;
    const dim3 grid(static_cast<unsigned>((tiles + 1) / 2), static_cast<unsigned>(n_groups));
    auto go = [&](auto tag) {
        using TS = decltype(tag);
        if (plan->feat == 0) hipLaunchKernelGGL((sweep_kernel<TS, 0>), grid, dim3(kBlock), 0, st, a);
        else if (plan->feat == 1) hipLaunchKernelGGL((sweep_kernel<TS, 1>), grid, dim3(kBlock), 0, st, a);
        else hipLaunchKernelGGL((sweep_kernel<TS, 3>), grid, dim3(kBlock), 0, st, a);
    };
    if (plan->dtype == RTPB_F64) go(double{});
    else go(float{});
    HIP_TRY(hipGetLastError());
    SpotArgs sa{nullptr, workspace, stats_out, gsize, n_groups, tiles};
    hipLaunchKernelGGL(spot_final_kernel, dim3(static_cast<unsigned>(n_groups)), dim3(kBlock), 0, st, sa);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipFreeAsync(dbuf, st));
    return RTPB_OK;
}

int rtpb_grid_interpolate(int32_t device, const rtpb_triangulation* tri, const double* xs, int64_t nx,
                          const double* ys, int64_t ny, double radius, double* phase_out, double* field_out,
                          void* stream) {
    int rc = check_device(device);
    if (rc) return rc;
    if (!tri || !xs || !ys || nx <= 0 || ny <= 0) return fail(RTPB_E_INVALID, "bad grid-interpolate arguments");
    if (tri->n_tri < 0 || (tri->n_tri > 0 && (!tri->transform || !tri->simplices || !tri->values)) ||
        tri->cells_x <= 0 || tri->cells_y <= 0 || !tri->cell_start || !tri->cell_tris || !(tri->cell_w > 0.0) ||
        !(tri->cell_h > 0.0))
        return fail(RTPB_E_INVALID, "bad triangulation descriptor");
    if (!phase_out && !field_out) return RTPB_OK;
    DeviceGuard g(device);
    const int64_t total = nx * ny;
    hipLaunchKernelGGL(grid_interp_kernel, dim3(static_cast<unsigned>((total + kBlock - 1) / kBlock)), dim3(kBlock),
                       0, static_cast<hipStream_t>(stream), *tri, xs, nx, ys, ny, radius, phase_out, field_out);
    HIP_TRY(hipGetLastError());
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
