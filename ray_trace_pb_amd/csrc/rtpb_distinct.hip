// rtpb_distinct.hip -- the distinct wavelengths of a device-resident bundle (the keys of the plan's
// RTPB_TABLE materials: Ebaf11 and user Material subclasses are evaluated by their own n() on the host at
// exactly these wavelengths).  One pass over the wavelength column into a small open-addressing hash set
// in device memory, instead of a full sort (torch.unique) of the column.
//
// Each wave deduplicates its 64 values in registers (ballot / leader broadcast), keeps the last few keys
// it inserted, and only inserts keys it has not seen with a global 64-bit compare-and-swap -- so a
// one-colour 50M-ray bundle costs a few thousand atomics, and the pass runs at the speed of reading the
// column (every 64-byte ray record is touched once).
#include "rtpb_internal.h"

using namespace rtpbi;

namespace {

constexpr uint64_t kEmpty = ~0ull;                       // a NaN payload canonicalisation never produces
constexpr uint64_t kNaNKey = 0x7ff8000000000000ull;      // every NaN wavelength -> one key
constexpr int kDistinctBlock = 256;
constexpr int kWaveCache = 4;

__device__ __forceinline__ uint64_t canon_key(double v) {
    if (v != v) return kNaNKey;
    if (v == 0.0) return 0ull;                           // -0.0 and +0.0 compare equal in the table lookup
    return static_cast<uint64_t>(__double_as_longlong(v));
}

__device__ __forceinline__ uint32_t slot_of(uint64_t k, uint32_t mask) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    return static_cast<uint32_t>(k) & mask;
}

struct DistinctArgs {
    const void* col;
    int64_t n, stride;                                   // elements between consecutive wavelengths
    unsigned long long* table;                           // slots (power of two), pre-filled with kEmpty
    uint32_t mask;
    uint32_t max_keys;                                   // insert at most this many (<= slots / 2)
    unsigned int* count;                                 // keys inserted; > max_keys = overflow
    int32_t f32;
};

constexpr unsigned int kOverflow = 0x40000000u;        // count value marking "more than max_keys keys"

__device__ __forceinline__ bool overflowed(const DistinctArgs& a) {
    return __hip_atomic_load(a.count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > a.max_keys;
}

__device__ void insert_key(const DistinctArgs& a, uint64_t k) {
    uint32_t s = slot_of(k, a.mask);
    for (uint32_t probe = 0; probe <= a.mask; ++probe) {
        const unsigned long long prev = atomicCAS(a.table + s, static_cast<unsigned long long>(kEmpty),
                                                  static_cast<unsigned long long>(k));
        if (prev == kEmpty) {
            if (atomicAdd(a.count, 1u) >= a.max_keys) atomicMax(a.count, kOverflow);
            return;
        }
        if (prev == k) return;
        s = (s + 1) & a.mask;
    }
    atomicMax(a.count, kOverflow);                       // table full (cannot happen below max_keys)
}

// each wave takes kUnroll consecutive 64-value groups per step: all kUnroll loads are issued before the
// first value is used, so every wave keeps several cache-line reads in flight
constexpr int kUnroll = 4;

__global__ __launch_bounds__(kDistinctBlock) void distinct_kernel(DistinctArgs a) {
    const int lane = threadIdx.x & 63;
    uint64_t cache[kWaveCache];
#pragma unroll
    for (int c = 0; c < kWaveCache; ++c) cache[c] = kEmpty;
    int next = 0;
    const int64_t step = static_cast<int64_t>(gridDim.x) * kDistinctBlock * kUnroll;
    for (int64_t i0 = (static_cast<int64_t>(blockIdx.x) * kDistinctBlock + (threadIdx.x & ~63)) * kUnroll; i0 < a.n;
         i0 += step) {
        uint64_t keys[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t i = i0 + 64 * u + lane;
            keys[u] = kEmpty;
            if (i < a.n) {
                const double v = a.f32 ? static_cast<double>(static_cast<const float*>(a.col)[i * a.stride])
                                       : static_cast<const double*>(a.col)[i * a.stride];
                keys[u] = canon_key(v);
            }
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const uint64_t key = keys[u];
            bool pending = key != kEmpty;
#pragma unroll
            for (int c = 0; c < kWaveCache; ++c) pending = pending && key != cache[c];
            // wave-uniform loop: the lowest pending lane's key is handled for every lane holding it
            uint64_t mask = __ballot(pending);
            while (mask) {
                const int leader = __ffsll(static_cast<unsigned long long>(mask)) - 1;
                const uint64_t lk = __shfl(key, leader);
                if (key == lk) pending = false;
                if (lane == leader && !overflowed(a)) insert_key(a, lk);
                cache[next] = lk;                        // uniform: every lane keeps the same cache
                next = (next + 1) % kWaveCache;
                mask = __ballot(pending);
            }
        }
        // more distinct keys than the caller wants: the answer is "overflow", stop reading
        if (__shfl(static_cast<int>(lane == 0 && overflowed(a)), 0)) break;
    }
}

}  // namespace

extern "C" {

int rtpb_distinct_keys(int32_t device, const void* col, int32_t dtype, int64_t n, int64_t stride, uint64_t* table,
                       int32_t table_slots, int32_t max_keys, uint32_t* count, void* stream) {
    int rc = check_device(device);
    if (rc) return rc;
    if (n < 0 || stride < 1 || !table || !count || (n > 0 && !col)) return fail(RTPB_E_INVALID, "bad distinct-keys arguments");
    if (dtype != RTPB_F64 && dtype != RTPB_F32) return fail(RTPB_E_INVALID, "bad dtype");
    if (table_slots < 2 || (table_slots & (table_slots - 1)))
        return fail(RTPB_E_INVALID, "table_slots must be a power of two >= 2");
    if (max_keys < 1 || max_keys > table_slots / 2) return fail(RTPB_E_INVALID, "max_keys must lie in [1, table_slots/2]");
    DeviceGuard g(device);
    hipStream_t st = static_cast<hipStream_t>(stream);
    HIP_TRY(hipMemsetAsync(table, 0xff, static_cast<size_t>(table_slots) * sizeof(uint64_t), st));
    HIP_TRY(hipMemsetAsync(count, 0, sizeof(uint32_t), st));
    if (n == 0) return RTPB_OK;
    DistinctArgs a{};
    a.col = col;
    a.n = n;
    a.stride = stride;
    a.table = reinterpret_cast<unsigned long long*>(table);
    a.mask = static_cast<uint32_t>(table_slots - 1);
    a.max_keys = static_cast<uint32_t>(max_keys);
    a.count = count;
    a.f32 = dtype == RTPB_F32;
    // enough waves to saturate HBM, few enough that the per-wave caches keep the atomics rare
    const int64_t need = (n + kDistinctBlock * kUnroll - 1) / (kDistinctBlock * kUnroll);
    const int64_t grid = need < 4096 ? need : 4096;
    hipLaunchKernelGGL(distinct_kernel, dim3(static_cast<unsigned>(grid)), dim3(kDistinctBlock), 0, st, a);
    HIP_TRY(hipGetLastError());
    return RTPB_OK;
}

}  // extern "C"
