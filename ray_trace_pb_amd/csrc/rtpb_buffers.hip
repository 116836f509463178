// rtpb_buffers.hip -- device buffers for large ray histories (rtpb_buffer_alloc / _free / _dlpack /
// _record_stream, ABI 6).
//
// A history is 2S+1 planes written concurrently by every wave (C3: 19 float32 planes of 1.6 GB).  That
// many-plane write pattern runs at a rate that depends on where the buffer's physical memory lies: into a
// physically contiguous allocation (hipDeviceMallocContiguous, and often the first large hipMalloc of a
// process on an unfragmented card) it is 15-20 % slower at full C3 size and ~45 % slower at quarter size,
// while a plain fill of the same memory is not (profiles/r03/placement/).  These buffers
// map their physical memory in chunks (64 MiB by default) whose order in the virtual range is a seeded
// shuffle (HIP virtual memory API), so the relative physical placement of the planes is randomised whatever
// the state of VRAM: every such buffer measured at the fast rate.
//
// Lifetime and streams (the semantics of PyTorch's caching allocator, made explicit):
//   * a buffer is allocated FOR a stream (its allocation stream); work on that stream is ordered anyway;
//   * rtpb_buffer_record_stream(ptr, s) marks a use on another stream s (torch's Tensor.record_stream, which
//     does nothing for memory torch did not allocate -- io.HistoryWriter and ray_trace_pb_amd.record_stream
//     call both);
//   * freeing (rtpb_buffer_free, or the DLPack deleter) records one event on the allocation stream and on
//     every recorded stream -- it never blocks;
//   * a freed buffer stays mapped in a per-device pool; the next allocation of the same size on that device
//     takes it and makes ITS stream wait (hipStreamWaitEvent, on the device) for those events, so no kernel
//     of the new owner can touch the memory before the previous owner's last recorded use has finished;
//   * the pool keeps only the most recently freed buffer per device (rtpb_set_tuning("buffer_pool_buffers")
//     sets k, 0 = none); older ones retire.  A retired buffer stays mapped until a call that may block
//     releases it: the next allocation that maps new memory (rtpb_buffer_alloc without a pooled match, or a
//     torch segment, rtpb_torch_alloc -- not while its stream is capturing a graph), rtpb_buffer_trim,
//     rtpb_shutdown.  Those synchronise the device and unmap every retired buffer; a free, a pooled
//     allocation and rtpb_buffer_held never block (ABI 8: a free inside a DLPack deleter, i.e. a Python
//     tensor's destructor, can run during stream capture).
//
// torch's own caching allocator can use the same memory (ABI 7): rtpb_torch_alloc / rtpb_torch_free are the
// allocation functions of a torch.cuda.memory.CUDAPluggableAllocator behind a torch.cuda.MemPool
// (ray_trace_pb_amd._engine.history_pool).  torch then owns streams, caching, record_stream, statistics and
// out-of-memory handling of those segments; the library only maps (alloc) and unmaps (free) them.
//
// Releasing a mapping always follows a device synchronisation: torch frees without a device sync, and a use on a
// stream never recorded may still be in flight (HIP's unmap, unlike hipFree, does not wait for it).  The
// virtual range of a buffer a kernel may have used is kept reserved (a range freed and reserved
// again took writes through its old translations in round 4); those dead ranges are counted
// (rtpb_buffer_stats), and once they exceed rtpb_set_tuning("buffer_dead_va_limit", bytes) new buffers are
// plain hipMalloc allocations (correct, without the shuffled placement).
#include "rtpb_internal.h"

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <vector>

using namespace rtpbi;

namespace {

struct Buffer {
    int dev = 0;
    void* va = nullptr;
    size_t size = 0, chunk = 0;
    bool plain = false;                                    // hipMalloc'd (dead-VA budget spent): hipFree
    std::vector<hipMemGenericAllocationHandle_t> chunks;   // created physical chunks
    std::vector<uint64_t> mapped;                          // virtual slot of each mapped chunk
    hipStream_t alloc_stream = nullptr;                    // the stream the current owner allocated it for
    std::vector<hipStream_t> used;                         // other streams recorded by the current owner
    std::vector<hipEvent_t> pending;                       // after free: the owner's last use on each stream
};

std::mutex g_mu;                                 // guards everything below
std::map<uintptr_t, Buffer*> g_live;             // buffers owned by a caller, by virtual address
std::vector<Buffer*> g_pool;                     // freed, still mapped, ready for reuse (newest last)
std::vector<Buffer*> g_retired;                  // freed, leaving the pool: destroyed once `pending` is done
size_t g_pool_keep = 1;                          // pooled buffers kept per device
std::map<uintptr_t, Buffer*> g_torch;            // live segments of torch MemPools (rtpb_torch_alloc)
uint64_t g_dead_va = 0;                          // reserved virtual bytes of released mappings (never reused)
uint64_t g_dead_ranges = 0, g_plain = 0, g_torch_allocs = 0, g_torch_frees = 0;
uint64_t g_dead_va_limit = 32ull << 40;          // beyond this, new buffers are plain hipMalloc allocations
std::atomic<uint64_t> g_torch_seed{0x7a11};      // shuffle seeds of torch-pool segments

int stream_device(hipStream_t s, int fallback) {
    int d = fallback;
    if (s != nullptr && hipStreamGetDevice(s, &d) != hipSuccess) d = fallback;
    return d;
}

void drop_events(Buffer* b) {
    for (hipEvent_t e : b->pending) (void)hipEventDestroy(e);
    b->pending.clear();
}

// Unmaps and releases the physical chunks of a buffer, after waiting for the recorded uses of its last owner
// (b->pending) and -- unless the caller has just done so (`synced`) -- for the whole device: a use on a stream
// nobody recorded may still be in flight, and an unmap does not wait for it.  `used`: a kernel may have touched
// the memory -- its virtual range then stays reserved (counted in g_dead_va); a buffer no kernel saw (an
// allocation that failed half way) frees it.  The Buffer object is deleted.
int destroy(Buffer* b, bool used = true, bool synced = false) {
    DeviceGuard g(b->dev);
    hipError_t e = hipSuccess;
    for (hipEvent_t ev : b->pending)
        if (hipEventSynchronize(ev) != hipSuccess) e = hipErrorUnknown;
    drop_events(b);
    if (used && !synced && hipDeviceSynchronize() != hipSuccess) e = hipErrorUnknown;
    if (b->plain) {
        if (b->va && hipFree(b->va) != hipSuccess) e = hipErrorUnknown;
    } else {
        for (uint64_t s : b->mapped)
            if (hipMemUnmap(static_cast<char*>(b->va) + s * b->chunk, b->chunk) != hipSuccess) e = hipErrorUnknown;
        for (auto h : b->chunks)
            if (hipMemRelease(h) != hipSuccess) e = hipErrorUnknown;
        if (b->va && !used) {
            if (hipMemAddressFree(b->va, b->size) != hipSuccess) e = hipErrorUnknown;
        } else if (b->va) {
            // The virtual range is NOT freed: a range freed and reserved again by a later buffer was seen to
            // take writes through translations still cached for the old mapping (partial histories,
            // profiles/r04/buffers_va_reuse.log).  Kept reserved it is never touched again; the cost is
            // address space, counted here and bounded by g_dead_va_limit.
            std::lock_guard<std::mutex> lk(g_mu);
            g_dead_va += b->size;
            ++g_dead_ranges;
        }
    }
    delete b;
    return e == hipSuccess ? RTPB_OK : fail(RTPB_E_HIP, "rtpb_buffer: releasing a mapping failed");
}

// Destroys `v`: one device synchronisation per device involved, then every unmap.
int destroy_all(const std::vector<Buffer*>& v) {
    int rc = RTPB_OK;
    std::vector<int> synced;
    for (Buffer* b : v) {
        if (std::find(synced.begin(), synced.end(), b->dev) != synced.end()) continue;
        DeviceGuard g(b->dev);
        if (hipDeviceSynchronize() != hipSuccess) rc = RTPB_E_HIP;
        synced.push_back(b->dev);
    }
    for (Buffer* b : v)
        if (destroy(b, true, true) != RTPB_OK) rc = RTPB_E_HIP;
    return rc;
}

// Every retired buffer (a blocking point: the device is synchronised before the unmaps).  Not while `stream`
// captures a graph -- a device synchronisation would invalidate the capture; the buffers wait for a later call.
int release_retired(hipStream_t stream) {
    if (stream != nullptr) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(stream, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
            (void)hipGetLastError();
            return RTPB_OK;
        }
    }
    std::vector<Buffer*> all;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        all.swap(g_retired);
    }
    return destroy_all(all);
}

// The owner's last use on each stream it used, as events (the free itself never waits).
int record_pending(Buffer* b) {
    std::vector<hipStream_t> streams{b->alloc_stream};
    for (hipStream_t s : b->used) streams.push_back(s);
    b->used.clear();
    int rc = RTPB_OK;
    for (hipStream_t s : streams) {
        DeviceGuard g(stream_device(s, b->dev));
        hipEvent_t ev = nullptr;
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
            rc = fail(RTPB_E_HIP, "rtpb_buffer_free: hipEventCreate failed");
            (void)hipDeviceSynchronize();       // no event: the conservative fallback
            continue;
        }
        if (hipEventRecord(ev, s) != hipSuccess) {
            (void)hipEventDestroy(ev);
            rc = fail(RTPB_E_HIP, "rtpb_buffer_free: hipEventRecord failed");
            (void)hipDeviceSynchronize();
            continue;
        }
        b->pending.push_back(ev);
    }
    return rc;
}

// Back to the pool (newest last); beyond g_pool_keep per device the oldest pooled buffers retire.
int release(Buffer* b) {
    int rc = record_pending(b);
    {
        std::lock_guard<std::mutex> lk(g_mu);
        g_live.erase(reinterpret_cast<uintptr_t>(b->va));
        g_pool.push_back(b);
        size_t held = 0;
        for (Buffer* p : g_pool) held += p->dev == b->dev;
        for (size_t k = 0; k < g_pool.size() && held > g_pool_keep;) {
            Buffer* p = g_pool[k];
            if (p->dev == b->dev && (p != b || g_pool_keep == 0)) {
                --held;
                g_retired.push_back(p);
                g_pool.erase(g_pool.begin() + static_cast<std::ptrdiff_t>(k));
            } else {
                ++k;
            }
        }
    }
    return rc;
}

// A pooled buffer of this size for `stream`: the stream waits (on the device) for the previous owner's uses.
Buffer* take_pooled(int dev, uint64_t size, uint64_t chunk, hipStream_t stream) {
    Buffer* b = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (size_t k = g_pool.size(); k-- > 0;) {
            Buffer* p = g_pool[k];
            if (p->dev == dev && p->size == size && p->chunk == chunk) {
                g_pool.erase(g_pool.begin() + static_cast<std::ptrdiff_t>(k));
                b = p;
                break;
            }
        }
    }
    if (!b) return nullptr;
    for (hipEvent_t ev : b->pending) {
        if (hipEventQuery(ev) == hipSuccess) continue;
        if (hipStreamWaitEvent(stream, ev, 0) != hipSuccess) (void)hipEventSynchronize(ev);
    }
    drop_events(b);
    return b;
}

// Every pooled and retired buffer of `dev` (-1: all devices), waiting for their last uses.
int trim_pool(int dev) {
    std::vector<Buffer*> all;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (auto* list : {&g_pool, &g_retired})
            for (size_t k = 0; k < list->size();) {
                if (dev < 0 || (*list)[k]->dev == dev) {
                    all.push_back((*list)[k]);
                    list->erase(list->begin() + static_cast<std::ptrdiff_t>(k));
                } else {
                    ++k;
                }
            }
    }
    return destroy_all(all);
}

void own(Buffer* b, hipStream_t stream) {
    b->alloc_stream = stream;
    b->used.clear();
    std::lock_guard<std::mutex> lk(g_mu);
    g_live[reinterpret_cast<uintptr_t>(b->va)] = b;
}

// splitmix64: the shuffle's generator
uint64_t mix(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// DLPack v0.8 (the ABI PyTorch's from_dlpack imports)
struct DLDevice { int32_t device_type; int32_t device_id; };
struct DLDataType { uint8_t code; uint8_t bits; uint16_t lanes; };
struct DLTensor {
    void* data;
    DLDevice device;
    int32_t ndim;
    DLDataType dtype;
    int64_t* shape;
    int64_t* strides;
    uint64_t byte_offset;
};
struct DLManagedTensor {
    DLTensor dl_tensor;
    void* manager_ctx;
    void (*deleter)(DLManagedTensor*);
};
constexpr int32_t kDLROCM = 10;
constexpr uint8_t kDLFloat = 2;

struct Managed {
    DLManagedTensor t;
    std::vector<int64_t> shape;
    Buffer* buf;
};

void managed_deleter(DLManagedTensor* t) {
    auto* m = static_cast<Managed*>(t->manager_ctx);
    (void)release(m->buf);
    delete m;
}

}  // namespace

namespace rtpbi {
// rtpb_set_tuning("buffer_pool_buffers", k): pooled buffers kept per device (>= 0)
int set_buffer_pool_keep(int64_t k) {
    if (k < 0 || k > 1024) return fail(RTPB_E_INVALID, "rtpb_set_tuning: buffer_pool_buffers must be 0..1024");
    {
        std::lock_guard<std::mutex> lk(g_mu);
        g_pool_keep = static_cast<size_t>(k);
    }
    return RTPB_OK;
}

// rtpb_set_tuning("buffer_dead_va_limit", bytes): reserved virtual bytes of released mappings before new
// buffers fall back to plain hipMalloc allocations
int set_buffer_dead_va_limit(int64_t bytes) {
    if (bytes < 0) return fail(RTPB_E_INVALID, "rtpb_set_tuning: buffer_dead_va_limit must be >= 0");
    std::lock_guard<std::mutex> lk(g_mu);
    g_dead_va_limit = static_cast<uint64_t>(bytes);
    return RTPB_OK;
}
}  // namespace rtpbi

namespace {

hipMemAllocationProp device_prop(int32_t device) {
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    return prop;
}

// Chunk size and count of a buffer of `bytes` (`chunk_bytes` 0: 64 MiB; a buffer smaller than one chunk is a
// single chunk of its own size, rounded to the allocation granularity); the caller has set the device.
int chunk_geometry(int32_t device, uint64_t bytes, uint64_t chunk_bytes, uint64_t* chunk, uint64_t* n,
                   uint64_t* gran_out = nullptr) {
    hipMemAllocationProp prop = device_prop(device);
    size_t gran = 0;
    HIP_TRY(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    gran = std::max<size_t>(gran, 1);
    auto round_up = [](uint64_t v, uint64_t m) { return (v + m - 1) / m * m; };
    const uint64_t want = chunk_bytes ? chunk_bytes : (64ull << 20);
    *chunk = round_up(std::min<uint64_t>(want, round_up(bytes, gran)), gran);
    *n = (bytes + *chunk - 1) / *chunk;
    if (gran_out) *gran_out = gran;
    return RTPB_OK;
}

// A new buffer of at least `bytes` on `device`: physical chunks mapped in a shuffled order into a fresh
// virtual range -- or, once the dead virtual ranges exceed g_dead_va_limit, one plain hipMalloc allocation.
// Retired buffers are released first (release_retired: unless `stream` is capturing).  Out of device memory,
// the library's pooled and retired buffers of the device are released once and the allocation retried.
int map_new(int32_t device, uint64_t bytes, uint64_t chunk_bytes, uint64_t seed, hipStream_t stream, Buffer** out) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail(RTPB_E_NODEV, "rtpb_buffer_alloc: no such device");
    DeviceGuard g(device);
    (void)release_retired(stream);
    const hipMemAllocationProp prop = device_prop(device);
    uint64_t chunk = 0, n = 0, gran = 1;
    const int rc = chunk_geometry(device, bytes, chunk_bytes, &chunk, &n, &gran);
    if (rc != RTPB_OK) return rc;
    auto* b = new Buffer;
    b->dev = device;
    b->size = n * chunk;
    b->chunk = chunk;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        b->plain = g_dead_va + b->size > g_dead_va_limit;
        g_plain += b->plain;
    }
    if (b->plain) {
        if (hipMalloc(&b->va, b->size) != hipSuccess &&
            (trim_pool(device) != RTPB_OK || hipMalloc(&b->va, b->size) != hipSuccess)) {
            b->va = nullptr;
            (void)destroy(b, false);
            return fail(RTPB_E_HIP, "rtpb_buffer_alloc: hipMalloc failed (out of device memory?)");
        }
        *out = b;
        return RTPB_OK;
    }
    // chunk-aligned virtual range when the chunk is a power of two (large translation fragments), else the
    // allocation granularity (a small buffer's single chunk)
    const uint64_t align = (chunk & (chunk - 1)) == 0 ? chunk : gran;
    if (hipMemAddressReserve(&b->va, b->size, align, nullptr, 0) != hipSuccess) {
        b->va = nullptr;
        (void)destroy(b, false);
        return fail(RTPB_E_HIP, "rtpb_buffer_alloc: hipMemAddressReserve failed");
    }
    std::vector<uint64_t> slot(n);
    for (uint64_t k = 0; k < n; ++k) slot[k] = k;
    uint64_t x = seed;
    for (uint64_t k = n; k > 1; --k) std::swap(slot[k - 1], slot[mix(x) % k]);     // Fisher-Yates
    b->chunks.reserve(n);
    b->mapped.reserve(n);
    bool trimmed = false;
    for (uint64_t k = 0; k < n; ++k) {
        hipMemGenericAllocationHandle_t h;
        if (hipMemCreate(&h, chunk, &prop, 0) != hipSuccess) {
            // out of memory: release the pooled and retired buffers of this device once and retry
            if (trimmed || trim_pool(device) != RTPB_OK || hipMemCreate(&h, chunk, &prop, 0) != hipSuccess) {
                (void)destroy(b, false);
                return fail(RTPB_E_HIP, "rtpb_buffer_alloc: hipMemCreate failed (out of device memory?)");
            }
            trimmed = true;
        }
        b->chunks.push_back(h);
        if (hipMemMap(static_cast<char*>(b->va) + slot[k] * chunk, chunk, 0, h, 0) != hipSuccess) {
            (void)destroy(b, false);
            return fail(RTPB_E_HIP, "rtpb_buffer_alloc: hipMemMap failed");
        }
        b->mapped.push_back(slot[k]);
    }
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    if (hipMemSetAccess(b->va, b->size, &acc, 1) != hipSuccess) {
        (void)destroy(b, false);
        return fail(RTPB_E_HIP, "rtpb_buffer_alloc: hipMemSetAccess failed");
    }
    *out = b;
    return RTPB_OK;
}

}  // namespace

extern "C" int rtpb_buffer_alloc(int32_t device, uint64_t bytes, uint64_t chunk_bytes, uint64_t seed, void* stream,
                                 void** ptr, void** handle) {
    if (!ptr || !handle || bytes == 0 || bytes > (1ull << 50))
        return fail(RTPB_E_INVALID, "rtpb_buffer_alloc: null output, zero size or more than 1 PiB");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail(RTPB_E_NODEV, "rtpb_buffer_alloc: no such device");
    const auto st = static_cast<hipStream_t>(stream);
    {
        DeviceGuard g(device);
        uint64_t chunk = 0, n = 0;
        const int rc = chunk_geometry(device, bytes, chunk_bytes, &chunk, &n);
        if (rc != RTPB_OK) return rc;
        if (Buffer* p = take_pooled(device, n * chunk, chunk, st)) {
            own(p, st);
            *ptr = p->va;
            *handle = p;
            return RTPB_OK;
        }
    }
    Buffer* b = nullptr;
    const int rc = map_new(device, bytes, chunk_bytes, seed, st, &b);
    if (rc != RTPB_OK) return rc;
    own(b, st);
    *ptr = b->va;
    *handle = b;
    return RTPB_OK;
}

// torch.cuda.memory.CUDAPluggableAllocator(librtpb.so, "rtpb_torch_alloc", "rtpb_torch_free"): a segment of a
// torch MemPool -- a fresh shuffled-chunk mapping (torch's caching allocator caches and reuses it).  NULL on
// failure (torch then frees its cached blocks and retries, or raises its out-of-memory error).
extern "C" void* rtpb_torch_alloc(int64_t size, int32_t device, void* stream) {
    if (size <= 0) return nullptr;
    Buffer* b = nullptr;
    if (map_new(device, static_cast<uint64_t>(size), 0, g_torch_seed.fetch_add(1), static_cast<hipStream_t>(stream),
                &b) != RTPB_OK)
        return nullptr;
    std::lock_guard<std::mutex> lk(g_mu);
    g_torch[reinterpret_cast<uintptr_t>(b->va)] = b;
    ++g_torch_allocs;
    return b->va;
}

extern "C" void rtpb_torch_free(void* ptr, int64_t size, int32_t device, void* stream) {
    (void)size, (void)device, (void)stream;
    Buffer* b = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_torch.find(reinterpret_cast<uintptr_t>(ptr));
        if (it == g_torch.end()) return;
        b = it->second;
        g_torch.erase(it);
        ++g_torch_frees;
    }
    (void)destroy(b);
}

extern "C" int rtpb_buffer_stats(int32_t device, uint64_t* out, int32_t n) {
    if (!out || n < 0) return fail(RTPB_E_INVALID, "rtpb_buffer_stats: null output");
    uint64_t v[8] = {};
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (const auto& kv : g_torch)
            if (device < 0 || kv.second->dev == device) {
                v[0] += kv.second->size;
                ++v[1];
            }
        v[2] = g_dead_va;
        v[3] = g_dead_ranges;
        v[4] = g_plain;
        v[5] = g_torch_allocs;
        v[6] = g_torch_frees;
        v[7] = g_dead_va_limit;
    }
    for (int32_t k = 0; k < n && k < 8; ++k) out[k] = v[k];
    return RTPB_OK;
}

extern "C" int rtpb_buffer_free(void* handle) {
    if (!handle) return fail(RTPB_E_INVALID, "rtpb_buffer_free: null handle");
    return release(static_cast<Buffer*>(handle));
}

extern "C" int rtpb_buffer_record_stream(const void* ptr, void* stream) {
    const auto p = reinterpret_cast<uintptr_t>(ptr);
    const auto st = static_cast<hipStream_t>(stream);
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_live.upper_bound(p);
    if (it == g_live.begin()) return 1;
    --it;
    Buffer* b = it->second;
    if (p >= it->first + b->size) return 1;                   // not inside a live history buffer
    if (st != b->alloc_stream && std::find(b->used.begin(), b->used.end(), st) == b->used.end())
        b->used.push_back(st);
    return RTPB_OK;
}

extern "C" int rtpb_buffer_trim(void) { return trim_pool(-1); }

extern "C" int rtpb_buffer_held(int32_t device, uint64_t* bytes, int32_t* buffers) {
    if (!bytes || !buffers) return fail(RTPB_E_INVALID, "rtpb_buffer_held: null output");
    uint64_t tot = 0;
    int32_t cnt = 0;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        for (auto* list : {&g_pool, &g_retired})
            for (Buffer* b : *list)
                if (device < 0 || b->dev == device) {
                    tot += b->size;
                    ++cnt;
                }
    }
    *bytes = tot;
    *buffers = cnt;
    return RTPB_OK;
}

extern "C" int rtpb_buffer_dlpack(void* handle, int32_t ndim, const int64_t* shape, int32_t dtype, void** managed) {
    if (!handle || !managed || ndim < 1 || ndim > 8 || !shape)
        return fail(RTPB_E_INVALID, "rtpb_buffer_dlpack: bad arguments");
    if (dtype != RTPB_F64 && dtype != RTPB_F32) return fail(RTPB_E_INVALID, "rtpb_buffer_dlpack: dtype");
    auto* b = static_cast<Buffer*>(handle);
    const uint64_t w = dtype == RTPB_F64 ? 8 : 4;
    uint64_t elems = 1;
    for (int k = 0; k < ndim; ++k) {
        if (shape[k] < 0) return fail(RTPB_E_INVALID, "rtpb_buffer_dlpack: negative extent");
        elems *= static_cast<uint64_t>(shape[k]);
    }
    if (elems * w > b->size) return fail(RTPB_E_INVALID, "rtpb_buffer_dlpack: shape exceeds the buffer");
    auto* m = new Managed;
    m->buf = b;
    m->shape.assign(shape, shape + ndim);
    m->t.dl_tensor.data = b->va;
    m->t.dl_tensor.device = DLDevice{kDLROCM, b->dev};
    m->t.dl_tensor.ndim = ndim;
    m->t.dl_tensor.dtype = DLDataType{kDLFloat, static_cast<uint8_t>(8 * w), 1};
    m->t.dl_tensor.shape = m->shape.data();
    m->t.dl_tensor.strides = nullptr;                 // C-contiguous
    m->t.dl_tensor.byte_offset = 0;
    m->t.manager_ctx = m;
    m->t.deleter = managed_deleter;
    *managed = &m->t;
    return RTPB_OK;
}

extern "C" int rtpb_buffer_dlpack_discard(void* managed) {
    if (!managed) return fail(RTPB_E_INVALID, "rtpb_buffer_dlpack_discard: null");
    auto* t = static_cast<DLManagedTensor*>(managed);
    t->deleter(t);
    return RTPB_OK;
}
