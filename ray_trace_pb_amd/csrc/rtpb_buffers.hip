// rtpb_buffers.hip -- device buffers for large ray histories (rtpb_buffer_alloc / _free / _dlpack, ABI 5).
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
// Lifetime: the caller frees a buffer with rtpb_buffer_free, or hands it to a DLPack importer
// (rtpb_buffer_dlpack) whose deleter frees it.  A freed buffer is kept, still mapped, in a per-process pool
// and handed out again to the next allocation of the same size on the same device -- stream-ordered reuse,
// as PyTorch's caching allocator does it (work queued on the same stream runs after the work that used the
// buffer before); a virtual range is never unmapped and then mapped again.  Besides the most recently freed
// buffer the pool holds at most a quarter of the device's memory; beyond that, and on rtpb_buffer_trim /
// rtpb_shutdown / an allocation that finds the device full, pooled buffers are released (after a device synchronisation: no kernel may still
// use memory being unmapped).  A released buffer's virtual range stays reserved and unused, so no
// translation cached by the GPU can ever point a new buffer at released memory.
#include "rtpb_internal.h"

#include <algorithm>
#include <mutex>
#include <vector>

using namespace rtpbi;

namespace {

struct Buffer {
    int dev = 0;
    void* va = nullptr;
    size_t size = 0, chunk = 0;
    std::vector<hipMemGenericAllocationHandle_t> chunks;   // created physical chunks
    std::vector<uint64_t> mapped;                          // virtual slot of each mapped chunk
};

// Unmaps and releases the physical chunks of a buffer no one uses; its virtual range stays reserved (never
// reused), the Buffer object is deleted.
int destroy(Buffer* b) {
    DeviceGuard g(b->dev);
    hipError_t e = hipDeviceSynchronize();
    for (uint64_t s : b->mapped)
        if (hipMemUnmap(static_cast<char*>(b->va) + s * b->chunk, b->chunk) != hipSuccess) e = hipErrorUnknown;
    for (auto h : b->chunks)
        if (hipMemRelease(h) != hipSuccess) e = hipErrorUnknown;
    delete b;
    return e == hipSuccess ? RTPB_OK : fail(RTPB_E_HIP, "rtpb_buffer: releasing a mapping failed");
}

std::mutex g_pool_mu;
std::vector<Buffer*> g_pool;                       // freed buffers, still mapped, ready for reuse

// Back to the pool (newest last); the oldest pooled buffers are released while the pool holds more than a
// quarter of the device's memory.
int release(Buffer* b) {
    size_t total = 0;
    {
        DeviceGuard g(b->dev);
        size_t free_b = 0;
        if (hipMemGetInfo(&free_b, &total) != hipSuccess) total = 0;
    }
    std::vector<Buffer*> drop;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        g_pool.push_back(b);
        uint64_t held = 0;
        for (Buffer* p : g_pool)
            if (p->dev == b->dev) held += p->size;
        for (size_t k = 0; k < g_pool.size() && held > total / 4;) {
            Buffer* p = g_pool[k];
            if (p->dev == b->dev && p != b) {
                held -= p->size;
                drop.push_back(p);
                g_pool.erase(g_pool.begin() + static_cast<std::ptrdiff_t>(k));
            } else {
                ++k;
            }
        }
    }
    int rc = RTPB_OK;
    for (Buffer* p : drop)
        if (destroy(p) != RTPB_OK) rc = RTPB_E_HIP;
    return rc;
}

Buffer* take_pooled(int dev, uint64_t size, uint64_t chunk) {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (size_t k = 0; k < g_pool.size(); ++k) {
        Buffer* b = g_pool[k];
        if (b->dev == dev && b->size == size && b->chunk == chunk) {
            g_pool.erase(g_pool.begin() + static_cast<std::ptrdiff_t>(k));
            return b;
        }
    }
    return nullptr;
}

int trim_pool() {
    std::vector<Buffer*> all;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        all.swap(g_pool);
    }
    int rc = RTPB_OK;
    for (Buffer* b : all)
        if (destroy(b) != RTPB_OK) rc = RTPB_E_HIP;
    return rc;
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

extern "C" int rtpb_buffer_alloc(int32_t device, uint64_t bytes, uint64_t chunk_bytes, uint64_t seed, void** ptr,
                                 void** handle) {
    if (!ptr || !handle || bytes == 0 || bytes > (1ull << 50))
        return fail(RTPB_E_INVALID, "rtpb_buffer_alloc: null output, zero size or more than 1 PiB");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail(RTPB_E_NODEV, "rtpb_buffer_alloc: no such device");
    DeviceGuard g(device);
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    size_t gran = 0;
    HIP_TRY(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
    gran = std::max<size_t>(gran, 1);
    auto round_up = [](uint64_t v, uint64_t m) { return (v + m - 1) / m * m; };
    const uint64_t want = chunk_bytes ? chunk_bytes : (64ull << 20);
    // a buffer smaller than one chunk is a single chunk of its own (rounded) size
    const uint64_t chunk = round_up(std::min<uint64_t>(want, round_up(bytes, gran)), gran);
    const uint64_t n = (bytes + chunk - 1) / chunk;
    if (Buffer* p = take_pooled(device, n * chunk, chunk)) {
        *ptr = p->va;
        *handle = p;
        return RTPB_OK;
    }
    auto* b = new Buffer;
    b->dev = device;
    b->size = n * chunk;
    b->chunk = chunk;
    // chunk-aligned virtual range when the chunk is a power of two (large translation fragments), else the
    // allocation granularity (a small buffer's single chunk)
    const uint64_t align = (chunk & (chunk - 1)) == 0 ? chunk : gran;
    if (hipMemAddressReserve(&b->va, b->size, align, nullptr, 0) != hipSuccess) {
        b->va = nullptr;
        (void)destroy(b);
        return fail(RTPB_E_HIP, "rtpb_buffer_alloc: hipMemAddressReserve failed");
    }
    std::vector<uint64_t> slot(n);
    for (uint64_t k = 0; k < n; ++k) slot[k] = k;
    uint64_t x = seed;
    for (uint64_t k = n; k > 1; --k) std::swap(slot[k - 1], slot[mix(x) % k]);     // Fisher-Yates
    b->chunks.reserve(n);
    b->mapped.reserve(n);
    for (uint64_t k = 0; k < n; ++k) {
        hipMemGenericAllocationHandle_t h;
        if (hipMemCreate(&h, chunk, &prop, 0) != hipSuccess) {
            // out of memory: release the pooled buffers' memory once and retry
            if (trim_pool() != RTPB_OK || hipMemCreate(&h, chunk, &prop, 0) != hipSuccess) {
                (void)destroy(b);
                return fail(RTPB_E_HIP, "rtpb_buffer_alloc: hipMemCreate failed (out of device memory?)");
            }
        }
        b->chunks.push_back(h);
        if (hipMemMap(static_cast<char*>(b->va) + slot[k] * chunk, chunk, 0, h, 0) != hipSuccess) {
            (void)destroy(b);
            return fail(RTPB_E_HIP, "rtpb_buffer_alloc: hipMemMap failed");
        }
        b->mapped.push_back(slot[k]);
    }
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    if (hipMemSetAccess(b->va, b->size, &acc, 1) != hipSuccess) {
        (void)destroy(b);
        return fail(RTPB_E_HIP, "rtpb_buffer_alloc: hipMemSetAccess failed");
    }
    *ptr = b->va;
    *handle = b;
    return RTPB_OK;
}

extern "C" int rtpb_buffer_free(void* handle) {
    if (!handle) return fail(RTPB_E_INVALID, "rtpb_buffer_free: null handle");
    return release(static_cast<Buffer*>(handle));
}

extern "C" int rtpb_buffer_trim(void) { return trim_pool(); }

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
