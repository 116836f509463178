// scatter_alloc.hip -- EXPERIMENT: a device buffer whose physical chunks are mapped into its virtual range in a
// shuffled order (HIP virtual memory API), so the physical placement of the history planes relative to each
// other is randomised at `chunk` granularity whatever the state of VRAM.  Built as a shared library for
// tools/placement_alloc.py:
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/_build/libscatter_alloc.so tools/scatter_alloc.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

struct Scatter {
    void* va = nullptr;
    size_t size = 0, chunk = 0;
    std::vector<hipMemGenericAllocationHandle_t> h;
};

extern "C" int scatter_alloc(int dev, size_t bytes, size_t chunk_bytes, uint64_t seed, void** out, void** handle) {
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    size_t g = 0;
    if (hipMemGetAllocationGranularity(&g, &prop, hipMemAllocationGranularityMinimum) != hipSuccess) return 1;
    const size_t chunk = (chunk_bytes + g - 1) / g * g;
    const size_t n = (bytes + chunk - 1) / chunk;
    auto* s = new Scatter;
    s->size = n * chunk;
    s->chunk = chunk;
    if (hipMemAddressReserve(&s->va, s->size, chunk, nullptr, 0) != hipSuccess) { delete s; return 2; }
    std::vector<size_t> perm(n);
    for (size_t k = 0; k < n; ++k) perm[k] = k;
    uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
    for (size_t k = n; k > 1; --k) {                     // Fisher-Yates, splitmix-style generator
        x += 0x9E3779B97F4A7C15ull;
        uint64_t z = x;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        const size_t j = static_cast<size_t>(z % k);
        std::swap(perm[k - 1], perm[j]);
    }
    s->h.resize(n);
    for (size_t k = 0; k < n; ++k) {
        if (hipMemCreate(&s->h[k], chunk, &prop, 0) != hipSuccess) return 3;
        if (hipMemMap(static_cast<char*>(s->va) + perm[k] * chunk, chunk, 0, s->h[k], 0) != hipSuccess) return 4;
    }
    hipMemAccessDesc acc = {};
    acc.location = prop.location;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    if (hipMemSetAccess(s->va, s->size, &acc, 1) != hipSuccess) return 5;
    *out = s->va;
    *handle = s;
    return 0;
}

extern "C" int scatter_free(void* handle) {
    auto* s = static_cast<Scatter*>(handle);
    hipMemUnmap(s->va, s->size);
    for (auto& h : s->h) hipMemRelease(h);
    hipMemAddressFree(s->va, s->size);
    delete s;
    return 0;
}
