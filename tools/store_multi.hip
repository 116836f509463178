// store_multi.hip -- write-only store patterns of the history kernels into caller-allocated buffers
// (experiment tool, never shipped; built as a shared library for tools/store_multi.py, which allocates many
// buffers with torch to compare placements).  One launch writes `planes` planes of `plane_bytes` each
// (plane stride = plane_bytes); every wave owns one `chunk_kib` KiB block per plane and writes plane 0, 1,
// ... in turn with 16-B-per-lane non-temporal stores (1 KiB per store instruction, the trace kernel's tile
// flush policy nt|sc1), sleeping `sleep` s_sleep units between planes (pacing like the arithmetic).
//
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/_build/libstore_multi.so tools/store_multi.hip
#include <hip/hip_runtime.h>

#include <cstdint>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int kChunks>
__global__ __launch_bounds__(64) void multi_kernel(char* out, int64_t plane_bytes, int planes, int64_t waves,
                                                   int sleep) {
    const int lane = threadIdx.x;
    const int64_t w = blockIdx.x;
    if (w >= waves) return;
    v4u acc = {static_cast<unsigned>(lane), 1u, 2u, 3u};
    for (int p = 0; p < planes; ++p) {
        char* base = out + p * plane_bytes + w * (kChunks * 1024);
        const __amdgpu_buffer_rsrc_t rsrc =
            __builtin_amdgcn_make_buffer_rsrc(base, static_cast<short>(0), kChunks * 1024, 0x00020000);
#pragma unroll
        for (int c = 0; c < kChunks; ++c)
            __builtin_amdgcn_raw_buffer_store_b128(acc + static_cast<unsigned>(c + p), rsrc, (c * 64 + lane) * 16, 0,
                                                   2 | 16);
        for (int k = 0; k < sleep; ++k) __builtin_amdgcn_s_sleep(8);
    }
}

extern "C" int store_multi(char* out, int64_t plane_bytes, int planes, int chunk_kib, int sleep, hipStream_t st) {
    const int64_t waves = plane_bytes / (chunk_kib * 1024);
    const dim3 grid(static_cast<unsigned>(waves)), block(64);
    switch (chunk_kib) {
    case 2: hipLaunchKernelGGL(multi_kernel<2>, grid, block, 0, st, out, plane_bytes, planes, waves, sleep); break;
    case 8: hipLaunchKernelGGL(multi_kernel<8>, grid, block, 0, st, out, plane_bytes, planes, waves, sleep); break;
    case 32: hipLaunchKernelGGL(multi_kernel<32>, grid, block, 0, st, out, plane_bytes, planes, waves, sleep); break;
    default: return 2;
    }
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
