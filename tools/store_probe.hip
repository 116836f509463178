// store_probe.hip -- write-only probe of the history kernels' store pattern at full config size (experiment
// tool, never shipped).  One launch writes `planes` planes of `plane_bytes` each (plane stride =
// plane_bytes), every wave owning one `chunk_kib` KiB block per plane and writing plane 0, 1, ... in turn
// with 16-B-per-lane non-temporal stores (1 KiB per store instruction), as the trace kernel's tile flush
// does.  planes = 1 is a plain fill of the same bytes.  Optionally each wave first reads `in_bytes_per_chunk`
// of an input stream (the trace kernel's ray records).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/store_probe tools/store_probe.hip
//   tools/store_probe TOTAL_BYTES PLANES CHUNK_KIB [REPS] [IN_BYTES_PER_WAVE]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                            \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int kChunks>
__global__ __launch_bounds__(64) void probe_kernel(char* out, const char* in, int64_t plane_bytes, int planes,
                                                   int64_t waves, int in_bytes) {
    const int lane = threadIdx.x;
    const int64_t w = blockIdx.x;
    if (w >= waves) return;
    v4u acc = {static_cast<unsigned>(lane), 1u, 2u, 3u};
    if (in_bytes > 0) {
        const v4u* src = reinterpret_cast<const v4u*>(in + w * static_cast<int64_t>(in_bytes));
        for (int k = lane; k < in_bytes / 16; k += 64) acc += src[k];
    }
    for (int p = 0; p < planes; ++p) {
        char* base = out + p * plane_bytes + w * (kChunks * 1024);
        const __amdgpu_buffer_rsrc_t rsrc =
            __builtin_amdgcn_make_buffer_rsrc(base, static_cast<short>(0), kChunks * 1024, 0x00020000);
#pragma unroll
        for (int c = 0; c < kChunks; ++c)
            __builtin_amdgcn_raw_buffer_store_b128(acc + static_cast<unsigned>(c + p), rsrc, (c * 64 + lane) * 16, 0, 2 | 16);
    }
}

template <int K>
float run(char* out, const char* in, int64_t plane_bytes, int planes, int reps, int in_bytes) {
    const int64_t waves = plane_bytes / (K * 1024);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    probe_kernel<K><<<dim3(static_cast<unsigned>(waves)), dim3(64)>>>(out, in, plane_bytes, planes, waves, in_bytes);
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r)
        probe_kernel<K><<<dim3(static_cast<unsigned>(waves)), dim3(64)>>>(out, in, plane_bytes, planes, waves, in_bytes);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s TOTAL_BYTES PLANES CHUNK_KIB [REPS] [IN_BYTES_PER_WAVE]\n", argv[0]);
        return 2;
    }
    const int64_t total = std::atoll(argv[1]);
    const int planes = std::atoi(argv[2]);
    const int chunk = std::atoi(argv[3]);
    const int reps = argc > 4 ? std::atoi(argv[4]) : 10;
    const int in_bytes = argc > 5 ? std::atoi(argv[5]) : 0;
    const int64_t plane_bytes = total / planes / (chunk * 1024) * (chunk * 1024);
    const int64_t waves = plane_bytes / (chunk * 1024);
    char* out = nullptr;
    char* in = nullptr;
    CHECK(hipMalloc(&out, plane_bytes * planes));
    if (in_bytes > 0) CHECK(hipMalloc(&in, waves * static_cast<int64_t>(in_bytes)));
    float ms = 0;
    switch (chunk) {
    case 1: ms = run<1>(out, in, plane_bytes, planes, reps, in_bytes); break;
    case 2: ms = run<2>(out, in, plane_bytes, planes, reps, in_bytes); break;
    case 4: ms = run<4>(out, in, plane_bytes, planes, reps, in_bytes); break;
    case 8: ms = run<8>(out, in, plane_bytes, planes, reps, in_bytes); break;
    case 16: ms = run<16>(out, in, plane_bytes, planes, reps, in_bytes); break;
    default: std::fprintf(stderr, "chunk must be 1, 2, 4, 8 or 16 KiB\n"); return 2;
    }
    const double bytes = static_cast<double>(plane_bytes) * planes + static_cast<double>(waves) * in_bytes;
    std::printf("planes %3d chunk %2d KiB in %4d B/wave  %9.4f ms  %7.0f GB/s  (%.2f GB)\n", planes, chunk, in_bytes,
                ms, bytes / ms / 1e6, bytes / 1e9);
    CHECK(hipFree(out));
    if (in) CHECK(hipFree(in));
    return 0;
}
