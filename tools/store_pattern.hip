// store_pattern.hip -- write-pattern microbenchmark for the trace kernel's output stream (experiment tool).
//
// The trace kernel writes P = 2S+1 history planes (N x 64 B each, plane stride N*64 B); each wave stores a
// 4 KiB contiguous chunk (64 records) into every plane, one plane after the other over its lifetime.  This
// tool times synthetic write-only kernels of the same total bytes with different shapes, to find which
// pattern the HBM write path prefers:
//   planes P (1 = one contiguous stream, like a fill), chunk bytes per wave per plane (4/8/16 KiB),
//   plane-stride padding, nt vs plain stores, waves per workgroup.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/store_pattern tools/store_pattern.hip && tools/store_pattern
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                            \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

typedef double v2d __attribute__((ext_vector_type(2)));

// Each wave owns `kChunks` consecutive 1 KiB store-instruction slots per plane (chunk = kChunks KiB) and
// writes plane 0, then plane 1, ... (plane-major inside the wave, like the trace kernel).  `spin` adds a
// dependent f64 chain between planes to emulate the per-surface compute.
template <int kChunks, bool NT>
__global__ __launch_bounds__(256) void planes_kernel(double* out, int64_t plane_stride_d, int planes, int64_t units,
                                                     int spin) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    if (wave * kChunks >= units) return;
    double acc = static_cast<double>(lane);
    for (int p = 0; p < planes; ++p) {
        for (int s = 0; s < spin; ++s) acc = acc * 1.0000001 + 0.5;
        v2d* base = reinterpret_cast<v2d*>(out + p * plane_stride_d) + wave * kChunks * 64;
#pragma unroll
        for (int c = 0; c < kChunks; ++c) {
            const v2d v = {acc, static_cast<double>(c)};
            if (NT) __builtin_nontemporal_store(v, base + c * 64 + lane);
            else base[c * 64 + lane] = v;
        }
    }
}

// Persistent grid-stride form: `gridDim.x` one-wave workgroups; wave w handles units w, w + W, w + 2W, ...
// (all planes of a unit before the next unit), so the concurrently running waves write the SAME plane at
// neighbouring addresses, as a fill does.
// 8-byte lanes (512 B per store instruction): `chunk` bytes per wave per stream in 512 B pieces.  With
// streams = 88 and chunk = 512 this is the trace kernel's SoA output shape (8 fields x 11 planes).
template <int kPieces>
__global__ __launch_bounds__(256) void narrow_kernel(double* out, int64_t stream_stride_d, int streams, int64_t units) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
    if (wave * kPieces >= units) return;
    const double v = static_cast<double>(lane);
    for (int p = 0; p < streams; ++p) {
        double* base = out + p * stream_stride_d + wave * kPieces * 64;
#pragma unroll
        for (int c = 0; c < kPieces; ++c) __builtin_nontemporal_store(v + c, base + c * 64 + lane);
    }
}

template <int kPieces>
float run_narrow(double* buf, int64_t stream_bytes, int streams, int block, int reps) {
    const int64_t units = stream_bytes / 512;
    const int64_t waves = (units + kPieces - 1) / kPieces;
    const dim3 grid(static_cast<unsigned>((waves * 64 + block - 1) / block));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    narrow_kernel<kPieces><<<grid, block>>>(buf, stream_bytes / 8, streams, units);
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) narrow_kernel<kPieces><<<grid, block>>>(buf, stream_bytes / 8, streams, units);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return ms / reps;
}

template <bool NT>
__global__ __launch_bounds__(64) void persistent_kernel(double* out, int64_t plane_stride_d, int planes, int64_t units,
                                                        int spin) {
    const int lane = threadIdx.x & 63;
    double acc = static_cast<double>(lane);
    for (int64_t u = blockIdx.x; u < units; u += gridDim.x) {
        for (int p = 0; p < planes; ++p) {
            for (int s = 0; s < spin; ++s) acc = acc * 1.0000001 + 0.5;
            v2d* base = reinterpret_cast<v2d*>(out + p * plane_stride_d) + u * 4 * 64;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const v2d v = {acc, static_cast<double>(c)};
                if (NT) __builtin_nontemporal_store(v, base + c * 64 + lane);
                else base[c * 64 + lane] = v;
            }
        }
    }
}

float run_persistent(double* buf, int64_t plane_bytes, int64_t stride_bytes, int planes, int nwaves, int spin,
                     int reps) {
    const int64_t units = plane_bytes / 4096;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    persistent_kernel<true><<<nwaves, 64>>>(buf, stride_bytes / 8, planes, units, spin);
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) persistent_kernel<true><<<nwaves, 64>>>(buf, stride_bytes / 8, planes, units, spin);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return ms / reps;
}

template <int kChunks, bool NT>
float run(double* buf, int64_t plane_bytes, int64_t stride_bytes, int planes, int block, int spin, int reps) {
    const int64_t units = plane_bytes / 1024;                 // 1 KiB store slots per plane
    const int64_t waves = (units + kChunks - 1) / kChunks;
    const int64_t threads = waves * 64;
    const dim3 grid(static_cast<unsigned>((threads + block - 1) / block));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    planes_kernel<kChunks, NT><<<grid, block>>>(buf, stride_bytes / 8, planes, units, spin);
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) planes_kernel<kChunks, NT><<<grid, block>>>(buf, stride_bytes / 8, planes, units, spin);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return ms / reps;
}

int main(int argc, char** argv) {
    const int64_t total = argc > 1 ? std::atoll(argv[1]) : 704000000LL;   // C2 history bytes
    const int reps = 50;
    double* buf;
    CHECK(hipMalloc(&buf, total + (64 << 20)));
    struct Case { const char* name; int planes; int chunks; bool nt; int64_t pad; int block; int spin; };
    std::vector<Case> cases = {
        {"fill-like  P=1  4K  nt", 1, 4, true, 0, 64, 0},
        {"fill-like  P=1 16K  nt", 1, 16, true, 0, 64, 0},
        {"trace-like P=11 4K  nt", 11, 4, true, 0, 64, 0},
        {"trace-like P=11 4K  plain", 11, 4, false, 0, 64, 0},
        {"P=11 8K  nt", 11, 8, true, 0, 64, 0},
        {"P=11 16K nt", 11, 16, true, 0, 64, 0},
        {"P=11 4K  nt wg256", 11, 4, true, 0, 256, 0},
        {"P=11 4K  nt pad+4K", 11, 4, true, 4096, 64, 0},
        {"P=11 4K  nt pad+1M+4K", 11, 4, true, (1 << 20) + 4096, 64, 0},
        {"P=2  4K  nt", 2, 4, true, 0, 64, 0},
        {"P=4  4K  nt", 4, 4, true, 0, 64, 0},
        {"P=11 4K  nt spin20", 11, 4, true, 0, 64, 20},
        {"P=11 16K nt spin20", 11, 16, true, 0, 64, 20},
        // persistent grid-stride (chunks = 4 KiB; `block` field = number of waves in the grid)
        {"persist P=1  W=5120", 1, -1, true, 0, 5120, 0},
        {"persist P=11 W=2048", 11, -1, true, 0, 2048, 0},
        {"persist P=11 W=5120", 11, -1, true, 0, 5120, 0},
        {"persist P=11 W=8192", 11, -1, true, 0, 8192, 0},
        {"persist P=11 W=5120 spin20", 11, -1, true, 0, 5120, 20},
        // 8-byte lanes: chunks = -8 means 8 pieces of 512 B (4 KiB) per stream, -1... handled below
        {"narrow P=11 4K wg64", 11, -8, true, 0, 64, 0},
        {"narrow P=11 4K wg256", 11, -8, true, 0, 256, 0},
        {"narrow P=88 512B wg64 (SoA)", 88, -9, true, 0, 64, 0},
        {"narrow P=88 512B wg256 (SoA)", 88, -9, true, 0, 256, 0},
        {"narrow P=1 4K wg64", 1, -8, true, 0, 64, 0},
    };
    for (int round = 0; round < 3; ++round) {
        for (const Case& c : cases) {
            const int64_t plane_bytes = (total / c.planes) / 16384 * 16384;
            const int64_t stride = plane_bytes + c.pad;
            float ms = 0;
#define DISPATCH(K)                                                                                   \
    ms = c.nt ? run<K, true>(buf, plane_bytes, stride, c.planes, c.block, c.spin, reps)               \
              : run<K, false>(buf, plane_bytes, stride, c.planes, c.block, c.spin, reps)
            if (c.chunks == -8) ms = run_narrow<8>(buf, plane_bytes, c.planes, c.block, reps);
            else if (c.chunks == -9) ms = run_narrow<1>(buf, plane_bytes, c.planes, c.block, reps);
            else if (c.chunks < 0) ms = run_persistent(buf, plane_bytes, stride, c.planes, c.block, c.spin, reps);
            else if (c.chunks == 4) DISPATCH(4);
            else if (c.chunks == 8) DISPATCH(8);
            else DISPATCH(16);
            const double bytes = static_cast<double>(plane_bytes) * c.planes;
            std::printf("round %d  %-26s  %8.4f ms  %7.0f GB/s\n", round, c.name, ms, bytes / ms / 1e6);
        }
    }
    CHECK(hipFree(buf));
    return 0;
}
