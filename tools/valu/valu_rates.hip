// valu_rates.hip -- issue cost of the VALU instructions the trace kernels are made of, measured on gfx950:
// cycles per wave64 instruction per SIMD when 4 waves per SIMD issue independent copies (8 chains per wave, so
// latency is hidden).  Each kernel times its loop with s_memtime (shader clock), so the number does not depend
// on the clock the package power allows.   usage: valu_rates [iterations]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); std::exit(1); } } while (0)

// 8 independent instructions of one kind per iteration; operands in v[0:31] as 8 register pairs (x) + 8 (y)
#define REP8(S) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)

template <int OP>
__global__ __launch_bounds__(256) void bench(int iters, double seed, unsigned long long* cyc, double* sink) {
    double a[8], b[8];
    int ia[8], ib[8];
    unsigned long long sm[8];
    float fa[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { a[k] = seed + threadIdx.x * 1e-3 + k; b[k] = 1.0 + k * 1e-6; ia[k] = threadIdx.x + k; ib[k] = 3 * k + 1; sm[k] = 0x5555ull << k; fa[k] = 0.f; }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#define FMA(k) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(a[k]) : "v"(b[k]));
#define ADD(k) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a[k]) : "v"(b[k]));
#define MUL(k) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a[k]) : "v"(b[k]));
#define RCP(k) asm volatile("v_rcp_f64 %0, %0" : "+v"(a[k]));
#define RSQ(k) asm volatile("v_rsq_f64 %0, %0" : "+v"(a[k]));
#define FIX(k) asm volatile("v_div_fixup_f64 %0, %0, %1, %1" : "+v"(a[k]) : "v"(b[k]));
#define FREXP(k) asm volatile("v_frexp_exp_i32_f64 %0, %1" : "=v"(ia[k]) : "v"(a[k]));
#define CLASS(k) asm volatile("v_cmp_class_f64_e64 %0, %1, %2" : "=s"(sm[k]) : "v"(a[k]), "v"(ia[k]));
#define CMPF(k) asm volatile("v_cmp_lt_f64_e64 %0, %1, %2" : "=s"(sm[k]) : "v"(a[k]), "v"(b[k]));
#define CMPU(k) asm volatile("v_cmp_lt_u32_e64 %0, %1, %2" : "=s"(sm[k]) : "v"(ia[k]), "v"(ib[k]));
#define ADDU(k) asm volatile("v_add_u32 %0, %0, %1" : "+v"(ia[k]) : "v"(ib[k]));
#define CND(k) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(ia[k]) : "v"(ib[k]), "s"(sm[k]));
#define MOV64(k) asm volatile("v_mov_b64 %0, %1" : "=v"(a[k]) : "v"(b[k]));
#define MOV32(k) asm volatile("v_mov_b32 %0, %1" : "=v"(ia[k]) : "v"(ib[k]));
#define MIN3(k) asm volatile("v_min3_i32 %0, %0, %1, %1" : "+v"(ia[k]) : "v"(ib[k]));
#define MINF(k) asm volatile("v_min_f64 %0, %0, %1" : "+v"(a[k]) : "v"(b[k]));
#define LDEXP(k) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(a[k]) : "v"(ia[k]));
#define CVT(k) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(fa[k]) : "v"(a[k]));
#define FMAC(k) asm volatile("v_fmac_f64 %0, %1, %1" : "+v"(a[k]) : "v"(b[k]));
        if constexpr (OP == 0) { REP8(FMA) }
        else if constexpr (OP == 1) { REP8(ADD) }
        else if constexpr (OP == 2) { REP8(MUL) }
        else if constexpr (OP == 3) { REP8(RCP) }
        else if constexpr (OP == 4) { REP8(RSQ) }
        else if constexpr (OP == 5) { REP8(FIX) }
        else if constexpr (OP == 6) { REP8(FREXP) }
        else if constexpr (OP == 7) { REP8(CLASS) }
        else if constexpr (OP == 8) { REP8(CMPF) }
        else if constexpr (OP == 9) { REP8(CMPU) }
        else if constexpr (OP == 10) { REP8(ADDU) }
        else if constexpr (OP == 11) { REP8(CND) }
        else if constexpr (OP == 12) { REP8(MOV64) }
        else if constexpr (OP == 13) { REP8(MOV32) }
        else if constexpr (OP == 14) { REP8(MIN3) }
        else if constexpr (OP == 15) { REP8(MINF) }
        else if constexpr (OP == 16) { REP8(LDEXP) }
        else if constexpr (OP == 17) { REP8(FMAC) }
        else if constexpr (OP == 18) { REP8(FMA) REP8(ADDU) }        // a 2:1 mix... (f64 then int)
        else if constexpr (OP == 19) { REP8(FMA) REP8(RCP) }         // transcendental beside f64 FMAs
        else if constexpr (OP == 20) { REP8(CVT) }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0; int si = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) { s += a[k] + fa[k]; si += ia[k] + int(sm[k] & 1); }
    sink[blockIdx.x * 256 + threadIdx.x] = s + si;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

static const char* kNames[] = {"v_fma_f64", "v_add_f64", "v_mul_f64", "v_rcp_f64", "v_rsq_f64", "v_div_fixup_f64",
                               "v_frexp_exp_i32_f64", "v_cmp_class_f64", "v_cmp_lt_f64", "v_cmp_lt_u32", "v_add_u32",
                               "v_cndmask_b32", "v_mov_b64", "v_mov_b32", "v_min3_i32", "v_min_f64", "v_ldexp_f64",
                               "v_fmac_f64", "8 v_fma_f64 + 8 v_add_u32", "8 v_fma_f64 + 8 v_rcp_f64", "v_cvt_f32_f64"};

template <int OP>
void run(int iters, int cus, int waves_per_simd) {
    const int blocks = cus * waves_per_simd;           // 4 waves per block = one per SIMD
    unsigned long long* cyc; double* sink;
    CHECK(hipMalloc(&cyc, sizeof(unsigned long long) * blocks * 4));
    CHECK(hipMalloc(&sink, sizeof(double) * blocks * 256));
    hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, 10, 1.0, cyc, sink);   // warm
    hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, iters, 1.0, cyc, sink);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0; CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> h(blocks * 4);
    CHECK(hipMemcpy(h.data(), cyc, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
    std::sort(h.begin(), h.end());
    const double med = double(h[h.size() / 2]);
    const int per_iter = (OP >= 18) ? 16 : 8;
    const double instr = double(iters) * per_iter;
    // waves_per_simd waves share a SIMD for (about) the whole loop
    std::printf("%-28s %7.2f cyc per wave-instruction per SIMD  (wave loop %.3g cyc, kernel %.3f ms, %.2f GHz implied)\n",
                kNames[OP], med / (instr * waves_per_simd),
                med, ms, med / (ms * 1e6));
    CHECK(hipFree(cyc)); CHECK(hipFree(sink));
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 20000;
    hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    std::printf("%s, %d CUs; W waves per SIMD (one 4-wave block per CU per W), 8 independent chains per wave; cycles "
                "= median s_memtime over a wave's loop / (its instructions x W)\n", p.gcnArchName, cus);
    for (int W : {1, 2, 4}) {
        std::printf("-- W = %d\n", W);
        run<0>(iters, cus, W); run<17>(iters, cus, W); run<1>(iters, cus, W); run<2>(iters, cus, W); run<3>(iters, cus, W);
        run<4>(iters, cus, W); run<5>(iters, cus, W); run<6>(iters, cus, W); run<7>(iters, cus, W); run<8>(iters, cus, W);
        run<9>(iters, cus, W); run<10>(iters, cus, W); run<11>(iters, cus, W); run<12>(iters, cus, W); run<13>(iters, cus, W);
        run<14>(iters, cus, W); run<15>(iters, cus, W); run<16>(iters, cus, W); run<18>(iters, cus, W); run<19>(iters, cus, W);
        run<20>(iters, cus, W);
    }
    return 0;
}
