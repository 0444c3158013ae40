// Per-CU L2 -> LDS fill rate of GEMM-shaped tile streams on gfx950 (no math): what bounds the
// small-M GEMMs of the training step.  Each workgroup streams the 64-deep K steps of one A tile row
// block (BM x 64) and one B block (BN x 64) from L2-resident bf16 matrices, NS stages in flight.
//   hipcc -O3 --offload-arch=gfx950 -o tools/bin/fill_bench tools/fill_bench.hip && tools/bin/fill_bench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_addr) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_addr)
                 : "memory");
}
__device__ __forceinline__ uint32_t lds_addr_of(const char* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int LPS, int MAXA>
__device__ __forceinline__ void wait_stages(int after) {
    if constexpr (MAXA > 0) {
        if (after >= MAXA) {
            wait_vm<MAXA * LPS>();
            return;
        }
        wait_stages<LPS, MAXA - 1>(after);
    } else {
        wait_vm<0>();
    }
}

// MODE 0: LDS-DMA (global_load_lds_dwordx4); MODE 1: global_load_dwordx4 -> ds_write_b128;
// MODE 2: global_load_dwordx4 only (L2 -> VGPR ceiling)
template <int BM, int BN, int NW, int NS, int MODE>
__global__ __launch_bounds__(64 * NW) void fill_kernel(const uint16_t* A, const uint16_t* B, int K, int passes,
                                                      int tiles_m, int tiles_n, unsigned* sink) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int STAGE = (BM + BN) * 64 * 2;
    constexpr int LPS = STAGE / 1024 / NW;  // DMA instructions per wave per stage
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tm = blockIdx.x % tiles_m, tn = (blockIdx.x / tiles_m) % tiles_n;
    const int nk = K / 64;
    unsigned acc = 0;
    auto issue = [&](int kt) {
        char* st = smem + (kt % NS) * STAGE;
        const int k0 = (kt % nk) * 64;
#pragma unroll
        for (int i = 0; i < LPS; ++i) {
            const int ib = (i * NW + wave) * 1024;
            const int o = ib + lane * 16;
            const int row = o / 128, c = (o % 128) / 16;
            const uint16_t* src = row < BM ? A + (size_t)(tm * BM + row) * K + k0 + c * 8
                                           : B + (size_t)(tn * BN + row - BM) * K + k0 + c * 8;
            if (MODE == 0) {
                glds16(src, __builtin_amdgcn_readfirstlane(lds_addr_of(st + ib)));
            } else {
                uint4 v = *reinterpret_cast<const uint4*>(src);
                if (MODE == 1) *reinterpret_cast<uint4*>(st + o) = v;
                else acc ^= v.x ^ v.y ^ v.z ^ v.w;
            }
        }
    };
    const int total = nk * passes;
    for (int s = 0; s < NS - 1; ++s) issue(s);
    for (int kt = 0; kt < total; ++kt) {
        if (MODE == 0) {
            const int after = min(NS - 2, total - 1 - kt);
            wait_stages<LPS, NS - 2>(after);
            __builtin_amdgcn_s_barrier();
        } else if (MODE == 1) {
            __syncthreads();
        }
        if (kt + NS - 1 < total) issue(kt + NS - 1);
    }
    wait_vm<0>();
    if (MODE == 2 && acc == 0x12345678u) sink[0] = acc;
}

template <int BM, int BN, int NW, int NS, int MODE>
void run(const char* name, const uint16_t* A, const uint16_t* B, int M, int N, int K, int passes, int wgs,
         unsigned* sink) {
    constexpr int STAGE = (BM + BN) * 64 * 2;
    const size_t lds = (size_t)NS * STAGE;
    hipFuncSetAttribute((const void*)fill_kernel<BM, BN, NW, NS, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)lds);
    auto launch = [&]() {
        hipLaunchKernelGGL((fill_kernel<BM, BN, NW, NS, MODE>), dim3(wgs), dim3(64 * NW), lds, 0, A, B, K, passes,
                           M / BM, N / BN, sink);
    };
    launch();
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    const int reps = 5;
    for (int r = 0; r < reps; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double bytes = (double)wgs * STAGE * (K / 64) * passes;
    const double s = ms * 1e-3 / reps;
    const int per_cu = (wgs + 255) / 256;
    printf("%-40s wgs %4d: %8.1f us  chip %6.2f TB/s  per-CU %6.1f GB/s (%d WG/CU)\n", name, wgs, s * 1e6,
           bytes / s / 1e12, bytes / s / 1e9 / std::min(wgs, 256), per_cu);
}

int main() {
    const int M = 2048, N = 3072, K = 768;
    uint16_t *A, *B;
    unsigned* sink;
    hipMalloc(&A, (size_t)M * K * 2);
    hipMalloc(&B, (size_t)N * K * 2);
    hipMalloc(&sink, 64);
    hipMemset(A, 0, (size_t)M * K * 2);
    hipMemset(B, 0, (size_t)N * K * 2);
    const int passes = 40;
    for (int wgs : {256, 512}) {
        run<64, 64, 4, 4, 0>("64x64 4w NS4 LDS-DMA", A, B, M, N, K, passes, wgs, sink);
        run<64, 64, 4, 8, 0>("64x64 4w NS8 LDS-DMA", A, B, M, N, K, passes, wgs, sink);
        run<64, 64, 4, 4, 1>("64x64 4w NS4 reg->ds_write", A, B, M, N, K, passes, wgs, sink);
        run<64, 64, 4, 4, 2>("64x64 4w load only", A, B, M, N, K, passes, wgs, sink);
        run<128, 128, 4, 3, 0>("128x128 4w NS3 LDS-DMA", A, B, M, N, K, passes, wgs, sink);
        run<128, 128, 8, 2, 0>("128x128 8w NS2 LDS-DMA", A, B, M, N, K, passes, wgs, sink);
        run<128, 128, 8, 4, 0>("128x128 8w NS4 LDS-DMA", A, B, M, N, K, passes, wgs, sink);
        run<128, 128, 8, 4, 2>("128x128 8w load only", A, B, M, N, K, passes, wgs, sink);
        run<256, 256, 8, 2, 0>("256x256 8w NS2 LDS-DMA", A, B, M, N, K, passes, wgs, sink);
        run<64, 64, 16, 4, 0>("64x64 16w NS4 LDS-DMA", A, B, M, N, K, passes, wgs, sink);
    }
    return 0;
}
