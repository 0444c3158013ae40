// Which packed-FP32 instruction forms go wrong beside MFMA waves on gfx950 (round 6)?  Each variant runs
// a dependent chain of one instruction form (inline asm, so the compiler cannot change it) on float pairs and is checked
// word for word against the host; alone and with MFMA waves from another kernel on the same CUs.
// Usage: pk_hazard <iters>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                        \
        }                                                                                   \
    } while (0)

typedef __attribute__((ext_vector_type(2))) float f2;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
constexpr int CHAIN = 32;

template <int V>
__global__ __launch_bounds__(256) void chain(f2* x, const f2* b, size_t n) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        f2 r = x[i];
        const f2 c = b[i];
#pragma unroll
        for (int k = 0; k < CHAIN; ++k) {
            if constexpr (V == 0) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(r) : "v"(c));
            if constexpr (V == 1) asm volatile("v_pk_add_f32 %0, %0, %1 op_sel:[0,1] op_sel_hi:[1,0]" : "+v"(r) : "v"(c));
            if constexpr (V == 2) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(r) : "v"(c));
            if constexpr (V == 3) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(r) : "v"(c));
            if constexpr (V == 4) {  // the same arithmetic as variant 0 through two unpacked instructions
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(r.x) : "v"(c.x));
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(r.y) : "v"(c.y));
            }
        }
        x[i] = r;
    }
}

static void host(int V, float& x, float& y, float cx, float cy) {
    for (int k = 0; k < CHAIN; ++k) {
        volatile float a = x, b = y;
        if (V == 0 || V == 4) { a = a + cx; b = b + cy; }
        if (V == 1) { a = a + cy; b = b + cx; }
        if (V == 2) { a = a * cx; b = b * cy; }
        if (V == 3) { a = std::fma((float)a, cx, cx); b = std::fma((float)b, cy, cy); }
        x = a;
        y = b;
    }
}

__global__ __launch_bounds__(256) void mfma_spin(float* out, int iters) {
    bf16x8 a, b;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        a[j] = (__bf16)(0.001f * (threadIdx.x + j));
        b[j] = (__bf16)(0.002f * (j + 1));
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < iters; ++k) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
    if (acc[0] == -1.f) out[threadIdx.x] = acc[1];
}

__global__ void compare(const float* got, const float* want, size_t n, unsigned* bad, unsigned* first) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        if (__float_as_uint(got[i]) != __float_as_uint(want[i])) {
            const unsigned k = atomicAdd(bad, 1u);
            if (k < 8) first[k] = (unsigned)i;
        }
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 100;
    const size_t n = 4u << 20;  // float pairs
    std::vector<float> hx(2 * n), hb(2 * n), want(2 * n);
    unsigned s = 7;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (s >> 8) * (1.0f / 16777216.0f); };
    for (size_t i = 0; i < 2 * n; ++i) {
        hx[i] = rnd() - 0.5f;
        hb[i] = 0.999f + 0.002f * rnd();
    }
    float *x, *x0, *b, *w, *sink;
    unsigned *bad, *first;
    CK(hipMalloc(&x, 8 * n));
    CK(hipMalloc(&x0, 8 * n));
    CK(hipMalloc(&b, 8 * n));
    CK(hipMalloc(&w, 8 * n));
    CK(hipMalloc(&sink, 4096));
    CK(hipMalloc(&bad, 4));
    CK(hipMalloc(&first, 32));
    CK(hipMemcpy(x0, hx.data(), 8 * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(b, hb.data(), 8 * n, hipMemcpyHostToDevice));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const char* names[] = {"v_pk_add_f32", "v_pk_add_f32 op_sel:[0,1] op_sel_hi:[1,0]", "v_pk_mul_f32", "v_pk_fma_f32",
                           "2 x v_add_f32 (unpacked)"};
    for (int V = 0; V < 5; ++V) {
        for (size_t i = 0; i < n; ++i) {
            float a = hx[2 * i], c = hx[2 * i + 1];
            host(V, a, c, hb[2 * i], hb[2 * i + 1]);
            want[2 * i] = a;
            want[2 * i + 1] = c;
        }
        CK(hipMemcpy(w, want.data(), 8 * n, hipMemcpyHostToDevice));
        for (int pressure = 0; pressure < 2; ++pressure) {
            unsigned tot = 0, f[8] = {0};
            bool have = false;
            for (int it = 0; it < iters; ++it) {
                CK(hipMemcpyAsync(x, x0, 8 * n, hipMemcpyDeviceToDevice, s1));
                CK(hipMemsetAsync(bad, 0, 4, s1));
                CK(hipStreamSynchronize(s1));
                if (pressure) hipLaunchKernelGGL(mfma_spin, dim3(1024), dim3(256), 0, s2, sink, 20000);
                switch (V) {
                    case 0: hipLaunchKernelGGL(chain<0>, dim3(2048), dim3(256), 0, s1, (f2*)x, (const f2*)b, n); break;
                    case 1: hipLaunchKernelGGL(chain<1>, dim3(2048), dim3(256), 0, s1, (f2*)x, (const f2*)b, n); break;
                    case 2: hipLaunchKernelGGL(chain<2>, dim3(2048), dim3(256), 0, s1, (f2*)x, (const f2*)b, n); break;
                    case 3: hipLaunchKernelGGL(chain<3>, dim3(2048), dim3(256), 0, s1, (f2*)x, (const f2*)b, n); break;
                    default: hipLaunchKernelGGL(chain<4>, dim3(2048), dim3(256), 0, s1, (f2*)x, (const f2*)b, n); break;
                }
                hipLaunchKernelGGL(compare, dim3(2048), dim3(256), 0, s1, x, w, 2 * n, bad, first);
                CK(hipStreamSynchronize(s1));
                CK(hipStreamSynchronize(s2));
                unsigned nb;
                CK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
                if (nb && !have) {
                    have = true;
                    CK(hipMemcpy(f, first, 32, hipMemcpyDeviceToHost));
                }
                tot += nb;
            }
            printf("%-44s %-18s wrong words %u of %zu\n", names[V], pressure ? "beside MFMA waves" : "alone", tot,
                   (size_t)iters * 2 * n);
            if (have) {
                printf("   first:");
                for (int k = 0; k < 8; ++k) printf(" %u(half %u, lane %u)", f[k], f[k] % 2, (f[k] / 2) % 64);
                printf("\n");
            }
            fflush(stdout);
        }
    }
    return 0;
}
