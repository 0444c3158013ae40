// Standalone HBM-rate experiment for the fused AdamW update (30 B/param) on gfx950: variants of the
// memory access pattern, timed with HIP events.  Build + run on the GPU box:
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/adamw_bench tools/adamw_bench.hip && /tmp/adamw_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ short f2bf(float x) {
    unsigned u = __float_as_uint(x);
    u += 0x7fff + ((u >> 16) & 1);
    return (short)(u >> 16);
}

struct Hyper {
    float decay, one_m_b1, b2, one_m_b2, eps, step_size, bc2_sqrt;
};

__device__ __forceinline__ void upd(f32x4& p, f32x4 g, f32x4& m, f32x4& v, s16x4& o, const Hyper& h) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        float x = p[j] * h.decay;
        float mj = m[j] + h.one_m_b1 * (g[j] - m[j]);
        float vj = v[j] * h.b2 + h.one_m_b2 * (g[j] * g[j]);
        x = x + (-h.step_size) * (mj / (sqrtf(vj) / h.bc2_sqrt + h.eps));
        p[j] = x;
        m[j] = mj;
        v[j] = vj;
        o[j] = f2bf(x);
    }
}

// G groups of float4 per thread per iteration; NT: nontemporal loads/stores
template <int G, int NTL, int NTS>
__global__ __launch_bounds__(256) void adamw_v(f32x4* p, const f32x4* g, f32x4* m, f32x4* v, s16x4* pb, size_t n4,
                                               Hyper h) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i0 = (size_t)blockIdx.x * 256 + threadIdx.x; i0 < n4; i0 += G * stride) {
        f32x4 P[G], Gr[G], M[G], V[G];
#pragma unroll
        for (int k = 0; k < G; ++k) {
            size_t i = i0 + k * stride;
            if (i < n4) {
                if (NTL) {
                    P[k] = __builtin_nontemporal_load(p + i);
                    Gr[k] = __builtin_nontemporal_load(g + i);
                    M[k] = __builtin_nontemporal_load(m + i);
                    V[k] = __builtin_nontemporal_load(v + i);
                } else {
                    P[k] = p[i];
                    Gr[k] = __builtin_nontemporal_load(g + i);
                    M[k] = m[i];
                    V[k] = v[i];
                }
            }
        }
#pragma unroll
        for (int k = 0; k < G; ++k) {
            size_t i = i0 + k * stride;
            if (i < n4) {
                s16x4 o;
                upd(P[k], Gr[k], M[k], V[k], o, h);
                if (NTS) {
                    __builtin_nontemporal_store(P[k], p + i);
                    __builtin_nontemporal_store(M[k], m + i);
                    __builtin_nontemporal_store(V[k], v + i);
                    __builtin_nontemporal_store(o, pb + i);
                } else {
                    p[i] = P[k];
                    m[i] = M[k];
                    v[i] = V[k];
                    pb[i] = o;
                }
            }
        }
    }
}

// pure streaming references: read 16 B / write 14 B per param without math
__global__ __launch_bounds__(256) void copy_ref(const f32x4* a, f32x4* b, size_t n4) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) b[i] = a[i];
}

template <typename K>
static float time_it(K k, int grid, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k(grid);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < reps; ++r) k(grid);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    const size_t n = 152848128, n4 = n / 4;
    f32x4 *p, *g, *m, *v;
    s16x4* pb;
    hipMalloc(&p, n * 4);
    hipMalloc(&g, n * 4);
    hipMalloc(&m, n * 4);
    hipMalloc(&v, n * 4);
    hipMalloc(&pb, n * 2);
    hipMemset(p, 0, n * 4);
    hipMemset(g, 0, n * 4);
    hipMemset(m, 0, n * 4);
    hipMemset(v, 0, n * 4);
    Hyper h{0.999999f, 0.1f, 0.999f, 0.001f, 1e-8f, 1e-4f, 0.03f};
    const double bytes = 30.0 * n;
    int grids[] = {1024, 2048, 4096, 8192, 16384, 0};
    auto run = [&](const char* name, auto launch) {
        for (int gi = 0; grids[gi]; ++gi) {
            float ms = time_it(launch, grids[gi], 10);
            printf("%-28s grid %6d  %7.1f us  %6.0f GB/s\n", name, grids[gi], ms * 1e3, bytes / (ms * 1e-3) / 1e9);
        }
    };
#define V(G, L, S)                                                                                             \
    run("G=" #G " ntload=" #L " ntstore=" #S, [&](int grid) {                                                  \
        hipLaunchKernelGGL((adamw_v<G, L, S>), dim3(grid), dim3(256), 0, 0, p, g, m, v, pb, n4, h);            \
    });
    V(1, 0, 0) V(2, 0, 0) V(4, 0, 0) V(2, 1, 0) V(2, 0, 1) V(2, 1, 1) V(4, 1, 1)
    {
        float ms = time_it([&](int grid) { hipLaunchKernelGGL(copy_ref, dim3(grid), dim3(256), 0, 0, p, m, n4); },
                           8192, 10);
        printf("copy 4B->4B (8 B/param)      %7.1f us  %6.0f GB/s\n", ms * 1e3, 8.0 * n / (ms * 1e-3) / 1e9);
    }
    return 0;
}
