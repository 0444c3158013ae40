// Cost of a cross-stream fork point on the producing stream: a chain of short kernels on stream A, each followed by
// (0) nothing, (1) hipEventRecord(ev, A) + hipStreamWaitEvent(B, ev) + a consumer kernel on B, or (2) the same event
// bound to the kernel itself through hipExtLaunchKernelGGL's stop event.  Prints the chain's time per link and
// checks that every consumer kernel saw its producer's value (ordering).
//   hipcc --offload-arch=gfx950 -O2 tools/event_gap.hip -o tools/bin/event_gap && tools/bin/event_gap
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

// producer: every workgroup spins ~`ns` then block 0 writes `val` to slot[i]
__global__ void producer(unsigned* slot, int i, unsigned val, long long cycles, float4* dirty, int nd) {
    // nd float4 per thread of dirty data (L2 write-back pressure at the fork); nd >= 1000: nd-1000 float4 written
    // with non-temporal stores; nd >= 2000: nd-2000 written through (sc1 buffer stores)
    const int mode = nd >= 2000 ? 2 : nd >= 1000 ? 1 : 0;
    const int n = nd - 1000 * mode;
    typedef __attribute__((ext_vector_type(4))) float f4;
    typedef unsigned u4v __attribute__((__vector_size__(16)));
    auto rs = __builtin_amdgcn_make_buffer_rsrc(dirty, 0, 0x7fffffff, 0x00020000);
    for (int k = 0; k < n; ++k) {
        const size_t e = ((size_t)blockIdx.x * n + k) * blockDim.x + threadIdx.x;
        const f4 v{(float)val, (float)k, 0.f, 0.f};
        if (mode == 1) __builtin_nontemporal_store(v, reinterpret_cast<f4*>(dirty + e));
        else if (mode == 2) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), rs, (int)(e * 16), 0, 16);
        else dirty[e] = make_float4(val, k, 0, 0);
    }
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) slot[i] = val;
}
// consumer: copies slot[i] to seen[i]
__global__ void consumer(const unsigned* slot, unsigned* seen, int i) {
    if (threadIdx.x == 0) seen[i] = slot[i];
}

int main() {
    const int N = 200, WG = 256;
    const long long cyc = 8000;  // ~4 us at ~2 GHz
    unsigned *slot, *seen;
    float4* dirty;
    CK(hipMalloc(&dirty, (size_t)WG * 256 * 64 * 16));
    CK(hipMalloc(&slot, N * 4));
    CK(hipMalloc(&seen, N * 4));
    hipStream_t A, B;
    CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
    std::vector<hipEvent_t> ev(N);
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence));
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    for (int nd : {0, 64, 1064, 2064})
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 3; ++mode) {
            CK(hipMemset(slot, 0, N * 4));
            CK(hipMemset(seen, 0, N * 4));
            CK(hipDeviceSynchronize());
            // keep the device busy while the host enqueues, so the host is never on the critical path
            hipLaunchKernelGGL(producer, dim3(1), dim3(64), 0, A, slot, 0, 0u, (long long)4000000, dirty, 0);
            CK(hipEventRecord(t0, A));
            for (int i = 0; i < N; ++i) {
                const unsigned val = 1000u * (mode + 1) + i;
                if (mode == 2) {
                    hipExtLaunchKernelGGL(producer, dim3(WG), dim3(256), 0, A, nullptr, ev[i], 0, slot, i, val, cyc, dirty, nd);
                } else {
                    hipLaunchKernelGGL(producer, dim3(WG), dim3(256), 0, A, slot, i, val, cyc, dirty, nd);
                    if (mode == 1) CK(hipEventRecord(ev[i], A));
                }
                if (mode >= 1) {
                    CK(hipStreamWaitEvent(B, ev[i], 0));
                    hipLaunchKernelGGL(consumer, dim3(1), dim3(64), 0, B, slot, seen, i);
                }
            }
            CK(hipEventRecord(t1, A));
            CK(hipDeviceSynchronize());
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, t0, t1));
            std::vector<unsigned> h(N);
            CK(hipMemcpy(h.data(), seen, N * 4, hipMemcpyDeviceToHost));
            int bad = 0;
            if (mode >= 1)
                for (int i = 0; i < N; ++i) bad += h[i] != 1000u * (mode + 1) + i;
            printf("dirty %d KB/WG mode %d (%s): %.2f us per link, consumer ordering errors %d\n", nd * 4, mode,
                   mode == 0 ? "no fork" : mode == 1 ? "hipEventRecord" : "ext launch stop event", 1000.f * ms / N, bad);
        }
    return 0;
}
