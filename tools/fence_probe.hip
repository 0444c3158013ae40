// Cross-stream hand-off probe (gfx950): is data written by a kernel on stream A always visible to a kernel on
// stream B that waits for an event recorded on A, for the event flavours the executor uses?
//
//   A: writer kernel (every workgroup, all XCDs) stores f(iter, i) over X (float4, plain or non-temporal)
//   A: event record  (flavour: kSyncEv = DisableTiming|DisableSystemFence, default = DisableTiming only,
//                     or the stop event of the writer's own hipExtLaunchKernel)
//   A: a busy kernel (keeps A's queue occupied, so no later packet on A flushes anything)
//   B: waits the event, checker kernel reads X (plain or non-temporal loads) and counts words != f(iter, i),
//      recording the first mismatches (index, observed, expected)
// Before the writer, a polluter kernel on B reads X with plain loads, so B's XCD L2s hold clean copies of the
// previous iteration's values (a missing invalidate shows up as those values).
// Usage: fence_probe <iters> [mib]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                        \
        }                                                                                   \
    } while (0)

typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ float val(unsigned it, size_t i) { return (float)((it * 2654435761u + (unsigned)i) & 0xFFFFFF); }

template <bool NT>
__global__ __launch_bounds__(256) void writer(float4* x, size_t n4, unsigned it) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        const f32x4 v = {val(it, 4 * i), val(it, 4 * i + 1), val(it, 4 * i + 2), val(it, 4 * i + 3)};
        if (NT) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(x + i));
        else *reinterpret_cast<f32x4*>(x + i) = v;
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void checker(const float4* x, size_t n4, unsigned it, unsigned* bad, unsigned* log) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        f32x4 v;
        if (NT) v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(x + i));
        else v = *reinterpret_cast<const f32x4*>(x + i);
        for (int c = 0; c < 4; ++c) {
            const float want = val(it, 4 * i + c);
            if (v[c] != want) {
                const unsigned k = atomicAdd(bad, 1u);
                if (k < 64) {
                    log[3 * k] = (unsigned)(4 * i + c);
                    log[3 * k + 1] = __float_as_uint(v[c]);
                    log[3 * k + 2] = __float_as_uint(want);
                }
            }
        }
    }
}

__global__ __launch_bounds__(256) void polluter(const float4* x, size_t n4, float* sink) {
    float s = 0.f;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        const float4 v = x[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == -1.2345f) sink[0] = s;  // never: keeps the loads
}

__global__ void busy(long long cycles) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
}

struct Variant {
    const char* name;
    unsigned ev_flags;
    bool bound;  // the event is the writer's hipExtLaunchKernel stop event
    bool nt_store, nt_load;
};

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 500;
    const size_t mib = argc > 2 ? (size_t)atoi(argv[2]) : 2;
    const size_t n4 = mib * (1 << 20) / 16;
    float4* x;
    unsigned *bad, *log;
    float* sink;
    CK(hipMalloc(&x, n4 * 16));
    CK(hipMalloc(&bad, 4));
    CK(hipMalloc(&log, 64 * 3 * 4));
    CK(hipMalloc(&sink, 4));
    hipStream_t A, B;
    CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
    const unsigned kSync = hipEventDisableTiming | hipEventDisableSystemFence;
    const Variant vs[] = {
        {"kSyncEv record, plain", kSync, false, false, false},
        {"kSyncEv record, nt", kSync, false, true, true},
        {"kSyncEv bound stop event, plain", kSync, true, false, false},
        {"kSyncEv bound stop event, nt", kSync, true, true, true},
        {"default record, plain", hipEventDisableTiming, false, false, false},
        {"default record, nt", hipEventDisableTiming, false, true, true},
    };
    const int grid = 1024;
    unsigned it = 1;
    for (const Variant& v : vs) {
        hipEvent_t ev;
        CK(hipEventCreateWithFlags(&ev, v.ev_flags));
        CK(hipMemset(bad, 0, 4));
        CK(hipDeviceSynchronize());
        for (int k = 0; k < iters; ++k, ++it) {
            hipLaunchKernelGGL(polluter, dim3(grid), dim3(256), 0, B, x, n4, sink);
            // the writer waits for the polluter (B) so B's L2 copies are older than the write
            hipEvent_t e0;
            CK(hipEventCreateWithFlags(&e0, hipEventDisableTiming));
            CK(hipEventRecord(e0, B));
            CK(hipStreamWaitEvent(A, e0, 0));
            if (v.bound) {
                if (v.nt_store) hipExtLaunchKernelGGL(writer<true>, dim3(grid), dim3(256), 0, A, nullptr, ev, 0, x, n4, it);
                else hipExtLaunchKernelGGL(writer<false>, dim3(grid), dim3(256), 0, A, nullptr, ev, 0, x, n4, it);
            } else {
                if (v.nt_store) hipLaunchKernelGGL(writer<true>, dim3(grid), dim3(256), 0, A, x, n4, it);
                else hipLaunchKernelGGL(writer<false>, dim3(grid), dim3(256), 0, A, x, n4, it);
                CK(hipEventRecord(ev, A));
            }
            hipLaunchKernelGGL(busy, dim3(1), dim3(64), 0, A, 20000LL);
            CK(hipStreamWaitEvent(B, ev, 0));
            if (v.nt_load) hipLaunchKernelGGL(checker<true>, dim3(grid), dim3(256), 0, B, x, n4, it, bad, log);
            else hipLaunchKernelGGL(checker<false>, dim3(grid), dim3(256), 0, B, x, n4, it, bad, log);
            CK(hipStreamSynchronize(B));
            CK(hipStreamSynchronize(A));
            CK(hipEventDestroy(e0));
        }
        unsigned nb = 0, lg[64 * 3];
        CK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(lg, log, sizeof(lg), hipMemcpyDeviceToHost));
        printf("%-36s iters %d  %.0f MiB  stale words %u\n", v.name, iters, (double)mib, nb);
        for (unsigned k = 0; k < nb && k < 8; ++k) {
            float o, w;
            memcpy(&o, &lg[3 * k + 1], 4);
            memcpy(&w, &lg[3 * k + 2], 4);
            printf("    word %u (mod 256: %u): got %.0f want %.0f\n", lg[3 * k], lg[3 * k] % 256, o, w);
        }
        fflush(stdout);
        CK(hipMemset(log, 0, sizeof(lg)));
        CK(hipEventDestroy(ev));
    }
    return 0;
}
