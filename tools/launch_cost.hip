// Host cost of one kernel launch through each HIP entry point (round 6: the training step issues ~480 launches
// and its host time is ~2.7 ms).  Launches an empty kernel taking a GemmArgs-sized (256 B) by-value struct, in
// batches of 256 with a stream sync between batches (only the enqueue is timed).
//   A: hipLaunchKernelGGL (the library's ERGM_LAUNCH); B: hipExtLaunchKernelGGL with a stop event (bound fork
//   points); C: hipModuleLaunchKernel with the hipFunction_t fetched once (hipGetFuncBySymbol), args by pointer;
//   D: hipModuleLaunchKernel, args as one packed buffer (HIP_LAUNCH_PARAM_BUFFER_POINTER)
// Usage: launch_cost
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                        \
        }                                                                                   \
    } while (0)

struct Args {
    float* out;
    int v[62];
};

__global__ void empty_kernel(Args a) {
    if (a.v[0] == 12345 && threadIdx.x == 0) a.out[blockIdx.x] = 1.f;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    float* out;
    CK(hipMalloc(&out, 4096 * 4));
    Args a{};
    a.out = out;
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    hipFunction_t f;
    CK(hipGetFuncBySymbol(&f, reinterpret_cast<const void*>(&empty_kernel)));
    const int BATCH = 256, ROUNDS = 40;
    const char* names[] = {"hipLaunchKernelGGL", "hipExtLaunchKernelGGL + stop event", "hipModuleLaunchKernel (params)",
                           "hipModuleLaunchKernel (packed buffer)"};
    for (int rep = 0; rep < 2; ++rep)
        for (int V = 0; V < 4; ++V) {
            double tot = 0;
            for (int r = 0; r < ROUNDS; ++r) {
                CK(hipStreamSynchronize(s));
                const auto t0 = std::chrono::steady_clock::now();
                for (int i = 0; i < BATCH; ++i) {
                    a.v[1] = i;
                    if (V == 0) {
                        hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, s, a);
                    } else if (V == 1) {
                        hipExtLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, s, nullptr, ev, 0, a);
                    } else if (V == 2) {
                        void* params[] = {&a};
                        CK(hipModuleLaunchKernel(f, 256, 1, 1, 256, 1, 1, 0, s, params, nullptr));
                    } else {
                        size_t sz = sizeof(a);
                        void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                                         HIP_LAUNCH_PARAM_END};
                        CK(hipModuleLaunchKernel(f, 256, 1, 1, 256, 1, 1, 0, s, nullptr, extra));
                    }
                }
                tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            }
            CK(hipStreamSynchronize(s));
            if (rep) printf("%-40s %.2f us per launch (host enqueue)\n", names[V], tot / (ROUNDS * BATCH));
        }
    CK(hipGetLastError());
    return 0;
}
