// Which part of the executor's three-stream fork/join pattern makes hipStreamEndCapture crash (round 6: a whole-step
// capture of the training forward segfaults in EndCapture, profiles/r06_graph_capture_segv.txt)?  Captures the forward's
// pattern — fork two streams off the capturing one with recorded events, one of them starting with a memset and
// waiting for the other, join both back — with the events created under different flags, instantiates the graph and
// replays it, checking the result.  Usage: capture_probe <variant>
//   0: events with flags 0; 1: hipEventDisableTiming; 2: | hipEventDisableSystemFence (the executor's); 3: as 2 with
//   a memset as the side stream's first captured operation (the executor's row-flag clear)
#include <hip/hip_runtime.h>

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

__global__ void add(float* x, float v, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) x[i] += v;
}

int main(int argc, char** argv) {
    const int V = argc > 1 ? atoi(argv[1]) : 0;
    const unsigned flags = V == 0 ? 0u : V == 1 ? hipEventDisableTiming : hipEventDisableTiming | hipEventDisableSystemFence;
    const int n = 1 << 16;
    float *a, *b, *c;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMalloc(&c, n * 4));
    hipStream_t s, f2, side;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&f2, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    hipEvent_t e_fork, e_emb, e_side, e_done;
    CK(hipEventCreateWithFlags(&e_fork, flags));
    CK(hipEventCreateWithFlags(&e_emb, flags));
    CK(hipEventCreateWithFlags(&e_side, flags));
    CK(hipEventCreateWithFlags(&e_done, flags));
    CK(hipMemset(a, 0, n * 4));
    CK(hipMemset(b, 0, n * 4));
    CK(hipMemset(c, 0, n * 4));
    CK(hipDeviceSynchronize());

    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    CK(hipEventRecord(e_fork, s));
    CK(hipStreamWaitEvent(f2, e_fork, 0));
    hipLaunchKernelGGL(add, dim3(n / 256), dim3(256), 0, f2, b, 1.f, n);
    CK(hipEventRecord(e_emb, f2));
    hipLaunchKernelGGL(add, dim3(n / 256), dim3(256), 0, s, a, 1.f, n);
    CK(hipEventRecord(e_fork, s));
    CK(hipStreamWaitEvent(side, e_fork, 0));
    CK(hipStreamWaitEvent(side, e_emb, 0));
    if (V == 3) CK(hipMemsetAsync(c, 0, n * 4, side));
    hipLaunchKernelGGL(add, dim3(n / 256), dim3(256), 0, side, c, 2.f, n);
    CK(hipEventRecord(e_side, side));
    CK(hipStreamWaitEvent(s, e_side, 0));
    CK(hipStreamWaitEvent(f2, e_side, 0));
    hipLaunchKernelGGL(add, dim3(n / 256), dim3(256), 0, f2, b, 1.f, n);
    hipLaunchKernelGGL(add, dim3(n / 256), dim3(256), 0, s, a, 1.f, n);
    CK(hipEventRecord(e_done, f2));
    CK(hipStreamWaitEvent(s, e_done, 0));
    hipLaunchKernelGGL(add, dim3(n / 256), dim3(256), 0, s, a, 1.f, n);
    printf("variant %d: ending capture\n", V);
    fflush(stdout);
    hipGraph_t g;
    CK(hipStreamEndCapture(s, &g));
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < 3; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    float ha, hb, hc;
    CK(hipMemcpy(&ha, a + 7, 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&hb, b + 7, 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&hc, c + 7, 4, hipMemcpyDeviceToHost));
    printf("variant %d: a %.0f (want 9) b %.0f (want 6) c %.0f (want %d)\n", V, ha, hb, hc, V == 3 ? 2 : 6);
    return 0;
}
