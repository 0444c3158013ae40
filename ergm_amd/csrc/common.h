// Internal helpers shared by the gfx950 kernels of libergm_hip.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <string>

#include "../../include/ergm_hip.h"

namespace ergm {

// ---- error state (thread-local; ergm_last_error reads it) ----------------------------------
void set_error(const char* fmt, ...);
int fail(int code, const char* fmt, ...);
int check_launch(const char* what);

#define ERGM_CHECK_ARG(cond, ...)                                   \
    do {                                                            \
        if (!(cond)) return ::ergm::fail(ERGM_EINVAL, __VA_ARGS__); \
    } while (0)
#define ERGM_TRY(expr)                 \
    do {                               \
        int _rc = (expr);              \
        if (_rc != ERGM_OK) return _rc; \
    } while (0)

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline int cdiv(int a, int b) { return (a + b - 1) / b; }

// ---- device types -----------------------------------------------------------------------
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef uint16_t bf16_t;  // storage type on the host side / in pointer arithmetic

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

__device__ __forceinline__ float bf2f(__bf16 x) { return (float)x; }
__device__ __forceinline__ __bf16 f2bf(float x) { return (__bf16)x; }  // RNE (v_cvt_pk_bf16_f32)

__device__ __forceinline__ float bits2f(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }

// fp8 weight quantisation jobs (quant.hip), batched over the matrices of one block
struct WqJob {
    const void* W;        // [K][ldw] f32 or bf16 (Conv1D [in, out]), see w_bf16
    uint8_t* Wt;          // [N][ldt] e4m3 (transposed)
    float* scale;         // [N]
    unsigned* amax;       // [N] |w| bit patterns, zeroed by the caller
    int ldw, K, N, ldt;
    int blk_amax, blk_q;  // first block of this job in each grid (set by quant_weights_fp8)
    int w_bf16;           // W is the bf16 shadow (the executor) rather than the f32 master
};
struct WqJobs {
    WqJob j[8];
    int n;
};

// wave-level reductions over 64 lanes, all VALU (no ds_bpermute round trips): DPP quad_perm [1,0,3,2]
// and [2,3,0,1], row_half_mirror and row_mirror inside each 16-lane row, then the gfx950 row swaps
// v_permlane16_swap / v_permlane32_swap across rows.  Every step combines a lane's value with its
// partner's by a commutative op, so all 64 lanes end with the bit-identical result.  Full waves only.
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <bool MAX>
__device__ __forceinline__ float wave_reduce(float v) {
    auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : a + b; };
    v = op(v, dpp_f32<0xB1>(v));   // quad_perm [1,0,3,2]
    v = op(v, dpp_f32<0x4E>(v));   // quad_perm [2,3,0,1]
    v = op(v, dpp_f32<0x141>(v));  // row_half_mirror
    v = op(v, dpp_f32<0x140>(v));  // row_mirror
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = op(__uint_as_float(r[0]), __uint_as_float(r[1]));
    r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return op(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float wave_sum(float v) { return wave_reduce<false>(v); }
__device__ __forceinline__ float wave_max(float v) { return wave_reduce<true>(v); }

// gelu_new (transformers NewGELUActivation): 0.5x(1+tanh(sqrt(2/pi)(x+0.044715x^3)))
__device__ __forceinline__ float gelu_new(float x) {
    const float k0 = 0.7978845608028654f;  // sqrt(2/pi)
    float u = k0 * (x + 0.044715f * x * x * x);
    return 0.5f * x * (1.0f + tanhf(u));
}
__device__ __forceinline__ float gelu_new_grad(float x) {
    const float k0 = 0.7978845608028654f;
    float x2 = x * x;
    float u = k0 * (x + 0.044715f * x2 * x);
    float t = tanhf(u);
    return 0.5f * (1.0f + t) + 0.5f * x * (1.0f - t * t) * k0 * (1.0f + 3.0f * 0.044715f * x2);
}

}  // namespace ergm
