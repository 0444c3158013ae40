// fp8 (OCP e4m3fn) quantisation for the config-5 forward GEMMs on gfx950 (BASELINE.json configs[4]:
// "GPT-2-medium backbone + 3-modality fusion, fp8 MFMA weight path").  Build-side: the reference trains
// in fp32 (src/main.py:62-68); SURVEY §8(c) states the fp8 tolerance.
//
// Scaling scheme (consumed by ergm_gemm_f8's epilogue):
//   activations  per row    scale[r] = max_c |X[r][c]| / 448,  Q[r][c] = e4m3(X[r][c] / scale[r])
//   weights      per output column of the Conv1D W[in][out]: scale[n] = max_k |W[k][n]| / 448, stored
//                transposed Wt[n][k] so both GEMM operands are k-contiguous
// 448 is the largest finite e4m3fn value; inputs are clamped to ±448 after the division so rounding can
// never reach the NaN code.  A row / column of zeros gets scale 1.  HBM-bound, one pass per tensor
// (weights: an amax pass and a quantise pass, both over L2-sized tiles).
#include "common.h"

namespace ergm {

__device__ __forceinline__ uint32_t fp8x4(float a, float b, float c, float d) {
    a = fminf(fmaxf(a, -448.f), 448.f);
    b = fminf(fmaxf(b, -448.f), 448.f);
    c = fminf(fmaxf(c, -448.f), 448.f);
    d = fminf(fmaxf(d, -448.f), 448.f);
    int q = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    q = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, q, true);
    return (uint32_t)q;
}

__device__ __forceinline__ uint8_t fp8x1(float a) {
    a = fminf(fmaxf(a, -448.f), 448.f);
    return (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(a, 0.f, 0, false) & 0xff);
}

__device__ __forceinline__ void load8(const void* X, bool bf16_in, size_t off, float* v) {
    if (bf16_in) {
        const bf16x8 x = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const __bf16*>(X) + off);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = bf2f(x[j]);
    } else {
        const float4 x0 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(X) + off);
        const float4 x1 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(X) + off + 4);
        v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
        v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
    }
}

// one row per wavefront; 8 consecutive columns per lane per pass (16-B bf16 / 32-B f32 loads)
template <bool BF16_IN>
__global__ __launch_bounds__(256) void quant_rows_kernel(const void* __restrict__ X, int ldx, int rows, int cols,
                                                         uint8_t* __restrict__ Q, int ldq, float* __restrict__ scale) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + wave;
    if (row >= rows) return;
    const size_t base = (size_t)row * ldx;
    float amax = 0.f;
    for (int c = lane * 8; c < cols; c += 512) {
        float v[8];
        load8(X, BF16_IN, base + c, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[j]));
    }
    amax = wave_max(amax);
    const float s = amax > 0.f ? amax / 448.f : 1.f;
    for (int c = lane * 8; c < cols; c += 512) {
        float v[8];
        load8(X, BF16_IN, base + c, v);
        uint2 o;
        o.x = fp8x4(v[0] / s, v[1] / s, v[2] / s, v[3] / s);
        o.y = fp8x4(v[4] / s, v[5] / s, v[6] / s, v[7] / s);
        *reinterpret_cast<uint2*>(Q + (size_t)row * ldq + c) = o;
    }
    if (lane == 0) scale[row] = s;
}

// Rows of at most NCH*512 columns: the row stays in registers (one read), same arithmetic as above.
template <bool BF16_IN, int NCH>
__global__ __launch_bounds__(256) void quant_rows_reg_kernel(const void* __restrict__ X, int ldx, int rows, int cols,
                                                             uint8_t* __restrict__ Q, int ldq, float* __restrict__ scale) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + wave;
    if (row >= rows) return;
    const size_t base = (size_t)row * ldx;
    float v[NCH][8];
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
        const int c = lane * 8 + i * 512;
        if (c < cols) {
            load8(X, BF16_IN, base + c, v[i]);
#pragma unroll
            for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v[i][j]));
        }
    }
    amax = wave_max(amax);
    const float s = amax > 0.f ? amax / 448.f : 1.f;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
        const int c = lane * 8 + i * 512;
        if (c < cols) {
            uint2 o;
            o.x = fp8x4(v[i][0] / s, v[i][1] / s, v[i][2] / s, v[i][3] / s);
            o.y = fp8x4(v[i][4] / s, v[i][5] / s, v[i][6] / s, v[i][7] / s);
            *reinterpret_cast<uint2*>(Q + (size_t)row * ldq + c) = o;
        }
    }
    if (lane == 0) scale[row] = s;
}

// ---- weights: batched over the matrices of one block (WqJobs in common.h) ------------------------

__device__ __forceinline__ int find_job(const WqJobs& J, int bid, bool q) {
    int k = 0;
#pragma unroll
    for (int i = 1; i < 8; ++i)
        if (i < J.n && bid >= (q ? J.j[i].blk_q : J.j[i].blk_amax)) k = i;
    return k;
}

constexpr int WQ_AMAX_COLS = 512;  // columns per amax block: 8 per lane (one 16-B bf16 load per row)
constexpr int WQ_AMAX_ROWS = 128;  // rows per amax block

// block = (job, 512-column tile, 128-row chunk): each lane keeps the running |w| max of 8 consecutive
// columns over every 4th row of the chunk; the 4 waves are merged through LDS and the result merged
// across chunks with atomicMax on the bit pattern (non-negative floats order like their bits: exact and
// order-independent)
__global__ __launch_bounds__(256) void wq_amax_kernel(WqJobs J) {
    __shared__ float red[4][WQ_AMAX_COLS];
    const int ji = find_job(J, blockIdx.x, false);
    const WqJob& jb = J.j[ji];
    const int local = blockIdx.x - jb.blk_amax;
    const int nt = (jb.N + WQ_AMAX_COLS - 1) / WQ_AMAX_COLS, kc = local / nt, n0 = (local % nt) * WQ_AMAX_COLS;
    const int lane = threadIdx.x & 63, rg = threadIdx.x >> 6;
    const int c = n0 + lane * 8;
    const int k0 = kc * WQ_AMAX_ROWS, k1 = min(jb.K, k0 + WQ_AMAX_ROWS);
    float m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = 0.f;
    if (c < jb.N) {
#pragma unroll 4
        for (int k = k0 + rg; k < k1; k += 4) {
            float v[8];
            load8(jb.W, jb.w_bf16, (size_t)k * jb.ldw + c, v);
#pragma unroll
            for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], fabsf(v[j]));
        }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) red[rg][lane * 8 + j] = m[j];
    __syncthreads();
    for (int i = threadIdx.x; i < WQ_AMAX_COLS; i += 256) {
        const float r = fmaxf(fmaxf(red[0][i], red[1][i]), fmaxf(red[2][i], red[3][i]));
        if (n0 + i < jb.N) atomicMax(jb.amax + n0 + i, __float_as_uint(r));
    }
}

// block = (job, 64-column tile, 64-row tile): thread = 4 consecutive rows x 4 consecutive columns
// (8-B bf16 / 16-B f32 loads), quantised with the column scales and packed per column into one dword
// of 4 k-consecutive bytes, transposed through LDS; then 64 rows of Wt (one per column) x 64 bytes
__global__ __launch_bounds__(256) void wq_quant_kernel(WqJobs J) {
    constexpr int LD = 80;  // bytes per LDS row (16-B aligned reads)
    __shared__ __attribute__((aligned(16))) uint8_t tile[64 * LD];
    const int ji = find_job(J, blockIdx.x, true);
    const WqJob& jb = J.j[ji];
    const int local = blockIdx.x - jb.blk_q;
    const int nt = jb.N / 64, kt = local / nt, n0 = (local % nt) * 64, k0 = kt * 64;
    const int nq = (threadIdx.x & 15) * 4, kq = (threadIdx.x >> 4) * 4;
    float s[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float amax = __uint_as_float(jb.amax[n0 + nq + j]);
        s[j] = amax > 0.f ? amax / 448.f : 1.f;
    }
    if (kt == 0 && kq == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) jb.scale[n0 + nq + j] = s[j];
    }
    float w[4][4];  // [row][column]
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int k = k0 + kq + r;
        const size_t idx = (size_t)k * jb.ldw + n0 + nq;
        if (k >= jb.K) {
            w[r][0] = w[r][1] = w[r][2] = w[r][3] = 0.f;
        } else if (jb.w_bf16) {
            const bf16x4 x = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const __bf16*>(jb.W) + idx);
#pragma unroll
            for (int j = 0; j < 4; ++j) w[r][j] = bf2f(x[j]);
        } else {
            const float4 x = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(jb.W) + idx);
            w[r][0] = x.x; w[r][1] = x.y; w[r][2] = x.z; w[r][3] = x.w;
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
        *reinterpret_cast<uint32_t*>(tile + (nq + j) * LD + kq) =
            fp8x4(w[0][j] / s[j], w[1][j] / s[j], w[2][j] / s[j], w[3][j] / s[j]);
    __syncthreads();
    const int n = threadIdx.x >> 2, q = threadIdx.x & 3;
    if (k0 + q * 16 < jb.K)
        *reinterpret_cast<uint4*>(jb.Wt + (size_t)(n0 + n) * jb.ldt + k0 + q * 16) =
            *reinterpret_cast<const uint4*>(tile + n * LD + q * 16);
}
int quant_weights_fp8(const WqJobs& J0, hipStream_t s) {
    WqJobs J = J0;
    ERGM_CHECK_ARG(J.n >= 1 && J.n <= 8, "quant_weights_fp8: 1..8 matrices per launch");
    int ba = 0, bq = 0;
    for (int i = 0; i < J.n; ++i) {
        WqJob& j = J.j[i];
        ERGM_CHECK_ARG(j.W && j.Wt && j.scale && j.amax && j.N % 64 == 0 && j.K % 64 == 0 && j.ldt >= j.K &&
                           j.ldt % 16 == 0 && j.ldw >= j.N && j.ldw % 8 == 0,
                       "quant_weights_fp8: bad matrix %d (K=%d N=%d)", i, j.K, j.N);
        j.blk_amax = ba;
        j.blk_q = bq;
        ba += cdiv(j.N, WQ_AMAX_COLS) * cdiv(j.K, WQ_AMAX_ROWS);
        bq += (j.N / 64) * (j.K / 64);
    }
    ERGM_LAUNCH(wq_amax_kernel, dim3(ba), dim3(256), 0, s, J);
    ERGM_LAUNCH(wq_quant_kernel, dim3(bq), dim3(256), 0, s, J);
    return check_launch("quant_weights_fp8");
}

// ---- MX-fp8 (OCP microscaling; common.h mx_*): e8m0 scale per 32 consecutive elements along K ----------
// Activations [rows][cols] -> Q [rows][ldq] e4m3 + S [rows][lds] e8m0 (block b = columns 32b..32b+31).  One row
// per wavefront, 8 columns per lane per pass: a block is 4 consecutive lanes.
template <bool BF16_IN>
__global__ __launch_bounds__(256) void mx_quant_rows_kernel(const void* __restrict__ X, int ldx, int rows, int cols,
                                                            uint8_t* __restrict__ Q, int ldq, uint8_t* __restrict__ S,
                                                            int lds) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + wave;
    if (row >= rows) return;
    const size_t base = (size_t)row * ldx;
    for (int c0 = 0; c0 < cols; c0 += 512) {  // cols % 32 == 0: a block is wholly in or out
        const int c = c0 + lane * 8;
        float v[8];
        if (c < cols) load8(X, BF16_IN, base + c, v);
        else {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = 0.f;
        }
        uint2 q;
        const int eb = mx_quant8_x4(v, q);
        if (c < cols) {
            *reinterpret_cast<uint2*>(Q + (size_t)row * ldq + c) = q;
            if ((lane & 3) == 0) S[mx_sidx(row, c >> 5, lds)] = (uint8_t)eb;
        }
    }
}

// Weights: MxJobs batched over one block's matrices.  Workgroup = (job, 64-row x 64-column tile of W); thread =
// 4 consecutive rows x 4 consecutive columns; column maxima of each 32-row block merged through LDS, then the
// quantised values packed per column (4 k-consecutive bytes) and written transposed through LDS as in
// wq_quant_kernel, with the block scales.
__device__ __forceinline__ int find_mx_job(const MxJobs& J, int bid) {
    int k = 0;
#pragma unroll
    for (int i = 1; i < 8; ++i)
        if (i < J.n && bid >= J.j[i].blk) k = i;
    return k;
}

__global__ __launch_bounds__(256) void mx_quant_weight_kernel(MxJobs J) {
    constexpr int LD = 80;
    __shared__ __attribute__((aligned(16))) uint8_t tile[64 * LD];
    __shared__ float red[16][64];
    __shared__ int ebs[2][64];
    const int ji = find_mx_job(J, blockIdx.x);
    const MxJob& jb = J.j[ji];
    const int local = blockIdx.x - jb.blk;
    const int nt = jb.N / 64, kt = local / nt, n0 = (local % nt) * 64, k0 = kt * 64;
    const int nq = (threadIdx.x & 15) * 4, kg = threadIdx.x >> 4, kq = kg * 4;
    float w[4][4];  // [row][column]
    float cm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const bf16x4 x = *reinterpret_cast<const bf16x4*>(jb.W + (size_t)(k0 + kq + r) * jb.ldw + n0 + nq);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            w[r][j] = bf2f(x[j]);
            cm[j] = fmaxf(cm[j], fabsf(w[r][j]));
        }
    }
    if (jb.Wr) {  // row form: a 32-column block is 8 consecutive threads (same row group kg)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float am = fmaxf(fmaxf(fabsf(w[r][0]), fabsf(w[r][1])), fmaxf(fabsf(w[r][2]), fabsf(w[r][3])));
            am = fmaxf(am, __shfl_xor(am, 1, 64));
            am = fmaxf(am, __shfl_xor(am, 2, 64));
            am = fmaxf(am, __shfl_xor(am, 4, 64));
            const int eb = mx_exp_biased(am);
            const float is = mx_inv_scale(eb);
            const size_t row = (size_t)(k0 + kq + r);
            *reinterpret_cast<uint32_t*>(jb.Wr + row * jb.ldr + n0 + nq) =
                mx_pack4(w[r][0] * is, w[r][1] * is, w[r][2] * is, w[r][3] * is);
            if ((threadIdx.x & 7) == 0) jb.scr[mx_sidx((int)row, (n0 + nq) >> 5, jb.ldsr)] = (uint8_t)eb;
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) red[kg][nq + j] = cm[j];
    __syncthreads();
    if (threadIdx.x < 128) {  // (block h, column n): max over the 8 row groups of the block
        const int h = threadIdx.x >> 6, n = threadIdx.x & 63;
        float m = red[8 * h][n];
#pragma unroll
        for (int i = 1; i < 8; ++i) m = fmaxf(m, red[8 * h + i][n]);
        const int eb = mx_exp_biased(m);
        ebs[h][n] = eb;
        jb.sc[mx_sidx(n0 + n, (k0 >> 5) + h, jb.lds)] = (uint8_t)eb;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float is = mx_inv_scale(ebs[kg >> 3][nq + j]);
        *reinterpret_cast<uint32_t*>(tile + (nq + j) * LD + kq) =
            mx_pack4(w[0][j] * is, w[1][j] * is, w[2][j] * is, w[3][j] * is);
    }
    __syncthreads();
    const int n = threadIdx.x >> 2, q = threadIdx.x & 3;
    *reinterpret_cast<uint4*>(jb.Wt + (size_t)(n0 + n) * jb.ldt + k0 + q * 16) =
        *reinterpret_cast<const uint4*>(tile + n * LD + q * 16);
}

int quant_weights_mx(const MxJobs& J0, hipStream_t s) {
    MxJobs J = J0;
    ERGM_CHECK_ARG(J.n >= 1 && J.n <= 8, "quant_weights_mx: 1..8 matrices per launch");
    int b = 0;
    for (int i = 0; i < J.n; ++i) {
        MxJob& j = J.j[i];
        ERGM_CHECK_ARG(j.W && j.Wt && j.sc && j.N % 64 == 0 && j.K % 64 == 0 && j.ldt >= j.K && j.ldt % 16 == 0 &&
                           j.ldw >= j.N && j.ldw % 4 == 0 && j.lds >= j.N,
                       "quant_weights_mx: bad matrix %d (K=%d N=%d)", i, j.K, j.N);
        ERGM_CHECK_ARG(!j.Wr || (j.scr && j.ldr >= j.N && j.ldr % 4 == 0 && j.ldsr >= j.K),
                       "quant_weights_mx: bad row-form output of matrix %d", i);
        j.blk = b;
        b += (j.N / 64) * (j.K / 64);
    }
    ERGM_LAUNCH(mx_quant_weight_kernel, dim3(b), dim3(256), 0, s, J);
    return check_launch("quant_weights_mx");
}

int quant_rows_mx(const void* X, int x_dtype, int ldx, int rows, int cols, void* Q, int ldq, void* S, int lds,
                  hipStream_t s) {
    ERGM_CHECK_ARG(X && Q && S && rows > 0 && cols > 0 && cols % 32 == 0 && ldx % 8 == 0 && ldx >= cols &&
                       ldq >= cols && ldq % 8 == 0 && lds >= rows,
                   "quant_rows_mx: bad argument");
    ERGM_CHECK_ARG(x_dtype == ERGM_BF16 || x_dtype == ERGM_F32, "quant_rows_mx: bad dtype");
    dim3 grid(cdiv(rows, 4));
    auto* q = reinterpret_cast<uint8_t*>(Q);
    auto* sc = reinterpret_cast<uint8_t*>(S);
    if (x_dtype == ERGM_BF16) ERGM_LAUNCH(mx_quant_rows_kernel<true>, grid, dim3(256), 0, s, X, ldx, rows, cols, q, ldq, sc, lds);
    else ERGM_LAUNCH(mx_quant_rows_kernel<false>, grid, dim3(256), 0, s, X, ldx, rows, cols, q, ldq, sc, lds);
    return check_launch("quant_rows_mx");
}

int quant_rows_fp8(const void* X, int x_dtype, int ldx, int rows, int cols, void* Q, int ldq, float* scale,
                   hipStream_t s) {
    ERGM_CHECK_ARG(X && Q && scale && rows > 0 && cols > 0 && cols % 8 == 0 && ldx % 8 == 0 && ldx >= cols &&
                       ldq >= cols && ldq % 8 == 0,
                   "quant_rows_fp8: bad argument");
    ERGM_CHECK_ARG(x_dtype == ERGM_BF16 || x_dtype == ERGM_F32, "quant_rows_fp8: bad dtype");
    dim3 grid(cdiv(rows, 4));
    auto* q = reinterpret_cast<uint8_t*>(Q);
    const int nch = cdiv(cols, 512);
    if (x_dtype == ERGM_BF16) {
        if (nch <= 2) ERGM_LAUNCH((quant_rows_reg_kernel<true, 2>), grid, dim3(256), 0, s, X, ldx, rows, cols, q, ldq, scale);
        else if (nch <= 4) ERGM_LAUNCH((quant_rows_reg_kernel<true, 4>), grid, dim3(256), 0, s, X, ldx, rows, cols, q, ldq, scale);
        else if (nch <= 8) ERGM_LAUNCH((quant_rows_reg_kernel<true, 8>), grid, dim3(256), 0, s, X, ldx, rows, cols, q, ldq, scale);
        else ERGM_LAUNCH(quant_rows_kernel<true>, grid, dim3(256), 0, s, X, ldx, rows, cols, q, ldq, scale);
    } else {
        ERGM_LAUNCH(quant_rows_kernel<false>, grid, dim3(256), 0, s, X, ldx, rows, cols, q, ldq, scale);
    }
    return check_launch("quant_rows_fp8");
}

}  // namespace ergm

using namespace ergm;

extern "C" int ergm_quant_rows_fp8(const void* X, int x_dtype, int ldx, int rows, int cols, void* Q, int ldq,
                                   float* scale, void* stream) {
    return quant_rows_fp8(X, x_dtype, ldx, rows, cols, Q, ldq, scale, as_stream(stream));
}

extern "C" int ergm_quant_weight_fp8(const void* W, int w_dtype, int ldw, int K, int N, void* Wt, int ldt,
                                     float* scale, void* amax_ws, void* stream) {
    ERGM_CHECK_ARG(amax_ws, "quant_weight_fp8: amax workspace (N x 4 bytes) required");
    ERGM_CHECK_ARG(w_dtype == ERGM_F32 || w_dtype == ERGM_BF16, "quant_weight_fp8: bad dtype");
    hipStream_t s = as_stream(stream);
    if (hipMemsetAsync(amax_ws, 0, (size_t)N * 4, s) != hipSuccess) return fail(ERGM_EHIP, "quant_weight_fp8: memset");
    WqJobs J{};
    J.n = 1;
    J.j[0] = WqJob{W, reinterpret_cast<uint8_t*>(Wt), scale, reinterpret_cast<unsigned*>(amax_ws), ldw, K, N, ldt, 0, 0,
                   w_dtype == ERGM_BF16};
    return quant_weights_fp8(J, s);
}

extern "C" int ergm_quant_rows_mx(const void* X, int x_dtype, int ldx, int rows, int cols, void* Q, int ldq, void* S,
                                  int lds, void* stream) {
    return quant_rows_mx(X, x_dtype, ldx, rows, cols, Q, ldq, S, lds, as_stream(stream));
}

extern "C" int ergm_quant_weight_mx(const void* W, int ldw, int K, int N, void* Wt, int ldt, void* S, int lds,
                                    void* Wr, int ldr, void* Sr, int ldsr, void* stream) {
    MxJobs J{};
    J.n = 1;
    J.j[0] = MxJob{reinterpret_cast<const __bf16*>(W), reinterpret_cast<uint8_t*>(Wt), reinterpret_cast<uint8_t*>(S), ldw,
                   K, N, ldt, lds, 0, reinterpret_cast<uint8_t*>(Wr), reinterpret_cast<uint8_t*>(Sr), ldr, ldsr};
    return quant_weights_mx(J, as_stream(stream));
}
