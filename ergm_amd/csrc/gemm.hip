// bf16 MFMA GEMM for gfx950 (CDNA4): every Conv1D / Linear contraction of the ERGM training step.
//
// Replaces transformers Conv1D.forward (addmm(b, x, W[in,out])) used at src/model.py:95-99,257-258,
// the tied lm_head nn.Linear (src/model.py:605,698) and their autograd backward GEMMs.
//
// C[M][N] = epilogue(alpha * Σ_k A(m,k) B(k,n)), A/B bf16, fp32 accumulate.
//   A storage: MK = A[m][k] (k contiguous) or KM = A[k][m]      (KM: weight-gradient GEMMs Xᵀ·dY)
//   B storage: NK = B[n][k] (Linear weight) or KN = B[k][n]    (Conv1D weight [in,out])
// Tiles of BM×BN×64 staged global→registers→LDS (double buffered, one barrier per K-step);
// 4 waves (2×2), each owning (BM/2)×(BN/2) as 16×16 MFMA tiles (v_mfma_f32_16x16x32_bf16).
// k-contiguous tiles are read row-wise with ds_read_b128 (16-B chunk XOR row&7 swizzle);
// m/n-contiguous tiles are read column-wise with ds_read_b64_tr_b16 (CDNA4 transpose read) under a
// row-dependent chunk XOR that keeps each 32-lane half conflict-free.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>

#include "common.h"
#include "tiles.h"

namespace ergm {


struct GemmArgs {
    const __bf16* A;
    const __bf16* B;
    void* C;
    int M, N, K;
    int lda, ldb, ldc;
    float alpha;
    const float* alpha_dev;
    const float* bias;
    const void* aux;
    int ld_aux;
    void* aux_out;
    int ld_aux_out;
    int tiles_m, tiles_n;
    int sweep_m;        // 1: consecutive tile ids walk M (B panel reused), 0: walk N
    int k_per_split;    // K range per blockIdx.z (multiple of 64)
    float* slab;        // split-K partials [z][M][N] (f32) or nullptr
    const float* a_scale;  // fp8 GEMM: per-row dequantisation scale of A [M] (nullptr: none)
    const float* b_scale;  // fp8 GEMM: per-column dequantisation scale of B [N]
    int nt_store;          // C written with non-temporal stores (streamed output)
    DropSite drop;         // BIAS_RESID: dropout of the residual branch (src/model.py:245,266), rows m, cols n
    float* colsum;         // KM x KN, EPI_NONE: bias gradient alpha·Σ_k B[k][n] -> colsum[n] (nullptr: none)
    float* colsum_part;    // split-K: per-split partial column sums [z][N] (combined by splitk_reduce_kernel)
    int xcd_split;         // split-K over 8 K slices, one per XCD: grid.x = 8·tiles, slice = blockIdx.x & 7, so
                           // every tile of one K slice shares an XCD's L2 (pipelined kernel only)
    // MX-fp8 GEMM (gemm_mx_kernel): e8m0 scales of every 32-element K block, A [M][ld_sa], B [N][ld_sb] bytes
    const uint8_t* a_mx;
    const uint8_t* b_mx;
    int ld_sa, ld_sb;
    // MX-fp8 copy of the (bf16) output C written by the epilogue: q_out [M][ld_q] e4m3, q_sc [M][ld_qs] e8m0
    uint8_t* q_out;
    uint8_t* q_sc;
    int ld_q, ld_qs;
};

template <int EPI, bool OUT_BF16>
__device__ __forceinline__ void epilogue_store(const GemmArgs& a, int m, int n, float v) {
    if (EPI == ERGM_EPI_BIAS || EPI == ERGM_EPI_BIAS_GELU || EPI == ERGM_EPI_BIAS_RESID) {
        if (a.bias) v += a.bias[n];
    }
    if (EPI == ERGM_EPI_BIAS_GELU) {
        float dg;
        v = gelu_new_fwd(v, dg);
        reinterpret_cast<__bf16*>(a.aux_out)[(size_t)m * a.ld_aux_out + n] = f2bf(dg);
    } else if (EPI == ERGM_EPI_BIAS_RESID) {
        if (a.drop.thresh) v = drop_keep1(a.drop, m, n) ? v * a.drop.scale : 0.f;
        v += reinterpret_cast<const float*>(a.aux)[(size_t)m * a.ld_aux + n];
    } else if (EPI == ERGM_EPI_GELU_BWD) {
        v *= bf2f(reinterpret_cast<const __bf16*>(a.aux)[(size_t)m * a.ld_aux + n]);  // stored gelu'(pre)
    }
    size_t idx = (size_t)m * a.ldc + n;
    if (OUT_BF16) {
        reinterpret_cast<__bf16*>(a.C)[idx] = f2bf(v);
    } else {
        float* c = reinterpret_cast<float*>(a.C);
        if (EPI == ERGM_EPI_ACCUM) v += c[idx];
        c[idx] = v;
    }
}

// Vectorized epilogue for 8 consecutive columns n..n+7 of row m (N % 8 == 0, n % 8 == 0).
// pre_bias / pre_aux: the bias (2 float4) and aux operand (BIAS_RESID: 2 float4 of the residual; GELU_BWD: one float4
// holding 8 bf16) of these 8 columns, loaded before the main loop (EpiPre) — nullptr: loaded here.
template <int EPI, bool OUT_BF16>
__device__ __forceinline__ void epilogue_store8(const GemmArgs& a, int m, int n, float* v,
                                                const float4* pre_bias = nullptr, const float4* pre_aux = nullptr) {
    if (EPI == ERGM_EPI_BIAS || EPI == ERGM_EPI_BIAS_GELU || EPI == ERGM_EPI_BIAS_RESID) {
        if (a.bias) {
            float4 b0 = pre_bias ? pre_bias[0] : *reinterpret_cast<const float4*>(a.bias + n);
            float4 b1 = pre_bias ? pre_bias[1] : *reinterpret_cast<const float4*>(a.bias + n + 4);
            v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
            v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
        }
    }
    if (EPI == ERGM_EPI_BIAS_GELU) {  // C = gelu_new(v), aux_out = gelu_new'(v) for the backward
        bf16x8 dgb;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float dg;
            v[j] = gelu_new_fwd(v[j], dg);
            dgb[j] = f2bf(dg);
        }
        *reinterpret_cast<bf16x8*>(reinterpret_cast<__bf16*>(a.aux_out) + (size_t)m * a.ld_aux_out + n) = dgb;
    } else if (EPI == ERGM_EPI_BIAS_RESID) {
        if (a.drop.thresh) {  // residual-branch dropout, then the residual add
            const unsigned k = drop_keep4(a.drop, m, n) | (drop_keep4(a.drop, m, n + 4) << 4);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = ((k >> j) & 1u) ? v[j] * a.drop.scale : 0.f;
        }
        const float* r = reinterpret_cast<const float*>(a.aux) + (size_t)m * a.ld_aux + n;
        float4 r0 = pre_aux ? pre_aux[0] : *reinterpret_cast<const float4*>(r);
        float4 r1 = pre_aux ? pre_aux[1] : *reinterpret_cast<const float4*>(r + 4);
        v[0] += r0.x; v[1] += r0.y; v[2] += r0.z; v[3] += r0.w;
        v[4] += r1.x; v[5] += r1.y; v[6] += r1.z; v[7] += r1.w;
    } else if (EPI == ERGM_EPI_GELU_BWD) {  // v · gelu_new'(pre), the derivative stored by the forward
        bf16x8 x = pre_aux ? __builtin_bit_cast(bf16x8, pre_aux[0])
                           : *reinterpret_cast<const bf16x8*>(reinterpret_cast<const __bf16*>(a.aux) + (size_t)m * a.ld_aux + n);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] *= bf2f(x[j]);
    }
    const size_t idx = (size_t)m * a.ldc + n;
    if (OUT_BF16) {
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            o[j] = f2bf(v[j]);
            v[j] = bf2f(o[j]);  // the stored value (an MX copy quantises exactly what the bf16 consumers read)
        }
        bf16x8* dst = reinterpret_cast<bf16x8*>(reinterpret_cast<__bf16*>(a.C) + idx);
        if (a.nt_store) __builtin_nontemporal_store(o, dst);
        else *dst = o;
    } else {
        float4* c = reinterpret_cast<float4*>(reinterpret_cast<float*>(a.C) + idx);
        float4 o0 = make_float4(v[0], v[1], v[2], v[3]), o1 = make_float4(v[4], v[5], v[6], v[7]);
        if (EPI == ERGM_EPI_ACCUM) {
            float4 p0 = c[0], p1 = c[1];
            o0.x += p0.x; o0.y += p0.y; o0.z += p0.z; o0.w += p0.w;
            o1.x += p1.x; o1.y += p1.y; o1.z += p1.z; o1.w += p1.w;
        }
        if (a.nt_store) {
            __builtin_nontemporal_store(f32x4{o0.x, o0.y, o0.z, o0.w}, reinterpret_cast<f32x4*>(c));
            __builtin_nontemporal_store(f32x4{o1.x, o1.y, o1.z, o1.w}, reinterpret_cast<f32x4*>(c + 1));
        } else {
            c[0] = o0;
            c[1] = o1;
        }
    }
}

// Epilogue operands loaded before the main loop: a BIAS_RESID / GELU_BWD epilogue reads the residual (f32) / the
// stored gelu' (bf16) of its tile and the bias, and at the end of the kernel those loads' latency is exposed (every
// wave waits for them with nothing left to overlap).  When store_tile gives each thread exactly one 8-column chunk per
// pass (WM·CPR == NT), the thread knows its chunks up front and loads them while the K loop runs: WGM·8 floats (or
// WGM·8 bf16) + 8 bias floats of registers.  Same values, same arithmetic: the output is bitwise unchanged.
template <int EPI, int BM, int BN, int WGM, int NT>
struct EpiPre {
    static constexpr int WM = BM / WGM, CPR = BN / 8;
    static constexpr int PER = EPI == ERGM_EPI_BIAS_RESID ? 2 : 1;  // float4 per chunk
    static constexpr bool ON = (EPI == ERGM_EPI_BIAS_RESID || EPI == ERGM_EPI_GELU_BWD) && WM * CPR == NT &&
                               WGM * PER <= 4;
    float4 aux[ON ? WGM * PER : 1];
    float4 bias[2];
    __device__ __forceinline__ void load(const GemmArgs& a, int m0, int n0) {
        if constexpr (ON) {
            if (a.slab) return;  // split-K partials: the reduce kernel applies the epilogue
            const int row = threadIdx.x / CPR, n = n0 + (threadIdx.x % CPR) * 8;
            if (n >= a.N) return;
            if (EPI == ERGM_EPI_BIAS_RESID && a.bias) {
                bias[0] = *reinterpret_cast<const float4*>(a.bias + n);
                bias[1] = *reinterpret_cast<const float4*>(a.bias + n + 4);
            }
#pragma unroll
            for (int p = 0; p < WGM; ++p) {
                const int m = m0 + p * WM + row;
                if (m >= a.M) continue;
                if constexpr (EPI == ERGM_EPI_BIAS_RESID) {
                    const float* r = reinterpret_cast<const float*>(a.aux) + (size_t)m * a.ld_aux + n;
                    aux[2 * p] = *reinterpret_cast<const float4*>(r);
                    aux[2 * p + 1] = *reinterpret_cast<const float4*>(r + 4);
                } else {
                    aux[p] = *reinterpret_cast<const float4*>(reinterpret_cast<const __bf16*>(a.aux) +
                                                              (size_t)m * a.ld_aux + n);
                }
            }
        }
    }
};

// Write a BM x BN accumulator tile (WGM x WGN waves, 16x16 MFMA fragments) through LDS so that every
// global store is a coalesced 16-B (bf16) / 32-B (f32) row piece instead of per-lane 2/4-B scatters
// (the per-lane form made the large GEMMs store-issue bound).  One wave-row (BM/WGM rows) per pass, so
// the staging buffer is (BM/WGM)*(BN+4) floats.  slab != nullptr: raw f32 split-K partials.
// MF: the accumulator fragments' MFMA shape — 16 (f32x4 per 16x16 fragment: lane l holds rows 4(l>>4)+r of column
// l&15) or 32 (f32x16 per 32x32 fragment: lane l holds rows (r&3) + 8(r>>2) + 4(l>>5) of column l&31).
template <int BM, int BN, int WGM, int WGN, int EPI, bool OUT_BF16, int FM, int FN, int NT = 64 * WGM * WGN,
          bool RS = false, bool QMX = false, int MF = 16, typename AccT = f32x4>
__device__ __forceinline__ void store_tile(const GemmArgs& a, char* lds, AccT (&acc)[FM][FN], int m0, int n0,
                                           float alpha, float* slab, const EpiPre<EPI, BM, BN, WGM, NT>* pre = nullptr) {
    // NT: every thread of the workgroup (a warp-specialised kernel adds producer waves, which only
    // help with the copy-out; accumulator fragments come from the WGM x WGN consumer waves)
    constexpr int LD = BN + 4;  // lanes l and l+16 (rows 4 apart) land 16 banks apart
    constexpr int WM = BM / WGM, WN = BN / WGN;
    float* t = reinterpret_cast<float*>(lds);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wm = wave / WGN, wn = wave % WGN;
    constexpr int CPR = BN / 8;  // 8-column chunks per row
#pragma unroll
    for (int pass = 0; pass < WGM; ++pass) {
        __syncthreads();
        if (wave < WGM * WGN && wm == pass) {
            if constexpr (MF == 16) {
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            t[(i * 16 + (lane >> 4) * 4 + r) * LD + wn * WN + j * 16 + (lane & 15)] = acc[i][j][r];
            } else {
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
#pragma unroll
                        for (int r = 0; r < 16; ++r)
                            t[(i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * LD + wn * WN + j * 32 + (lane & 31)] =
                                acc[i][j][r];
            }
        }
        __syncthreads();
        for (int c = threadIdx.x; c < WM * CPR; c += NT) {
            const int row = c / CPR, col = (c % CPR) * 8;
            const int m = m0 + pass * WM + row, n = n0 + col;
            if constexpr (QMX) {  // every lane reaches the block's shuffles (WM·CPR is a multiple of NT here)
                static_assert(BN % 32 == 0 && (WM * CPR) % NT == 0, "MX epilogue: whole 32-column blocks per pass");
                const bool ok = m < a.M && n < a.N;
                const float4 x0 = *reinterpret_cast<const float4*>(t + row * LD + col);
                const float4 x1 = *reinterpret_cast<const float4*>(t + row * LD + col + 4);
                float v[8] = {x0.x * alpha, x0.y * alpha, x0.z * alpha, x0.w * alpha,
                              x1.x * alpha, x1.y * alpha, x1.z * alpha, x1.w * alpha};
                if (ok) epilogue_store8<EPI, OUT_BF16>(a, m, n, v);
                else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) v[j] = 0.f;
                }
                uint2 q;
                const int eb = mx_quant8_x4(v, q);
                if (ok) {
                    *reinterpret_cast<uint2*>(a.q_out + (size_t)m * a.ld_q + n) = q;
                    if ((c & 3) == 0) a.q_sc[mx_sidx(m, n >> 5, a.ld_qs)] = (uint8_t)eb;
                }
                continue;
            }
            if (m >= a.M || n >= a.N) continue;
            const float4 x0 = *reinterpret_cast<const float4*>(t + row * LD + col);
            const float4 x1 = *reinterpret_cast<const float4*>(t + row * LD + col + 4);
            if (slab) {
                float4* d = reinterpret_cast<float4*>(slab + (size_t)m * a.N + n);
                d[0] = x0;
                d[1] = x1;
            } else {
                float v[8] = {x0.x * alpha, x0.y * alpha, x0.z * alpha, x0.w * alpha,
                              x1.x * alpha, x1.y * alpha, x1.z * alpha, x1.w * alpha};
                if constexpr (RS) {  // fp8 dequantisation: row scale of A times column scale of B
                    const float sa = a.a_scale[m];
                    const float4 b0 = *reinterpret_cast<const float4*>(a.b_scale + n);
                    const float4 b1 = *reinterpret_cast<const float4*>(a.b_scale + n + 4);
                    const float sb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
                    for (int j = 0; j < 8; ++j) v[j] *= sa * sb[j];
                }
                if constexpr (EpiPre<EPI, BM, BN, WGM, NT>::ON) {
                    if (pre) {  // c == threadIdx.x: this thread's chunk of pass `pass`, loaded before the K loop
                        constexpr int PER = EpiPre<EPI, BM, BN, WGM, NT>::PER;
                        epilogue_store8<EPI, OUT_BF16>(a, m, n, v, pre->bias, pre->aux + PER * pass);
                        continue;
                    }
                }
                epilogue_store8<EPI, OUT_BF16>(a, m, n, v);
            }
        }
    }
}

// LDS-free epilogue for tiles computed with SWAPPED MFMA operands (mfma(B-frag, A-frag) = Cᵀ fragments:
// lane (g = l>>4, i = l&15) holds C[m = 16·blk + i][n = 16·j + 4g + r], r = 0..3, i.e. 4 consecutive
// columns of one row).  v_permlane16_swap of fragments (i, i+1) exchanges the odd 16-lane rows of the
// first with the even rows of the second, after which every lane holds 8 consecutive columns of one row
// (block i + (g & 1), columns 16j + 8(g >> 1) ..+7): one 8-wide epilogue store per fragment pair, no LDS
// staging and no barriers.
template <int WGN, int EPI, bool OUT_BF16, int FM, int FN, int WM, int WN>
__device__ __forceinline__ void store_tile_direct(const GemmArgs& a, f32x4 (&acc)[FM][FN], int m0, int n0,
                                                  float alpha) {
    static_assert(FM % 2 == 0, "direct store pairs row fragments");
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wm = wave / WGN, wn = wave % WGN;
    const int g = lane >> 4, i16 = lane & 15;
#pragma unroll
    for (int i = 0; i < FM; i += 2)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            float v[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][j][r]),
                                                           __float_as_uint(acc[i + 1][j][r]), false, false);
                v[r] = __uint_as_float(sw[0]) * alpha;
                v[4 + r] = __uint_as_float(sw[1]) * alpha;
            }
            const int m = m0 + wm * WM + (i + (g & 1)) * 16 + i16;
            const int n = n0 + wn * WN + j * 16 + 8 * (g >> 1);
            if (m < a.M && n < a.N) epilogue_store8<EPI, OUT_BF16>(a, m, n, v);
        }
}

// bijective XCD-grouping remap: blocks b, b+8, ... share an XCD; give each XCD a contiguous range.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int NX = 8;
    if (nwg < NX) return bid;
    int xcd = bid % NX, idx = bid / NX;
    int q = nwg / NX, r = nwg % NX;
    int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + idx;
}

template <int BM, int BN, bool A_KM, bool B_KN, int EPI, bool OUT_BF16>
__global__ __launch_bounds__(GEMM_THREADS) void gemm_kernel(GemmArgs a) {
    constexpr int WM = BM / 2, WN = BN / 2;
    constexpr int FM = WM / 16, FN = WN / 16;
    constexpr int A_BYTES = BM * GEMM_BK * 2, B_BYTES = BN * GEMM_BK * 2;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int STAGE = A_BYTES + B_BYTES;

    const int nwg = a.tiles_m * a.tiles_n;
    const int id = xcd_remap(blockIdx.x, nwg);
    int tm, tn;
    if (a.sweep_m) { tm = id % a.tiles_m; tn = id / a.tiles_m; }
    else { tn = id % a.tiles_n; tm = id / a.tiles_n; }
    const int m0 = tm * BM, n0 = tn * BN;
    const int kbeg = blockIdx.z * a.k_per_split;
    const int kend = min(a.K, kbeg + a.k_per_split);
    const int nk = (kend - kbeg + GEMM_BK - 1) / GEMM_BK;

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int wm = wave >> 1, wn = wave & 1;

    TileLoader<BM, A_KM> la;
    TileLoader<BN, B_KN> lb;
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (nk > 0) {
        la.load(a.A, a.lda, m0, kbeg, a.M, kend);
        lb.load(a.B, a.ldb, n0, kbeg, a.N, kend);
        la.store(smem);
        lb.store(smem + A_BYTES);
    }
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = kt & 1;
        const bool more = kt + 1 < nk;
        if (more) {
            la.load(a.A, a.lda, m0, kbeg + (kt + 1) * GEMM_BK, a.M, kend);
            lb.load(a.B, a.ldb, n0, kbeg + (kt + 1) * GEMM_BK, a.N, kend);
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 fa[FM], fb[FN];
#pragma unroll
            for (int i = 0; i < FM; ++i) fa[i] = la.frag(smem + cur * STAGE, wm * WM + i * 16, ks);
#pragma unroll
            for (int j = 0; j < FN; ++j) fb[j] = lb.frag(smem + cur * STAGE + A_BYTES, wn * WN + j * 16, ks);
#pragma unroll
            for (int i = 0; i < FM; ++i)
#pragma unroll
                for (int j = 0; j < FN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
        if (more) {
            la.store(smem + (cur ^ 1) * STAGE);
            lb.store(smem + (cur ^ 1) * STAGE + A_BYTES);
        }
        __syncthreads();
    }

    float alpha = a.alpha;
    if (a.alpha_dev) alpha *= *a.alpha_dev;
    float* slab = a.slab ? a.slab + (size_t)blockIdx.z * a.M * a.N : nullptr;
    if (a.N % 8 == 0 && (a.slab || a.ldc % 8 == 0)) {
        store_tile<BM, BN, 2, 2, EPI, OUT_BF16, FM, FN>(a, smem, acc, m0, n0, alpha, slab);
        return;
    }
    const int lane_ = threadIdx.x & 63, wave_ = threadIdx.x >> 6;
    const int rbase = m0 + (wave_ >> 1) * WM + (lane_ >> 4) * 4;
    const int cbase = n0 + (wave_ & 1) * WN + (lane_ & 15);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                int m = rbase + i * 16 + r, n = cbase + j * 16;
                if (m >= a.M || n >= a.N) continue;
                if (slab) slab[(size_t)m * a.N + n] = acc[i][j][r];
                else epilogue_store<EPI, OUT_BF16>(a, m, n, alpha * acc[i][j][r]);
            }
}

// ------------------------------------------------------------------------------------------
// Pipelined variant: NS-stage LDS ring filled by LDS-DMA (GldsTile, tiles.h), counted waits, raw barrier.
// The body takes its workgroup index `bid` (the tile, before the XCD remap) so that a grouped launch can run
// several problems in one grid (gemm_dw2_kernel).
// IL = 1: the next stage's DMA pieces are issued between this step's fragment reads and MFMAs (half after the
// first K half's reads, half after the second's) instead of all of them right after the barrier, so the wave's
// LDS reads are in flight while the pieces queue at the texture unit and the fill overlaps the MFMAs.
// MF = 32: v_mfma_f32_32x32x16_bf16 on 32x32 fragments (tile images in swizzle family 1, tiles.h frag32), half the
// MFMA instructions of the 16x16x32 form for the same wave tile; no in-loop bias sums, staged epilogue only.
template <int BM, int BN, int WGM, int WGN, int NS, bool A_KM, bool B_KN, int EPI, bool OUT_BF16, bool DIRECT = false,
          int IL = 0, int MF = 16>
__device__ __forceinline__ void gemm_pipe_body(const GemmArgs& a, const int bid) {
    static_assert(MF == 16 || (MF == 32 && !DIRECT && IL == 0), "32x32x16 MFMA: staged epilogue, no interleaved issue");
    constexpr int SW = MF == 32 ? 1 : 0;
    constexpr int NW = WGM * WGN;
    constexpr int WM = BM / WGM, WN = BN / WGN;
    constexpr int FM = WM / MF, FN = WN / MF;
    static_assert(FM >= 1 && FN >= 1 && FM * MF == WM && FN * MF == WN, "wave tile must be a multiple of the MFMA tile");
    constexpr int A_BYTES = BM * GEMM_BK * 2, B_BYTES = BN * GEMM_BK * 2;
    constexpr int STAGE = A_BYTES + B_BYTES;
    constexpr int LPS = GldsTile<BM, A_KM, NW>::PER_WAVE + GldsTile<BN, B_KN, NW>::PER_WAVE;  // vmcnt per stage
    static_assert(NS >= 2 && NS <= 8 && (NS - 2) * LPS <= 63, "2..8 stages, vmcnt <= 63");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int nwg = a.tiles_m * a.tiles_n;
    // K slice zs: blockIdx.z, or (xcd_split) the XCD the workgroup runs on — workgroup b goes to XCD b % 8,
    // so the tiles of one slice share that XCD's L2 and each operand slice is fetched once
    const int zs = a.xcd_split ? (bid & 7) : (int)blockIdx.z;
    const int id = a.xcd_split ? (bid >> 3) : xcd_remap(bid, nwg);
    if (id >= nwg) return;
    int tm, tn;
    if (a.sweep_m) { tm = id % a.tiles_m; tn = id / a.tiles_m; }
    else { tn = id % a.tiles_n; tm = id / a.tiles_n; }
    const int m0 = tm * BM, n0 = tn * BN;
    const int kbeg = zs * a.k_per_split;
    const int kend = min(a.K, kbeg + a.k_per_split);
    const int nk = (kend - kbeg) / GEMM_BK;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave / WGN, wn = wave % WGN;

    using AccT = std::conditional_t<MF == 32, f32x16, f32x4>;
    AccT acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = AccT{};

    auto issue_stage = [&](int kt) {
        char* st = smem + (kt % NS) * STAGE;
        const int k0 = kbeg + kt * GEMM_BK;
        GldsTile<BM, A_KM, NW, SW>::issue(st, a.A, a.lda, m0, a.M, k0, wave);
        GldsTile<BN, B_KN, NW, SW>::issue(st + A_BYTES, a.B, a.ldb, n0, a.N, k0, wave);
    };
    constexpr int PA = GldsTile<BM, A_KM, NW>::PER_WAVE;
    auto issue_piece = [&](int kt, int p) {  // piece p of this wave's LPS pieces of stage kt (A's first)
        char* st = smem + (kt % NS) * STAGE;
        const int k0 = kbeg + kt * GEMM_BK;
        if (p < PA) GldsTile<BM, A_KM, NW, SW>::issue_piece(st, a.A, a.lda, m0, a.M, k0, wave, p);
        else GldsTile<BN, B_KN, NW, SW>::issue_piece(st + A_BYTES, a.B, a.ldb, n0, a.N, k0, wave, p - PA);
    };
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
        if (s < nk) issue_stage(s);

    EpiPre<EPI, BM, BN, WGM, 64 * NW> pre;
    if constexpr (!DIRECT) pre.load(a, m0, n0);
    FragReader<BM, A_KM, SW> la;
    FragReader<BN, B_KN, SW> lb;
    // weight-gradient bias: the waves of the last tile row with wm == 0 also sum the B (dY) fragments they
    // read: lane l holds B[k = 8(l>>4) .. +7][n = l & 15] of each 16-column fragment (16x16x32 form only)
    constexpr bool CS = A_KM && B_KN && EPI == ERGM_EPI_NONE && !OUT_BF16 && MF == 16;
    const bool do_cs = CS && a.colsum && tm == a.tiles_m - 1 && wm == 0;
    float cs[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) cs[j] = 0.f;
    // two copies of the main loop: only the summing waves carry the dot products (a runtime flag inside
    // one loop made the compiler unswitch it and raised the register count for every tile)
    auto main_loop = [&](auto sum_tag) {
        constexpr bool SUM = decltype(sum_tag)::value;
        for (int kt = 0; kt < nk; ++kt) {
            // stages this wave issued after kt: min(NS-2, nk-1-kt); wait until stage kt has landed
            const int after = min(NS - 2, nk - 1 - kt);
            wait_stages<LPS, NS - 2>(after);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the slot to refill are done
            __builtin_amdgcn_s_barrier();
            const bool refill = kt + NS - 1 < nk;
            if (!IL && refill) issue_stage(kt + NS - 1);
            const char* st = smem + (kt % NS) * STAGE;
            if constexpr (MF == 32) {
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    bf16x8 fa[FM], fb[FN];
#pragma unroll
                    for (int i = 0; i < FM; ++i) fa[i] = la.frag32(st, wm * WM + i * 32, kk);
#pragma unroll
                    for (int j = 0; j < FN; ++j) fb[j] = lb.frag32(st + A_BYTES, wn * WN + j * 32, kk);
#pragma unroll
                    for (int i = 0; i < FM; ++i)
#pragma unroll
                        for (int j = 0; j < FN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
                }
            } else {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                bf16x8 fa[FM], fb[FN];
#pragma unroll
                for (int i = 0; i < FM; ++i) fa[i] = la.frag(st, wm * WM + i * 16, ks);
#pragma unroll
                for (int j = 0; j < FN; ++j) fb[j] = lb.frag(st + A_BYTES, wn * WN + j * 16, ks);
                if constexpr (IL != 0) {
                    constexpr int H = (LPS + 1) / 2;
                    if (refill) {
#pragma unroll
                        for (int p = ks * H; p < (ks + 1) * H && p < LPS; ++p) issue_piece(kt + NS - 1, p);
                    }
                }
                if constexpr (SUM) {  // packed bf16 dot products against ones: 4 v_dot2 per fragment
                    const bf16x2 one = {(__bf16)1.0f, (__bf16)1.0f};
#pragma unroll
                    for (int j = 0; j < FN; ++j) {
                        float t = cs[j];
                        t = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(fb[j], fb[j], 0, 1), one, t, false);
                        t = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(fb[j], fb[j], 2, 3), one, t, false);
                        t = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(fb[j], fb[j], 4, 5), one, t, false);
                        t = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(fb[j], fb[j], 6, 7), one, t, false);
                        cs[j] = t;
                    }
                }
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j) {
                        if constexpr (DIRECT)  // Cᵀ fragments (store_tile_direct)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
                        else
                            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
                    }
            }
            }
        }
    };
    if constexpr (CS) {
        if (do_cs) main_loop(std::true_type{});
        else main_loop(std::false_type{});
    } else {
        main_loop(std::false_type{});
    }
    float alpha = a.alpha;
    if (a.alpha_dev) alpha *= *a.alpha_dev;
    if constexpr (CS) {
        if (do_cs) {  // sum the four 16-lane rows (k groups), lane position (column) preserved
            const int lane = threadIdx.x & 63;
            float* dst = a.slab ? a.colsum_part + (size_t)zs * a.N : a.colsum;
            const float sc = a.slab ? 1.0f : alpha;  // split-K: the reduce kernel applies alpha
#pragma unroll
            for (int j = 0; j < FN; ++j) {
                float v = cs[j];
                auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
                v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
                r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
                v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
                const int n = n0 + wn * WN + j * 16 + lane;
                if (lane < 16 && n < a.N) dst[n] = sc * v;
            }
        }
    }
    if constexpr (DIRECT) {
        store_tile_direct<WGN, EPI, OUT_BF16, FM, FN, WM, WN>(a, acc, m0, n0, alpha);
    } else {
        float* slab = a.slab ? a.slab + (size_t)zs * a.M * a.N : nullptr;
        store_tile<BM, BN, WGM, WGN, EPI, OUT_BF16, FM, FN, 64 * WGM * WGN, false, false, MF>(a, smem, acc, m0, n0, alpha,
                                                                                           slab, &pre);
    }
}

// Intra-workgroup split-K (KS2): 2·WGM·WGN waves in two groups of WGM×WGN.  Each barrier interval consumes a
// PAIR of 64-deep K steps — group 0 the first, group 1 the second, on the same output tile — and refills one pair
// slot; every wave of the workgroup issues its share of the DMA pieces, so a tile has twice the issuers of the
// 4-wave kernel (the LDS-DMA fill, not the MFMA, bounds these tiles: ~25 GB/s landing per issuing wave) and half
// the serial K steps.  At the end group 1's accumulators go through LDS into group 0's (acc_even + acc_odd per
// element, fixed order: deterministic), then the staged epilogue with all waves copying out.  An odd K-step count
// ends with a half-empty pair whose second half re-loads the first half's K step (so every pair issues the same
// number of pieces and the counted waits stay exact) and group 1 skips it.
template <int BM, int BN, int WGM, int WGN, int NS, bool A_KM, bool B_KN, int EPI, bool OUT_BF16>
__device__ __forceinline__ void gemm_ks2_body(const GemmArgs& a, const int bid) {
    constexpr int NW = WGM * WGN;  // waves per group
    constexpr int NT = 2 * NW;     // waves per workgroup
    constexpr int WM = BM / WGM, WN = BN / WGN;
    constexpr int FM = WM / 16, FN = WN / 16;
    constexpr int A_BYTES = BM * GEMM_BK * 2, B_BYTES = BN * GEMM_BK * 2;
    constexpr int HALF = A_BYTES + B_BYTES;  // one 64-deep K step
    constexpr int STAGE = 2 * HALF;          // a pair
    constexpr int LPS = 2 * (GldsTile<BM, A_KM, NT>::PER_WAVE + GldsTile<BN, B_KN, NT>::PER_WAVE);
    static_assert(NS >= 2 && NS <= 8 && (NS - 2) * LPS <= 63, "2..8 stages, vmcnt <= 63");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int nwg = a.tiles_m * a.tiles_n;
    const int zs = (int)blockIdx.z;
    const int id = xcd_remap(bid, nwg);
    if (id >= nwg) return;
    int tm, tn;
    if (a.sweep_m) { tm = id % a.tiles_m; tn = id / a.tiles_m; }
    else { tn = id % a.tiles_n; tm = id / a.tiles_n; }
    const int m0 = tm * BM, n0 = tn * BN;
    const int kbeg = zs * a.k_per_split;
    const int kend = min(a.K, kbeg + a.k_per_split);
    const int nk = (kend - kbeg) / GEMM_BK;
    const int npair = (nk + 1) / 2;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int grp = wave / NW, wv = wave % NW;
    const int wm = wv / WGN, wn = wv % WGN;

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto issue_pair = [&](int kp) {
        char* st = smem + (kp % NS) * STAGE;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int kt = min(2 * kp + h, nk - 1);  // the odd tail's second half re-loads the last step
            const int k0 = kbeg + kt * GEMM_BK;
            GldsTile<BM, A_KM, NT>::issue(st + h * HALF, a.A, a.lda, m0, a.M, k0, wave);
            GldsTile<BN, B_KN, NT>::issue(st + h * HALF + A_BYTES, a.B, a.ldb, n0, a.N, k0, wave);
        }
    };
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
        if (s < npair) issue_pair(s);

    FragReader<BM, A_KM> la;
    FragReader<BN, B_KN> lb;
    for (int kp = 0; kp < npair; ++kp) {
        wait_stages<LPS, NS - 2>(min(NS - 2, npair - 1 - kp));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (kp + NS - 1 < npair) issue_pair(kp + NS - 1);
        if (2 * kp + grp < nk) {
            const char* st = smem + (kp % NS) * STAGE + grp * HALF;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                bf16x8 fa[FM], fb[FN];
#pragma unroll
                for (int i = 0; i < FM; ++i) fa[i] = la.frag(st, wm * WM + i * 16, ks);
#pragma unroll
                for (int j = 0; j < FN; ++j) fb[j] = lb.frag(st + A_BYTES, wn * WN + j * 16, ks);
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
            }
        }
    }
    // group 1's partial tile into group 0's through LDS ([fragment register][lane] floats: conflict-free)
    const int lane = threadIdx.x & 63;
    float* red = reinterpret_cast<float*>(smem);
    __syncthreads();
    if (grp == 1) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) red[(((wv * FM + i) * FN + j) * 4 + r) * 64 + lane] = acc[i][j][r];
    }
    __syncthreads();
    if (grp == 0) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[i][j][r] += red[(((wv * FM + i) * FN + j) * 4 + r) * 64 + lane];
    }
    float alpha = a.alpha;
    if (a.alpha_dev) alpha *= *a.alpha_dev;
    float* slab = a.slab ? a.slab + (size_t)zs * a.M * a.N : nullptr;
    // store_tile opens with a barrier (group 0's reads of `red` are done before the staging reuse); only the
    // group-0 waves hold accumulators, every wave helps with the copy-out
    store_tile<BM, BN, WGM, WGN, EPI, OUT_BF16, FM, FN, 64 * NT>(a, smem, acc, m0, n0, alpha, slab);
}

template <int BM, int BN, int WGM, int WGN, int NS, bool A_KM, bool B_KN, int EPI, bool OUT_BF16>
__global__ __launch_bounds__(128 * WGM * WGN) void gemm_ks2_kernel(GemmArgs a) {
    gemm_ks2_body<BM, BN, WGM, WGN, NS, A_KM, B_KN, EPI, OUT_BF16>(a, blockIdx.x);
}

template <int BM, int BN, int WGM, int WGN, int NS, bool A_KM, bool B_KN, int EPI, bool OUT_BF16, bool DIRECT = false,
          int IL = 0, int MF = 16>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm_pipe_kernel(GemmArgs a) {
    gemm_pipe_body<BM, BN, WGM, WGN, NS, A_KM, B_KN, EPI, OUT_BF16, DIRECT, IL, MF>(a, blockIdx.x);
}

// Two weight-gradient GEMMs (KM x KN, f32 out, no split) in ONE launch: workgroups [0, b1) run problem 0
// (those past its tile count exit), [b1, b1 + tiles of problem 1) run problem 1.  A block's dW GEMMs
// are issued in pairs on the side stream, and each alone has 126-168 tiles — fewer than the 256 CUs —
// so as two launches the pair's second half waits for the first to drain; as one grid both fill the chip
// together.  b1 is a multiple of 8, so the XCD remap of problem 1 sees the same block -> XCD pattern.
struct GemmArgs2 {
    GemmArgs a[2];
    int b1;
};
template <int BM, int BN, int WGM, int WGN, int NS, int IL = 0, int EPI = ERGM_EPI_NONE, int MF = 16>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm_dw2_kernel(GemmArgs2 g) {
    const int b = blockIdx.x;
    const int pr = b < g.b1 ? 0 : 1;
    const int bb = pr == 0 ? b : b - g.b1;
    if (pr == 0 && b >= g.a[0].tiles_m * g.a[0].tiles_n) return;
    gemm_pipe_body<BM, BN, WGM, WGN, NS, true, true, EPI, false, false, IL, MF>(g.a[pr], bb);
}

// Warp-specialised variant: NP producer waves only issue the LDS-DMA fills, the WGM x WGN consumer
// waves only read fragments and run MFMAs.  In gemm_pipe_kernel every wave issues its share of the
// DMAs and then computes, so the DMA issue time (the per-CU fill path sustains ~100-120 GB/s, about
// 150 ns per 16 KiB stage: tools/fill_bench.hip) adds to the compute time of every K step; split
// across waves it overlaps instead, and a K step costs max(fill, compute).  One s_barrier per K step:
// producers arrive once their DMAs of stage kt have landed, consumers once they are done reading
// the slot the next fill overwrites.
template <int BM, int BN, int WGM, int WGN, int NP, int NS, bool A_KM, bool B_KN, int EPI, bool OUT_BF16>
__global__ __launch_bounds__(64 * (WGM * WGN + NP)) void gemm_ws_kernel(GemmArgs a) {
    constexpr int NC = WGM * WGN;
    constexpr int WM = BM / WGM, WN = BN / WGN;
    constexpr int FM = WM / 16, FN = WN / 16;
    constexpr int A_BYTES = BM * GEMM_BK * 2, B_BYTES = BN * GEMM_BK * 2;
    constexpr int STAGE = A_BYTES + B_BYTES;
    constexpr int LPS = GldsTile<BM, A_KM, NP>::PER_WAVE + GldsTile<BN, B_KN, NP>::PER_WAVE;  // per producer
    static_assert(NS >= 2 && NS <= 8 && (NS - 2) * LPS <= 63, "2..8 stages, vmcnt <= 63");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int nwg = a.tiles_m * a.tiles_n;
    const int id = xcd_remap(blockIdx.x, nwg);
    int tm, tn;
    if (a.sweep_m) { tm = id % a.tiles_m; tn = id / a.tiles_m; }
    else { tn = id % a.tiles_n; tm = id / a.tiles_n; }
    const int m0 = tm * BM, n0 = tn * BN;
    const int kbeg = blockIdx.z * a.k_per_split;
    const int kend = min(a.K, kbeg + a.k_per_split);
    const int nk = (kend - kbeg) / GEMM_BK;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool producer = wave >= NC;
    const int pw = wave - NC;
    const int wm = wave / WGN, wn = wave % WGN;

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto issue_stage = [&](int kt) {
        char* st = smem + (kt % NS) * STAGE;
        const int k0 = kbeg + kt * GEMM_BK;
        GldsTile<BM, A_KM, NP>::issue(st, a.A, a.lda, m0, a.M, k0, pw);
        GldsTile<BN, B_KN, NP>::issue(st + A_BYTES, a.B, a.ldb, n0, a.N, k0, pw);
    };
    if (producer) {
#pragma unroll
        for (int s = 0; s < NS - 1; ++s)
            if (s < nk) issue_stage(s);
    }
    FragReader<BM, A_KM> la;
    FragReader<BN, B_KN> lb;
    for (int kt = 0; kt < nk; ++kt) {
        if (producer) wait_stages<LPS, NS - 2>(min(NS - 2, nk - 1 - kt));  // stage kt landed
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");         // reads of slot kt-1 done
        __builtin_amdgcn_s_barrier();
        if (producer) {
            if (kt + NS - 1 < nk) issue_stage(kt + NS - 1);
        } else {
            const char* st = smem + (kt % NS) * STAGE;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                bf16x8 fa[FM], fb[FN];
#pragma unroll
                for (int i = 0; i < FM; ++i) fa[i] = la.frag(st, wm * WM + i * 16, ks);
#pragma unroll
                for (int j = 0; j < FN; ++j) fb[j] = lb.frag(st + A_BYTES, wn * WN + j * 16, ks);
#pragma unroll
                for (int i = 0; i < FM; ++i)
#pragma unroll
                    for (int j = 0; j < FN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
            }
        }
    }
    float alpha = a.alpha;
    if (a.alpha_dev) alpha *= *a.alpha_dev;
    float* slab = a.slab ? a.slab + (size_t)blockIdx.z * a.M * a.N : nullptr;
    // store_tile opens with a barrier: the last stage's reads are done before the staging reuse
    store_tile<BM, BN, WGM, WGN, EPI, OUT_BF16, FM, FN, 64 * (NC + NP)>(a, smem, acc, m0, n0, alpha, slab);
}

// ------------------------------------------------------------------------------------------
// fp8 (OCP e4m3fn) GEMM for the config-5 forward: A [M][K] and B [N][K] bytes (k contiguous: the
// activations as produced, the weights stored transposed by ergm_quant_weight_fp8), one
// v_mfma_scale_f32_16x16x128_f8f6f4 per 16x16 output fragment per 128-deep K step with unit block
// scales (e8m0 127 = 2^0) — the block-scaled instruction runs e4m3 at twice the bf16 MFMA rate, the
// unscaled fp8 forms only at the bf16 rate (MI355X_MICROARCH.md, matrix cores).  Dequantisation by the
// per-row scale of A and per-column scale of B happens once, in the epilogue.
// A 128-byte K step has the byte layout of the bf16 kernels' 64-element step, so the same LDS-DMA
// ring (GldsTile on a 2-byte view) and XOR swizzle stage it; lane l reads the 32 bytes of row l&15 at
// k-offset 32·(l>>4) (two 16-B chunks).
typedef __attribute__((ext_vector_type(8))) int i32x8;

template <int ROWS>
__device__ __forceinline__ i32x8 frag_f8(const char* lds, int ro) {
    const int lane = threadIdx.x & 63;
    const int row = ro + (lane & 15), g = lane >> 4;
    const char* base = lds + row * 128;
    const int sw = swz_row(row);
    const uint4 lo = *reinterpret_cast<const uint4*>(base + (((2 * g) ^ sw) << 4));
    const uint4 hi = *reinterpret_cast<const uint4*>(base + (((2 * g + 1) ^ sw) << 4));
    return i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
}

// MX operand fragment: the block-scaled 16x16x128 MFMA reads a lane's 8 dwords as K positions {16g..16g+15} (dwords
// 0-3) and {64+16g..64+16g+15} (dwords 4-7), g = lane >> 4, and applies the scale of lane group G to K positions
// [32G, 32G+32) (measured: tools/mx_debug2.py).  Reading 16-B chunks g and g+4 of the row makes those positions
// the row's memory order, so lane group G's scale byte is that of the 128-deep step's 32-element block G.
__device__ __forceinline__ i32x8 frag_mx(const char* lds, int ro) {
    const int lane = threadIdx.x & 63;
    const int row = ro + (lane & 15), g = lane >> 4;
    const char* base = lds + row * 128;
    const int sw = swz_row(row);
    const uint4 lo = *reinterpret_cast<const uint4*>(base + ((g ^ sw) << 4));
    const uint4 hi = *reinterpret_cast<const uint4*>(base + (((g + 4) ^ sw) << 4));
    return i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
}

template <int BM, int BN, int WGM, int WGN, int NS, int EPI, bool OUT_BF16>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm_f8_kernel(GemmArgs a) {
    constexpr int NW = WGM * WGN;
    constexpr int WM = BM / WGM, WN = BN / WGN;
    constexpr int FM = WM / 16, FN = WN / 16;
    constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128;
    constexpr int STAGE = A_BYTES + B_BYTES;
    constexpr int LPS = GldsTile<BM, false, NW>::PER_WAVE + GldsTile<BN, false, NW>::PER_WAVE;
    static_assert(NS >= 2 && NS <= 8 && (NS - 2) * LPS <= 63, "2..8 stages, vmcnt <= 63");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int nwg = a.tiles_m * a.tiles_n;
    const int id = xcd_remap(blockIdx.x, nwg);
    int tm, tn;
    if (a.sweep_m) { tm = id % a.tiles_m; tn = id / a.tiles_m; }
    else { tn = id % a.tiles_n; tm = id / a.tiles_n; }
    const int m0 = tm * BM, n0 = tn * BN;
    const int nk = a.K / 128;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave / WGN, wn = wave % WGN;
    // 2-byte views: a 128-byte K step is "64 elements" of the bf16 staging code
    const __bf16* A2 = a.A;
    const __bf16* B2 = a.B;
    const int lda2 = a.lda / 2, ldb2 = a.ldb / 2;

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto issue_stage = [&](int kt) {
        char* st = smem + (kt % NS) * STAGE;
        const int k0 = kt * 64;
        GldsTile<BM, false, NW>::issue(st, A2, lda2, m0, a.M, k0, wave);
        GldsTile<BN, false, NW>::issue(st + A_BYTES, B2, ldb2, n0, a.N, k0, wave);
    };
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
        if (s < nk) issue_stage(s);
    for (int kt = 0; kt < nk; ++kt) {
        wait_stages<LPS, NS - 2>(min(NS - 2, nk - 1 - kt));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (kt + NS - 1 < nk) issue_stage(kt + NS - 1);
        const char* st = smem + (kt % NS) * STAGE;
        i32x8 fa[FM], fb[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) fa[i] = frag_f8<BM>(st, wm * WM + i * 16);
#pragma unroll
        for (int j = 0; j < FN; ++j) fb[j] = frag_f8<BN>(st + A_BYTES, wn * WN + j * 16);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fa[i], fb[j], acc[i][j], 0, 0, 0, 127, 0,
                                                                              127);
    }
    float alpha = a.alpha;
    if (a.alpha_dev) alpha *= *a.alpha_dev;
    store_tile<BM, BN, WGM, WGN, EPI, OUT_BF16, FM, FN, 64 * NW, true>(a, smem, acc, m0, n0, alpha, nullptr);
}

// MX-fp8 GEMM (OCP microscaling, config 5's forward): A [M][K] and B [N][K] e4m3 bytes (k contiguous) with an
// e8m0 scale per 32-element K block of every row of A (a_mx, pitch ld_sa rows) and of B (b_mx, pitch ld_sb rows) in
// the K-step-major layout of common.h mx_sidx, consumed by the MFMA itself: v_mfma_scale_f32_16x16x128_f8f6f4
// applies lane group G's scale byte to K [32G, 32G+32) of the 128-deep step (frag_mx).  The scales of a stage
// (4 bytes per row: the 4 blocks of a 128-deep step, 256 contiguous bytes per 64 rows) ride in the same LDS ring
// behind the operand tiles, filled by 4-byte-per-lane
// LDS-DMA (one 64-row piece per wave-instruction; with more waves than pieces the spare waves re-issue piece
// 0, identical bytes, so every wave issues the same count and the counted waits stay exact).  No
// per-row / per-column dequantisation in the epilogue; QMX: the epilogue also writes an MX copy of its bf16
// output (the next fp8 GEMM's A operand).
template <int BM, int BN, int WGM, int WGN, int NS, int EPI, bool OUT_BF16, bool QMX>
__global__ __launch_bounds__(64 * WGM * WGN) void gemm_mx_kernel(GemmArgs a) {
    constexpr int NW = WGM * WGN;
    constexpr int WM = BM / WGM, WN = BN / WGN;
    constexpr int FM = WM / 16, FN = WN / 16;
    constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128;
    constexpr int SC_BYTES = (BM + BN) * 4;
    constexpr int STAGE = A_BYTES + B_BYTES + SC_BYTES;
    constexpr int NSP = (BM + BN) / 64;                // scale pieces per stage (64 rows each)
    constexpr int SPW = (NSP + NW - 1) / NW;           // per wave
    constexpr int LPS = GldsTile<BM, false, NW>::PER_WAVE + GldsTile<BN, false, NW>::PER_WAVE + SPW;
    static_assert(NS >= 2 && NS <= 8 && (NS - 2) * LPS <= 63, "2..8 stages, vmcnt <= 63");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int nwg = a.tiles_m * a.tiles_n;
    const int id = xcd_remap(blockIdx.x, nwg);
    int tm, tn;
    if (a.sweep_m) { tm = id % a.tiles_m; tn = id / a.tiles_m; }
    else { tn = id % a.tiles_n; tm = id / a.tiles_n; }
    const int m0 = tm * BM, n0 = tn * BN;
    const int nk = a.K / 128;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int wm = wave / WGN, wn = wave % WGN;
    const __bf16* A2 = a.A;
    const __bf16* B2 = a.B;
    const int lda2 = a.lda / 2, ldb2 = a.ldb / 2;

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto issue_stage = [&](int kt) {
        char* st = smem + (kt % NS) * STAGE;
        const int k0 = kt * 64;
        GldsTile<BM, false, NW>::issue(st, A2, lda2, m0, a.M, k0, wave);
        GldsTile<BN, false, NW>::issue(st + A_BYTES, B2, ldb2, n0, a.N, k0, wave);
#pragma unroll
        for (int i = 0; i < SPW; ++i) {
            int p = wave + i * NW;
            if (p >= NSP) p = 0;  // spare wave: re-issue piece 0 (same bytes, same destination)
            const bool isb = p * 64 >= BM;
            const int r = (isb ? p * 64 - BM : p * 64) + lane;
            const uint8_t* src = isb ? a.b_mx + ((size_t)kt * a.ld_sb + min(n0 + r, a.N - 1)) * 4
                                     : a.a_mx + ((size_t)kt * a.ld_sa + min(m0 + r, a.M - 1)) * 4;
            glds4(src, __builtin_amdgcn_readfirstlane(lds_addr_of(st + A_BYTES + B_BYTES + p * 256)));
        }
    };
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
        if (s < nk) issue_stage(s);
    const int g = lane >> 4, r16 = lane & 15;
    for (int kt = 0; kt < nk; ++kt) {
        wait_stages<LPS, NS - 2>(min(NS - 2, nk - 1 - kt));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (kt + NS - 1 < nk) issue_stage(kt + NS - 1);
        const char* st = smem + (kt % NS) * STAGE;
        const uint32_t* sc = reinterpret_cast<const uint32_t*>(st + A_BYTES + B_BYTES);
        i32x8 fa[FM], fb[FN];
        int sa[FM], sb[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
            fa[i] = frag_mx(st, wm * WM + i * 16);
            sa[i] = (int)(sc[wm * WM + i * 16 + r16] >> (8 * g));
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) {
            fb[j] = frag_mx(st + A_BYTES, wn * WN + j * 16);
            sb[j] = (int)(sc[BM + wn * WN + j * 16 + r16] >> (8 * g));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fa[i], fb[j], acc[i][j], 0, 0, 0, sa[i], 0,
                                                                              sb[j]);
    }
    float alpha = a.alpha;
    if (a.alpha_dev) alpha *= *a.alpha_dev;
    store_tile<BM, BN, WGM, WGN, EPI, OUT_BF16, FM, FN, 64 * NW, false, QMX>(a, smem, acc, m0, n0, alpha, nullptr);
}

// split-K combine: C = epilogue(alpha * Σ_z slab[z]) in z order (deterministic).
template <int EPI, bool OUT_BF16>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmArgs a, int splits) {
    size_t total = (size_t)a.M * a.N;
    float alpha = a.alpha;
    if (a.alpha_dev) alpha *= *a.alpha_dev;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        float s = 0.f;
        for (int z = 0; z < splits; ++z) s += a.slab[(size_t)z * total + i];
        int m = (int)(i / a.N), n = (int)(i % a.N);
        epilogue_store<EPI, OUT_BF16>(a, m, n, alpha * s);
    }
    if (a.colsum && a.colsum_part) {  // the weight-gradient bias: per-split column sums, in z order
        for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < a.N; n += gridDim.x * blockDim.x) {
            float s = 0.f;
            for (int z = 0; z < splits; ++z) s += a.colsum_part[(size_t)z * a.N + n];
            a.colsum[n] = alpha * s;
        }
    }
}

// Bias gradient for the kernels without the in-GEMM column sum (register-staged / warp-specialised
// configurations): out[n] = alpha·Σ_k B[k][n], B = [K][ldb] bf16; 4 row groups per column, fixed-order
// combine (deterministic).
__global__ __launch_bounds__(256) void colsum_kn_kernel(const __bf16* __restrict__ B, int K, int N, int ldb,
                                                        float alpha, const float* alpha_dev, float* __restrict__ out) {
    __shared__ float part[4][64];
    const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int n = blockIdx.x * 64 + c;
    float s = 0.f;
    if (n < N)
        for (int k = g; k < K; k += 4) s += bf2f(B[(size_t)k * ldb + n]);
    part[g][c] = s;
    __syncthreads();
    if (g == 0 && n < N) {
        const float al = alpha_dev ? alpha * *alpha_dev : alpha;
        out[n] = al * (((part[0][c] + part[1][c]) + part[2][c]) + part[3][c]);
    }
}

// ------------------------------------------------------------------------------------------
// host dispatch
// ------------------------------------------------------------------------------------------
// Pipelined-kernel configurations (tile BM x BN, wave grid WGM x WGN, LDS stages NS).
struct PipeCfg {
    int bm, bn, wgm, wgn, ns;
    int np = 0;      // > 0: warp-specialised kernel with np producer waves
    bool direct = false;  // LDS-free epilogue (store_tile_direct); split-K partials keep the staged one
    int il = 0;      // 1: next-stage DMA pieces interleaved with the step's reads / MFMAs (gemm_pipe_body IL)
    int ks = 1;      // 2: intra-workgroup split-K over two wave groups (gemm_ks2_body; ns counts K-step pairs)
    int mf = 16;     // 32: v_mfma_f32_32x32x16_bf16 on 32x32 fragments (gemm_pipe_body MF; pipelined kernel only)
};
static constexpr PipeCfg kCfgs[] = {
    {64, 64, 2, 2, 4},     // 0
    {128, 128, 2, 2, 3},   // 1
    {128, 128, 2, 2, 2},   // 2
    {128, 128, 2, 4, 3},   // 3  8 waves (64x32 each)
    {256, 128, 4, 2, 3},   // 4  8 waves (64x64 each)
    {128, 256, 2, 4, 3},   // 5  8 waves (64x64 each)
    {256, 256, 4, 2, 2},   // 6  8 waves (64x128 each)
    {128, 64, 2, 2, 4},    // 7
    {64, 128, 2, 2, 4},    // 8
    {256, 128, 4, 2, 2},   // 9
    {128, 128, 4, 2, 2},   // 10 8 waves (32x64 each)
    {64, 64, 2, 2, 8},     // 11 deep: 7 stages (112 KiB) in flight
    {128, 64, 2, 2, 6},    // 12
    {64, 128, 2, 2, 6},    // 13
    {128, 128, 2, 2, 4},   // 14
    {128, 128, 4, 2, 4},   // 15 8 waves
    // warp-specialised (consumer grid + 4 producer waves)
    {64, 64, 2, 2, 4, 4},    // 16
    {64, 64, 2, 2, 6, 4},    // 17
    {128, 64, 2, 2, 5, 4},   // 18
    {64, 128, 2, 2, 5, 4},   // 19
    {128, 128, 2, 2, 4, 4},  // 20
    {128, 128, 4, 2, 4, 4},  // 21
    // LDS-free epilogue variants
    {256, 256, 4, 2, 2, 0, true},  // 22 the LM-head tile of cfg 6
    {128, 128, 4, 2, 2, 0, true},  // 23 cfg 10
    {128, 128, 2, 2, 2, 0, true},  // 24 cfg 2
    // interleaved DMA issue (IL) variants of the automatic plans' configurations
    {64, 64, 2, 2, 4, 0, false, 1},     // 25 cfg 0
    {128, 128, 2, 2, 2, 0, false, 1},   // 26 cfg 2
    {128, 128, 2, 4, 3, 0, false, 1},   // 27 cfg 3
    {256, 256, 4, 2, 2, 0, false, 1},   // 28 cfg 6
    {64, 128, 2, 2, 4, 0, false, 1},    // 29 cfg 8
    {128, 128, 4, 2, 2, 0, false, 1},   // 30 cfg 10
    {128, 128, 2, 2, 4, 0, false, 1},   // 31 cfg 14
    {128, 128, 2, 2, 3, 0, false, 1},   // 32 cfg 1
    // intra-workgroup split-K (KS2, 8 waves as two K groups of 2x2; ns = K-step PAIRS in the ring)
    {64, 64, 2, 2, 2, 0, false, 0, 2},    // 33  64 KB
    {64, 64, 2, 2, 3, 0, false, 0, 2},    // 34  96 KB
    {64, 128, 2, 2, 2, 0, false, 0, 2},   // 35  96 KB
    {128, 64, 2, 2, 2, 0, false, 0, 2},   // 36  96 KB
    {128, 128, 2, 2, 2, 0, false, 0, 2},  // 37 128 KB
    // v_mfma_f32_32x32x16_bf16 twins of the pipelined configurations (round 6, verdict r05 #2)
    {64, 64, 2, 2, 4, 0, false, 0, 1, 32},     // 38 cfg 0
    {128, 128, 2, 2, 2, 0, false, 0, 1, 32},   // 39 cfg 2
    {128, 128, 4, 2, 2, 0, false, 0, 1, 32},   // 40 cfg 10 (32 x 64 per wave)
    {128, 64, 2, 2, 4, 0, false, 0, 1, 32},    // 41 cfg 7
    {64, 128, 2, 2, 4, 0, false, 0, 1, 32},    // 42 cfg 8
    {128, 128, 4, 2, 4, 0, false, 0, 1, 32},   // 43 cfg 15
    {256, 256, 4, 2, 2, 0, false, 0, 1, 32},   // 44 cfg 6 (64 x 128 per wave)
    {64, 64, 2, 2, 8, 0, false, 0, 1, 32},     // 45 cfg 11
    {128, 128, 2, 4, 3, 0, false, 0, 1, 32},   // 46 cfg 3 (64 x 32 per wave)
};
static constexpr int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);

static thread_local int g_force_cfg = -1;    // ergm_gemm_tune: -1 = automatic
static thread_local int g_force_split = 0;

struct GemmPlan {
    int cfg;    // index into kCfgs, or -1: register-staged fallback kernel
    int bm, bn;
    int split, kps;
    bool xcd = false;  // split 8 with one K slice per XCD (GemmArgs::xcd_split)
};

static long tiles_of(int M, int N, int bm, int bn) { return (long)cdiv(M, bm) * cdiv(N, bn); }

// Layout / epilogue / output-type combinations instantiated for the pipelined kernels (the ones the
// training step issues); everything else runs on the register-staged kernel.
static constexpr bool combo_ok(bool akm, bool bkn, int e, bool ob) {
    return (!akm && bkn && (e == ERGM_EPI_BIAS || e == ERGM_EPI_BIAS_GELU) && ob) ||
           (!akm && bkn && e == ERGM_EPI_BIAS_RESID && !ob) || (!akm && bkn && e == ERGM_EPI_NONE && !ob) ||
           (!akm && !bkn && e == ERGM_EPI_NONE) || (!akm && !bkn && e == ERGM_EPI_GELU_BWD && ob) ||
           (akm && bkn && e == ERGM_EPI_NONE && !ob);
}

static bool pipe_ok(const ergm_gemm_desc* d) {
    // the pipelined path needs K % 64 == 0 and 16-B vector epilogue access (N, ldc, aux lds % 8)
    return d->K % GEMM_BK == 0 && d->N % 8 == 0 && d->ldc % 8 == 0 && (!d->aux || d->ld_aux % 8 == 0) &&
           (!d->aux_out || d->ld_aux_out % 8 == 0);
}

// Per-shape configuration overrides (ergm_gemm_set_override): measured in the running training step
// (tools/step_tune.py), where per-kernel isolated timings do not predict the concurrent step.  Keyed on
// (M, N, K, layouts); a small fixed table, written from the host only (plan creation / tuning).
struct GemmOverride {
    int M, N, K, al, bl, cfg, split;
};
static constexpr int kMaxOverrides = 64;
static GemmOverride g_over[kMaxOverrides];
static int g_n_over = 0;
static std::mutex g_over_mu;

// Built-in entries measured by tools/step_tune.py inside the bench step (interleaved A/B against the
// automatic choice; profiles/r01_step_tune_*.json).  Runtime overrides take precedence.
static constexpr GemmOverride kStepTuned[] = {
    // config 2 (GPT-2-small, B=16, S=128; forward GEMMs run per batch half, M = 1024)
    {3073, 768, 2048, ERGM_KM, ERGM_KN, 15, 1},  // mlp c_proj weight gradient (+ the bias row); cfg 2 until round 4's
                                                 // re-tune (profiles/r04_experiments.txt #24)
    {769, 2304, 2048, ERGM_KM, ERGM_KN, 2, 1},   // c_attn weight gradient (+ the bias row)
    {3072, 768, 2048, ERGM_KM, ERGM_KN, 2, 1},   // the same with the in-GEMM bias column sums
    {768, 2304, 2048, ERGM_KM, ERGM_KN, 2, 1},
    {1024, 2304, 768, ERGM_MK, ERGM_KN, 3, 1},   // c_attn forward
    {2048, 768, 3072, ERGM_MK, ERGM_NK, 8, 1},   // c_fc data gradient
    {2048, 768, 2304, ERGM_MK, ERGM_NK, 15, 1},  // c_attn data gradient (cfg 8 until round 4's re-tune)
    {769, 3072, 2048, ERGM_KM, ERGM_KN, 15, 1},  // c_fc weight gradient (+ the bias row; round 4)
    {769, 768, 2048, ERGM_KM, ERGM_KN, 16, 1},   // attn c_proj / q / cross c_proj weight gradients: the warp-
                                                 // specialised 64 x 64 tile, launched singly (round 5's pass over the
                                                 // KS2 / IL / warp-specialised configurations: -0.6 %, profiles/
                                                 // r05_experiments.txt #16; cfg 11 in pairs since round 4)
    {1025, 1024, 4096, ERGM_KM, ERGM_KN, 15, 1}, // GPT-2-medium attention c_proj weight gradient (C5)
    {1024, 1024, 4096, ERGM_KM, ERGM_KN, 15, 1},
    // config 5 (GPT-2-medium, B=32, T=4096) data gradients, round 5's re-tune on the current build (tools/step_tune.py
    // --config c5: 21.53 -> 21.11 ms/step in the tuner, profiles/r05_step_tune_c5.txt)
    {4096, 1024, 4096, ERGM_MK, ERGM_NK, 15, 1}, // c_fc data gradient (cfg 2 since round 1's pass 2)
    {4096, 4096, 1024, ERGM_MK, ERGM_NK, 6, 1},  // mlp c_proj data gradient (GELU' epilogue)
    {4096, 1024, 3072, ERGM_MK, ERGM_NK, 2, 1},  // c_attn data gradient
    {50304, 768, 4096, ERGM_KM, ERGM_KN, 4, 1},  // LM-head weight gradient at T = 4096 (C4)
    // config 4 (S = 512, T = 4096), round 4's re-tune (profiles/r04_step_tune_c4.txt, experiments #26)
    {4096, 3072, 768, ERGM_MK, ERGM_NK, 2, 1},   // mlp c_proj data gradient (GELU' epilogue)
    {4096, 768, 2304, ERGM_MK, ERGM_NK, 14, 1},  // c_attn data gradient
    {769, 2304, 4096, ERGM_KM, ERGM_KN, 15, 1},  // c_attn weight gradient (+ the bias row)
    {769, 768, 4096, ERGM_KM, ERGM_KN, 15, 1},   // E x E weight gradients (+ the bias row)
};

static bool find_override(const ergm_gemm_desc* d, int& cfg, int& split) {
    std::lock_guard<std::mutex> lk(g_over_mu);
    for (int i = 0; i < g_n_over; ++i) {
        const GemmOverride& o = g_over[i];
        if (o.M == d->M && o.N == d->N && o.K == d->K && o.al == d->a_layout && o.bl == d->b_layout) {
            cfg = o.cfg;
            split = o.split;
            return true;
        }
    }
    for (const GemmOverride& o : kStepTuned) {
        if (o.M == d->M && o.N == d->N && o.K == d->K && o.al == d->a_layout && o.bl == d->b_layout) {
            cfg = o.cfg;
            split = o.split;
            return true;
        }
    }
    return false;
}

// Shape trace (ergm_gemm_trace): the distinct (M, N, K, layouts) of the ergm_gemm calls since enabled.
static bool g_trace_on = false;
static int g_trace[256][5];
static int g_trace_n = 0;

static void trace_shape(const ergm_gemm_desc* d) {
    std::lock_guard<std::mutex> lk(g_over_mu);
    if (!g_trace_on) return;
    for (int i = 0; i < g_trace_n; ++i)
        if (g_trace[i][0] == d->M && g_trace[i][1] == d->N && g_trace[i][2] == d->K && g_trace[i][3] == d->a_layout &&
            g_trace[i][4] == d->b_layout)
            return;
    if (g_trace_n < 256) {
        int* t = g_trace[g_trace_n++];
        t[0] = d->M; t[1] = d->N; t[2] = d->K; t[3] = d->a_layout; t[4] = d->b_layout;
    }
}

static GemmPlan plan_gemm(const ergm_gemm_desc* d) {
    GemmPlan p;
    const int M = d->M, N = d->N, K = d->K;
    int split = 1;
    int ocfg = -1, osplit = 1;
    const bool pipe = pipe_ok(d) &&
                      combo_ok(d->a_layout == ERGM_KM, d->b_layout == ERGM_KN, d->epilogue, d->c_dtype == ERGM_BF16);
    if (pipe && g_force_cfg < 0 && d->split_k == 0 && find_override(d, ocfg, osplit)) {
        p.cfg = ocfg;
        split = osplit;
    } else if (!pipe) {
        p.cfg = -1;
        const long t128 = tiles_of(M, N, 128, 128), t64 = tiles_of(M, N, 64, 64);
        p.bm = p.bn = t128 >= 240 ? 128 : 64;
        if (p.bm == 64 && t64 < 200 && K >= 1024 && d->split_k != 1)
            split = std::max(1, std::min((int)((400 + t64 - 1) / t64), K / 512));
    } else if (g_force_cfg >= 0 && g_force_cfg < kNumCfgs) {
        p.cfg = g_force_cfg;
        split = std::max(1, g_force_split);
    } else {
        // Tile choice per shape class, from tools/gemm_tune.py on MI355X (gpurun_out/gemm_tune.json,
        // summarized in DESIGN.md): the 256x256 8-wave tile for the vocabulary-wide LM head, 8-wave
        // 128x128 (32x64 per wave, 2 stages) for mid/large activation GEMMs, 4-wave 128x128 for large
        // weight gradients (A = activations^T), deep K split 4 ways, 64x64 without split otherwise
        // (split-K's extra reduce launch cost more than it saved at these sizes).
        const long t128 = tiles_of(M, N, 128, 128);
        const bool km = d->a_layout == ERGM_KM;
        if (K >= 32768 && t128 < 240 && d->split_k != 1) {
            // contraction over the vocabulary (LM-head dX) / the stacked caption K/V at config 5: the
            // 256x256 tile, split until ~256 workgroups (c6s10 at C2: 240 workgroups, LM-head dX 195 -> 172
            // us in-step, profiles/r01_lmhead_probe.txt; c6s5 at C4, c6s4 at C5)
            p.cfg = 6;
            split = (int)std::max(1L, std::min(16L, 256 / std::max(1L, tiles_of(M, N, 256, 256))));
            // (one K slice per XCD — each operand slice fetched into one L2 once — measured slower for the LM-head
            // dX at C2 with 256x256 tiles, round 3: 200 vs 177 us in-step, and with 256x192 tiles, round 4: the
            // step +0.7 %; profiles/r04_experiments.txt #8.  GemmArgs::xcd_split keeps the kernel side of it.)
        } else if (K >= 4096 && t128 < 240 && d->split_k != 1) {
            p.cfg = 2;
            // weight gradients over T >= 4096 tokens (config 5): split only the smallest outputs
            split = km ? (t128 < 100 ? 3 : 1) : std::max(1, std::min(4, K / 1024));
        } else if (t128 >= 4000) {
            p.cfg = 6;
        } else if (t128 >= 140) {
            p.cfg = km ? 2 : (K >= 3072 ? 14 : 10);
        } else {
            p.cfg = 0;
        }
    }
    if (p.cfg >= 0) {
        p.bm = kCfgs[p.cfg].bm;
        p.bn = kCfgs[p.cfg].bn;
    }
    if (d->split_k > 1) split = d->split_k;
    int kps = cdiv(cdiv(K, split), GEMM_BK) * GEMM_BK;
    split = cdiv(K, kps);
    if (p.xcd && split != 8) p.xcd = false;
    p.split = split;
    p.kps = kps;
    return p;
}

template <int C, bool AKM, bool BKN, int EPI, bool OB>
static void launch_pipe_cfg(const GemmArgs& a, int split, hipStream_t s) {
    constexpr PipeCfg c = kCfgs[C];
    constexpr int nthreads = 64 * (c.wgm * c.wgn * c.ks + c.np);
    constexpr size_t lds = std::max((size_t)c.ns * c.ks * (c.bm + c.bn) * GEMM_BK * 2,
                                    (size_t)(c.bm / c.wgm) * (c.bn + 4) * 4);
    using KSplit = decltype(&gemm_pipe_kernel<16, 16, 1, 1, 2, AKM, BKN, ERGM_EPI_NONE, false>);
    KSplit k_split, k_full;
    if constexpr (c.ks == 2) {
        k_split = gemm_ks2_kernel<c.bm, c.bn, c.wgm, c.wgn, c.ns, AKM, BKN, ERGM_EPI_NONE, false>;
        k_full = gemm_ks2_kernel<c.bm, c.bn, c.wgm, c.wgn, c.ns, AKM, BKN, EPI, OB>;
    } else if constexpr (c.np > 0) {
        k_split = gemm_ws_kernel<c.bm, c.bn, c.wgm, c.wgn, c.np, c.ns, AKM, BKN, ERGM_EPI_NONE, false>;
        k_full = gemm_ws_kernel<c.bm, c.bn, c.wgm, c.wgn, c.np, c.ns, AKM, BKN, EPI, OB>;
    } else {
        k_split = gemm_pipe_kernel<c.bm, c.bn, c.wgm, c.wgn, c.ns, AKM, BKN, ERGM_EPI_NONE, false, false, c.il, c.mf>;
        k_full = gemm_pipe_kernel<c.bm, c.bn, c.wgm, c.wgn, c.ns, AKM, BKN, EPI, OB, c.direct, c.il, c.mf>;
    }
    static bool attr = (hipFuncSetAttribute((const void*)k_split, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                        hipFuncSetAttribute((const void*)k_full, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                        true);
    (void)attr;
    dim3 grid(a.tiles_m * a.tiles_n, 1, split);
    if (a.xcd_split) grid = dim3(8 * a.tiles_m * a.tiles_n, 1, 1);  // split == 8, slice = XCD
    ERGM_LAUNCH(split > 1 ? k_split : k_full, grid, dim3(nthreads), lds, s, a);
}

template <bool AKM, bool BKN, int EPI, bool OB>
static void launch_pipe(const GemmArgs& a, int cfg, int split, hipStream_t s) {
    switch (cfg) {
        case 0: launch_pipe_cfg<0, AKM, BKN, EPI, OB>(a, split, s); break;
        case 1: launch_pipe_cfg<1, AKM, BKN, EPI, OB>(a, split, s); break;
        case 2: launch_pipe_cfg<2, AKM, BKN, EPI, OB>(a, split, s); break;
        case 3: launch_pipe_cfg<3, AKM, BKN, EPI, OB>(a, split, s); break;
        case 4: launch_pipe_cfg<4, AKM, BKN, EPI, OB>(a, split, s); break;
        case 5: launch_pipe_cfg<5, AKM, BKN, EPI, OB>(a, split, s); break;
        case 6: launch_pipe_cfg<6, AKM, BKN, EPI, OB>(a, split, s); break;
        case 7: launch_pipe_cfg<7, AKM, BKN, EPI, OB>(a, split, s); break;
        case 8: launch_pipe_cfg<8, AKM, BKN, EPI, OB>(a, split, s); break;
        case 9: launch_pipe_cfg<9, AKM, BKN, EPI, OB>(a, split, s); break;
        case 10: launch_pipe_cfg<10, AKM, BKN, EPI, OB>(a, split, s); break;
        case 11: launch_pipe_cfg<11, AKM, BKN, EPI, OB>(a, split, s); break;
        case 12: launch_pipe_cfg<12, AKM, BKN, EPI, OB>(a, split, s); break;
        case 13: launch_pipe_cfg<13, AKM, BKN, EPI, OB>(a, split, s); break;
        case 14: launch_pipe_cfg<14, AKM, BKN, EPI, OB>(a, split, s); break;
        case 15: launch_pipe_cfg<15, AKM, BKN, EPI, OB>(a, split, s); break;
        case 16: launch_pipe_cfg<16, AKM, BKN, EPI, OB>(a, split, s); break;
        case 17: launch_pipe_cfg<17, AKM, BKN, EPI, OB>(a, split, s); break;
        case 18: launch_pipe_cfg<18, AKM, BKN, EPI, OB>(a, split, s); break;
        case 19: launch_pipe_cfg<19, AKM, BKN, EPI, OB>(a, split, s); break;
        case 20: launch_pipe_cfg<20, AKM, BKN, EPI, OB>(a, split, s); break;
        case 21: launch_pipe_cfg<21, AKM, BKN, EPI, OB>(a, split, s); break;
        case 22: launch_pipe_cfg<22, AKM, BKN, EPI, OB>(a, split, s); break;
        case 23: launch_pipe_cfg<23, AKM, BKN, EPI, OB>(a, split, s); break;
        case 24: launch_pipe_cfg<24, AKM, BKN, EPI, OB>(a, split, s); break;
        case 25: launch_pipe_cfg<25, AKM, BKN, EPI, OB>(a, split, s); break;
        case 26: launch_pipe_cfg<26, AKM, BKN, EPI, OB>(a, split, s); break;
        case 27: launch_pipe_cfg<27, AKM, BKN, EPI, OB>(a, split, s); break;
        case 28: launch_pipe_cfg<28, AKM, BKN, EPI, OB>(a, split, s); break;
        case 29: launch_pipe_cfg<29, AKM, BKN, EPI, OB>(a, split, s); break;
        case 30: launch_pipe_cfg<30, AKM, BKN, EPI, OB>(a, split, s); break;
        case 31: launch_pipe_cfg<31, AKM, BKN, EPI, OB>(a, split, s); break;
        case 32: launch_pipe_cfg<32, AKM, BKN, EPI, OB>(a, split, s); break;
        case 33: launch_pipe_cfg<33, AKM, BKN, EPI, OB>(a, split, s); break;
        case 34: launch_pipe_cfg<34, AKM, BKN, EPI, OB>(a, split, s); break;
        case 35: launch_pipe_cfg<35, AKM, BKN, EPI, OB>(a, split, s); break;
        case 36: launch_pipe_cfg<36, AKM, BKN, EPI, OB>(a, split, s); break;
        case 37: launch_pipe_cfg<37, AKM, BKN, EPI, OB>(a, split, s); break;
        case 38: launch_pipe_cfg<38, AKM, BKN, EPI, OB>(a, split, s); break;
        case 39: launch_pipe_cfg<39, AKM, BKN, EPI, OB>(a, split, s); break;
        case 40: launch_pipe_cfg<40, AKM, BKN, EPI, OB>(a, split, s); break;
        case 41: launch_pipe_cfg<41, AKM, BKN, EPI, OB>(a, split, s); break;
        case 42: launch_pipe_cfg<42, AKM, BKN, EPI, OB>(a, split, s); break;
        case 43: launch_pipe_cfg<43, AKM, BKN, EPI, OB>(a, split, s); break;
        case 44: launch_pipe_cfg<44, AKM, BKN, EPI, OB>(a, split, s); break;
        case 45: launch_pipe_cfg<45, AKM, BKN, EPI, OB>(a, split, s); break;
        default: launch_pipe_cfg<46, AKM, BKN, EPI, OB>(a, split, s); break;
    }
}

// register-staged fallback (K % 64 != 0, odd N / leading dims, rarely used layout/epilogue pairs)
template <int BM, int BN, bool AKM, bool BKN, int EPI, bool OB>
static void launch_reg(const GemmArgs& a, int split, hipStream_t s) {
    constexpr size_t lds = std::max((size_t)2 * (BM + BN) * GEMM_BK * 2, (size_t)BM * (BN + 4) * 4);
    static bool attr = (hipFuncSetAttribute((const void*)gemm_kernel<BM, BN, AKM, BKN, EPI, OB>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                        hipFuncSetAttribute((const void*)gemm_kernel<BM, BN, AKM, BKN, ERGM_EPI_NONE, false>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                        true);
    (void)attr;
    dim3 grid(a.tiles_m * a.tiles_n, 1, split);
    if (split > 1)
        ERGM_LAUNCH((gemm_kernel<BM, BN, AKM, BKN, ERGM_EPI_NONE, false>), grid, dim3(GEMM_THREADS), lds, s, a);
    else
        ERGM_LAUNCH((gemm_kernel<BM, BN, AKM, BKN, EPI, OB>), grid, dim3(GEMM_THREADS), lds, s, a);
}

template <bool AKM, bool BKN, int EPI, bool OB>
static void launch_reg_any(const GemmArgs& a, const GemmPlan& p, hipStream_t s) {
    if (p.bm == 128) launch_reg<128, 128, AKM, BKN, EPI, OB>(a, p.split, s);
    else launch_reg<64, 64, AKM, BKN, EPI, OB>(a, p.split, s);
}

// Layout/epilogue pairs the training step issues get the pipelined kernel family.
template <bool AKM, bool BKN, int EPI, bool OB>
static constexpr bool pipe_combo() {
    return combo_ok(AKM, BKN, EPI, OB);
}

template <bool AKM, bool BKN, int EPI, bool OB>
static void launch_any(const GemmArgs& a, const GemmPlan& p, hipStream_t s) {
    if constexpr (pipe_combo<AKM, BKN, EPI, OB>()) {
        if (p.cfg >= 0) {
            launch_pipe<AKM, BKN, EPI, OB>(a, p.cfg, p.split, s);
            return;
        }
    }
    launch_reg_any<AKM, BKN, EPI, OB>(a, p, s);
}

template <int EPI, bool OB>
static void launch_layout(const GemmArgs& a, const GemmPlan& p, int al, int bl, hipStream_t s) {
    if (al == ERGM_MK && bl == ERGM_NK) launch_any<false, false, EPI, OB>(a, p, s);
    else if (al == ERGM_MK && bl == ERGM_KN) launch_any<false, true, EPI, OB>(a, p, s);
    else if (al == ERGM_KM && bl == ERGM_NK) launch_any<true, false, EPI, OB>(a, p, s);
    else launch_any<true, true, EPI, OB>(a, p, s);
}

template <int EPI, bool OB>
static void launch_reduce(const GemmArgs& a, int split, hipStream_t s) {
    size_t total = (size_t)a.M * a.N;
    int blocks = (int)std::min<size_t>((total + 255) / 256, 4096);
    ERGM_LAUNCH((splitk_reduce_kernel<EPI, OB>), dim3(blocks), dim3(256), 0, s, a, split);
}

}  // namespace ergm

using namespace ergm;

namespace ergm {
// fp8 configurations (tile, wave grid, stages); a stage is (BM + BN) x 128 bytes
struct F8Cfg {
    int bm, bn, wgm, wgn, ns;
};
static constexpr F8Cfg kF8Cfgs[] = {
    {128, 128, 2, 2, 3},  // 0
    {256, 128, 4, 2, 3},  // 1  8 waves
    {128, 128, 4, 2, 3},  // 2  8 waves (32x64 each)
    {256, 256, 4, 2, 2},  // 3  8 waves (64x128 each)
    {64, 64, 2, 2, 4},    // 4
};
static constexpr int kNumF8Cfgs = sizeof(kF8Cfgs) / sizeof(kF8Cfgs[0]);
static thread_local int g_force_f8_cfg = -1;

template <int C, int EPI, bool OB>
static void launch_f8_cfg(const GemmArgs& a, hipStream_t s) {
    constexpr F8Cfg c = kF8Cfgs[C];
    constexpr size_t lds = std::max((size_t)c.ns * (c.bm + c.bn) * 128, (size_t)(c.bm / c.wgm) * (c.bn + 4) * 4);
    auto k = gemm_f8_kernel<c.bm, c.bn, c.wgm, c.wgn, c.ns, EPI, OB>;
    static bool attr = (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), true);
    (void)attr;
    ERGM_LAUNCH(k, dim3(a.tiles_m * a.tiles_n), dim3(64 * c.wgm * c.wgn), lds, s, a);
}

template <int EPI, bool OB>
static void launch_f8(const GemmArgs& a, int cfg, hipStream_t s) {
    switch (cfg) {
        case 0: launch_f8_cfg<0, EPI, OB>(a, s); break;
        case 1: launch_f8_cfg<1, EPI, OB>(a, s); break;
        case 2: launch_f8_cfg<2, EPI, OB>(a, s); break;
        case 3: launch_f8_cfg<3, EPI, OB>(a, s); break;
        default: launch_f8_cfg<4, EPI, OB>(a, s); break;
    }
}

// Per-shape overrides of the fp8 / MX tile configuration (ergm_gemm_f8_set_override: the in-step tuner) and the
// built-in entries it measured; keyed on (M, N, K).
struct F8Override {
    int M, N, K, cfg;
};
static constexpr int kMaxF8Overrides = 32;
static F8Override g_f8_over[kMaxF8Overrides];
static int g_n_f8_over = 0;
static constexpr F8Override kF8StepTuned[] = {
    // config 5 (GPT-2-medium, B=32, S=128; forward chains of M = 2048): the MX c_fc GEMM on the 256 x 256 tile
    // (tools/step_tune.py --config c5 --f8: 21.06 -> 20.85 ms/step, profiles/r05_step_tune_c5_f8.txt)
    {2048, 4096, 1024, 3},
};

static int plan_f8(int M, int N, int K) {
    if (g_force_f8_cfg >= 0) return g_force_f8_cfg;
    {
        std::lock_guard<std::mutex> lk(g_over_mu);
        for (int i = 0; i < g_n_f8_over; ++i)
            if (g_f8_over[i].M == M && g_f8_over[i].N == N && g_f8_over[i].K == K) return g_f8_over[i].cfg;
    }
    for (const F8Override& o : kF8StepTuned)
        if (o.cfg >= 0 && o.M == M && o.N == N && o.K == K) return o.cfg;
    const long t128 = tiles_of(M, N, 128, 128);
    if (t128 >= 4000) return 3;
    if (t128 >= 512) return 1;
    if (t128 >= 140) return 2;
    return 4;
}

}  // namespace ergm

namespace ergm {
template <int C, int EPI, bool OB, bool QMX>
static void launch_mx_cfg(const GemmArgs& a, hipStream_t s) {
    constexpr F8Cfg c = kF8Cfgs[C];
    constexpr size_t stage = (size_t)(c.bm + c.bn) * 132;  // operand bytes (128 per row) + scale bytes (4 per row)
    constexpr size_t lds = std::max((size_t)c.ns * stage, (size_t)(c.bm / c.wgm) * (c.bn + 4) * 4);
    auto k = gemm_mx_kernel<c.bm, c.bn, c.wgm, c.wgn, c.ns, EPI, OB, QMX>;
    static bool attr = (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), true);
    (void)attr;
    ERGM_LAUNCH(k, dim3(a.tiles_m * a.tiles_n), dim3(64 * c.wgm * c.wgn), lds, s, a);
}
template <int EPI, bool OB, bool QMX>
static void launch_mx(const GemmArgs& a, int cfg, hipStream_t s) {
    switch (cfg) {
        case 0: launch_mx_cfg<0, EPI, OB, QMX>(a, s); break;
        case 1: launch_mx_cfg<1, EPI, OB, QMX>(a, s); break;
        case 2: launch_mx_cfg<2, EPI, OB, QMX>(a, s); break;
        case 3: launch_mx_cfg<3, EPI, OB, QMX>(a, s); break;
        default: launch_mx_cfg<4, EPI, OB, QMX>(a, s); break;
    }
}
}  // namespace ergm

extern "C" int ergm_gemm_mx(const ergm_gemm_desc* d, const void* A, const void* a_scale, int ld_sa, const void* B,
                            const void* b_scale, int ld_sb, void* C, void* q_out, void* q_scale, int ld_q, int ld_qs,
                            void* stream) {
    using namespace ergm;
    ERGM_CHECK_ARG(d && A && B && C && a_scale && b_scale, "ergm_gemm_mx: null argument");
    ERGM_CHECK_ARG(d->M > 0 && d->N > 0 && d->K > 0 && d->K % 128 == 0, "ergm_gemm_mx: K=%d must be a multiple of 128",
                   d->K);
    ERGM_CHECK_ARG(d->a_layout == ERGM_MK && d->b_layout == ERGM_NK, "ergm_gemm_mx: A [M][K] and B [N][K] only");
    ERGM_CHECK_ARG(d->lda >= d->K && d->ldb >= d->K && d->lda % 16 == 0 && d->ldb % 16 == 0,
                   "ergm_gemm_mx: lda/ldb >= K, multiples of 16 bytes");
    ERGM_CHECK_ARG(ld_sa >= d->M && ld_sb >= d->N, "ergm_gemm_mx: scale pitches ld_sa >= M, ld_sb >= N (rows)");
    ERGM_CHECK_ARG(aligned16(A) && aligned16(B) && (reinterpret_cast<uintptr_t>(a_scale) & 3) == 0 &&
                       (reinterpret_cast<uintptr_t>(b_scale) & 3) == 0,
                   "ergm_gemm_mx: operand / scale alignment");
    ERGM_CHECK_ARG(d->N % 8 == 0 && d->ldc % 8 == 0 && d->ldc >= d->N, "ergm_gemm_mx: N, ldc multiples of 8");
    ERGM_CHECK_ARG(d->c_dtype == ERGM_F32 || d->c_dtype == ERGM_BF16, "ergm_gemm_mx: bad c_dtype");
    const int e = d->epilogue;
    const bool bf_epi = e == ERGM_EPI_BIAS || e == ERGM_EPI_BIAS_GELU || e == ERGM_EPI_GELU_BWD;
    ERGM_CHECK_ARG(e == ERGM_EPI_NONE || (bf_epi && d->c_dtype == ERGM_BF16) ||
                       (e == ERGM_EPI_BIAS_RESID && d->c_dtype == ERGM_F32),
                   "ergm_gemm_mx: epilogue %d with c_dtype %d not supported", e, d->c_dtype);
    ERGM_CHECK_ARG(!(e == ERGM_EPI_BIAS_RESID || e == ERGM_EPI_GELU_BWD) || (d->aux && d->ld_aux % 8 == 0),
                   "ergm_gemm_mx: epilogue %d needs aux", e);
    ERGM_CHECK_ARG(e != ERGM_EPI_BIAS_GELU || (d->aux_out && d->ld_aux_out % 8 == 0), "ergm_gemm_mx: GELU needs aux_out");
    ERGM_CHECK_ARG(!q_out || (q_scale && (e == ERGM_EPI_BIAS_GELU || e == ERGM_EPI_GELU_BWD) && d->N % 32 == 0 &&
                              ld_q >= d->N && ld_q % 8 == 0 && ld_qs >= d->M),
                   "ergm_gemm_mx: the MX copy of C needs a GELU / GELU' epilogue, N % 32 == 0 and its buffers");
    {  // the shape trace lists the fp8 / MX GEMMs with a_layout 16 (ergm_gemm_f8_set_override's keys)
        ergm_gemm_desc t = *d;
        t.a_layout = 16;
        trace_shape(&t);
    }
    const int cfg = plan_f8(d->M, d->N, d->K);
    GemmArgs a;
    memset(&a, 0, sizeof(a));
    a.A = reinterpret_cast<const __bf16*>(A);
    a.B = reinterpret_cast<const __bf16*>(B);
    a.C = C;
    a.M = d->M; a.N = d->N; a.K = d->K;
    a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc;
    a.alpha = d->alpha; a.alpha_dev = d->alpha_dev;
    a.bias = d->bias; a.aux = d->aux; a.ld_aux = d->ld_aux;
    a.aux_out = d->aux_out; a.ld_aux_out = d->ld_aux_out;
    a.tiles_m = cdiv(d->M, kF8Cfgs[cfg].bm);
    a.tiles_n = cdiv(d->N, kF8Cfgs[cfg].bn);
    a.sweep_m = (long)d->M < (long)d->N ? 1 : 0;
    a.a_mx = reinterpret_cast<const uint8_t*>(a_scale);
    a.b_mx = reinterpret_cast<const uint8_t*>(b_scale);
    a.ld_sa = ld_sa; a.ld_sb = ld_sb;
    a.q_out = reinterpret_cast<uint8_t*>(q_out);
    a.q_sc = reinterpret_cast<uint8_t*>(q_scale);
    a.ld_q = ld_q; a.ld_qs = ld_qs;
    ERGM_TRY(check_dropout(d->dropout));
    ERGM_CHECK_ARG(!d->dropout || d->dropout->p == 0.f || e == ERGM_EPI_BIAS_RESID,
                   "ergm_gemm_mx: dropout applies to the BIAS_RESID epilogue only");
    a.drop = drop_site_of(d->dropout, d->N);
    hipStream_t s = as_stream(stream);
    const bool ob = d->c_dtype == ERGM_BF16;
    switch (e) {
        case ERGM_EPI_NONE:
            if (ob) launch_mx<ERGM_EPI_NONE, true, false>(a, cfg, s);
            else launch_mx<ERGM_EPI_NONE, false, false>(a, cfg, s);
            break;
        case ERGM_EPI_BIAS: launch_mx<ERGM_EPI_BIAS, true, false>(a, cfg, s); break;
        case ERGM_EPI_BIAS_GELU:
            if (q_out) launch_mx<ERGM_EPI_BIAS_GELU, true, true>(a, cfg, s);
            else launch_mx<ERGM_EPI_BIAS_GELU, true, false>(a, cfg, s);
            break;
        case ERGM_EPI_GELU_BWD:
            if (q_out) launch_mx<ERGM_EPI_GELU_BWD, true, true>(a, cfg, s);
            else launch_mx<ERGM_EPI_GELU_BWD, true, false>(a, cfg, s);
            break;
        default: launch_mx<ERGM_EPI_BIAS_RESID, false, false>(a, cfg, s); break;
    }
    return check_launch("ergm_gemm_mx");
}

extern "C" int ergm_gemm_f8_set_override(int M, int N, int K, int cfg) {
    using namespace ergm;
    ERGM_CHECK_ARG(cfg >= -1 && cfg < kNumF8Cfgs, "gemm_f8_set_override: cfg in [-1, %d)", kNumF8Cfgs);
    std::lock_guard<std::mutex> lk(g_over_mu);
    for (int i = 0; i < g_n_f8_over; ++i)
        if (g_f8_over[i].M == M && g_f8_over[i].N == N && g_f8_over[i].K == K) {
            if (cfg < 0) g_f8_over[i] = g_f8_over[--g_n_f8_over];
            else g_f8_over[i].cfg = cfg;
            return ERGM_OK;
        }
    if (cfg < 0) return ERGM_OK;
    ERGM_CHECK_ARG(g_n_f8_over < kMaxF8Overrides, "gemm_f8_set_override: table full");
    g_f8_over[g_n_f8_over++] = F8Override{M, N, K, cfg};
    return ERGM_OK;
}

extern "C" int ergm_gemm_f8_tune(int cfg) {
    ERGM_CHECK_ARG(cfg >= -1 && cfg < ergm::kNumF8Cfgs, "gemm_f8_tune: cfg in [-1, %d)", ergm::kNumF8Cfgs);
    ergm::g_force_f8_cfg = cfg;
    return ERGM_OK;
}

extern "C" int ergm_gemm_f8(const ergm_gemm_desc* d, const void* A, const float* a_scale, const void* B,
                            const float* b_scale, void* C, void* stream) {
    using namespace ergm;
    ERGM_CHECK_ARG(d && A && B && C && a_scale && b_scale, "ergm_gemm_f8: null argument");
    ERGM_CHECK_ARG(d->M > 0 && d->N > 0 && d->K > 0 && d->K % 128 == 0, "ergm_gemm_f8: K=%d must be a multiple of 128",
                   d->K);
    ERGM_CHECK_ARG(d->a_layout == ERGM_MK && d->b_layout == ERGM_NK, "ergm_gemm_f8: A [M][K] and B [N][K] only");
    ERGM_CHECK_ARG(d->lda >= d->K && d->ldb >= d->K && d->lda % 16 == 0 && d->ldb % 16 == 0,
                   "ergm_gemm_f8: lda/ldb >= K, multiples of 16 bytes");
    ERGM_CHECK_ARG(aligned16(A) && aligned16(B) && aligned16(b_scale), "ergm_gemm_f8: 16-byte alignment");
    ERGM_CHECK_ARG(d->N % 8 == 0 && d->ldc % 8 == 0 && d->ldc >= d->N, "ergm_gemm_f8: N, ldc multiples of 8");
    ERGM_CHECK_ARG(d->c_dtype == ERGM_F32 || d->c_dtype == ERGM_BF16, "ergm_gemm_f8: bad c_dtype");
    const int e = d->epilogue;
    ERGM_CHECK_ARG((e == ERGM_EPI_NONE || e == ERGM_EPI_BIAS || e == ERGM_EPI_BIAS_GELU) ? d->c_dtype == ERGM_BF16 ||
                       e == ERGM_EPI_NONE
                                                                                        : e == ERGM_EPI_BIAS_RESID &&
                                                                                              d->c_dtype == ERGM_F32,
                   "ergm_gemm_f8: epilogue %d with c_dtype %d not supported", e, d->c_dtype);
    ERGM_CHECK_ARG(e != ERGM_EPI_BIAS_RESID || (d->aux && d->ld_aux % 8 == 0), "ergm_gemm_f8: residual needs aux");
    ERGM_CHECK_ARG(e != ERGM_EPI_BIAS_GELU || (d->aux_out && d->ld_aux_out % 8 == 0), "ergm_gemm_f8: GELU needs aux_out");
    {  // the shape trace lists the fp8 / MX GEMMs with a_layout 16 (ergm_gemm_f8_set_override's keys)
        ergm_gemm_desc t = *d;
        t.a_layout = 16;
        trace_shape(&t);
    }
    const int cfg = plan_f8(d->M, d->N, d->K);
    GemmArgs a;
    memset(&a, 0, sizeof(a));
    a.A = reinterpret_cast<const __bf16*>(A);
    a.B = reinterpret_cast<const __bf16*>(B);
    a.C = C;
    a.M = d->M; a.N = d->N; a.K = d->K;
    a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc;
    a.alpha = d->alpha; a.alpha_dev = d->alpha_dev;
    a.bias = d->bias; a.aux = d->aux; a.ld_aux = d->ld_aux;
    a.aux_out = d->aux_out; a.ld_aux_out = d->ld_aux_out;
    a.tiles_m = cdiv(d->M, kF8Cfgs[cfg].bm);
    a.tiles_n = cdiv(d->N, kF8Cfgs[cfg].bn);
    a.sweep_m = (long)d->M < (long)d->N ? 1 : 0;
    a.a_scale = a_scale;
    a.b_scale = b_scale;
    ERGM_TRY(check_dropout(d->dropout));
    ERGM_CHECK_ARG(!d->dropout || d->dropout->p == 0.f || e == ERGM_EPI_BIAS_RESID,
                   "ergm_gemm_f8: dropout applies to the BIAS_RESID epilogue only");
    a.drop = drop_site_of(d->dropout, d->N);
    hipStream_t s = as_stream(stream);
    const bool ob = d->c_dtype == ERGM_BF16;
    switch (e) {
        case ERGM_EPI_NONE:
            if (ob) launch_f8<ERGM_EPI_NONE, true>(a, cfg, s);
            else launch_f8<ERGM_EPI_NONE, false>(a, cfg, s);
            break;
        case ERGM_EPI_BIAS: launch_f8<ERGM_EPI_BIAS, true>(a, cfg, s); break;
        case ERGM_EPI_BIAS_GELU: launch_f8<ERGM_EPI_BIAS_GELU, true>(a, cfg, s); break;
        default: launch_f8<ERGM_EPI_BIAS_RESID, false>(a, cfg, s); break;
    }
    return check_launch("ergm_gemm_f8");
}

extern "C" int ergm_gemm_tune(int cfg, int split) {
    ERGM_CHECK_ARG(cfg >= -1 && cfg < kNumCfgs && split >= 0, "gemm_tune: cfg in [-1, %d), split >= 0", kNumCfgs);
    g_force_cfg = cfg;
    g_force_split = split;
    return ERGM_OK;
}

extern "C" size_t ergm_gemm_workspace_size(const ergm_gemm_desc* d) {
    if (!d) return 0;
    GemmPlan p = plan_gemm(d);
    if (p.split <= 1) return 0;
    return (size_t)p.split * d->M * d->N * sizeof(float) + (d->bias_grad ? (size_t)p.split * d->N * sizeof(float) : 0);
}

extern "C" int ergm_gemm_set_override(int M, int N, int K, int a_layout, int b_layout, int cfg, int split) {
    ERGM_CHECK_ARG(cfg >= -1 && cfg < kNumCfgs && split >= 1 && split <= 16, "gemm_set_override: cfg in [-1, %d)",
                   kNumCfgs);
    std::lock_guard<std::mutex> lk(g_over_mu);
    for (int i = 0; i < g_n_over; ++i) {
        GemmOverride& o = g_over[i];
        if (o.M == M && o.N == N && o.K == K && o.al == a_layout && o.bl == b_layout) {
            if (cfg < 0) {
                o = g_over[--g_n_over];
            } else {
                o.cfg = cfg;
                o.split = split;
            }
            return ERGM_OK;
        }
    }
    if (cfg < 0) return ERGM_OK;
    ERGM_CHECK_ARG(g_n_over < kMaxOverrides, "gemm_set_override: table full");
    g_over[g_n_over++] = GemmOverride{M, N, K, a_layout, b_layout, cfg, split};
    return ERGM_OK;
}

extern "C" int ergm_gemm_trace(int on, int* shapes, int max_shapes) {
    std::lock_guard<std::mutex> lk(g_over_mu);
    const int n = g_trace_n;
    if (shapes)
        for (int i = 0; i < n && i < max_shapes; ++i)
            for (int j = 0; j < 5; ++j) shapes[i * 5 + j] = g_trace[i][j];
    if (on && !g_trace_on) g_trace_n = 0;
    g_trace_on = on != 0;
    return n;
}

namespace ergm {
// Kernel arguments of one planned GEMM (split-K slabs are set by the caller).
static GemmArgs make_args(const ergm_gemm_desc* d, const void* A, const void* B, void* C, const GemmPlan& p) {
    GemmArgs a;
    a.A = reinterpret_cast<const __bf16*>(A);
    a.B = reinterpret_cast<const __bf16*>(B);
    a.C = C;
    a.M = d->M; a.N = d->N; a.K = d->K;
    a.lda = d->lda; a.ldb = d->ldb; a.ldc = d->ldc;
    a.alpha = d->alpha; a.alpha_dev = d->alpha_dev;
    a.bias = d->bias; a.aux = d->aux; a.ld_aux = d->ld_aux;
    a.aux_out = d->aux_out; a.ld_aux_out = d->ld_aux_out;
    a.tiles_m = cdiv(d->M, p.bm); a.tiles_n = cdiv(d->N, p.bn);
    // stream the larger operand once: walk along the dimension of the smaller operand
    a.sweep_m = (long)d->M < (long)d->N ? 1 : 0;
    a.k_per_split = p.kps;
    a.slab = nullptr;
    a.a_scale = a.b_scale = nullptr;
    a.drop = drop_site_of(d->dropout, d->N);
    // the vocabulary-wide bf16 logits (206 MB at C2) are streamed out with non-temporal stores so they
    // do not evict the operands of the kernels running beside the LM head (C2 step +0.5-1 %,
    // profiles/r01_overlap_experiments.txt #14) ... and so are the f32 weight gradients (A = activationsᵀ),
    // consumed later by the optimizer / the all-reduce (C5 +0.4-0.8 %, C2 neutral: #17)
    static const bool nt_wide = [] {  // ERGM_NT_WIDE=0: vocabulary-wide bf16 outputs (the logits) stored normally (A/B)
        const char* e = getenv("ERGM_NT_WIDE");
        return !e || atoi(e) != 0;
    }();
    a.nt_store = (nt_wide && d->c_dtype == ERGM_BF16 && d->N >= 32768) ||
                 (d->c_dtype == ERGM_F32 && d->a_layout == ERGM_KM && d->epilogue == ERGM_EPI_NONE);
    // the in-GEMM bias gradient runs in the pipelined (non-warp-specialised) kernels; others use a column-sum pass
    const bool cs_in = d->bias_grad && p.cfg >= 0 && kCfgs[p.cfg].np == 0 && kCfgs[p.cfg].ks == 1 && kCfgs[p.cfg].mf == 16;
    a.colsum = cs_in ? d->bias_grad : nullptr;
    a.colsum_part = nullptr;
    a.xcd_split = p.xcd && p.cfg >= 0 && kCfgs[p.cfg].np == 0 && kCfgs[p.cfg].ks == 1 && kCfgs[p.cfg].mf == 16 ? 1 : 0;
    return a;
}
}  // namespace ergm

namespace ergm {
// Argument checks of ergm_gemm (also applied to each problem of a grouped launch).
static int validate_desc(const ergm_gemm_desc* d, const void* A, const void* B, const void* C) {
    ERGM_CHECK_ARG(d && A && B && C, "ergm_gemm: null argument");
    ERGM_CHECK_ARG(d->M > 0 && d->N > 0 && d->K > 0, "ergm_gemm: bad shape M=%d N=%d K=%d", d->M, d->N, d->K);
    // k-contiguous operands are read in 8-element chunks along K; with both operands k-major (rows = k,
    // the weight-gradient layout) any K works
    ERGM_CHECK_ARG(d->K % 8 == 0 || (d->a_layout == ERGM_KM && d->b_layout == ERGM_KN),
                   "ergm_gemm: K=%d must be a multiple of 8 unless a_layout = KM and b_layout = KN", d->K);
    ERGM_CHECK_ARG(d->lda % 8 == 0 && d->ldb % 8 == 0, "ergm_gemm: lda/ldb must be multiples of 8 elements");
    ERGM_CHECK_ARG(aligned16(A) && aligned16(B), "ergm_gemm: A/B must be 16-byte aligned");
    ERGM_CHECK_ARG(d->a_layout == ERGM_MK || d->a_layout == ERGM_KM, "ergm_gemm: bad a_layout");
    ERGM_CHECK_ARG(d->b_layout == ERGM_NK || d->b_layout == ERGM_KN, "ergm_gemm: bad b_layout");
    ERGM_CHECK_ARG(d->a_layout == ERGM_MK ? d->lda >= d->K : d->lda >= d->M, "ergm_gemm: lda too small");
    ERGM_CHECK_ARG(d->b_layout == ERGM_NK ? d->ldb >= d->K : d->ldb >= d->N, "ergm_gemm: ldb too small");
    // m/n-contiguous operands are staged in whole 16-B chunks: the row must hold round_up(M|N, 8)
    ERGM_CHECK_ARG(d->a_layout == ERGM_MK || d->lda >= ((d->M + 7) & ~7), "ergm_gemm: KM layout needs lda >= round8(M)");
    ERGM_CHECK_ARG(d->b_layout == ERGM_NK || d->ldb >= ((d->N + 7) & ~7), "ergm_gemm: KN layout needs ldb >= round8(N)");
    ERGM_CHECK_ARG(d->ldc >= d->N, "ergm_gemm: ldc < N");
    ERGM_CHECK_ARG(d->c_dtype == ERGM_F32 || d->c_dtype == ERGM_BF16, "ergm_gemm: bad c_dtype");
    int e = d->epilogue;
    ERGM_CHECK_ARG(e >= ERGM_EPI_NONE && e <= ERGM_EPI_ACCUM, "ergm_gemm: bad epilogue %d", e);
    ERGM_CHECK_ARG(!(e == ERGM_EPI_BIAS_RESID || e == ERGM_EPI_ACCUM) || d->c_dtype == ERGM_F32,
                   "ergm_gemm: residual/accumulate epilogues need f32 C");
    ERGM_CHECK_ARG(!(e == ERGM_EPI_BIAS_RESID || e == ERGM_EPI_GELU_BWD) || d->aux, "ergm_gemm: epilogue needs aux");
    ERGM_CHECK_ARG(e != ERGM_EPI_BIAS_GELU || d->aux_out, "ergm_gemm: BIAS_GELU needs aux_out");
    ERGM_TRY(check_dropout(d->dropout));
    ERGM_CHECK_ARG(!d->dropout || d->dropout->p == 0.f || e == ERGM_EPI_BIAS_RESID,
                   "ergm_gemm: dropout applies to the BIAS_RESID epilogue only");
    ERGM_CHECK_ARG(!d->bias_grad || (d->a_layout == ERGM_KM && d->b_layout == ERGM_KN && e == ERGM_EPI_NONE &&
                                     d->c_dtype == ERGM_F32),
                   "ergm_gemm: bias_grad needs a_layout KM, b_layout KN, epilogue NONE and f32 C");

    return ERGM_OK;
}
}  // namespace ergm

extern "C" int ergm_gemm(const ergm_gemm_desc* d, const void* A, const void* B, void* C, void* ws,
                         size_t ws_bytes, void* stream) {
    ERGM_TRY(validate_desc(d, A, B, C));
    const int e = d->epilogue;
    trace_shape(d);
    GemmPlan p = plan_gemm(d);
    GemmArgs a = make_args(d, A, B, C, p);
    const bool cs_in = a.colsum != nullptr;
    hipStream_t s = as_stream(stream);
    if (p.split > 1) {
        size_t need = (size_t)p.split * d->M * d->N * sizeof(float) + (d->bias_grad ? (size_t)p.split * d->N * 4 : 0);
        ERGM_CHECK_ARG(ws && ws_bytes >= need, "ergm_gemm: split-K %d needs %zu workspace bytes (got %zu)", p.split,
                       need, ws_bytes);
        a.slab = reinterpret_cast<float*>(ws);
        if (cs_in) a.colsum_part = a.slab + (size_t)p.split * d->M * d->N;
    }
    const bool ob = d->c_dtype == ERGM_BF16;
#define ERGM_EPI_CASE(E)                                                  \
    case E:                                                               \
        if (ob) launch_layout<E, true>(a, p, d->a_layout, d->b_layout, s); \
        else launch_layout<E, false>(a, p, d->a_layout, d->b_layout, s);   \
        if (p.split > 1) {                                                \
            if (ob) launch_reduce<E, true>(a, p.split, s);                 \
            else launch_reduce<E, false>(a, p.split, s);                   \
        }                                                                 \
        break;
    switch (e) {
        ERGM_EPI_CASE(ERGM_EPI_NONE)
        ERGM_EPI_CASE(ERGM_EPI_BIAS)
        ERGM_EPI_CASE(ERGM_EPI_BIAS_GELU)
        ERGM_EPI_CASE(ERGM_EPI_BIAS_RESID)
        ERGM_EPI_CASE(ERGM_EPI_GELU_BWD)
        ERGM_EPI_CASE(ERGM_EPI_ACCUM)
    }
#undef ERGM_EPI_CASE
    if (d->bias_grad && !cs_in)
        ERGM_LAUNCH(colsum_kn_kernel, dim3(cdiv(d->N, 64)), dim3(256), 0, s, a.B, d->K, d->N, d->ldb, d->alpha,
                           d->alpha_dev, d->bias_grad);
    return check_launch("ergm_gemm");
}

namespace ergm {
template <int C, int EPI = ERGM_EPI_NONE>
static void launch_dw2_cfg(const GemmArgs2& g, int nblocks, hipStream_t s) {
    constexpr PipeCfg c = kCfgs[C];
    static_assert(c.np == 0 && !c.direct, "grouped dW launch: pipelined kernels with the staged epilogue only");
    constexpr size_t lds = std::max((size_t)c.ns * (c.bm + c.bn) * GEMM_BK * 2, (size_t)(c.bm / c.wgm) * (c.bn + 4) * 4);
    auto k = gemm_dw2_kernel<c.bm, c.bn, c.wgm, c.wgn, c.ns, c.il, EPI, c.mf>;
    static bool attr = (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), true);
    (void)attr;
    ERGM_LAUNCH(k, dim3(nblocks), dim3(64 * c.wgm * c.wgn), lds, s, g);
}

// Two weight-gradient GEMMs (a_layout KM, b_layout KN, epilogue NONE, f32 C) in one launch when both plan
// to the same unsplit pipelined configuration; ERGM_EUNSUPPORTED (nothing launched) otherwise, and the caller
// issues them one by one.  launch = false: only the check.  Same kernel body and tile order as ergm_gemm: the results are bit-identical.
int gemm_dw_pair(const ergm_gemm_desc* const d[2], const void* const A[2], const void* const B[2], void* const C[2],
                 void* stream, bool launch) {
    for (int i = 0; i < 2; ++i) {
        ERGM_TRY(validate_desc(d[i], A[i], B[i], C[i]));
        if (d[i]->a_layout != ERGM_KM || d[i]->b_layout != ERGM_KN || d[i]->epilogue != ERGM_EPI_NONE ||
            d[i]->c_dtype != ERGM_F32 || d[i]->split_k > 1 || !pipe_ok(d[i]))
            return ERGM_EUNSUPPORTED;
    }
    GemmPlan p[2] = {plan_gemm(d[0]), plan_gemm(d[1])};
    const int cfg = p[0].cfg;
    if (cfg < 0 || (cfg >= 16 && cfg < 38 && kCfgs[cfg].il == 0) || kCfgs[cfg].ks != 1 || p[1].cfg != cfg ||
        p[0].split != 1 ||
        p[1].split != 1 ||
        p[0].xcd || p[1].xcd || kCfgs[cfg].np != 0 || kCfgs[cfg].direct)
        return ERGM_EUNSUPPORTED;
    // only pairs whose problems each leave CUs idle: grouping two chip-filling GEMMs measured slower (C5:
    // 264 + 288 tiles, step +1.2 %); C2's pairs (150 + 168, 156 + 156 tiles) gain 0.4 %
    if (tiles_of(d[0]->M, d[0]->N, p[0].bm, p[0].bn) >= 256 || tiles_of(d[1]->M, d[1]->N, p[1].bm, p[1].bn) >= 256)
        return ERGM_EUNSUPPORTED;
    if (!launch) return ERGM_OK;
    trace_shape(d[0]);
    trace_shape(d[1]);
    GemmArgs2 g;
    for (int i = 0; i < 2; ++i) g.a[i] = make_args(d[i], A[i], B[i], C[i], p[i]);
    const int n0 = g.a[0].tiles_m * g.a[0].tiles_n, n1 = g.a[1].tiles_m * g.a[1].tiles_n;
    g.b1 = (n0 + 7) & ~7;
    const int nb = g.b1 + n1;
    hipStream_t s = as_stream(stream);
    switch (cfg) {
        case 0: launch_dw2_cfg<0>(g, nb, s); break;
        case 1: launch_dw2_cfg<1>(g, nb, s); break;
        case 2: launch_dw2_cfg<2>(g, nb, s); break;
        case 3: launch_dw2_cfg<3>(g, nb, s); break;
        case 4: launch_dw2_cfg<4>(g, nb, s); break;
        case 5: launch_dw2_cfg<5>(g, nb, s); break;
        case 6: launch_dw2_cfg<6>(g, nb, s); break;
        case 7: launch_dw2_cfg<7>(g, nb, s); break;
        case 8: launch_dw2_cfg<8>(g, nb, s); break;
        case 9: launch_dw2_cfg<9>(g, nb, s); break;
        case 10: launch_dw2_cfg<10>(g, nb, s); break;
        case 11: launch_dw2_cfg<11>(g, nb, s); break;
        case 12: launch_dw2_cfg<12>(g, nb, s); break;
        case 13: launch_dw2_cfg<13>(g, nb, s); break;
        case 14: launch_dw2_cfg<14>(g, nb, s); break;
        case 15: launch_dw2_cfg<15>(g, nb, s); break;
        case 25: launch_dw2_cfg<25>(g, nb, s); break;
        case 26: launch_dw2_cfg<26>(g, nb, s); break;
        case 27: launch_dw2_cfg<27>(g, nb, s); break;
        case 29: launch_dw2_cfg<29>(g, nb, s); break;
        case 30: launch_dw2_cfg<30>(g, nb, s); break;
        case 31: launch_dw2_cfg<31>(g, nb, s); break;
        case 32: launch_dw2_cfg<32>(g, nb, s); break;
        case 38: launch_dw2_cfg<38>(g, nb, s); break;
        case 39: launch_dw2_cfg<39>(g, nb, s); break;
        case 40: launch_dw2_cfg<40>(g, nb, s); break;
        case 41: launch_dw2_cfg<41>(g, nb, s); break;
        case 42: launch_dw2_cfg<42>(g, nb, s); break;
        case 43: launch_dw2_cfg<43>(g, nb, s); break;
        case 44: launch_dw2_cfg<44>(g, nb, s); break;
        case 45: launch_dw2_cfg<45>(g, nb, s); break;
        case 46: launch_dw2_cfg<46>(g, nb, s); break;
        default: return ERGM_EUNSUPPORTED;
    }
    return check_launch("gemm_dw_pair");
}
}  // namespace ergm
