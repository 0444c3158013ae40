// Fused multi-head attention (head_dim 64) forward/backward for gfx950.
//
// Replaces GPT2Attention._attn (src/model.py:119-148): W = QKᵀ / sqrt(d); causal
// where(tril, W, finfo.min) for self-attention; additive all-zero encoder mask for the cross path
// (src/model.py:484-489, elided); softmax; O = W·V — and its autograd backward.  _split_heads /
// _merge_heads (src/model.py:190-198) are folded into addressing: Q/K/V/O are token-major
// [b*S + s][h*64 + d] slices of the Conv1D outputs.
//
// Forward (flash-style, online softmax): one workgroup = 4 waves = 64 queries of one (b, h); each
// wave owns 16 queries.  Scores are computed SWAPPED, Sᵀ = K·Qᵀ (v_mfma_f32_16x16x32_bf16), so a
// lane holds 16 keys of ONE query: row max/sum are lane-local + two xor-shuffles.  The output is also
// kept transposed, Oᵀ = Vᵀ·Pᵀ: P feeds the MFMA B operand straight from registers (k-order
// permuted identically on both operands) and Vᵀ comes from the LDS V tile by ds_read_b64_tr_b16.
// Backward: δ = rowsum(dO·O) kernel, dK/dV kernel (workgroup = 64 keys, loops over query tiles, P
// recomputed from the forward LSE) + dQ kernel (workgroup = 64 queries, loops over key tiles); no
// atomics, deterministic.  The tiled kernels stream their 64-row tiles through a 3-stage LDS ring filled
// by LDS-DMA (tiles.h GldsTile: two tiles in flight while one is consumed, one barrier per tile); causal
// grids start with the longest rows.
// The backward of sequences of at most 128 (the training path: S = 128 tokens, 128 caption rows) takes
// the fused short kernel instead: one 8-wave workgroup per (b, h) holding every operand in LDS, the whole
// backward in one launch; it evaluates every product in the same order as the tiled kernels
// (bit-identical).  The forward is tiled at every length.
// Softmax arithmetic in the exp2 domain (v_exp_f32 is 2^x): exp(scale·s − shift) = exp2(fma(s, c, −shift·log2e))
// with c = scale·log2e, one FMA + one v_exp per score; tiles a wave sees entirely unmasked (uniform
// test per wave and tile) skip the mask compares.
#include "common.h"
#include "tiles.h"

#include <cstdlib>

namespace ergm {

constexpr int AT_D = 64;       // head dim
constexpr int AT_T = 64;       // tile rows (queries or keys)
constexpr int AT_TILE_BYTES = AT_T * AT_D * 2;  // 8 KiB
constexpr int AT_MAX_SQ_DROP = 1024;            // dropout: keep-bit words a tiled backward stages in LDS

// 64x64 bf16 tile in LDS, 128-B rows, 16-B chunk c of row r stored at chunk c ^ (r & 7):
// conflict-free for both ds_read_b128 row reads and the ds_read_b64_tr_b16 reads below.
__device__ __forceinline__ int tile_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

// Row-read operand fragment (16x16x32): lane l gets X[row0 + (l&15)][32ks + 8(l>>4) + j].
__device__ __forceinline__ bf16x8 row_frag(const char* lds, int row0, int ks) {
    const int lane = threadIdx.x & 63;
    int row = row0 + (lane & 15);
    return *reinterpret_cast<const bf16x8*>(lds + tile_off(row, ks * 4 + (lane >> 4)));
}

// Transposed operand fragment over 32 tile rows starting at krow0 (the MFMA k dim) and 16 columns
// starting at col0 (the MFMA m dim): lane l (g = l>>4, i = l&15) gets element j =
//   X[krow0 + 4g + j][col0 + i]        (j < 4)
//   X[krow0 + 16 + 4g + j-4][col0 + i] (j >= 4)
// — the same permuted k order as the P/dS register fragments (pack_p).
__device__ __forceinline__ bf16x8 tr_frag(const char* lds, int krow0, int col0) {
    const int lane = threadIdx.x & 63;
    const int i = lane & 15, g = lane >> 4;
    const int col = col0 + 4 * (i & 3);
    const int ch = col >> 3, sub = (col & 7) * 2;
    const int r1 = krow0 + 4 * g + (i >> 2), r2 = r1 + 16;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, lds + tile_off(r1, ch) + sub));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, lds + tile_off(r2, ch) + sub));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
}

// Register fragment holding rows [16*(2s)+4g .. +3] and [16*(2s+1)+4g .. +3] of a 16x16 accumulator
// pair (accumulator row = (l>>4)*4 + r), i.e. the k order tr_frag uses.
__device__ __forceinline__ bf16x8 pack_p(const f32x4& a, const f32x4& b) {
    bf16x8 r;
    r[0] = f2bf(a[0]); r[1] = f2bf(a[1]); r[2] = f2bf(a[2]); r[3] = f2bf(a[3]);
    r[4] = f2bf(b[0]); r[5] = f2bf(b[1]); r[6] = f2bf(b[2]); r[7] = f2bf(b[3]);
    return r;
}

__device__ __forceinline__ bf16x8 load_frag_global(const __bf16* base, int ld, int row, int nrows, int col) {
    if (row < nrows) return *reinterpret_cast<const bf16x8*>(base + (size_t)row * ld + col);
    bf16x8 z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = f2bf(0.f);
    return z;
}

#define MFMA16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

struct AttnArgs {
    const __bf16 *q, *k, *v, *o, *dout;
    __bf16 *out, *dq, *dk, *dv;
    float *lse, *delta;
    int B, H, Sq, Sk;
    int ldq, ldk, ldv, ldo, lddo, lddq, lddk, lddv;
    float scale;
    // attention-probability dropout (src/model.py:142): the forward draws the keep bits (Philox,
    // common.h; row = (b·H + h)·Sq + q, col = key) and stores them, one u64 per (row, 64-key tile), bit
    // key mod 64 — the backward reads them back.  mbits == nullptr: no dropout.
    DropSite drop;
    uint64_t* mbits;
    int mwords;  // u64 words per row = ceil(Sk / 64)
    // MX-fp8 copy of the forward output (config 5): e4m3 [row][ldqm] and e8m0 scales in common.h's mx_sidx
    // layout (pitch qpitch rows), row = b·Sq + q; nullptr: none
    uint8_t *qmx, *qms;
    int ldqm, qpitch;
    // fused short backward (attn_bwd_short_kernel<.., GEMM_DO = true>): dO of head h is formed in the kernel as
    // dO = gA·Wᵀ over K_g (the residual branch's c_proj data gradient, src/model.py:245 — gA = the branch's output
    // gradient [B·Sq][lda_g], gW = the c_proj weight [H·64][ldw_g] (Conv1D [in, out], row i = dO column i)) instead of
    // being read from `dout`
    const __bf16* gA;
    const __bf16* gW;
    int lda_g, ldw_g, K_g;
    // fused cross-attention forward (attn_fwd_qgemm_kernel): Q of head h formed in the kernel as
    // bf16(gA·gW + gbias) over K_g (the query projection, src/model.py:311-329: gA = LN_x output [B·Sq][lda_g],
    // gW = the Conv1D weight [K_g][ldw_g], column h·64 + d), also stored to `q` for the backward
    const float* gbias;
};

// Dropout factor of one probability: 1/(1-p) kept, 0 dropped.
__device__ __forceinline__ float keep_scale(unsigned bits, int j, float scale) { return ((bits >> j) & 1u) ? scale : 0.f; }

constexpr float AT_LOG2E = 1.4426950408889634f;

// All-reduce over the 4 16-lane rows of a wave (lanes l, l^16, l^32, l^48) with the gfx950 row swaps
// (v_permlane16_swap / v_permlane32_swap: VALU, no LDS round trip as ds_bpermute would take).  Each
// swap of x with itself yields (x of the even row, x of the odd row) in every lane, so every lane
// combines the same two values in the same order.
__device__ __forceinline__ float rows_max(float x) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
    r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float rows_sum(float x) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    x = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// exp(scale·s − shift) given c = scale·log2e and shift2 = shift·log2e.
__device__ __forceinline__ float exp_sc(float s, float c, float shift2) {
    return __builtin_amdgcn_exp2f(fmaf(s, c, -shift2));
}

// One 64-key tile of the online-softmax forward for this lane's query q (keys key0..key0+63 of the
// staged sK / sV tiles): scores, running max / sum update, Oᵀ += Vᵀ·Pᵀ.  m is the running max of the
// RAW scores (before the 1/sqrt(d) scale).  MASK=false: every key of the tile is valid for every query
// of the wave.
// DROP: P·keep/(1-p) feeds the PV product (the row sum l stays undropped: softmax, then dropout), and
// the tile's keep bits of this lane's query are OR-combined over its 4 lane rows into *mword (the u64
// of (row, key tile); written by the g == 0 lanes).
template <bool CAUSAL, bool MASK, bool DROP>
__device__ __forceinline__ void fwd_kv_tile(const char* sK, const char* sV, int key0, int q, int Sk, float c,
                                            const bf16x8 (&qf)[2], f32x4 (&o)[4], float& m, float& l,
                                            const DropSite& drop, int64_t arow, uint64_t* mword) {
    const int g = (threadIdx.x & 63) >> 4;
    f32x4 s[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
        s[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
        s[kb] = MFMA16(row_frag(sK, kb * 16, 0), qf[0], s[kb]);
        s[kb] = MFMA16(row_frag(sK, kb * 16, 1), qf[1], s[kb]);
    }
    // s[kb][r] = score(key = key0 + kb*16 + 4g + r, query q)
    float mx = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float x = s[kb][r];
            if (MASK) {
                const int key = key0 + kb * 16 + 4 * g + r;
                const bool masked = key >= Sk || (CAUSAL && key > q);
                x = masked ? -INFINITY : x;
                s[kb][r] = x;
            }
            mx = fmaxf(mx, x);
        }
    mx = rows_max(mx);
    const float mnew = fmaxf(m, mx);
    const float m2 = (mnew == -INFINITY ? 0.f : mnew) * c;
    const float alpha = exp_sc(m, c, m2);
    float rs = 0.f;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float p = exp_sc(s[kb][r], c, m2);
            s[kb][r] = p;
            rs += p;
        }
    rs = rows_sum(rs);
    l = l * alpha + rs;
    m = mnew;
#pragma unroll
    for (int d = 0; d < 4; ++d) o[d] *= alpha;
    if constexpr (DROP) {
        uint32_t lo = 0, hi = 0;  // keys key0+0..31 / key0+32..63 of this query
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
            const unsigned kb4 = drop_keep4(drop, arow, key0 + kb * 16 + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r) s[kb][r] *= keep_scale(kb4, r, drop.scale);
            const uint32_t sh = (uint32_t)kb4 << (16 * (kb & 1) + 4 * g);
            if (kb < 2) lo |= sh;
            else hi |= sh;
        }
        auto r16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
        lo = r16[0] | r16[1];
        r16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
        hi = r16[0] | r16[1];
        auto r32 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
        lo = r32[0] | r32[1];
        r32 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
        hi = r32[0] | r32[1];
        if (g == 0 && mword) *mword = ((uint64_t)hi << 32) | lo;
    }
    // Oᵀ[d][q] += Σ_key V[key][d] P[q][key]
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        bf16x8 pb = pack_p(s[2 * half], s[2 * half + 1]);
#pragma unroll
        for (int d = 0; d < 4; ++d) o[d] = MFMA16(tr_frag(sV, 32 * half, d * 16), pb, o[d]);
    }
}

// Keys key0..key0+63 against the wave's queries qw0..qw0+15: does any pair need the mask?
template <bool CAUSAL>
__device__ __forceinline__ bool tile_masked(int key0, int Sk, int qw0) {
    return key0 + AT_T > Sk || (CAUSAL && key0 + AT_T - 1 > qw0);
}

template <bool CAUSAL, bool DROP>
__device__ __forceinline__ void fwd_tile(const char* sK, const char* sV, int key0, int q, int qw0, int Sk, float c,
                                         const bf16x8 (&qf)[2], f32x4 (&o)[4], float& m, float& l,
                                         const DropSite& drop, int64_t arow, uint64_t* mword) {
    if (tile_masked<CAUSAL>(key0, Sk, qw0))
        fwd_kv_tile<CAUSAL, true, DROP>(sK, sV, key0, q, Sk, c, qf, o, m, l, drop, arow, mword);
    else
        fwd_kv_tile<CAUSAL, false, DROP>(sK, sV, key0, q, Sk, c, qf, o, m, l, drop, arow, mword);
}

// Keep bits of (row, key) pairs stored by the forward: u64 word of (row, key tile), bit key mod 64.
__device__ __forceinline__ float stored_keep(const uint64_t* mrow, int key, float scale) {
    return ((mrow[key >> 6] >> (key & 63)) & 1ull) ? scale : 0.f;
}

// Normalised output row (bf16) and the log-sum-exp (natural log, scaled scores) of this lane's query.
__device__ __forceinline__ void fwd_store(const AttnArgs& a, int b, int h, int q, const f32x4 (&o)[4], float m,
                                          float l) {
    const int g = (threadIdx.x & 63) >> 4;
    const float inv = l > 0.f ? 1.0f / l : 0.f;
    if (a.qmx) {  // MX copy of the stored bf16 row: block 0 = dims 0-31 (d = 0, 1), block 1 = 32-63, each spread over
                  // the 4 lanes of this query (l, l^16, l^32, l^48); all lanes take part in the row reductions
        const bool live = q < a.Sq;
        const size_t row = (size_t)b * a.Sq + q;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            float v[2][4];
            float am = 0.f;
#pragma unroll
            for (int dd = 0; dd < 2; ++dd)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    v[dd][r] = live ? bf2f(f2bf(o[2 * half + dd][r] * inv)) : 0.f;
                    am = fmaxf(am, fabsf(v[dd][r]));
                }
            am = rows_max(am);
            const int eb = mx_exp_biased(am);
            const float is = mx_inv_scale(eb);
            if (live) {
#pragma unroll
                for (int dd = 0; dd < 2; ++dd)
                    *reinterpret_cast<uint32_t*>(a.qmx + row * a.ldqm + h * AT_D + (2 * half + dd) * 16 + 4 * g) =
                        mx_pack4(v[dd][0] * is, v[dd][1] * is, v[dd][2] * is, v[dd][3] * is);
                if (g == 0) a.qms[mx_sidx((int)row, 2 * h + half, a.qpitch)] = (uint8_t)eb;
            }
        }
    }
    if (q >= a.Sq) return;
    __bf16* Ob = a.out + ((size_t)b * a.Sq + q) * a.ldo + h * AT_D;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        bf16x4 w;
#pragma unroll
        for (int r = 0; r < 4; ++r) w[r] = f2bf(o[d][r] * inv);
        *reinterpret_cast<bf16x4*>(Ob + d * 16 + 4 * g) = w;
    }
    if (g == 0) a.lse[((size_t)b * a.H + h) * a.Sq + q] = m * a.scale + logf(l);
}

// dK/dV contribution of one 64-query tile (Q, dO, LSE, δ staged) for this lane's key: P recomputed,
// dS = P∘(dP − δ); dVᵀ += dOᵀ·Pᵀ, dKᵀ += Qᵀ·dSᵀ.  tS (optional): dS also stored key-major, bf16, at
// tile row krow (the fused short backward reuses it for dQ).  MASK=false: no pair of the tile is masked.
// Keep bits of the dropout backward (DROP): mcol points at the u64 word of (query q0, this lane's key
// tile); word of query q0 + i at mcol[i·mstride], bit kbit = key mod 64.  With dropout P̃ = P·Z
// (Z = keep/(1-p)) feeds dV, and dS = P∘(dP̃∘Z − δ) (δ = rowsum(dO∘O) is unchanged).
struct DropBits {
    const uint64_t* mcol;
    int mstride, kbit;
    float scale;
};

template <bool CAUSAL, bool MASK, bool DROP, bool PRE = false>
__device__ __forceinline__ void dkv_tile(const char* sQ, const char* sdO, const float* sL, const float* sD, int q0,
                                         int key, int Sq, int Sk, float c, const bf16x8 (&kf)[2],
                                         const bf16x8 (&vf)[2], f32x4 (&dk)[4], f32x4 (&dv)[4], char* tS, int krow,
                                         const DropBits& db) {
    const int g = (threadIdx.x & 63) >> 4;
    f32x4 p[4], ds[4];
#pragma unroll
    for (int qb = 0; qb < 4; ++qb) {
        f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
        s = MFMA16(row_frag(sQ, qb * 16, 0), kf[0], s);
        s = MFMA16(row_frag(sQ, qb * 16, 1), kf[1], s);
        f32x4 dp = f32x4{0.f, 0.f, 0.f, 0.f};
        dp = MFMA16(row_frag(sdO, qb * 16, 0), vf[0], dp);
        dp = MFMA16(row_frag(sdO, qb * 16, 1), vf[1], dp);
        // element r: query q0 + qb*16 + 4g + r, key `key`
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int ql = qb * 16 + 4 * g + r;
            float pv = exp_sc(s[r], c, PRE ? sL[ql] : sL[ql] * AT_LOG2E);  // PRE: sL holds LSE·log2e (short kernel)
            if (MASK) {
                const int qq = q0 + ql;
                const bool masked = qq >= Sq || key >= Sk || (CAUSAL && key > qq);
                pv = masked ? 0.f : pv;
            }
            if constexpr (DROP) {
                // PRE (the short kernel): its staged keep bits are zero past Sq, so the word is read unguarded
                const float z = (PRE || q0 + ql < Sq)
                                    ? (((db.mcol[(size_t)ql * db.mstride] >> db.kbit) & 1ull) ? db.scale : 0.f)
                                    : 0.f;
                p[qb][r] = pv * z;
                ds[qb][r] = pv * (dp[r] * z - sD[ql]);
            } else {
                p[qb][r] = pv;
                ds[qb][r] = pv * (dp[r] - sD[ql]);
            }
        }
        if (tS) {  // dS[key][q..q+3] -> key-major LDS tile (one 8-byte store per lane)
            bf16x4 w;
#pragma unroll
            for (int r = 0; r < 4; ++r) w[r] = f2bf(ds[qb][r]);
            const int qc = qb * 16 + 4 * g;  // query column inside the tile
            *reinterpret_cast<bf16x4*>(tS + tile_off(krow, qc >> 3) + (qc & 7) * 2) = w;
        }
    }
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        bf16x8 pb = pack_p(p[2 * half], p[2 * half + 1]);
        bf16x8 sb = pack_p(ds[2 * half], ds[2 * half + 1]);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            dv[d] = MFMA16(tr_frag(sdO, 32 * half, d * 16), pb, dv[d]);
            dk[d] = MFMA16(tr_frag(sQ, 32 * half, d * 16), sb, dk[d]);
        }
    }
}

// Queries q0..q0+63 against the wave's keys kw0..kw0+15: does any pair need the mask?
template <bool CAUSAL>
__device__ __forceinline__ bool dkv_masked(int q0, int Sq, int kw0, int Sk) {
    return q0 + AT_T > Sq || kw0 + 16 > Sk || (CAUSAL && kw0 + 15 > q0);
}

template <bool CAUSAL, bool DROP, bool PRE = false>
__device__ __forceinline__ void dkv_step(const char* sQ, const char* sdO, const float* sL, const float* sD, int q0,
                                         int key, int kw0, int Sq, int Sk, float c, const bf16x8 (&kf)[2],
                                         const bf16x8 (&vf)[2], f32x4 (&dk)[4], f32x4 (&dv)[4], char* tS, int krow,
                                         const DropBits& db) {
    if (dkv_masked<CAUSAL>(q0, Sq, kw0, Sk))
        dkv_tile<CAUSAL, true, DROP, PRE>(sQ, sdO, sL, sD, q0, key, Sq, Sk, c, kf, vf, dk, dv, tS, krow, db);
    else
        dkv_tile<CAUSAL, false, DROP, PRE>(sQ, sdO, sL, sD, q0, key, Sq, Sk, c, kf, vf, dk, dv, tS, krow, db);
}

// dQ contribution of one 64-key tile for this lane's query (lq2 = LSE·log2e, dl = δ).  DROP: mword =
// the stored keep bits of (this query, this key tile).
template <bool CAUSAL, bool MASK, bool DROP>
__device__ __forceinline__ void dq_tile(const char* sK, const char* sV, int key0, int q, int Sq, int Sk, float c,
                                        float lq2, float dl, const bf16x8 (&qf)[2], const bf16x8 (&dof)[2],
                                        f32x4 (&dq)[4], uint64_t mword, float dscale) {
    const int g = (threadIdx.x & 63) >> 4;
    f32x4 ds[4];
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
        f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
        s = MFMA16(row_frag(sK, kb * 16, 0), qf[0], s);
        s = MFMA16(row_frag(sK, kb * 16, 1), qf[1], s);
        f32x4 dp = f32x4{0.f, 0.f, 0.f, 0.f};
        dp = MFMA16(row_frag(sV, kb * 16, 0), dof[0], dp);
        dp = MFMA16(row_frag(sV, kb * 16, 1), dof[1], dp);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float pv = exp_sc(s[r], c, lq2);
            if (MASK) {
                const int key = key0 + kb * 16 + 4 * g + r;
                const bool masked = key >= Sk || q >= Sq || (CAUSAL && key > q);
                pv = masked ? 0.f : pv;
            }
            if constexpr (DROP) {
                const float z = ((mword >> (kb * 16 + 4 * g + r)) & 1ull) ? dscale : 0.f;
                ds[kb][r] = pv * (dp[r] * z - dl);
            } else {
                ds[kb][r] = pv * (dp[r] - dl);
            }
        }
    }
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        bf16x8 sb = pack_p(ds[2 * half], ds[2 * half + 1]);
#pragma unroll
        for (int d = 0; d < 4; ++d) dq[d] = MFMA16(tr_frag(sK, 32 * half, d * 16), sb, dq[d]);
    }
}

// Tile of a tiled-kernel workgroup, XCD-aware: workgroups are dispatched round-robin over the 8 XCDs
// (linear id mod 8), so the (b, h) pairs are split into 8 contiguous groups, one per XCD, and all row
// blocks of a pair run on the XCD whose L2 holds that pair's K/V (or Q/dO); within an XCD, row block 0
// of every pair is dispatched first (callers map it to the longest causal rows).
struct AttnBlock {
    int x, h, b;
};
__device__ __forceinline__ AttnBlock attn_block() {
    const int nx = gridDim.x, P = gridDim.y * gridDim.z;
    AttnBlock r;
    if ((P & 7) == 0) {
        const int L = blockIdx.x + nx * (blockIdx.y + gridDim.y * blockIdx.z);
        const int per = P >> 3, j = L >> 3;
        const int pair = (L & 7) * per + j % per;
        r.x = j / per;
        r.h = pair % gridDim.y;
        r.b = pair / gridDim.y;
    } else {
        r.x = blockIdx.x;
        r.h = blockIdx.y;
        r.b = blockIdx.z;
    }
    return r;
}

using AttnTile = GldsTile<AT_T, false, 4>;      // one 64x64 bf16 tile: 2 LDS-DMA wave-instructions per wave

// Make the compiler wait for a register operand loaded before the ring prologue: its own vmcnt wait then
// sits here, not inside the loop (where it would drain the untracked LDS-DMA ring every iteration).
__device__ __forceinline__ void vm_ready(const bf16x8& x) {
    typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
    asm volatile("" ::"v"(__builtin_bit_cast(u32x4, x)));
}
__device__ __forceinline__ void vm_ready(float x) { asm volatile("" ::"v"(x)); }

// Ring step: wait until this wave's DMA for the current stage landed (`after` younger stages may stay in
// flight), finish this wave's LDS reads of the slot about to be refilled, then one workgroup barrier.
template <int LPS, int NS>
__device__ __forceinline__ void ring_sync(int after) {
    wait_stages<LPS, NS - 2>(after);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

template <bool CAUSAL, int NS, bool DROP>
__global__ __launch_bounds__(256, DROP ? 3 : 4) void attn_fwd_kernel(AttnArgs a) {
    __shared__ __attribute__((aligned(16))) char ring[NS * 2 * AT_TILE_BYTES];  // [stage][K|V]
    const AttnBlock blk = attn_block();
    const int b = blk.b, h = blk.h;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int i16 = lane & 15, g = lane >> 4;
    const int qblk = (CAUSAL ? gridDim.x - 1 - blk.x : blk.x) * AT_T;
    const int q = qblk + wave * 16 + i16;  // this lane's query
    const float c = a.scale * AT_LOG2E;
    const __bf16* Qb = a.q + (size_t)b * a.Sq * a.ldq + h * AT_D;
    const __bf16* Kb = a.k + (size_t)b * a.Sk * a.ldk + h * AT_D;
    const __bf16* Vb = a.v + (size_t)b * a.Sk * a.ldv + h * AT_D;

    // Qᵀ as the B operand: lane l needs Q[q][32ks + 8g + j]
    bf16x8 qf[2];
    qf[0] = load_frag_global(Qb, a.ldq, q, a.Sq, 8 * g);
    qf[1] = load_frag_global(Qb, a.ldq, q, a.Sq, 32 + 8 * g);
    vm_ready(qf[0]);
    vm_ready(qf[1]);

    f32x4 o[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, l = 0.f;

    int nkt = (a.Sk + AT_T - 1) / AT_T;
    if (CAUSAL) {
        int qlast = min(a.Sq, qblk + AT_T) - 1;
        nkt = min(nkt, qlast / AT_T + 1);
    }
    auto issue = [&](int kt) {
        char* st = ring + (kt % NS) * 2 * AT_TILE_BYTES;
        AttnTile::issue(st, Kb, a.ldk, kt * AT_T, a.Sk, 0, wave);
        AttnTile::issue(st + AT_TILE_BYTES, Vb, a.ldv, kt * AT_T, a.Sk, 0, wave);
    };
    const int64_t arow = ((int64_t)b * a.H + h) * a.Sq + q;  // dropout row of this lane's query
    uint64_t* mrow = DROP && q < a.Sq ? a.mbits + arow * a.mwords : nullptr;
    for (int s = 0; s < NS - 1 && s < nkt; ++s) issue(s);
    for (int kt = 0; kt < nkt; ++kt) {
        ring_sync<4, NS>(min(NS - 2, nkt - 1 - kt));
        if (kt + NS - 1 < nkt) issue(kt + NS - 1);
        const char* st = ring + (kt % NS) * 2 * AT_TILE_BYTES;
        fwd_tile<CAUSAL, DROP>(st, st + AT_TILE_BYTES, kt * AT_T, q, qblk + wave * 16, a.Sk, c, qf, o, m, l, a.drop,
                               arow, mrow ? mrow + kt : nullptr);
    }
    fwd_store(a, b, h, q, o, m, l);
}

// Cross-attention forward with the query projection inside (non-causal): the workgroup of (query block, h, b)
// first forms its 64 x 64 Q tile = bf16(LN_x rows · Wq[:, h·64 ..] + bias) on its 4 waves (2 x 2 grid of 32 x 32,
// 64-deep K steps through a 3-stage LDS-DMA ring: the product order of the GEMM's 64x64 configuration, so Q is
// bitwise the q GEMM's output), stores it (the backward's operand) and stages it in LDS for the Q fragments, then
// runs attn_fwd_kernel's key loop over the same ring.  One launch and one Q round trip fewer per block and chain on
// the forward, which is latency-bound (profiles/r04_experiments.txt #10).
constexpr int QG_STAGES = 3;
constexpr int QG_STAGE = 2 * AT_TILE_BYTES;  // A 64 x 64 + W 64 x 64 (bf16)

template <int NS, bool DROP>
__global__ __launch_bounds__(256, 2) void attn_fwd_qgemm_kernel(AttnArgs a) {
    constexpr int RING = QG_STAGES * QG_STAGE > NS * 2 * AT_TILE_BYTES ? QG_STAGES * QG_STAGE : NS * 2 * AT_TILE_BYTES;
    __shared__ __attribute__((aligned(16))) char ring[RING];
    __shared__ __attribute__((aligned(16))) char sQ[AT_TILE_BYTES];
    const AttnBlock blk = attn_block();
    const int b = blk.b, h = blk.h;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int i16 = lane & 15, g = lane >> 4;
    const int qblk = blk.x * AT_T;
    const int q = qblk + wave * 16 + i16;  // this lane's query
    const float c = a.scale * AT_LOG2E;
    {
        using TA = GldsTile<AT_T, false, 4>;  // LN_x rows, k contiguous
        using TW = GldsTile<AT_D, true, 4>;   // Wq [k][n]: n contiguous
        constexpr int LPS = TA::PER_WAVE + TW::PER_WAVE;
        const __bf16* gA = a.gA + (size_t)b * a.Sq * a.lda_g;
        const int nk = a.K_g / GEMM_BK;
        auto issue = [&](int kt) {
            char* st = ring + (kt % QG_STAGES) * QG_STAGE;
            TA::issue(st, gA, a.lda_g, qblk, a.Sq, kt * GEMM_BK, wave);
            TW::issue(st + AT_TILE_BYTES, a.gW, a.ldw_g, h * AT_D, a.H * AT_D, kt * GEMM_BK, wave);
        };
        for (int s = 0; s < QG_STAGES - 1 && s < nk; ++s) issue(s);
        const int wm = wave >> 1, wn = wave & 1;
        FragReader<AT_T, false> fa_r;
        FragReader<AT_D, true> fb_r;
        f32x4 acc[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int kt = 0; kt < nk; ++kt) {
            wait_stages<LPS, QG_STAGES - 2>(min(QG_STAGES - 2, nk - 1 - kt));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if (kt + QG_STAGES - 1 < nk) issue(kt + QG_STAGES - 1);
            const char* st = ring + (kt % QG_STAGES) * QG_STAGE;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                bf16x8 fa[2], fb[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) fa[i] = fa_r.frag(st, wm * 32 + i * 16, ks);
#pragma unroll
                for (int j = 0; j < 2; ++j) fb[j] = fb_r.frag(st + AT_TILE_BYTES, wn * 32 + j * 16, ks);
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[i][j] = MFMA16(fa[i], fb[j], acc[i][j]);
            }
        }
        // Q = bf16(acc + bias) (the GEMM's EPI_BIAS arithmetic): to the global q (rows < Sq) and the LDS tile
        // (rows >= Sq zero, as attn_fwd_kernel loads them)
        __bf16* Qg = const_cast<__bf16*>(a.q) + ((size_t)b * a.Sq + qblk) * a.ldq + h * AT_D;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int col = wn * 32 + j * 16 + i16;
                const float bias = a.gbias[h * AT_D + col];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = wm * 32 + i * 16 + 4 * g + r;
                    const bool live = qblk + row < a.Sq;
                    const __bf16 v = f2bf(acc[i][j][r] + bias);
                    if (live) Qg[(size_t)row * a.ldq + col] = v;
                    *reinterpret_cast<__bf16*>(sQ + tile_off(row, col >> 3) + (col & 7) * 2) = live ? v : f2bf(0.f);
                }
            }
        __syncthreads();  // Q staged; every wave is done with the GEMM's ring
    }
    bf16x8 qf[2];
    qf[0] = row_frag(sQ, wave * 16, 0);
    qf[1] = row_frag(sQ, wave * 16, 1);

    const __bf16* Kb = a.k + (size_t)b * a.Sk * a.ldk + h * AT_D;
    const __bf16* Vb = a.v + (size_t)b * a.Sk * a.ldv + h * AT_D;
    f32x4 o[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, l = 0.f;
    const int nkt = (a.Sk + AT_T - 1) / AT_T;
    auto issue = [&](int kt) {
        char* st = ring + (kt % NS) * 2 * AT_TILE_BYTES;
        AttnTile::issue(st, Kb, a.ldk, kt * AT_T, a.Sk, 0, wave);
        AttnTile::issue(st + AT_TILE_BYTES, Vb, a.ldv, kt * AT_T, a.Sk, 0, wave);
    };
    const int64_t arow = ((int64_t)b * a.H + h) * a.Sq + q;  // dropout row of this lane's query
    uint64_t* mrow = DROP && q < a.Sq ? a.mbits + arow * a.mwords : nullptr;
    for (int s = 0; s < NS - 1 && s < nkt; ++s) issue(s);
    for (int kt = 0; kt < nkt; ++kt) {
        ring_sync<4, NS>(min(NS - 2, nkt - 1 - kt));
        if (kt + NS - 1 < nkt) issue(kt + NS - 1);
        const char* st = ring + (kt % NS) * 2 * AT_TILE_BYTES;
        fwd_tile<false, DROP>(st, st + AT_TILE_BYTES, kt * AT_T, q, qblk + wave * 16, a.Sk, c, qf, o, m, l, a.drop, arow,
                              mrow ? mrow + kt : nullptr);
    }
    fwd_store(a, b, h, q, o, m, l);
}

// δ[b,h,q] = Σ_d dO·O: 4 threads per (token, head), 16 dims each, partials combined (p0+p1)+(p2+p3) —
// the order attn_bwd_short_kernel uses, so both backward paths see bit-identical δ.
__global__ __launch_bounds__(256) void attn_delta_kernel(AttnArgs a) {
    const size_t n = (size_t)a.B * a.Sq * a.H * 4;
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const int part = (int)(i & 3);
    const size_t row = i >> 2;  // (b*Sq + q)*H + h
    const int h = (int)(row % a.H);
    const size_t tok = row / a.H;
    float s = 0.f;
    if (i < n) {
        const __bf16* dd = a.dout + tok * a.lddo + h * AT_D + part * 16;
        const __bf16* od = a.o + tok * a.ldo + h * AT_D + part * 16;
        const bf16x8 x0 = *reinterpret_cast<const bf16x8*>(dd), x1 = *reinterpret_cast<const bf16x8*>(dd + 8);
        const bf16x8 y0 = *reinterpret_cast<const bf16x8*>(od), y1 = *reinterpret_cast<const bf16x8*>(od + 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) s += bf2f(x0[j]) * bf2f(y0[j]);
#pragma unroll
        for (int j = 0; j < 8; ++j) s += bf2f(x1[j]) * bf2f(y1[j]);
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (i < n && part == 0) {
        const int bb = (int)(tok / a.Sq), q = (int)(tok % a.Sq);
        a.delta[((size_t)bb * a.H + h) * a.Sq + q] = s;
    }
}

// dK, dV: workgroup = 64 keys of one (b, h), each wave 16 keys; loop over query tiles.  A ring stage holds
// the Q and dO tiles and the tile's 64 LSE and δ values (one 256-B DMA per wave: waves 0/2 LSE, 1/3 δ).
template <bool CAUSAL, int NS, bool DROP>
__global__ __launch_bounds__(256, DROP ? 2 : 3) void attn_bwd_dkv_kernel(AttnArgs a) {
    constexpr int STAGE = 2 * AT_TILE_BYTES + 4 * AT_T * 4;
    __shared__ __attribute__((aligned(16))) char ring[NS * STAGE];
    const AttnBlock blk = attn_block();
    const int b = blk.b, h = blk.h;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int i16 = lane & 15, g = lane >> 4;
    const int kblk = blk.x * AT_T;
    const int key = kblk + wave * 16 + i16;  // this lane's key (MFMA n index)
    const __bf16* Qb = a.q + (size_t)b * a.Sq * a.ldq + h * AT_D;
    const __bf16* dOb = a.dout + (size_t)b * a.Sq * a.lddo + h * AT_D;
    const __bf16* Kb = a.k + (size_t)b * a.Sk * a.ldk + h * AT_D;
    const __bf16* Vb = a.v + (size_t)b * a.Sk * a.ldv + h * AT_D;
    const float* rowv = ((wave & 1) ? a.delta : a.lse) + ((size_t)b * a.H + h) * a.Sq;
    const float c = a.scale * AT_LOG2E;

    // Kᵀ / Vᵀ as B operands: lane l needs K[key][32ks + 8g + j]
    bf16x8 kf[2], vf[2];
    kf[0] = load_frag_global(Kb, a.ldk, key, a.Sk, 8 * g);
    kf[1] = load_frag_global(Kb, a.ldk, key, a.Sk, 32 + 8 * g);
    vf[0] = load_frag_global(Vb, a.ldv, key, a.Sk, 8 * g);
    vf[1] = load_frag_global(Vb, a.ldv, key, a.Sk, 32 + 8 * g);
    vm_ready(kf[0]); vm_ready(kf[1]); vm_ready(vf[0]); vm_ready(vf[1]);

    f32x4 dk[4], dv[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        dk[d] = f32x4{0.f, 0.f, 0.f, 0.f};
        dv[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const int qt0 = CAUSAL ? kblk / AT_T : 0;
    const int n = (a.Sq + AT_T - 1) / AT_T - qt0;  // query tiles of this workgroup
    auto issue = [&](int i) {
        char* st = ring + (i % NS) * STAGE;
        const int q0 = (qt0 + i) * AT_T;
        AttnTile::issue(st, Qb, a.ldq, q0, a.Sq, 0, wave);
        AttnTile::issue(st + AT_TILE_BYTES, dOb, a.lddo, q0, a.Sq, 0, wave);
        glds4(rowv + min(q0 + lane, a.Sq - 1),
              __builtin_amdgcn_readfirstlane(lds_addr_of(st + 2 * AT_TILE_BYTES + wave * AT_T * 4)));
    };
    // dropout keep bits of this workgroup's key tile for every query (u64 per query), staged in LDS
    // before the ring starts (a plain load inside the loop would make the compiler drain the untracked
    // LDS-DMA ring at every use)
    __shared__ uint64_t smask[DROP ? AT_MAX_SQ_DROP : 1];
    if constexpr (DROP) {
        const uint64_t* src = a.mbits + ((size_t)b * a.H + h) * a.Sq * a.mwords + blk.x;
        for (int i = threadIdx.x; i < a.Sq; i += 256) smask[i] = src[(size_t)i * a.mwords];
        __syncthreads();
    }
    for (int s = 0; s < NS - 1 && s < n; ++s) issue(s);
    DropBits db{nullptr, 1, key & 63, a.drop.scale};
    for (int i = 0; i < n; ++i) {
        ring_sync<5, NS>(min(NS - 2, n - 1 - i));
        if (i + NS - 1 < n) issue(i + NS - 1);
        const char* sQ = ring + (i % NS) * STAGE;
        const char* sdO = sQ + AT_TILE_BYTES;
        const float* sL = reinterpret_cast<const float*>(sQ + 2 * AT_TILE_BYTES);
        const float* sD = sL + AT_T;
        if (DROP) db.mcol = smask + (qt0 + i) * AT_T;
        dkv_step<CAUSAL, DROP>(sQ, sdO, sL, sD, (qt0 + i) * AT_T, key, kblk + wave * 16, a.Sq, a.Sk, c, kf, vf, dk, dv,
                               nullptr, 0, db);
    }
    if (key < a.Sk) {
        size_t tok = (size_t)b * a.Sk + key;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            bf16x4 wk, wv;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                wk[r] = f2bf(dk[d][r] * a.scale);
                wv[r] = f2bf(dv[d][r]);
            }
            *reinterpret_cast<bf16x4*>(a.dk + tok * a.lddk + h * AT_D + d * 16 + 4 * g) = wk;
            *reinterpret_cast<bf16x4*>(a.dv + tok * a.lddv + h * AT_D + d * 16 + 4 * g) = wv;
        }
    }
}

// dQ: workgroup = 64 queries, each wave 16 queries; loop over key tiles (K, V through the ring).
template <bool CAUSAL, int NS, bool DROP>
__global__ __launch_bounds__(256) void attn_bwd_dq_kernel(AttnArgs a) {
    __shared__ __attribute__((aligned(16))) char ring[NS * 2 * AT_TILE_BYTES];
    const AttnBlock blk = attn_block();
    const int b = blk.b, h = blk.h;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int i16 = lane & 15, g = lane >> 4;
    const int qblk = (CAUSAL ? gridDim.x - 1 - blk.x : blk.x) * AT_T;
    const int q = qblk + wave * 16 + i16;
    const __bf16* Qb = a.q + (size_t)b * a.Sq * a.ldq + h * AT_D;
    const __bf16* dOb = a.dout + (size_t)b * a.Sq * a.lddo + h * AT_D;
    const __bf16* Kb = a.k + (size_t)b * a.Sk * a.ldk + h * AT_D;
    const __bf16* Vb = a.v + (size_t)b * a.Sk * a.ldv + h * AT_D;
    const size_t sidx = ((size_t)b * a.H + h) * a.Sq + q;
    const float lq = q < a.Sq ? a.lse[sidx] : 0.f;
    const float dq_delta = q < a.Sq ? a.delta[sidx] : 0.f;
    const float c = a.scale * AT_LOG2E, lq2 = lq * AT_LOG2E;

    bf16x8 qf[2], dof[2];
    qf[0] = load_frag_global(Qb, a.ldq, q, a.Sq, 8 * g);
    qf[1] = load_frag_global(Qb, a.ldq, q, a.Sq, 32 + 8 * g);
    dof[0] = load_frag_global(dOb, a.lddo, q, a.Sq, 8 * g);
    dof[1] = load_frag_global(dOb, a.lddo, q, a.Sq, 32 + 8 * g);
    vm_ready(qf[0]); vm_ready(qf[1]); vm_ready(dof[0]); vm_ready(dof[1]);
    vm_ready(lq); vm_ready(dq_delta);

    f32x4 dq[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    int nkt = (a.Sk + AT_T - 1) / AT_T;
    if (CAUSAL) {
        int qlast = min(a.Sq, qblk + AT_T) - 1;
        nkt = min(nkt, qlast / AT_T + 1);
    }
    auto issue = [&](int kt) {
        char* st = ring + (kt % NS) * 2 * AT_TILE_BYTES;
        AttnTile::issue(st, Kb, a.ldk, kt * AT_T, a.Sk, 0, wave);
        AttnTile::issue(st + AT_TILE_BYTES, Vb, a.ldv, kt * AT_T, a.Sk, 0, wave);
    };
    // dropout keep bits of the workgroup's 64 queries (mwords u64 each), staged in LDS before the ring
    __shared__ uint64_t smask[DROP ? AT_MAX_SQ_DROP : 1];
    if constexpr (DROP) {
        const uint64_t* src = a.mbits + (((size_t)b * a.H + h) * a.Sq + qblk) * a.mwords;
        const int nw = (min(a.Sq, qblk + AT_T) - qblk) * a.mwords;
        for (int i = threadIdx.x; i < nw; i += 256) smask[i] = src[i];
        __syncthreads();
    }
    for (int s = 0; s < NS - 1 && s < nkt; ++s) issue(s);
    for (int kt = 0; kt < nkt; ++kt) {
        ring_sync<4, NS>(min(NS - 2, nkt - 1 - kt));
        if (kt + NS - 1 < nkt) issue(kt + NS - 1);
        const char* sK = ring + (kt % NS) * 2 * AT_TILE_BYTES;
        const char* sV = sK + AT_TILE_BYTES;
        const int key0 = kt * AT_T;
        const uint64_t mw = DROP && q < a.Sq ? smask[(q - qblk) * a.mwords + kt] : 0ull;
        if (tile_masked<CAUSAL>(key0, a.Sk, qblk + wave * 16) || qblk + wave * 16 + 16 > a.Sq)
            dq_tile<CAUSAL, true, DROP>(sK, sV, key0, q, a.Sq, a.Sk, c, lq2, dq_delta, qf, dof, dq, mw, a.drop.scale);
        else
            dq_tile<CAUSAL, false, DROP>(sK, sV, key0, q, a.Sq, a.Sk, c, lq2, dq_delta, qf, dof, dq, mw, a.drop.scale);
    }
    if (q < a.Sq) {
        __bf16* out = a.dq + ((size_t)b * a.Sq + q) * a.lddq + h * AT_D;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            bf16x4 w;
#pragma unroll
            for (int r = 0; r < 4; ++r) w[r] = f2bf(dq[d][r] * a.scale);
            *reinterpret_cast<bf16x4*>(out + d * 16 + 4 * g) = w;
        }
    }
}

// ---- short sequences (Sq, Sk <= 128): the whole backward of one (b, h) in one workgroup ----------
// 8 waves.  Q, dO, K, V (up to 128 rows each) are staged in LDS once; δ and the LSE per query too.
// Phase 1 (keys-major): wave w owns keys 16w..16w+15 and accumulates dK, dV over every query, as
// attn_bwd_dkv_kernel does, and also stores its dS (bf16) key-major into LDS.  Phase 2 (queries-
// major): wave w owns queries 16w..16w+15: dQᵀ = Kᵀ·dSᵀ, both operands read transposed from LDS.
// One launch instead of two, no re-staging of Q/dO per key tile, no recomputation of P for dQ.
constexpr int AS_MAX = 128;                          // max Sq / Sk of the fused path
constexpr int AS_TILES = AS_MAX / AT_T;              // 64-row tiles per operand
constexpr int AS_OPER = AS_TILES * AT_TILE_BYTES;    // 16 KiB per staged operand
// LDS: Q, dO, K, V staged, the dS tiles [key][query], then LSE, δ and the dropout keep bits of the (b, h)
// ([query][AS_TILES] u64): 99 KiB.  (Placing the dS tiles over V's staging — dead once every wave holds its V
// fragments — brings it to 83 KiB, room beside one 64-KiB GEMM tile of the concurrent weight-gradient stream; the
// co-residency measured level at C2 and -1.5 % at C5, profiles/r04_experiments.txt #13.)
constexpr int AS_DS = AS_TILES * AS_TILES * AT_TILE_BYTES;  // 32 KiB
constexpr int AS_SMALL = 2 * AS_MAX * 4 + AS_MAX * AS_TILES * 8;  // LSE, δ, keep bits: 3 KiB
constexpr int AS_LDS = AS_SMALL + 4 * AS_OPER + AS_DS;

// 128 rows x 64 dims of a token-major operand as two swizzled 64-row tiles (rows >= nrows are zero):
// the loads are issued first (2 x 16 B per thread), then written to LDS, so several staged operands
// can have all their loads in flight together (load_rows ... load_rows, then put_rows ...).
struct Rows128 {
    uint4 v[2];
};
__device__ __forceinline__ Rows128 load_rows(const __bf16* base, int ld, int nrows) {
    Rows128 r;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int c = threadIdx.x + i * 512, row = c >> 3, ch = c & 7;
        r.v[i] = row < nrows ? *reinterpret_cast<const uint4*>(base + (size_t)row * ld + ch * 8) : make_uint4(0, 0, 0, 0);
    }
    return r;
}
__device__ __forceinline__ void put_rows(char* lds, const Rows128& r) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int c = threadIdx.x + i * 512, row = c >> 3, ch = c & 7;
        *reinterpret_cast<uint4*>(lds + (row >> 6) * AT_TILE_BYTES + tile_off(row & 63, ch)) = r.v[i];
    }
}

// GEMM_DO: the fused form.  dO [Sq][64] of (b, h) = gA[b·Sq ..][0, K_g) · gW[h·64 ..][0, K_g)ᵀ on the 8 waves (4 x 2
// grid of 32 x 32, v_mfma_f32_16x16x32_bf16, 64-deep K steps through a 2-stage LDS-DMA ring, the same product order as
// ergm_gemm, so dO is bitwise the c_proj data-gradient GEMM's bf16 output) while Q, K, V and O are loaded, then
// rounded to bf16 straight into the staged dO tiles — one launch and one HBM round trip fewer on the backward's
// critical chain, and dO never goes to memory.  The 3-stage ring occupies the dO, dS, K and V staging (72 of 80 KiB):
// K and V are held in registers over the GEMM and staged after it, and the dO tiles are written once every wave has
// left the ring, so the fused form needs no more LDS than the plain one.
constexpr int AS_GA = AS_MAX * GEMM_BK * 2;            // 16 KiB: a 128 x 64 gA stage
constexpr int AS_GW = AT_D * GEMM_BK * 2;              // 8 KiB: a 64 x 64 gW stage
constexpr int AS_GSTAGES = 3;
constexpr int AS_RING = AS_GSTAGES * (AS_GA + AS_GW);  // 72 KiB
static_assert(AS_RING <= 3 * AS_OPER + AS_DS, "the GEMM ring fits over the dO, dS, K and V staging");

template <bool CAUSAL, bool DROP, bool GEMM_DO = false>
__global__ __launch_bounds__(512) void attn_bwd_short_kernel(AttnArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // the per-query arrays first and the most-read tiles next, so their accesses stay within the 64-KiB reach of
    // the ds_read / ds_write immediate offset (no per-access address arithmetic)
    float* sL = reinterpret_cast<float*>(smem);        // LSE·log2e per query
    float* sD = sL + AS_MAX;                           // δ per query
    uint64_t* sM = reinterpret_cast<uint64_t*>(sD + AS_MAX);  // dropout keep bits [query][AS_TILES]
    char* sQ = smem + AS_SMALL;
    char* sdO = sQ + AS_OPER;
    char* sdS = sdO + AS_OPER;                         // tile (kt, qt) at (kt*2 + qt)*8 KiB, [key][query]
    char* sK = sdS + AS_DS;
    char* sV = sK + AS_OPER;
    const int b = blockIdx.z, h = blockIdx.y;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int i16 = lane & 15, g = lane >> 4;
    const __bf16* Qb = a.q + (size_t)b * a.Sq * a.ldq + h * AT_D;
    const __bf16* dOb = a.dout + (size_t)b * a.Sq * a.lddo + h * AT_D;
    const __bf16* Kb = a.k + (size_t)b * a.Sk * a.ldk + h * AT_D;
    const __bf16* Vb = a.v + (size_t)b * a.Sk * a.ldv + h * AT_D;
    if constexpr (GEMM_DO) {
        using TA = GldsTile<AS_MAX, false, 8>;
        using TW = GldsTile<AT_D, false, 8>;
        constexpr int LPS = TA::PER_WAVE + TW::PER_WAVE;
        char* ring = sdO;
        const __bf16* gA = a.gA + (size_t)b * a.Sq * a.lda_g;
        const int nk = a.K_g / GEMM_BK;
        auto issue = [&](int kt) {
            char* st = ring + (kt % AS_GSTAGES) * (AS_GA + AS_GW);
            TA::issue(st, gA, a.lda_g, 0, a.Sq, kt * GEMM_BK, wave);
            TW::issue(st + AS_GA, a.gW, a.ldw_g, h * AT_D, a.H * AT_D, kt * GEMM_BK, wave);
        };
        for (int s0 = 0; s0 < AS_GSTAGES - 1 && s0 < nk; ++s0) issue(s0);
        // Q, K, V rows, O for δ and the LSE / keep bits, all in flight beside the GEMM's first stage
        const Rows128 rq = load_rows(Qb, a.ldq, a.Sq);
        const Rows128 rk = load_rows(Kb, a.ldk, a.Sk);
        const Rows128 rv = load_rows(Vb, a.ldv, a.Sk);
        uint64_t mv = 0;
        if constexpr (DROP) {
            const int qq = threadIdx.x / AS_TILES, w = threadIdx.x % AS_TILES;
            if (qq < a.Sq && w < a.mwords) mv = a.mbits[(((size_t)b * a.H + h) * a.Sq + qq) * a.mwords + w];
        }
        const int ql = threadIdx.x >> 2, part = threadIdx.x & 3;
        bf16x8 y0, y1;
        float lse = 0.f;
        if (ql < a.Sq) {
            const __bf16* od = a.o + ((size_t)b * a.Sq + ql) * a.ldo + h * AT_D + part * 16;
            y0 = *reinterpret_cast<const bf16x8*>(od);
            y1 = *reinterpret_cast<const bf16x8*>(od + 8);
            lse = a.lse[((size_t)b * a.H + h) * a.Sq + ql];
        }
        put_rows(sQ, rq);
        if (DROP && threadIdx.x < AS_MAX * AS_TILES) sM[threadIdx.x] = mv;
        // dO = gA·gWᵀ: wave (wm, wn) owns rows 32wm.., columns 32wn.. of the 128 x 64 tile
        const int wm = wave >> 1, wn = wave & 1;
        FragReader<AS_MAX, false> fa_r;
        FragReader<AT_D, false> fb_r;
        f32x4 acc[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int kt = 0; kt < nk; ++kt) {
            wait_stages<LPS, AS_GSTAGES - 2>(min(AS_GSTAGES - 2, nk - 1 - kt));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if (kt + AS_GSTAGES - 1 < nk) issue(kt + AS_GSTAGES - 1);
            const char* st = ring + (kt % AS_GSTAGES) * (AS_GA + AS_GW);
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                bf16x8 fa[2], fb[2];
#pragma unroll
                for (int i = 0; i < 2; ++i) fa[i] = fa_r.frag(st, wm * 32 + i * 16, ks);
#pragma unroll
                for (int j = 0; j < 2; ++j) fb[j] = fb_r.frag(st + AS_GA, wn * 32 + j * 16, ks);
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[i][j] = MFMA16(fa[i], fb[j], acc[i][j]);
            }
        }
        __syncthreads();  // every wave is done with the ring, which covers the dO tiles
        // bf16(dO) into the staged tiles: element (row, col) of the C fragment layout (row 4(l>>4) + r, col l & 15)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = wm * 32 + i * 16 + 4 * g + r, col = wn * 32 + j * 16 + i16;
                    *reinterpret_cast<__bf16*>(sdO + (row >> 6) * AT_TILE_BYTES + tile_off(row & 63, col >> 3) +
                                               (col & 7) * 2) = f2bf(acc[i][j][r]);
                }
        __syncthreads();  // every wave is done with the ring: K and V take its place
        put_rows(sK, rk);
        put_rows(sV, rv);
        // δ[q] = Σ_d dO·O in the non-fused kernel's order (4 threads per query, 16 dims each)
        float dsum = 0.f;
        if (ql < a.Sq) {
            const char* t = sdO + (ql >> 6) * AT_TILE_BYTES;
            const bf16x8 x0 = *reinterpret_cast<const bf16x8*>(t + tile_off(ql & 63, part * 2));
            const bf16x8 x1 = *reinterpret_cast<const bf16x8*>(t + tile_off(ql & 63, part * 2 + 1));
#pragma unroll
            for (int j = 0; j < 8; ++j) dsum += bf2f(x0[j]) * bf2f(y0[j]);
#pragma unroll
            for (int j = 0; j < 8; ++j) dsum += bf2f(x1[j]) * bf2f(y1[j]);
        }
        dsum += __shfl_xor(dsum, 1, 64);
        dsum += __shfl_xor(dsum, 2, 64);
        if (part == 0) {
            sL[ql] = lse * AT_LOG2E;
            sD[ql] = dsum;
        }
    } else {
        const Rows128 rq = load_rows(Qb, a.ldq, a.Sq);
        const Rows128 rdo = load_rows(dOb, a.lddo, a.Sq);
        const Rows128 rk = load_rows(Kb, a.ldk, a.Sk);
        const Rows128 rv = load_rows(Vb, a.ldv, a.Sk);
        uint64_t mv = 0;  // one keep-bit word per thread (Sq * AS_TILES <= 256 < 512 threads)
        if constexpr (DROP) {
            const int qq = threadIdx.x / AS_TILES, w = threadIdx.x % AS_TILES;
            if (qq < a.Sq && w < a.mwords) mv = a.mbits[(((size_t)b * a.H + h) * a.Sq + qq) * a.mwords + w];
        }
        // δ[q] = Σ_d dO·O (4 threads per query, 16 dims each) and the forward LSE
        const int ql = threadIdx.x >> 2, part = threadIdx.x & 3;
        bf16x8 x0, x1, y0, y1;
        float lse = 0.f;
        if (ql < a.Sq) {
            const __bf16* od = a.o + ((size_t)b * a.Sq + ql) * a.ldo + h * AT_D + part * 16;
            const __bf16* dd = dOb + (size_t)ql * a.lddo + part * 16;
            x0 = *reinterpret_cast<const bf16x8*>(dd);
            x1 = *reinterpret_cast<const bf16x8*>(dd + 8);
            y0 = *reinterpret_cast<const bf16x8*>(od);
            y1 = *reinterpret_cast<const bf16x8*>(od + 8);
            lse = a.lse[((size_t)b * a.H + h) * a.Sq + ql];
        }
        put_rows(sQ, rq);
        put_rows(sdO, rdo);
        put_rows(sK, rk);
        put_rows(sV, rv);
        if (DROP && threadIdx.x < AS_MAX * AS_TILES) sM[threadIdx.x] = mv;
        float dsum = 0.f;
        if (ql < a.Sq) {
#pragma unroll
            for (int j = 0; j < 8; ++j) dsum += bf2f(x0[j]) * bf2f(y0[j]);
#pragma unroll
            for (int j = 0; j < 8; ++j) dsum += bf2f(x1[j]) * bf2f(y1[j]);
        }
        dsum += __shfl_xor(dsum, 1, 64);
        dsum += __shfl_xor(dsum, 2, 64);
        if (part == 0) {
            sL[ql] = lse * AT_LOG2E;
            sD[ql] = dsum;
        }
    }
    __syncthreads();

    // ---- phase 1: this wave's 16 keys
    const float c = a.scale * AT_LOG2E;
    {
        const int key = wave * 16 + i16;
        const int kt = wave >> 2;                      // key tile of this wave
        const int krow = (wave & 3) * 16 + i16;        // row inside that tile
        bf16x8 kf[2], vf[2];
        kf[0] = row_frag(sK + kt * AT_TILE_BYTES, (wave & 3) * 16, 0);
        kf[1] = row_frag(sK + kt * AT_TILE_BYTES, (wave & 3) * 16, 1);
        vf[0] = row_frag(sV + kt * AT_TILE_BYTES, (wave & 3) * 16, 0);
        vf[1] = row_frag(sV + kt * AT_TILE_BYTES, (wave & 3) * 16, 1);
        f32x4 dk[4], dv[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            dk[d] = f32x4{0.f, 0.f, 0.f, 0.f};
            dv[d] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        const int nqt = (a.Sq + AT_T - 1) / AT_T;
        DropBits db{nullptr, AS_TILES, key & 63, a.drop.scale};
        for (int qt = CAUSAL ? kt : 0; qt < nqt; ++qt) {
            const char* tQ = sQ + qt * AT_TILE_BYTES;
            const char* tdO = sdO + qt * AT_TILE_BYTES;
            char* tS = sdS + (kt * AS_TILES + qt) * AT_TILE_BYTES;
            if (DROP) db.mcol = sM + qt * AT_T * AS_TILES + kt;
            dkv_step<CAUSAL, DROP, true>(tQ, tdO, sL + qt * AT_T, sD + qt * AT_T, qt * AT_T, key, wave * 16, a.Sq, a.Sk, c, kf,
                                   vf, dk, dv, tS, krow, db);
        }
        if (key < a.Sk) {
            size_t tok = (size_t)b * a.Sk + key;
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                bf16x4 wk, wv;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    wk[r] = f2bf(dk[d][r] * a.scale);
                    wv[r] = f2bf(dv[d][r]);
                }
                *reinterpret_cast<bf16x4*>(a.dk + tok * a.lddk + h * AT_D + d * 16 + 4 * g) = wk;
                *reinterpret_cast<bf16x4*>(a.dv + tok * a.lddv + h * AT_D + d * 16 + 4 * g) = wv;
            }
        }
    }
    __syncthreads();

    // ---- phase 2: this wave's 16 queries, dQᵀ[d][q] = Σ_key K[key][d] dS[key][q]
    {
        const int q = wave * 16 + i16;
        const int qt = wave >> 2, qc0 = (wave & 3) * 16;
        f32x4 dq[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int nkt = CAUSAL ? qt + 1 : (a.Sk + AT_T - 1) / AT_T;
        for (int kt = 0; kt < nkt; ++kt) {
            const char* tK = sK + kt * AT_TILE_BYTES;
            const char* tS = sdS + (kt * AS_TILES + qt) * AT_TILE_BYTES;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                // rows (keys) of a tile the causal phase 1 never wrote are skipped whole (kt > qt);
                // inside a diagonal tile masked entries were stored as 0
                bf16x8 sb = tr_frag(tS, 32 * half, qc0);
#pragma unroll
                for (int d = 0; d < 4; ++d) dq[d] = MFMA16(tr_frag(tK, 32 * half, d * 16), sb, dq[d]);
            }
        }
        if (q < a.Sq) {
            __bf16* out = a.dq + ((size_t)b * a.Sq + q) * a.lddq + h * AT_D;
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                bf16x4 w;
#pragma unroll
                for (int r = 0; r < 4; ++r) w[r] = f2bf(dq[d][r] * a.scale);
                *reinterpret_cast<bf16x4*>(out + d * 16 + 4 * g) = w;
            }
        }
    }
}

static int check_common(const void* q, const void* k, const void* v, int B, int H, int Sq, int Sk, int ldq, int ldk,
                        int ldv, int causal) {
    ERGM_CHECK_ARG(q && k && v, "attn: null argument");
    ERGM_CHECK_ARG(B > 0 && H > 0 && Sq > 0 && Sk > 0, "attn: bad shape");
    ERGM_CHECK_ARG(!causal || Sq == Sk, "attn: causal needs Sq == Sk");
    ERGM_CHECK_ARG(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0, "attn: leading dims must be multiples of 8");
    ERGM_CHECK_ARG(ldq >= H * AT_D && ldk >= H * AT_D && ldv >= H * AT_D, "attn: leading dim < H*64");
    ERGM_CHECK_ARG(aligned16(q) && aligned16(k) && aligned16(v), "attn: pointers must be 16-byte aligned");
    return ERGM_OK;
}

}  // namespace ergm

using namespace ergm;

namespace {
bool g_attn_generic = false;  // ergm_attn_tune: force the tiled kernels even for short sequences
// ergm_attn_tune: ring stages of the tiled kernels (0: per-kernel defaults)
int g_attn_ns = 0;

template <bool CAUSAL, int NS, bool DROP>
void launch_tiled_fwd(dim3 grid, hipStream_t s, const AttnArgs& a) {
    ERGM_LAUNCH((attn_fwd_kernel<CAUSAL, NS, DROP>), grid, dim3(256), 0, s, a);
}
// Defaults: 2 stages everywhere (tools/attn_bench.py at the C4 shape: forward fastest at 2, the dK/dV
// kernel then fits 3 waves per SIMD without spills; dQ 3 isolated, 2 inside the C4 step, #20).
template <bool CAUSAL, bool DROP>
void tiled_fwd(dim3 grid, hipStream_t s, const AttnArgs& a) {
    if (g_attn_ns == 3) launch_tiled_fwd<CAUSAL, 3, DROP>(grid, s, a);
    else if (g_attn_ns == 4) launch_tiled_fwd<CAUSAL, 4, DROP>(grid, s, a);
    else launch_tiled_fwd<CAUSAL, 2, DROP>(grid, s, a);
}
template <bool CAUSAL, bool DROP>
void tiled_bwd(dim3 gk, dim3 gq, hipStream_t s, const AttnArgs& a) {
    const int ns_kv = g_attn_ns ? g_attn_ns : 2, ns_q = g_attn_ns ? g_attn_ns : 2;
    if (ns_kv == 3) ERGM_LAUNCH((attn_bwd_dkv_kernel<CAUSAL, 3, DROP>), gk, dim3(256), 0, s, a);
    else if (ns_kv == 4) ERGM_LAUNCH((attn_bwd_dkv_kernel<CAUSAL, 4, DROP>), gk, dim3(256), 0, s, a);
    else ERGM_LAUNCH((attn_bwd_dkv_kernel<CAUSAL, 2, DROP>), gk, dim3(256), 0, s, a);
    if (ns_q == 2) ERGM_LAUNCH((attn_bwd_dq_kernel<CAUSAL, 2, DROP>), gq, dim3(256), 0, s, a);
    else if (ns_q == 4) ERGM_LAUNCH((attn_bwd_dq_kernel<CAUSAL, 4, DROP>), gq, dim3(256), 0, s, a);
    else ERGM_LAUNCH((attn_bwd_dq_kernel<CAUSAL, 3, DROP>), gq, dim3(256), 0, s, a);
}
// Dropout fields of AttnArgs from the C-ABI descriptor (rows (b·H + h)·Sq + q, cols Sk).
int set_drop(AttnArgs& a, const ergm_dropout* d, void* keep_bits) {
    ERGM_TRY(check_dropout(d));
    a.drop = drop_site_of(d, a.Sk);
    a.mwords = (a.Sk + 63) / 64;
    a.mbits = a.drop.thresh ? reinterpret_cast<uint64_t*>(keep_bits) : nullptr;
    ERGM_CHECK_ARG(!a.drop.thresh || keep_bits, "attn: dropout needs the keep-bit buffer");
    ERGM_CHECK_ARG(!a.drop.thresh || (a.Sq <= AT_MAX_SQ_DROP && a.Sk <= AT_MAX_SQ_DROP),
                   "attn: dropout supports Sq, Sk <= %d", AT_MAX_SQ_DROP);
    return ERGM_OK;
}
}

extern "C" int ergm_attn_tune(int force_generic) {
    const int ns = (force_generic >> 4) & 15;
    ERGM_CHECK_ARG(ns == 0 || ns == 2 || ns == 3 || ns == 4, "attn_tune: ring stages must be 2, 3 or 4");
    g_attn_generic = (force_generic & 1) != 0;
    g_attn_ns = ns;
    return ERGM_OK;
}

namespace ergm {
// ergm_attn_fwd + the MX-fp8 copy of its output (the executor's config-5 forward: the c_proj GEMMs' A operand)
int attn_fwd_mx(const void* q, const void* k, const void* v, void* o, float* lse, int B, int H, int Sq, int Sk, int ldq,
                int ldk, int ldv, int ldo, int causal, const ergm_dropout* dropout, void* keep_bits, uint8_t* qmx,
                uint8_t* qms, int ldqm, int qpitch, hipStream_t s);
}

extern "C" int ergm_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int H, int Sq,
                             int Sk, int ldq, int ldk, int ldv, int ldo, int causal, const ergm_dropout* dropout,
                             void* keep_bits, void* stream) {
    return ergm::attn_fwd_mx(q, k, v, o, lse, B, H, Sq, Sk, ldq, ldk, ldv, ldo, causal, dropout, keep_bits, nullptr,
                             nullptr, 0, 0, as_stream(stream));
}

int ergm::attn_fwd_mx(const void* q, const void* k, const void* v, void* o, float* lse, int B, int H, int Sq, int Sk,
                      int ldq, int ldk, int ldv, int ldo, int causal, const ergm_dropout* dropout, void* keep_bits,
                      uint8_t* qmx, uint8_t* qms, int ldqm, int qpitch, hipStream_t s) {
    ERGM_TRY(check_common(q, k, v, B, H, Sq, Sk, ldq, ldk, ldv, causal));
    ERGM_CHECK_ARG(o && lse && ldo % 4 == 0 && ldo >= H * AT_D, "attn_fwd: bad output");
    AttnArgs a{};
    a.q = (const __bf16*)q; a.k = (const __bf16*)k; a.v = (const __bf16*)v;
    a.out = (__bf16*)o; a.lse = lse;
    a.B = B; a.H = H; a.Sq = Sq; a.Sk = Sk;
    a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.ldo = ldo;
    a.scale = 0.125f;  // 1/sqrt(64): exact, so x*scale == x / 8.0 (src/model.py:122-125)
    ERGM_TRY(set_drop(a, dropout, keep_bits));
    ERGM_CHECK_ARG(!qmx || (qms && ldqm >= H * AT_D && ldqm % 4 == 0 && qpitch >= B * Sq), "attn_fwd: bad MX output");
    a.qmx = qmx; a.qms = qms; a.ldqm = ldqm; a.qpitch = qpitch;
    // every length takes the tiled kernel: at S = 128 its 2x more workgroups beat the one-workgroup-per-
    // (b, h) form inside the concurrent step (C2 +1.6 %, C5 +0.4 %; profiles/r01_overlap_experiments.txt #19)
    dim3 grid(cdiv(Sq, AT_T), H, B);
    const bool drop = a.mbits != nullptr;
    if (causal) drop ? tiled_fwd<true, true>(grid, s, a) : tiled_fwd<true, false>(grid, s, a);
    else drop ? tiled_fwd<false, true>(grid, s, a) : tiled_fwd<false, false>(grid, s, a);
    return check_launch("attn_fwd");
}

extern "C" int ergm_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                             const float* lse, float* delta, void* dq, void* dk, void* dv, int B, int H, int Sq,
                             int Sk, int ldq, int ldk, int ldv, int ldo, int lddo, int lddq, int lddk, int lddv,
                             int causal, const ergm_dropout* dropout, const void* keep_bits, void* stream) {
    ERGM_TRY(check_common(q, k, v, B, H, Sq, Sk, ldq, ldk, ldv, causal));
    ERGM_CHECK_ARG(o && dout && lse && delta && dq && dk && dv, "attn_bwd: null argument");
    ERGM_CHECK_ARG(ldo % 8 == 0 && lddo % 8 == 0 && lddq % 4 == 0 && lddk % 4 == 0 && lddv % 4 == 0,
                   "attn_bwd: bad leading dims");
    ERGM_CHECK_ARG(aligned16(o) && aligned16(dout), "attn_bwd: O/dO must be 16-byte aligned");
    AttnArgs a{};
    a.q = (const __bf16*)q; a.k = (const __bf16*)k; a.v = (const __bf16*)v;
    a.o = (const __bf16*)o; a.dout = (const __bf16*)dout;
    a.dq = (__bf16*)dq; a.dk = (__bf16*)dk; a.dv = (__bf16*)dv;
    a.lse = (float*)lse; a.delta = delta;
    a.B = B; a.H = H; a.Sq = Sq; a.Sk = Sk;
    a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.ldo = ldo; a.lddo = lddo;
    a.lddq = lddq; a.lddk = lddk; a.lddv = lddv;
    a.scale = 0.125f;
    ERGM_TRY(set_drop(a, dropout, const_cast<void*>(keep_bits)));
    const bool drop = a.mbits != nullptr;
    hipStream_t s = as_stream(stream);
    if (Sq <= AS_MAX && Sk <= AS_MAX && !g_attn_generic) {
        static bool attr_set = false;  // benign race: idempotent attribute writes
        if (!attr_set) {
            const void* ks[4] = {(const void*)attn_bwd_short_kernel<true, false>,
                                 (const void*)attn_bwd_short_kernel<false, false>,
                                 (const void*)attn_bwd_short_kernel<true, true>,
                                 (const void*)attn_bwd_short_kernel<false, true>};
            for (const void* k : ks)
                if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, AS_LDS) != hipSuccess)
                    return fail(ERGM_EHIP, "attn_bwd: cannot raise dynamic LDS limit");
            attr_set = true;
        }
        dim3 grid(1, H, B);
        if (causal) {
            if (drop) ERGM_LAUNCH((attn_bwd_short_kernel<true, true>), grid, dim3(512), AS_LDS, s, a);
            else ERGM_LAUNCH((attn_bwd_short_kernel<true, false>), grid, dim3(512), AS_LDS, s, a);
        } else {
            if (drop) ERGM_LAUNCH((attn_bwd_short_kernel<false, true>), grid, dim3(512), AS_LDS, s, a);
            else ERGM_LAUNCH((attn_bwd_short_kernel<false, false>), grid, dim3(512), AS_LDS, s, a);
        }
        return check_launch("attn_bwd");
    }
    dim3 gk(cdiv(Sk, AT_T), H, B), gq(cdiv(Sq, AT_T), H, B);
    ERGM_LAUNCH(attn_delta_kernel, dim3(cdiv(B * Sq * H * 4, 256)), dim3(256), 0, s, a);
    if (causal) drop ? tiled_bwd<true, true>(gk, gq, s, a) : tiled_bwd<true, false>(gk, gq, s, a);
    else drop ? tiled_bwd<false, true>(gk, gq, s, a) : tiled_bwd<false, false>(gk, gq, s, a);
    return check_launch("attn_bwd");
}

namespace ergm {
bool attn_bwd_fusable(int Sq, int Sk, int K) { return Sq <= AS_MAX && Sk <= AS_MAX && !g_attn_generic && K > 0 && K % GEMM_BK == 0; }

// The executor's fused form of "dO = dY·Wᵀ (the c_proj data gradient) ; ergm_attn_bwd(.., dO, ..)" for short
// sequences (attn_bwd_fusable): attn_bwd_short_kernel<.., GEMM_DO = true>.  Bitwise the two launches' results (the
// GEMM's product order is ergm_gemm's, δ is summed as in the unfused kernel); no dO or δ is written.
int attn_bwd_fused(const void* q, const void* k, const void* v, const void* o, const void* dy, int lddy, const void* w,
                   int ldw, int K, const float* lse, void* dq, void* dk, void* dv, int B, int H, int Sq, int Sk, int ldq,
                   int ldk, int ldv, int ldo, int lddq, int lddk, int lddv, int causal, const ergm_dropout* dropout,
                   const void* keep_bits, hipStream_t s) {
    ERGM_TRY(check_common(q, k, v, B, H, Sq, Sk, ldq, ldk, ldv, causal));
    ERGM_CHECK_ARG(attn_bwd_fusable(Sq, Sk, K), "attn_bwd_fused: shape not fusable");
    ERGM_CHECK_ARG(o && dy && w && lse && dq && dk && dv, "attn_bwd_fused: null argument");
    ERGM_CHECK_ARG(ldo % 8 == 0 && lddy % 8 == 0 && ldw % 8 == 0 && lddy >= K && ldw >= K && lddq % 4 == 0 &&
                       lddk % 4 == 0 && lddv % 4 == 0,
                   "attn_bwd_fused: bad leading dims");
    ERGM_CHECK_ARG(aligned16(o) && aligned16(dy) && aligned16(w), "attn_bwd_fused: O/dY/W must be 16-byte aligned");
    AttnArgs a{};
    a.q = (const __bf16*)q; a.k = (const __bf16*)k; a.v = (const __bf16*)v;
    a.o = (const __bf16*)o;
    a.dq = (__bf16*)dq; a.dk = (__bf16*)dk; a.dv = (__bf16*)dv;
    a.lse = (float*)lse;
    a.B = B; a.H = H; a.Sq = Sq; a.Sk = Sk;
    a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.ldo = ldo;
    a.lddq = lddq; a.lddk = lddk; a.lddv = lddv;
    a.scale = 0.125f;
    a.gA = (const __bf16*)dy; a.gW = (const __bf16*)w;
    a.lda_g = lddy; a.ldw_g = ldw; a.K_g = K;
    ERGM_TRY(set_drop(a, dropout, const_cast<void*>(keep_bits)));
    const bool drop = a.mbits != nullptr;
    static bool attr_set = false;  // benign race: idempotent attribute writes
    if (!attr_set) {
        const void* ks[4] = {(const void*)attn_bwd_short_kernel<true, false, true>,
                             (const void*)attn_bwd_short_kernel<false, false, true>,
                             (const void*)attn_bwd_short_kernel<true, true, true>,
                             (const void*)attn_bwd_short_kernel<false, true, true>};
        for (const void* kf : ks)
            if (hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, AS_LDS) != hipSuccess)
                return fail(ERGM_EHIP, "attn_bwd_fused: cannot raise dynamic LDS limit");
        attr_set = true;
    }
    dim3 grid(1, H, B);
    if (causal) {
        if (drop) ERGM_LAUNCH((attn_bwd_short_kernel<true, true, true>), grid, dim3(512), AS_LDS, s, a);
        else ERGM_LAUNCH((attn_bwd_short_kernel<true, false, true>), grid, dim3(512), AS_LDS, s, a);
    } else {
        if (drop) ERGM_LAUNCH((attn_bwd_short_kernel<false, true, true>), grid, dim3(512), AS_LDS, s, a);
        else ERGM_LAUNCH((attn_bwd_short_kernel<false, false, true>), grid, dim3(512), AS_LDS, s, a);
    }
    return check_launch("attn_bwd_fused");
}
}  // namespace ergm

namespace ergm {
// The executor's fused form of "q = LN_x·Wq + bq ; ergm_attn_fwd(q, K, V, ..., causal = 0)" (attn_fwd_qgemm_kernel):
// bitwise the two launches' q, O, LSE and keep bits.
int attn_fwd_qgemm(const void* x, int ldx, const void* w, int ldw, const float* bias, int K, void* q, int ldq,
                   const void* k, const void* v, void* o, float* lse, int B, int H, int Sq, int Sk, int ldk, int ldv,
                   int ldo, const ergm_dropout* dropout, void* keep_bits, hipStream_t s) {
    ERGM_TRY(check_common(q, k, v, B, H, Sq, Sk, ldq, ldk, ldv, 0));
    ERGM_CHECK_ARG(x && w && bias && o && lse, "attn_fwd_qgemm: null argument");
    ERGM_CHECK_ARG(K > 0 && K % GEMM_BK == 0 && ldx % 8 == 0 && ldx >= K && ldw % 8 == 0 && ldw >= H * AT_D,
                   "attn_fwd_qgemm: bad K / leading dims");
    ERGM_CHECK_ARG(aligned16(x) && aligned16(w), "attn_fwd_qgemm: x / w must be 16-byte aligned");
    ERGM_CHECK_ARG(ldo % 4 == 0 && ldo >= H * AT_D, "attn_fwd_qgemm: bad output");
    AttnArgs a{};
    a.q = (const __bf16*)q; a.k = (const __bf16*)k; a.v = (const __bf16*)v;
    a.out = (__bf16*)o; a.lse = lse;
    a.B = B; a.H = H; a.Sq = Sq; a.Sk = Sk;
    a.ldq = ldq; a.ldk = ldk; a.ldv = ldv; a.ldo = ldo;
    a.scale = 0.125f;
    a.gA = (const __bf16*)x; a.gW = (const __bf16*)w; a.gbias = bias;
    a.lda_g = ldx; a.ldw_g = ldw; a.K_g = K;
    ERGM_TRY(set_drop(a, dropout, keep_bits));
    dim3 grid(cdiv(Sq, AT_T), H, B);
    if (a.mbits) ERGM_LAUNCH((attn_fwd_qgemm_kernel<2, true>), grid, dim3(256), 0, s, a);
    else ERGM_LAUNCH((attn_fwd_qgemm_kernel<2, false>), grid, dim3(256), 0, s, a);
    return check_launch("attn_fwd_qgemm");
}
}  // namespace ergm
