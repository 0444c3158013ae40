// LayerNorm forward/backward and deterministic column sums for gfx950.
//
// Replaces nn.LayerNorm (ln_1 / ln_cross_attn / ln_2 / ln_f: src/model.py:276,278,282,392, applied at
// :298,318,332,578) and its autograd backward; column sums give Conv1D bias gradients, the LayerNorm
// dγ/dβ reductions and the wpe gradient (Σ over batch of the embedding gradient).
// Row-per-wavefront: each lane owns NV float4 column groups of the row (coalesced 1 KiB per
// wave-instruction), reductions by 64-lane xor shuffles; HBM-bound.
#include "common.h"

namespace ergm {

constexpr int LN_WAVES_BWD = 8;  // one row per wave: 8 waves per CU in flight at T = 2048
// rows per workgroup: one per wave (two per wave, 128 workgroups at T = 2048, halves the partials the dγ/dβ reduce
// reads but cost +0.8 % at C2 and +3.7 % at C5: profiles/r05_experiments.txt #13)
constexpr int LN_ROWS_PER_BLOCK_BWD = 8;

template <int NV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, __bf16* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int rows, int E, int ldy, float eps, uint8_t* __restrict__ yq,
                                                     int ldq, float* __restrict__ qscale, uint8_t* __restrict__ qmx,
                                                     int ld_qmx) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + wave;
    if (row >= rows) return;
    const float* xr = x + (size_t)row * E;
    float4 v[NV], gv[NV], bv[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {  // every load issued before the first reduction
        int c = (i * 64 + lane) * 4;
        const bool in = c < E;
        v[i] = in ? *reinterpret_cast<const float4*>(xr + c) : make_float4(0, 0, 0, 0);
        gv[i] = in ? *reinterpret_cast<const float4*>(gamma + c) : make_float4(0, 0, 0, 0);
        bv[i] = in ? *reinterpret_cast<const float4*>(beta + c) : make_float4(0, 0, 0, 0);
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) s += (v[i].x + v[i].y) + (v[i].z + v[i].w);
    const float inv_e = 1.0f / (float)E;
    const float mean = wave_sum(s) * inv_e;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        int c = (i * 64 + lane) * 4;
        if (c < E) {
            float a = v[i].x - mean, b = v[i].y - mean, cc = v[i].z - mean, d = v[i].w - mean;
            q += (a * a + b * b) + (cc * cc + d * d);
        }
    }
    const float var = wave_sum(q) * inv_e;
    const float rstd = 1.0f / sqrtf(var + eps);
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        int c = (i * 64 + lane) * 4;
        if (c < E) {
            const float4 g = gv[i], b = bv[i];
            v[i].x = (v[i].x - mean) * rstd * g.x + b.x;
            v[i].y = (v[i].y - mean) * rstd * g.y + b.y;
            v[i].z = (v[i].z - mean) * rstd * g.z + b.z;
            v[i].w = (v[i].w - mean) * rstd * g.w + b.w;
            bf16x4 o;
            o[0] = f2bf(v[i].x);
            o[1] = f2bf(v[i].y);
            o[2] = f2bf(v[i].z);
            o[3] = f2bf(v[i].w);
            *reinterpret_cast<bf16x4*>(y + (size_t)row * ldy + c) = o;
            amax = fmaxf(amax, fmaxf(fmaxf(fabsf(v[i].x), fabsf(v[i].y)), fmaxf(fabsf(v[i].z), fabsf(v[i].w))));
        }
    }
    if (yq && qmx) {  // MX-fp8 copy (config 5): a 32-column block is 8 consecutive lanes of one float4 group
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            const int c = (i * 64 + lane) * 4;
            const bool in = c < E;  // E % 32 == 0: a block is wholly in or out
            float am = in ? fmaxf(fmaxf(fabsf(v[i].x), fabsf(v[i].y)), fmaxf(fabsf(v[i].z), fabsf(v[i].w))) : 0.f;
            am = fmaxf(am, __shfl_xor(am, 1, 64));
            am = fmaxf(am, __shfl_xor(am, 2, 64));
            am = fmaxf(am, __shfl_xor(am, 4, 64));
            const int eb = mx_exp_biased(am);
            const float is = mx_inv_scale(eb);
            if (in) {
                *reinterpret_cast<uint32_t*>(yq + (size_t)row * ldq + c) =
                    mx_pack4(v[i].x * is, v[i].y * is, v[i].z * is, v[i].w * is);
                if ((lane & 7) == 0) qmx[mx_sidx(row, c >> 5, ld_qmx)] = (uint8_t)eb;
            }
        }
    } else if (yq) {  // fp8 copy for the config-5 forward GEMMs (row scale, quant.hip's scheme)
        amax = wave_max(amax);
        const float sc = amax > 0.f ? amax / 448.f : 1.f;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            int c = (i * 64 + lane) * 4;
            if (c < E) {
                float a = fminf(fmaxf(v[i].x / sc, -448.f), 448.f), b = fminf(fmaxf(v[i].y / sc, -448.f), 448.f);
                float cc = fminf(fmaxf(v[i].z / sc, -448.f), 448.f), d = fminf(fmaxf(v[i].w / sc, -448.f), 448.f);
                int qq = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
                qq = __builtin_amdgcn_cvt_pk_fp8_f32(cc, d, qq, true);
                *reinterpret_cast<int*>(yq + (size_t)row * ldq + c) = qq;
            }
        }
        if (lane == 0) qscale[row] = sc;
    }
    if (lane == 0) {
        mean_out[row] = mean;
        rstd_out[row] = rstd;
    }
}

// dx = rstd·(g − mean(g) − x̂·mean(g·x̂)), g = dy·γ;  dres += dx;  partial dγ = Σ dy·x̂, dβ = Σ dy.
// dres_b = bf16(dres), or with `drop` the gradient reaching the residual branch that produced this
// residual-stream tensor through its dropout: bf16(dres·keep/(1-p)) (src/model.py:245,266,506; the
// keep bits recomputed, common.h drop_keep4).
// DYB: dy is the bf16 output of the data-gradient GEMM (the per-block LayerNorms), else f32 (ln_f: the LM-head
// and emotion-head gradients summed in f32).
template <int NV, bool DYB>
__global__ __launch_bounds__(64 * LN_WAVES_BWD) void ln_bwd_kernel(const void* __restrict__ dy_, const float* __restrict__ x,
                                                     const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
                                                     const float* __restrict__ gamma, float* __restrict__ dres,
                                                     __bf16* __restrict__ dres_b, float* __restrict__ part_g,
                                                     float* __restrict__ part_b, int rows, int E, DropSite drop,
                                                     int drop_res, uint8_t* __restrict__ qmx, uint8_t* __restrict__ qmx_s,
                                                     int ld_qs) {
    __shared__ float red[LN_WAVES_BWD][NV * 256];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float4 pg[NV], pb[NV], gm[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        pg[i] = make_float4(0, 0, 0, 0);
        pb[i] = make_float4(0, 0, 0, 0);
        int c = (i * 64 + lane) * 4;
        gm[i] = c < E ? *reinterpret_cast<const float4*>(gamma + c) : make_float4(0, 0, 0, 0);
    }
    const float inv_e = 1.0f / (float)E;
    // each wave owns RPW rows and issues every load of all of them (x, dy and the residual gradient it
    // adds into) before the first reduction, so the HBM latency is paid once
    constexpr int RPW = LN_ROWS_PER_BLOCK_BWD / LN_WAVES_BWD;
    const int r0 = blockIdx.x * LN_ROWS_PER_BLOCK_BWD + wave * RPW;
    float4 xh[RPW][NV], d[RPW][NV], o[RPW][NV];
    float mu[RPW], rs[RPW];
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
        const int row = r0 + j;
        const bool live = row < rows;
        mu[j] = live ? mean_in[row] : 0.f;
        rs[j] = live ? rstd_in[row] : 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            int c = (i * 64 + lane) * 4;
            if (live && c < E) {
                xh[j][i] = *reinterpret_cast<const float4*>(x + (size_t)row * E + c);
                if constexpr (DYB) {
                    const bf16x4 b = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const __bf16*>(dy_) +
                                                                      (size_t)row * E + c);
                    d[j][i] = make_float4(bf2f(b[0]), bf2f(b[1]), bf2f(b[2]), bf2f(b[3]));
                } else {
                    d[j][i] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(dy_) + (size_t)row * E + c);
                }
                o[j][i] = *reinterpret_cast<const float4*>(dres + (size_t)row * E + c);
            } else {
                xh[j][i] = d[j][i] = o[j][i] = make_float4(0, 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
        const int row = r0 + j;
        float s1 = 0.f, s2 = 0.f;
        float4 g[NV];
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            float4& h = xh[j][i];
            const float4 dv = d[j][i];
            h = make_float4((h.x - mu[j]) * rs[j], (h.y - mu[j]) * rs[j], (h.z - mu[j]) * rs[j], (h.w - mu[j]) * rs[j]);
            g[i] = make_float4(dv.x * gm[i].x, dv.y * gm[i].y, dv.z * gm[i].z, dv.w * gm[i].w);
            s1 += (g[i].x * h.x + g[i].y * h.y) + (g[i].z * h.z + g[i].w * h.w);
            s2 += (g[i].x + g[i].y) + (g[i].z + g[i].w);
            pg[i].x += dv.x * h.x; pg[i].y += dv.y * h.y;
            pg[i].z += dv.z * h.z; pg[i].w += dv.w * h.w;
            pb[i].x += dv.x; pb[i].y += dv.y; pb[i].z += dv.z; pb[i].w += dv.w;
        }
        const float c1 = wave_sum(s1) * inv_e, c2 = wave_sum(s2) * inv_e;
        if (row >= rows) continue;
        const float r = rs[j];
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            int c = (i * 64 + lane) * 4;
            if (c < E) {
                float4 v = o[j][i];
                const float4 h = xh[j][i];
                v.x += r * (g[i].x - c2 - h.x * c1);
                v.y += r * (g[i].y - c2 - h.y * c1);
                v.z += r * (g[i].z - c2 - h.z * c1);
                v.w += r * (g[i].w - c2 - h.w * c1);
                if (drop_res && drop.thresh) {  // final residual gradient taken through the branch dropout
                    const unsigned k = drop_keep4(drop, row, c);
                    v.x = (k & 1u) ? v.x * drop.scale : 0.f;
                    v.y = (k & 2u) ? v.y * drop.scale : 0.f;
                    v.z = (k & 4u) ? v.z * drop.scale : 0.f;
                    v.w = (k & 8u) ? v.w * drop.scale : 0.f;
                }
                *reinterpret_cast<float4*>(dres + (size_t)row * E + c) = v;
                if (dres_b) {
                    bf16x4 ob;
                    float4 u = v;
                    if (drop.thresh && !drop_res) {
                        const unsigned k = drop_keep4(drop, row, c);
                        u.x = (k & 1u) ? u.x * drop.scale : 0.f;
                        u.y = (k & 2u) ? u.y * drop.scale : 0.f;
                        u.z = (k & 4u) ? u.z * drop.scale : 0.f;
                        u.w = (k & 8u) ? u.w * drop.scale : 0.f;
                    }
                    ob[0] = f2bf(u.x); ob[1] = f2bf(u.y); ob[2] = f2bf(u.z); ob[3] = f2bf(u.w);
                    *reinterpret_cast<bf16x4*>(dres_b + (size_t)row * E + c) = ob;
                    if (qmx) {  // MX-fp8 copy of the stored bf16 values (config 5's fp8 data-gradient GEMMs): a
                                // 32-column block is 8 consecutive lanes (E % 32 == 0, so a block is wholly in)
                        const float w0 = bf2f(ob[0]), w1 = bf2f(ob[1]), w2 = bf2f(ob[2]), w3 = bf2f(ob[3]);
                        float am = fmaxf(fmaxf(fabsf(w0), fabsf(w1)), fmaxf(fabsf(w2), fabsf(w3)));
                        am = fmaxf(am, __shfl_xor(am, 1, 64));
                        am = fmaxf(am, __shfl_xor(am, 2, 64));
                        am = fmaxf(am, __shfl_xor(am, 4, 64));
                        const int eb = mx_exp_biased(am);
                        const float is = mx_inv_scale(eb);
                        *reinterpret_cast<uint32_t*>(qmx + (size_t)row * E + c) = mx_pack4(w0 * is, w1 * is, w2 * is, w3 * is);
                        if ((lane & 7) == 0) qmx_s[mx_sidx(row, c >> 5, ld_qs)] = (uint8_t)eb;
                    }
                }
            }
        }
    }
    // cross-wave reduction of the partial column sums (fixed order → deterministic): dγ then dβ through one
    // [waves][E] buffer, so the workgroup holds 24 KB of LDS (at E = 768) and fits beside the GEMM tiles of the
    // concurrent weight-gradient stream
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (h) __syncthreads();  // dγ's reads of the buffer are done
#pragma unroll
        for (int i = 0; i < NV; ++i) {
            int c = (i * 64 + lane) * 4;
            *reinterpret_cast<float4*>(&red[wave][c]) = h ? pb[i] : pg[i];
        }
        __syncthreads();
        float* out = h ? part_b : part_g;
        for (int c = threadIdx.x; c < E; c += 64 * LN_WAVES_BWD) {
            float a = red[0][c];
#pragma unroll
            for (int w = 1; w < LN_WAVES_BWD; ++w) a += red[w][c];
            out[(size_t)blockIdx.x * E + c] = a;
        }
    }
}

// dγ / dβ: sum the per-block partials (fixed order).  grid (cdiv(E,64), 2), 1024 threads: 64 columns x
// 16 row lanes, each lane with 16 partial rows in flight per round (one HBM latency per 256 partials).
struct LnReduceJobs {  // up to 4 LayerNorms' (partials, dγ, dβ) reduced by one launch (blockIdx.z)
    const float* part_g[4];
    const float* part_b[4];
    float* dgamma[4];
    float* dbeta[4];
};

// 256-thread blocks (32 columns x 8 row lanes): small enough to find free wave slots beside the GEMMs running
// concurrently on the other streams (a 1024-thread block needs a whole CU's slots and waited behind long GEMM tiles
// at config-5 sizes).  Each lane keeps LN_RED_LOADS partial rows in flight per round, so the training step's 256
// partial rows (T = 2048) are one round: one memory latency per launch instead of two (round 4: 16 per lane).
constexpr int LN_RED_LOADS = 32;
__global__ __launch_bounds__(256) void ln_param_reduce_kernel(LnReduceJobs jobs, int nparts, int E) {
    __shared__ float red[8][32];
    const int z = blockIdx.z;
    const float* part = blockIdx.y == 0 ? jobs.part_g[z] : jobs.part_b[z];
    float* out = blockIdx.y == 0 ? jobs.dgamma[z] : jobs.dbeta[z];
    const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
    const int c = blockIdx.x * 32 + cl;
    float acc = 0.f;
    for (int base = 0; base < nparts; base += 8 * LN_RED_LOADS) {
        float v[LN_RED_LOADS];
#pragma unroll
        for (int j = 0; j < LN_RED_LOADS; ++j) {
            const int r = base + rl + 8 * j;
            v[j] = c < E && r < nparts ? __builtin_nontemporal_load(part + (size_t)r * E + c) : 0.f;
        }
#pragma unroll
        for (int w = 1; w < LN_RED_LOADS; w <<= 1)
#pragma unroll
            for (int j = 0; j < LN_RED_LOADS; j += 2 * w) v[j] += v[j + w];
        acc += v[0];
    }
    red[rl][cl] = acc;
    __syncthreads();
    if (rl == 0 && c < E) {
        float t[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) t[j] = red[j][cl];
#pragma unroll
        for (int w = 1; w < 8; w <<= 1)
#pragma unroll
            for (int j = 0; j < 8; j += 2 * w) t[j] += t[j + w];
        out[c] = t[0];
    }
}

// ---- column sums: out[c] (+)= Σ_r X[r][c] -------------------------------------------------
constexpr int CS_ROWS = 64;  // rows per partial block

template <bool BF16_IN>
__global__ __launch_bounds__(256) void colsum_partial_kernel(const void* __restrict__ X, int rows, int cols, int ldx,
                                                             float* __restrict__ part, float* __restrict__ out,
                                                             int accumulate, int direct) {
    // block: 64 column groups (4 cols each) x 4 row lanes; blockIdx.x: 256-column slab, y: row chunk
    __shared__ float4 red[4][64];
    const int cg = threadIdx.x & 63, rl = threadIdx.x >> 6;
    const int c = (blockIdx.x * 64 + cg) * 4;
    const int r0 = blockIdx.y * CS_ROWS;
    float4 s = make_float4(0, 0, 0, 0);
    if (c < cols) {
        for (int r = r0 + rl; r < min(rows, r0 + CS_ROWS); r += 4) {
            float4 v;
            if (BF16_IN) {
                bf16x4 b = *reinterpret_cast<const bf16x4*>(reinterpret_cast<const __bf16*>(X) + (size_t)r * ldx + c);
                v = make_float4(bf2f(b[0]), bf2f(b[1]), bf2f(b[2]), bf2f(b[3]));
            } else {
                v = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(X) + (size_t)r * ldx + c);
            }
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
    }
    red[rl][cg] = s;
    __syncthreads();
    if (rl == 0 && c < cols) {
        float4 t = red[0][cg];
#pragma unroll
        for (int k = 1; k < 4; ++k) {
            t.x += red[k][cg].x; t.y += red[k][cg].y; t.z += red[k][cg].z; t.w += red[k][cg].w;
        }
        if (direct) {
            float4* o = reinterpret_cast<float4*>(out + c);
            if (accumulate) {
                float4 p = *o;
                t.x += p.x; t.y += p.y; t.z += p.z; t.w += p.w;
            }
            *o = t;
        } else {
            *reinterpret_cast<float4*>(part + (size_t)blockIdx.y * cols + c) = t;
        }
    }
}

__global__ __launch_bounds__(256) void colsum_final_kernel(const float* __restrict__ part, int nparts, int cols,
                                                           float* __restrict__ out, int accumulate) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= cols) return;
    float s = 0.f;
    for (int p = 0; p < nparts; ++p) s += part[(size_t)p * cols + c];
    if (accumulate) s += out[c];
    out[c] = s;
}

int colsum_impl(const void* X, bool bf16_in, int rows, int cols, int ldx, float* out, int accumulate, float* ws,
                size_t ws_bytes, hipStream_t s) {
    int nparts = cdiv(rows, CS_ROWS);
    dim3 grid(cdiv(cols, 256), nparts);
    bool direct = nparts == 1;
    if (!direct) {
        size_t need = (size_t)nparts * cols * sizeof(float);
        ERGM_CHECK_ARG(ws && ws_bytes >= need, "colsum: workspace %zu < %zu", ws_bytes, need);
    }
    if (bf16_in)
        ERGM_LAUNCH(colsum_partial_kernel<true>, grid, dim3(256), 0, s, X, rows, cols, ldx, ws, out, accumulate,
                           (int)direct);
    else
        ERGM_LAUNCH(colsum_partial_kernel<false>, grid, dim3(256), 0, s, X, rows, cols, ldx, ws, out, accumulate,
                           (int)direct);
    if (!direct)
        ERGM_LAUNCH(colsum_final_kernel, dim3(cdiv(cols, 256)), dim3(256), 0, s, ws, nparts, cols, out,
                           accumulate);
    return check_launch("colsum");
}

size_t colsum_ws(int rows, int cols) {
    int nparts = cdiv(rows, CS_ROWS);
    return nparts > 1 ? (size_t)nparts * cols * sizeof(float) : 0;
}

}  // namespace ergm

using namespace ergm;

namespace ergm {
int layernorm_fwd_ld(const float* x, const float* gamma, const float* beta, void* y, int ldy, float* mean, float* rstd,
                     int rows, int E, float eps, hipStream_t s, void* yq, int ldq, float* qscale, void* qmx, int ld_qmx) {
    ERGM_CHECK_ARG(!yq || ((qscale || qmx) && ldq >= E && ldq % 4 == 0), "layernorm_fwd: bad fp8 output");
    ERGM_CHECK_ARG(!qmx || (E % 32 == 0 && ld_qmx >= rows), "layernorm_fwd: bad MX-fp8 output");
    auto* qm = reinterpret_cast<uint8_t*>(qmx);
    auto* q8 = reinterpret_cast<uint8_t*>(yq);
    ERGM_CHECK_ARG(x && gamma && beta && y && mean && rstd, "layernorm_fwd: null argument");
    ERGM_CHECK_ARG(rows > 0 && E > 0 && E % 4 == 0 && E <= 1024, "layernorm_fwd: unsupported E=%d", E);
    ERGM_CHECK_ARG(ldy >= E && ldy % 4 == 0, "layernorm_fwd: bad ldy");
    dim3 grid(cdiv(rows, 4));
    int nv = cdiv(E, 256);
    auto* yb = reinterpret_cast<__bf16*>(y);
    switch (nv) {
        case 1: ERGM_LAUNCH(ln_fwd_kernel<1>, grid, dim3(256), 0, s, x, gamma, beta, yb, mean, rstd, rows, E, ldy, eps, q8, ldq, qscale, qm, ld_qmx); break;
        case 2: ERGM_LAUNCH(ln_fwd_kernel<2>, grid, dim3(256), 0, s, x, gamma, beta, yb, mean, rstd, rows, E, ldy, eps, q8, ldq, qscale, qm, ld_qmx); break;
        case 3: ERGM_LAUNCH(ln_fwd_kernel<3>, grid, dim3(256), 0, s, x, gamma, beta, yb, mean, rstd, rows, E, ldy, eps, q8, ldq, qscale, qm, ld_qmx); break;
        default: ERGM_LAUNCH(ln_fwd_kernel<4>, grid, dim3(256), 0, s, x, gamma, beta, yb, mean, rstd, rows, E, ldy, eps, q8, ldq, qscale, qm, ld_qmx); break;
    }
    return check_launch("layernorm_fwd");
}

// p[r*ld + col] = 1, p[r*ld + col+1 .. col+7] = 0: the constant "ones" column that turns a weight-
// gradient GEMM Xᵀ·dY into [dW; db] (row K of the augmented product is Σ_t dY[t]).
__global__ void ones_col_kernel(__bf16* p, int rows, int ld, int col) {
    int r = blockIdx.x * 256 + threadIdx.x;
    if (r >= rows) return;
    bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = f2bf(j == 0 ? 1.f : 0.f);
    *reinterpret_cast<bf16x8*>(p + (size_t)r * ld + col) = v;
}

int fill_ones_col(void* p, int rows, int ld, int col, hipStream_t s) {
    ERGM_CHECK_ARG(p && rows > 0 && col % 8 == 0 && ld >= col + 8, "fill_ones_col: bad argument");
    ERGM_LAUNCH(ones_col_kernel, dim3(cdiv(rows, 256)), dim3(256), 0, s, reinterpret_cast<__bf16*>(p), rows, ld,
                       col);
    return check_launch("fill_ones_col");
}
}  // namespace ergm

extern "C" int ergm_layernorm_fwd(const float* x, const float* gamma, const float* beta, void* y, float* mean,
                                  float* rstd, int rows, int E, float eps, void* stream) {
    return layernorm_fwd_ld(x, gamma, beta, y, E, mean, rstd, rows, E, eps, as_stream(stream), nullptr, 0, nullptr,
                            nullptr, 0);
}

namespace ergm {
int ln_bwd_nparts(int rows);
}
extern "C" size_t ergm_layernorm_bwd_workspace_size(int rows, int E) {
    int nb = ln_bwd_nparts(rows);
    return 2 * (size_t)nb * E * sizeof(float);
}

namespace ergm {
// Main LayerNorm-backward pass only: dres += dx, dres_bf16, and per-block dγ/dβ partials
// (part_g/part_b: ln_bwd_nparts(rows) x E floats each), reduced later by layernorm_param_reduce.
// drop_res: the updated dres is final and itself goes through `drop` (dres_bf16 then gets the same values).
int ln_bwd_rows_per_part() { return LN_ROWS_PER_BLOCK_BWD; }
int ln_bwd_nparts(int rows) { return cdiv(rows, ln_bwd_rows_per_part()); }

int layernorm_bwd_main(const void* dy, int dy_bf16, const float* x, const float* mean, const float* rstd,
                       const float* gamma, float* dres, void* dres_bf16, float* part_g, float* part_b, int rows, int E,
                       hipStream_t s, const DropSite& drop, int drop_res, void* qmx, void* qmx_s, int ld_qs) {
    ERGM_CHECK_ARG(dy && x && mean && rstd && gamma && dres && part_g && part_b, "layernorm_bwd: null argument");
    ERGM_CHECK_ARG(rows > 0 && E > 0 && E % 4 == 0 && E <= 1024, "layernorm_bwd: unsupported E=%d", E);
    ERGM_CHECK_ARG(!qmx || (dres_bf16 && qmx_s && E % 32 == 0 && ld_qs >= rows), "layernorm_bwd: bad MX-fp8 output");
    auto* q8 = reinterpret_cast<uint8_t*>(qmx);
    auto* qs = reinterpret_cast<uint8_t*>(qmx_s);
    const int nb = ln_bwd_nparts(rows);
    auto* db = reinterpret_cast<__bf16*>(dres_bf16);
#define LN_BWD_LAUNCH(NV, B)                                                                                     \
    ERGM_LAUNCH((ln_bwd_kernel<NV, B>), dim3(nb), dim3(64 * LN_WAVES_BWD), 0, s, dy, x, mean, rstd, gamma, dres, db,   \
                part_g, part_b, rows, E, drop, drop_res, q8, qs, ld_qs)
    switch (cdiv(E, 256) * 2 + (dy_bf16 ? 1 : 0)) {
        case 2: LN_BWD_LAUNCH(1, false); break;
        case 3: LN_BWD_LAUNCH(1, true); break;
        case 4: LN_BWD_LAUNCH(2, false); break;
        case 5: LN_BWD_LAUNCH(2, true); break;
        case 6: LN_BWD_LAUNCH(3, false); break;
        case 7: LN_BWD_LAUNCH(3, true); break;
        case 8: LN_BWD_LAUNCH(4, false); break;
        default: LN_BWD_LAUNCH(4, true); break;
    }
#undef LN_BWD_LAUNCH
    return check_launch("layernorm_bwd");
}

int layernorm_param_reduce_n(int n, const float* const* part_g, const float* const* part_b, int rows, int E,
                             float* const* dgamma, float* const* dbeta, hipStream_t s) {
    ERGM_CHECK_ARG(n >= 1 && n <= 4, "layernorm_param_reduce: 1..4 jobs per launch");
    LnReduceJobs j{};
    for (int i = 0; i < n; ++i) {
        ERGM_CHECK_ARG(part_g[i] && part_b[i] && dgamma[i] && dbeta[i], "layernorm_param_reduce: null argument");
        j.part_g[i] = part_g[i]; j.part_b[i] = part_b[i]; j.dgamma[i] = dgamma[i]; j.dbeta[i] = dbeta[i];
    }
    ERGM_LAUNCH(ln_param_reduce_kernel, dim3(cdiv(E, 32), 2, n), dim3(256), 0, s, j, ln_bwd_nparts(rows), E);
    return check_launch("layernorm_param_reduce");
}

int layernorm_param_reduce(const float* part_g, const float* part_b, int rows, int E, float* dgamma, float* dbeta,
                           hipStream_t s) {
    return layernorm_param_reduce_n(1, &part_g, &part_b, rows, E, &dgamma, &dbeta, s);
}
}  // namespace ergm

extern "C" int ergm_layernorm_bwd(const float* dy, const float* x, const float* mean, const float* rstd,
                                  const float* gamma, float* dres, void* dres_bf16, float* dgamma, float* dbeta,
                                  void* ws, size_t ws_bytes, int rows, int E, const ergm_dropout* dropout,
                                  void* stream) {
    ERGM_CHECK_ARG(dgamma && dbeta, "layernorm_bwd: null argument");
    ERGM_TRY(check_dropout(dropout));
    ERGM_CHECK_ARG(ws && ws_bytes >= ergm_layernorm_bwd_workspace_size(rows, E), "layernorm_bwd: workspace too small");
    const int nb = ln_bwd_nparts(rows);
    float* pg = reinterpret_cast<float*>(ws);
    float* pb = pg + (size_t)nb * E;
    hipStream_t s = as_stream(stream);
    ERGM_TRY(layernorm_bwd_main(dy, 0, x, mean, rstd, gamma, dres, dres_bf16, pg, pb, rows, E, s, drop_site_of(dropout, E), 0,
                                 nullptr, nullptr, 0));
    return layernorm_param_reduce(pg, pb, rows, E, dgamma, dbeta, s);
}

extern "C" size_t ergm_colsum_workspace_size(int rows, int cols) { return colsum_ws(rows, cols); }

extern "C" int ergm_colsum(const void* X, int x_dtype, int rows, int cols, int ldx, float* out, int accumulate,
                           void* ws, size_t ws_bytes, void* stream) {
    ERGM_CHECK_ARG(X && out, "colsum: null argument");
    ERGM_CHECK_ARG(rows > 0 && cols > 0 && cols % 4 == 0 && ldx % 4 == 0 && ldx >= cols, "colsum: bad shape");
    ERGM_CHECK_ARG(x_dtype == ERGM_F32 || x_dtype == ERGM_BF16, "colsum: bad dtype");
    return colsum_impl(X, x_dtype == ERGM_BF16, rows, cols, ldx, out, accumulate, reinterpret_cast<float*>(ws),
                       ws_bytes, as_stream(stream));
}
