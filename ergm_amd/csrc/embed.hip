// Token / position / token-type embeddings with visual+audio fusion, and their backward, for gfx950.
//
// Forward replaces src/model.py:459-463 (wte(input_ids), wte(caption_ids)), :495-498 (per-sample
// Python loop adding imgs[i][0] to position 0 and auds[i] to position 1 — 2B tiny launches in the
// reference, one fused pass here) and :500-504 (+ wpe(arange(S)) + wte(token_type_ids)).
// Backward replaces the autograd Embedding backward into the tied wte (lm_head shares it) and wpe.
// Determinism: the 3·B·S (row, source) entries are sorted by (vocab id, entry index) in one LDS
// bitonic sort; each segment of equal ids is then summed in entry order by one workgroup — no float
// atomics (the token-type rows would otherwise take ~B·S/2 colliding adds each).
#include "common.h"

#include <algorithm>

namespace ergm {

template <int NV>
__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ ids, const int64_t* __restrict__ tt,
                                                        const int64_t* __restrict__ cap_ids, const float* __restrict__ wte,
                                                        const float* __restrict__ wpe, const float* __restrict__ vis,
                                                        int ld_vis, const float* __restrict__ aud,
                                                        float* __restrict__ h0, __bf16* __restrict__ cap, int ld_cap,
                                                        int B, int S, int E, int V, DropSite drop) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int t = blockIdx.x * 4 + wave;
    if (t >= B * S) return;
    const int b = t / S, s = t % S;
    const int64_t id = ids[t];
    const int64_t ty = tt ? tt[t] : -1;
    const int64_t cid = cap_ids[t];
    const bool ok_id = id >= 0 && id < V, ok_ty = ty >= 0 && ty < V, ok_c = cid >= 0 && cid < V;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        int c = (i * 64 + lane) * 4;
        if (c >= E) continue;
        float4 x = ok_id ? *reinterpret_cast<const float4*>(wte + (size_t)id * E + c) : make_float4(0, 0, 0, 0);
        if (vis && s == 0) {
            float4 f = *reinterpret_cast<const float4*>(vis + (size_t)b * ld_vis + c);
            x.x += f.x; x.y += f.y; x.z += f.z; x.w += f.w;
        } else if (aud && s == 1) {
            float4 f = *reinterpret_cast<const float4*>(aud + (size_t)b * E + c);
            x.x += f.x; x.y += f.y; x.z += f.z; x.w += f.w;
        }
        float4 p = *reinterpret_cast<const float4*>(wpe + (size_t)s * E + c);
        x.x += p.x; x.y += p.y; x.z += p.z; x.w += p.w;
        if (ok_ty) {
            float4 y = *reinterpret_cast<const float4*>(wte + (size_t)ty * E + c);
            x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w;
        }
        if (drop.thresh) {  // self.drop(hidden_states), src/model.py:506
            const unsigned k = drop_keep4(drop, t, c);
            x.x = (k & 1u) ? x.x * drop.scale : 0.f;
            x.y = (k & 2u) ? x.y * drop.scale : 0.f;
            x.z = (k & 4u) ? x.z * drop.scale : 0.f;
            x.w = (k & 8u) ? x.w * drop.scale : 0.f;
        }
        *reinterpret_cast<float4*>(h0 + (size_t)t * E + c) = x;
        float4 cv = ok_c ? *reinterpret_cast<const float4*>(wte + (size_t)cid * E + c) : make_float4(0, 0, 0, 0);
        bf16x4 cb;
        cb[0] = f2bf(cv.x); cb[1] = f2bf(cv.y); cb[2] = f2bf(cv.z); cb[3] = f2bf(cv.w);
        *reinterpret_cast<bf16x4*>(cap + (size_t)t * ld_cap + c) = cb;
    }
}

constexpr int SORT_MAX = 16384;  // entries one workgroup sorts in LDS (128 KiB of u64)

// keys = (vocab id << 32) | entry, entry in [0, 3T): [0,T) input ids, [T,2T) token types, [2T,3T) captions,
// sorted ascending over npad = next_pow2(3T) slots (padding keys ~0 sort last) by a bitonic network.
// One workgroup per chunk of `chunk` = min(npad, SORT_MAX) slots runs every compare of the network that
// stays inside its chunk, in LDS: merge_size = 0 generates the chunk's keys from the ids and runs stages
// 2..chunk; merge_size > chunk loads the chunk and runs the strides < chunk of that stage (the larger
// strides are embed_sort_global_kernel passes).  Directions come from global indices, so the chunks
// compose into the one global network (and a single chunk is the whole sort).  Slots g < n_out are
// written back; row_flag (optional, pre-zeroed, one byte per vocab row), on the last launch only, is set
// for every row the lookups touch.
__global__ __launch_bounds__(1024) void embed_sort_kernel(const int64_t* __restrict__ ids, const int64_t* __restrict__ tt,
                                                          const int64_t* __restrict__ cap_ids, int T, int V, int chunk,
                                                          int merge_size, uint64_t* __restrict__ out, int n_out,
                                                          uint8_t* __restrict__ row_flag) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint64_t* key = reinterpret_cast<uint64_t*>(smem);
    const int n = 3 * T;
    const int base = blockIdx.x * chunk;
    for (int i = threadIdx.x; i < chunk; i += 1024) {
        const int g = base + i;
        uint64_t k = ~0ull;
        if (merge_size) {
            k = out[g];
        } else if (g < n) {
            int src = g / T, t = g - src * T;
            int64_t id = src == 0 ? ids[t] : (src == 1 ? (tt ? tt[t] : -1) : cap_ids[t]);
            if (id >= 0 && id < V) k = ((uint64_t)id << 32) | (uint64_t)g;
        }
        key[i] = k;
    }
    __syncthreads();
    auto stage = [&](int size, int stride) {
        for (int i = threadIdx.x; i < chunk / 2; i += 1024) {
            int lo = 2 * i - (i & (stride - 1));
            int hi = lo + stride;
            bool up = ((base + lo) & size) == 0;
            uint64_t a = key[lo], b = key[hi];
            if ((a > b) == up) {
                key[lo] = b;
                key[hi] = a;
            }
        }
        __syncthreads();
    };
    if (merge_size) {
        for (int stride = chunk >> 1; stride > 0; stride >>= 1) stage(merge_size, stride);
    } else {
        for (int size = 2; size <= chunk; size <<= 1)
            for (int stride = size >> 1; stride > 0; stride >>= 1) stage(size, stride);
    }
    for (int i = threadIdx.x; i < chunk; i += 1024) {
        const int g = base + i;
        if (g >= n_out) continue;
        const uint64_t k = key[i];
        out[g] = k;
        if (row_flag && k != ~0ull) row_flag[k >> 32] = 1;
    }
}

// one compare-exchange step of stage `size` at a stride >= the chunk (pairs span chunks)
__global__ __launch_bounds__(256) void embed_sort_global_kernel(uint64_t* __restrict__ key, int npad, int size,
                                                                int stride) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= npad / 2) return;
    const int lo = 2 * i - (i & (stride - 1));
    const int hi = lo + stride;
    const bool up = (lo & size) == 0;
    const uint64_t a = key[lo], b = key[hi];
    if ((a > b) == up) {
        key[lo] = b;
        key[hi] = a;
    }
}

// Pass 1: one workgroup per chunk of SEG_CH sorted positions.  Every maximal run of equal ids inside
// the chunk is summed in position order and written to part[run start].  The chunk's rows are all
// loaded before the (ordered) sum, so the SEG_CH row reads are in flight together.
constexpr int SEG_CH = 16;

__device__ __forceinline__ const float* seg_row(uint64_t key, int T, const float* dh0, const float* dcap, int E) {
    int e = (int)(uint32_t)key;
    return e < 2 * T ? dh0 + (size_t)(e < T ? e : e - T) * E : dcap + (size_t)(e - 2 * T) * E;
}

template <int NC>
__global__ __launch_bounds__(256) void embed_runsum_kernel(const uint64_t* __restrict__ keys, int n, int T,
                                                           const float* __restrict__ dh0, const float* __restrict__ dcap,
                                                           float* __restrict__ part, int E) {
    const int p0 = blockIdx.x * SEG_CH;
    if (keys[p0] == ~0ull) return;
    uint64_t kq[SEG_CH];
    float v[SEG_CH][NC];
#pragma unroll
    for (int q = 0; q < SEG_CH; ++q) {
        kq[q] = p0 + q < n ? keys[p0 + q] : ~0ull;
        const float* row = kq[q] != ~0ull ? seg_row(kq[q], T, dh0, dcap, E) : nullptr;
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            const int c = threadIdx.x + j * 256;
            v[q][j] = row && c < E ? row[c] : 0.f;
        }
    }
    float acc[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) acc[j] = 0.f;
    int start = p0;
    uint32_t id = (uint32_t)(kq[0] >> 32);
#pragma unroll
    for (int q = 0; q < SEG_CH; ++q) {
        if (kq[q] == ~0ull) break;
        const uint32_t iq = (uint32_t)(kq[q] >> 32);
        if (iq != id) {
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                const int c = threadIdx.x + j * 256;
                if (c < E) part[(size_t)start * E + c] = acc[j];
                acc[j] = 0.f;
            }
            start = p0 + q;
            id = iq;
        }
#pragma unroll
        for (int j = 0; j < NC; ++j) acc[j] += v[q][j];
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        const int c = threadIdx.x + j * 256;
        if (c < E) part[(size_t)start * E + c] = acc[j];
    }
}

// Pass 2: one workgroup per sorted position; segment heads add their run partials (the run at the
// head, then one run per following chunk while the id continues) in order to dwte[id].
template <int NC>
__global__ __launch_bounds__(256) void embed_segsum_kernel(const uint64_t* __restrict__ keys, int n,
                                                           const float* __restrict__ part, float* __restrict__ dwte,
                                                           const int* __restrict__ row_pos, int E) {
    const int p = blockIdx.x;
    const uint64_t k = keys[p];
    if (k == ~0ull) return;
    const uint32_t id = (uint32_t)(k >> 32);
    if (p > 0 && (uint32_t)(keys[p - 1] >> 32) == id) return;
    float acc[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        int c = threadIdx.x + j * 256;
        acc[j] = c < E ? part[(size_t)p * E + c] : 0.f;
    }
    // the run continues into chunk q while keys[q] (the chunk's first key) still has this id; keys are
    // sorted, so that holds for a prefix of the following chunks: fetch 8 chunk partials at a time
    constexpr int G = 8;
    for (int q0 = (p / SEG_CH + 1) * SEG_CH; q0 < n; q0 += G * SEG_CH) {
        bool more[G];
        float v[G][NC];
#pragma unroll
        for (int i = 0; i < G; ++i) {
            const int q = q0 + i * SEG_CH;
            const uint64_t kq = q < n ? keys[q] : ~0ull;
            more[i] = kq != ~0ull && (uint32_t)(kq >> 32) == id;
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                const int c = threadIdx.x + j * 256;
                v[i][j] = more[i] && c < E ? part[(size_t)q * E + c] : 0.f;
            }
        }
#pragma unroll
        for (int i = 0; i < G; ++i)
#pragma unroll
            for (int j = 0; j < NC; ++j) acc[j] += v[i][j];
        if (!more[G - 1]) break;
    }
    // dense: accumulate into dwte[id]; compact (row_pos given): the zeroed slot row_pos[id] of dwte
    float* dst = dwte + (size_t)(row_pos ? row_pos[id] : id) * E;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
        int c = threadIdx.x + j * 256;
        if (c < E) dst[c] += acc[j];
    }
}

// ---- compact lookup rows (data parallelism) ------------------------------------------------------
// The lookup part of the tied-wte gradient lives in the rows the batch touched.  Under data
// parallelism the union of those rows over all ranks (flags all-reduced with MAX) is numbered by an
// exclusive prefix sum, the lookup sums go to compact[pos[row]], and only that compact block is
// all-reduced and added back — instead of a second all-reduce of the whole [V, E] gradient.

// pos[r] = number of flagged rows before r; count[0] = total.  One workgroup (n <= 1024 * 1024).
__global__ __launch_bounds__(1024) void rows_scan_kernel(const uint8_t* __restrict__ flag, int n, int* __restrict__ pos,
                                                         int* __restrict__ count) {
    __shared__ int part[1024];
    const int per = (n + 1023) / 1024;
    const int r0 = threadIdx.x * per, r1 = min(n, r0 + per);
    int c = 0;
    for (int r = r0; r < r1; ++r) c += flag[r] != 0;
    part[threadIdx.x] = c;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // inclusive Hillis-Steele scan
        int v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    int run = threadIdx.x ? part[threadIdx.x - 1] : 0;
    for (int r = r0; r < r1; ++r) {
        pos[r] = run;
        run += flag[r] != 0;
    }
    if (threadIdx.x == 1023) count[0] = part[1023];
}

// mode 0: compact[pos[r]] = 0;  mode 1: dst[r] += compact[pos[r]]   (flagged rows r only)
__global__ __launch_bounds__(256) void rows_compact_kernel(const uint8_t* __restrict__ flag, const int* __restrict__ pos,
                                                           int n, int row4, float4* __restrict__ compact,
                                                           float4* __restrict__ dst, int mode) {
    for (int r = blockIdx.x; r < n; r += gridDim.x) {
        if (!flag[r]) continue;
        float4* c = compact + (size_t)pos[r] * row4;
        for (int j = threadIdx.x; j < row4; j += 256) {
            if (mode == 0) {
                c[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            } else {
                float4 a = dst[(size_t)r * row4 + j], b = c[j];
                a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
                dst[(size_t)r * row4 + j] = a;
            }
        }
    }
}

int colsum_impl(const void* X, bool bf16_in, int rows, int cols, int ldx, float* out, int accumulate, float* ws,
                size_t ws_bytes, hipStream_t s);
size_t colsum_ws(int rows, int cols);

static int next_pow2(int x) {
    int p = 1;
    while (p < x) p <<= 1;
    return p;
}

}  // namespace ergm

using namespace ergm;

namespace ergm {
int embed_fwd_ld(const int64_t* ids, const int64_t* tt, const int64_t* cap_ids, const float* wte, const float* wpe,
                 const float* vis, int ld_vis, const float* aud, float* h0, void* cap, int ld_cap, int B, int S, int E,
                 int V, hipStream_t s, const DropSite& drop) {
    ERGM_CHECK_ARG(ids && cap_ids && wte && wpe && h0 && cap, "embed_fwd: null argument");
    ERGM_CHECK_ARG(B > 0 && S > 0 && E > 0 && E % 4 == 0 && E <= 1024 && V > 0, "embed_fwd: bad shape");
    ERGM_CHECK_ARG((vis == nullptr) == (aud == nullptr), "embed_fwd: visual and audio features go together");
    ERGM_CHECK_ARG(!vis || (ld_vis >= E && ld_vis % 4 == 0), "embed_fwd: bad ld_vis");
    const int T = B * S;
    dim3 grid(cdiv(T, 4));
    ERGM_CHECK_ARG(ld_cap >= E && ld_cap % 4 == 0, "embed_fwd: bad ld_cap");
    auto* cb = reinterpret_cast<__bf16*>(cap);
    switch (cdiv(E, 256)) {
        case 1: ERGM_LAUNCH(embed_fwd_kernel<1>, grid, dim3(256), 0, s, ids, tt, cap_ids, wte, wpe, vis, ld_vis, aud, h0, cb, ld_cap, B, S, E, V, drop); break;
        case 2: ERGM_LAUNCH(embed_fwd_kernel<2>, grid, dim3(256), 0, s, ids, tt, cap_ids, wte, wpe, vis, ld_vis, aud, h0, cb, ld_cap, B, S, E, V, drop); break;
        case 3: ERGM_LAUNCH(embed_fwd_kernel<3>, grid, dim3(256), 0, s, ids, tt, cap_ids, wte, wpe, vis, ld_vis, aud, h0, cb, ld_cap, B, S, E, V, drop); break;
        default: ERGM_LAUNCH(embed_fwd_kernel<4>, grid, dim3(256), 0, s, ids, tt, cap_ids, wte, wpe, vis, ld_vis, aud, h0, cb, ld_cap, B, S, E, V, drop); break;
    }
    return check_launch("embed_fwd");
}
}  // namespace ergm

extern "C" int ergm_embed_fwd(const int64_t* ids, const int64_t* tt, const int64_t* cap_ids, const float* wte,
                              const float* wpe, const float* vis, int ld_vis, const float* aud, float* h0, void* cap,
                              int B, int S, int E, int V, const ergm_dropout* dropout, void* stream) {
    ERGM_TRY(check_dropout(dropout));
    return embed_fwd_ld(ids, tt, cap_ids, wte, wpe, vis, ld_vis, aud, h0, cap, E, B, S, E, V, as_stream(stream),
                        drop_site_of(dropout, E));
}

namespace ergm {
// sorted-key slots: 3T when one workgroup sorts them all, else the padded network width
int embed_sort_capacity(int T) { return 3 * T <= SORT_MAX ? 3 * T : next_pow2(3 * T); }
}  // namespace ergm

static size_t keys_bytes(int T) { return ((size_t)embed_sort_capacity(T) * sizeof(uint64_t) + 255) & ~(size_t)255; }

extern "C" size_t ergm_embed_bwd_workspace_size(int T) {
    // sorted keys + one partial row per sorted position (run sums); E <= 1024
    return keys_bytes(T) + (size_t)3 * T * 1024 * sizeof(float);
}

namespace ergm {
// Sort the lookups of one batch by vocabulary row (only needs the ids: the training executor runs it
// during the forward, off the critical path) and flag the touched rows.
int embed_bwd_sort(const int64_t* ids, const int64_t* tt, const int64_t* cap_ids, int T, int V, uint64_t* keys,
                   uint8_t* row_flag, int n_flag, hipStream_t s) {
    ERGM_CHECK_ARG(ids && cap_ids && keys, "embed_bwd: null argument");
    ERGM_CHECK_ARG(T > 0 && 3 * T <= (1 << 30), "embed_bwd: bad token count %d", T);
    ERGM_CHECK_ARG(!row_flag || n_flag >= V, "embed_bwd: row_flag shorter than the vocabulary");
    static bool attr_set = false;  // benign race: idempotent attribute write
    if (!attr_set) {
        if (hipFuncSetAttribute((const void*)embed_sort_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                SORT_MAX * (int)sizeof(uint64_t)) != hipSuccess)
            return fail(ERGM_EHIP, "embed_bwd: cannot raise dynamic LDS limit");
        attr_set = true;
    }
    if (row_flag && hipMemsetAsync(row_flag, 0, (size_t)n_flag, s) != hipSuccess)
        return fail(ERGM_EHIP, "embed_bwd: memset");
    const int n = 3 * T, npad = next_pow2(n);
    const int chunk = std::min(npad, SORT_MAX), nch = npad / chunk;
    const size_t lds = (size_t)chunk * sizeof(uint64_t);
    // (keys holds embed_sort_capacity(T) slots: n for one chunk, npad for several)
    ERGM_LAUNCH(embed_sort_kernel, dim3(nch), dim3(1024), lds, s, ids, tt, cap_ids, T, V, chunk, 0, keys,
                       nch > 1 ? npad : n, nch > 1 ? nullptr : row_flag);
    for (int size = 2 * chunk; size <= npad; size <<= 1) {
        for (int stride = size >> 1; stride >= chunk; stride >>= 1)
            ERGM_LAUNCH(embed_sort_global_kernel, dim3(cdiv(npad / 2, 256)), dim3(256), 0, s, keys, npad, size,
                               stride);
        const bool last = size == npad;
        ERGM_LAUNCH(embed_sort_kernel, dim3(nch), dim3(1024), lds, s, ids, tt, cap_ids, T, V, chunk, size, keys,
                           last ? n : npad, last ? row_flag : nullptr);
    }
    return check_launch("embed_bwd_sort");
}

// dwte[id] += Σ (ordered) of the lookup gradients of each sorted run; dwpe = Σ_b dh0[b].
// part: 3T x E floats of scratch (reused, once the runs are summed, by the dwpe column sums).
int embed_bwd_sums(const uint64_t* keys, int B, int S, int E, const float* dh0, const float* dcap, float* dwte,
                   float* dwpe, float* part, const int* row_pos, hipStream_t s) {
    const int T = B * S, n = 3 * T;
    dim3 g1(cdiv(n, SEG_CH)), g2(n);
#define ERGM_SEG(NC)                                                                                         \
    ERGM_LAUNCH(embed_runsum_kernel<NC>, g1, dim3(256), 0, s, keys, n, T, dh0, dcap, part, E);         \
    ERGM_LAUNCH(embed_segsum_kernel<NC>, g2, dim3(256), 0, s, keys, n, part, dwte, row_pos, E);
    switch (cdiv(E, 256)) {
        case 1: ERGM_SEG(1) break;
        case 2: ERGM_SEG(2) break;
        case 3: ERGM_SEG(3) break;
        default: ERGM_SEG(4) break;
    }
#undef ERGM_SEG
    ERGM_TRY(check_launch("embed_bwd"));
    // dwpe[s][e] = Σ_b dh0[b][s][e]   (rows b of [B][S*E])
    return colsum_impl(dh0, false, B, S * E, S * E, dwpe, 0, part, (size_t)n * E * sizeof(float), s);
}
}  // namespace ergm

extern "C" int ergm_embed_bwd(const int64_t* ids, const int64_t* tt, const int64_t* cap_ids, const float* dh0,
                              const float* dcap, float* dwte, float* dwpe, void* ws, size_t ws_bytes, int B, int S, int E,
                              int V, void* stream) {
    ERGM_CHECK_ARG(ids && cap_ids && dh0 && dcap && dwte && dwpe, "embed_bwd: null argument");
    ERGM_CHECK_ARG(B > 0 && S > 0 && E > 0 && E % 4 == 0 && E <= 1024, "embed_bwd: bad shape");
    const int T = B * S;
    ERGM_CHECK_ARG(ws && ws_bytes >= ergm_embed_bwd_workspace_size(T), "embed_bwd: workspace too small");
    hipStream_t s = as_stream(stream);
    uint64_t* keys = reinterpret_cast<uint64_t*>(ws);
    ERGM_TRY(embed_bwd_sort(ids, tt, cap_ids, T, V, keys, nullptr, 0, s));
    float* part = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + keys_bytes(T));
    return embed_bwd_sums(keys, B, S, E, dh0, dcap, dwte, dwpe, part, nullptr, s);
}

extern "C" int ergm_rows_scan(const void* row_flag, int n, int* pos, int* count, void* stream) {
    ERGM_CHECK_ARG(row_flag && pos && count && n > 0 && n <= 1024 * 1024, "rows_scan: bad argument");
    ERGM_LAUNCH(rows_scan_kernel, dim3(1), dim3(1024), 0, as_stream(stream), (const uint8_t*)row_flag, n, pos,
                       count);
    return check_launch("rows_scan");
}

extern "C" int ergm_rows_compact(const void* row_flag, const int* pos, int n, int row_len, float* compact, float* dst,
                                 int mode, void* stream) {
    ERGM_CHECK_ARG(row_flag && pos && compact && n > 0 && row_len > 0 && row_len % 4 == 0, "rows_compact: bad argument");
    ERGM_CHECK_ARG(mode == 0 || (mode == 1 && dst), "rows_compact: mode 0 (zero) or 1 (scatter-add into dst)");
    ERGM_CHECK_ARG(aligned16(compact) && (!dst || aligned16(dst)), "rows_compact: 16-byte alignment");
    ERGM_LAUNCH(rows_compact_kernel, dim3(std::min(n, 8192)), dim3(256), 0, as_stream(stream),
                       (const uint8_t*)row_flag, pos, n, row_len / 4, (float4*)compact, (float4*)dst, mode);
    return check_launch("rows_compact");
}

// ---- feature projection operands (build-side config 5: feat_dim != n_embd) --------
namespace ergm {

// out[m][b][k] (bf16, [2][Bp][ld]) = bf16(src_m[b][k]) for b < B, 0 for the pad rows b in [B, Bp);
// src_0 = the visual row 0 (vis + b*ld_vis), src_1 = the audio vector (aud + b*Fd).  Column Fd is the
// constant 1 of the fused-bias weight-gradient GEMM, columns Fd+1 .. ld-1 are 0.
__global__ __launch_bounds__(256) void feat_pack_kernel(const float* __restrict__ vis, int ld_vis,
                                                        const float* __restrict__ aud, __bf16* __restrict__ out,
                                                        int B, int Bp, int Fd, int ld) {
    const int row = blockIdx.x;  // m * Bp + b
    const int m = row / Bp, b = row % Bp;
    const float* src = b < B ? (m == 0 ? vis + (size_t)b * ld_vis : aud + (size_t)b * Fd) : nullptr;
    __bf16* dst = out + (size_t)row * ld;
    for (int k = threadIdx.x; k < ld; k += 256) {
        float v = k < Fd ? (src ? src[k] : 0.f) : (k == Fd ? 1.f : 0.f);
        dst[k] = f2bf(v);
    }
}

// d[m][b][n] (bf16, [2][Bp][E]) = bf16(dh0[b*S + m][n]) for b < B (the gradient reaching the
// projected visual (m=0, position 0) and audio (m=1, position 1) vectors), 0 for the pad rows.
__global__ __launch_bounds__(256) void proj_grad_pack_kernel(const float* __restrict__ dh0, __bf16* __restrict__ d,
                                                             int B, int Bp, int S, int E) {
    const int row = blockIdx.x;
    const int m = row / Bp, b = row % Bp;
    for (int n = threadIdx.x; n < E; n += 256)
        d[(size_t)row * E + n] = f2bf(b < B ? dh0[((size_t)b * S + m) * E + n] : 0.f);
}

int feat_pack(const float* vis, int ld_vis, const float* aud, void* out, int B, int Bp, int Fd, int ld,
              hipStream_t s) {
    ERGM_CHECK_ARG(vis && aud && out && B > 0 && Bp >= B && ld > Fd, "feat_pack: bad argument");
    ERGM_LAUNCH(feat_pack_kernel, dim3(2 * Bp), dim3(256), 0, s, vis, ld_vis, aud,
                       reinterpret_cast<__bf16*>(out), B, Bp, Fd, ld);
    return check_launch("feat_pack");
}

int proj_grad_pack(const float* dh0, void* d, int B, int Bp, int S, int E, hipStream_t s) {
    ERGM_CHECK_ARG(dh0 && d && B > 0 && Bp >= B && S >= 2, "proj_grad_pack: bad argument");
    ERGM_LAUNCH(proj_grad_pack_kernel, dim3(2 * Bp), dim3(256), 0, s, dh0, reinterpret_cast<__bf16*>(d), B, Bp,
                       S, E);
    return check_launch("proj_grad_pack");
}

}  // namespace ergm

// ---- feature pooling (data_process/feature_extraction.py:63,69) -------------
// out[b][d] = mean over the valid frames t < len_b of x[b][t][d]: the torch.mean(last_hidden_state,
// dim=1) the reference applies offline to wav2vec2 (audio) and BLIP-vision (keyframe) encoder outputs,
// on the GPU, with optional per-sample lengths for padded audio.  Block = 64 feature columns x 4 frame
// groups (coalesced 64-column rows); the 4 partial sums are combined in a fixed order (deterministic).
namespace ergm {
template <bool BF16>
__global__ __launch_bounds__(256) void feat_pool_kernel(const void* __restrict__ x, int T, int D, long ld_t,
                                                        long ld_b, const int* __restrict__ lengths,
                                                        float* __restrict__ out, int ld_out) {
    __shared__ float red[4][64];
    const int b = blockIdx.y, col = threadIdx.x & 63, rg = threadIdx.x >> 6;
    const int d = blockIdx.x * 64 + col;
    const int n = lengths ? max(0, min(T, lengths[b])) : T;
    float s = 0.f;
    if (d < D) {
        for (int t = rg; t < n; t += 4) {
            const size_t i = (size_t)b * ld_b + (size_t)t * ld_t + d;
            s += BF16 ? bf2f(reinterpret_cast<const __bf16*>(x)[i]) : reinterpret_cast<const float*>(x)[i];
        }
    }
    red[rg][col] = s;
    __syncthreads();
    if (rg == 0 && d < D) {
        const float tot = (red[0][col] + red[1][col]) + (red[2][col] + red[3][col]);
        out[(size_t)b * ld_out + d] = n > 0 ? tot / (float)n : 0.f;
    }
}
}  // namespace ergm

extern "C" int ergm_feat_pool(const void* x, int x_dtype, int B, int T, int D, long ld_t, long ld_b,
                              const int* lengths, float* out, int ld_out, void* stream) {
    using namespace ergm;
    ERGM_CHECK_ARG(x && out && B > 0 && T > 0 && D > 0 && ld_t >= D && ld_b >= (long)T * ld_t && ld_out >= D,
                   "feat_pool: bad shape");
    ERGM_CHECK_ARG(x_dtype == ERGM_F32 || x_dtype == ERGM_BF16, "feat_pool: bad dtype");
    dim3 grid(cdiv(D, 64), B);
    hipStream_t s = as_stream(stream);
    if (x_dtype == ERGM_BF16)
        ERGM_LAUNCH(feat_pool_kernel<true>, grid, dim3(256), 0, s, x, T, D, ld_t, ld_b, lengths, out, ld_out);
    else
        ERGM_LAUNCH(feat_pool_kernel<false>, grid, dim3(256), 0, s, x, T, D, ld_t, ld_b, lengths, out, ld_out);
    return check_launch("feat_pool");
}
