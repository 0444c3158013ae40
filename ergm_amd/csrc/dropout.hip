// Dropout for gfx950: the keep masks of nn.Dropout (src/model.py:142 attention probabilities, :245
// attention / cross-attention resid_dropout, :266 MLP dropout, :506 embedding dropout) as a pure
// function of (seed, forward number, site, element) — common.h drop_keep4, Philox4x32-10.
//
// The fused kernels generate the bits they need inline (embedding forward, the residual GEMM epilogue,
// the LayerNorm backward, the attention forward); this file holds the stand-alone forms: the mask
// itself as bits (ergm_dropout_mask: tests replay it through the CPU oracle, and it is the
// definition the fused kernels are checked against) and the in-place application to an f32 tensor
// (ergm_dropout_apply: the executor's embedding-dropout backward).
#include "common.h"

#include <cmath>

namespace ergm {

DropSite make_drop_site(uint64_t seed, uint32_t offset, uint32_t site, float p, int64_t row0, int64_t cols) {
    DropSite d{};
    d.key0 = (uint32_t)seed;
    d.key1 = (uint32_t)(seed >> 32);
    d.site = site;
    d.offset = offset;
    const double t = std::nearbyint((double)p * 4294967296.0);
    d.thresh = p <= 0.f ? 0u : (t >= 4294967295.0 ? 4294967295u : (uint32_t)t);
    d.scale = p <= 0.f ? 1.f : 1.0f / (1.0f - p);
    d.row0 = row0;
    d.cols4 = (cols + 3) / 4;
    return d;
}

// bits[r][w] (words_per_row = ceil(cols/32)): bit j of word w = keep(r, 32w + j); pad bits 0.
__global__ __launch_bounds__(256) void dropout_mask_kernel(DropSite d, int rows, int cols, int wpr,
                                                           uint32_t* __restrict__ bits) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)rows * wpr) return;
    const int r = (int)(i / wpr), w = (int)(i % wpr);
    uint32_t word = 0;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        const int c = 32 * w + 4 * g;
        if (c < cols) {
            unsigned k = d.thresh ? drop_keep4(d, r, c) : 0xFu;
            const int valid = cols - c;
            if (valid < 4) k &= (1u << valid) - 1u;
            word |= k << (4 * g);
        }
    }
    bits[i] = word;
}

// x[r][c] = keep(r, c) ? x·scale : 0 (f32, row stride ld, cols % 4 == 0)
__global__ __launch_bounds__(256) void dropout_apply_kernel(DropSite d, float* __restrict__ x, int rows, int cols,
                                                            int ld) {
    const int cg = cols / 4;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)rows * cg) return;
    const int r = (int)(i / cg), c = (int)(i % cg) * 4;
    float4* p = reinterpret_cast<float4*>(x + (size_t)r * ld + c);
    const unsigned k = drop_keep4(d, r, c);
    float4 v = *p;
    v.x = (k & 1u) ? v.x * d.scale : 0.f;
    v.y = (k & 2u) ? v.y * d.scale : 0.f;
    v.z = (k & 4u) ? v.z * d.scale : 0.f;
    v.w = (k & 8u) ? v.w * d.scale : 0.f;
    *p = v;
}

int dropout_apply_f32(const DropSite& d, float* x, int rows, int cols, int ld, hipStream_t s) {
    if (d.thresh == 0) return ERGM_OK;
    ERGM_CHECK_ARG(x && rows > 0 && cols > 0 && cols % 4 == 0 && ld % 4 == 0 && ld >= cols && aligned16(x),
                   "dropout_apply: bad argument");
    const int64_t n = (int64_t)rows * (cols / 4);
    ERGM_LAUNCH(dropout_apply_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, d, x, rows, cols, ld);
    return check_launch("dropout_apply");
}

DropSite drop_site_of(const ergm_dropout* d, int64_t cols) {
    if (!d || !(d->p > 0.f)) return DropSite{};
    return make_drop_site(d->seed, d->offset, d->site, d->p, d->row0, cols);
}

int check_dropout(const ergm_dropout* d) {
    ERGM_CHECK_ARG(!d || (d->p >= 0.f && d->p < 1.f), "dropout: p must be in [0, 1)");
    return ERGM_OK;
}

}  // namespace ergm

using namespace ergm;

extern "C" int ergm_dropout_mask(const ergm_dropout* d, int rows, int cols, uint32_t* bits, void* stream) {
    ERGM_CHECK_ARG(d && bits && rows > 0 && cols > 0, "dropout_mask: bad argument");
    ERGM_TRY(check_dropout(d));
    const DropSite s = make_drop_site(d->seed, d->offset, d->site, d->p, d->row0, cols);
    const int wpr = (cols + 31) / 32;
    const int64_t n = (int64_t)rows * wpr;
    ERGM_LAUNCH(dropout_mask_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, as_stream(stream), s, rows,
                       cols, wpr, bits);
    return check_launch("dropout_mask");
}

extern "C" int ergm_dropout_apply(const ergm_dropout* d, float* x, int rows, int cols, int ld, void* stream) {
    ERGM_CHECK_ARG(d, "dropout_apply: null descriptor");
    ERGM_TRY(check_dropout(d));
    return dropout_apply_f32(drop_site_of(d, cols), x, rows, cols, ld, as_stream(stream));
}
