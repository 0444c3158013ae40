// LDS tile staging for the GEMM kernels (gemm.hip): bf16 operand tiles of ROWS x 64 (k contiguous) or 64 x ROWS (rows contiguous) with
// XOR-swizzled 16-B chunks, filled either through registers (TileLoader) or by LDS-DMA
// (global_load_lds_dwordx4, GldsTile) with the swizzle applied on the source address, and read as
// v_mfma_f32_16x16x32_bf16 operand fragments (ds_read_b128, or ds_read_b64_tr_b16 for the transposed
// image).  Counted waits: wait_vm / wait_stages.
#pragma once

#include "common.h"

namespace ergm {

constexpr int GEMM_BK = 64;
constexpr int GEMM_THREADS = 256;

// XOR swizzles (chunk = 16 bytes).
__device__ __forceinline__ int swz_row(int row) { return row & 7; }  // 128-B rows, row reads
// transposed-read tiles: rows {8g+q} (g=0,1; q=0..3) of a half-wave must hit distinct slots
__device__ __forceinline__ int swz_tr16(int k) { return ((k & 3) | ((k >> 1) & 4)) << 1; }        // 256-B rows
__device__ __forceinline__ int swz_tr8(int k) { return (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) << 1; }  // 128-B rows

// Swizzle family SW of a tile image (the DMA writes and the fragment reads of one kernel use the same one):
//   SW 0 — the v_mfma_f32_16x16x32_bf16 reads above;
//   SW 1 — the v_mfma_f32_32x32x16_bf16 reads (frag32): a row read (ds_read_b128, lanes 0-31 rows r0..r0+31 of one
//   16-B chunk) is conflict-free in each of the instruction's four 16-lane groups with chunk ^ ((row >> 1) & 7); a
//   transposed read (ds_read_b64_tr_b16, a 32-lane half takes 4 k-rows x 32 columns = 4 chunks per row) with chunk ^
//   4·(k & 3) on rows of >= 256 B and chunk ^ 4·((k >> 1) & 1) on 128-B rows (cdna_hip_programming.md T10, §2).
template <bool TRANS, int CPR, int SW>
__device__ __forceinline__ int swz_of(int row) {
    if constexpr (SW == 0) return TRANS ? (CPR == 16 ? swz_tr16(row) : swz_tr8(row)) : swz_row(row);
    else return TRANS ? (CPR == 8 ? ((row >> 1) & 1) << 2 : (row & 3) << 2) : (row >> 1) & 7;
}

template <int ROWS, bool TRANS, int SW = 0>
struct TileLoader {
    // ROWS = tile extent along M (A) or N (B).  !TRANS: tile [ROWS][64] (k contiguous);
    // TRANS: tile [64][ROWS] (ROWS contiguous).
    static constexpr int CHUNKS = ROWS * GEMM_BK / 8;       // 16-B chunks per tile
    static constexpr int PER_THREAD = CHUNKS / GEMM_THREADS;
    static constexpr int CPR = TRANS ? ROWS / 8 : 8;         // chunks per LDS row
    static constexpr int ROW_BYTES = CPR * 16;
    static_assert(PER_THREAD >= 1, "tile too small");

    uint4 regs[PER_THREAD];

    // global → registers. base: operand pointer, ld: leading dim, r0: tile origin along ROWS dim,
    // k0: K origin, R: extent along ROWS dim (M or N), K: contraction extent (k_end).
    __device__ __forceinline__ void load(const __bf16* base, int ld, int r0, int k0, int R, int Kend) {
#pragma unroll
        for (int i = 0; i < PER_THREAD; ++i) {
            int c = threadIdx.x + i * GEMM_THREADS;
            int lrow = c / CPR, lc = c % CPR;
            bool ok;
            const __bf16* p;
            if (!TRANS) {  // row = r, chunk along k
                int r = r0 + lrow, k = k0 + lc * 8;
                ok = (r < R) && (k < Kend);
                p = base + (size_t)r * ld + k;
            } else {       // row = k, chunk along r
                int k = k0 + lrow, r = r0 + lc * 8;
                ok = (k < Kend) && (r < R);
                p = base + (size_t)k * ld + r;
            }
            regs[i] = ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
        }
    }
    __device__ __forceinline__ void store(char* lds) const {
#pragma unroll
        for (int i = 0; i < PER_THREAD; ++i) {
            int c = threadIdx.x + i * GEMM_THREADS;
            int lrow = c / CPR, lc = c % CPR;
            const int pc = lc ^ swz_of<TRANS, CPR, SW>(lrow);
            *reinterpret_cast<uint4*>(lds + lrow * ROW_BYTES + pc * 16) = regs[i];
        }
    }
    // MFMA 16x16x32 operand fragment for the 16 rows starting at `ro` (tile-relative), k-step ks.
    // Lane l gets element j = X[ro + (l&15)][32ks + 8(l>>4) + j].
    __device__ __forceinline__ bf16x8 frag(const char* lds, int ro, int ks) const {
        const int lane = threadIdx.x & 63;
        if (!TRANS) {
            int row = ro + (lane & 15);
            int ch = ks * 4 + (lane >> 4);
            return *reinterpret_cast<const bf16x8*>(lds + row * ROW_BYTES + ((ch ^ swz_of<TRANS, CPR, SW>(row)) << 4));
        } else {
            int i16 = lane & 15, g = lane >> 4;
            int k = ks * 32 + 8 * g + (i16 >> 2);
            int col = ro + 4 * (i16 & 3);
            int ch = col >> 3;
            int sub = (col & 7) * 2;  // byte offset within chunk (0 or 8)
            int s1 = swz_of<TRANS, CPR, SW>(k);
            int s2 = swz_of<TRANS, CPR, SW>(k + 4);
            const char* p1 = lds + k * ROW_BYTES + ((ch ^ s1) << 4) + sub;
            const char* p2 = lds + (k + 4) * ROW_BYTES + ((ch ^ s2) << 4) + sub;
            s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, p1));
            s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, p2));
            typedef __attribute__((ext_vector_type(8))) short s16x8;
            s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            return __builtin_bit_cast(bf16x8, r);
        }
    }
    // MFMA 32x32x16 operand fragment for the 32 rows starting at `ro`, 16-deep k-step kk (0..3) of the 64-deep stage.
    // Lane l gets element j = X[ro + (l&31)][16kk + 8(l>>5) + j] (the v_mfma_f32_32x32x16_bf16 A / B lane map).
    __device__ __forceinline__ bf16x8 frag32(const char* lds, int ro, int kk) const {
        const int lane = threadIdx.x & 63;
        if (!TRANS) {
            const int row = ro + (lane & 31);
            const int ch = kk * 2 + (lane >> 5);
            return *reinterpret_cast<const bf16x8*>(lds + row * ROW_BYTES + ((ch ^ swz_of<TRANS, CPR, SW>(row)) << 4));
        } else {
            // per 16-lane group G: rows k0..k0+3 (then +4..+7) of the 16 columns ro + 16(G&1) ...; lane 4q+p addresses
            // row q, columns 4p..4p+3, and receives its column's 4 rows (T10)
            const int i16 = lane & 15, G = lane >> 4;
            const int k = kk * 16 + 8 * (G >> 1) + (i16 >> 2);
            const int col = ro + 16 * (G & 1) + 4 * (i16 & 3);
            const int ch = col >> 3;
            const int sub = (col & 7) * 2;
            const char* p1 = lds + k * ROW_BYTES + ((ch ^ swz_of<TRANS, CPR, SW>(k)) << 4) + sub;
            const char* p2 = lds + (k + 4) * ROW_BYTES + ((ch ^ swz_of<TRANS, CPR, SW>(k + 4)) << 4) + sub;
            s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, p1));
            s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, p2));
            typedef __attribute__((ext_vector_type(8))) short s16x8;
            s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            return __builtin_bit_cast(bf16x8, r);
        }
    }
};


// ------------------------------------------------------------------------------------------
// Pipelined staging: NS-stage LDS ring filled by global_load_lds_dwordx4 (LDS-DMA, no VGPR staging).
// The DMA writes each wave-instruction's 64 x 16 B lane-linearly, so the XOR swizzles above are applied
// to the per-lane SOURCE address (same involution on the read).  Stage kt is consumed after a counted
// s_waitcnt vmcnt (the younger stages stay in flight) and a raw s_barrier; the freed slot is refilled
// right after that barrier.  Out-of-range rows/columns are CLAMPED to valid memory (never masked), so
// every wave issues the same number of DMA instructions per stage and the counts stay exact; clamped
// data only reaches output rows/columns that are not stored.  Requires K % 64 == 0.
template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Wait until at most `after` stages (LPS DMA instructions each) of this wave are still in flight.
template <int LPS, int MAXA>
__device__ __forceinline__ void wait_stages(int after) {
    if constexpr (MAXA > 0) {
        if (after >= MAXA) {
            wait_vm<MAXA * LPS>();
            return;
        }
        wait_stages<LPS, MAXA - 1>(after);
    } else {
        wait_vm<0>();
    }
}

// One 16-B-per-lane LDS-DMA: LDS[lds_addr + 16*lane] = *gsrc.  Issued from inline asm so hipcc does
// not track it (it would otherwise drain vmcnt before every later ds_read); completion is covered by
// the explicit counted waits.  M0 is saved/set/restored inside the one statement (guide §5.7).
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_addr) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_addr)
                 : "memory");
}

// 4-B-per-lane LDS-DMA: LDS[lds_addr + 4*lane] = *gsrc (a 256-B row of floats per wave-instruction).
__device__ __forceinline__ void glds4(const void* gsrc, uint32_t lds_addr) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_addr)
                 : "memory");
}

__device__ __forceinline__ uint32_t lds_addr_of(const char* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

template <int ROWS, bool TRANS, int NWAVES, int SW = 0>
struct GldsTile {
    static constexpr int BYTES = ROWS * GEMM_BK * 2;
    static constexpr int PER_WAVE = BYTES / 1024 / NWAVES;   // wave-instructions per wave per stage
    static constexpr int CPR = TRANS ? ROWS / 8 : 8;
    static constexpr int ROW_BYTES = CPR * 16;
    static_assert(PER_WAVE >= 1 && PER_WAVE * 1024 * NWAVES == BYTES, "tile / wave count mismatch");

    // r0: tile origin along M|N; Rlim: M|N (valid extent); k0: K origin of the stage.
    // Piece i (0 <= i < PER_WAVE) of this wave's share of the stage: one 1-KiB wave-instruction.
    __device__ __forceinline__ static void issue_piece(char* lds, const __bf16* base, int ld, int r0, int Rlim, int k0,
                                                       int wave, int i) {
        const int lane = threadIdx.x & 63;
        const int ib = (i * NWAVES + wave) * 1024;
        const int o = ib + lane * 16;
        const int row = o / ROW_BYTES, pc = (o % ROW_BYTES) >> 4;
        const __bf16* src;
        if (!TRANS) {
            const int c = pc ^ swz_of<TRANS, CPR, SW>(row);
            const int r = min(r0 + row, Rlim - 1);
            src = base + (size_t)r * ld + k0 + c * 8;
        } else {
            const int c = pc ^ swz_of<TRANS, CPR, SW>(row);
            const int col = min(r0 + c * 8, ((Rlim + 7) & ~7) - 8);
            src = base + (size_t)(k0 + row) * ld + col;
        }
        glds16(src, __builtin_amdgcn_readfirstlane(lds_addr_of(lds + ib)));
    }
    __device__ __forceinline__ static void issue(char* lds, const __bf16* base, int ld, int r0, int Rlim, int k0,
                                                 int wave) {
#pragma unroll
        for (int i = 0; i < PER_WAVE; ++i) issue_piece(lds, base, ld, r0, Rlim, k0, wave, i);
    }
};

// Fragment reader for a staged tile (any wave count): same LDS image and swizzles as TileLoader.
template <int ROWS, bool TRANS, int SW = 0>
using FragReader = TileLoader<ROWS, TRANS, SW>;

}  // namespace ergm
