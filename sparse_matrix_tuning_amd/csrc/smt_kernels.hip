// smt_kernels.hip — gfx950 (MI355X, CDNA4) kernels of the SMT block-sparse fine-tuning hot path
// and the extern "C" ABI declared in include/smt_hip.h.
//
// Kernels (reference lines they restate, relative to yudaohai666/Sparse_Matrix_Tuning):
//   wgrad_partial / wgrad_reduce   deepspeed/smt/smt.py:382-404  per-tile weight gradient, bf16 MFMA
//   tile_copy<GATHER/SCATTER>      deepspeed/smt/smt.py:317-325 / 332-341
//   grad_accumulate                deepspeed/fine_tune.py:724-741, 751-764
//   block_score                    deepspeed/smt/smt_helper.py:67-78, 233-251
//   sq_norm_partial / final        DeepSpeed gradient_clipping (deepspeed_helpers.py:87), external
//   adamw_fused                    DeepSpeed FusedAdam (adam_w_mode) step, external, + W scatter
//
// Layout conventions: a "tile" is one 256x256 block; a tile buffer is [n_tiles*256, 256] row-major
// (tile i occupies rows i*256..i*256+255, exactly the selected_weight layout of smt.py:312-325).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>

#include "smt_hip.h"
#include "fp8_math.h"

namespace {

constexpr int kTile = SMT_BLOCK_DIM;          // 256
constexpr int kTileElems = kTile * kTile;     // 65536

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(SMT_E_LAUNCH, "%s: %s", what, hipGetErrorString(e));
    return SMT_OK;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

__device__ __forceinline__ float bf16_bits_to_f32(uint32_t b) { return __uint_as_float(b << 16); }

// Round-to-nearest-even f32 -> bf16 through the compiler's cast (v_cvt_pk_bf16_f32 on gfx950,
// NaN-preserving; MI355X_MICROARCH.md "Correctness boundaries").
__device__ __forceinline__ uint16_t f32_to_bf16_bits(float f) {
    __bf16 b = (__bf16)f;
    return __builtin_bit_cast(uint16_t, b);
}

__device__ __forceinline__ float half_bits_to_f32(uint16_t h) {
    return (float)__builtin_bit_cast(_Float16, h);
}

// Operand formats of the tile wgrad. The reference runs linearZ in the model's dtype
// (fine_tune.py:955-959 --dtype bf16 | fp16 | fp32; deepspeed_helpers.py:53-61), so the per-sample
// partials are rounded to that dtype (smt.py:397-404). FMT 0 = bf16, 1 = fp16 (the same 16-bit
// staging, transposed reads and slabs; only the MFMA and the roundings differ), 2 = fp32 operands
// (wgrad_f32_kernel; "rounding" a partial to fp32 is the identity).
constexpr int kFmtBF16 = 0, kFmtF16 = 1, kFmtF32 = 2;

__device__ __forceinline__ uint16_t f32_to_half_bits(float f) {
    const _Float16 h = (_Float16)f;                        // round to nearest even, overflow to inf
    return __builtin_bit_cast(uint16_t, h);
}

template <int FMT>
__device__ __forceinline__ uint16_t to16(float f) { return FMT == kFmtF16 ? f32_to_half_bits(f) : f32_to_bf16_bits(f); }

template <int FMT>
__device__ __forceinline__ float from16(uint32_t b) {
    return FMT == kFmtF16 ? half_bits_to_f32((uint16_t)b) : bf16_bits_to_f32(b);
}

// a partial rounded to the operand dtype (fp32 operands: unchanged)
template <int FMT>
__device__ __forceinline__ float round_op(float v) { return FMT == kFmtF32 ? v : from16<FMT>(to16<FMT>(v)); }

// ------------------------------------------------------------------------------------------------
// Per-tile weight gradient (smt.py:397-404):
//   C[m][n] = sum_t g[t][r*256+m] * x[t][c*256+n],  m,n in [0,256)
// One 512-thread workgroup (8 waves as 2(M) x 4(N), 128x64 outputs per wave, 8 accumulators of
// v_mfma_f32_32x32x16_bf16) owns a whole 256x256 tile for one contiguous chunk of T rows and
// writes its fp32 partial to a slab; wgrad_reduce sums the slabs in a fixed order.
// Both operands arrive K-major ([t][feature] rows of 512 B), so the LDS images are [k][256] and
// every MFMA fragment is fetched by ds_read_b64_tr_b16 (transposed read, cdna_hip_programming T10).
// Image swizzle: byte (k, b) -> k*512 + (b ^ ((k&3)<<6)). A 32-lane half of a tr read covers rows
// k0..k0+3 x one aligned 64-B column chunk, which the XOR spreads over the four 64-B quarters of the
// 256-B bank row: conflict-free. Staged through registers (global_load_dwordx4 -> ds_write_b128,
// issue-early / write-late, T14) with one barrier per 64-row stage and two LDS buffers.
// ------------------------------------------------------------------------------------------------
constexpr int kWgThreads = 512;
constexpr int kBK = 64;                        // T rows per stage
constexpr int kRowBytes = kTile * 2;           // 512
constexpr int kImgBytes = kBK * kRowBytes;     // 32 KiB per operand per stage
constexpr int kChunksPerThread = (kImgBytes / 16) / kWgThreads;   // 4 x 16 B per operand
static_assert(kChunksPerThread == 4, "staging geometry");

__device__ __forceinline__ uint32_t img_off(uint32_t k, uint32_t byte_in_row) {
    return k * kRowBytes + (byte_in_row ^ ((k & 3u) << 6));
}

typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));

// one 32x32x16 MFMA on 16-bit fragments in operand format FMT (the fragments are raw 16-bit lanes)
template <int FMT>
__device__ __forceinline__ f32x16_t mfma16(const bf16x8_t& a, const bf16x8_t& b, const f32x16_t& c) {
    if constexpr (FMT == kFmtF16)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b),
                                                      c, 0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8_t tr_frag(const uint8_t* img, uint32_t k, uint32_t byte_in_row) {
    s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(img + img_off(k, byte_in_row)));
    s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(img + img_off(k + 4, byte_in_row)));
    // whole-vector bit casts: element-wise __bf16 bit_casts of vector lanes miscompile (all lanes
    // came back equal to element 0 on ROCm 7.2 / gfx950)
    const s16x8_t both = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8_t, both);
}

// Epilogue modes: partial slab (S > 1), or the final tile written directly (S == 1). kOutSlabBF16:
// the reference rounding's per-sample partial when one workgroup computes a whole sample (kps == 1):
// rounded to bf16 in the epilogue, as smt.py:397-404 rounds it, so its slab takes half the bytes.
enum WgradOut { kOutSlab = 0, kOutF32 = 1, kOutBF16 = 2, kOutSlabBF16 = 3 };

// Where a workgroup's accumulators go: the fp32 partial slab (tile, s) of a split tile (S > 1), or
// the final tile itself (S == 1; fp32 or bf16 per OUT).
template <int OUT>
__device__ __forceinline__ void* wgrad_dst(void* out_ptr, int tile, int s, int S) {
    if (OUT == kOutSlab) return static_cast<float*>(out_ptr) + (int64_t)(tile * S + s) * kTileElems;
    if (OUT == kOutSlabBF16) return static_cast<uint16_t*>(out_ptr) + (int64_t)(tile * S + s) * kTileElems;
    if (OUT == kOutF32) return static_cast<float*>(out_ptr) + (int64_t)tile * kTileElems;
    return static_cast<uint16_t*>(out_ptr) + (int64_t)tile * kTileElems;
}

// Epilogue of the wgrad kernels. They issue their MFMAs as x-slice x g-slice, so each accumulator
// holds C^T: acc[mb][nb][i] = C[m][n] with m = wm0 + mb*32 + (lane&31), n = wn0 + nb*32 +
// 8*(i>>2) + 4*(lane>>5) + (i&3), (wm0, wn0) = the wave's origin in the tile. Each lane then holds
// runs of 4 consecutive columns of one row, so the stores are 16-B (fp32) or 8-B (bf16) vectors
// instead of 16 scalar stores per accumulator -- the store tail is issue-bound (cdna_hip_programming
// T21). For the bf16 slab the two half-waves' 4-column runs are paired by v_permlane32_swap into
// 8-column rows: one 16-B store per lane per pair of runs.
template <int OUT, int MB, int FMT = kFmtBF16>
__device__ __forceinline__ void wgrad_store_t(f32x16_t (&acc)[MB][2], void* __restrict__ dst,
                                              int wm0, int wn0, int lane, int accumulate) {
    const int r = lane & 31;
    const int h = lane >> 5;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
            const int m = wm0 + mb * 32 + r;
            const int n0 = wn0 + nb * 32;
            const f32x16_t& a = acc[mb][nb];
            if (OUT == kOutSlabBF16) {
                uint16_t* row = static_cast<uint16_t*>(dst) + m * kTile + n0;
#pragma unroll
                for (int g = 0; g < 4; g += 2) {
                    uint32_t lo0 = to16<FMT>(a[4 * g]) | ((uint32_t)to16<FMT>(a[4 * g + 1]) << 16);
                    uint32_t lo1 = to16<FMT>(a[4 * g + 2]) | ((uint32_t)to16<FMT>(a[4 * g + 3]) << 16);
                    uint32_t hi0 = to16<FMT>(a[4 * g + 4]) | ((uint32_t)to16<FMT>(a[4 * g + 5]) << 16);
                    uint32_t hi1 = to16<FMT>(a[4 * g + 6]) | ((uint32_t)to16<FMT>(a[4 * g + 7]) << 16);
                    // vdst = run g, src = run g+1: lanes 0-31 end with columns 8g..8g+7 of their row,
                    // lanes 32-63 with columns 8(g+1)..8(g+1)+7
                    const auto s0 = __builtin_amdgcn_permlane32_swap(lo0, hi0, false, false);
                    const auto s1 = __builtin_amdgcn_permlane32_swap(lo1, hi1, false, false);
                    uint4 w;
                    w.x = s0[0]; w.y = s1[0]; w.z = s0[1]; w.w = s1[1];
                    *reinterpret_cast<uint4*>(row + 8 * (g + h)) = w;
                }
            } else if (OUT == kOutSlab || OUT == kOutF32) {
                float* row = static_cast<float*>(dst) + m * kTile + n0;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    float4* p = reinterpret_cast<float4*>(row + 8 * g + 4 * h);
                    float4 v = make_float4(a[4 * g], a[4 * g + 1], a[4 * g + 2], a[4 * g + 3]);
                    if (OUT == kOutF32 && accumulate) {
                        const float4 o = *p;
                        v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
                    }
                    *p = v;
                }
            } else {
                uint16_t* row = static_cast<uint16_t*>(dst) + m * kTile + n0;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    uint2* p = reinterpret_cast<uint2*>(row + 8 * g + 4 * h);
                    float v0 = a[4 * g], v1 = a[4 * g + 1], v2 = a[4 * g + 2], v3 = a[4 * g + 3];
                    if (accumulate) {
                        const uint2 o = *p;
                        v0 += from16<FMT>(o.x & 0xffffu); v1 += from16<FMT>(o.x >> 16);
                        v2 += from16<FMT>(o.y & 0xffffu); v3 += from16<FMT>(o.y >> 16);
                    }
                    uint2 w;
                    w.x = to16<FMT>(v0) | ((uint32_t)to16<FMT>(v1) << 16);
                    w.y = to16<FMT>(v2) | ((uint32_t)to16<FMT>(v3) << 16);
                    *p = w;
                }
            }
        }
}

// One tile of a wgrad launch: its operand column slices and its output. A launch covers the tiles
// of one module (BATCH = false: int32 [n][2] table of (row_block, col_block), module m[0]) or of up
// to SMT_WGRAD_MAX_MODULES modules that share T (BATCH = true: int32 [n][4] table of (module,
// row_block, col_block, tile index in that module's output)). Everything here is workgroup-uniform.
struct WgradModules { smt_wgrad_module m[SMT_WGRAD_MAX_MODULES]; };
struct WgradMxModules { smt_wgrad_mx_module m[SMT_WGRAD_MAX_MODULES]; };   // the MX-fp8 kernels

struct WgradTile {
    const uint16_t* g;       // grad_out column slice r: element (t, j) at g[t * ldg + j]
    const uint16_t* x;       // input column block c: element (t, j) at x[t * ldx + j]
    int64_t ldg, ldx;
    void* out;               // the final tile (S == 1 epilogue and the reduce)
    int accumulate;
};

template <bool BATCH, int OUT_BYTES>
__device__ __forceinline__ WgradTile wgrad_tile(const WgradModules& mods, const int32_t* __restrict__ tab, int tile) {
    WgradTile t;
    int mi = 0, r, c, ti;
    if (BATCH) {
        mi = tab[4 * tile]; r = tab[4 * tile + 1]; c = tab[4 * tile + 2]; ti = tab[4 * tile + 3];
    } else {
        r = tab[2 * tile]; c = tab[2 * tile + 1]; ti = tile;
    }
    const smt_wgrad_module& m = mods.m[mi];
    t.ldg = m.ld_grad_out;
    t.ldx = m.ld_x;
    t.g = static_cast<const uint16_t*>(m.grad_out) + (int64_t)r * kTile;
    t.x = static_cast<const uint16_t*>(m.x) + (int64_t)c * m.x_block_stride;
    t.out = static_cast<uint8_t*>(m.grad_tiles) + (int64_t)ti * kTileElems * OUT_BYTES;
    t.accumulate = m.accumulate;
    return t;
}

// Rows [t_begin, t_end) of split s. Default (seq == 0): contiguous chunks of T. Reference rounding
// (seq > 0, smt.py:397-404 rounds every per-sample [256, 256] partial to bf16): split s = sample *
// kps + j covers piece j (chunk rows) of one seq-row sample, so no split crosses a sample boundary
// and the reduce can rebuild each sample's partial before rounding it.
__device__ __forceinline__ void wgrad_span(int s, int64_t T, int64_t chunk, int64_t seq, int kps,
                                           int64_t& t_begin, int64_t& t_end) {
    if (seq > 0) {
        const int smp = s / kps, j = s - smp * kps;
        const int64_t lim = (int64_t)(smp + 1) * seq;
        t_begin = (int64_t)smp * seq + (int64_t)j * chunk;
        t_end = (t_begin + chunk < lim) ? (t_begin + chunk) : lim;
    } else {
        t_begin = (int64_t)s * chunk;
        t_end = (t_begin + chunk < T) ? (t_begin + chunk) : T;
    }
}

template <int OUT, bool BATCH, int FMT = kFmtBF16>
__global__ __launch_bounds__(kWgThreads, 2)
void wgrad_partial_kernel(const WgradModules mods, int64_t T, int64_t chunk, int S, int64_t seq, int kps, int n_tiles,
                          const int32_t* __restrict__ tile_tab, const int32_t* __restrict__ order,
                          float* __restrict__ slab) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * 2 * kImgBytes];   // 128 KiB, one array

    // XCD-aware, chunk-major schedule. Workgroups are dealt round-robin over the 8 XCDs (b and b+8
    // share one); the bijective remap (cdna_hip_programming T1) gives each XCD a CONTIGUOUS run of
    // logical ids L = s*n_tiles + i: the tiles of (about) one T-chunk, in `order` (the host sorts
    // tiles so that those sharing an x column-block / g row-block are adjacent). Tiles running on
    // one XCD therefore stream the same rows at the same time and re-read shared slices from that
    // XCD's L2 instead of HBM. Placement only changes speed, never results.
    const int total = n_tiles * S;
    const int b = blockIdx.x;
    const int q8 = total >> 3, r8 = total & 7, xcd = b & 7;
    const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    const int s = L / n_tiles;
    const int li = L - s * n_tiles;
    const int tile = order != nullptr ? order[li] : li;
    const WgradTile tt = wgrad_tile<BATCH, OUT == kOutBF16 ? 2 : 4>(mods, tile_tab, tile);
    int64_t t_begin, t_end;
    wgrad_span(s, T, chunk, seq, kps, t_begin, t_end);
    const int nst = (t_end > t_begin) ? (int)((t_end - t_begin + kBK - 1) / kBK) : 0;

    const uint16_t* gb = tt.g;
    const uint16_t* xb = tt.x;
    const int64_t ldg = tt.ldg, ldx = tt.ldx;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave >> 2;          // 0..1 -> rows wm*128
    const int wn = wave & 3;           // 0..3 -> cols wn*64

    uint4 ra[kChunksPerThread], rb[kChunksPerThread];

    auto gload = [&](int st) {
        const int64_t t0 = t_begin + (int64_t)st * kBK;
        if (t0 + kBK <= t_end) {
#pragma unroll
            for (int i = 0; i < kChunksPerThread; ++i) {
                const int cid = tid + kWgThreads * i;
                const int64_t t = t0 + (cid >> 5);
                const int e = (cid & 31) * 8;
                ra[i] = *reinterpret_cast<const uint4*>(gb + t * ldg + e);
                rb[i] = *reinterpret_cast<const uint4*>(xb + t * ldx + e);
            }
        } else {
#pragma unroll
            for (int i = 0; i < kChunksPerThread; ++i) {
                const int cid = tid + kWgThreads * i;
                const int64_t t = t0 + (cid >> 5);
                const int e = (cid & 31) * 8;
                if (t < t_end) {
                    ra[i] = *reinterpret_cast<const uint4*>(gb + t * ldg + e);
                    rb[i] = *reinterpret_cast<const uint4*>(xb + t * ldx + e);
                } else {
                    ra[i] = make_uint4(0, 0, 0, 0);
                    rb[i] = make_uint4(0, 0, 0, 0);
                }
            }
        }
    };
    auto swrite = [&](int buf) {
        uint8_t* A = lds + buf * 2 * kImgBytes;
        uint8_t* B = A + kImgBytes;
#pragma unroll
        for (int i = 0; i < kChunksPerThread; ++i) {
            const int cid = tid + kWgThreads * i;
            const uint32_t off = img_off((uint32_t)(cid >> 5), (uint32_t)(cid & 31) * 16u);
            *reinterpret_cast<uint4*>(A + off) = ra[i];
            *reinterpret_cast<uint4*>(B + off) = rb[i];
        }
    };

    f32x16_t acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    // tr-read lane geometry: group gi = lane>>4 covers feature offset 16*(gi&1) and k offset
    // 8*(gi>>1); lane 4q+p of the group supplies row q, features 4p..4p+3 (T10).
    const int gi = lane >> 4;
    const int q = (lane >> 2) & 3;
    const int p = lane & 3;
    const uint32_t feat_byte = 2u * (16u * (gi & 1) + 4u * p);
    const uint32_t krow = 8u * (gi >> 1) + q;

    if (nst > 0) {
        gload(0);
        swrite(0);
    }
    __syncthreads();

    for (int st = 0; st < nst; ++st) {
        const int buf = st & 1;
        if (st + 1 < nst) gload(st + 1);
        const uint8_t* A = lds + buf * 2 * kImgBytes;
        const uint8_t* B = A + kImgBytes;
#pragma unroll
        for (int ks = 0; ks < kBK / 16; ++ks) {
            bf16x8_t af[4], bfr[2];
#pragma unroll
            for (int mb = 0; mb < 4; ++mb)
                af[mb] = tr_frag(A, ks * 16 + krow, 2u * (wm * 128 + mb * 32) + feat_byte);
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
                bfr[nb] = tr_frag(B, ks * 16 + krow, 2u * (wn * 64 + nb * 32) + feat_byte);
#pragma unroll
            for (int mb = 0; mb < 4; ++mb)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb)
                    acc[mb][nb] = mfma16<FMT>(bfr[nb], af[mb], acc[mb][nb]);
        }
        if (st + 1 < nst) swrite(buf ^ 1);
        __syncthreads();
    }

    wgrad_store_t<OUT, 4, FMT>(acc, (OUT == kOutSlab || OUT == kOutSlabBF16) ? wgrad_dst<OUT>(slab, tile, s, S) : tt.out,
                          wm * 128, wn * 64, lane, tt.accumulate);
}

// ------------------------------------------------------------------------------------------------
// LDS-DMA variant of the same tile GEMM (default). Operands go HBM -> LDS with
// buffer_load_dwordx4 ... lds (no VGPR staging), 32-row stages in a 4-slot LDS ring with TWO stages
// in flight while one is computed (counted s_waitcnt vmcnt + raw s_barrier: cdna_hip_programming
// §5 "Pipelining across barriers"). The register-staged kernel above keeps only one 64 KiB stage in
// flight per CU, which measured as latency-bound at ~25 GB/s per CU.
// The LDS image stays lane-linear per DMA instruction (1 KiB = two 512-B rows); the XOR swizzle of
// the image is applied to each lane's SOURCE address instead (rule 21), so the transposed reads are
// unchanged. Rows past the chunk end read as zeros through the buffer descriptor's range check.
// ------------------------------------------------------------------------------------------------
constexpr int kDmaBK = 32;                                 // rows per stage
constexpr int kDmaImg = kDmaBK * kRowBytes;                // 16 KiB per operand per stage
constexpr int kDmaSlotBytes = 2 * kDmaImg;                 // A + B
// ring slots: (SLOTS - 2) stages in flight + 1 computing + 1 WAR margin. 4 slots (128 KiB, 2 stages
// in flight) is the default: 5 slots (160 KiB, the whole LDS of a gfx950 CU, 3 in flight) measured
// 1-10 % SLOWER at 4-436 tiles, T = 32768 (profiles/r02_wgrad_ring_depth.jsonl): the kernel is not
// bound by the bytes in flight per CU.
constexpr int kDmaSlotsDefault = 4;
// Measured, not kept (profiles/r03_wgrad_stagger_ab.jsonl, scripts/ab_wgrad_batch.sh on bench-shaped
// batches): waves 4-7 one k-step behind their SIMD partners (MI355X_MICROARCH "Two waves per SIMD",
// item 9), with and without s_setprio 1 on the lagging half: 1-3 % slower, bit-identical tiles.

// s_waitcnt vmcnt(n) for a run-time n in {0, 4, 8, 12} (the immediate must be a constant)
__device__ __forceinline__ void wait_vm_stages(int stages_in_flight) {
    switch (stages_in_flight) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    }
}

typedef __attribute__((address_space(3))) uint8_t lds_u8_t;

// One 1 KiB LDS-DMA: lane l's 16 B from rsrc+voff land at LDS byte lds_base + 16*l. Inline asm on
// purpose: hipcc then does not see an LDS write it cannot disambiguate from the ring slot being read
// (with the builtin it puts s_waitcnt vmcnt(0) before every ds_read, draining the 2-deep pipeline);
// completion is tracked by the hand-counted vmcnt in the loop. M0 is saved / restored inside the
// statement (cdna_hip_programming §5.7). Default cache policy: the non-temporal one measured the same
// on the bench's batched launches (profiles/r02_wgrad_nt_ab.jsonl).
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, uint32_t lds_base, int voff) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(lds_base) : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const uint8_t* p) {
    return (uint32_t)(uintptr_t)(const lds_u8_t*)p;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base, int64_t bytes) {
    // every descriptor input made provably wave-uniform (T20): no waterfall loops
    const uint64_t a = (uint64_t)(uintptr_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const int n = __builtin_amdgcn_readfirstlane((int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}

template <int OUT, int SLOTS, bool BATCH, int FMT = kFmtBF16>
__global__ __launch_bounds__(kWgThreads, 1)
void wgrad_dma_kernel(const WgradModules mods, int64_t T, int64_t chunk, int S, int64_t seq, int kps, int n_tiles,
                      const int32_t* __restrict__ tile_tab, const int32_t* __restrict__ order,
                      float* __restrict__ slab) {
    static_assert(SLOTS >= 3 && SLOTS <= 5, "ring depth");
    constexpr int AHEAD = SLOTS - 2;                       // stages in flight beside the one computed
    __shared__ __attribute__((aligned(16))) uint8_t lds[SLOTS * kDmaSlotBytes];   // one array (T-trap 4a)

    const int total = n_tiles * S;
    const int b = blockIdx.x;
    const int q8 = total >> 3, r8 = total & 7, xcd = b & 7;
    const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    const int s = L / n_tiles;
    const int li = L - s * n_tiles;
    const int tile = order != nullptr ? order[li] : li;
    const WgradTile tt = wgrad_tile<BATCH, OUT == kOutBF16 ? 2 : 4>(mods, tile_tab, tile);
    const int64_t ldg = tt.ldg, ldx = tt.ldx;
    int64_t t_begin, t_end;
    wgrad_span(s, T, chunk, seq, kps, t_begin, t_end);
    const int rows = (t_end > t_begin) ? (int)(t_end - t_begin) : 0;
    const int nst = (rows + kDmaBK - 1) / kDmaBK;

    // descriptors over this chunk's rows of the two column slices (host guarantees rows*ld*2 < 2^31)
    const __amdgpu_buffer_rsrc_t rg = uniform_rsrc(tt.g + t_begin * ldg, (int64_t)rows * ldg * 2);
    const __amdgpu_buffer_rsrc_t rx = uniform_rsrc(tt.x + t_begin * ldx, (int64_t)rows * ldx * 2);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2;
    const int wn = wave & 3;

    // DMA geometry: wave w fills image rows 4w .. 4w+3 of each operand (two 1 KiB instructions);
    // lane l of instruction j lands at image row k = 4w + 2j + (l>>5), physical byte 16*(l&31),
    // which holds logical byte (16*(l&31)) ^ ((k&3) << 6) of that row.
    int voff_g[2], voff_x[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int k = 4 * wave + 2 * j + (lane >> 5);
        const int lb = (16 * (lane & 31)) ^ ((k & 3) << 6);
        voff_g[j] = (int)(k * ldg * 2) + lb;
        voff_x[j] = (int)(k * ldx * 2) + lb;
    }
    const int step_g = (int)(kDmaBK * ldg * 2), step_x = (int)(kDmaBK * ldx * 2);

    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(lds));
    auto issue = [&](int st) {
        const uint32_t slot = lds0 + (uint32_t)((st % SLOTS) * kDmaSlotBytes);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t row0 = (uint32_t)(4 * wave + 2 * j) * kRowBytes;
            dma16(rg, __builtin_amdgcn_readfirstlane(slot + row0), voff_g[j] + st * step_g);
            dma16(rx, __builtin_amdgcn_readfirstlane(slot + kDmaImg + row0), voff_x[j] + st * step_x);
        }
    };

    f32x16_t acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    const int gi = lane >> 4;
    const int q = (lane >> 2) & 3;
    const int p = lane & 3;
    const uint32_t feat_byte = 2u * (16u * (gi & 1) + 4u * p);
    const uint32_t krow = 8u * (gi >> 1) + q;

#pragma unroll
    for (int i = 0; i < AHEAD; ++i)
        if (i < nst) issue(i);
    for (int st = 0; st < nst; ++st) {
        // 4 DMA instructions per wave per stage: stage st has landed once at most 4 * (stages issued
        // after it) are outstanding
        if (st + AHEAD < nst) {
            issue(st + AHEAD);
            wait_vm_stages(AHEAD);
        } else {
            wait_vm_stages(nst - 1 - st);
        }
        __builtin_amdgcn_s_barrier();                              // every wave's DMA for stage st landed
        __builtin_amdgcn_sched_barrier(0);
        const uint8_t* A = lds + (st % SLOTS) * kDmaSlotBytes;
        const uint8_t* B = A + kDmaImg;
#pragma unroll
        for (int ks = 0; ks < kDmaBK / 16; ++ks) {
            bf16x8_t af[4], bfr[2];
#pragma unroll
            for (int mb = 0; mb < 4; ++mb)
                af[mb] = tr_frag(A, ks * 16 + krow, 2u * (wm * 128 + mb * 32) + feat_byte);
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
                bfr[nb] = tr_frag(B, ks * 16 + krow, 2u * (wn * 64 + nb * 32) + feat_byte);
            // x slice as A, g slice as B: the accumulators hold C^T, whose per-lane runs of 4
            // consecutive columns give wgrad_store_t its vector stores
#pragma unroll
            for (int mb = 0; mb < 4; ++mb)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb)
                    acc[mb][nb] = mfma16<FMT>(bfr[nb], af[mb], acc[mb][nb]);
        }
    }
    wgrad_store_t<OUT, 4, FMT>(acc, (OUT == kOutSlab || OUT == kOutSlabBF16) ? wgrad_dst<OUT>(slab, tile, s, S) : tt.out,
                          wm * 128, wn * 64, lane, tt.accumulate);
}

// ------------------------------------------------------------------------------------------------
// Quarter-tile variant for modules with few tiles (the HBM-bound regime: no two tiles share an
// operand slice). A 256-thread workgroup owns one 128x128 quarter of a tile for one chunk of T rows
// (4 waves as 2x2, 64x64 outputs each = 2x2 accumulators of v_mfma_f32_32x32x16_bf16), so a tile
// splits 4 ways over its OUTPUT before it splits over T: 4x fewer split-K slabs for the same number
// of workgroups, and two workgroups fit per CU (64 KiB LDS each: a 4-slot ring of 32-row stages of
// two 32 x 128 bf16 half-slices). The four quarters of a (tile, chunk) are consecutive logical ids,
// so they run on one XCD at the same time and each half-slice is read from HBM once and from L2 by
// the quarter beside it. Same LDS-DMA / transposed-read machinery and swizzle as wgrad_dma_kernel;
// slabs use the same [tile][S][256][256] layout, so wgrad_reduce_kernel is shared.
// ------------------------------------------------------------------------------------------------
constexpr int kQThreads = 256;
constexpr int kQRowBytes = 128 * 2;                         // 256 B: one half-slice row
constexpr int kQImg = kDmaBK * kQRowBytes;                  // 8 KiB per operand per stage
constexpr int kQSlotBytes = 2 * kQImg;
constexpr int kQSlots = 4;

__device__ __forceinline__ uint32_t qimg_off(uint32_t k, uint32_t byte_in_row) {
    return k * kQRowBytes + (byte_in_row ^ ((k & 3u) << 6));
}

__device__ __forceinline__ bf16x8_t qtr_frag(const uint8_t* img, uint32_t k, uint32_t byte_in_row) {
    s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(img + qimg_off(k, byte_in_row)));
    s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(img + qimg_off(k + 4, byte_in_row)));
    const s16x8_t both = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8_t, both);
}

template <int OUT, int QS, bool BATCH, int FMT = kFmtBF16>
__global__ __launch_bounds__(kQThreads, 2)
void wgrad_quarter_kernel(const WgradModules mods, int64_t T, int64_t chunk, int S, int64_t seq, int kps, int n_tiles,
                          const int32_t* __restrict__ tile_tab, const int32_t* __restrict__ order,
                          float* __restrict__ slab) {
    static_assert(QS >= 3 && QS <= 5, "ring depth");
    constexpr int AHEAD = QS - 2;                          // stages in flight beside the one computed
    __shared__ __attribute__((aligned(16))) uint8_t lds[QS * kQSlotBytes];          // 64 KiB (4 slots), one array

    // logical id L = (s * n_tiles + i) * 4 + quarter, dealt XCD-contiguously (bijective remap)
    const int total = n_tiles * S * 4;
    const int b = blockIdx.x;
    const int q8 = total >> 3, r8 = total & 7, xcd = b & 7;
    const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    const int qd = L & 3;
    const int ts = L >> 2;
    const int s = ts / n_tiles;
    const int li = ts - s * n_tiles;
    const int tile = order != nullptr ? order[li] : li;
    const int qm = qd >> 1, qn = qd & 1;
    const WgradTile tt = wgrad_tile<BATCH, OUT == kOutBF16 ? 2 : 4>(mods, tile_tab, tile);
    const int64_t ldg = tt.ldg, ldx = tt.ldx;
    int64_t t_begin, t_end;
    wgrad_span(s, T, chunk, seq, kps, t_begin, t_end);
    const int rows = (t_end > t_begin) ? (int)(t_end - t_begin) : 0;
    const int nst = (rows + kDmaBK - 1) / kDmaBK;

    const __amdgpu_buffer_rsrc_t rg = uniform_rsrc(tt.g + t_begin * ldg + qm * 128, (int64_t)rows * ldg * 2);
    const __amdgpu_buffer_rsrc_t rx = uniform_rsrc(tt.x + t_begin * ldx + qn * 128, (int64_t)rows * ldx * 2);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1;
    const int wn = wave & 1;

    // DMA geometry: wave w fills image rows 8w .. 8w+7 of each operand (two 1 KiB instructions of
    // 4 rows x 256 B); lane l of instruction j lands at row k = 8w + 4j + (l>>4), physical byte
    // 16*(l&15), which holds logical byte (16*(l&15)) ^ ((k&3) << 6) of that row.
    int voff_g[2], voff_x[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int k = 8 * wave + 4 * j + (lane >> 4);
        const int lb = (16 * (lane & 15)) ^ ((k & 3) << 6);
        voff_g[j] = (int)(k * ldg * 2) + lb;
        voff_x[j] = (int)(k * ldx * 2) + lb;
    }
    const int step_g = (int)(kDmaBK * ldg * 2), step_x = (int)(kDmaBK * ldx * 2);

    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(lds));
    auto issue = [&](int st) {
        const uint32_t slot = lds0 + (uint32_t)((st % QS) * kQSlotBytes);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t row0 = (uint32_t)(8 * wave + 4 * j) * kQRowBytes;
            dma16(rg, __builtin_amdgcn_readfirstlane(slot + row0), voff_g[j] + st * step_g);
            dma16(rx, __builtin_amdgcn_readfirstlane(slot + kQImg + row0), voff_x[j] + st * step_x);
        }
    };

    f32x16_t acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    const int gi = lane >> 4;
    const int q = (lane >> 2) & 3;
    const int p = lane & 3;
    const uint32_t feat_byte = 2u * (16u * (gi & 1) + 4u * p);
    const uint32_t krow = 8u * (gi >> 1) + q;

#pragma unroll
    for (int i = 0; i < AHEAD; ++i)
        if (i < nst) issue(i);
    for (int st = 0; st < nst; ++st) {
        // 4 DMA instructions per wave per stage (as wgrad_dma_kernel)
        if (st + AHEAD < nst) {
            issue(st + AHEAD);
            wait_vm_stages(AHEAD);
        } else {
            wait_vm_stages(nst - 1 - st);
        }
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        const uint8_t* A = lds + (st % QS) * kQSlotBytes;
        const uint8_t* B = A + kQImg;
#pragma unroll
        for (int ks = 0; ks < kDmaBK / 16; ++ks) {
            bf16x8_t af[2], bfr[2];
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
                af[mb] = qtr_frag(A, ks * 16 + krow, 2u * (wm * 64 + mb * 32) + feat_byte);
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
                bfr[nb] = qtr_frag(B, ks * 16 + krow, 2u * (wn * 64 + nb * 32) + feat_byte);
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb)
                    acc[mb][nb] = mfma16<FMT>(bfr[nb], af[mb], acc[mb][nb]);
        }
    }
    wgrad_store_t<OUT, 2, FMT>(acc, (OUT == kOutSlab || OUT == kOutSlabBF16) ? wgrad_dst<OUT>(slab, tile, s, S) : tt.out,
                          qm * 128 + wm * 64, qn * 128 + wn * 64, lane, tt.accumulate);
}

// ------------------------------------------------------------------------------------------------
// fp32 operands (the reference's --dtype fp32, fine_tune.py:955-959): exact f32 products on
// v_mfma_f32_32x32x2_f32 (1/16 of the bf16 rate, cdna_hip_programming "FP32-input MFMA"). A workgroup
// of 4 waves owns one 128x128 quarter of a tile for one split of T, as wgrad_quarter_kernel (same
// XCD-contiguous logical ids, slabs and reduce); each wave 64x64 = 2x2 accumulators. The operand
// lane maps of the f32 form (A[i = l&31][k = l>>5], B[k = l>>5][j = l&31]) are rows of the K-major
// slices themselves: lanes 0-31 read 32 consecutive floats of row t, lanes 32-63 of row t+1, so the
// fragments come straight from global memory (128-B coalesced pieces, L1/L2-shared by the waves and
// quarters that read the same slice) with no LDS image and no transpose. x is A and g is B, so the
// accumulators hold C^T as in the 16-bit kernels and wgrad_store_t is shared. kUnroll row pairs are
// loaded ahead of the MFMAs that consume them.
// ------------------------------------------------------------------------------------------------
constexpr int kF32Threads = 256;
constexpr int kF32Unroll = 8;                              // row pairs (K = 2 each) per loaded batch

template <int OUT, bool BATCH>
__global__ __launch_bounds__(kF32Threads, 2)
void wgrad_f32_kernel(const WgradModules mods, int64_t T, int64_t chunk, int S, int64_t seq, int kps, int n_tiles,
                      const int32_t* __restrict__ tile_tab, const int32_t* __restrict__ order,
                      float* __restrict__ slab) {
    const int total = n_tiles * S * 4;
    const int b = blockIdx.x;
    const int q8 = total >> 3, r8 = total & 7, xcd = b & 7;
    const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    const int qd = L & 3;
    const int ts = L >> 2;
    const int s = ts / n_tiles;
    const int li = ts - s * n_tiles;
    const int tile = order != nullptr ? order[li] : li;
    const int qm = qd >> 1, qn = qd & 1;
    int mi = 0, r, c, ti;
    if (BATCH) {
        mi = tile_tab[4 * tile]; r = tile_tab[4 * tile + 1]; c = tile_tab[4 * tile + 2]; ti = tile_tab[4 * tile + 3];
    } else {
        r = tile_tab[2 * tile]; c = tile_tab[2 * tile + 1]; ti = tile;
    }
    const smt_wgrad_module& m = mods.m[mi];
    const int64_t ldg = m.ld_grad_out, ldx = m.ld_x;
    const float* gb = static_cast<const float*>(m.grad_out) + (int64_t)r * kTile;
    const float* xb = static_cast<const float*>(m.x) + (int64_t)c * m.x_block_stride;
    int64_t t_begin, t_end;
    wgrad_span(s, T, chunk, seq, kps, t_begin, t_end);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int m0 = qm * 128 + (wave >> 1) * 64;            // the wave's origin in the tile (rows: g)
    const int n0 = qn * 128 + (wave & 1) * 64;             // (columns: x)
    const int kr = lane >> 5, cl = lane & 31;

    f32x16_t acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    typedef float Frags[kF32Unroll][2];
    auto load = [&](Frags& ga, Frags& xa, int64_t t0) {    // kF32Unroll row pairs from row t0 on
        // buffer loads over this batch's rows: 32-bit lane offsets, and the descriptor's range check
        // reads the rows past the split's end as zeros (no per-load branch); the second 32-column
        // half of a fragment is the same address + 128 B
        const int64_t nrows = (t_end - t0 < 2 * kF32Unroll) ? (t_end - t0) : 2 * kF32Unroll;
        const __amdgpu_buffer_rsrc_t rg = uniform_rsrc(gb + t0 * ldg, nrows * ldg * 4);
        const __amdgpu_buffer_rsrc_t rx = uniform_rsrc(xb + t0 * ldx, nrows * ldx * 4);
        int og = (int)((kr * ldg + m0 + cl) * 4), ox = (int)((kr * ldx + n0 + cl) * 4);
        const int sg = (int)(2 * ldg * 4), sx = (int)(2 * ldx * 4);
#pragma unroll
        for (int u = 0; u < kF32Unroll; ++u) {
            ga[u][0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rg, og, 0, 0));
            ga[u][1] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rg, og + 128, 0, 0));
            xa[u][0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, ox, 0, 0));
            xa[u][1] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, ox + 128, 0, 0));
            og += sg;
            ox += sx;
        }
    };
    auto compute = [&](const Frags& ga, const Frags& xa) {
#pragma unroll
        for (int u = 0; u < kF32Unroll; ++u)
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb)
                    acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[u][nb], ga[u][mb], acc[mb][nb], 0, 0, 0);
    };
    // two register batches: the next batch's loads are in flight under the current batch's MFMAs
    constexpr int kStep = 2 * kF32Unroll;
    Frags g0, x0, g1, x1;
    if (t_begin < t_end) load(g0, x0, t_begin);
    for (int64_t t0 = t_begin; t0 < t_end; t0 += 2 * kStep) {
        const bool more1 = t0 + kStep < t_end;
        if (more1) load(g1, x1, t0 + kStep);
        compute(g0, x0);
        if (!more1) break;
        if (t0 + 2 * kStep < t_end) load(g0, x0, t0 + 2 * kStep);
        compute(g1, x1);
    }
    void* out = static_cast<uint8_t*>(m.grad_tiles) + (int64_t)ti * kTileElems * 4;
    wgrad_store_t<OUT, 2, kFmtF32>(acc, OUT == kOutSlab ? wgrad_dst<OUT>(slab, tile, s, S) : out, m0, n0, lane,
                                   m.accumulate);
}

// Sum the S partial slabs of one tile in order s = 0..S-1 (deterministic) and write the tile (this
// workgroup's 1024 of its elements). kps > 0 (reference rounding, wgrad_span): the slabs come in
// groups of kps per sample; each sample's partial (its kps slabs summed in fp32) is rounded to bf16,
// the samples are summed in order in fp32 and the sum is rounded to bf16 once more (smt.py:397-404:
// bf16 matmul per sample, then torch.sum(dim=0) of the bf16 partials, accumulated in fp32), before
// the optional accumulation into the output (autograd's add into .grad).
template <bool OUT_F32, bool SLAB16 = false, int FMT = kFmtBF16>
__device__ __forceinline__ void wgrad_reduce_tile(const float* __restrict__ slab, int S, int kps, int tile,
                                                  void* __restrict__ tile_out, int accumulate) {
    const int e = (((blockIdx.x & 63) << 8) + threadIdx.x) * 4;
    const float* src = slab + (int64_t)tile * S * kTileElems + e;
    float4 sum;
    if (SLAB16) {
        // kps == 1: every slab IS a sample's bf16-rounded partial (kOutSlabBF16); sum them in sample
        // order in fp32 and round once more (the same arithmetic as the fp32-slab branch below)
        const uint16_t* s16 = reinterpret_cast<const uint16_t*>(slab) + (int64_t)tile * S * kTileElems + e;
        sum = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
        for (int s = 0; s < S; ++s) {                      // unrolled: several slab loads in flight
            const uint2 v = *reinterpret_cast<const uint2*>(s16 + (int64_t)s * kTileElems);
            sum.x += from16<FMT>(v.x & 0xffffu); sum.y += from16<FMT>(v.x >> 16);
            sum.z += from16<FMT>(v.y & 0xffffu); sum.w += from16<FMT>(v.y >> 16);
        }
        sum.x = round_op<FMT>(sum.x); sum.y = round_op<FMT>(sum.y);
        sum.z = round_op<FMT>(sum.z); sum.w = round_op<FMT>(sum.w);
    } else if (kps <= 0) {
        sum = *reinterpret_cast<const float4*>(src);
#pragma unroll 4
        for (int s = 1; s < S; ++s) {
            const float4 v = *reinterpret_cast<const float4*>(src + (int64_t)s * kTileElems);
            sum.x += v.x; sum.y += v.y; sum.z += v.z; sum.w += v.w;
        }
    } else {
        sum = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
        for (int s0 = 0; s0 < S; s0 += kps) {
            float4 part = *reinterpret_cast<const float4*>(src + (int64_t)s0 * kTileElems);
            for (int j = 1; j < kps; ++j) {
                const float4 v = *reinterpret_cast<const float4*>(src + (int64_t)(s0 + j) * kTileElems);
                part.x += v.x; part.y += v.y; part.z += v.z; part.w += v.w;
            }
            sum.x += round_op<FMT>(part.x); sum.y += round_op<FMT>(part.y);
            sum.z += round_op<FMT>(part.z); sum.w += round_op<FMT>(part.w);
        }
        sum.x = round_op<FMT>(sum.x); sum.y = round_op<FMT>(sum.y);
        sum.z = round_op<FMT>(sum.z); sum.w = round_op<FMT>(sum.w);
    }
    const int64_t o = e;
    void* out = tile_out;
    if (OUT_F32) {
        float4* dst = reinterpret_cast<float4*>(static_cast<float*>(out) + o);
        if (accumulate) {
            const float4 a = *dst;
            sum.x += a.x; sum.y += a.y; sum.z += a.z; sum.w += a.w;
        }
        *dst = sum;
    } else {
        uint2* dst = reinterpret_cast<uint2*>(static_cast<uint16_t*>(out) + o);
        if (accumulate) {
            const uint2 a = *dst;
            sum.x += from16<FMT>(a.x & 0xffffu);
            sum.y += from16<FMT>(a.x >> 16);
            sum.z += from16<FMT>(a.y & 0xffffu);
            sum.w += from16<FMT>(a.y >> 16);
        }
        uint2 w;
        w.x = (uint32_t)to16<FMT>(sum.x) | ((uint32_t)to16<FMT>(sum.y) << 16);
        w.y = (uint32_t)to16<FMT>(sum.z) | ((uint32_t)to16<FMT>(sum.w) << 16);
        *dst = w;
    }
}

// 64 workgroups x 256 threads x 4 elements per tile; tile i's output = out + i tiles
template <bool OUT_F32, bool SLAB16 = false, int FMT = kFmtBF16>
__global__ __launch_bounds__(256)
void wgrad_reduce_kernel(const float* __restrict__ slab, int S, int kps, void* __restrict__ out, int accumulate) {
    const int tile = blockIdx.x >> 6;
    wgrad_reduce_tile<OUT_F32, SLAB16, FMT>(slab, S, kps, tile, static_cast<uint8_t*>(out) + (int64_t)tile * kTileElems * (OUT_F32 ? 4 : 2),
                               accumulate);
}

// the same over an MX batch
template <bool OUT_F32>
__global__ __launch_bounds__(256)
void wgrad_reduce_mx_batch_kernel(const float* __restrict__ slab, int S, const WgradMxModules mods,
                                  const int32_t* __restrict__ tile_tab) {
    const int tile = blockIdx.x >> 6;
    const int m = tile_tab[4 * tile];
    const int ti = tile_tab[4 * tile + 3];
    wgrad_reduce_tile<OUT_F32>(slab, S, 0, tile,
                               static_cast<uint8_t*>(mods.m[m].grad_tiles) + (int64_t)ti * kTileElems * (OUT_F32 ? 4 : 2),
                               mods.m[m].accumulate);
}

// the same over a batch: each tile's output and accumulate flag from its module (wgrad_tile)
template <bool OUT_F32, bool SLAB16 = false, int FMT = kFmtBF16>
__global__ __launch_bounds__(256)
void wgrad_reduce_batch_kernel(const float* __restrict__ slab, int S, int kps, const WgradModules mods,
                               const int32_t* __restrict__ tile_tab) {
    const int tile = blockIdx.x >> 6;
    const WgradTile tt = wgrad_tile<true, OUT_F32 ? 4 : 2>(mods, tile_tab, tile);
    wgrad_reduce_tile<OUT_F32, SLAB16, FMT>(slab, S, kps, tile, tt.out, tt.accumulate);
}

// ------------------------------------------------------------------------------------------------
// MX-fp8 tile weight gradient (BASELINE config 5, SURVEY §8(f) row 2: the reference has no fp8,
// fine_tune.py:955-959, so the bar is the bf16 tile path, not the reference).
//
// Operand format ("MX column blocks"), written by mx_quant_cols_kernel from a bf16 [T, C] matrix for
// a list of 256-column blocks, K-major so that no transpose is needed on the way to the MFMA:
//   q[blk][t/64][f][t%64]  e4m3 (OCP), f in [0,256), t in [0, ldq), rows T..ldq-1 zero; ldq % 64 == 0
//                     (K-major in 64-token panels: one stage of the wgrad is 16 KiB contiguous)
//   s[blk][t/32][f]   e8m0 shared exponent of the 32 values q[blk][f][32j .. 32j+31]
// value(t, f) = e4m3(q) * 2^(s - 127). The exponent is the smallest e with amax <= 448 * 2^e, so
// nothing saturates (amax = the 32 values' max |x|; e = -127 for an all-zero group; computed from
// the bits of amax, exact), and q = e4m3_rne(x * 2^-e) (a power-of-two multiply: exact).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int mx_exponent(float amax) {
    const uint32_t b = __float_as_uint(amax);
    const int ef = (int)((b >> 23) & 255u);
    if (ef == 0) return -127;                              // zero or fp32-subnormal amax
    const int e = ef - 127 - 8 + ((b & 0x7fffffu) > 0x600000u ? 1 : 0);   // 448 = 1.75 * 2^8
    return e < -127 ? -127 : e;
}

// One workgroup per (column block, ROWS rows of T). The [ROWS][256] bf16 slab is staged through
// LDS with coalesced 16-B row loads; LDS chunk ch of row r is stored at ch ^ (((r >> 4) & 3) << 2)
// so that the column reads below are conflict-free. Then LPF = ROWS/16 lanes share one column f:
// lane c quantises rows 16c .. 16c+15 of it (the 32-row group's amax is one shuffle with the
// neighbour lane) and the LPF lanes write the column's ROWS bytes of q[blk][f] as one contiguous
// run (ROWS = 128: whole 128-B lines).
__device__ __forceinline__ int mx_slab_off(int r, int f) {
    return r * kTile + ((((f >> 3) ^ (((r >> 4) & 3) << 2))) << 3) + (f & 7);
}

template <int ROWS>
__global__ __launch_bounds__(256)
void mx_quant_cols_kernel(const uint16_t* __restrict__ x, int64_t ldx, int64_t T, const int32_t* __restrict__ blocks,
                          int64_t ldq, uint8_t* __restrict__ q, uint8_t* __restrict__ sc) {
    constexpr int LPF = ROWS / 16;                          // lanes per column
    constexpr int FPP = 256 / LPF;                          // columns per pass
    __shared__ __attribute__((aligned(16))) uint16_t slab[ROWS * kTile];
    const int blk = blockIdx.x;
    const int64_t t0 = (int64_t)blockIdx.y * ROWS;
    const int tid = threadIdx.x;
    const uint16_t* src = x + (int64_t)blocks[blk] * kTile;
#pragma unroll
    for (int i = 0; i < ROWS * 32 / 256; ++i) {               // ROWS rows x 32 chunks of 16 B
        const int cid = tid + 256 * i;
        const int rr = cid >> 5, ch = cid & 31;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (t0 + rr < T) v = *reinterpret_cast<const uint4*>(src + (t0 + rr) * ldx + ch * 8);
        *reinterpret_cast<uint4*>(&slab[mx_slab_off(rr, ch * 8)]) = v;
    }
    __syncthreads();
    const int c = tid % LPF;                                 // 16-row run of the column
    const bool live = t0 + 16 * c < ldq;                     // the last workgroup may be half empty
#pragma unroll
    for (int pass = 0; pass < LPF; ++pass) {
        const int f = pass * FPP + tid / LPF;
        float v[16];
        float amax = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            v[k] = bf16_bits_to_f32(slab[mx_slab_off(16 * c + k, f)]);
            amax = fmaxf(amax, fabsf(v[k]));
        }
        amax = fmaxf(amax, __shfl_xor(amax, 1, 64));         // the other half of the 32-row group
        const int e = mx_exponent(amax);
        const float inv = __uint_as_float((uint32_t)(127 - e) << 23);     // 2^-e, e in [-127, 121]
        uint4 w;
        w.x = pack4(v[0] * inv, v[1] * inv, v[2] * inv, v[3] * inv);
        w.y = pack4(v[4] * inv, v[5] * inv, v[6] * inv, v[7] * inv);
        w.z = pack4(v[8] * inv, v[9] * inv, v[10] * inv, v[11] * inv);
        w.w = pack4(v[12] * inv, v[13] * inv, v[14] * inv, v[15] * inv);
        if (live) {
            const int64_t t = t0 + 16 * c;
            *reinterpret_cast<uint4*>(q + (((int64_t)blk * (ldq >> 6) + (t >> 6)) * kTile + f) * 64 + (t & 63)) = w;
            if ((c & 1) == 0) sc[((int64_t)blk * (ldq >> 5) + (t0 >> 5) + (c >> 1)) * kTile + f] = (uint8_t)(e + 127);
        }
    }
}

// The MX wgrad: C[m][n] = sum_t A(t, m) * B(t, n) over the MX column blocks of g (A, the tile's row
// block) and x (B, its column block), one 512-thread workgroup per (tile, T-chunk), 8 waves as
// 2(M) x 4(N) with 128x64 outputs each = 8 accumulators of v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 x
// e4m3, per-lane e8m0 scales): 2x the bf16 MFMA rate and half the operand bytes of the bf16 kernel.
// Lane l of a 32x32x64 operand holds row (l & 31) and two 16-token runs of it (see mx_frag): two
// ds_read_b128 from an LDS image of [256 rows][64 B] per 64-token stage, with chunk c of row f
// stored at chunk c ^ ((f >> 2) & 3) (16 lanes of a b128 read then cover all 64 banks once); the
// lane's scale is the exponent of (its row, k-block 2*stage + (l >> 5)).
// Stages stream through a 4-slot LDS-DMA ring (2 stages in flight, counted vmcnt, raw s_barrier)
// exactly as wgrad_dma_kernel; slabs / epilogue / reduce are shared with it.
constexpr int kMxBK = 64;                                   // tokens per stage = one MFMA K step
constexpr int kMxImg = kTile * kMxBK;                       // 16 KiB per operand per stage
constexpr int kMxSlotBytes = 2 * kMxImg + 2 * 2 * kTile;    // + 2 k-blocks x 256 exponents per operand
constexpr int kMxSlots = 4;

typedef int i32x8_t __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) uint4 lds_u4_t;

__device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t rsrc, uint32_t lds_base, int voff) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "buffer_load_dword %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(lds_base) : "memory");
}

// s_waitcnt vmcnt for a run-time count in {0, 4, 5, 8, 10}
__device__ __forceinline__ void wait_vm_n(int n) {
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    }
}

// Lane (row, h) of a 32x32x64 f8 operand: bytes 0-15 are k = 16h .. 16h+15, bytes 16-31 are
// k = 32 + 16h .. 32 + 16h + 15 (measured with one-hot operands: scripts/mx_probe.py), and its
// scale is the exponent of k-block h (k = 32h .. 32h+31). 16-B chunk c of a 64-token row holds
// tokens 16c .. 16c+15, so the lane reads chunks h and 2 + h.
__device__ __forceinline__ i32x8_t mx_frag(const uint8_t* img, int row, int h) {
    const int sw = (row >> 2) & 3;
    const uint4 lo = *reinterpret_cast<const uint4*>(img + row * kMxBK + ((h ^ sw) << 4));
    const uint4 hi = *reinterpret_cast<const uint4*>(img + row * kMxBK + (((2 + h) ^ sw) << 4));
    i32x8_t f;
    f[0] = (int)lo.x; f[1] = (int)lo.y; f[2] = (int)lo.z; f[3] = (int)lo.w;
    f[4] = (int)hi.x; f[5] = (int)hi.y; f[6] = (int)hi.z; f[7] = (int)hi.w;
    return f;
}

// One tile of an MX wgrad launch (one module, or a batch: as WgradTile). The operands are the
// module's MX row blocks of g (qa/sa, block r) and column blocks of x (qb/sb, block c).

struct WgradMxTile {
    const uint8_t *qa, *sa, *qb, *sb;    // this tile's blocks
    void* out;
    int accumulate;
};

template <bool BATCH, int OUT_BYTES>
__device__ __forceinline__ WgradMxTile wgrad_mx_tile(const WgradMxModules& mods, const int32_t* __restrict__ tab,
                                                     int tile, int64_t ldq) {
    int mi = 0, r, c, ti;
    if (BATCH) {
        mi = tab[4 * tile]; r = tab[4 * tile + 1]; c = tab[4 * tile + 2]; ti = tab[4 * tile + 3];
    } else {
        r = tab[2 * tile]; c = tab[2 * tile + 1]; ti = tile;
    }
    const smt_wgrad_mx_module& m = mods.m[mi];
    const int64_t blk_bytes = (int64_t)kTile * ldq, sc_bytes = (ldq >> 5) * kTile;
    WgradMxTile t;
    t.qa = static_cast<const uint8_t*>(m.qg) + r * blk_bytes;
    t.sa = static_cast<const uint8_t*>(m.sg) + r * sc_bytes;
    t.qb = static_cast<const uint8_t*>(m.qx) + c * blk_bytes;
    t.sb = static_cast<const uint8_t*>(m.sx) + c * sc_bytes;
    t.out = static_cast<uint8_t*>(m.grad_tiles) + (int64_t)ti * kTileElems * OUT_BYTES;
    t.accumulate = m.accumulate;
    return t;
}

template <int OUT, bool BATCH>
__global__ __launch_bounds__(kWgThreads, 1)
void wgrad_mx_kernel(const WgradMxModules mods, int64_t ldq, int64_t chunk, int S, int n_tiles,
                     const int32_t* __restrict__ tile_tab, const int32_t* __restrict__ order, float* __restrict__ slab) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kMxSlots * kMxSlotBytes];   // 132 KiB, one array

    const int total = n_tiles * S;
    const int b = blockIdx.x;
    const int q8 = total >> 3, r8 = total & 7, xcd = b & 7;
    const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    const int s = L / n_tiles;
    const int li = L - s * n_tiles;
    const int tile = order != nullptr ? order[li] : li;
    const WgradMxTile tt = wgrad_mx_tile<BATCH, OUT == kOutBF16 ? 2 : 4>(mods, tile_tab, tile, ldq);
    const int64_t t_begin = (int64_t)s * chunk;
    const int64_t t_end = (t_begin + chunk < ldq) ? (t_begin + chunk) : ldq;
    const int nst = (t_end > t_begin) ? (int)((t_end - t_begin) / kMxBK) : 0;   // ldq, chunk % 64 == 0

    const int64_t blk_bytes = (int64_t)kTile * ldq;       // = (ldq / 64) panels of 16 KiB
    const int64_t sc_bytes = (ldq >> 5) * kTile;
    const __amdgpu_buffer_rsrc_t rqa = uniform_rsrc(tt.qa + t_begin * kTile, blk_bytes - t_begin * kTile);
    const __amdgpu_buffer_rsrc_t rqb = uniform_rsrc(tt.qb + t_begin * kTile, blk_bytes - t_begin * kTile);
    const __amdgpu_buffer_rsrc_t rsa = uniform_rsrc(tt.sa + (t_begin >> 5) * kTile, sc_bytes - (t_begin >> 5) * kTile);
    const __amdgpu_buffer_rsrc_t rsb = uniform_rsrc(tt.sb + (t_begin >> 5) * kTile, sc_bytes - (t_begin >> 5) * kTile);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 2;
    const int wn = wave & 3;

    // DMA geometry: instruction j of wave w fills image rows 16*(2w+j) .. +15 (1 KiB, contiguous in the
    // 64-token panel of the block); lane l lands at row 16*(2w+j) + (l>>2), physical chunk l&3, which
    // holds logical chunk (l&3) ^ ((row>>2)&3).
    int voff[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int row = 16 * (2 * wave + j) + (lane >> 2);
        voff[j] = row * kMxBK + ((((lane & 3) ^ ((row >> 2) & 3))) << 4);
    }
    // exponents: waves 0-3 each move one 256-B k-block row (A kb0, A kb1, B kb0, B kb1) per stage
    const int sc_kb = wave & 1;
    const int sc_voff = sc_kb * kTile + 4 * lane;
    const int per_stage = wave < 4 ? 5 : 4;                 // DMA instructions per stage of this wave

    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(lds));
    auto issue = [&](int st) {
        const uint32_t slot = lds0 + (uint32_t)((st % kMxSlots) * kMxSlotBytes);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t row0 = (uint32_t)(2 * wave + j) * 1024u;
            dma16(rqa, __builtin_amdgcn_readfirstlane(slot + row0), voff[j] + st * kMxImg);
            dma16(rqb, __builtin_amdgcn_readfirstlane(slot + kMxImg + row0), voff[j] + st * kMxImg);
        }
        if (wave < 2)
            dma4(rsa, __builtin_amdgcn_readfirstlane(slot + 2 * kMxImg + sc_kb * kTile), sc_voff + st * 2 * kTile);
        else if (wave < 4)
            dma4(rsb, __builtin_amdgcn_readfirstlane(slot + 2 * kMxImg + 2 * kTile + sc_kb * kTile), sc_voff + st * 2 * kTile);
    };

    f32x16_t acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    const int r32 = lane & 31;
    const int h = lane >> 5;
    if (nst > 0) issue(0);
    if (nst > 1) issue(1);
    for (int st = 0; st < nst; ++st) {
        if (st + 2 < nst) {
            issue(st + 2);
            wait_vm_n(2 * per_stage);                       // stage st landed (st+1, st+2 in flight)
        } else if (st + 1 < nst) {
            wait_vm_n(per_stage);
        } else {
            wait_vm_n(0);
        }
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        const uint8_t* A = lds + (st % kMxSlots) * kMxSlotBytes;
        const uint8_t* B = A + kMxImg;
        const uint8_t* SA = A + 2 * kMxImg + h * kTile;     // this lane's k-block of the stage
        const uint8_t* SB = SA + 2 * kTile;
        i32x8_t af[4], bfr[2];
        int as[4], bs[2];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
            const int row = wm * 128 + mb * 32 + r32;
            af[mb] = mx_frag(A, row, h);
            as[mb] = SA[row];
        }
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
            const int col = wn * 64 + nb * 32 + r32;
            bfr[nb] = mx_frag(B, col, h);
            bs[nb] = SB[col];
        }
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
                acc[mb][nb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bfr[nb], af[mb], acc[mb][nb],
                                                                               0, 0, 0, bs[nb], 0, as[mb]);
    }
    wgrad_store_t<OUT, 4>(acc, (OUT == kOutSlab || OUT == kOutSlabBF16) ? wgrad_dst<OUT>(slab, tile, s, S) : tt.out,
                          wm * 128, wn * 64, lane, tt.accumulate);
}

// Quarter-tile MX variant for modules with few tiles (the fill-bound regime, as wgrad_quarter_kernel):
// 256 threads (4 waves as 2x2, 64x64 outputs each = 2x2 accumulators), one 128x128 quarter of a tile
// per workgroup, 4-slot ring of 64-token stages of two [128 rows][64 B] images + 2 x 256 B of
// exponents (66 KiB: two workgroups per CU). Logical ids, schedule, slabs and epilogue as
// wgrad_quarter_kernel; fragment / scale maps as wgrad_mx_kernel.
constexpr int kMxQImg = 128 * kMxBK;                        // 8 KiB per operand per stage
constexpr int kMxQSlotBytes = 2 * kMxQImg + 2 * 256;

template <int OUT, bool BATCH>
__global__ __launch_bounds__(kQThreads, 2)
void wgrad_mx_quarter_kernel(const WgradMxModules mods, int64_t ldq, int64_t chunk, int S, int n_tiles,
                             const int32_t* __restrict__ tile_tab, const int32_t* __restrict__ order,
                             float* __restrict__ slab) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kMxSlots * kMxQSlotBytes];  // 66 KiB, one array

    const int total = n_tiles * S * 4;
    const int b = blockIdx.x;
    const int q8 = total >> 3, r8 = total & 7, xcd = b & 7;
    const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
    const int qd = L & 3;
    const int ts = L >> 2;
    const int s = ts / n_tiles;
    const int li = ts - s * n_tiles;
    const int tile = order != nullptr ? order[li] : li;
    const int qm = qd >> 1, qn = qd & 1;
    const WgradMxTile tt = wgrad_mx_tile<BATCH, OUT == kOutBF16 ? 2 : 4>(mods, tile_tab, tile, ldq);
    const int64_t t_begin = (int64_t)s * chunk;
    const int64_t t_end = (t_begin + chunk < ldq) ? (t_begin + chunk) : ldq;
    const int nst = (t_end > t_begin) ? (int)((t_end - t_begin) / kMxBK) : 0;

    const int64_t blk_bytes = (int64_t)kTile * ldq;
    const int64_t sc_bytes = (ldq >> 5) * kTile;
    // this quarter's 128 rows of the A / B blocks
    const __amdgpu_buffer_rsrc_t rqa = uniform_rsrc(tt.qa + t_begin * kTile + qm * 128 * kMxBK,
                                                    blk_bytes - t_begin * kTile - qm * 128 * kMxBK);
    const __amdgpu_buffer_rsrc_t rqb = uniform_rsrc(tt.qb + t_begin * kTile + qn * 128 * kMxBK,
                                                    blk_bytes - t_begin * kTile - qn * 128 * kMxBK);
    const __amdgpu_buffer_rsrc_t rsa = uniform_rsrc(tt.sa + (t_begin >> 5) * kTile, sc_bytes - (t_begin >> 5) * kTile);
    const __amdgpu_buffer_rsrc_t rsb = uniform_rsrc(tt.sb + (t_begin >> 5) * kTile, sc_bytes - (t_begin >> 5) * kTile);

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave >> 1;
    const int wn = wave & 1;

    // image DMA: instruction j of wave w fills rows 16*(2w+j) .. +15 of each 128-row image (1 KiB
    // contiguous in the panel layout)
    int voff[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int row = 16 * (2 * wave + j) + (lane >> 2);
        voff[j] = row * kMxBK + ((((lane & 3) ^ ((row >> 2) & 3))) << 4);
    }
    // exponents: wave 0 moves A's, wave 1 B's: lanes 0-31 the quarter's 128 B of k-block 2st,
    // lanes 32-63 those of k-block 2st+1
    const int sc_voff = (lane >> 5) * kTile + (wave == 0 ? qm : qn) * 128 + 4 * (lane & 31);
    const int per_stage = wave < 2 ? 5 : 4;

    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(lds));
    auto issue = [&](int st) {
        const uint32_t slot = lds0 + (uint32_t)((st % kMxSlots) * kMxQSlotBytes);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const uint32_t row0 = (uint32_t)(2 * wave + j) * 1024u;
            dma16(rqa, __builtin_amdgcn_readfirstlane(slot + row0), voff[j] + st * kMxImg);
            dma16(rqb, __builtin_amdgcn_readfirstlane(slot + kMxQImg + row0), voff[j] + st * kMxImg);
        }
        if (wave == 0)
            dma4(rsa, __builtin_amdgcn_readfirstlane(slot + 2 * kMxQImg), sc_voff + st * 2 * kTile);
        else if (wave == 1)
            dma4(rsb, __builtin_amdgcn_readfirstlane(slot + 2 * kMxQImg + 256), sc_voff + st * 2 * kTile);
    };

    f32x16_t acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    const int r32 = lane & 31;
    const int h = lane >> 5;
    if (nst > 0) issue(0);
    if (nst > 1) issue(1);
    for (int st = 0; st < nst; ++st) {
        if (st + 2 < nst) {
            issue(st + 2);
            wait_vm_n(2 * per_stage);
        } else if (st + 1 < nst) {
            wait_vm_n(per_stage);
        } else {
            wait_vm_n(0);
        }
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        const uint8_t* A = lds + (st % kMxSlots) * kMxQSlotBytes;
        const uint8_t* B = A + kMxQImg;
        const uint8_t* SA = A + 2 * kMxQImg + h * 128;     // this lane's k-block of the stage
        const uint8_t* SB = SA + 256;
        i32x8_t af[2], bfr[2];
        int as[2], bs[2];
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
            const int row = wm * 64 + mb * 32 + r32;
            af[mb] = mx_frag(A, row, h);
            as[mb] = SA[row];
        }
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
            const int col = wn * 64 + nb * 32 + r32;
            bfr[nb] = mx_frag(B, col, h);
            bs[nb] = SB[col];
        }
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
                acc[mb][nb] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bfr[nb], af[mb], acc[mb][nb],
                                                                               0, 0, 0, bs[nb], 0, as[mb]);
    }
    wgrad_store_t<OUT, 2>(acc, (OUT == kOutSlab || OUT == kOutSlabBF16) ? wgrad_dst<OUT>(slab, tile, s, S) : tt.out,
                          qm * 128 + wm * 64, qn * 128 + wn * 64, lane, tt.accumulate);
}

// ------------------------------------------------------------------------------------------------
// Tile gather / scatter (smt.py:317-325 and 332-341): 16 B per thread, 32 workgroups per tile.
// ------------------------------------------------------------------------------------------------
template <bool SCATTER, int ELEM_BYTES>
__global__ __launch_bounds__(256)
void tile_copy_kernel(uint8_t* __restrict__ weight, int64_t ld_weight, const int32_t* __restrict__ tile_rc,
                      uint8_t* __restrict__ tiles) {
    constexpr int kVec = 16 / ELEM_BYTES;                      // elements per 16 B
    constexpr int kChunksPerRow = kTile / kVec;                // 32 or 64
    constexpr int kChunksPerTile = kTile * kChunksPerRow;      // 8192 or 16384
    constexpr int kWgPerTile = kChunksPerTile / 256;           // 32 or 64
    const int tile = blockIdx.x / kWgPerTile;
    const int chunk = (blockIdx.x - tile * kWgPerTile) * 256 + threadIdx.x;
    const int m = chunk / kChunksPerRow;
    const int n = (chunk - m * kChunksPerRow) * kVec;
    const int r = tile_rc[2 * tile];
    const int c = tile_rc[2 * tile + 1];
    uint4* w = reinterpret_cast<uint4*>(weight + (((int64_t)r * kTile + m) * ld_weight + (int64_t)c * kTile + n) * ELEM_BYTES);
    uint4* t = reinterpret_cast<uint4*>(tiles + ((int64_t)tile * kTileElems + (int64_t)m * kTile + n) * ELEM_BYTES);
    if (SCATTER) *w = *t;
    else *t = *w;
}


// ------------------------------------------------------------------------------------------------
// Warm-up accumulation (fine_tune.py:731-741): dst = float(src) (first step) or dst += float(src).
// 4096 elements per workgroup (256 threads x 2 passes x 8); entries found by binary search over
// chunk_begin. One IEEE fp32 add of a widened bf16/fp16 value per element: bit-identical to the
// CPU `acc += grad.cpu().to(torch.float32)` of the reference.
// ------------------------------------------------------------------------------------------------
constexpr int kAccChunk = 4096;

__device__ __forceinline__ int find_acc_entry(const smt_accum_entry* e, int n, int64_t chunk) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (e[mid].chunk_begin <= chunk) lo = mid; else hi = mid - 1;
    }
    return lo;
}

template <int DT>
__device__ __forceinline__ float load_elem(const void* p, int64_t i) {
    if (DT == SMT_DTYPE_BF16) return bf16_bits_to_f32(static_cast<const uint16_t*>(p)[i]);
    if (DT == SMT_DTYPE_FP16) return half_bits_to_f32(static_cast<const uint16_t*>(p)[i]);
    return static_cast<const float*>(p)[i];
}

template <int DT>
__device__ __forceinline__ void load8(const void* p, int64_t i, float (&v)[8]) {
    if (DT == SMT_DTYPE_FP32) {
        const float4 a = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
        const float4 b = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
        const uint4 a = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(p) + i);
        const uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (DT == SMT_DTYPE_BF16) {
                v[2 * j] = bf16_bits_to_f32(w[j] & 0xffffu);
                v[2 * j + 1] = bf16_bits_to_f32(w[j] >> 16);
            } else {
                v[2 * j] = half_bits_to_f32((uint16_t)(w[j] & 0xffffu));
                v[2 * j + 1] = half_bits_to_f32((uint16_t)(w[j] >> 16));
            }
        }
    }
}

template <int DT>
__device__ void accumulate_chunk(const smt_accum_entry& ent, int64_t base) {
    const bool vec = ((reinterpret_cast<uintptr_t>(ent.src) | reinterpret_cast<uintptr_t>(ent.dst)) & 15u) == 0;
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
        const int64_t i0 = base + pass * 2048 + threadIdx.x * 8;
        if (i0 >= ent.n) continue;
        if (vec && i0 + 8 <= ent.n) {
            float v[8];
            load8<DT>(ent.src, i0, v);
            float4* d = reinterpret_cast<float4*>(ent.dst + i0);
            float4 a = ent.assign ? make_float4(0.f, 0.f, 0.f, 0.f) : d[0];
            float4 b = ent.assign ? make_float4(0.f, 0.f, 0.f, 0.f) : d[1];
            if (ent.assign) {
                a = make_float4(v[0], v[1], v[2], v[3]);
                b = make_float4(v[4], v[5], v[6], v[7]);
            } else {
                a.x += v[0]; a.y += v[1]; a.z += v[2]; a.w += v[3];
                b.x += v[4]; b.y += v[5]; b.z += v[6]; b.w += v[7];
            }
            d[0] = a;
            d[1] = b;
        } else {
            for (int j = 0; j < 8; ++j) {
                const int64_t i = i0 + j;
                if (i < ent.n) {
                    const float v = load_elem<DT>(ent.src, i);
                    ent.dst[i] = ent.assign ? v : ent.dst[i] + v;
                }
            }
        }
    }
}

__global__ __launch_bounds__(256)
void grad_accumulate_kernel(const smt_accum_entry* __restrict__ entries, int n_entries) {
    const int64_t chunk = blockIdx.x;
    const smt_accum_entry ent = entries[find_acc_entry(entries, n_entries, chunk)];
    const int64_t base = (chunk - ent.chunk_begin) * kAccChunk;
    if (ent.src_dtype == SMT_DTYPE_BF16) accumulate_chunk<SMT_DTYPE_BF16>(ent, base);
    else if (ent.src_dtype == SMT_DTYPE_FP16) accumulate_chunk<SMT_DTYPE_FP16>(ent, base);
    else accumulate_chunk<SMT_DTYPE_FP32>(ent, base);
}

// ------------------------------------------------------------------------------------------------
// Block scores (smt_helper.py:67-78, 233-251): one 256-thread workgroup per 256x256 block of an
// fp32 gradient; float4 row loads (a wave covers one 1 KiB row), fp64 accumulation, wave shuffle
// then LDS reduction in a fixed order. Writes, per block, the fp64 sum of the reference's terms
// (g for mean_abs, |g| for abs_mean / L1, the fp32-rounded g*g of `g.abs()**2` for L2) and the fp64
// sum of their magnitudes. The host turns the first into mean / abs / sqrt and rounds to fp32; the
// second bounds how far ATen's fp32 reduction of the same terms can be from it (smt_helper.py).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int find_score_entry(const smt_score_entry* e, int n, int64_t blk) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (e[mid].block_begin <= blk) lo = mid; else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// contract(off): the L2 term is the fp32-rounded square, never fused into the fp64 add
#pragma clang fp contract(off)
template <int STRAT>
__device__ __forceinline__ double score_term(float f) {
    if (STRAT == SMT_SCORE_MEAN_ABS) return (double)f;
    if (STRAT == SMT_SCORE_L2) return (double)(f * f);             // the fp32 square of `g.abs()**2`
    return (double)fabsf(f);
}

// acc.x = sum of terms, acc.y = sum of |terms| (only differs from acc.x for mean_abs)
template <int STRAT>
__device__ double2 block_partial(const float* __restrict__ src, int64_t ld) {
    const int col = (threadIdx.x & 63) * 4;
    const int row0 = threadIdx.x >> 6;
    double s = 0.0, m = 0.0;
#pragma unroll 4
    for (int it = 0; it < kTile / 4; ++it) {
        const float4 v = *reinterpret_cast<const float4*>(src + (int64_t)(row0 + 4 * it) * ld + col);
        s += score_term<STRAT>(v.x) + score_term<STRAT>(v.y) + score_term<STRAT>(v.z) + score_term<STRAT>(v.w);
        if (STRAT == SMT_SCORE_MEAN_ABS)
            m += (double)fabsf(v.x) + (double)fabsf(v.y) + (double)fabsf(v.z) + (double)fabsf(v.w);
    }
    return make_double2(s, STRAT == SMT_SCORE_MEAN_ABS ? m : s);
}

__global__ __launch_bounds__(256)
void block_score_kernel(const smt_score_entry* __restrict__ entries, int n_entries) {
    __shared__ double part[2][4];
    const int64_t blk = blockIdx.x;
    const smt_score_entry ent = entries[find_score_entry(entries, n_entries, blk)];
    const int64_t local = blk - ent.block_begin;
    const int bi = (int)(local / ent.d2);
    const int bj = (int)(local - (int64_t)bi * ent.d2);
    const float* src = ent.src + (int64_t)bi * kTile * ent.ld + (int64_t)bj * kTile;
    double2 acc;
    switch (ent.strategy) {
        case SMT_SCORE_MEAN_ABS: acc = block_partial<SMT_SCORE_MEAN_ABS>(src, ent.ld); break;
        case SMT_SCORE_L2: acc = block_partial<SMT_SCORE_L2>(src, ent.ld); break;
        default: acc = block_partial<SMT_SCORE_ABS_MEAN>(src, ent.ld); break;
    }
    acc.x = wave_sum(acc.x);
    acc.y = wave_sum(acc.y);
    if ((threadIdx.x & 63) == 0) {
        part[0][threadIdx.x >> 6] = acc.x;
        part[1][threadIdx.x >> 6] = acc.y;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        reinterpret_cast<double2*>(ent.out)[local] =
            make_double2((part[0][0] + part[0][1]) + (part[0][2] + part[0][3]),
                         (part[1][0] + part[1][1]) + (part[1][2] + part[1][3]));
    }
}
#pragma clang fp contract(fast)

// ------------------------------------------------------------------------------------------------
// Global squared L2 norm of the flat fp32 gradient (deterministic two-pass, fp64).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256)
void sq_norm_partial_kernel(const float* __restrict__ x, int64_t n, double* __restrict__ partials) {
    __shared__ double part[4];
    double acc = 0.0;
    const int64_t n4 = ((reinterpret_cast<uintptr_t>(x) & 15u) == 0) ? n / 4 : 0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const float4 v = reinterpret_cast<const float4*>(x)[i];
        acc += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    }
    for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        acc += (double)x[i] * x[i];
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) partials[blockIdx.x] = (part[0] + part[1]) + (part[2] + part[3]);
}

__global__ __launch_bounds__(256)
void sq_norm_final_kernel(const double* __restrict__ partials, int n, double* __restrict__ out) {
    __shared__ double part[4];
    double acc = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) acc += partials[i];
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) out[0] = (part[0] + part[1]) + (part[2] + part[3]);
}

// ------------------------------------------------------------------------------------------------
// Fused clip + AdamW + bf16 cast + scatter into W. 8 elements per thread; in tile mode 32
// workgroups per 256x256 tile (8 tile rows per workgroup) so the W destination is one scalar
// descriptor per workgroup and every W store is a 16-B piece of a 512-B tile row.
// ------------------------------------------------------------------------------------------------
struct AdamStep {
    float lr, b1, b2, eps, wd, bc1, bc2;
    int mode;
    __device__ __forceinline__ void apply(float g, float& p, float& m, float& v) const {
        if (mode == SMT_ADAM_DEEPSPEED) {
            m = b1 * m + (1.f - b1) * g;
            v = b2 * v + (1.f - b2) * g * g;
            const float denom = sqrtf(v / bc2) + eps;
            const float update = (m / bc1) / denom + wd * p;
            p = p - lr * update;
        } else {
            p = p * (1.f - lr * wd);
            m = m + (1.f - b1) * (g - m);
            v = v * b2 + (1.f - b2) * g * g;
            const float denom = sqrtf(v) / sqrtf(bc2) + eps;
            p = p - (lr / bc1) * (m / denom);
        }
    }
};

// the updated values in the parameter dtype (ABI v12: the reference's --dtype, fine_tune.py:955-959):
// 8 elements are 16 B of bf16 / fp16 (a) or 32 B of fp32 (a, b)
struct Packed8 {
    uint4 a, b;
};

template <int PDT>
__device__ __forceinline__ uint16_t param16(float f) {
    return PDT == SMT_DTYPE_FP16 ? f32_to_half_bits(f) : f32_to_bf16_bits(f);
}

template <int PDT>
__device__ __forceinline__ void pack8(const float (&p)[8], Packed8& out) {
    if (PDT == SMT_DTYPE_FP32) {
        out.a = make_uint4(__float_as_uint(p[0]), __float_as_uint(p[1]), __float_as_uint(p[2]), __float_as_uint(p[3]));
        out.b = make_uint4(__float_as_uint(p[4]), __float_as_uint(p[5]), __float_as_uint(p[6]), __float_as_uint(p[7]));
    } else {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            w[j] = (uint32_t)param16<PDT>(p[2 * j]) | ((uint32_t)param16<PDT>(p[2 * j + 1]) << 16);
        out.a = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

// 8 consecutive elements at element i of a parameter-dtype buffer
template <int PDT>
__device__ __forceinline__ void store8(void* base, int64_t i, const Packed8& v) {
    if (PDT == SMT_DTYPE_FP32) {
        uint4* d = reinterpret_cast<uint4*>(static_cast<float*>(base) + i);
        d[0] = v.a;
        d[1] = v.b;
    } else {
        *reinterpret_cast<uint4*>(static_cast<uint16_t*>(base) + i) = v.a;
    }
}

template <int PDT>
__device__ __forceinline__ void store1(void* base, int64_t i, float p) {
    if (PDT == SMT_DTYPE_FP32) static_cast<float*>(base)[i] = p;
    else static_cast<uint16_t*>(base)[i] = param16<PDT>(p);
}

template <int GDT, int PDT>
__device__ __forceinline__ void adam8(const void* grad, float* master, float* m, float* v, void* param,
                                      int64_t f, float gscale, const AdamStep& st, Packed8* packed) {
    float g[8];
    load8<GDT>(grad, f, g);
    float4* P = reinterpret_cast<float4*>(master + f);
    float4* M = reinterpret_cast<float4*>(m + f);
    float4* V = reinterpret_cast<float4*>(v + f);
    float4 p0 = P[0], p1 = P[1], m0 = M[0], m1 = M[1], v0 = V[0], v1 = V[1];
    float pp[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
    float mm[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
    float vv[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) st.apply(g[j] * gscale, pp[j], mm[j], vv[j]);
    P[0] = make_float4(pp[0], pp[1], pp[2], pp[3]); P[1] = make_float4(pp[4], pp[5], pp[6], pp[7]);
    M[0] = make_float4(mm[0], mm[1], mm[2], mm[3]); M[1] = make_float4(mm[4], mm[5], mm[6], mm[7]);
    V[0] = make_float4(vv[0], vv[1], vv[2], vv[3]); V[1] = make_float4(vv[4], vv[5], vv[6], vv[7]);
    pack8<PDT>(pp, *packed);
    store8<PDT>(param, f, *packed);
}

// norm_sq: squared global norm of the EFFECTIVE gradient (after grad_scale), fp64.
__device__ __forceinline__ float clip_scale(const double* norm_sq, float max_norm, float grad_scale) {
    float s = grad_scale;
    if (norm_sq != nullptr && max_norm > 0.f) {
        // DeepSpeed: clip = (total_norm + 1e-6) / max_norm; grads *= 1/clip when clip > 1.
        const float total = (float)sqrt(*norm_sq);
        const float clip = (total + 1e-6f) / max_norm;
        if (clip > 1.f) s = grad_scale / clip;
    }
    return s;
}

template <int GDT, int PDT>
__global__ __launch_bounds__(256)
void adamw_tiles_kernel(const void* __restrict__ grad, float* __restrict__ master, float* __restrict__ m,
                        float* __restrict__ v, void* __restrict__ param,
                        const smt_tile_desc* __restrict__ tiles, const double* __restrict__ norm_sq,
                        smt_adamw_args a) {
    const int tile = blockIdx.x >> 5;
    const int local = (((blockIdx.x & 31) << 8) + threadIdx.x) * 8;   // element within the tile
    const smt_tile_desc d = tiles[tile];
    const int64_t f = d.flat_offset + local;
    const AdamStep st{a.lr, a.beta1, a.beta2, a.eps, a.weight_decay, a.bias_correction1, a.bias_correction2, a.mode};
    const float gscale = clip_scale(norm_sq, a.max_grad_norm, a.grad_scale);
    Packed8 packed;
    adam8<GDT, PDT>(grad, master, m, v, param, f, gscale, st, &packed);
    if (d.weight != nullptr) {
        const int row = local >> 8;
        const int col = local & 255;
        store8<PDT>(d.weight, ((int64_t)d.row_block * kTile + row) * d.ld_weight + (int64_t)d.col_block * kTile + col,
                    packed);
    }
}

template <int GDT, int PDT>
__global__ __launch_bounds__(256)
void adamw_flat_kernel(const void* __restrict__ grad, float* __restrict__ master, float* __restrict__ m,
                       float* __restrict__ v, void* __restrict__ param, int64_t n,
                       const double* __restrict__ norm_sq, smt_adamw_args a) {
    const int64_t f = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
    if (f >= n) return;
    const AdamStep st{a.lr, a.beta1, a.beta2, a.eps, a.weight_decay, a.bias_correction1, a.bias_correction2, a.mode};
    const float gscale = clip_scale(norm_sq, a.max_grad_norm, a.grad_scale);
    if (f + 8 <= n) {
        Packed8 packed;
        adam8<GDT, PDT>(grad, master, m, v, param, f, gscale, st, &packed);
    } else {
        for (int64_t i = f; i < n; ++i) {
            float pp = master[i], mm = m[i], vv = v[i];
            st.apply(load_elem<GDT>(grad, i) * gscale, pp, mm, vv);
            master[i] = pp; m[i] = mm; v[i] = vv;
            store1<PDT>(param, i, pp);
        }
    }
}

// Multi-tensor flat AdamW: one launch over every dense parameter of the warm-up full fine-tune
// (DeepSpeed FusedAdam's multi_tensor_apply, external). Workgroup w covers 2048 elements of the
// tensor t with block_start[t] <= w < block_start[t+1] (binary search over the n+1 prefix).
template <int GDT, int PDT>
__global__ __launch_bounds__(256)
void adamw_multi_kernel(const smt_adamw_tensor* __restrict__ tensors, const int64_t* __restrict__ block_start,
                        int32_t n_tensors, const double* __restrict__ norm_sq, smt_adamw_args a) {
    const int64_t w = blockIdx.x;
    int lo = 0, hi = n_tensors - 1;
    while (lo < hi) {                                   // last t with block_start[t] <= w
        const int mid = (lo + hi + 1) >> 1;
        if (block_start[mid] <= w) lo = mid; else hi = mid - 1;
    }
    const smt_adamw_tensor d = tensors[lo];
    const int64_t f = ((w - block_start[lo]) * 256 + threadIdx.x) * 8;
    if (f >= d.n) return;
    const AdamStep st{a.lr, a.beta1, a.beta2, a.eps, a.weight_decay, a.bias_correction1, a.bias_correction2, a.mode};
    const float gscale = clip_scale(norm_sq, a.max_grad_norm, a.grad_scale);
    if (f + 8 <= d.n) {
        Packed8 packed;
        adam8<GDT, PDT>(d.grad, d.master, d.exp_avg, d.exp_avg_sq, d.param, f, gscale, st, &packed);
    } else {
        for (int64_t i = f; i < d.n; ++i) {
            float pp = d.master[i], mm = d.exp_avg[i], vv = d.exp_avg_sq[i];
            st.apply(load_elem<GDT>(d.grad, i) * gscale, pp, mm, vv);
            d.master[i] = pp; d.exp_avg[i] = mm; d.exp_avg_sq[i] = vv;
            store1<PDT>(d.param, i, pp);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Channel path (smt.py:185-296, smt_helper.py:149-230, fine_tune.py:636-667).
// ------------------------------------------------------------------------------------------------
// Row gather / scatter of the selected rows (smt.py:200-204 gather, 211-213 per-forward write-back):
// rows_buf[i, :] <-> W[rows[i], :]. One workgroup per (row, 4 KiB slice), 16 B per thread.
constexpr int kRowSliceBytes = 4096;

template <bool SCATTER>
__global__ __launch_bounds__(256)
void row_copy_kernel(uint8_t* __restrict__ weight, int64_t ld_w_bytes, const int32_t* __restrict__ rows,
                     uint8_t* __restrict__ buf, int64_t ld_b_bytes, int64_t row_bytes, int32_t slices) {
    const int64_t i = blockIdx.x / slices;
    const int64_t off = (int64_t)(blockIdx.x - i * slices) * kRowSliceBytes + threadIdx.x * 16;
    if (off >= row_bytes) return;
    const int64_t r = rows[i];
    uint4* w = reinterpret_cast<uint4*>(weight + r * ld_w_bytes + off);
    uint4* b = reinterpret_cast<uint4*>(buf + i * ld_b_bytes + off);
    if (SCATTER) *w = *b;
    else *b = *w;
}

// partial_input of linearChannel.forward (smt.py:225-233): out[t, j] = x[t, cols[j]] for j < n_cols,
// 0 for n_cols <= j < ld_out (zero columns pad the operand to a whole number of 256-blocks for the
// tile wgrad). Each workgroup stages up to 4 rows of x (their first n_in elements) into LDS with
// coalesced 16-B loads, then each thread gathers 8 consecutive outputs from LDS and writes them as
// one 16-B store (the previous version gathered 2-B elements from global memory: 0.15 of HBM).
__global__ __launch_bounds__(256)
void column_gather_kernel(const uint16_t* __restrict__ x, int64_t ld_x, int64_t n_in, int64_t T,
                          const int32_t* __restrict__ cols, int32_t n_cols, uint16_t* __restrict__ out,
                          int64_t ld_out, int rows) {
    extern __shared__ __attribute__((aligned(16))) uint16_t rowbuf[];      // [rows][n_in8]
    const int64_t n_in8 = (n_in + 7) & ~(int64_t)7;
    const int64_t t0 = (int64_t)blockIdx.x * rows;
    const int tid = threadIdx.x;
    const int64_t chunks = n_in8 >> 3;
    for (int r = 0; r < rows; ++r) {
        const int64_t t = t0 + r;
        if (t >= T) break;
        const uint16_t* xr = x + t * ld_x;
        for (int64_t k = tid; k < chunks; k += 256) {
            if (8 * k + 8 <= n_in) {
                *reinterpret_cast<uint4*>(rowbuf + r * n_in8 + 8 * k) = *reinterpret_cast<const uint4*>(xr + 8 * k);
            } else {
                for (int64_t e = 8 * k; e < n_in8; ++e) rowbuf[r * n_in8 + e] = e < n_in ? xr[e] : 0;
            }
        }
    }
    __syncthreads();
    const int64_t vec_per_row = ld_out >> 3;
    for (int r = 0; r < rows; ++r) {
        const int64_t t = t0 + r;
        if (t >= T) break;
        const uint16_t* br = rowbuf + r * n_in8;
        for (int64_t v = tid; v < vec_per_row; v += 256) {
            const int j0 = (int)(v * 8);
            int idx[8];
            if (j0 + 8 <= n_cols) {                               // 8 indices as two 16-B loads
                const int4 a = *reinterpret_cast<const int4*>(cols + j0);
                const int4 b = *reinterpret_cast<const int4*>(cols + j0 + 4);
                idx[0] = a.x; idx[1] = a.y; idx[2] = a.z; idx[3] = a.w;
                idx[4] = b.x; idx[5] = b.y; idx[6] = b.z; idx[7] = b.w;
            } else {
#pragma unroll
                for (int q = 0; q < 8; ++q) idx[q] = j0 + q < n_cols ? cols[j0 + q] : -1;
            }
            uint32_t w[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t lo = idx[2 * q] >= 0 ? br[idx[2 * q]] : 0u;
                const uint32_t hi = idx[2 * q + 1] >= 0 ? br[idx[2 * q + 1]] : 0u;
                w[q] = lo | (hi << 16);
            }
            *reinterpret_cast<uint4*>(out + t * ld_out + j0) = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
}

// The same gather with the rows staged by LDS-DMA (buffer_load ... lds): a row is ppr 1 KiB pieces
// (one wave instruction each; the last may run past n_in into the row's padding or the next row,
// bytes the gather never indexes; past the last row's n_in elements the descriptor returns zeros). All R * ppr
// pieces of a workgroup are in flight at once without passing through registers (the round-3
// attempt to issue a thread's loads ahead in registers ran 1.65x slower). Each thread then loads
// its 8 output indices once and gathers them from every staged row.
template <int R>
__global__ __launch_bounds__(256)
void column_gather_dma_kernel(const uint16_t* __restrict__ x, int64_t ld_x, int64_t n_in, int64_t T, int ppr,
                              const int32_t* __restrict__ cols, int32_t n_cols, uint16_t* __restrict__ out,
                              int64_t ld_out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t cg_lds[];          // [R][ppr * 1 KiB]
    const int64_t t0 = (int64_t)blockIdx.x * R;
    const int rows = (int)(T - t0 < R ? T - t0 : R);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // the descriptor ends at the last row's n_in-th element: a piece running past it reads zeros,
    // never memory past a column-slice view's allocation
    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(x + t0 * ld_x, (int64_t)(rows - 1) * ld_x * 2 + n_in * 2);
    const uint32_t lds0 = __builtin_amdgcn_readfirstlane(lds_addr(cg_lds));
    const int row_stride = ppr * 1024;
    for (int p = wave; p < rows * ppr; p += 4) {
        const int r = p / ppr, c = p - r * ppr;
        dma16(rs, __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(r * row_stride + c * 1024)),
              (int)(r * ld_x * 2 + c * 1024 + lane * 16));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int64_t vec_per_row = ld_out >> 3;
    for (int64_t v = tid; v < vec_per_row; v += 256) {
        const int j0 = (int)(v * 8);
        int idx[8];
        if (j0 + 8 <= n_cols) {
            const int4 a = *reinterpret_cast<const int4*>(cols + j0);
            const int4 b = *reinterpret_cast<const int4*>(cols + j0 + 4);
            idx[0] = a.x; idx[1] = a.y; idx[2] = a.z; idx[3] = a.w;
            idx[4] = b.x; idx[5] = b.y; idx[6] = b.z; idx[7] = b.w;
        } else {
#pragma unroll
            for (int q = 0; q < 8; ++q) idx[q] = j0 + q < n_cols ? cols[j0 + q] : -1;
        }
        for (int r = 0; r < rows; ++r) {
            const uint16_t* br = reinterpret_cast<const uint16_t*>(cg_lds + r * row_stride);
            uint32_t w[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t lo = idx[2 * q] >= 0 ? br[idx[2 * q]] : 0u;
                const uint32_t hi = idx[2 * q + 1] >= 0 ? br[idx[2 * q + 1]] : 0u;
                w[q] = lo | (hi << 16);
            }
            *reinterpret_cast<uint4*>(out + (t0 + r) * ld_out + j0) = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
}

// Transposed tile scatter: Wt[c*256 + j, r*256 + k] = tile[k, j] for every descriptor (weight = the
// transposed copy Wt = W^T of a frozen W, ld_weight its row stride, (row_block, col_block) = the
// tile's (r, c) in W, flat_offset = the tile in the bf16 source). Keeps the transposed copies that
// the data-gradient GEMMs read (g @ W as the TN product g @ Wt^T) in step with the tiles. One
// workgroup per 64x64 sub-block, transposed through LDS.
__global__ __launch_bounds__(256)
void tile_scatter_t_kernel(const smt_tile_desc* __restrict__ descs, const uint16_t* __restrict__ src) {
    __shared__ __attribute__((aligned(16))) uint16_t sub[64][72];      // 144-B rows
    const int tile = blockIdx.x >> 4;
    const int sb = blockIdx.x & 15;
    const int k0 = (sb >> 2) * 64, j0 = (sb & 3) * 64;               // sub-block origin (tile row k, col j)
    const smt_tile_desc d = descs[tile];
    if (d.weight == nullptr) return;
    const uint16_t* t = src + d.flat_offset;
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = tid; i < 512; i += 256) {
        const int k = i >> 3, ch = i & 7;
        *reinterpret_cast<uint4*>(&sub[k][ch * 8]) =
            *reinterpret_cast<const uint4*>(t + (int64_t)(k0 + k) * kTile + j0 + ch * 8);
    }
    __syncthreads();
    uint16_t* w = static_cast<uint16_t*>(d.weight);
#pragma unroll
    for (int i = tid; i < 512; i += 256) {
        const int j = i >> 3, ch = i & 7;
        uint32_t p[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            p[q] = (uint32_t)sub[ch * 8 + 2 * q][j] | ((uint32_t)sub[ch * 8 + 2 * q + 1][j] << 16);
        *reinterpret_cast<uint4*>(w + ((int64_t)d.col_block * kTile + j0 + j) * d.ld_weight +
                                  (int64_t)d.row_block * kTile + k0 + ch * 8) = make_uint4(p[0], p[1], p[2], p[3]);
    }
}

// The 256-column blocks of x that a module's tiles read, block-major:
// out[j, t, k] = x[t, col_blocks[j]*256 + k]. linearZ saves this [n_cb, T, 256] copy for its
// backward instead of the whole input (the tile wgrad reads nothing else), each block's rows
// contiguous so that the wgrad's x stages are contiguous 16 KiB reads. 16 B per thread; one wave
// covers two (row, block) pairs of 512 contiguous bytes on both sides.
__global__ __launch_bounds__(256)
void colblock_gather_kernel(const uint16_t* __restrict__ x, int64_t ld_x, int64_t T,
                            const int32_t* __restrict__ col_blocks, int32_t n_cb, uint16_t* __restrict__ out) {
    const int64_t per_row = (int64_t)n_cb * 32;                  // 16-B chunks per output row
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t t = v / per_row;
    if (t >= T) return;
    const int r = (int)(v - t * per_row);
    const int j = r >> 5, ch = r & 31;
    const uint4 val = *reinterpret_cast<const uint4*>(x + t * ld_x + (int64_t)col_blocks[j] * kTile + ch * 8);
    *reinterpret_cast<uint4*>(out + ((int64_t)j * T + t) * kTile + ch * 8) = val;     // block-major [n_cb][T][256]
}

// Activation harvest, the forward hook of fine_tune.py:636-667: the reference keeps, per key, the
// fp32 [B, S, in] tensor `feat[key] = |x|` (first step) / `feat[key] += |x|` (later steps). Same
// state here, elementwise in HBM: acc[b, s, c] = (assign ? 0 : acc[b, s, c]) + float(|x[b, s, c]|),
// one fp32 add per element exactly as the CPU `+=` (|x| of a bf16/fp16 value is exact in fp32).
// One thread per 8 contiguous channels: one 16-B (bf16) or 32-B (fp32) load, 32 B read-modify-write.
template <int DT>
__global__ __launch_bounds__(256)
void act_accumulate_kernel(const void* __restrict__ x, int64_t ld_x, int64_t sb, int32_t S,
                           int32_t n_cols, int64_t rows, float* __restrict__ acc, int32_t assign) {
    const int64_t groups = n_cols >> 3;
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t row = v / groups;                       // row = b * S + s
    if (row >= rows) return;
    const int64_t c0 = (v - row * groups) * 8;
    const int64_t b = row / S, s = row - b * S;
    float e[8];
    load8<DT>(x, b * sb + s * ld_x + c0, e);
    float4* a = reinterpret_cast<float4*>(acc + row * n_cols + c0);
    float4 lo = assign ? make_float4(0.f, 0.f, 0.f, 0.f) : a[0];
    float4 hi = assign ? make_float4(0.f, 0.f, 0.f, 0.f) : a[1];
    lo.x += fabsf(e[0]); lo.y += fabsf(e[1]); lo.z += fabsf(e[2]); lo.w += fabsf(e[3]);
    hi.x += fabsf(e[4]); hi.y += fabsf(e[5]); hi.z += fabsf(e[6]); hi.w += fabsf(e[7]);
    a[0] = lo;
    a[1] = hi;
}

// Column statistic of the harvested activations (smt_helper.py:167-184): the reference sums |acc|
// over the batch (`torch.sum(act.abs(), dim=0)`, fp32) and reduces the [S, in] result over the
// sequence. Here, in fp64 (nearly exact): out[c] = sum_s A_s (mean_abs / abs_mean / L1) or
// sum_s A_s^2 (L2) with A_s = sum_b |acc[b, s, c]|. The host divides by S / takes the square root,
// rounds to fp32 once, and bounds the reference's fp32 value around it (smt_helper.py). Two passes
// for parallelism (a [16, 2048, 5120] accumulator is 671 MB): thread (c, p) sums rows
// s in [32p, 32p+32) into partials[p][c]; then out[c] = sum_p partials[p][c], p ascending. A wave
// reads 256 contiguous bytes of a row per (b, s).
constexpr int kChanRows = 32;

__global__ __launch_bounds__(256)
void channel_partial_kernel(const float* __restrict__ acc, int32_t B, int32_t S, int32_t n_cols, int32_t square,
                            double* __restrict__ partials) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= n_cols) return;
    const int p = blockIdx.y;
    const int s0 = p * kChanRows, s1 = min(S, s0 + kChanRows);
    const int64_t bstride = (int64_t)S * n_cols;
    double tot = 0.0;
    for (int s = s0; s < s1; ++s) {
        const float* q = acc + (int64_t)s * n_cols + c;
        double a = 0.0;
        for (int b = 0; b < B; ++b) a += (double)fabsf(q[b * bstride]);
        tot += square ? a * a : a;
    }
    partials[(int64_t)p * n_cols + c] = tot;
}

__global__ __launch_bounds__(256)
void channel_final_kernel(const double* __restrict__ partials, int32_t P, int32_t n_cols, double* __restrict__ out) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= n_cols) return;
    double tot = 0.0;
    for (int p = 0; p < P; ++p) tot += partials[(int64_t)p * n_cols + c];
    out[c] = tot;
}
#pragma clang fp contract(fast)

// Split of T over workgroups for one tile set. One 512-thread workgroup fits per CU (128 KiB LDS),
// so the launch runs in rounds of 256 workgroups; pick S in [1, 64] (chunks >= 512 rows, multiple of
// the 64-row stage) minimising the modelled time below, ties to the smaller S. E.g. at T = 32768:
// n = 27 -> S = 9 (243 workgroups, one round); n = 436 -> S = 4 (7 rounds of T/4 instead of 2 rounds
// of T). S == 1: the tile is written straight from the accumulators.
constexpr int kCUs = 256;
// ------------------------------------------------------------------------------------------------
// Channel mean in ATen's CPU summation order (smt_helper.py:167-176 as the reference computes it:
// torch.sum(act.abs(), dim=0) then torch.mean(., dim=0), i.e. sum then div_ by S on the CPU).
// Both are outer reductions of a contiguous fp32 tensor, which ATen's cascade_sum (SumKernel.cpp,
// multi_row_sum) computes per output column with 4 accumulator levels of 2^p rows,
// p = max(4, ceil_log2(n) / 4): rows are added one by one into level 0 from 0.0f; after every full
// chunk of 2^p rows level j-1 is added into level j and cleared, climbing while the row count is a
// multiple of 2^(p*j); the tail rows go into level 0; finally level 0 += level 1, += level 2,
// += level 3. Each output column is reduced by one thread in that order whatever the thread count
// (parallel_dim_reduction splits the columns). The host checks the result against the reference
// expression once per shape before trusting it (smt_helper.channel_scores_exact).
// Pass 1: one thread per (chunk of the S reduction, column): the chunk's row sum, each row value
// itself the cascade over B. Pass 2: one thread per column replays the levels over the chunks.
// ------------------------------------------------------------------------------------------------
__host__ __device__ inline int cascade_level_power(int64_t n) {
    int lg = 0;
    while (((int64_t)1 << lg) < n) ++lg;                  // ceil_log2 (0 for n <= 1)
    return (lg / 4) > 4 ? (lg / 4) : 4;
}

// the cascade of ATen over n strided values (fp32, no contraction: additions only)
__device__ __forceinline__ float cascade_sum_strided(const float* __restrict__ p, int64_t stride, int64_t n, int lp,
                                                     bool absval) {
    const int64_t step = (int64_t)1 << lp;
    const int64_t mask = step - 1;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int64_t i = 0;
    while (i + step <= n) {
        for (int64_t j = 0; j < step; ++j, ++i) {
            const float v = p[i * stride];
            acc[0] = __fadd_rn(acc[0], absval ? fabsf(v) : v);
        }
        for (int j = 1; j < 4; ++j) {
            acc[j] = __fadd_rn(acc[j], acc[j - 1]);
            acc[j - 1] = 0.f;
            if ((i & (mask << (j * lp))) != 0) break;
        }
    }
    for (; i < n; ++i) {
        const float v = p[i * stride];
        acc[0] = __fadd_rn(acc[0], absval ? fabsf(v) : v);
    }
    for (int j = 1; j < 4; ++j) acc[0] = __fadd_rn(acc[0], acc[j]);
    return acc[0];
}

// pass 1: chunk q < n_full of the S reduction is rows [q*2^lpS, (q+1)*2^lpS); chunk n_full is the tail
__global__ __launch_bounds__(256)
void channel_aten_chunks_kernel(const float* __restrict__ acc, int B, int S, int C, int lpS, int lpB,
                                float* __restrict__ chunks) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    const int q = blockIdx.y;
    const int64_t step = (int64_t)1 << lpS;
    const int64_t r0 = (int64_t)q * step;
    const int64_t r1 = r0 + step < S ? r0 + step : S;
    const int64_t bs = (int64_t)S * C;
    float sum = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
        const float v = cascade_sum_strided(acc + r * C + c, bs, B, lpB, true);   // torch.sum(act.abs(), 0)
        sum = __fadd_rn(sum, v);                           // .abs() of a non-negative sum: the same value
    }
    chunks[(int64_t)q * C + c] = sum;
}

// pass 2: the level replay over the chunks, then the mean's division by S
__global__ __launch_bounds__(256)
void channel_aten_levels_kernel(const float* __restrict__ chunks, int S, int C, int lpS, float* __restrict__ out) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    if (c >= C) return;
    const int64_t step = (int64_t)1 << lpS;
    const int64_t mask = step - 1;
    const int64_t n_full = S / step;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    int64_t i = 0;
    for (int64_t q = 0; q < n_full; ++q) {
        i += step;
        acc[0] = chunks[q * C + c];                        // the chunk summed from 0.0f into level 0
        for (int j = 1; j < 4; ++j) {
            acc[j] = __fadd_rn(acc[j], acc[j - 1]);
            acc[j - 1] = 0.f;
            if ((i & (mask << (j * lpS))) != 0) break;
        }
    }
    if (S % step) acc[0] = chunks[n_full * C + c];         // the tail rows, from 0.0f
    for (int j = 1; j < 4; ++j) acc[0] = __fadd_rn(acc[0], acc[j]);
    out[c] = __fdiv_rn(acc[0], (float)S);                  // sum(...).div_(S)
}

// S splits of `chunk` rows each; seq > 0: the reference-rounding split (kps pieces per seq-row sample)
struct WgradSplit { int S; int64_t chunk; bool quarter; int64_t seq; int kps; };

// Quarter-tile kernel for modules with at most this many tiles. Measured at T = 32768
// (profiles/r02_wgrad_quarter.jsonl): 1.1-1.2x faster than the full-tile kernel at 1-8 tiles, even
// at 16, slower from 27.
constexpr int kQuarterMaxTiles = 8;
int quarter_max_tiles() { return kQuarterMaxTiles; }

// row_bytes: operand bytes per T row of one tile (1 KiB bf16, 512 B MX-fp8)
WgradSplit wgrad_split(int64_t T, int32_t n_tiles, bool allow_quarter = true, double row_bytes = 1024.0) {
    WgradSplit sp{1, kBK, false, 0, 0};
    if (T <= 0 || n_tiles <= 0) return sp;
    const int64_t s_max = std::max<int64_t>(1, std::min<int64_t>(64, (T + 511) / 512));
    int64_t S = 1;
    if (allow_quarter && n_tiles <= quarter_max_tiles()) {
        // quarter tiles, two workgroups per CU: fill the 512 workgroup slots once, never more (a
        // 513th workgroup is a second round: n = 6 with ceil(512/24) = 22 ran 57 us, floor = 21 fits)
        sp.quarter = true;
        S = std::min<int64_t>(s_max, std::max<int64_t>(1, (2 * kCUs) / (4 * n_tiles)));
    } else {
        // Time model (measured rates): a workgroup streams its 1 KiB/row of g+x slices at ~25 GB/s per
        // CU and, when S > 1, writes a 256 KiB fp32 slab; the reduce re-reads the n*S slabs (~5 TB/s).
        double best = 1e30;
        for (int64_t cand = 1; cand <= s_max; ++cand) {
            const int64_t rounds = (n_tiles * cand + kCUs - 1) / kCUs;
            const double rows = std::ceil((double)T / (double)cand);
            const double slab = cand > 1 ? 262144.0 : 0.0;
            const double t_wg = (rows * row_bytes + slab) / 25e9;
            const double t_red = cand > 1 ? (double)n_tiles * cand * 262144.0 * 2.0 / 5e12 : 0.0;
            const double cost = (double)rounds * t_wg + t_red;
            if (cost < best * (1.0 - 1e-6)) { best = cost; S = cand; }
        }
    }
    int64_t chunk = (T + S - 1) / S;
    chunk = (chunk + kBK - 1) / kBK * kBK;
    sp.S = (int)((T + chunk - 1) / chunk);
    sp.chunk = chunk;
    return sp;
}

// Reference-rounding split (T = n_samples * seq): every sample is cut into kps pieces of `chunk`
// rows (a multiple of 32, the LDS-DMA stage), kps doubled until the launch fills the chip (256
// full-tile or 512 quarter-tile workgroup slots) or a piece would drop below 64 rows. Always the
// slab path (S = n_samples * kps >= 1): the reduce rebuilds and rounds each sample's partial.
WgradSplit wgrad_split_seq(int64_t T, int64_t seq, int32_t n_tiles) {
    WgradSplit sp{1, seq, false, seq, 1};
    if (T <= 0 || n_tiles <= 0 || seq <= 0 || T % seq) return sp;
    const int64_t n_samples = T / seq;
    sp.quarter = n_tiles <= quarter_max_tiles();
    const int64_t slots = sp.quarter ? 2 * kCUs : kCUs;
    const int64_t per_split = sp.quarter ? 4 : 1;
    int64_t k = 1;
    while ((int64_t)n_tiles * n_samples * k * per_split < slots && seq / (2 * k) >= 64) k *= 2;
    int64_t chunk = (seq + k - 1) / k;
    chunk = (chunk + 31) / 32 * 32;
    sp.chunk = chunk;
    sp.kps = (int)((seq + chunk - 1) / chunk);
    sp.S = (int)(n_samples * sp.kps);
    return sp;
}

}  // namespace

// ================================================================================================
// C ABI
// ================================================================================================
// AdamW launches per (grad dtype, parameter dtype), dispatched by smt_adamw_step / _multi below
template <int GDT, int PDT>
static void adamw_launch(bool tiled, int64_t blocks, const void* grad, float* master, float* exp_avg,
                         float* exp_avg_sq, void* param, const smt_tile_desc* tiles_dev, int64_t n_elems,
                         const double* grad_sq_norm_dev, const smt_adamw_args& a, hipStream_t stream) {
    if (tiled)
        hipLaunchKernelGGL((adamw_tiles_kernel<GDT, PDT>), dim3((unsigned)blocks), dim3(256), 0, stream, grad, master,
                           exp_avg, exp_avg_sq, param, tiles_dev, grad_sq_norm_dev, a);
    else
        hipLaunchKernelGGL((adamw_flat_kernel<GDT, PDT>), dim3((unsigned)blocks), dim3(256), 0, stream, grad, master,
                           exp_avg, exp_avg_sq, param, n_elems, grad_sq_norm_dev, a);
}

template <int GDT, int PDT>
static void adamw_multi_launch(int64_t n_blocks, const smt_adamw_tensor* tensors_dev, const int64_t* block_start_dev,
                               int32_t n_tensors, const double* grad_sq_norm_dev, const smt_adamw_args& a,
                               hipStream_t stream) {
    hipLaunchKernelGGL((adamw_multi_kernel<GDT, PDT>), dim3((unsigned)n_blocks), dim3(256), 0, stream, tensors_dev,
                       block_start_dev, n_tensors, grad_sq_norm_dev, a);
}

extern "C" {

const char* smt_last_error(void) { return g_err; }

int smt_abi_version(void) { return 13; }

size_t smt_wgrad_workspace_bytes(int64_t T, int32_t n_tiles) {
    if (T <= 0 || n_tiles <= 0) return 0;
    const WgradSplit sp = wgrad_split(T, n_tiles);
    if (sp.S == 1) return 0;                      // written straight from the accumulators
    return (size_t)n_tiles * (size_t)sp.S * (size_t)kTileElems * sizeof(float);
}

}  // extern "C"

namespace {

// Launch the tile wgrad of `n_tiles` tiles (one module, or a batch) and, when split, its reduce.
// max_ld: the largest leading dimension of any operand (the LDS-DMA kernels' 32-bit buffer offsets
// need chunk * ld * 2 < 2^31, otherwise the register-staged kernel, which addresses with 64 bits).
// FMT: the operands' format (kFmtBF16 / kFmtF16: the 16-bit kernels; kFmtF32: wgrad_f32_kernel, on
// the same split, slabs and reduce, so the workspace sizes do not depend on the format).
template <bool BATCH, int FMT>
int wgrad_launch_fmt(const WgradModules& mods, int64_t T, int64_t max_ld, const int32_t* tab, const int32_t* order,
                     int32_t n_tiles, int32_t out_dtype, void* workspace, size_t workspace_bytes, hipStream_t stream,
                     int64_t seq) {
    const WgradSplit sp = seq > 0 ? wgrad_split_seq(T, seq, n_tiles) : wgrad_split(T, n_tiles);
    const bool use_slab = sp.S > 1 || sp.seq > 0;       // reference rounding always reduces
    const dim3 grid(n_tiles * sp.S), block(kWgThreads);
    const dim3 qgrid(n_tiles * sp.S * 4), qblock(kQThreads);
    // the LDS-DMA kernels address a split's rows with 32-bit buffer offsets; past that, the
    // register-staged kernel (64-bit addresses)
    const bool dma = sp.chunk * max_ld * 2 < (int64_t)0x7fffffff;
    const bool quarter = dma && sp.quarter;
    // reference rounding with one workgroup per sample piece (kps == 1): the LDS-DMA kernels round
    // each sample's partial to the 16-bit operand format themselves and write half-size slabs
    // (SMT_WGRAD_SLAB16=0: fp32)
    static const bool slab16_ok = [] { const char* e = getenv("SMT_WGRAD_SLAB16"); return !(e && atoi(e) == 0); }();
    const bool slab16 = FMT != kFmtF32 && slab16_ok && dma && sp.seq > 0 && sp.kps == 1;
    float* slab = nullptr;
    if (use_slab) {
        const size_t need = (size_t)n_tiles * sp.S * kTileElems * sizeof(float);
        if (!workspace || workspace_bytes < need)
            return fail(SMT_E_WORKSPACE, "smt_tile_wgrad: workspace %zu < %zu bytes", workspace_bytes, need);
        if (!aligned16(workspace)) return fail(SMT_E_ALIGN, "smt_tile_wgrad: workspace not 16-byte aligned");
        slab = static_cast<float*>(workspace);
    }
    if constexpr (FMT == kFmtF32) {
        const dim3 fgrid(n_tiles * sp.S * 4), fblock(kF32Threads);
        if (!use_slab) hipLaunchKernelGGL((wgrad_f32_kernel<kOutF32, BATCH>), fgrid, fblock, 0, stream, mods, T,
                                          sp.chunk, sp.S, sp.seq, sp.kps, n_tiles, tab, order, slab);
        else hipLaunchKernelGGL((wgrad_f32_kernel<kOutSlab, BATCH>), fgrid, fblock, 0, stream, mods, T, sp.chunk,
                                sp.S, sp.seq, sp.kps, n_tiles, tab, order, slab);
        const int rc = check_launch("wgrad_f32_kernel");
        if (rc || !use_slab) return rc;
    } else {
#define SMT_WGRAD_LAUNCH(OUT)                                                                                     \
    do {                                                                                                          \
        if (!dma) hipLaunchKernelGGL((wgrad_partial_kernel<OUT, BATCH, FMT>), grid, block, 0, stream, mods, T,    \
                                     sp.chunk, sp.S, sp.seq, sp.kps, n_tiles, tab, order, slab);                  \
        else if (quarter) hipLaunchKernelGGL((wgrad_quarter_kernel<OUT, kQSlots, BATCH, FMT>), qgrid, qblock, 0,   \
                                     stream, mods, T, sp.chunk, sp.S, sp.seq, sp.kps, n_tiles, tab, order, slab); \
        else hipLaunchKernelGGL((wgrad_dma_kernel<OUT, kDmaSlotsDefault, BATCH, FMT>), grid, block, 0, stream,     \
                                mods, T, sp.chunk, sp.S, sp.seq, sp.kps, n_tiles, tab, order, slab);              \
    } while (0)
        if (!use_slab) {
            if (out_dtype == SMT_DTYPE_FP32) SMT_WGRAD_LAUNCH(kOutF32);
            else SMT_WGRAD_LAUNCH(kOutBF16);
            return check_launch("wgrad kernel");
        }
        if (slab16) {
            // the LDS-DMA kernels only (dma is true here)
            if (quarter) hipLaunchKernelGGL((wgrad_quarter_kernel<kOutSlabBF16, kQSlots, BATCH, FMT>), qgrid, qblock, 0,
                                            stream, mods, T, sp.chunk, sp.S, sp.seq, sp.kps, n_tiles, tab, order, slab);
            else hipLaunchKernelGGL((wgrad_dma_kernel<kOutSlabBF16, kDmaSlotsDefault, BATCH, FMT>), grid, block, 0,
                                    stream, mods, T, sp.chunk, sp.S, sp.seq, sp.kps, n_tiles, tab, order, slab);
        } else {
            SMT_WGRAD_LAUNCH(kOutSlab);
        }
#undef SMT_WGRAD_LAUNCH
        const int rc = check_launch("wgrad kernel");
        if (rc) return rc;
    }
    const dim3 rgrid(n_tiles * 64), rblock(256);
    const int kps = sp.seq > 0 ? sp.kps : 0;
#define SMT_WGRAD_REDUCE(F32, S16)                                                                                 \
    do {                                                                                                          \
        if (BATCH) hipLaunchKernelGGL((wgrad_reduce_batch_kernel<F32, S16, FMT>), rgrid, rblock, 0, stream, slab,  \
                                      sp.S, kps, mods, tab);                                                      \
        else hipLaunchKernelGGL((wgrad_reduce_kernel<F32, S16, FMT>), rgrid, rblock, 0, stream, slab, sp.S, kps,   \
                                mods.m[0].grad_tiles, mods.m[0].accumulate);                                      \
    } while (0)
    if constexpr (FMT == kFmtF32) {
        SMT_WGRAD_REDUCE(true, false);
    } else {
        if (out_dtype == SMT_DTYPE_FP32) {
            if (slab16) SMT_WGRAD_REDUCE(true, true);
            else SMT_WGRAD_REDUCE(true, false);
        } else {
            if (slab16) SMT_WGRAD_REDUCE(false, true);
            else SMT_WGRAD_REDUCE(false, false);
        }
    }
#undef SMT_WGRAD_REDUCE
    return check_launch("wgrad_reduce_kernel");
}

// The operand format from SMT_DTYPE_* (checked by the entry points against out_dtype).
template <bool BATCH>
int wgrad_launch(const WgradModules& mods, int64_t T, int64_t max_ld, const int32_t* tab, const int32_t* order,
                 int32_t n_tiles, int32_t out_dtype, void* workspace, size_t workspace_bytes, hipStream_t stream,
                 int64_t seq = 0, int32_t operand_dtype = SMT_DTYPE_BF16) {
    switch (operand_dtype) {
        case SMT_DTYPE_FP16:
            return wgrad_launch_fmt<BATCH, kFmtF16>(mods, T, max_ld, tab, order, n_tiles, out_dtype, workspace,
                                                    workspace_bytes, stream, seq);
        case SMT_DTYPE_FP32:
            return wgrad_launch_fmt<BATCH, kFmtF32>(mods, T, max_ld, tab, order, n_tiles, out_dtype, workspace,
                                                    workspace_bytes, stream, seq);
        default:
            return wgrad_launch_fmt<BATCH, kFmtBF16>(mods, T, max_ld, tab, order, n_tiles, out_dtype, workspace,
                                                     workspace_bytes, stream, seq);
    }
}

// out_dtype allowed for an operand format: the operand dtype itself (the reference's grad dtype,
// smt.py:382-385) or fp32 (the engine's sink)
bool wgrad_dtypes_ok(int32_t operand_dtype, int32_t out_dtype) {
    if (out_dtype == SMT_DTYPE_FP32) return operand_dtype == SMT_DTYPE_BF16 || operand_dtype == SMT_DTYPE_FP16 ||
                                            operand_dtype == SMT_DTYPE_FP32;
    return (operand_dtype == SMT_DTYPE_BF16 || operand_dtype == SMT_DTYPE_FP16) && out_dtype == operand_dtype;
}

// argument checks shared by the single-module and batched entry points
int check_wgrad_module(const char* fn, const smt_wgrad_module& m) {
    if (!m.grad_out || !m.x || !m.grad_tiles) return fail(SMT_E_INVALID, "%s: null operand or output", fn);
    if (!aligned16(m.grad_out) || !aligned16(m.x) || (m.ld_grad_out & 7) || (m.ld_x & 7) || !aligned16(m.grad_tiles))
        return fail(SMT_E_ALIGN, "%s: operands need 16-byte aligned rows (ld %% 8 == 0) and a 16-byte aligned output", fn);
    if (m.ld_grad_out < kTile || m.ld_x < kTile)
        return fail(SMT_E_INVALID, "%s: leading dimensions %lld / %lld below 256", fn, (long long)m.ld_grad_out,
                    (long long)m.ld_x);
    if (m.x_block_stride < kTile || (m.x_block_stride & 7))
        return fail(SMT_E_INVALID, "%s: x_block_stride %lld (>= 256, %% 8 == 0)", fn, (long long)m.x_block_stride);
    return SMT_OK;
}

}  // namespace

extern "C" {

int smt_tile_wgrad(const void* grad_out, int64_t ld_grad_out, const void* x, int64_t ld_x, int64_t x_block_stride, int64_t T,
                   const int32_t* tile_rc_dev, const int32_t* order_dev, int32_t n_tiles, void* grad_tiles,
                   int32_t out_dtype, int32_t accumulate, void* workspace, size_t workspace_bytes, hipStream_t stream) {
    if (n_tiles < 0 || T < 0) return fail(SMT_E_INVALID, "smt_tile_wgrad: negative size (T=%lld, n_tiles=%d)", (long long)T, n_tiles);
    if (n_tiles == 0) return SMT_OK;
    if (out_dtype != SMT_DTYPE_BF16 && out_dtype != SMT_DTYPE_FP32)
        return fail(SMT_E_INVALID, "smt_tile_wgrad: out_dtype %d not supported", out_dtype);
    if (!tile_rc_dev || !grad_tiles) return fail(SMT_E_INVALID, "smt_tile_wgrad: null tile table or output");
    if (!aligned16(grad_tiles)) return fail(SMT_E_ALIGN, "smt_tile_wgrad: output not 16-byte aligned");
    if (T == 0) {
        if (accumulate) return SMT_OK;
        const size_t bytes = (size_t)n_tiles * kTileElems * (out_dtype == SMT_DTYPE_FP32 ? 4 : 2);
        hipError_t e = hipMemsetAsync(grad_tiles, 0, bytes, stream);
        return e == hipSuccess ? SMT_OK : fail(SMT_E_LAUNCH, "smt_tile_wgrad: memset: %s", hipGetErrorString(e));
    }
    if (!grad_out || !x) return fail(SMT_E_INVALID, "smt_tile_wgrad: null operand");
    if (!aligned16(grad_out) || !aligned16(x) || (ld_grad_out & 7) || (ld_x & 7))
        return fail(SMT_E_ALIGN, "smt_tile_wgrad: operands need 16-byte aligned rows (ld %% 8 == 0)");
    if (x_block_stride < kTile || (x_block_stride & 7))
        return fail(SMT_E_INVALID, "smt_tile_wgrad: x_block_stride %lld (>= 256, %% 8 == 0)", (long long)x_block_stride);
    WgradModules mods{};
    mods.m[0] = smt_wgrad_module{grad_out, x, ld_grad_out, ld_x, x_block_stride, grad_tiles, accumulate ? 1 : 0, 0};
    const int64_t max_ld = ld_grad_out > ld_x ? ld_grad_out : ld_x;
    return wgrad_launch<false>(mods, T, max_ld, tile_rc_dev, order_dev, n_tiles, out_dtype, workspace, workspace_bytes, stream);
}

size_t smt_wgrad_batch_workspace_bytes(int64_t T, int32_t n_tiles) { return smt_wgrad_workspace_bytes(T, n_tiles); }

}  // extern "C"

namespace {

int wgrad_batch_entry(const char* fn, const smt_wgrad_module* modules, int32_t n_modules, int64_t T, int64_t seq,
                      const int32_t* tile_tab_dev, const int32_t* order_dev, int32_t n_tiles, int32_t out_dtype,
                      void* workspace, size_t workspace_bytes, hipStream_t stream) {
    if (n_tiles < 0 || T < 0 || n_modules < 0)
        return fail(SMT_E_INVALID, "%s: negative size (T=%lld, n_tiles=%d, n_modules=%d)", fn, (long long)T, n_tiles, n_modules);
    if (n_tiles == 0) return SMT_OK;
    if (n_modules == 0 || n_modules > SMT_WGRAD_MAX_MODULES || !modules)
        return fail(SMT_E_INVALID, "%s: %d modules (1..%d)", fn, n_modules, SMT_WGRAD_MAX_MODULES);
    const int32_t operand_dtype = modules[0].operand_dtype;
    if (!wgrad_dtypes_ok(operand_dtype, out_dtype))
        return fail(SMT_E_INVALID, "%s: operand dtype %d with out_dtype %d not supported", fn, operand_dtype, out_dtype);
    if (!tile_tab_dev) return fail(SMT_E_INVALID, "%s: null tile table", fn);
    if (T == 0) return fail(SMT_E_INVALID, "%s: T = 0 (use smt_tile_wgrad per module)", fn);
    if (seq < 0 || (seq > 0 && T % seq))
        return fail(SMT_E_INVALID, "%s: T = %lld is not a whole number of %lld-row samples", fn, (long long)T,
                    (long long)seq);
    WgradModules mods{};
    int64_t max_ld = 0;
    for (int i = 0; i < n_modules; ++i) {
        const int rc = check_wgrad_module(fn, modules[i]);
        if (rc) return rc;
        if (modules[i].operand_dtype != operand_dtype)
            return fail(SMT_E_INVALID, "%s: modules of one launch need one operand dtype (%d, %d)", fn,
                        modules[i].operand_dtype, operand_dtype);
        mods.m[i] = modules[i];
        mods.m[i].accumulate = modules[i].accumulate ? 1 : 0;
        max_ld = std::max(max_ld, std::max(modules[i].ld_grad_out, modules[i].ld_x));
    }
    return wgrad_launch<true>(mods, T, max_ld, tile_tab_dev, order_dev, n_tiles, out_dtype, workspace, workspace_bytes,
                              stream, seq, operand_dtype);
}

}  // namespace

extern "C" {

int smt_tile_wgrad_batch(const smt_wgrad_module* modules, int32_t n_modules, int64_t T, const int32_t* tile_tab_dev,
                         const int32_t* order_dev, int32_t n_tiles, int32_t out_dtype, void* workspace,
                         size_t workspace_bytes, hipStream_t stream) {
    return wgrad_batch_entry("smt_tile_wgrad_batch", modules, n_modules, T, 0, tile_tab_dev, order_dev, n_tiles,
                             out_dtype, workspace, workspace_bytes, stream);
}

size_t smt_wgrad_seq_workspace_bytes(int64_t T, int64_t seq_len, int32_t n_tiles) {
    if (T <= 0 || n_tiles <= 0 || seq_len <= 0 || T % seq_len) return 0;
    const WgradSplit sp = wgrad_split_seq(T, seq_len, n_tiles);
    return (size_t)n_tiles * (size_t)sp.S * (size_t)kTileElems * sizeof(float);
}

int smt_tile_wgrad_batch_seq(const smt_wgrad_module* modules, int32_t n_modules, int64_t T, int64_t seq_len,
                             const int32_t* tile_tab_dev, const int32_t* order_dev, int32_t n_tiles,
                             int32_t out_dtype, void* workspace, size_t workspace_bytes, hipStream_t stream) {
    if (seq_len <= 0) return fail(SMT_E_INVALID, "smt_tile_wgrad_batch_seq: seq_len %lld <= 0", (long long)seq_len);
    return wgrad_batch_entry("smt_tile_wgrad_batch_seq", modules, n_modules, T, seq_len, tile_tab_dev, order_dev,
                             n_tiles, out_dtype, workspace, workspace_bytes, stream);
}

size_t smt_wgrad_mx_workspace_bytes(int64_t ldq, int32_t n_tiles) {
    if (ldq <= 0 || n_tiles <= 0) return 0;
    const WgradSplit sp = wgrad_split(ldq, n_tiles, true, 512.0);
    if (sp.S == 1) return 0;
    return (size_t)n_tiles * (size_t)sp.S * (size_t)kTileElems * sizeof(float);
}

int smt_mx_quant_cols(const void* x, int64_t ld_x, int64_t T, const int32_t* blocks_dev, int32_t n_blocks,
                      int64_t ldq, void* q, void* scales, hipStream_t stream) {
    if (T < 0 || n_blocks < 0 || ldq < 0) return fail(SMT_E_INVALID, "smt_mx_quant_cols: negative size");
    if (ldq % 64 || ldq < T) return fail(SMT_E_INVALID, "smt_mx_quant_cols: ldq %lld must be a multiple of 64 and >= T %lld",
                                         (long long)ldq, (long long)T);
    if (n_blocks == 0 || ldq == 0) return SMT_OK;
    if (!x || !blocks_dev || !q || !scales) return fail(SMT_E_INVALID, "smt_mx_quant_cols: null pointer");
    if (!aligned16(x) || (ld_x & 7) || !aligned16(q))
        return fail(SMT_E_ALIGN, "smt_mx_quant_cols: 16-byte aligned rows required (ld %% 8 == 0)");
    // 64 rows per workgroup (32 and 128 measured no faster)
    constexpr int rows = 64;
    const int64_t wgs = (ldq + rows - 1) / rows;
    if (wgs > 65535) return fail(SMT_E_INVALID, "smt_mx_quant_cols: T too large");
    hipLaunchKernelGGL(mx_quant_cols_kernel<rows>, dim3(n_blocks, (unsigned)wgs), dim3(256), 0, stream,
                       static_cast<const uint16_t*>(x), ld_x, T, blocks_dev, ldq, static_cast<uint8_t*>(q),
                       static_cast<uint8_t*>(scales));
    return check_launch("mx_quant_cols_kernel");
}

}  // extern "C"

namespace {

template <bool BATCH>
int wgrad_mx_launch(const WgradMxModules& mods, int64_t ldq, const int32_t* tab, const int32_t* order, int32_t n_tiles,
                    int32_t out_dtype, void* workspace, size_t workspace_bytes, hipStream_t stream) {
    const WgradSplit sp = wgrad_split(ldq, n_tiles, true, 512.0);
    const dim3 grid(n_tiles * sp.S), block(kWgThreads);
    const dim3 qgrid(n_tiles * sp.S * 4), qblock(kQThreads);
    float* slab = nullptr;
    if (sp.S > 1) {
        const size_t need = (size_t)n_tiles * sp.S * kTileElems * sizeof(float);
        if (!workspace || workspace_bytes < need)
            return fail(SMT_E_WORKSPACE, "smt_tile_wgrad_mx: workspace %zu < %zu bytes", workspace_bytes, need);
        if (!aligned16(workspace)) return fail(SMT_E_ALIGN, "smt_tile_wgrad_mx: workspace not 16-byte aligned");
        slab = static_cast<float*>(workspace);
    }
#define SMT_WGRAD_MX(OUT)                                                                                       \
    do {                                                                                                        \
        if (sp.quarter) hipLaunchKernelGGL((wgrad_mx_quarter_kernel<OUT, BATCH>), qgrid, qblock, 0, stream, mods, ldq, \
                                           sp.chunk, sp.S, n_tiles, tab, order, slab);                          \
        else hipLaunchKernelGGL((wgrad_mx_kernel<OUT, BATCH>), grid, block, 0, stream, mods, ldq, sp.chunk, sp.S,     \
                                n_tiles, tab, order, slab);                                                     \
    } while (0)
    if (sp.S == 1) {
        if (out_dtype == SMT_DTYPE_FP32) SMT_WGRAD_MX(kOutF32);
        else SMT_WGRAD_MX(kOutBF16);
        return check_launch("wgrad_mx_kernel");
    }
    SMT_WGRAD_MX(kOutSlab);
#undef SMT_WGRAD_MX
    int rc = check_launch("wgrad_mx_kernel");
    if (rc) return rc;
    const dim3 rgrid(n_tiles * 64), rblock(256);
    if (BATCH) {
        if (out_dtype == SMT_DTYPE_FP32)
            hipLaunchKernelGGL(wgrad_reduce_mx_batch_kernel<true>, rgrid, rblock, 0, stream, slab, sp.S, mods, tab);
        else
            hipLaunchKernelGGL(wgrad_reduce_mx_batch_kernel<false>, rgrid, rblock, 0, stream, slab, sp.S, mods, tab);
    } else {
        const smt_wgrad_mx_module& m = mods.m[0];
        if (out_dtype == SMT_DTYPE_FP32)
            hipLaunchKernelGGL(wgrad_reduce_kernel<true>, rgrid, rblock, 0, stream, slab, sp.S, 0, m.grad_tiles, m.accumulate);
        else
            hipLaunchKernelGGL(wgrad_reduce_kernel<false>, rgrid, rblock, 0, stream, slab, sp.S, 0, m.grad_tiles, m.accumulate);
    }
    return check_launch("wgrad_reduce_kernel");
}

int check_mx_module(const char* fn, const smt_wgrad_mx_module& m) {
    if (!m.qg || !m.sg || !m.qx || !m.sx || !m.grad_tiles) return fail(SMT_E_INVALID, "%s: null operand or output", fn);
    if (!aligned16(m.qg) || !aligned16(m.qx) || !aligned16(m.sg) || !aligned16(m.sx) || !aligned16(m.grad_tiles))
        return fail(SMT_E_ALIGN, "%s: operands / output not 16-byte aligned", fn);
    return SMT_OK;
}

}  // namespace

extern "C" {

int smt_tile_wgrad_mx(const void* qg, const void* sg, const void* qx, const void* sx, int64_t ldq,
                      const int32_t* tile_rc_dev, const int32_t* order_dev, int32_t n_tiles, void* grad_tiles,
                      int32_t out_dtype, int32_t accumulate, void* workspace, size_t workspace_bytes,
                      hipStream_t stream) {
    if (n_tiles < 0 || ldq < 0) return fail(SMT_E_INVALID, "smt_tile_wgrad_mx: negative size");
    if (n_tiles == 0) return SMT_OK;
    if (ldq % 64) return fail(SMT_E_INVALID, "smt_tile_wgrad_mx: ldq %lld not a multiple of 64", (long long)ldq);
    if (out_dtype != SMT_DTYPE_BF16 && out_dtype != SMT_DTYPE_FP32)
        return fail(SMT_E_INVALID, "smt_tile_wgrad_mx: out_dtype %d not supported", out_dtype);
    if (!tile_rc_dev || !grad_tiles) return fail(SMT_E_INVALID, "smt_tile_wgrad_mx: null tile table or output");
    if (!aligned16(grad_tiles)) return fail(SMT_E_ALIGN, "smt_tile_wgrad_mx: output not 16-byte aligned");
    if (ldq == 0) {
        if (accumulate) return SMT_OK;
        const size_t bytes = (size_t)n_tiles * kTileElems * (out_dtype == SMT_DTYPE_FP32 ? 4 : 2);
        hipError_t e = hipMemsetAsync(grad_tiles, 0, bytes, stream);
        return e == hipSuccess ? SMT_OK : fail(SMT_E_LAUNCH, "smt_tile_wgrad_mx: memset: %s", hipGetErrorString(e));
    }
    if (!qg || !sg || !qx || !sx) return fail(SMT_E_INVALID, "smt_tile_wgrad_mx: null operand");
    if (!aligned16(qg) || !aligned16(qx) || !aligned16(sg) || !aligned16(sx))
        return fail(SMT_E_ALIGN, "smt_tile_wgrad_mx: operands not 16-byte aligned");
    if ((int64_t)kTile * ldq >= (int64_t)0x7fffffff) return fail(SMT_E_INVALID, "smt_tile_wgrad_mx: T too large for 32-bit offsets");
    WgradMxModules mods{};
    mods.m[0] = smt_wgrad_mx_module{qg, sg, qx, sx, grad_tiles, accumulate ? 1 : 0, 0};
    return wgrad_mx_launch<false>(mods, ldq, tile_rc_dev, order_dev, n_tiles, out_dtype, workspace, workspace_bytes, stream);
}

int smt_tile_wgrad_mx_batch(const smt_wgrad_mx_module* modules, int32_t n_modules, int64_t ldq,
                            const int32_t* tile_tab_dev, const int32_t* order_dev, int32_t n_tiles,
                            int32_t out_dtype, void* workspace, size_t workspace_bytes, hipStream_t stream) {
    static const char* fn = "smt_tile_wgrad_mx_batch";
    if (n_tiles < 0 || ldq < 0 || n_modules < 0) return fail(SMT_E_INVALID, "%s: negative size", fn);
    if (n_tiles == 0) return SMT_OK;
    if (n_modules == 0 || n_modules > SMT_WGRAD_MAX_MODULES || !modules)
        return fail(SMT_E_INVALID, "%s: %d modules (1..%d)", fn, n_modules, SMT_WGRAD_MAX_MODULES);
    if (ldq <= 0 || ldq % 64) return fail(SMT_E_INVALID, "%s: ldq %lld (a positive multiple of 64)", fn, (long long)ldq);
    if ((int64_t)kTile * ldq >= (int64_t)0x7fffffff) return fail(SMT_E_INVALID, "%s: T too large for 32-bit offsets", fn);
    if (out_dtype != SMT_DTYPE_BF16 && out_dtype != SMT_DTYPE_FP32)
        return fail(SMT_E_INVALID, "%s: out_dtype %d not supported", fn, out_dtype);
    if (!tile_tab_dev) return fail(SMT_E_INVALID, "%s: null tile table", fn);
    WgradMxModules mods{};
    for (int i = 0; i < n_modules; ++i) {
        const int rc = check_mx_module(fn, modules[i]);
        if (rc) return rc;
        mods.m[i] = modules[i];
        mods.m[i].accumulate = modules[i].accumulate ? 1 : 0;
    }
    return wgrad_mx_launch<true>(mods, ldq, tile_tab_dev, order_dev, n_tiles, out_dtype, workspace, workspace_bytes, stream);
}

static int tile_copy(bool scatter, void* weight, int64_t ld_weight, int32_t elem_bytes, const int32_t* tile_rc_dev,
                     int32_t n_tiles, void* tiles, hipStream_t stream) {
    const char* name = scatter ? "smt_tile_scatter" : "smt_tile_gather";
    if (n_tiles < 0) return fail(SMT_E_INVALID, "%s: negative n_tiles", name);
    if (n_tiles == 0) return SMT_OK;
    if (!weight || !tile_rc_dev || !tiles) return fail(SMT_E_INVALID, "%s: null pointer", name);
    if (elem_bytes != 2 && elem_bytes != 4) return fail(SMT_E_INVALID, "%s: elem_bytes %d", name, elem_bytes);
    if (!aligned16(weight) || !aligned16(tiles) || ((ld_weight * elem_bytes) & 15))
        return fail(SMT_E_ALIGN, "%s: weight/tiles need 16-byte aligned rows", name);
    uint8_t* w = static_cast<uint8_t*>(weight);
    uint8_t* t = static_cast<uint8_t*>(tiles);
    const int wg_per_tile = kTileElems * elem_bytes / 16 / 256;
    dim3 grid(n_tiles * wg_per_tile);
    if (elem_bytes == 2) {
        if (scatter) hipLaunchKernelGGL((tile_copy_kernel<true, 2>), grid, dim3(256), 0, stream, w, ld_weight, tile_rc_dev, t);
        else hipLaunchKernelGGL((tile_copy_kernel<false, 2>), grid, dim3(256), 0, stream, w, ld_weight, tile_rc_dev, t);
    } else {
        if (scatter) hipLaunchKernelGGL((tile_copy_kernel<true, 4>), grid, dim3(256), 0, stream, w, ld_weight, tile_rc_dev, t);
        else hipLaunchKernelGGL((tile_copy_kernel<false, 4>), grid, dim3(256), 0, stream, w, ld_weight, tile_rc_dev, t);
    }
    return check_launch(name);
}

int smt_tile_gather(const void* weight, int64_t ld_weight, int32_t elem_bytes, const int32_t* tile_rc_dev,
                    int32_t n_tiles, void* tiles, hipStream_t stream) {
    return tile_copy(false, const_cast<void*>(weight), ld_weight, elem_bytes, tile_rc_dev, n_tiles, tiles, stream);
}

int smt_tile_scatter(void* weight, int64_t ld_weight, int32_t elem_bytes, const int32_t* tile_rc_dev,
                     int32_t n_tiles, const void* tiles, hipStream_t stream) {
    return tile_copy(true, weight, ld_weight, elem_bytes, tile_rc_dev, n_tiles, const_cast<void*>(tiles), stream);
}

int smt_grad_accumulate(const smt_accum_entry* entries_dev, int32_t n_entries, int64_t total_chunks, hipStream_t stream) {
    if (n_entries < 0 || total_chunks < 0) return fail(SMT_E_INVALID, "smt_grad_accumulate: negative size");
    if (n_entries == 0 || total_chunks == 0) return SMT_OK;
    if (!entries_dev) return fail(SMT_E_INVALID, "smt_grad_accumulate: null entry table");
    if (total_chunks > 0x7fffffffLL) return fail(SMT_E_INVALID, "smt_grad_accumulate: too many chunks");
    hipLaunchKernelGGL(grad_accumulate_kernel, dim3((unsigned)total_chunks), dim3(256), 0, stream, entries_dev, n_entries);
    return check_launch("grad_accumulate_kernel");
}

int smt_block_score(const smt_score_entry* entries_dev, int32_t n_entries, int64_t total_blocks, hipStream_t stream) {
    if (n_entries < 0 || total_blocks < 0) return fail(SMT_E_INVALID, "smt_block_score: negative size");
    if (n_entries == 0 || total_blocks == 0) return SMT_OK;
    if (!entries_dev) return fail(SMT_E_INVALID, "smt_block_score: null entry table");
    if (total_blocks > 0x7fffffffLL) return fail(SMT_E_INVALID, "smt_block_score: too many blocks");
    hipLaunchKernelGGL(block_score_kernel, dim3((unsigned)total_blocks), dim3(256), 0, stream, entries_dev, n_entries);
    return check_launch("block_score_kernel");
}

int smt_sq_norm(const float* x, int64_t n, double* partials_dev, int32_t n_partials, double* out_dev, hipStream_t stream) {
    if (n < 0 || n_partials <= 0) return fail(SMT_E_INVALID, "smt_sq_norm: bad sizes (n=%lld, n_partials=%d)", (long long)n, n_partials);
    if (!partials_dev || !out_dev || (n > 0 && !x)) return fail(SMT_E_INVALID, "smt_sq_norm: null pointer");
    hipLaunchKernelGGL(sq_norm_partial_kernel, dim3(n_partials), dim3(256), 0, stream, x, n, partials_dev);
    int rc = check_launch("sq_norm_partial_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(sq_norm_final_kernel, dim3(1), dim3(256), 0, stream, partials_dev, n_partials, out_dev);
    return check_launch("sq_norm_final_kernel");
}

// (grad dtype, parameter dtype) pairs of the AdamW kernels: bf16 / fp16 gradients of a parameter of
// the same dtype, or fp32 gradients (the engine's packed tile buffer) of any parameter dtype
static bool adamw_dtypes_ok(int gdt, int pdt) {
    const bool p_ok = pdt == SMT_DTYPE_BF16 || pdt == SMT_DTYPE_FP16 || pdt == SMT_DTYPE_FP32;
    return p_ok && (gdt == SMT_DTYPE_FP32 || ((gdt == SMT_DTYPE_BF16 || gdt == SMT_DTYPE_FP16) && gdt == pdt));
}

static int adamw_args_ok(const char* fn, const smt_adamw_args* args) {
    if (!args) return fail(SMT_E_INVALID, "%s: null args", fn);
    if (!adamw_dtypes_ok(args->grad_dtype, args->param_dtype))
        return fail(SMT_E_INVALID, "%s: grad_dtype %d with param_dtype %d not supported", fn, args->grad_dtype,
                    args->param_dtype);
    if (args->mode != SMT_ADAM_DEEPSPEED && args->mode != SMT_ADAM_TORCH)
        return fail(SMT_E_INVALID, "%s: mode %d", fn, args->mode);
    if (!(args->bias_correction1 > 0.f) || !(args->bias_correction2 > 0.f))
        return fail(SMT_E_INVALID, "%s: bias corrections must be > 0", fn);
    return SMT_OK;
}

// F(GDT, PDT) for the runtime pair (adamw_dtypes_ok checked)
#define SMT_ADAMW_DISPATCH(gdt, pdt, F)                                                                      \
    do {                                                                                                    \
        if ((gdt) == SMT_DTYPE_FP32) {                                                                       \
            if ((pdt) == SMT_DTYPE_FP32) F(SMT_DTYPE_FP32, SMT_DTYPE_FP32);                                   \
            else if ((pdt) == SMT_DTYPE_FP16) F(SMT_DTYPE_FP32, SMT_DTYPE_FP16);                              \
            else F(SMT_DTYPE_FP32, SMT_DTYPE_BF16);                                                          \
        } else if ((gdt) == SMT_DTYPE_FP16) {                                                                \
            F(SMT_DTYPE_FP16, SMT_DTYPE_FP16);                                                               \
        } else {                                                                                            \
            F(SMT_DTYPE_BF16, SMT_DTYPE_BF16);                                                               \
        }                                                                                                   \
    } while (0)

int smt_adamw_step(const void* grad, float* master, float* exp_avg, float* exp_avg_sq, void* param,
                   const smt_tile_desc* tiles_dev, int32_t n_tiles, int64_t n_elems, const double* grad_sq_norm_dev,
                   const smt_adamw_args* args, hipStream_t stream) {
    if (int rc = adamw_args_ok("smt_adamw_step", args)) return rc;
    const bool tiled = tiles_dev != nullptr;
    if (tiled ? n_tiles < 0 : n_elems < 0) return fail(SMT_E_INVALID, "smt_adamw_step: negative size");
    if ((tiled && n_tiles == 0) || (!tiled && n_elems == 0)) return SMT_OK;
    if (!grad || !master || !exp_avg || !exp_avg_sq || !param) return fail(SMT_E_INVALID, "smt_adamw_step: null buffer");
    if (!aligned16(grad) || !aligned16(master) || !aligned16(exp_avg) || !aligned16(exp_avg_sq) || !aligned16(param))
        return fail(SMT_E_ALIGN, "smt_adamw_step: buffers must be 16-byte aligned");
    const smt_adamw_args a = *args;
    const int64_t blocks = tiled ? (int64_t)n_tiles * 32 : (n_elems + 2047) / 2048;
    if (blocks > 0x7fffffffLL) return fail(SMT_E_INVALID, "smt_adamw_step: too many elements");
#define SMT_ADAMW_STEP(G, P) \
    adamw_launch<G, P>(tiled, blocks, grad, master, exp_avg, exp_avg_sq, param, tiles_dev, n_elems, grad_sq_norm_dev, a, stream)
    SMT_ADAMW_DISPATCH(a.grad_dtype, a.param_dtype, SMT_ADAMW_STEP);
#undef SMT_ADAMW_STEP
    return check_launch(tiled ? "adamw_tiles_kernel" : "adamw_flat_kernel");
}

int smt_adamw_multi(const smt_adamw_tensor* tensors_dev, const int64_t* block_start_dev, int32_t n_tensors,
                    int64_t n_blocks, const double* grad_sq_norm_dev, const smt_adamw_args* args, hipStream_t stream) {
    if (int rc = adamw_args_ok("smt_adamw_multi", args)) return rc;
    if (n_tensors < 0 || n_blocks < 0) return fail(SMT_E_INVALID, "smt_adamw_multi: negative size");
    if (n_tensors == 0 || n_blocks == 0) return SMT_OK;
    if (!tensors_dev || !block_start_dev) return fail(SMT_E_INVALID, "smt_adamw_multi: null table");
    if (n_blocks > 0x7fffffffLL) return fail(SMT_E_INVALID, "smt_adamw_multi: too many elements");
    const smt_adamw_args a = *args;
#define SMT_ADAMW_MULTI(G, P) \
    adamw_multi_launch<G, P>(n_blocks, tensors_dev, block_start_dev, n_tensors, grad_sq_norm_dev, a, stream)
    SMT_ADAMW_DISPATCH(a.grad_dtype, a.param_dtype, SMT_ADAMW_MULTI);
#undef SMT_ADAMW_MULTI
    return check_launch("adamw_multi_kernel");
}

static int row_copy(bool scatter, void* weight, int64_t ld_weight, int32_t elem_bytes, int64_t n_cols,
                    const int32_t* rows_dev, int32_t n_rows, void* rows, int64_t ld_rows, hipStream_t stream) {
    const char* name = scatter ? "smt_row_scatter" : "smt_row_gather";
    if (n_rows < 0 || n_cols < 0) return fail(SMT_E_INVALID, "%s: negative size", name);
    if (n_rows == 0 || n_cols == 0) return SMT_OK;
    if (!weight || !rows_dev || !rows) return fail(SMT_E_INVALID, "%s: null pointer", name);
    if (elem_bytes != 2 && elem_bytes != 4) return fail(SMT_E_INVALID, "%s: elem_bytes %d", name, elem_bytes);
    if (ld_weight < n_cols || ld_rows < n_cols) return fail(SMT_E_INVALID, "%s: leading dimension < n_cols", name);
    const int64_t row_bytes = n_cols * elem_bytes;
    if (!aligned16(weight) || !aligned16(rows) || ((ld_weight * elem_bytes) & 15) || ((ld_rows * elem_bytes) & 15) ||
        (row_bytes & 15))
        return fail(SMT_E_ALIGN, "%s: rows must be 16-byte aligned and a multiple of 16 bytes", name);
    const int64_t slices = (row_bytes + kRowSliceBytes - 1) / kRowSliceBytes;
    const int64_t blocks = slices * n_rows;
    if (blocks > 0x7fffffffLL) return fail(SMT_E_INVALID, "%s: too many rows", name);
    uint8_t* w = static_cast<uint8_t*>(weight);
    uint8_t* b = static_cast<uint8_t*>(rows);
    if (scatter)
        hipLaunchKernelGGL(row_copy_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, stream, w, ld_weight * elem_bytes,
                           rows_dev, b, ld_rows * elem_bytes, row_bytes, (int32_t)slices);
    else
        hipLaunchKernelGGL(row_copy_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, stream, w, ld_weight * elem_bytes,
                           rows_dev, b, ld_rows * elem_bytes, row_bytes, (int32_t)slices);
    return check_launch(name);
}

int smt_row_gather(const void* weight, int64_t ld_weight, int32_t elem_bytes, int64_t n_cols,
                   const int32_t* rows_dev, int32_t n_rows, void* rows, int64_t ld_rows, hipStream_t stream) {
    return row_copy(false, const_cast<void*>(weight), ld_weight, elem_bytes, n_cols, rows_dev, n_rows, rows, ld_rows, stream);
}

int smt_row_scatter(void* weight, int64_t ld_weight, int32_t elem_bytes, int64_t n_cols,
                    const int32_t* rows_dev, int32_t n_rows, const void* rows, int64_t ld_rows, hipStream_t stream) {
    return row_copy(true, weight, ld_weight, elem_bytes, n_cols, rows_dev, n_rows, const_cast<void*>(rows), ld_rows, stream);
}

int smt_column_gather(const void* x, int64_t ld_x, int64_t n_in, int64_t T, const int32_t* cols_dev, int32_t n_cols,
                      void* out, int64_t ld_out, hipStream_t stream) {
    if (T < 0 || n_cols < 0 || ld_out < n_cols || n_in < 0) return fail(SMT_E_INVALID, "smt_column_gather: bad sizes");
    if (T == 0 || ld_out == 0) return SMT_OK;
    if (!x || !out || (n_cols > 0 && !cols_dev)) return fail(SMT_E_INVALID, "smt_column_gather: null pointer");
    if (!aligned16(out) || (ld_out & 7)) return fail(SMT_E_ALIGN, "smt_column_gather: out rows must be 16-byte aligned (ld_out %% 8 == 0)");
    if (!aligned16(x) || (ld_x & 7) || n_in > ld_x)
        return fail(SMT_E_ALIGN, "smt_column_gather: x rows must be 16-byte aligned (ld_x %% 8 == 0) and n_in <= ld_x");
    // rows staged per workgroup: up to 4, within a 64 KiB LDS stage
    const int64_t row_bytes = ((n_in + 7) & ~(int64_t)7) * 2;
    const int rows = row_bytes * 4 <= 65536 ? 4 : row_bytes * 2 <= 65536 ? 2 : 1;
    if (row_bytes > 65536) return fail(SMT_E_INVALID, "smt_column_gather: rows of %lld elements exceed the LDS stage", (long long)n_in);
    if (n_cols > 0 && ((uintptr_t)cols_dev & 15)) return fail(SMT_E_ALIGN, "smt_column_gather: cols not 16-byte aligned");
    // LDS-DMA staging of 4 rows per workgroup (profiles/r04_h_column_gather_ab.jsonl: 82 us against 120
    // for register staging and 90 for 8 rows); register staging where the rows do not fit the 64 KiB
    // stage or the 32-bit buffer offsets
    const int64_t ppr = (n_in * 2 + 1023) / 1024;
    if (ppr * 1024 * 4 <= 65536 && ld_x * 2 * 8 < 0x7fffffffLL) {
        constexpr int R = 4;
        const int64_t nb = (T + R - 1) / R;
        if (nb > 0x7fffffffLL) return fail(SMT_E_INVALID, "smt_column_gather: too large");
        const size_t lds = (size_t)(R * ppr * 1024);
        hipLaunchKernelGGL(column_gather_dma_kernel<R>, dim3((unsigned)nb), dim3(256), lds, stream,
                           static_cast<const uint16_t*>(x), ld_x, n_in, T, (int)ppr, cols_dev, n_cols,
                           static_cast<uint16_t*>(out), ld_out);
        return check_launch("column_gather_dma_kernel");
    }
    const int64_t blocks = (T + rows - 1) / rows;
    if (blocks > 0x7fffffffLL) return fail(SMT_E_INVALID, "smt_column_gather: too large");
    hipLaunchKernelGGL(column_gather_kernel, dim3((unsigned)blocks), dim3(256), (size_t)(rows * row_bytes), stream,
                       static_cast<const uint16_t*>(x), ld_x, n_in, T, cols_dev, n_cols, static_cast<uint16_t*>(out), ld_out,
                       rows);
    return check_launch("column_gather_kernel");
}

int smt_tile_scatter_t(const smt_tile_desc* descs_dev, int32_t n_tiles, const void* tiles, hipStream_t stream) {
    if (n_tiles < 0) return fail(SMT_E_INVALID, "smt_tile_scatter_t: negative n_tiles");
    if (n_tiles == 0) return SMT_OK;
    if (!descs_dev || !tiles) return fail(SMT_E_INVALID, "smt_tile_scatter_t: null pointer");
    if (!aligned16(tiles)) return fail(SMT_E_ALIGN, "smt_tile_scatter_t: tiles not 16-byte aligned");
    hipLaunchKernelGGL(tile_scatter_t_kernel, dim3((unsigned)n_tiles * 16u), dim3(256), 0, stream, descs_dev,
                       static_cast<const uint16_t*>(tiles));
    return check_launch("tile_scatter_t_kernel");
}

int smt_colblock_gather(const void* x, int64_t ld_x, int64_t T, const int32_t* col_blocks_dev, int32_t n_cb,
                        void* out, hipStream_t stream) {
    if (T < 0 || n_cb < 0 || ld_x < 0) return fail(SMT_E_INVALID, "smt_colblock_gather: negative size");
    if (T == 0 || n_cb == 0) return SMT_OK;
    if (!x || !out || !col_blocks_dev) return fail(SMT_E_INVALID, "smt_colblock_gather: null pointer");
    if (!aligned16(x) || !aligned16(out) || (ld_x & 7))
        return fail(SMT_E_ALIGN, "smt_colblock_gather: 16-byte aligned rows required (ld_x %% 8 == 0)");
    const int64_t blocks = (T * (int64_t)n_cb * 32 + 255) / 256;
    if (blocks > 0x7fffffffLL) return fail(SMT_E_INVALID, "smt_colblock_gather: too large");
    hipLaunchKernelGGL(colblock_gather_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                       static_cast<const uint16_t*>(x), ld_x, T, col_blocks_dev, n_cb, static_cast<uint16_t*>(out));
    return check_launch("colblock_gather_kernel");
}

int smt_act_accumulate(const void* x, int32_t x_dtype, int64_t ld_x, int64_t batch_stride, int32_t B, int32_t S,
                       int32_t n_cols, float* acc, int32_t assign, hipStream_t stream) {
    if (B < 0 || S < 0 || n_cols < 0) return fail(SMT_E_INVALID, "smt_act_accumulate: negative size");
    if (B == 0 || S == 0 || n_cols == 0) return SMT_OK;
    if (!acc || !x) return fail(SMT_E_INVALID, "smt_act_accumulate: null pointer");
    if (x_dtype != SMT_DTYPE_BF16 && x_dtype != SMT_DTYPE_FP16 && x_dtype != SMT_DTYPE_FP32)
        return fail(SMT_E_INVALID, "smt_act_accumulate: x_dtype %d", x_dtype);
    const int64_t vec = x_dtype == SMT_DTYPE_FP32 ? 4 : 8;
    if ((n_cols & 7) || !aligned16(acc) || !aligned16(x) || (ld_x % vec) || (batch_stride % vec))
        return fail(SMT_E_ALIGN, "smt_act_accumulate: needs n_cols %% 8 == 0 and 16-byte aligned rows");
    const int64_t rows = (int64_t)B * S;
    const int64_t blocks = (rows * (n_cols >> 3) + 255) / 256;
    if (blocks > 0x7fffffffLL) return fail(SMT_E_INVALID, "smt_act_accumulate: too large");
    const dim3 grid((unsigned)blocks), block(256);
    if (x_dtype == SMT_DTYPE_BF16)
        hipLaunchKernelGGL(act_accumulate_kernel<SMT_DTYPE_BF16>, grid, block, 0, stream, x, ld_x, batch_stride, S, n_cols, rows, acc, assign);
    else if (x_dtype == SMT_DTYPE_FP16)
        hipLaunchKernelGGL(act_accumulate_kernel<SMT_DTYPE_FP16>, grid, block, 0, stream, x, ld_x, batch_stride, S, n_cols, rows, acc, assign);
    else
        hipLaunchKernelGGL(act_accumulate_kernel<SMT_DTYPE_FP32>, grid, block, 0, stream, x, ld_x, batch_stride, S, n_cols, rows, acc, assign);
    return check_launch("act_accumulate_kernel");
}

size_t smt_channel_score_workspace_bytes(int32_t S, int32_t n_cols) {
    if (S <= 0 || n_cols <= 0) return 0;
    return (size_t)((S + kChanRows - 1) / kChanRows) * (size_t)n_cols * sizeof(double);
}

int smt_channel_score(const float* acc, int32_t B, int32_t S, int32_t n_cols, int32_t strategy, double* partials,
                      size_t partial_bytes, double* out, hipStream_t stream) {
    if (B < 0 || S < 0 || n_cols < 0) return fail(SMT_E_INVALID, "smt_channel_score: negative size");
    if (strategy < SMT_SCORE_MEAN_ABS || strategy > SMT_SCORE_L2) return fail(SMT_E_INVALID, "smt_channel_score: strategy %d", strategy);
    if (n_cols == 0) return SMT_OK;
    if (!out || (B > 0 && S > 0 && !acc)) return fail(SMT_E_INVALID, "smt_channel_score: null pointer");
    if (S == 0) {
        hipError_t e = hipMemsetAsync(out, 0, (size_t)n_cols * sizeof(double), stream);
        return e == hipSuccess ? SMT_OK : fail(SMT_E_LAUNCH, "smt_channel_score: memset: %s", hipGetErrorString(e));
    }
    const size_t need = smt_channel_score_workspace_bytes(S, n_cols);
    if (!partials || partial_bytes < need)
        return fail(SMT_E_WORKSPACE, "smt_channel_score: workspace %zu < %zu bytes", partial_bytes, need);
    const int P = (S + kChanRows - 1) / kChanRows;
    if (P > 65535) return fail(SMT_E_INVALID, "smt_channel_score: S too large");
    hipLaunchKernelGGL(channel_partial_kernel, dim3((n_cols + 255) / 256, P), dim3(256), 0, stream, acc, B, S, n_cols,
                       (int32_t)(strategy == SMT_SCORE_L2), partials);
    int rc = check_launch("channel_partial_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(channel_final_kernel, dim3((n_cols + 255) / 256), dim3(256), 0, stream, partials, P, n_cols, out);
    return check_launch("channel_final_kernel");
}

size_t smt_channel_mean_aten_workspace_bytes(int32_t S, int32_t n_cols) {
    if (S <= 0 || n_cols <= 0) return 0;
    const int64_t step = (int64_t)1 << cascade_level_power(S);
    return (size_t)(S / step + 1) * (size_t)n_cols * sizeof(float);
}

int smt_channel_mean_aten(const float* acc, int32_t B, int32_t S, int32_t n_cols, float* workspace,
                          size_t workspace_bytes, float* out, hipStream_t stream) {
    static const char* fn = "smt_channel_mean_aten";
    if (B <= 0 || S <= 0 || n_cols <= 0) return fail(SMT_E_INVALID, "%s: sizes must be positive", fn);
    if (!acc || !out || !workspace) return fail(SMT_E_INVALID, "%s: null pointer", fn);
    const size_t need = smt_channel_mean_aten_workspace_bytes(S, n_cols);
    if (workspace_bytes < need) return fail(SMT_E_WORKSPACE, "%s: workspace %zu < %zu bytes", fn, workspace_bytes, need);
    const int lpS = cascade_level_power(S), lpB = cascade_level_power(B);
    const int64_t n_chunks = S / ((int64_t)1 << lpS) + ((S % ((int64_t)1 << lpS)) ? 1 : 0);
    if (n_chunks > 65535) return fail(SMT_E_INVALID, "%s: S too large", fn);
    const dim3 g1((n_cols + 255) / 256, (unsigned)n_chunks), g2((n_cols + 255) / 256);
    hipLaunchKernelGGL(channel_aten_chunks_kernel, g1, dim3(256), 0, stream, acc, B, S, n_cols, lpS, lpB, workspace);
    int rc = check_launch("channel_aten_chunks_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(channel_aten_levels_kernel, g2, dim3(256), 0, stream, workspace, S, n_cols, lpS, out);
    return check_launch("channel_aten_levels_kernel");
}

}  // extern "C"
