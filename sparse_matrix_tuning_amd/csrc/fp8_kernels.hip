// fp8_kernels.hip — gfx950 OCP e4m3 quantisation for the SMT fp8 path (BASELINE config 5,
// SURVEY §8(f) row 2). C ABI: include/smt_fp8.h.
//
// The frozen linear weights of the decoder layers get e4m3 copies with one fp32 scale per row
// (W [out, in], the forward operand) and per column (written transposed as W^T [in, out], the data-
// gradient operand); activations and output gradients are quantised per row (token) before each
// GEMM. hipBLASLt then runs the rowwise-scaled fp8 GEMMs (2.4-2.9 PF/s on the LLaMA-3-8B shapes
// against 1.4-1.6 PF/s bf16, profiles/r01_fp8_probe.jsonl).
//
// scale = amax * fp32(1/448) (1 when amax == 0); q = e4m3_rne(x / scale), IEEE fp32 division and
// v_cvt_pk_fp8_f32 (round to nearest even, OCP e4m3 on gfx950), clamped to +-448 first, so the
// bytes equal torch's (x.float() / scale).to(torch.float8_e4m3fn).

#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>

#include "smt_fp8.h"
#include "silu_math.h"
#include "fp8_math.h"

namespace {

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
    if (e != hipSuccess) return fail(-4, "%s: %s", what, hipGetErrorString(e));
    return 0;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

__device__ __forceinline__ float bf(uint32_t b16) { return __uint_as_float(b16 << 16); }

struct F8 { float v[8]; };

__device__ __forceinline__ F8 unpack8(const uint4 a) {
    F8 r;
    const uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) { r.v[2 * j] = bf(w[j] & 0xffffu); r.v[2 * j + 1] = bf(w[j] >> 16); }
    return r;
}

__device__ __forceinline__ F8 ld8(const uint16_t* p) {
    const uint4 a = *reinterpret_cast<const uint4*>(p);
    F8 r;
    const uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) { r.v[2 * j] = bf(w[j] & 0xffffu); r.v[2 * j + 1] = bf(w[j] >> 16); }
    return r;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
    return v;
}

// One wave per row: pass 1 the row's amax, pass 2 (the row again, L2-served) the conversion.
__global__ __launch_bounds__(256)
void quant_rows_kernel(const uint16_t* __restrict__ x, int64_t ldx, int64_t rows, int cols,
                       const int32_t* __restrict__ row_blocks, int64_t n_sel, uint8_t* __restrict__ out, int64_t ldo,
                       float* __restrict__ scales) {
    const int lane = threadIdx.x & 63;
    const int64_t idx = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (idx >= n_sel) return;
    const int64_t row = row_blocks ? (int64_t)row_blocks[idx >> 8] * 256 + (idx & 255) : idx;
    if (row >= rows) return;
    const uint16_t* xr = x + row * ldx;
    const int nch = cols >> 3;
    float amax = 0.f;
    for (int c = lane; c < nch; c += 64) {
        const F8 v = ld8(xr + c * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(v.v[j]));
    }
    amax = wave_max(amax);
    const float scale = amax > 0.f ? amax * kInvE4M3Max : 1.f;
    if (lane == 0) scales[row] = scale;
    uint8_t* orow = out + row * ldo;
    for (int c = lane; c < nch; c += 64) {
        const F8 v = ld8(xr + c * 8);
        uint2 w;
        w.x = pack4(qv(v.v[0], scale), qv(v.v[1], scale), qv(v.v[2], scale), qv(v.v[3], scale));
        w.y = pack4(qv(v.v[4], scale), qv(v.v[5], scale), qv(v.v[6], scale), qv(v.v[7], scale));
        *reinterpret_cast<uint2*>(orow + c * 8) = w;
    }
}

// Single-pass variant for rows of at most 64 * MAXC * 8 elements: the lane keeps its 16-B chunks of
// the row in registers between the amax reduction and the conversion (one HBM read instead of two).
template <int MAXC>
__global__ __launch_bounds__(256)
void quant_rows_reg_kernel(const uint16_t* __restrict__ x, int64_t ldx, int64_t rows, int cols,
                           const int32_t* __restrict__ row_blocks, int64_t n_sel, uint8_t* __restrict__ out,
                           int64_t ldo, float* __restrict__ scales) {
    const int lane = threadIdx.x & 63;
    const int64_t idx = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (idx >= n_sel) return;
    const int64_t row = row_blocks ? (int64_t)row_blocks[idx >> 8] * 256 + (idx & 255) : idx;
    if (row >= rows) return;
    const uint16_t* xr = x + row * ldx;
    const int nch = cols >> 3;
    uint4 buf[MAXC];
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
        const int c = lane + 64 * i;
        buf[i] = c < nch ? *reinterpret_cast<const uint4*>(xr + c * 8) : make_uint4(0u, 0u, 0u, 0u);
    }
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
        const uint32_t w[4] = {buf[i].x, buf[i].y, buf[i].z, buf[i].w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
            amax = fmaxf(amax, fmaxf(fabsf(bf(w[j] & 0xffffu)), fabsf(bf(w[j] >> 16))));
    }
    amax = wave_max(amax);
    const float scale = amax > 0.f ? amax * kInvE4M3Max : 1.f;
    if (lane == 0) scales[row] = scale;
    uint8_t* orow = out + row * ldo;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
        const int c = lane + 64 * i;
        if (c < nch) {
            const uint32_t w[4] = {buf[i].x, buf[i].y, buf[i].z, buf[i].w};
            uint2 o;
            o.x = pack4(qv(bf(w[0] & 0xffffu), scale), qv(bf(w[0] >> 16), scale),
                        qv(bf(w[1] & 0xffffu), scale), qv(bf(w[1] >> 16), scale));
            o.y = pack4(qv(bf(w[2] & 0xffffu), scale), qv(bf(w[2] >> 16), scale),
                        qv(bf(w[3] & 0xffffu), scale), qv(bf(w[3] >> 16), scale));
            *reinterpret_cast<uint2*>(orow + c * 8) = o;
        }
    }
}

// Wide rows (the 14336-wide MLP activations and gradients): one 256-thread workgroup per row, each
// thread holding CPT 16-B chunks in registers (7 at 14336), the row maximum combined through LDS.
// One wave per row with 28 chunks in flight ran latency-bound at 3.3 TB/s.
template <int CPT>
__global__ __launch_bounds__(256)
void quant_rows_wg_kernel(const uint16_t* __restrict__ x, int64_t ldx, int64_t rows, int cols,
                          const int32_t* __restrict__ row_blocks, int64_t n_sel, uint8_t* __restrict__ out,
                          int64_t ldo, float* __restrict__ scales) {
    __shared__ float wmax[4];
    const int tid = threadIdx.x;
    const int64_t idx = blockIdx.x;
    const int64_t row = row_blocks ? (int64_t)row_blocks[idx >> 8] * 256 + (idx & 255) : idx;
    if (row >= rows) return;                                  // uniform per workgroup
    const uint16_t* xr = x + row * ldx;
    const int nch = cols >> 3;
    uint4 buf[CPT];
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
        const int c = tid + 256 * i;
        buf[i] = c < nch ? *reinterpret_cast<const uint4*>(xr + c * 8) : make_uint4(0u, 0u, 0u, 0u);
    }
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
        const uint32_t w[4] = {buf[i].x, buf[i].y, buf[i].z, buf[i].w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
            amax = fmaxf(amax, fmaxf(fabsf(bf(w[j] & 0xffffu)), fabsf(bf(w[j] >> 16))));
    }
    amax = wave_max(amax);
    if ((tid & 63) == 0) wmax[tid >> 6] = amax;
    __syncthreads();
    amax = fmaxf(fmaxf(wmax[0], wmax[1]), fmaxf(wmax[2], wmax[3]));
    const float scale = amax > 0.f ? amax * kInvE4M3Max : 1.f;
    if (tid == 0) scales[row] = scale;
    uint8_t* orow = out + row * ldo;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
        const int c = tid + 256 * i;
        if (c < nch) {
            const uint32_t w[4] = {buf[i].x, buf[i].y, buf[i].z, buf[i].w};
            uint2 o;
            o.x = pack4(qv(bf(w[0] & 0xffffu), scale), qv(bf(w[0] >> 16), scale),
                        qv(bf(w[1] & 0xffffu), scale), qv(bf(w[1] >> 16), scale));
            o.y = pack4(qv(bf(w[2] & 0xffffu), scale), qv(bf(w[2] >> 16), scale),
                        qv(bf(w[3] & 0xffffu), scale), qv(bf(w[3] >> 16), scale));
            *reinterpret_cast<uint2*>(orow + c * 8) = o;
        }
    }
}

// Row-wise over a concatenation of up to 4 bf16 sources [src0 | src1 | ...] (the output gradients
// of the linears that share one input: q/k/v or gate/up), one scale per row over all of them; the
// fp8 rows are written concatenated, ready for ONE data-gradient GEMM against the jointly quantised
// transposed weights. One NT-thread workgroup per row, CPT chunks of 8 per thread held in registers.
// UNIFORM: every source is a whole number of 64-chunk wave spans (cols % 512 == 0), so the source of
// a wave's chunks is wave-uniform and its pointer / stride come from scalar registers.
struct CatSrcs {
    const uint16_t* p[4];
    int64_t ld[4];
    int off[5];                        // chunk offsets (8 elements per chunk), off[n] = total
    int n;
};

template <int CPT, int NT, bool UNIFORM>
__global__ __launch_bounds__(NT)
void quant_rows_cat_kernel(CatSrcs src, int64_t rows, uint8_t* __restrict__ out, int64_t ldo, float* __restrict__ scales) {
    constexpr int NW = NT / 64;
    __shared__ float wmax[NW];
    const int tid = threadIdx.x;
    const int64_t row = blockIdx.x;
    if (row >= rows) return;
    const int nch = src.off[src.n];
    uint4 buf[CPT];
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
        const int c = tid + NT * i;
        int k = (c >= src.off[1]) + (c >= src.off[2]) + (c >= src.off[3]);
        if (UNIFORM) k = __builtin_amdgcn_readfirstlane(k);
        if (c < nch)
            buf[i] = *reinterpret_cast<const uint4*>(src.p[k] + row * src.ld[k] + (int64_t)(c - src.off[k]) * 8);
        else
            buf[i] = make_uint4(0u, 0u, 0u, 0u);
    }
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
        const uint32_t w[4] = {buf[i].x, buf[i].y, buf[i].z, buf[i].w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
            amax = fmaxf(amax, fmaxf(fabsf(bf(w[j] & 0xffffu)), fabsf(bf(w[j] >> 16))));
    }
    amax = wave_max(amax);
    if ((tid & 63) == 0) wmax[tid >> 6] = amax;
    __syncthreads();
    amax = wmax[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) amax = fmaxf(amax, wmax[w]);
    const float scale = amax > 0.f ? amax * kInvE4M3Max : 1.f;
    if (tid == 0) scales[row] = scale;
    uint8_t* orow = out + row * ldo;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
        const int c = tid + NT * i;
        if (c < nch) {
            const uint32_t w[4] = {buf[i].x, buf[i].y, buf[i].z, buf[i].w};
            uint2 o;
            o.x = pack4(qv(bf(w[0] & 0xffffu), scale), qv(bf(w[0] >> 16), scale),
                        qv(bf(w[1] & 0xffffu), scale), qv(bf(w[1] >> 16), scale));
            o.y = pack4(qv(bf(w[2] & 0xffffu), scale), qv(bf(w[2] >> 16), scale),
                        qv(bf(w[3] & 0xffffu), scale), qv(bf(w[3] >> 16), scale));
            *reinterpret_cast<uint2*>(orow + c * 8) = o;
        }
    }
}

// SwiGLU backward fused with the per-row quantisation of its two outputs for the gate/up group's
// joint data-gradient GEMM (fp8.Fp8Group): per token row, dgate and dup are computed exactly as
// llama_kernels.hip swiglu_bwd_kernel does (same fp32 formula, same bf16 roundings), the row's amax
// is taken over the bf16 values of BOTH, and they are written as one e4m3 row [dgate | dup] with one
// scale -- bit-identical to smt_swiglu_bwd followed by smt_quant_rows_cat_e4m3, without writing
// and re-reading the bf16 gradients (written too only when grad_gate / grad_up are non-null: an SMT
// gate/up module needs them for its tile weight gradient). With a position map (gpos / upos: int32
// per 256-column block, -1 = not written) only the mapped blocks are written, block b at column
// 256 * gpos[b] of a packed [rows, ldg] gradient: the blocks an MX tile gradient reads, and none of
// the rest. One 512-thread workgroup per row.
__device__ __forceinline__ uint32_t tobf16(float f) { return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)f); }
__device__ __forceinline__ float rbf16(float f) { return bf(tobf16(f)); }

template <int CPT>
__global__ __launch_bounds__(512)
void swiglu_bwd_quant_kernel(const uint16_t* __restrict__ g, const uint16_t* __restrict__ u,
                             const uint16_t* __restrict__ dh, int64_t ld, int cols, uint8_t* __restrict__ out,
                             int64_t ldo, float* __restrict__ scales, uint16_t* __restrict__ dg_out,
                             const int32_t* __restrict__ gpos, int64_t ldg, uint16_t* __restrict__ du_out,
                             const int32_t* __restrict__ upos, int64_t ldu) {
    __shared__ float wmax[8];
    const int tid = threadIdx.x;
    const int64_t row = blockIdx.x;
    const int nch = cols >> 3;
    uint4 dgv[CPT], duv[CPT];                           // the row's bf16 dgate / dup, 8 per chunk
    uint4 graw[CPT], uraw[CPT], hraw[CPT];              // every load of the row issued before any math
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
        const int c = tid + 512 * i;
        const int64_t off = row * ld + (int64_t)c * 8;
        const bool in = c < nch;
        graw[i] = in ? *reinterpret_cast<const uint4*>(g + off) : make_uint4(0u, 0u, 0u, 0u);
        uraw[i] = in ? *reinterpret_cast<const uint4*>(u + off) : make_uint4(0u, 0u, 0u, 0u);
        hraw[i] = in ? *reinterpret_cast<const uint4*>(dh + off) : make_uint4(0u, 0u, 0u, 0u);
    }
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
        const int c = tid + 512 * i;
        uint32_t og[4] = {0u, 0u, 0u, 0u}, ou[4] = {0u, 0u, 0u, 0u};
        if (c < nch) {
            const F8 gv = unpack8(graw[i]), uv = unpack8(uraw[i]), hv = unpack8(hraw[i]);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float x = gv.v[j];
                const float sig = smt_sigmoid(x);
                const float sl = rbf16(x * sig);
                const float ds = rbf16(hv.v[j] * uv.v[j]);
                const float vu = rbf16(hv.v[j] * sl);
                const float vg = rbf16(ds * sig * (1.0f + x * (1.0f - sig)));
                amax = fmaxf(amax, fmaxf(fabsf(vg), fabsf(vu)));
                og[j >> 1] |= tobf16(vg) << (16 * (j & 1));
                ou[j >> 1] |= tobf16(vu) << (16 * (j & 1));
            }
        }
        dgv[i] = make_uint4(og[0], og[1], og[2], og[3]);
        duv[i] = make_uint4(ou[0], ou[1], ou[2], ou[3]);
    }
    amax = wave_max(amax);
    if ((tid & 63) == 0) wmax[tid >> 6] = amax;
    __syncthreads();
    amax = wmax[0];
#pragma unroll
    for (int w = 1; w < 8; ++w) amax = fmaxf(amax, wmax[w]);
    const float scale = amax > 0.f ? amax * kInvE4M3Max : 1.f;
    if (tid == 0) scales[row] = scale;
    uint8_t* orow = out + row * ldo;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
        const int c = tid + 512 * i;
        if (c < nch) {
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                const uint4 v = half ? duv[i] : dgv[i];
                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
                uint2 o;
                o.x = pack4(qv(bf(w[0] & 0xffffu), scale), qv(bf(w[0] >> 16), scale),
                            qv(bf(w[1] & 0xffffu), scale), qv(bf(w[1] >> 16), scale));
                o.y = pack4(qv(bf(w[2] & 0xffffu), scale), qv(bf(w[2] >> 16), scale),
                            qv(bf(w[3] & 0xffffu), scale), qv(bf(w[3] >> 16), scale));
                *reinterpret_cast<uint2*>(orow + (int64_t)half * cols + c * 8) = o;
            }
            if (dg_out) {
                const int64_t col = gpos ? 256LL * gpos[c >> 5] + 8 * (c & 31) : 8LL * c;
                if (col >= 0 && col + 8 <= ldg) *reinterpret_cast<uint4*>(dg_out + row * ldg + col) = dgv[i];
            }
            if (du_out) {
                const int64_t col = upos ? 256LL * upos[c >> 5] + 8 * (c & 31) : 8LL * c;
                if (col >= 0 && col + 8 <= ldu) *reinterpret_cast<uint4*>(du_out + row * ldu + col) = duv[i];
            }
        }
    }
}

// SwiGLU forward fused with the per-row quantisation of its output (the down_proj input of the fp8
// path): h = bf16(bf16(silu(gate)) * up) exactly as llama_kernels.hip swiglu_fwd_kernel, then one
// e4m3 row + scale per token -- bit-identical to smt_swiglu_fwd + smt_quant_rows_e4m3. The bf16 h is
// written only when h_out is non-null (an SMT down_proj reads its input columns for the tile weight
// gradient; a frozen one reads only the fp8 copy). One 512-thread workgroup per row.
template <int CPT>
__global__ __launch_bounds__(512)
void swiglu_fwd_quant_kernel(const uint16_t* __restrict__ g, const uint16_t* __restrict__ u, int64_t ld, int cols,
                             uint8_t* __restrict__ out, int64_t ldo, float* __restrict__ scales,
                             uint16_t* __restrict__ h_out) {
    __shared__ float wmax[8];
    const int tid = threadIdx.x;
    const int64_t row = blockIdx.x;
    const int nch = cols >> 3;
    uint4 hv[CPT];
    uint4 graw[CPT], uraw[CPT];                         // every load of the row issued before any math
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
        const int c = tid + 512 * i;
        const int64_t off = row * ld + (int64_t)c * 8;
        const bool in = c < nch;
        graw[i] = in ? *reinterpret_cast<const uint4*>(g + off) : make_uint4(0u, 0u, 0u, 0u);
        uraw[i] = in ? *reinterpret_cast<const uint4*>(u + off) : make_uint4(0u, 0u, 0u, 0u);
    }
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
        const int c = tid + 512 * i;
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        if (c < nch) {
            const F8 gv = unpack8(graw[i]), uv = unpack8(uraw[i]);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float sl = rbf16(gv.v[j] * smt_sigmoid(gv.v[j]));
                const float hh = rbf16(sl * uv.v[j]);
                amax = fmaxf(amax, fabsf(hh));
                w[j >> 1] |= tobf16(hh) << (16 * (j & 1));
            }
        }
        hv[i] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    amax = wave_max(amax);
    if ((tid & 63) == 0) wmax[tid >> 6] = amax;
    __syncthreads();
    amax = wmax[0];
#pragma unroll
    for (int w = 1; w < 8; ++w) amax = fmaxf(amax, wmax[w]);
    const float scale = amax > 0.f ? amax * kInvE4M3Max : 1.f;
    if (tid == 0) scales[row] = scale;
    uint8_t* orow = out + row * ldo;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
        const int c = tid + 512 * i;
        if (c < nch) {
            const uint32_t w[4] = {hv[i].x, hv[i].y, hv[i].z, hv[i].w};
            uint2 o;
            o.x = pack4(qv(bf(w[0] & 0xffffu), scale), qv(bf(w[0] >> 16), scale),
                        qv(bf(w[1] & 0xffffu), scale), qv(bf(w[1] >> 16), scale));
            o.y = pack4(qv(bf(w[2] & 0xffffu), scale), qv(bf(w[2] >> 16), scale),
                        qv(bf(w[3] & 0xffffu), scale), qv(bf(w[3] >> 16), scale));
            *reinterpret_cast<uint2*>(orow + c * 8) = o;
            if (h_out) *reinterpret_cast<uint4*>(h_out + row * ld + (int64_t)c * 8) = hv[i];
        }
    }
}

constexpr int kSlabRows = 64;
constexpr int kSlabLd = 256 + 8;             // 528-B LDS rows
constexpr int kSegRows = 256;                // rows of W one workgroup covers (4 slabs)

// Per-input-column quantisation of W [rows, cols] into out_t = W^T [cols, rows] (one scale per column
// of W), over the 256-column blocks listed in col_blocks (all when null). Grid: (column block,
// 256-row segment), so a 14336-row W spreads over 56 x n_blocks workgroups instead of n_blocks.
// Three passes that need no scratch: the column amaxes are reduced into `scales` itself (atomicMax
// on the bits of non-negative floats) after zeroing it, the quantise pass reads them, and a last
// pass turns each amax into the scale in place.
__device__ __forceinline__ int col_block_of(const int32_t* col_blocks, int i) { return col_blocks ? col_blocks[i] : i; }

__global__ __launch_bounds__(256)
void cols_t_zero_kernel(const int32_t* __restrict__ col_blocks, float* __restrict__ scales) {
    scales[(int64_t)col_block_of(col_blocks, blockIdx.x) * 256 + threadIdx.x] = 0.f;
}

__global__ __launch_bounds__(256)
void cols_t_amax_kernel(const uint16_t* __restrict__ w, int64_t ldw, int rows, const int32_t* __restrict__ col_blocks,
                        float* __restrict__ scales) {
    __shared__ float red[8][256];
    const int cb = col_block_of(col_blocks, blockIdx.x);
    const int tid = threadIdx.x, chunk = tid & 31, rg = tid >> 5;
    const int r0 = blockIdx.y * kSegRows, r1 = min(rows, r0 + kSegRows);
    const uint16_t* base = w + (int64_t)cb * 256 + chunk * 8;
    float m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = 0.f;
#pragma unroll 4
    for (int r = r0 + rg; r < r1; r += 8) {
        const F8 v = ld8(base + (int64_t)r * ldw);
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], fabsf(v.v[j]));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) red[rg][chunk * 8 + j] = m[j];
    __syncthreads();
    float amax = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) amax = fmaxf(amax, red[g][tid]);
    atomicMax(reinterpret_cast<unsigned int*>(scales) + (int64_t)cb * 256 + tid, __float_as_uint(amax));
}

__device__ __forceinline__ float scale_of_amax(float amax) { return amax > 0.f ? amax * kInvE4M3Max : 1.f; }

__global__ __launch_bounds__(256)
void cols_t_quant_kernel(const uint16_t* __restrict__ w, int64_t ldw, int rows, const int32_t* __restrict__ col_blocks,
                         const float* __restrict__ amaxes, uint8_t* __restrict__ out_t, int64_t ldo) {
    __shared__ __attribute__((aligned(16))) uint16_t slab[kSlabRows][kSlabLd];
    const int cb = col_block_of(col_blocks, blockIdx.x);
    const int tid = threadIdx.x;
    const int64_t col = (int64_t)cb * 256 + tid;
    const float scale = scale_of_amax(amaxes[col]);
    const uint16_t* base = w + (int64_t)cb * 256;
    uint8_t* orow = out_t + col * ldo;
    const int seg0 = blockIdx.y * kSegRows, seg1 = min(rows, seg0 + kSegRows);
    for (int r0 = seg0; r0 < seg1; r0 += kSlabRows) {
        __syncthreads();                                     // the previous slab is consumed
#pragma unroll
        for (int i = tid; i < kSlabRows * 32; i += 256) {
            const int rr = i >> 5, ch = i & 31;
            *reinterpret_cast<uint4*>(&slab[rr][ch * 8]) =
                *reinterpret_cast<const uint4*>(base + (int64_t)(r0 + rr) * ldw + ch * 8);
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kSlabRows / 16; ++q) {
            uint32_t wd[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int rr = q * 16 + k * 4;
                wd[k] = pack4(qv(bf(slab[rr][tid]), scale), qv(bf(slab[rr + 1][tid]), scale),
                              qv(bf(slab[rr + 2][tid]), scale), qv(bf(slab[rr + 3][tid]), scale));
            }
            *reinterpret_cast<uint4*>(orow + r0 + q * 16) = make_uint4(wd[0], wd[1], wd[2], wd[3]);
        }
    }
}

__global__ __launch_bounds__(256)
void cols_t_finalize_kernel(const int32_t* __restrict__ col_blocks, float* __restrict__ scales) {
    float* s = scales + (int64_t)col_block_of(col_blocks, blockIdx.x) * 256 + threadIdx.x;
    *s = scale_of_amax(*s);
}

}  // namespace

extern "C" {

const char* smt_fp8_last_error(void) { return g_err; }

int smt_quant_rows_e4m3(const void* x, int64_t ld_x, int64_t rows, int32_t cols, const int32_t* row_blocks_dev,
                        int32_t n_row_blocks, void* out, int64_t ld_out, float* scales, hipStream_t stream) {
    if (rows < 0 || cols <= 0 || (cols & 7) || ld_x < cols || ld_out < cols || n_row_blocks < 0)
        return fail(-1, "smt_quant_rows_e4m3: bad sizes rows=%lld cols=%d (cols %% 8 == 0)", (long long)rows, cols);
    const int64_t n_sel = row_blocks_dev ? (int64_t)n_row_blocks * 256 : rows;
    if (n_sel == 0) return 0;
    if (!x || !out || !scales) return fail(-1, "smt_quant_rows_e4m3: null pointer");
    if (!aligned16(x) || (ld_x & 7) || (reinterpret_cast<uintptr_t>(out) & 7) || (ld_out & 7))
        return fail(-2, "smt_quant_rows_e4m3: 16-byte aligned bf16 rows and 8-byte aligned fp8 rows required");
    const int64_t blocks = (n_sel + 3) / 4;
    if (blocks > 0x7fffffffLL || n_sel > 0x7fffffffLL) return fail(-1, "smt_quant_rows_e4m3: too many rows");
    const uint16_t* px = static_cast<const uint16_t*>(x);
    uint8_t* po = static_cast<uint8_t*>(out);
    const int nch = cols >> 3;
    if (nch <= 64 * 2)
        hipLaunchKernelGGL(quant_rows_reg_kernel<2>, dim3((unsigned)blocks), dim3(256), 0, stream, px, ld_x, rows, cols,
                           row_blocks_dev, n_sel, po, ld_out, scales);
    else if (nch <= 64 * 8)
        hipLaunchKernelGGL(quant_rows_reg_kernel<8>, dim3((unsigned)blocks), dim3(256), 0, stream, px, ld_x, rows, cols,
                           row_blocks_dev, n_sel, po, ld_out, scales);
    else if (nch <= 256 * 8)
        hipLaunchKernelGGL(quant_rows_wg_kernel<8>, dim3((unsigned)n_sel), dim3(256), 0, stream, px, ld_x, rows, cols,
                           row_blocks_dev, n_sel, po, ld_out, scales);
    else
        hipLaunchKernelGGL(quant_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, px, ld_x, rows, cols,
                           row_blocks_dev, n_sel, po, ld_out, scales);
    return check_launch("quant_rows_kernel");
}

int smt_quant_rows_cat_e4m3(const smt_quant_src* srcs, int32_t n_src, int64_t rows, void* out, int64_t ld_out,
                            float* scales, hipStream_t stream) {
    if (n_src < 1 || n_src > 4 || rows < 0) return fail(-1, "smt_quant_rows_cat_e4m3: 1..4 sources, rows >= 0");
    if (rows == 0) return 0;
    if (!srcs || !out || !scales) return fail(-1, "smt_quant_rows_cat_e4m3: null pointer");
    CatSrcs c{};
    c.n = n_src;
    int total = 0;
    for (int k = 0; k < 4; ++k) {
        c.off[k] = total;
        if (k < n_src) {
            const smt_quant_src& s = srcs[k];
            if (!s.ptr || s.cols <= 0 || (s.cols & 7) || s.ld < s.cols || (s.ld & 7) || !aligned16(s.ptr))
                return fail(-2, "smt_quant_rows_cat_e4m3: source %d needs 16-byte aligned bf16 rows, cols %% 8 == 0", k);
            c.p[k] = static_cast<const uint16_t*>(s.ptr);
            c.ld[k] = s.ld;
            total += s.cols / 8;
        } else {
            c.p[k] = nullptr;
            c.ld[k] = 0;
        }
    }
    c.off[4] = total;
    for (int k = n_src; k < 4; ++k) c.off[k] = total;
    if (total > 512 * 8) return fail(-1, "smt_quant_rows_cat_e4m3: %d columns > 32768", total * 8);
    if (ld_out < (int64_t)total * 8 || (ld_out & 7) || (reinterpret_cast<uintptr_t>(out) & 7))
        return fail(-2, "smt_quant_rows_cat_e4m3: ld_out must cover the concatenation, 8-byte aligned");
    if (rows > 0x7fffffffLL) return fail(-1, "smt_quant_rows_cat_e4m3: too many rows");
    bool uniform = true;
    for (int k = 0; k < n_src; ++k) uniform = uniform && (c.off[k + 1] - c.off[k]) % 64 == 0;
    const dim3 grid((unsigned)rows);
    uint8_t* po = static_cast<uint8_t*>(out);
#define SMT_CAT(CPT, NT)                                                                                         \
    do {                                                                                                         \
        if (uniform)                                                                                             \
            hipLaunchKernelGGL((quant_rows_cat_kernel<CPT, NT, true>), grid, dim3(NT), 0, stream, c, rows, po,    \
                               ld_out, scales);                                                                  \
        else                                                                                                     \
            hipLaunchKernelGGL((quant_rows_cat_kernel<CPT, NT, false>), grid, dim3(NT), 0, stream, c, rows, po,   \
                               ld_out, scales);                                                                  \
    } while (0)
    if (total <= 4 * 256) SMT_CAT(4, 256);
    else if (total <= 8 * 256) SMT_CAT(8, 256);
    else SMT_CAT(8, 512);
#undef SMT_CAT
    return check_launch("quant_rows_cat_kernel");
}

int smt_swiglu_fwd_quant_e4m3(const void* gate, const void* up, int64_t rows, int32_t cols, void* out, int64_t ld_out,
                              float* scales, void* h_out, hipStream_t stream) {
    if (rows < 0 || cols <= 0 || (cols & 7) || cols > 512 * 4 * 8)
        return fail(-1, "smt_swiglu_fwd_quant_e4m3: bad sizes rows=%lld cols=%d (cols %% 8 == 0, <= 16384)",
                    (long long)rows, cols);
    if (rows == 0) return 0;
    if (!gate || !up || !out || !scales) return fail(-1, "smt_swiglu_fwd_quant_e4m3: null pointer");
    if (!aligned16(gate) || !aligned16(up) || (h_out && !aligned16(h_out)) ||
        (reinterpret_cast<uintptr_t>(out) & 7) || (ld_out & 7) || ld_out < cols)
        return fail(-2, "smt_swiglu_fwd_quant_e4m3: 16-byte aligned bf16 rows, 8-byte aligned fp8 rows");
    if (rows > 0x7fffffffLL) return fail(-1, "smt_swiglu_fwd_quant_e4m3: too many rows");
    const uint16_t *pg = static_cast<const uint16_t*>(gate), *pu = static_cast<const uint16_t*>(up);
    uint8_t* po = static_cast<uint8_t*>(out);
    uint16_t* ph = static_cast<uint16_t*>(h_out);
    if ((cols >> 3) <= 512 * 2)
        hipLaunchKernelGGL(swiglu_fwd_quant_kernel<2>, dim3((unsigned)rows), dim3(512), 0, stream, pg, pu,
                           (int64_t)cols, cols, po, ld_out, scales, ph);
    else
        hipLaunchKernelGGL(swiglu_fwd_quant_kernel<4>, dim3((unsigned)rows), dim3(512), 0, stream, pg, pu,
                           (int64_t)cols, cols, po, ld_out, scales, ph);
    return check_launch("swiglu_fwd_quant_kernel");
}

}  // extern "C"

namespace {

int swiglu_bwd_quant_launch(const char* fn, const void* gate, const void* up, const void* grad_out, int64_t rows,
                            int32_t cols, void* out, int64_t ld_out, float* scales, void* grad_gate,
                            const int32_t* gate_pos, int64_t ld_gate, void* grad_up, const int32_t* up_pos,
                            int64_t ld_up, hipStream_t stream) {
    if (rows < 0 || cols <= 0 || (cols & 7) || cols > 512 * 4 * 8)
        return fail(-1, "%s: bad sizes rows=%lld cols=%d (cols %% 8 == 0, <= 16384)", fn, (long long)rows, cols);
    if ((gate_pos || up_pos) && (cols % 256))
        return fail(-1, "%s: a block position map needs cols %% 256 == 0 (cols=%d)", fn, cols);
    if ((grad_gate && (ld_gate < (gate_pos ? 256 : cols) || (ld_gate & 7))) ||
        (grad_up && (ld_up < (up_pos ? 256 : cols) || (ld_up & 7))))
        return fail(-1, "%s: bad gradient row strides %lld / %lld", fn, (long long)ld_gate, (long long)ld_up);
    if (rows == 0) return 0;
    if (!gate || !up || !grad_out || !out || !scales) return fail(-1, "%s: null pointer", fn);
    if (!aligned16(gate) || !aligned16(up) || !aligned16(grad_out) || (grad_gate && !aligned16(grad_gate)) ||
        (grad_up && !aligned16(grad_up)) || (reinterpret_cast<uintptr_t>(out) & 7) || (ld_out & 7) ||
        ld_out < 2LL * cols)
        return fail(-2, "%s: 16-byte aligned bf16 rows, 8-byte aligned fp8 rows of >= 2*cols", fn);
    if (rows > 0x7fffffffLL) return fail(-1, "%s: too many rows", fn);
    const uint16_t *pg = static_cast<const uint16_t*>(gate), *pu = static_cast<const uint16_t*>(up),
                   *ph = static_cast<const uint16_t*>(grad_out);
    uint8_t* po = static_cast<uint8_t*>(out);
    uint16_t *dg = static_cast<uint16_t*>(grad_gate), *du = static_cast<uint16_t*>(grad_up);
    const int nch = cols >> 3;
    if (nch <= 512 * 2)
        hipLaunchKernelGGL(swiglu_bwd_quant_kernel<2>, dim3((unsigned)rows), dim3(512), 0, stream, pg, pu, ph,
                           (int64_t)cols, cols, po, ld_out, scales, dg, gate_pos, ld_gate, du, up_pos, ld_up);
    else
        hipLaunchKernelGGL(swiglu_bwd_quant_kernel<4>, dim3((unsigned)rows), dim3(512), 0, stream, pg, pu, ph,
                           (int64_t)cols, cols, po, ld_out, scales, dg, gate_pos, ld_gate, du, up_pos, ld_up);
    return check_launch("swiglu_bwd_quant_kernel");
}

}  // namespace

extern "C" {

int smt_swiglu_bwd_quant_e4m3(const void* gate, const void* up, const void* grad_out, int64_t rows, int32_t cols,
                              void* out, int64_t ld_out, float* scales, void* grad_gate, void* grad_up,
                              hipStream_t stream) {
    return swiglu_bwd_quant_launch("smt_swiglu_bwd_quant_e4m3", gate, up, grad_out, rows, cols, out, ld_out, scales,
                                   grad_gate, nullptr, cols, grad_up, nullptr, cols, stream);
}

int smt_swiglu_bwd_quant_e4m3_packed(const void* gate, const void* up, const void* grad_out, int64_t rows,
                                     int32_t cols, void* out, int64_t ld_out, float* scales, void* grad_gate,
                                     const int32_t* gate_pos, int64_t ld_gate, void* grad_up, const int32_t* up_pos,
                                     int64_t ld_up, hipStream_t stream) {
    return swiglu_bwd_quant_launch("smt_swiglu_bwd_quant_e4m3_packed", gate, up, grad_out, rows, cols, out, ld_out,
                                   scales, grad_gate, gate_pos, ld_gate, grad_up, up_pos, ld_up, stream);
}

int smt_quant_cols_t_e4m3(const void* w, int64_t ld_w, int32_t rows, int32_t cols, const int32_t* col_blocks_dev,
                          int32_t n_col_blocks, void* out_t, int64_t ld_out, float* scales, hipStream_t stream) {
    if (rows <= 0 || cols <= 0 || (cols % 256) || (rows % kSlabRows) || ld_w < cols || ld_out < rows || n_col_blocks < 0)
        return fail(-1, "smt_quant_cols_t_e4m3: bad sizes rows=%d cols=%d (cols %% 256 == 0, rows %% 64 == 0)", rows, cols);
    const int nb = col_blocks_dev ? n_col_blocks : cols / 256;
    if (nb == 0) return 0;
    if (!w || !out_t || !scales) return fail(-1, "smt_quant_cols_t_e4m3: null pointer");
    if (!aligned16(w) || (ld_w & 7) || !aligned16(out_t) || (ld_out & 15))
        return fail(-2, "smt_quant_cols_t_e4m3: 16-byte aligned rows required (ld_w %% 8 == 0, ld_out %% 16 == 0)");
    const uint16_t* pw = static_cast<const uint16_t*>(w);
    const dim3 grid2((unsigned)nb, (unsigned)((rows + kSegRows - 1) / kSegRows));
    hipLaunchKernelGGL(cols_t_zero_kernel, dim3((unsigned)nb), dim3(256), 0, stream, col_blocks_dev, scales);
    hipLaunchKernelGGL(cols_t_amax_kernel, grid2, dim3(256), 0, stream, pw, ld_w, rows, col_blocks_dev, scales);
    hipLaunchKernelGGL(cols_t_quant_kernel, grid2, dim3(256), 0, stream, pw, ld_w, rows, col_blocks_dev, scales,
                       static_cast<uint8_t*>(out_t), ld_out);
    hipLaunchKernelGGL(cols_t_finalize_kernel, dim3((unsigned)nb), dim3(256), 0, stream, col_blocks_dev, scales);
    return check_launch("quant_cols_t kernels");
}

}  // extern "C"
