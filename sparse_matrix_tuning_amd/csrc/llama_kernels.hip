// llama_kernels.hip — gfx950 fused elementwise kernels for the HF LLaMA decoder that carries the SMT
// modules in the training step (bench / trainer). They replace the eager op chains of
// transformers' LlamaRMSNorm.forward, apply_rotary_pos_emb and LlamaMLP's act_fn(gate) * up, which
// the rocprof step breakdown shows as ~27 % of an SMT step (3.6 k elementwise dispatches, each a full
// HBM pass over [B*S, hidden] or [B*S, intermediate] tensors, several in fp32).
//
// Numerics follow the eager bf16 op sequence, including every intermediate bf16 rounding, so the
// outputs match the eager module to (at most) an ulp from reduction order / exp implementation.
// All loads and stores are 16 B per lane; rows are processed one wave (64 lanes) per row.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdarg.h>
#include <stdio.h>

#include "smt_hip.h"
#include "smt_model_ops.h"
#include "silu_math.h"
#include "fp8_math.h"
#include "smt_fp8.h"

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

// 16-bit storage formats: F = SMT_DTYPE_BF16 (0) or SMT_DTYPE_FP16 (2), the model's dtype (the
// reference's --dtype bf16 | fp16, fine_tune.py:955-959, deepspeed_helpers.py:53-58). The eager chains
// round to the model's dtype at the same points in both formats, so every kernel below is a template on
// F with one body; the fp8 producer fusions (QUANT) exist for bf16 models only.
template <int F> __device__ __forceinline__ float u2f(uint32_t b16) {         // 16-bit bits -> fp32 (exact)
    if constexpr (F == SMT_DTYPE_FP16) return (float)__builtin_bit_cast(_Float16, (uint16_t)b16);
    else return __uint_as_float(b16 << 16);
}
template <int F> __device__ __forceinline__ uint32_t f2u(float f) {           // fp32 -> 16-bit bits (RNE)
    if constexpr (F == SMT_DTYPE_FP16) return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)f);
    else return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)f);
}
// round through F. For fp16 the rounded bits pass an empty asm: hipcc otherwise shrinks
// float(half(a * b)) + c to a half multiply and contracts it with the add into v_pk_fma_f16, dropping
// the product's rounding that the eager chain performs (rope_fp16 differed from eager by it). bf16
// has no native arithmetic to shrink to, and its code is unchanged.
template <int F> __device__ __forceinline__ float rnd(float f) {
    uint32_t b = f2u<F>(f);
    if constexpr (F == SMT_DTYPE_FP16) asm("" : "+v"(b));
    return u2f<F>(b);
}

struct F8 { float v[8]; };

template <int F> __device__ __forceinline__ F8 unpack8(const uint4 a) {
    F8 r;
    const uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) { r.v[2 * j] = u2f<F>(w[j] & 0xffffu); r.v[2 * j + 1] = u2f<F>(w[j] >> 16); }
    return r;
}

template <int F> __device__ __forceinline__ F8 ld8(const uint16_t* p) {
    return unpack8<F>(*reinterpret_cast<const uint4*>(p));
}

// 16-bit bits of 8 floats (RNE; exact for values that are in the format already) and back
template <int F> __device__ __forceinline__ uint4 pack8(const F8& r) {
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) w[j] = f2u<F>(r.v[2 * j]) | (f2u<F>(r.v[2 * j + 1]) << 16);
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Row values kept in registers by the register-resident kernels: fp32 (PACK = false) or packed
// 16-bit bits (PACK = true; exact for values that are in the format already).
template <int F> __device__ __forceinline__ F8 rnd8(const F8& v) {
    F8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r.v[j] = rnd<F>(v.v[j]);
    return r;
}
template <bool PACK, int F> struct RowReg;
template <int F> struct RowReg<false, F> {
    typedef F8 T;
    static __device__ __forceinline__ T keep(const uint4 raw) { return unpack8<F>(raw); }
    static __device__ __forceinline__ T put(const F8& v) { return v; }
    static __device__ __forceinline__ F8 get(const T& v) { return v; }
};
template <int F> struct RowReg<true, F> {
    typedef uint4 T;
    static __device__ __forceinline__ T keep(const uint4 raw) { return raw; }
    static __device__ __forceinline__ T put(const F8& v) { return pack8<F>(v); }
    static __device__ __forceinline__ F8 get(const T& v) { return unpack8<F>(v); }
};

template <int F> __device__ __forceinline__ void st8(uint16_t* p, const F8& r) {
    *reinterpret_cast<uint4*>(p) = pack8<F>(r);
}

__device__ __forceinline__ float wave_max_f(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
    return v;
}

__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// ------------------------------------------------------------------------------------------------
// RMSNorm (LlamaRMSNorm.forward):  xf = float(x); r = rsqrt(mean(xf^2) + eps);
//                                  y = bf16(float(w) * float(bf16(xf * r)))
// ------------------------------------------------------------------------------------------------
template <int F>
__global__ __launch_bounds__(256)
void rmsnorm_fwd_kernel(const uint16_t* __restrict__ x, int64_t ldx, const uint16_t* __restrict__ w,
                        uint16_t* __restrict__ y, int64_t ldy, float* __restrict__ rstd,
                        int64_t rows, int H, float eps) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const uint16_t* xr = x + row * ldx;
    const int nch = H >> 3;
    float ss = 0.f;
    for (int c = lane; c < nch; c += 64) {
        const F8 v = ld8<F>(xr + c * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += v.v[j] * v.v[j];
    }
    ss = wave_sum_f(ss);
    const float r = 1.0f / sqrtf(ss / (float)H + eps);
    if (lane == 0) rstd[row] = r;
    uint16_t* yr = y + row * ldy;
    for (int c = lane; c < nch; c += 64) {
        const F8 v = ld8<F>(xr + c * 8);
        const F8 wv = ld8<F>(w + c * 8);
        F8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o.v[j] = wv.v[j] * rnd<F>(v.v[j] * r);
        st8<F>(yr + c * 8, o);
    }
}

// Backward of the eager chain: dn = bf16(dy * w); dx = bf16(r*dn - xf * r^3 * sum(dn*xf) / H), for
// any hidden % 8 == 0 (the register-resident kernels below cover hidden % 512 == 0). Waves stride
// over rows.
template <int F>
__global__ __launch_bounds__(256)
void rmsnorm_bwd_kernel(const uint16_t* __restrict__ dy, int64_t lddy, const uint16_t* __restrict__ x, int64_t ldx,
                        const uint16_t* __restrict__ w, const float* __restrict__ rstd,
                        uint16_t* __restrict__ dx, int64_t lddx, int64_t rows, int H) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t n_waves = (int64_t)gridDim.x * 4;
    const int nch = H >> 3;
    for (int64_t row = wave; row < rows; row += n_waves) {
        const float r = rstd[row];
        const uint16_t* xr = x + row * ldx;
        const uint16_t* dyr = dy + row * lddy;
        float dot = 0.f;
        for (int c = lane; c < nch; c += 64) {
            const F8 xv = ld8<F>(xr + c * 8), gv = ld8<F>(dyr + c * 8), wv = ld8<F>(w + c * 8);
#pragma unroll
            for (int j = 0; j < 8; ++j) dot += rnd<F>(gv.v[j] * wv.v[j]) * xv.v[j];
        }
        dot = wave_sum_f(dot);
        const float coef = r * r * r * dot / (float)H;
        uint16_t* dxr = dx + row * lddx;
        for (int c = lane; c < nch; c += 64) {
            const F8 xv = ld8<F>(xr + c * 8), gv = ld8<F>(dyr + c * 8), wv = ld8<F>(w + c * 8);
            F8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) o.v[j] = r * rnd<F>(gv.v[j] * wv.v[j]) - xv.v[j] * coef;
            st8<F>(dxr + c * 8, o);
        }
    }
}

// dw = bf16(sum over the waves' partials), in a fixed order: stage 1 sums each chunk of kDwChunk
// partial rows (in row order) into the chunk's first row, stage 2 the chunk sums in chunk order.
// (One thread per column over all 4096 partial rows took 1.1 ms per call: 16 workgroups of
// serial loads.)
constexpr int kDwChunk = 64;

__global__ __launch_bounds__(256)
void rmsnorm_dw_chunk_kernel(float* __restrict__ partial, int64_t n_waves, int H) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    if (col >= H) return;
    const int64_t r0 = (int64_t)blockIdx.y * kDwChunk;
    const int64_t r1 = r0 + kDwChunk < n_waves ? r0 + kDwChunk : n_waves;
    float s = 0.f;
    for (int64_t i = r0; i < r1; ++i) s += partial[i * H + col];
    partial[r0 * H + col] = s;
}

template <int F>
__global__ __launch_bounds__(256)
void rmsnorm_dw_kernel(const float* __restrict__ partial, int64_t n_waves, int H, uint16_t* __restrict__ dw) {
    const int col = blockIdx.x * 256 + threadIdx.x;
    if (col >= H) return;
    float s = 0.f;
    for (int64_t i = 0; i < n_waves; i += kDwChunk) s += partial[i * H + col];
    dw[col] = (uint16_t)f2u<F>(s);
}

// Register-resident variants (hidden = 512 * CPL, CPL <= 16): one wave per row keeps its 8 * CPL
// values in registers, so each input is read from HBM once (the generic kernels above read the row
// twice). Same arithmetic and the same per-lane accumulation order, so the results are bit-identical
// to them.
//
// Forward with an optional fused residual add (LlamaDecoderLayer: h = residual + attn_out, then
// post_attention_layernorm(h)): h = bf16(x + res) is written out as well and normalised.
template <int CPL, bool ADD, bool QUANT = false, int F = SMT_DTYPE_BF16>
__global__ __launch_bounds__(256)
void rmsnorm_fwd_reg_kernel(const uint16_t* __restrict__ x, int64_t ldx, const uint16_t* __restrict__ res, int64_t ldr,
                            const uint16_t* __restrict__ w, uint16_t* __restrict__ h, int64_t ldh,
                            uint16_t* __restrict__ y, int64_t ldy, float* __restrict__ rstd, int64_t rows, int H,
                            float eps, uint8_t* __restrict__ q8, int64_t ldq, float* __restrict__ qscale) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    F8 v[CPL];
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int c = lane + 64 * k;
        v[k] = ld8<F>(x + row * ldx + c * 8);
        if (ADD) {
            const F8 rv = ld8<F>(res + row * ldr + c * 8);
#pragma unroll
            for (int j = 0; j < 8; ++j) v[k].v[j] = rnd<F>(v[k].v[j] + rv.v[j]);
            st8<F>(h + row * ldh + c * 8, v[k]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) ss += v[k].v[j] * v[k].v[j];
    }
    ss = wave_sum_f(ss);
    const float r = 1.0f / sqrtf(ss / (float)H + eps);
    if (lane == 0) rstd[row] = r;
    if (!QUANT) {
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            const int c = lane + 64 * k;
            const F8 wv = ld8<F>(w + c * 8);
            F8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) o.v[j] = wv.v[j] * rnd<F>(v[k].v[j] * r);
            st8<F>(y + row * ldy + c * 8, o);
        }
        return;
    }
    // QUANT: the bf16 output (kept in registers) also as one e4m3 row + scale, exactly as
    // smt_quant_rows_e4m3 would quantise it; the bf16 row is stored only when y is non-null
    float amax = 0.f;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int c = lane + 64 * k;
        const F8 wv = ld8<F>(w + c * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            v[k].v[j] = rnd<F>(wv.v[j] * rnd<F>(v[k].v[j] * r));
            amax = fmaxf(amax, fabsf(v[k].v[j]));
        }
        if (y) st8<F>(y + row * ldy + c * 8, v[k]);
    }
    amax = wave_max_f(amax);
    const float scale = e4m3_scale(amax);
    if (lane == 0) qscale[row] = scale;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int c = lane + 64 * k;
        uint2 o;
        o.x = pack4(qv(v[k].v[0], scale), qv(v[k].v[1], scale), qv(v[k].v[2], scale), qv(v[k].v[3], scale));
        o.y = pack4(qv(v[k].v[4], scale), qv(v[k].v[5], scale), qv(v[k].v[6], scale), qv(v[k].v[7], scale));
        *reinterpret_cast<uint2*>(q8 + row * ldq + c * 8) = o;
    }
}

// Backward without weight grad; with ADD the gradient reaching the norm's input by the residual path
// is added as autograd would: dx = bf16(bf16(dx_norm) + dres). The residual gradient is loaded up
// front, beside the row's other loads (profiles/r04_v_norm_bwd_preload_ab.jsonl: 193-197 -> 189-190 us).
template <int CPL, bool ADD, bool QUANT = false, int F = SMT_DTYPE_BF16>
__global__ __launch_bounds__(256, CPL <= 10 ? 2 : 1)        // two waves per SIMD up to hidden 5120
void rmsnorm_bwd_reg_kernel(const uint16_t* __restrict__ dy, int64_t lddy, const uint16_t* __restrict__ x, int64_t ldx,
                            const uint16_t* __restrict__ w, const float* __restrict__ rstd,
                            const uint16_t* __restrict__ dres, int64_t lddr, uint16_t* __restrict__ dx, int64_t lddx,
                            int64_t rows, int H, uint8_t* __restrict__ q8 = nullptr, int64_t ldq = 0,
                            float* __restrict__ qscale = nullptr) {
    const int lane = threadIdx.x & 63;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float r = rstd[row];
    // the row's x and bf16(dy * w) stay in registers; above CPL 8 as packed bf16 (both are bf16
    // values, so this is exact): half the registers of fp32 copies, two waves per SIMD at CPL 10
    // instead of one (at CPL 8 the fp32 copies fit two waves, and the packing only adds ALU work)
    constexpr bool PACK = CPL > 8;
    typename RowReg<PACK, F>::T xr[CPL], gr[CPL];
    // up to CPL 8 the residual gradient's row is loaded with x and dy (32 more registers): issued
    // in the second pass, each load waited behind the dx stores issued before it (vmcnt counts both)
    constexpr bool PRE = ADD && !PACK;
    uint4 drr[PRE ? CPL : 1];
    if constexpr (PRE) {
#pragma unroll
        for (int k = 0; k < CPL; ++k) drr[k] = *reinterpret_cast<const uint4*>(dres + row * lddr + (lane + 64 * k) * 8);
    }
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int c = lane + 64 * k;
        const uint4 xraw = *reinterpret_cast<const uint4*>(x + row * ldx + c * 8);
        xr[k] = RowReg<PACK, F>::keep(xraw);
        const F8 xv = unpack8<F>(xraw), gv = ld8<F>(dy + row * lddy + c * 8), wv = ld8<F>(w + c * 8);
        F8 gw;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            gw.v[j] = rnd<F>(gv.v[j] * wv.v[j]);
            dot += gw.v[j] * xv.v[j];
        }
        gr[k] = RowReg<PACK, F>::put(gw);
    }
    if constexpr (PRE) {
        // opaque from here on: hipcc would otherwise re-issue (rematerialise) the read-only loads in pass 2
#pragma unroll
        for (int k = 0; k < CPL; ++k)
            asm volatile("" : "+v"(drr[k].x), "+v"(drr[k].y), "+v"(drr[k].z), "+v"(drr[k].w));
    }
    dot = wave_sum_f(dot);
    const float coef = r * r * r * dot / (float)H;
    if constexpr (PACK) asm volatile("" ::: "memory");   // the residual-gradient loads stay in this pass
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
        const int c = lane + 64 * k;
        const F8 xv = RowReg<PACK, F>::get(xr[k]), gw = RowReg<PACK, F>::get(gr[k]);
        F8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o.v[j] = r * gw.v[j] - xv.v[j] * coef;
        if (ADD) {
            F8 dr;
            if constexpr (PRE) dr = unpack8<F>(drr[k]);
            else dr = ld8<F>(dres + row * lddr + c * 8);
#pragma unroll
            for (int j = 0; j < 8; ++j) o.v[j] = rnd<F>(o.v[j]) + dr.v[j];
        }
        st8<F>(dx + row * lddx + c * 8, o);
        if (QUANT) gr[k] = RowReg<PACK, F>::put(rnd8<F>(o));   // the stored bf16 dx, kept for the e4m3 pass
    }
    if (QUANT) {
        // dx also as one e4m3 row + scale (the data-gradient GEMM operand of the fp8 linear that
        // consumes this gradient), exactly as smt_quant_rows_e4m3 would quantise the stored dx
        float amax = 0.f;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            const F8 d = RowReg<PACK, F>::get(gr[k]);
#pragma unroll
            for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(d.v[j]));
        }
        amax = wave_max_f(amax);
        const float scale = e4m3_scale(amax);
        if (lane == 0) qscale[row] = scale;
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
            const int c = lane + 64 * k;
            const F8 d = RowReg<PACK, F>::get(gr[k]);
            uint2 q;
            q.x = pack4(qv(d.v[0], scale), qv(d.v[1], scale), qv(d.v[2], scale), qv(d.v[3], scale));
            q.y = pack4(qv(d.v[4], scale), qv(d.v[5], scale), qv(d.v[6], scale), qv(d.v[7], scale));
            *reinterpret_cast<uint2*>(q8 + row * ldq + c * 8) = q;
        }
    }
}

// The weight gradient of the full fine-tuning warm-up: dw = bf16(sum_rows bf16(dy * bf16(x * r))),
// the eager chain's terms. Its own pass over x and dy (the dx pass stays the register-resident
// kernel, one row per wave): a thread owns 8 columns of one chunk of `rows_per_chunk` rows and adds
// that chunk's terms in row order into dw_partial[chunk]; the chunks are then summed in chunk order.
// (Fusing the column sums into the dx kernel needs 8 * CPL fp32 accumulators per lane beside the
// row: ~390 registers at hidden 4096, one wave per SIMD, 2.9 TB/s.)
template <int F>
__global__ __launch_bounds__(256)
void rmsnorm_dw_rows_kernel(const uint16_t* __restrict__ dy, int64_t lddy, const uint16_t* __restrict__ x,
                            int64_t ldx, const float* __restrict__ rstd, float* __restrict__ dw_partial,
                            int64_t rows, int64_t rows_per_chunk, int H) {
    const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
    if (c >= H) return;
    const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
    const int64_t r1 = r0 + rows_per_chunk < rows ? r0 + rows_per_chunk : rows;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll 4
    for (int64_t row = r0; row < r1; ++row) {
        const float r = rstd[row];
        const F8 xv = ld8<F>(x + row * ldx + c), gv = ld8<F>(dy + row * lddy + c);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += rnd<F>(gv.v[j] * rnd<F>(xv.v[j] * r));
    }
    float4* d = reinterpret_cast<float4*>(dw_partial + (int64_t)blockIdx.y * H + c);
    d[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    d[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
}

// ------------------------------------------------------------------------------------------------
// RoPE (apply_rotary_pos_emb): per element pair (d, d+D/2) of one head row,
//   lo' = bf16(bf16(lo*c_lo) + bf16(-hi*s_lo)),  hi' = bf16(bf16(hi*c_hi) + bf16(lo*s_hi))
// backward:
//   dlo = bf16(bf16(dlo'*c_lo) + bf16(dhi'*s_hi)), dhi = bf16(bf16(dhi'*c_hi) - bf16(dlo'*s_lo))
// Tensors are [B, H, S, D] with element strides (sb, sh, ss, 1); cos/sin [B, S, D] (cb, cs, 1).
// One thread per 8 pairs; the q and k tensors share one launch.
// ------------------------------------------------------------------------------------------------
struct RopeT {
    const uint16_t* in; uint16_t* out;
    int64_t sb, sh, ss;     // input strides
    int64_t ob, oh, os;     // output strides
    int H;
};

// One (b, head) row block per blockIdx.y (q heads first, then k heads: wave-uniform), the
// (s, 8-pair chunk) index on blockIdx.x * 256 + tid with 32-bit arithmetic (the flat 64-bit
// div / mod chain of a 1-D grid cost more than the bytes).
template <bool BWD, int F>
__device__ __forceinline__ void rope_row(const RopeT& t, const uint16_t* cos, const uint16_t* sin, int64_t cb,
                                         int64_t cs, int64_t b, int h, int idx, int S, int D) {
    const int half = D >> 1;
    const int cpr = half >> 3;                        // 8-pair chunks per head row
    const int s = idx / cpr;
    if (s >= S) return;
    const int d = (idx - s * cpr) * 8;
    const uint16_t* ip = t.in + b * t.sb + h * t.sh + (int64_t)s * t.ss;
    uint16_t* op = t.out + b * t.ob + h * t.oh + (int64_t)s * t.os;
    const uint16_t* cp = cos + b * cb + (int64_t)s * cs;
    const uint16_t* sp = sin + b * cb + (int64_t)s * cs;
    const F8 lo = ld8<F>(ip + d), hi = ld8<F>(ip + half + d);
    const F8 clo = ld8<F>(cp + d), chi = ld8<F>(cp + half + d), slo = ld8<F>(sp + d), shi = ld8<F>(sp + half + d);
    F8 olo, ohi;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        if (!BWD) {
            olo.v[j] = rnd<F>(lo.v[j] * clo.v[j]) + rnd<F>(-hi.v[j] * slo.v[j]);
            ohi.v[j] = rnd<F>(hi.v[j] * chi.v[j]) + rnd<F>(lo.v[j] * shi.v[j]);
        } else {
            olo.v[j] = rnd<F>(lo.v[j] * clo.v[j]) + rnd<F>(hi.v[j] * shi.v[j]);
            ohi.v[j] = rnd<F>(hi.v[j] * chi.v[j]) - rnd<F>(lo.v[j] * slo.v[j]);
        }
    }
    st8<F>(op + d, olo);
    st8<F>(op + half + d, ohi);
}

// Head-grouped variant: a thread rotates the same (s, 8-pair chunk) of kRopeHG consecutive heads, so
// its cos / sin chunks (4 x 16 B) are loaded once per group instead of once per head (the loads per
// element pair drop from 6 to 2.5). blockIdx.y = b * (q groups + k groups) + group.
constexpr int kRopeHG = 8;
template <bool BWD, int F>
__global__ __launch_bounds__(256)
void rope_hg_kernel(RopeT q, RopeT k, const uint16_t* __restrict__ cos, const uint16_t* __restrict__ sin,
                    int64_t cb, int64_t cs, int S, int D) {
    const int qg = q.H / kRopeHG, groups = qg + k.H / kRopeHG;
    const int y = blockIdx.y;
    const int64_t b = y / groups;
    const int g = y - (int)b * groups;
    const RopeT& t = g < qg ? q : k;
    const int h0 = (g < qg ? g : g - qg) * kRopeHG;
    const int half = D >> 1;
    const int cpr = half >> 3;
    const int idx = blockIdx.x * 256 + threadIdx.x;
    const int s = idx / cpr;
    if (s >= S) return;
    const int d = (idx - s * cpr) * 8;
    const uint16_t* cp = cos + b * cb + (int64_t)s * cs;
    const uint16_t* sp = sin + b * cb + (int64_t)s * cs;
    const F8 clo = ld8<F>(cp + d), chi = ld8<F>(cp + half + d), slo = ld8<F>(sp + d), shi = ld8<F>(sp + half + d);
#pragma unroll 4
    for (int h = h0; h < h0 + kRopeHG; ++h) {
        const uint16_t* ip = t.in + b * t.sb + h * t.sh + (int64_t)s * t.ss;
        uint16_t* op = t.out + b * t.ob + h * t.oh + (int64_t)s * t.os;
        const F8 lo = ld8<F>(ip + d), hi = ld8<F>(ip + half + d);
        F8 olo, ohi;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (!BWD) {
                olo.v[j] = rnd<F>(lo.v[j] * clo.v[j]) + rnd<F>(-hi.v[j] * slo.v[j]);
                ohi.v[j] = rnd<F>(hi.v[j] * chi.v[j]) + rnd<F>(lo.v[j] * shi.v[j]);
            } else {
                olo.v[j] = rnd<F>(lo.v[j] * clo.v[j]) + rnd<F>(hi.v[j] * shi.v[j]);
                ohi.v[j] = rnd<F>(hi.v[j] * chi.v[j]) - rnd<F>(lo.v[j] * slo.v[j]);
            }
        }
        st8<F>(op + d, olo);
        st8<F>(op + half + d, ohi);
    }
}

template <bool BWD, int F>
__global__ __launch_bounds__(256)
void rope_kernel(RopeT q, RopeT k, const uint16_t* __restrict__ cos, const uint16_t* __restrict__ sin,
                 int64_t cb, int64_t cs, int64_t B, int S, int D) {
    const int heads = q.H + k.H;
    const int y = blockIdx.y;                         // b * heads + head
    const int64_t b = y / heads;
    const int hh = y - (int)b * heads;
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (hh < q.H) rope_row<BWD, F>(q, cos, sin, cb, cs, b, hh, idx, S, D);
    else rope_row<BWD, F>(k, cos, sin, cb, cs, b, hh - q.H, idx, S, D);
}

// ------------------------------------------------------------------------------------------------
// SwiGLU (act_fn(gate) * up with act_fn = SiLU):
//   s = bf16(g / (1 + exp(-g))), h = bf16(s * u)
// backward: ds = bf16(dh*u), du = bf16(dh*s), dg = bf16(ds * sig * (1 + g*(1 - sig)))
// ------------------------------------------------------------------------------------------------
template <int F>
__global__ __launch_bounds__(256)
void swiglu_fwd_kernel(const uint16_t* __restrict__ g, const uint16_t* __restrict__ u, uint16_t* __restrict__ h,
                       int64_t n8) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n8) return;
    const F8 gv = ld8<F>(g + i * 8), uv = ld8<F>(u + i * 8);
    F8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float s = rnd<F>(gv.v[j] * smt_sigmoid(gv.v[j]));
        o.v[j] = s * uv.v[j];
    }
    st8<F>(h + i * 8, o);
}

// Column blocks of a norm's or SwiGLU's output rebuilt from the producer's own saved operands
// (activation policy "selective": linearZ keeps no copy of these inputs between forward and
// backward). Same block-major layout as smt_colblock_gather (out[j][t][256]) and the producers'
// arithmetic, so the values are bit-identical to the gathered ones:
//   OP 0 (RMSNorm): out = bf16(float(w) * float(bf16(x * rstd)))   (rmsnorm_fwd_kernel, _reg_kernel)
//   OP 1 (SwiGLU):  out = bf16(float(bf16(g * sigmoid(g))) * u)    (swiglu_fwd_kernel)
// 16 B per thread, a wave covers two 512-B row pieces.
template <int OP, int F>
__global__ __launch_bounds__(256)
void colblock_recompute_kernel(const uint16_t* __restrict__ a, int64_t lda, const uint16_t* __restrict__ b, int64_t ldb,
                               const uint16_t* __restrict__ w, const float* __restrict__ rstd, int64_t T,
                               const int32_t* __restrict__ col_blocks, int32_t n_cb, uint16_t* __restrict__ out) {
    const int64_t per_row = (int64_t)n_cb * 32;
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t t = v / per_row;
    if (t >= T) return;
    const int r = (int)(v - t * per_row);
    const int j = r >> 5, ch = r & 31;
    const int64_t c = (int64_t)col_blocks[j] * 256 + ch * 8;
    const F8 av = ld8<F>(a + t * lda + c);
    F8 o;
    if (OP == 0) {
        const float rs = rstd[t];
        const F8 wv = ld8<F>(w + c);
#pragma unroll
        for (int k = 0; k < 8; ++k) o.v[k] = wv.v[k] * rnd<F>(av.v[k] * rs);
    } else {
        const F8 bv = ld8<F>(b + t * ldb + c);
#pragma unroll
        for (int k = 0; k < 8; ++k) o.v[k] = rnd<F>(av.v[k] * smt_sigmoid(av.v[k])) * bv.v[k];
    }
    st8<F>(out + ((int64_t)j * T + t) * 256 + ch * 8, o);
}

template <int F>
__global__ __launch_bounds__(256)
void swiglu_bwd_kernel(const uint16_t* __restrict__ g, const uint16_t* __restrict__ u, const uint16_t* __restrict__ dh,
                       uint16_t* __restrict__ dg, uint16_t* __restrict__ du, int64_t n8) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n8) return;
    const F8 gv = ld8<F>(g + i * 8), uv = ld8<F>(u + i * 8), hv = ld8<F>(dh + i * 8);
    F8 og, ou;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float x = gv.v[j];
        const float sig = smt_sigmoid(x);
        const float s = rnd<F>(x * sig);
        const float ds = rnd<F>(hv.v[j] * uv.v[j]);
        ou.v[j] = hv.v[j] * s;
        og.v[j] = ds * sig * (1.0f + x * (1.0f - sig));
    }
    st8<F>(dg + i * 8, og);
    st8<F>(du + i * 8, ou);
}

// ------------------------------------------------------------------------------------------------
// Causal-LM cross entropy (transformers ForCausalLMLoss: logits.float() -> log_softmax -> nll with
// ignore_index). The eager chain writes an fp32 copy of the [rows, vocab] logits (16.8 GB at
// B16 x S2048 x V128256), a log_softmax output of the same size, and an fp32 gradient cast back to
// bf16. Here the forward reads the bf16 logits once (per-row online max / sum of exp, one workgroup
// per row) and the backward reads them once more and writes the bf16 gradient.
// Softmax arithmetic in the log2 domain: y = x * log2(e), exp via v_exp_f32.
// ------------------------------------------------------------------------------------------------
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;
constexpr float kNegInf = -__builtin_huge_valf();
constexpr int kCeThreads = 256;

// (m, s): running max of the log2-scaled logits and sum of exp2(y - m)
__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
    const float M = fmaxf(m, m2);
    if (M == kNegInf) return;                           // both still empty
    s = s * __builtin_amdgcn_exp2f(m - M) + s2 * __builtin_amdgcn_exp2f(m2 - M);
    m = M;
}

__device__ __forceinline__ void lse_chunk(const F8& v, float& m, float& s) {
    float y[8];
    float cm = kNegInf;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        y[j] = v.v[j] * kLog2e;
        cm = fmaxf(cm, y[j]);
    }
    if (cm > m) {
        s *= __builtin_amdgcn_exp2f(m - cm);
        m = cm;
    }
    if (m == kNegInf) return;                           // every logit so far is -inf
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __builtin_amdgcn_exp2f(y[j] - m);
}

template <int F>
__global__ __launch_bounds__(kCeThreads)
void ce_fwd_kernel(const uint16_t* __restrict__ logits, int64_t ld, const int64_t* __restrict__ labels, int64_t V,
                   int64_t ignore_index, float* __restrict__ lse, float* __restrict__ loss) {
    __shared__ float wm[kCeThreads / 64], wsum[kCeThreads / 64];
    const int64_t row = blockIdx.x;
    const uint16_t* xr = logits + row * ld;
    const int tid = threadIdx.x;
    const int64_t n8 = V >> 3;
    float m = kNegInf, s = 0.f;
    int64_t c = tid;
    for (; c + 3 * kCeThreads < n8; c += 4 * kCeThreads) {     // 4 x 16 B in flight per lane
        const F8 a = ld8<F>(xr + c * 8), b = ld8<F>(xr + (c + kCeThreads) * 8);
        const F8 d = ld8<F>(xr + (c + 2 * kCeThreads) * 8), e = ld8<F>(xr + (c + 3 * kCeThreads) * 8);
        lse_chunk(a, m, s);
        lse_chunk(b, m, s);
        lse_chunk(d, m, s);
        lse_chunk(e, m, s);
    }
    for (; c < n8; c += kCeThreads) lse_chunk(ld8<F>(xr + c * 8), m, s);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const float m2 = __shfl_xor(m, off, 64), s2 = __shfl_xor(s, off, 64);
        lse_merge(m, s, m2, s2);
    }
    if ((tid & 63) == 0) {
        wm[tid >> 6] = m;
        wsum[tid >> 6] = s;
    }
    __syncthreads();
    if (tid == 0) {
#pragma unroll
        for (int w = 1; w < kCeThreads / 64; ++w) lse_merge(m, s, wm[w], wsum[w]);
        const float l = (m + log2f(s)) * kLn2;
        lse[row] = l;
        const int64_t lab = labels[row];
        float out;
        if (lab == ignore_index) out = 0.f;
        else if (lab < 0 || lab >= V) out = __builtin_nanf("");
        else out = l - u2f<F>((uint32_t)xr[lab]);
        loss[row] = out;
    }
}

__device__ __forceinline__ F8 ce_grad8(const F8& v, int64_t col0, int64_t lab, float l2, float w) {
    F8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float p = __builtin_amdgcn_exp2f(fmaf(v.v[j], kLog2e, -l2)) * w;
        o.v[j] = (col0 + j == lab) ? p - w : p;
    }
    return o;
}

template <int F>
__global__ __launch_bounds__(kCeThreads)
void ce_bwd_kernel(const uint16_t* logits, int64_t ld, const int64_t* __restrict__ labels,
                   const float* __restrict__ lse, const float* __restrict__ scale, int64_t V, int64_t ignore_index,
                   uint16_t* dlogits, int64_t ldd) {
    // logits and dlogits may alias (in place): no __restrict__ on them; each thread reads its 8-element
    // chunks before it writes the same chunks, and no two threads touch one chunk
    const int64_t row = blockIdx.x;
    const int64_t lab = labels[row];
    const float w = (lab == ignore_index) ? 0.f : scale[0];
    const float l2 = lse[row] * kLog2e;
    const uint16_t* xr = logits + row * ld;
    uint16_t* dr = dlogits + row * ldd;
    const int64_t n8 = V >> 3;
    int64_t c = threadIdx.x;
    for (; c + kCeThreads < n8; c += 2 * kCeThreads) {
        const F8 a = ld8<F>(xr + c * 8), b = ld8<F>(xr + (c + kCeThreads) * 8);
        st8<F>(dr + c * 8, ce_grad8(a, c * 8, lab, l2, w));
        st8<F>(dr + (c + kCeThreads) * 8, ce_grad8(b, (c + kCeThreads) * 8, lab, l2, w));
    }
    for (; c < n8; c += kCeThreads) st8<F>(dr + c * 8, ce_grad8(ld8<F>(xr + c * 8), c * 8, lab, l2, w));
}

template <bool ADD, int F>
int fwd_reg_dispatch(int cpl, dim3 grid, hipStream_t stream, const uint16_t* x, int64_t ldx, const uint16_t* r, int64_t ldr,
                     const uint16_t* w, uint16_t* h, int64_t ldh, uint16_t* y, int64_t ldy, float* rstd, int64_t rows,
                     int H, float eps) {
#define FWD_REG(C) case C: hipLaunchKernelGGL((rmsnorm_fwd_reg_kernel<C, ADD, false, F>), grid, dim3(256), 0, stream, x, ldx, r, ldr, w, h, ldh, y, ldy, rstd, rows, H, eps, nullptr, 0, nullptr); break;
    switch (cpl) {
        FWD_REG(1) FWD_REG(2) FWD_REG(3) FWD_REG(4) FWD_REG(5) FWD_REG(6) FWD_REG(7) FWD_REG(8)
        FWD_REG(9) FWD_REG(10) FWD_REG(11) FWD_REG(12) FWD_REG(13) FWD_REG(14) FWD_REG(15) FWD_REG(16)
        default: return fail(-1, "rmsnorm: hidden %d", H);
    }
#undef FWD_REG
    return check_launch("rmsnorm_fwd_reg_kernel");
}

template <int F>
int launch_fwd_reg(bool add, const void* x, int64_t ldx, const void* r, int64_t ldr, const void* w, void* h, int64_t ldh,
                   void* y, int64_t ldy, float* rstd, int64_t rows, int H, float eps, hipStream_t stream) {
    const dim3 grid((unsigned)((rows + 3) / 4));
    const int cpl = H / 512;
    if (add)
        return fwd_reg_dispatch<true, F>(cpl, grid, stream, (const uint16_t*)x, ldx, (const uint16_t*)r, ldr,
                                         (const uint16_t*)w, (uint16_t*)h, ldh, (uint16_t*)y, ldy, rstd, rows, H, eps);
    return fwd_reg_dispatch<false, F>(cpl, grid, stream, (const uint16_t*)x, ldx, nullptr, 0, (const uint16_t*)w, nullptr,
                                      0, (uint16_t*)y, ldy, rstd, rows, H, eps);
}

template <bool ADD, int F>
int bwd_reg_dispatch(int cpl, dim3 grid, hipStream_t stream, const uint16_t* dy, int64_t lddy, const uint16_t* x, int64_t ldx,
                     const uint16_t* w, const float* rstd, const uint16_t* dres, int64_t lddr, uint16_t* dx, int64_t lddx,
                     int64_t rows, int H) {
#define BWD_REG(C) case C: hipLaunchKernelGGL((rmsnorm_bwd_reg_kernel<C, ADD, false, F>), grid, dim3(256), 0, stream, dy, lddy, x, ldx, w, rstd, dres, lddr, dx, lddx, rows, H, nullptr, 0, nullptr); break;
    switch (cpl) {
        BWD_REG(1) BWD_REG(2) BWD_REG(3) BWD_REG(4) BWD_REG(5) BWD_REG(6) BWD_REG(7) BWD_REG(8)
        BWD_REG(9) BWD_REG(10) BWD_REG(11) BWD_REG(12) BWD_REG(13) BWD_REG(14) BWD_REG(15) BWD_REG(16)
        default: return fail(-1, "rmsnorm: hidden %d", H);
    }
#undef BWD_REG
    return check_launch("rmsnorm_bwd_reg_kernel");
}

template <int F>
int launch_bwd_reg(bool add, const void* dy, int64_t lddy, const void* x, int64_t ldx, const void* w, const float* rstd,
                   const void* dres, int64_t lddr, void* dx, int64_t lddx, int64_t rows, int H, hipStream_t stream) {
    const dim3 grid((unsigned)((rows + 3) / 4));
    const int cpl = H / 512;
    if (add)
        return bwd_reg_dispatch<true, F>(cpl, grid, stream, (const uint16_t*)dy, lddy, (const uint16_t*)x, ldx,
                                         (const uint16_t*)w, rstd, (const uint16_t*)dres, lddr, (uint16_t*)dx, lddx, rows, H);
    return bwd_reg_dispatch<false, F>(cpl, grid, stream, (const uint16_t*)dy, lddy, (const uint16_t*)x, ldx,
                                      (const uint16_t*)w, rstd, nullptr, 0, (uint16_t*)dx, lddx, rows, H);
}

// dx (with dres: + the residual-path gradient) by the register-resident kernel, then dw: chunk
// partials over rows (at most smt_rmsnorm_bwd_waves(rows) chunks: the caller's partial buffer)
// and the fixed-order reduction.
template <int F>
int launch_bwd_dw(const void* dres, int64_t lddr, const void* dy, int64_t lddy, const void* x, int64_t ldx,
                  const void* w, const float* rstd, void* dx, int64_t lddx, float* dw_partial, void* dw, int64_t rows,
                  int H, hipStream_t stream) {
    if (!dw_partial || !dw || (H % 512) || H > 8192)
        return fail(-1, "smt_rmsnorm_bwd: weight grad needs hidden %% 512 == 0, <= 8192 and a partial buffer");
    int rc = launch_bwd_reg<F>(dres != nullptr, dy, lddy, x, ldx, w, rstd, dres, lddr, dx, lddx, rows, H, stream);
    if (rc) return rc;
    const int64_t cap = smt_rmsnorm_bwd_waves(rows);
    int64_t per = (rows + cap - 1) / cap;
    if (per < 64) per = 64;
    const int64_t n_chunks = (rows + per - 1) / per;
    const unsigned col_blocks = (unsigned)((H / 8 + 255) / 256);
    hipLaunchKernelGGL(rmsnorm_dw_rows_kernel<F>, dim3(col_blocks, (unsigned)n_chunks), dim3(256), 0, stream,
                       (const uint16_t*)dy, lddy, (const uint16_t*)x, ldx, rstd, dw_partial, rows, per, H);
    rc = check_launch("rmsnorm_dw_rows_kernel");
    if (rc) return rc;
    const unsigned out_blocks = (unsigned)((H + 255) / 256);
    hipLaunchKernelGGL(rmsnorm_dw_chunk_kernel, dim3(out_blocks, (unsigned)((n_chunks + kDwChunk - 1) / kDwChunk)),
                       dim3(256), 0, stream, dw_partial, n_chunks, H);
    rc = check_launch("rmsnorm_dw_chunk_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(rmsnorm_dw_kernel<F>, dim3(out_blocks), dim3(256), 0, stream, (const float*)dw_partial, n_chunks, H,
                       (uint16_t*)dw);
    return check_launch("rmsnorm_dw_kernel");
}

// The entry points below take the model's 16-bit dtype (ABI v13: SMT_DTYPE_BF16 or SMT_DTYPE_FP16) and
// run the matching instance of one template body.
#define SMT_FMT_CALL(what, dtype, fn, ...)                                                                     \
    ((dtype) == SMT_DTYPE_BF16   ? fn<SMT_DTYPE_BF16>(__VA_ARGS__)                                              \
     : (dtype) == SMT_DTYPE_FP16 ? fn<SMT_DTYPE_FP16>(__VA_ARGS__)                                              \
                                 : fail(-1, "%s: dtype %d is not a 16-bit format (SMT_DTYPE_BF16 / SMT_DTYPE_FP16)", \
                                        what, (int)(dtype)))

template <int F>
int ce_fwd_impl(const void* logits, int64_t ld, const int64_t* labels, int64_t rows, int64_t vocab, int64_t ignore_index,
                float* lse, float* loss, hipStream_t stream) {
    hipLaunchKernelGGL(ce_fwd_kernel<F>, dim3((unsigned)rows), dim3(kCeThreads), 0, stream, (const uint16_t*)logits, ld,
                       labels, vocab, ignore_index, lse, loss);
    return check_launch("ce_fwd_kernel");
}

template <int F>
int ce_bwd_impl(const void* logits, int64_t ld, const int64_t* labels, const float* lse, const float* scale, int64_t rows,
                int64_t vocab, int64_t ignore_index, void* dlogits, int64_t ld_d, hipStream_t stream) {
    hipLaunchKernelGGL(ce_bwd_kernel<F>, dim3((unsigned)rows), dim3(kCeThreads), 0, stream, (const uint16_t*)logits, ld,
                       labels, lse, scale, vocab, ignore_index, (uint16_t*)dlogits, ld_d);
    return check_launch("ce_bwd_kernel");
}

template <int F>
int rmsnorm_fwd_impl(const void* x, int64_t ld_x, const void* weight, void* y, int64_t ld_y, float* rstd, int64_t rows,
                     int32_t hidden, float eps, hipStream_t stream) {
    if (hidden % 512 == 0 && hidden <= 8192)
        return launch_fwd_reg<F>(false, x, ld_x, nullptr, 0, weight, nullptr, 0, y, ld_y, rstd, rows, hidden, eps, stream);
    hipLaunchKernelGGL(rmsnorm_fwd_kernel<F>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream,
                       (const uint16_t*)x, ld_x, (const uint16_t*)weight, (uint16_t*)y, ld_y, rstd, rows, hidden, eps);
    return check_launch("rmsnorm_fwd_kernel");
}

template <int F>
int rmsnorm_bwd_impl(const void* dy, int64_t ld_dy, const void* x, int64_t ld_x, const void* weight, const float* rstd,
                     void* dx, int64_t ld_dx, float* dw_partial, void* dw, int64_t rows, int32_t hidden, hipStream_t stream) {
    if (dw != nullptr)
        return launch_bwd_dw<F>(nullptr, 0, dy, ld_dy, x, ld_x, weight, rstd, dx, ld_dx, dw_partial, dw, rows, hidden,
                                stream);
    if (hidden % 512 == 0 && hidden <= 8192)
        return launch_bwd_reg<F>(false, dy, ld_dy, x, ld_x, weight, rstd, nullptr, 0, dx, ld_dx, rows, hidden, stream);
    const int n_waves = smt_rmsnorm_bwd_waves(rows);
    hipLaunchKernelGGL(rmsnorm_bwd_kernel<F>, dim3(n_waves / 4), dim3(256), 0, stream, (const uint16_t*)dy, ld_dy,
                       (const uint16_t*)x, ld_x, (const uint16_t*)weight, rstd, (uint16_t*)dx, ld_dx, rows, hidden);
    return check_launch("rmsnorm_bwd_kernel");
}

template <int F>
int rope_impl(bool bwd, const RopeT& tq, const RopeT& tk, const void* cos, const void* sin, int64_t cos_sb, int64_t cos_ss,
              int64_t B, int32_t S, int32_t D, int64_t per_row, hipStream_t stream) {
    // cos / sin loaded once per kRopeHG heads (profiles/r04_nn_rope_hg_ab.jsonl: 141 -> 125 us); one
    // head per thread when the head counts are not multiples of it
    if (tq.H % kRopeHG == 0 && tk.H % kRopeHG == 0) {
        const dim3 hgrid((unsigned)((per_row + 255) / 256), (unsigned)(B * (tq.H + tk.H) / kRopeHG));
        if (bwd)
            hipLaunchKernelGGL((rope_hg_kernel<true, F>), hgrid, dim3(256), 0, stream, tq, tk, (const uint16_t*)cos,
                               (const uint16_t*)sin, cos_sb, cos_ss, S, D);
        else
            hipLaunchKernelGGL((rope_hg_kernel<false, F>), hgrid, dim3(256), 0, stream, tq, tk, (const uint16_t*)cos,
                               (const uint16_t*)sin, cos_sb, cos_ss, S, D);
        return check_launch("rope_hg_kernel");
    }
    const dim3 grid((unsigned)((per_row + 255) / 256), (unsigned)(B * (tq.H + tk.H)));
    if (bwd)
        hipLaunchKernelGGL((rope_kernel<true, F>), grid, dim3(256), 0, stream, tq, tk, (const uint16_t*)cos,
                           (const uint16_t*)sin, cos_sb, cos_ss, B, S, D);
    else
        hipLaunchKernelGGL((rope_kernel<false, F>), grid, dim3(256), 0, stream, tq, tk, (const uint16_t*)cos,
                           (const uint16_t*)sin, cos_sb, cos_ss, B, S, D);
    return check_launch("rope_kernel");
}

template <int F>
int swiglu_fwd_impl(const void* gate, const void* up, void* out, int64_t n8, hipStream_t stream) {
    hipLaunchKernelGGL(swiglu_fwd_kernel<F>, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, stream,
                       (const uint16_t*)gate, (const uint16_t*)up, (uint16_t*)out, n8);
    return check_launch("swiglu_fwd_kernel");
}

template <int F>
int swiglu_bwd_impl(const void* gate, const void* up, const void* grad_out, void* grad_gate, void* grad_up, int64_t n8,
                    hipStream_t stream) {
    hipLaunchKernelGGL(swiglu_bwd_kernel<F>, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, stream,
                       (const uint16_t*)gate, (const uint16_t*)up, (const uint16_t*)grad_out, (uint16_t*)grad_gate,
                       (uint16_t*)grad_up, n8);
    return check_launch("swiglu_bwd_kernel");
}

template <int F>
int colblock_recompute_impl(int32_t op, const void* a, int64_t ld_a, const void* b, int64_t ld_b, const void* weight,
                            const float* rstd, int64_t T, const int32_t* col_blocks_dev, int32_t n_cb, void* out,
                            int64_t blocks, hipStream_t stream) {
    if (op == SMT_RECOMPUTE_RMSNORM)
        hipLaunchKernelGGL((colblock_recompute_kernel<0, F>), dim3((unsigned)blocks), dim3(256), 0, stream,
                           (const uint16_t*)a, ld_a, nullptr, (int64_t)0, (const uint16_t*)weight, rstd, T, col_blocks_dev,
                           n_cb, (uint16_t*)out);
    else
        hipLaunchKernelGGL((colblock_recompute_kernel<1, F>), dim3((unsigned)blocks), dim3(256), 0, stream,
                           (const uint16_t*)a, ld_a, (const uint16_t*)b, ld_b, nullptr, nullptr, T, col_blocks_dev, n_cb,
                           (uint16_t*)out);
    return check_launch("colblock_recompute_kernel");
}

}  // namespace

extern "C" {

const char* smt_model_ops_last_error(void) { return g_err; }

int smt_ce_fwd(const void* logits, int64_t ld, const int64_t* labels, int64_t rows, int64_t vocab,
               int64_t ignore_index, float* lse, float* loss, int32_t dtype, hipStream_t stream) {
    if (rows < 0 || vocab <= 0 || (vocab & 7) || ld < vocab)
        return fail(-1, "smt_ce_fwd: bad sizes rows=%lld vocab=%lld ld=%lld (vocab %% 8 == 0, ld >= vocab)",
                    (long long)rows, (long long)vocab, (long long)ld);
    if (rows == 0) return 0;
    if (!logits || !labels || !lse || !loss) return fail(-1, "smt_ce_fwd: null pointer");
    if (!aligned16(logits) || (ld & 7)) return fail(-2, "smt_ce_fwd: 16-byte aligned rows required");
    if (rows > 0x7fffffffLL) return fail(-1, "smt_ce_fwd: too many rows");
    return SMT_FMT_CALL("smt_ce_fwd", dtype, ce_fwd_impl, logits, ld, labels, rows, vocab, ignore_index, lse, loss, stream);
}

int smt_ce_bwd(const void* logits, int64_t ld, const int64_t* labels, const float* lse, const float* scale,
               int64_t rows, int64_t vocab, int64_t ignore_index, void* dlogits, int64_t ld_d, int32_t dtype,
               hipStream_t stream) {
    if (rows < 0 || vocab <= 0 || (vocab & 7) || ld < vocab || ld_d < vocab)
        return fail(-1, "smt_ce_bwd: bad sizes rows=%lld vocab=%lld", (long long)rows, (long long)vocab);
    if (rows == 0) return 0;
    if (!logits || !labels || !lse || !scale || !dlogits) return fail(-1, "smt_ce_bwd: null pointer");
    if (!aligned16(logits) || !aligned16(dlogits) || (ld & 7) || (ld_d & 7))
        return fail(-2, "smt_ce_bwd: 16-byte aligned rows required");
    if (rows > 0x7fffffffLL) return fail(-1, "smt_ce_bwd: too many rows");
    if (dlogits == logits && ld_d != ld) return fail(-1, "smt_ce_bwd: in place needs ld_d == ld");
    return SMT_FMT_CALL("smt_ce_bwd", dtype, ce_bwd_impl, logits, ld, labels, lse, scale, rows, vocab, ignore_index,
                        dlogits, ld_d, stream);
}

int smt_rmsnorm_fwd(const void* x, int64_t ld_x, const void* weight, void* y, int64_t ld_y, float* rstd,
                    int64_t rows, int32_t hidden, float eps, int32_t dtype, hipStream_t stream) {
    if (rows < 0 || hidden <= 0 || (hidden & 7)) return fail(-1, "smt_rmsnorm_fwd: bad sizes rows=%lld hidden=%d", (long long)rows, hidden);
    if (rows == 0) return 0;
    if (!x || !weight || !y || !rstd) return fail(-1, "smt_rmsnorm_fwd: null pointer");
    if (!aligned16(x) || !aligned16(weight) || !aligned16(y) || (ld_x & 7) || (ld_y & 7))
        return fail(-2, "smt_rmsnorm_fwd: 16-byte aligned rows required");
    return SMT_FMT_CALL("smt_rmsnorm_fwd", dtype, rmsnorm_fwd_impl, x, ld_x, weight, y, ld_y, rstd, rows, hidden, eps,
                        stream);
}

int smt_rmsnorm_fwd_quant_e4m3(const void* x, int64_t ld_x, const void* residual, int64_t ld_r, const void* weight,
                               void* h, int64_t ld_h, void* y, int64_t ld_y, float* rstd, void* out, int64_t ld_out,
                               float* scales, int64_t rows, int32_t hidden, float eps, hipStream_t stream) {
    const int cpl = hidden / 512;
    if (rows < 0 || hidden <= 0 || hidden % 512 || (cpl != 2 && cpl != 4 && cpl != 8 && cpl != 16))
        return fail(-1, "smt_rmsnorm_fwd_quant_e4m3: hidden %d must be 1024, 2048, 4096 or 8192", hidden);
    if (rows == 0) return 0;
    if (!x || !weight || !rstd || !out || !scales || (residual && !h))
        return fail(-1, "smt_rmsnorm_fwd_quant_e4m3: null pointer");
    if (!aligned16(x) || (ld_x & 7) || !aligned16(weight) || (residual && (!aligned16(residual) || (ld_r & 7))) ||
        (h && (!aligned16(h) || (ld_h & 7))) || (y && (!aligned16(y) || (ld_y & 7))) ||
        (reinterpret_cast<uintptr_t>(out) & 7) || (ld_out & 7) || ld_out < hidden)
        return fail(-2, "smt_rmsnorm_fwd_quant_e4m3: 16-byte aligned bf16 rows, 8-byte aligned fp8 rows");
    const dim3 grid((unsigned)((rows + 3) / 4));
    const uint16_t *px = (const uint16_t*)x, *pr = (const uint16_t*)residual, *pw = (const uint16_t*)weight;
    uint16_t *ph = (uint16_t*)h, *py = (uint16_t*)y;
    uint8_t* po = (uint8_t*)out;
#define FWDQ(C)                                                                                                        \
    case C:                                                                                                            \
        if (residual)                                                                                                  \
            hipLaunchKernelGGL((rmsnorm_fwd_reg_kernel<C, true, true>), grid, dim3(256), 0, stream, px, ld_x, pr, ld_r,  \
                               pw, ph, ld_h, py, ld_y, rstd, rows, hidden, eps, po, ld_out, scales);                   \
        else                                                                                                           \
            hipLaunchKernelGGL((rmsnorm_fwd_reg_kernel<C, false, true>), grid, dim3(256), 0, stream, px, ld_x, nullptr,  \
                               (int64_t)0, pw, nullptr, (int64_t)0, py, ld_y, rstd, rows, hidden, eps, po, ld_out,      \
                               scales);                                                                                \
        break;
    switch (cpl) { FWDQ(2) FWDQ(4) FWDQ(8) FWDQ(16) }
#undef FWDQ
    return check_launch("rmsnorm_fwd_reg_kernel<quant>");
}

int smt_add_rmsnorm_fwd(const void* x, int64_t ld_x, const void* residual, int64_t ld_r, const void* weight, void* h,
                        int64_t ld_h, void* y, int64_t ld_y, float* rstd, int64_t rows, int32_t hidden, float eps,
                        int32_t dtype, hipStream_t stream) {
    if (rows < 0 || hidden <= 0 || hidden % 512 || hidden > 8192)
        return fail(-1, "smt_add_rmsnorm_fwd: hidden %d must be a multiple of 512, <= 8192", hidden);
    if (rows == 0) return 0;
    if (!x || !residual || !weight || !h || !y || !rstd) return fail(-1, "smt_add_rmsnorm_fwd: null pointer");
    if (!aligned16(x) || !aligned16(residual) || !aligned16(weight) || !aligned16(h) || !aligned16(y) ||
        (ld_x & 7) || (ld_r & 7) || (ld_h & 7) || (ld_y & 7))
        return fail(-2, "smt_add_rmsnorm_fwd: 16-byte aligned rows required");
    return SMT_FMT_CALL("smt_add_rmsnorm_fwd", dtype, launch_fwd_reg, true, x, ld_x, residual, ld_r, weight, h, ld_h, y,
                        ld_y, rstd, rows, hidden, eps, stream);
}

int smt_rmsnorm_bwd_add(const void* dy, int64_t ld_dy, const void* x, int64_t ld_x, const void* weight, const float* rstd,
                        const void* dres, int64_t ld_dres, void* dx, int64_t ld_dx, int64_t rows, int32_t hidden,
                        int32_t dtype, hipStream_t stream) {
    if (rows < 0 || hidden <= 0 || hidden % 512 || hidden > 8192)
        return fail(-1, "smt_rmsnorm_bwd_add: hidden %d must be a multiple of 512, <= 8192", hidden);
    if (rows == 0) return 0;
    if (!dy || !x || !weight || !rstd || !dres || !dx) return fail(-1, "smt_rmsnorm_bwd_add: null pointer");
    if (!aligned16(dy) || !aligned16(x) || !aligned16(weight) || !aligned16(dres) || !aligned16(dx) || (ld_dy & 7) ||
        (ld_x & 7) || (ld_dres & 7) || (ld_dx & 7))
        return fail(-2, "smt_rmsnorm_bwd_add: 16-byte aligned rows required");
    return SMT_FMT_CALL("smt_rmsnorm_bwd_add", dtype, launch_bwd_reg, true, dy, ld_dy, x, ld_x, weight, rstd, dres,
                        ld_dres, dx, ld_dx, rows, hidden, stream);
}

int smt_rmsnorm_bwd_add_quant_e4m3(const void* dy, int64_t ld_dy, const void* x, int64_t ld_x, const void* weight,
                                   const float* rstd, const void* dres, int64_t ld_dres, void* dx, int64_t ld_dx,
                                   void* out, int64_t ld_out, float* scales, int64_t rows, int32_t hidden,
                                   hipStream_t stream) {
    const int cpl = hidden / 512;
    if (rows < 0 || hidden <= 0 || hidden % 512 || (cpl != 2 && cpl != 4 && cpl != 8 && cpl != 16))
        return fail(-1, "smt_rmsnorm_bwd_add_quant_e4m3: hidden %d must be 1024, 2048, 4096 or 8192", hidden);
    if (rows == 0) return 0;
    if (!dy || !x || !weight || !rstd || !dres || !dx || !out || !scales)
        return fail(-1, "smt_rmsnorm_bwd_add_quant_e4m3: null pointer");
    if (!aligned16(dy) || !aligned16(x) || !aligned16(weight) || !aligned16(dres) || !aligned16(dx) || (ld_dy & 7) ||
        (ld_x & 7) || (ld_dres & 7) || (ld_dx & 7) || (reinterpret_cast<uintptr_t>(out) & 7) || (ld_out & 7) ||
        ld_out < hidden)
        return fail(-2, "smt_rmsnorm_bwd_add_quant_e4m3: 16-byte aligned bf16 rows, 8-byte aligned fp8 rows");
    const dim3 grid((unsigned)((rows + 3) / 4));
    const uint16_t *pdy = (const uint16_t*)dy, *px = (const uint16_t*)x, *pw = (const uint16_t*)weight,
                   *pr = (const uint16_t*)dres;
    uint16_t* pdx = (uint16_t*)dx;
    uint8_t* po = (uint8_t*)out;
#define BWDQ(C)                                                                                                       \
    case C:                                                                                                           \
        hipLaunchKernelGGL((rmsnorm_bwd_reg_kernel<C, true, true>), grid, dim3(256), 0, stream, pdy, ld_dy, px, ld_x, \
                           pw, rstd, pr, ld_dres, pdx, ld_dx, rows, hidden, po, ld_out, scales);                      \
        break;
    switch (cpl) { BWDQ(2) BWDQ(4) BWDQ(8) BWDQ(16) }
#undef BWDQ
    return check_launch("rmsnorm_bwd_reg_kernel<quant>");
}

int smt_rmsnorm_bwd_waves(int64_t rows) {
    const int64_t want = rows < 4096 ? rows : 4096;
    return (int)(want < 4 ? 4 : (want + 3) / 4 * 4);
}

int smt_rmsnorm_bwd(const void* dy, int64_t ld_dy, const void* x, int64_t ld_x, const void* weight, const float* rstd,
                    void* dx, int64_t ld_dx, float* dw_partial, void* dw, int64_t rows, int32_t hidden, int32_t dtype,
                    hipStream_t stream) {
    if (rows < 0 || hidden <= 0 || (hidden & 7)) return fail(-1, "smt_rmsnorm_bwd: bad sizes");
    if (rows == 0) return 0;
    if (!dy || !x || !weight || !rstd || !dx) return fail(-1, "smt_rmsnorm_bwd: null pointer");
    if (!aligned16(dy) || !aligned16(x) || !aligned16(weight) || !aligned16(dx) || (ld_dy & 7) || (ld_x & 7) || (ld_dx & 7))
        return fail(-2, "smt_rmsnorm_bwd: 16-byte aligned rows required");
    return SMT_FMT_CALL("smt_rmsnorm_bwd", dtype, rmsnorm_bwd_impl, dy, ld_dy, x, ld_x, weight, rstd, dx, ld_dx,
                        dw_partial, dw, rows, hidden, stream);
}

int smt_rmsnorm_bwd_add_dw(const void* dy, int64_t ld_dy, const void* x, int64_t ld_x, const void* weight,
                           const float* rstd, const void* dres, int64_t ld_dres, void* dx, int64_t ld_dx,
                           float* dw_partial, void* dw, int64_t rows, int32_t hidden, int32_t dtype,
                           hipStream_t stream) {
    if (rows < 0 || hidden <= 0 || (hidden & 7)) return fail(-1, "smt_rmsnorm_bwd_add_dw: bad sizes");
    if (rows == 0) return 0;
    if (!dy || !x || !weight || !rstd || !dx || !dres) return fail(-1, "smt_rmsnorm_bwd_add_dw: null pointer");
    if (!aligned16(dy) || !aligned16(x) || !aligned16(weight) || !aligned16(dx) || !aligned16(dres) || (ld_dy & 7) ||
        (ld_x & 7) || (ld_dx & 7) || (ld_dres & 7))
        return fail(-2, "smt_rmsnorm_bwd_add_dw: 16-byte aligned rows required");
    return SMT_FMT_CALL("smt_rmsnorm_bwd_add_dw", dtype, launch_bwd_dw, dres, ld_dres, dy, ld_dy, x, ld_x, weight, rstd, dx,
                        ld_dx, dw_partial, dw, rows, hidden, stream);
}

static int rope(bool bwd, const smt_rope_tensor* q, const smt_rope_tensor* k, const void* cos, const void* sin,
                int64_t cos_sb, int64_t cos_ss, int64_t B, int32_t S, int32_t D, int32_t dtype, hipStream_t stream) {
    if (!q || !k || !cos || !sin) return fail(-1, "smt_rope: null pointer");
    if (B < 0 || S < 0 || D <= 0 || (D & 15)) return fail(-1, "smt_rope: head_dim %d must be a multiple of 16", D);
    RopeT tq{(const uint16_t*)q->in, (uint16_t*)q->out, q->in_sb, q->in_sh, q->in_ss, q->out_sb, q->out_sh, q->out_ss, q->heads};
    RopeT tk{(const uint16_t*)k->in, (uint16_t*)k->out, k->in_sb, k->in_sh, k->in_ss, k->out_sb, k->out_sh, k->out_ss, k->heads};
    const void* ptrs[] = {q->in, q->out, k->in, k->out, cos, sin};
    for (const void* p : ptrs) if (!aligned16(p)) return fail(-2, "smt_rope: 16-byte alignment required");
    const int64_t strides[] = {q->in_sb, q->in_sh, q->in_ss, q->out_sb, q->out_sh, q->out_ss,
                               k->in_sb, k->in_sh, k->in_ss, k->out_sb, k->out_sh, k->out_ss, cos_sb, cos_ss};
    for (int64_t s : strides) if (s & 7) return fail(-2, "smt_rope: strides must be multiples of 8 elements");
    const int64_t rows = B * (int64_t)(q->heads + k->heads);
    const int64_t per_row = (int64_t)S * (D / 16);
    if (rows == 0 || per_row == 0) return 0;
    if (rows > 65535 || per_row > 0x7fffffffLL - 255)
        return fail(-1, "smt_rope: %lld (batch x heads) rows of %lld chunks exceed the grid", (long long)rows,
                    (long long)per_row);
    return SMT_FMT_CALL("smt_rope", dtype, rope_impl, bwd, tq, tk, cos, sin, cos_sb, cos_ss, B, S, D, per_row, stream);
}

int smt_rope_fwd(const smt_rope_tensor* q, const smt_rope_tensor* k, const void* cos, const void* sin,
                 int64_t cos_sb, int64_t cos_ss, int64_t B, int32_t S, int32_t D, int32_t dtype, hipStream_t stream) {
    return rope(false, q, k, cos, sin, cos_sb, cos_ss, B, S, D, dtype, stream);
}

int smt_rope_bwd(const smt_rope_tensor* dq, const smt_rope_tensor* dk, const void* cos, const void* sin,
                 int64_t cos_sb, int64_t cos_ss, int64_t B, int32_t S, int32_t D, int32_t dtype, hipStream_t stream) {
    return rope(true, dq, dk, cos, sin, cos_sb, cos_ss, B, S, D, dtype, stream);
}

int smt_swiglu_fwd(const void* gate, const void* up, void* out, int64_t n, int32_t dtype, hipStream_t stream) {
    if (n < 0 || (n & 7)) return fail(-1, "smt_swiglu_fwd: n %lld must be a multiple of 8", (long long)n);
    if (n == 0) return 0;
    if (!aligned16(gate) || !aligned16(up) || !aligned16(out)) return fail(-2, "smt_swiglu_fwd: alignment");
    return SMT_FMT_CALL("smt_swiglu_fwd", dtype, swiglu_fwd_impl, gate, up, out, n / 8, stream);
}

int smt_swiglu_bwd(const void* gate, const void* up, const void* grad_out, void* grad_gate, void* grad_up, int64_t n,
                   int32_t dtype, hipStream_t stream) {
    if (n < 0 || (n & 7)) return fail(-1, "smt_swiglu_bwd: n %lld must be a multiple of 8", (long long)n);
    if (n == 0) return 0;
    if (!aligned16(gate) || !aligned16(up) || !aligned16(grad_out) || !aligned16(grad_gate) || !aligned16(grad_up))
        return fail(-2, "smt_swiglu_bwd: alignment");
    return SMT_FMT_CALL("smt_swiglu_bwd", dtype, swiglu_bwd_impl, gate, up, grad_out, grad_gate, grad_up, n / 8, stream);
}

int smt_colblock_recompute(int32_t op, const void* a, int64_t ld_a, const void* b, int64_t ld_b, const void* weight,
                           const float* rstd, int64_t T, const int32_t* col_blocks_dev, int32_t n_cb, void* out,
                           int32_t dtype, hipStream_t stream) {
    if (op != SMT_RECOMPUTE_RMSNORM && op != SMT_RECOMPUTE_SWIGLU)
        return fail(-1, "smt_colblock_recompute: unknown op %d", (int)op);
    if (T < 0 || n_cb < 0 || ld_a < 0 || ld_b < 0) return fail(-1, "smt_colblock_recompute: negative size");
    if (T == 0 || n_cb == 0) return 0;
    if (!a || !out || !col_blocks_dev) return fail(-1, "smt_colblock_recompute: null pointer");
    if (op == SMT_RECOMPUTE_RMSNORM && (!weight || !rstd)) return fail(-1, "smt_colblock_recompute: null weight/rstd");
    if (op == SMT_RECOMPUTE_SWIGLU && !b) return fail(-1, "smt_colblock_recompute: null up operand");
    if (!aligned16(a) || !aligned16(out) || (ld_a & 7) || (op == SMT_RECOMPUTE_SWIGLU && (!aligned16(b) || (ld_b & 7))) ||
        (op == SMT_RECOMPUTE_RMSNORM && !aligned16(weight)))
        return fail(-2, "smt_colblock_recompute: 16-byte aligned rows required");
    const int64_t blocks = (T * n_cb * 32 + 255) / 256;
    if (blocks > 0x7fffffffLL) return fail(-1, "smt_colblock_recompute: too large");
    return SMT_FMT_CALL("smt_colblock_recompute", dtype, colblock_recompute_impl, op, a, ld_a, b, ld_b, weight, rstd, T,
                        col_blocks_dev, n_cb, out, blocks, stream);
}

}  // extern "C"
