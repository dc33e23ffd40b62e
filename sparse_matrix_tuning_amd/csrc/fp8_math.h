// e4m3 (OCP float8_e4m3fn) helpers shared by the quantisation kernels (fp8_kernels.hip) and the
// producers that quantise their own output (llama_kernels.hip: RMSNorm).
#pragma once
#include <stdint.h>

constexpr float kE4M3Max = 448.f;
constexpr float kInvE4M3Max = 1.f / 448.f;          // fp32-rounded reciprocal: scale = amax * (1/448)

// x / scale, correctly rounded (so bit-identical to torch's IEEE division) without a per-element
// division: with rs = RN(1/scale), q0 = RN(x * rs) is within an ulp of the quotient, the residual
// x - q0 * scale is exact in one FMA, and RN(q0 + residual * rs) is the correctly rounded quotient
// (Markstein). 1/scale is loop-invariant per row / column, so the one real division is hoisted.
// The quotient stays within +-448 (|x| <= amax = 448 * scale), far from overflow and underflow.
__device__ __forceinline__ float qv(float x, float scale) {
    const float rs = 1.f / scale;
    const float q0 = x * rs;
    const float r = __builtin_fmaf(-q0, scale, x);
    return __builtin_amdgcn_fmed3f(__builtin_fmaf(r, rs, q0), kE4M3Max, -kE4M3Max);
}

// four values -> four e4m3 bytes (little endian: a is byte 0)
__device__ __forceinline__ uint32_t pack4(float a, float b, float c, float d) {
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
    return (uint32_t)w;
}

// the scale of a row / column with this amax (1 for an all-zero one)
__device__ __forceinline__ float e4m3_scale(float amax) { return amax > 0.f ? amax * kInvE4M3Max : 1.f; }
