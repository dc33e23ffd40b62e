// SiLU pieces shared by every SwiGLU kernel (llama_kernels.hip, and the fp8 fusions in
// fp8_kernels.hip, which must produce bit-identical bf16 values to the unfused kernels).
// sigmoid(x) = 1 / (1 + 2^(-x log2 e)) with the hardware v_exp_f32 / v_rcp_f32 (about 1 ulp each)
// instead of the libm-accurate expf and an IEEE division: a few fp32 ulps from transformers' eager
// silu (x / (1 + exp(-x))), i.e. after the bf16 rounding an occasional one-step difference, which
// the tests bound (tests/test_gpu_fused_llama.py, <= 1e-3 of the values one bf16 step apart).
#pragma once

__device__ __forceinline__ float smt_sigmoid(float x) {
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-x * 1.4426950408889634f));
}
