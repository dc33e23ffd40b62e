/*
 * smt_attention.h — C-ABI of the gfx950 causal flash attention (forward + backward) used by the SMT
 * training step (csrc/attn_kernels.hip, same library libsmt_hip.so).
 *
 * Auxiliary to the SMT hot path (smt_hip.h): it replaces the attention of the HF transformers LLaMA
 * decoder that carries the SMT modules (the reference trains that model through
 * AutoModelForCausalLM, deepspeed/fine_tune.py:150-155; transformers' sdpa attention dispatches to
 * aotriton on this torch build). Causal, grouped-query (Hq = G * Hkv), head_dim 128, bf16 in / out,
 * fp32 softmax statistics.
 *
 * Tensors are addressed by element strides (d-stride 1, rows 16-byte aligned):
 *   q, o, dq, do   element (b, h, s, d) at base + b*sb + h*sh + s*ss + d,  h < Hq
 *   k, v, dk, dv   element (b, h, s, d) at base + b*sb + h*sh + s*ss + d,  h < Hkv
 *   lse, delta     fp32 [B][Hq][S]; lse in log2 units of the scaled scores:
 *                  lse = log2(sum_j exp2(scale*log2(e) * q.k_j))
 * Returns 0 or a negative code; smt_attn_last_error() holds the message.
 */
#ifndef SMT_ATTENTION_H
#define SMT_ATTENTION_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SMT_ATTN_HEAD_DIM 128

typedef struct smt_attn_tensor {
    void* ptr;
    int64_t sb, sh, ss;             /* element strides of batch, head, sequence */
} smt_attn_tensor;

typedef struct smt_attn_shape {
    int32_t B, Hq, Hkv, S;
    float scale;                    /* softmax scale, usually 1/sqrt(128) */
    int32_t pad_;
} smt_attn_shape;

const char* smt_attn_last_error(void);

/* o = softmax(scale * q k^T + causal mask) v ; lse as above. */
int smt_attn_fwd(const smt_attn_tensor* q, const smt_attn_tensor* k, const smt_attn_tensor* v,
                 const smt_attn_tensor* o, float* lse, const smt_attn_shape* shape, hipStream_t stream);

/*
 * Gradients of smt_attn_fwd. delta_ws: fp32 [B][Hq][S] workspace (delta = rowsum(do * o)).
 * dk / dv sum the G query heads that share a key/value head (no atomics; deterministic).
 */
int smt_attn_bwd(const smt_attn_tensor* q, const smt_attn_tensor* k, const smt_attn_tensor* v,
                 const smt_attn_tensor* o, const smt_attn_tensor* d_o, const float* lse, float* delta_ws,
                 const smt_attn_tensor* dq, const smt_attn_tensor* dk, const smt_attn_tensor* dv,
                 const smt_attn_shape* shape, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SMT_ATTENTION_H */
