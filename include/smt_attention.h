/*
 * smt_attention.h — C-ABI of the gfx950 causal flash attention (forward + backward) used by the SMT
 * training step (csrc/attn_kernels.hip, same library libsmt_hip.so).
 *
 * Auxiliary to the SMT hot path (smt_hip.h): it replaces the attention of the HF transformers LLaMA
 * decoder that carries the SMT modules (the reference trains that model through
 * AutoModelForCausalLM, deepspeed/fine_tune.py:150-155; transformers' sdpa attention dispatches to
 * aotriton on this torch build). Causal, grouped-query (Hq = G * Hkv), head_dim 128, 16-bit in / out
 * (shape->dtype: SMT_DTYPE_BF16 or, since ABI v13, SMT_DTYPE_FP16 -- the reference's --dtype,
 * fine_tune.py:955-959), fp32 softmax statistics; P and dS are rounded to that format for their
 * products.
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
    int32_t dtype;                  /* ABI v13 (was padding, 0): SMT_DTYPE_BF16 (0) or SMT_DTYPE_FP16 (2) */
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

/*
 * The same with a key mask (ABI v8): the attention of a padded batch, as transformers builds it from
 * the 2-D attention_mask the reference's collator passes (input_ids != pad_token_id,
 * deepspeed/helpers/helper.py:194-204), combined with the causal mask. key_mask: device uint64
 * [B][key_mask_ld], key_mask_ld >= ceil(S / 64); bit (j & 63) of word b*key_mask_ld + (j >> 6) set =
 * key j of batch b takes part. The mask may have holes anywhere (a pad id can occur inside a
 * sequence). A query row whose visible keys are all masked gets o = 0, lse = +inf and zero
 * gradients (torch's safe softmax). key_mask NULL = smt_attn_fwd / smt_attn_bwd.
 */
int smt_attn_fwd_kmask(const smt_attn_tensor* q, const smt_attn_tensor* k, const smt_attn_tensor* v,
                       const smt_attn_tensor* o, float* lse, const uint64_t* key_mask, int64_t key_mask_ld,
                       const smt_attn_shape* shape, hipStream_t stream);
int smt_attn_bwd_kmask(const smt_attn_tensor* q, const smt_attn_tensor* k, const smt_attn_tensor* v,
                       const smt_attn_tensor* o, const smt_attn_tensor* d_o, const float* lse, float* delta_ws,
                       const smt_attn_tensor* dq, const smt_attn_tensor* dk, const smt_attn_tensor* dv,
                       const uint64_t* key_mask, int64_t key_mask_ld, const smt_attn_shape* shape,
                       hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SMT_ATTENTION_H */
