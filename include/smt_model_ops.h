/*
 * smt_model_ops.h — C-ABI of the fused LLaMA elementwise kernels used by the SMT training step
 * (csrc/llama_kernels.hip, same library libsmt_hip.so). Auxiliary to the SMT hot path (smt_hip.h):
 * they replace eager op chains of the HF transformers LLaMA decoder that carries the SMT modules
 * (the reference trains that model through AutoModelForCausalLM, deepspeed/fine_tune.py:150-155):
 *   smt_rmsnorm_fwd/bwd   transformers LlamaRMSNorm.forward (+ autograd of its op chain)
 *   smt_add_rmsnorm_fwd / smt_rmsnorm_bwd_add   LlamaDecoderLayer's residual add fused into the
 *                         post-attention RMSNorm (forward) and its gradient sum (backward)
 *   smt_rope_fwd/bwd      transformers apply_rotary_pos_emb
 *   smt_swiglu_fwd/bwd    transformers LlamaMLP.forward: act_fn(gate_proj(x)) * up_proj(x), act = SiLU
 * 16-byte aligned rows; every intermediate rounding of the eager chain to the model's dtype is kept.
 * ABI v13: every entry point below (except the fp8 producer fusions of smt_fp8.h, bf16 models only)
 * takes `dtype`, the model's 16-bit format -- SMT_DTYPE_BF16 (0) or SMT_DTYPE_FP16 (2) of smt_hip.h,
 * the reference's --dtype bf16 | fp16 (fine_tune.py:955-959) -- and reads and writes every 16-bit
 * tensor in it; the formulas below write "bf16(...)" for "rounded to that format". Any other value
 * fails with SMT_E_INVALID.
 * Return 0 or a negative code; smt_model_ops_last_error() holds the message.
 */
#ifndef SMT_MODEL_OPS_H
#define SMT_MODEL_OPS_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

/* A [B, heads, S, D] 16-bit tensor and its output, element strides (d-stride 1). */
typedef struct smt_rope_tensor {
    const void* in;
    void* out;
    int64_t in_sb, in_sh, in_ss;
    int64_t out_sb, out_sh, out_ss;
    int32_t heads;
    int32_t pad_;
} smt_rope_tensor;

const char* smt_model_ops_last_error(void);

/* y = w * bf16(x * rsqrt(mean(x^2) + eps)); rstd[rows] (fp32) saved for the backward. */
int smt_rmsnorm_fwd(const void* x, int64_t ld_x, const void* weight, void* y, int64_t ld_y, float* rstd,
                    int64_t rows, int32_t hidden, float eps, int32_t dtype, hipStream_t stream);

/* LlamaDecoderLayer's `h = residual + attn_out; post_attention_layernorm(h)` in one pass:
 * h = bf16(x + residual) is written to h and normalised into y (rstd saved). hidden % 512 == 0, <= 8192. */
int smt_add_rmsnorm_fwd(const void* x, int64_t ld_x, const void* residual, int64_t ld_r, const void* weight, void* h,
                        int64_t ld_h, void* y, int64_t ld_y, float* rstd, int64_t rows, int32_t hidden, float eps,
                        int32_t dtype, hipStream_t stream);

/* RMSNorm backward (no weight grad) plus the gradient reaching the same input by the residual path:
 * dx = bf16(bf16(dx_norm) + dres), as autograd's sum of the two. hidden % 512 == 0, <= 8192. */
int smt_rmsnorm_bwd_add(const void* dy, int64_t ld_dy, const void* x, int64_t ld_x, const void* weight, const float* rstd,
                        const void* dres, int64_t ld_dres, void* dx, int64_t ld_dx, int64_t rows, int32_t hidden,
                        int32_t dtype, hipStream_t stream);

/* Number of waves (and rows of dw_partial) smt_rmsnorm_bwd uses for `rows` rows. */
int smt_rmsnorm_bwd_waves(int64_t rows);

/* dx (and, if dw != NULL, dw via dw_partial[smt_rmsnorm_bwd_waves(rows)][hidden] fp32). */
int smt_rmsnorm_bwd(const void* dy, int64_t ld_dy, const void* x, int64_t ld_x, const void* weight, const float* rstd,
                    void* dx, int64_t ld_dx, float* dw_partial, void* dw, int64_t rows, int32_t hidden,
                    int32_t dtype, hipStream_t stream);

/* smt_rmsnorm_bwd with the weight gradient AND the residual-path gradient (the full fine-tuning
 * warm-up's LlamaDecoderLayer norms): dx = bf16(bf16(dx_norm) + dres), dw = bf16(sum_rows bf16(dy *
 * bf16(x * rstd))) via dw_partial[smt_rmsnorm_bwd_waves(rows)][hidden] fp32 (overwritten).
 * hidden % 512 == 0, <= 8192. (ABI 7) */
int smt_rmsnorm_bwd_add_dw(const void* dy, int64_t ld_dy, const void* x, int64_t ld_x, const void* weight,
                           const float* rstd, const void* dres, int64_t ld_dres, void* dx, int64_t ld_dx,
                           float* dw_partial, void* dw, int64_t rows, int32_t hidden, int32_t dtype,
                           hipStream_t stream);

/* q/k rotary embedding (one launch for both); cos/sin [B, S, D] with strides (cos_sb, cos_ss, 1). */
int smt_rope_fwd(const smt_rope_tensor* q, const smt_rope_tensor* k, const void* cos, const void* sin,
                 int64_t cos_sb, int64_t cos_ss, int64_t B, int32_t S, int32_t D, int32_t dtype, hipStream_t stream);
int smt_rope_bwd(const smt_rope_tensor* dq, const smt_rope_tensor* dk, const void* cos, const void* sin,
                 int64_t cos_sb, int64_t cos_ss, int64_t B, int32_t S, int32_t D, int32_t dtype, hipStream_t stream);

/* out = bf16(silu(gate)) * up ; backward recomputes silu from gate. n % 8 == 0. */
int smt_swiglu_fwd(const void* gate, const void* up, void* out, int64_t n, int32_t dtype, hipStream_t stream);
int smt_swiglu_bwd(const void* gate, const void* up, const void* grad_out, void* grad_gate, void* grad_up, int64_t n,
                   int32_t dtype, hipStream_t stream);

/* Activation policy "selective" (ABI 9): the 256-column blocks linearZ's tile weight gradient reads,
 * rebuilt in the backward from the producer's saved operands instead of kept from the forward
 * (deepspeed/smt/smt.py:351-358 keeps them as ctx.list1). Same block-major output as
 * smt_colblock_gather (out[j][t][256] = value[t, col_blocks[j]*256 + k]) and bit-identical values:
 *   SMT_RECOMPUTE_RMSNORM: value = bf16(float(w) * float(bf16(a * rstd[t])))   (smt_rmsnorm_fwd's y)
 *   SMT_RECOMPUTE_SWIGLU:  value = bf16(float(bf16(silu(a))) * b)            (smt_swiglu_fwd's out)
 * a / b: [T, >= cols] bf16 rows with leading dimensions ld_a / ld_b; weight: the norm's [cols] bf16;
 * rstd: the norm's saved [T] fp32; col_blocks_dev: device int32 [n_cb]. */
#define SMT_RECOMPUTE_RMSNORM 0
#define SMT_RECOMPUTE_SWIGLU 1
int smt_colblock_recompute(int32_t op, const void* a, int64_t ld_a, const void* b, int64_t ld_b, const void* weight,
                           const float* rstd, int64_t T, const int32_t* col_blocks_dev, int32_t n_cb, void* out,
                           int32_t dtype, hipStream_t stream);

/* Causal-LM cross entropy over 16-bit logits [rows, vocab] (transformers ForCausalLMLoss:
 * logits.float() -> log_softmax -> nll), without materialising fp32 logits.
 * Forward:  lse[r] = logsumexp(float(logits[r, :]));  loss[r] = lse[r] - float(logits[r, label[r]]),
 *           0 where label[r] == ignore_index, NaN where the label is outside [0, vocab).
 * Backward: dlogits[r, j] = bf16((exp(logits[r, j] - lse[r]) - [j == label[r]]) * scale[0]),
 *           0 on ignored rows. `scale` is a device float (d loss / normaliser), so no host sync.
 *           `dlogits` may be `logits` itself (ld_d == ld): every element is read and then written
 *           by the same thread (the fused LM head + loss runs it in place over a chunk's logits).
 * vocab % 8 == 0, 16-byte aligned rows. */
int smt_ce_fwd(const void* logits, int64_t ld, const int64_t* labels, int64_t rows, int64_t vocab,
               int64_t ignore_index, float* lse, float* loss, int32_t dtype, hipStream_t stream);
int smt_ce_bwd(const void* logits, int64_t ld, const int64_t* labels, const float* lse, const float* scale,
               int64_t rows, int64_t vocab, int64_t ignore_index, void* dlogits, int64_t ld_d, int32_t dtype,
               hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SMT_MODEL_OPS_H */
