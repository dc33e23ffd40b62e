/*
 * smt_fp8.h — C-ABI of the fp8 (OCP e4m3) quantisation kernels of the SMT fp8 path
 * (BASELINE.json config 5; csrc/fp8_kernels.hip, same library libsmt_hip.so).
 *
 * The reference has no fp8 anywhere (bf16/fp16/fp32 only, deepspeed/fine_tune.py:955-959), so this
 * path has no reference counterpart: parity is stated against the build's own bf16 path.
 * The frozen weights of the decoder layers are kept as e4m3 copies with one fp32 scale per row
 * (forward, W [out, in]) and per column (data gradient, written transposed as W^T [in, out]), and the
 * activations / output gradients are quantised per row (token) on the fly; the GEMMs then run as
 * hipBLASLt rowwise-scaled fp8 GEMMs. After every optimizer step the rows / columns that the
 * updated 256x256 tiles touch are re-quantised from the bf16 W (whose tiles the AdamW epilogue wrote).
 *
 * Quantisation (both kernels): scale = amax * fp32(1/448) (1 when amax == 0), q = e4m3_rne(x / scale),
 * with x / scale an IEEE fp32 division, so the bytes equal torch's
 * (x.float() / scale).to(torch.float8_e4m3fn).
 * Return 0 or a negative code; smt_fp8_last_error() holds the message.
 */
#ifndef SMT_FP8_H
#define SMT_FP8_H

#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* smt_fp8_last_error(void);

/*
 * Row-wise: out[r, 0:cols] = e4m3(x[r, 0:cols] / scales[r]) for every row r of x (bf16 [rows, ld_x]),
 * or, when row_blocks_dev != NULL, only for the rows of the listed 256-row blocks (device int32 [n]).
 * out: fp8 bytes [rows, ld_out]; scales: fp32 [rows]. cols % 8 == 0; 16-byte aligned bf16 rows.
 */
int smt_quant_rows_e4m3(const void* x, int64_t ld_x, int64_t rows, int32_t cols, const int32_t* row_blocks_dev,
                        int32_t n_row_blocks, void* out, int64_t ld_out, float* scales, hipStream_t stream);

/* One bf16 source of a row-wise concatenation. */
typedef struct smt_quant_src {
    const void* ptr;                /* bf16 [rows, ld], 16-byte aligned rows */
    int64_t ld;
    int32_t cols;                   /* % 8 == 0 */
    int32_t pad_;
} smt_quant_src;

/*
 * Row-wise over the concatenation [src_0 | ... | src_{n-1}] (1 <= n <= 4, <= 32768 columns in all):
 * one scale per row over all sources; out: fp8 [rows, ld_out] holding the concatenated row.
 * (The output gradients of linears that share one input -- q/k/v, gate/up -- for ONE joint
 * data-gradient GEMM.)
 */
int smt_quant_rows_cat_e4m3(const smt_quant_src* srcs, int32_t n_src, int64_t rows, void* out, int64_t ld_out,
                            float* scales, hipStream_t stream);

/*
 * Column-wise, transposed: out_t[c, 0:rows] = e4m3(w[0:rows, c] / scales[c]) for every column c of
 * w (bf16 [rows, ld_w], cols % 256 == 0), or only the columns of the listed 256-column blocks.
 * out_t: fp8 bytes [cols, ld_out] (the transposed matrix); scales: fp32 [cols]. rows % 64 == 0.
 */
int smt_quant_cols_t_e4m3(const void* w, int64_t ld_w, int32_t rows, int32_t cols, const int32_t* col_blocks_dev,
                          int32_t n_col_blocks, void* out_t, int64_t ld_out, float* scales, hipStream_t stream);

/* RMSNorm forward (smt_rmsnorm_fwd; with residual != NULL smt_add_rmsnorm_fwd, h = bf16(x + residual))
 * that also writes its bf16 output y as one e4m3 row per token: out[rows, hidden] + scales[rows],
 * bit-identical to the bf16 kernel followed by smt_quant_rows_e4m3. y may be NULL when no consumer
 * reads the bf16 output (a frozen fp8 q/k/v or gate/up group). hidden in {1024, 2048, 4096, 8192}.
 * (Defined in llama_kernels.hip next to the RMSNorm kernels.) */
int smt_rmsnorm_fwd_quant_e4m3(const void* x, int64_t ld_x, const void* residual, int64_t ld_r, const void* weight,
                               void* h, int64_t ld_h, void* y, int64_t ld_y, float* rstd, void* out, int64_t ld_out,
                               float* scales, int64_t rows, int32_t hidden, float eps, hipStream_t stream);

/* smt_rmsnorm_bwd_add (RMSNorm backward plus the residual gradient, dx = bf16(bf16(dx_norm) + dres))
 * that also writes dx as one e4m3 row per token (out[rows, hidden] + scales[rows]) for the fp8
 * linear consuming that gradient (o_proj, down_proj), bit-identical to smt_quant_rows_e4m3 of dx.
 * hidden in {1024, 2048, 4096, 8192}. (Defined in llama_kernels.hip.) */
int smt_rmsnorm_bwd_add_quant_e4m3(const void* dy, int64_t ld_dy, const void* x, int64_t ld_x, const void* weight,
                                   const float* rstd, const void* dres, int64_t ld_dres, void* dx, int64_t ld_dx,
                                   void* out, int64_t ld_out, float* scales, int64_t rows, int32_t hidden,
                                   hipStream_t stream);

/* SwiGLU forward (smt_swiglu_fwd's formula and roundings) fused with the per-row quantisation of
 * its output: out[rows, cols] e4m3 + scales[rows], bit-identical to smt_swiglu_fwd followed by
 * smt_quant_rows_e4m3; the bf16 output is written to h_out only when it is non-NULL.
 * gate / up / h_out contiguous [rows, cols] bf16, cols % 8 == 0, <= 16384. */
int smt_swiglu_fwd_quant_e4m3(const void* gate, const void* up, int64_t rows, int32_t cols, void* out, int64_t ld_out,
                              float* scales, void* h_out, hipStream_t stream);

/* SwiGLU backward (transformers LlamaMLP, act = SiLU; the formula and bf16 roundings of
 * smt_swiglu_bwd in smt_model_ops.h) fused with the per-row quantisation of [grad_gate | grad_up]:
 * out[rows, 2*cols] e4m3 (ld_out >= 2*cols) with one scale per row over both, bit-identical to
 * smt_swiglu_bwd + smt_quant_rows_cat_e4m3. gate / up / grad_out are contiguous [rows, cols] bf16;
 * grad_gate / grad_up (same layout) are written only when non-NULL. cols % 8 == 0, <= 16384. */
int smt_swiglu_bwd_quant_e4m3(const void* gate, const void* up, const void* grad_out, int64_t rows, int32_t cols,
                              void* out, int64_t ld_out, float* scales, void* grad_gate, void* grad_up,
                              hipStream_t stream);

/* smt_swiglu_bwd_quant_e4m3 writing only some 256-column blocks of grad_gate / grad_up (fp8 path, an
 * SMT gate/up module with MX tile gradients: the blocks its tiles read, in its row-block order, so
 * the full bf16 gradient the data-gradient GEMM never reads is not written). gate_pos / up_pos:
 * device int32 [cols / 256], the block's position in the packed gradient or -1 (NULL: every block, at
 * its own column); grad_x is [rows, ld_x] bf16 and block b lands at column 256 * pos[b] (positions
 * past ld_x / 256 are not written). cols % 256 == 0 with a map. Replaces the reference's bf16
 * grad_output of gate/up, which linearZ.backward slices per tile (smt.py:382-404). */
int smt_swiglu_bwd_quant_e4m3_packed(const void* gate, const void* up, const void* grad_out, int64_t rows,
                                     int32_t cols, void* out, int64_t ld_out, float* scales, void* grad_gate,
                                     const int32_t* gate_pos, int64_t ld_gate, void* grad_up, const int32_t* up_pos,
                                     int64_t ld_up, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SMT_FP8_H */
