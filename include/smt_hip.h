/*
 * smt_hip.h — C-ABI of the MI355X (gfx950) SMT block-sparse fine-tuning hot path.
 *
 * Every entry point takes borrowed device pointers, sizes and a hipStream_t, never
 * allocates or frees caller memory (workspaces are passed in), is enqueued on the
 * given stream without a host synchronisation, and returns 0 on success or a
 * negative SMT_E* code; smt_last_error() then returns a thread-local message.
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * yudaohai666/Sparse_Matrix_Tuning snapshot):
 *   smt_tile_gather       deepspeed/smt/smt.py:317-325   tile copy W -> selected_weight
 *   smt_tile_scatter      deepspeed/smt/smt.py:332-341   per-forward write-back tiles -> W
 *                         (also smt.py:429-439, the merge in convert_matrix_sparsity_to_linear_layer)
 *   smt_tile_wgrad        deepspeed/smt/smt.py:382-404   per-tile sum_b g[b,:,rows]^T x[b,:,cols]
 *   smt_tile_wgrad_batch  the same, for the tiles of several modules in one launch (ABI v6)
 *   smt_tile_wgrad_batch_seq  the same with the reference's rounding: every per-sample [256, 256]
 *                         partial rounded to bf16, then the batch sum (smt.py:397-404, ABI v8)
 *   smt_tile_scatter_t    deepspeed/smt/smt.py:332-341 / 406   write-back into the transposed copy W^T
 *                         that the data-gradient GEMM grad_input = g @ W reads (as g @ (W^T)^T)
 *   smt_colblock_gather   deepspeed/smt/smt.py:351-358   ctx.list1: the input column slices linearZ keeps
 *                         for its backward (block-major copy of the distinct 256-column blocks)
 *   smt_grad_accumulate   deepspeed/fine_tune.py:724-741, 751-764   warm-up fp32 grad harvest
 *   smt_block_score       deepspeed/smt/smt_helper.py:67-78, 233-251   per-256x256-block scores
 *                         (fp64 sum + magnitude sum: the host bounds ATen's fp32 value with them)
 *   smt_sq_norm           DeepSpeed bf16/ZeRO global grad-norm for gradient_clipping=1.0
 *                         (deepspeed/helpers/deepspeed_helpers.py:87; DeepSpeed 0.16.5, external)
 *   smt_adamw_step        DeepSpeed FusedAdam(adam_w_mode=True) step over the tiles
 *                         (deepspeed/fine_tune.py:352,361-363,773; DeepSpeed 0.16.5, external),
 *                         fused with clip, bf16 cast and the tile -> W scatter
 *   smt_mx_quant_cols,    MX-fp8 (e4m3 + e8m0 per 32 tokens) column blocks and the tile weight
 *   smt_tile_wgrad_mx     gradient over them (config 5's fp8 tiles; no reference counterpart);
 *   smt_tile_wgrad_mx_batch  the same for several modules in one launch (ABI v6)
 *   smt_adamw_multi       the same step over many dense parameters in one launch (the warm-up
 *                         full fine-tune's FusedAdam multi_tensor_apply, fine_tune.py:352-363)
 *   Channel path (activation-selected rows; SURVEY §8(f) row 1, ABI v3):
 *   smt_row_gather        deepspeed/smt/smt.py:200-204   selected_weight[i, :] = W[index_list[i], :]
 *   smt_row_scatter       deepspeed/smt/smt.py:211-213   per-forward write-back rows -> W
 *   smt_column_gather     deepspeed/smt/smt.py:225-233   partial_input[:, :, i] = input[:, :, index_list[i]]
 *   smt_act_accumulate    deepspeed/fine_tune.py:636-667 (cache_input_hook: the fp32 [B, S, in]
 *                         accumulator `feat[key] (+)= |x|` over steps)
 *   smt_channel_score     deepspeed/smt/smt_helper.py:167-184   per-channel statistic (batch sum of
 *                         smt_helper.py:170, then the sequence reduction) in fp64
 *   smt_channel_mean_aten deepspeed/smt/smt_helper.py:167-176   the mean statistic in ATen's own CPU
 *                         summation order (bit-identical values; ABI v6)
 */
#ifndef SMT_HIP_H
#define SMT_HIP_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SMT_BLOCK_DIM 256           /* deepspeed/smt/smt.py:22 Block_dimension */

/* status codes */
#define SMT_OK 0
#define SMT_E_INVALID (-1)          /* bad argument (null pointer, negative size, bad enum) */
#define SMT_E_ALIGN (-2)            /* pointer / leading dimension not 16-byte aligned */
#define SMT_E_WORKSPACE (-3)        /* workspace too small */
#define SMT_E_LAUNCH (-4)           /* hipLaunchKernel / hipGetLastError failure */

/* element dtypes */
#define SMT_DTYPE_BF16 0
#define SMT_DTYPE_FP32 1
#define SMT_DTYPE_FP16 2

/* block-score strategies, smt_helper.py:71-78 (term = what the reference's fp32 reduction adds) */
#define SMT_SCORE_MEAN_ABS 0        /* mean(dim=(1,3)).abs()  -> term g                   */
#define SMT_SCORE_ABS_MEAN 1        /* abs().mean(dim=(1,3))  -> term |g|                 */
#define SMT_SCORE_L1 2              /* abs().sum(dim=(1,3))   -> term |g|                 */
#define SMT_SCORE_L2 3              /* sqrt(sum(abs()**2))    -> term fp32(g*g)           */

/* AdamW update formulas */
#define SMT_ADAM_DEEPSPEED 0        /* DeepSpeed FusedAdam ADAM_MODE_1 (decoupled decay inside update) */
#define SMT_ADAM_TORCH 1            /* torch.optim.AdamW (decay applied to p before the update)        */

/* One 256x256 tile of a flat tile-major parameter buffer and where it lives in W. */
typedef struct smt_tile_desc {
    void* weight;                   /* W base (row-major, the AdamW step's param_dtype) or NULL: no scatter */
    int64_t ld_weight;              /* W row stride in elements                       */
    int32_t row_block;              /* index[0] of smt.py:318                         */
    int32_t col_block;              /* index[1] of smt.py:318                         */
    int64_t flat_offset;            /* element offset of the tile in the flat buffers */
} smt_tile_desc;

/* One warm-up accumulator update: dst[i] (+)= float(src[i]) for i < n. */
typedef struct smt_accum_entry {
    const void* src;                /* gradient (dtype src_dtype)                 */
    float* dst;                     /* fp32 accumulator                           */
    int64_t n;                      /* elements                                   */
    int64_t chunk_begin;            /* exclusive prefix of ceil(n / 4096) chunks  */
    int32_t src_dtype;              /* SMT_DTYPE_*                                */
    int32_t assign;                 /* 1: dst = src (first step, fine_tune.py:731-734); 0: dst += src */
} smt_accum_entry;

/* One gradient matrix [d1*256, d2*256] (fp32, row stride ld) to score per 256x256 block. */
typedef struct smt_score_entry {
    const float* src;
    int64_t ld;
    int32_t d1, d2;                 /* block grid, smt_helper.py:57-58            */
    int64_t block_begin;            /* exclusive prefix of d1*d2                  */
    double* out;                    /* d1*d2 pairs {sum of terms, sum of |terms|}, row-major (ABI v4) */
    int32_t strategy;               /* SMT_SCORE_*                                */
    int32_t pad_;
} smt_score_entry;

typedef struct smt_adamw_args {
    float lr, beta1, beta2, eps, weight_decay;
    float bias_correction1;         /* 1 - beta1^step (1.0 if bias_correction off) */
    float bias_correction2;         /* 1 - beta2^step                              */
    float max_grad_norm;            /* <= 0: no clipping                           */
    float grad_scale;               /* multiplies every gradient (1/world for DP average; with fp16
                                       loss scaling also 1/loss_scale)                       */
    int32_t mode;                   /* SMT_ADAM_*                                  */
    int32_t grad_dtype;             /* SMT_DTYPE_FP32 (any param_dtype), or SMT_DTYPE_BF16 / _FP16
                                       equal to param_dtype                                  */
    int32_t param_dtype;            /* ABI v12: SMT_DTYPE_BF16, _FP16 or _FP32, the dtype of the
                                       parameter (and W) values written -- the reference's
                                       --dtype (fine_tune.py:955-959, deepspeed_helpers.py:53-61) */
    int32_t reserved;               /* 0                                           */
} smt_adamw_args;

typedef struct smt_adamw_tensor {
    const void* grad;               /* n gradient elements (args->grad_dtype)     */
    float* master;                  /* n fp32 master values                       */
    float* exp_avg;
    float* exp_avg_sq;
    void* param;                    /* n parameter values of args->param_dtype (written) */
    int64_t n;
} smt_adamw_tensor;                 /* all five buffers 16-byte aligned          */

const char* smt_last_error(void);
/* 13: the fused LLaMA ops (smt_model_ops.h) and the flash attention (smt_attention.h) take the
 *     model's 16-bit dtype, bf16 or fp16 (the reference's --dtype fp16, fine_tune.py:955-959);
 * 12: smt_adamw_args.param_dtype; 11: smt_wgrad_module.operand_dtype. */
int smt_abi_version(void);

/* Workspace bytes smt_tile_wgrad needs for T rows and n_tiles tiles. */
size_t smt_wgrad_workspace_bytes(int64_t T, int32_t n_tiles);

/*
 * grad_tiles[i] (+)= sum_{t<T} grad_out[t, r_i*256 : r_i*256+256]^T  X_{c_i}[t, 0:256]
 * grad_out [T, ld_grad_out] bf16 row-major; X_c = x + c * x_block_stride, rows of ld_x elements:
 * x_block_stride = 256 for a row-major x [T, ld_x], or T*256 (ld_x = 256) for the block-major copy
 * smt_colblock_gather writes (each block a contiguous [T, 256]); tile_rc_dev: device int32 [n_tiles][2];
 * order_dev: optional device int32 [n_tiles] permutation giving the SCHEDULE order of the tiles
 * (tiles sharing a column / row block adjacent, for L2 reuse); NULL = index order. Results do not
 * depend on it. grad_tiles: [n_tiles*256, 256] row-major of out_dtype (bf16 or fp32). fp32 MFMA
 * accumulation over the whole T, one rounding at the end (the reference rounds each per-sample
 * partial to bf16 first). Deterministic (fixed split and summation order).
 */
int smt_tile_wgrad(const void* grad_out, int64_t ld_grad_out,
                   const void* x, int64_t ld_x, int64_t x_block_stride, int64_t T,
                   const int32_t* tile_rc_dev, const int32_t* order_dev, int32_t n_tiles,
                   void* grad_tiles, int32_t out_dtype, int32_t accumulate,
                   void* workspace, size_t workspace_bytes, hipStream_t stream);

/*
 * One module of a batched tile wgrad (smt_tile_wgrad_batch): the operands and output of one
 * smt_tile_wgrad call (same meaning as its arguments), plus the module's accumulate flag.
 */
#define SMT_WGRAD_MAX_MODULES 16
typedef struct smt_wgrad_module {
    const void* grad_out;           /* [T, ld_grad_out] of operand_dtype                            */
    const void* x;                  /* block c at x + c * x_block_stride, rows of ld_x              */
    int64_t ld_grad_out;
    int64_t ld_x;
    int64_t x_block_stride;
    void* grad_tiles;               /* this module's [n_m*256, 256] output of out_dtype            */
    int32_t accumulate;             /* add to grad_tiles instead of overwriting                     */
    int32_t operand_dtype;          /* ABI v11 (was reserved, 0): SMT_DTYPE_BF16 (0), _FP16 or _FP32,
                                       one per launch -- the reference's --dtype (fine_tune.py:955-959).
                                       out_dtype is that dtype (16-bit operands) or SMT_DTYPE_FP32    */
} smt_wgrad_module;                 /* 56 bytes                                                     */

/* Workspace bytes smt_tile_wgrad_batch needs for T rows and n_tiles tiles over all its modules. */
size_t smt_wgrad_batch_workspace_bytes(int64_t T, int32_t n_tiles);

/*
 * The tile weight gradients of up to SMT_WGRAD_MAX_MODULES SMT modules that share T (every linear of
 * a decoder sees the same B*S rows) in ONE launch: for tile i of tile_tab_dev (device int32
 * [n_tiles][4] = (module m, row_block r, col_block c, tile index k in module m's output)),
 *   modules[m].grad_tiles[k] (+)= sum_{t<T} grad_out_m[t, r*256 : r*256+256]^T  X_{m,c}[t, 0:256]
 * exactly as smt_tile_wgrad computes it per module (smt.py:382-404; same kernels, same split and
 * summation order for the same T and total tile count). `modules` is a HOST array of n_modules
 * entries, passed to the kernels by value. Batching makes one launch of the ~8 tiles a module of a
 * spread selection carries plus those of its neighbours: fewer split-K slabs per tile and one launch
 * instead of several (the engine batches consecutive backward calls).
 * Operands bf16 or fp16 (the 16-bit kernels: bf16 / f16 MFMA, fp32 accumulation) or fp32 (exact f32
 * MFMA, v_mfma_f32_32x32x2_f32), per the modules' operand_dtype (ABI v11); smt_tile_wgrad is bf16.
 */
int smt_tile_wgrad_batch(const smt_wgrad_module* modules, int32_t n_modules, int64_t T,
                         const int32_t* tile_tab_dev, const int32_t* order_dev, int32_t n_tiles,
                         int32_t out_dtype, void* workspace, size_t workspace_bytes, hipStream_t stream);

/* Workspace bytes smt_tile_wgrad_batch_seq needs (T = n_samples * seq_len rows, n_tiles tiles). */
size_t smt_wgrad_seq_workspace_bytes(int64_t T, int64_t seq_len, int32_t n_tiles);

/*
 * smt_tile_wgrad_batch with the reference's rounding (ABI v8; opt-in parity mode). The T rows are
 * T / seq_len samples of seq_len rows (linearZ's 3-D input [B, S, in] flattened, so seq_len = S), and
 * each tile's gradient is computed exactly as smt.py:397-404 rounds it: one [256, 256] product per
 * sample accumulated in fp32 and rounded to bf16 (torch.matmul of bf16), the B bf16 partials summed in
 * fp32 in sample order and rounded to bf16 (torch.sum(dim=0)), then, with accumulate, added to the
 * output (autograd's accumulation into .grad). An fp32 output holds that bf16 value exactly. fp16
 * operands round to fp16 in the same places; for fp32 operands the roundings are the identity (each
 * sample's fp32 partial, summed in sample order in fp32). T must be
 * a whole number of samples (SMT_E_INVALID otherwise). Deterministic; about n_samples / S times the
 * default mode's fp32 slab traffic.
 */
int smt_tile_wgrad_batch_seq(const smt_wgrad_module* modules, int32_t n_modules, int64_t T, int64_t seq_len,
                             const int32_t* tile_tab_dev, const int32_t* order_dev, int32_t n_tiles,
                             int32_t out_dtype, void* workspace, size_t workspace_bytes, hipStream_t stream);

/*
 * out[j, t, 0:256] = x[t, c_j*256 : c_j*256+256] for the n_cb column blocks c_j of col_blocks_dev
 * (device int32); x [T, ld_x] row-major, out [n_cb, T, 256] block-major (ABI v5; was [T, n_cb*256]),
 * 16-bit elements: each block's rows contiguous for smt_tile_wgrad (x_block_stride = T*256).
 */
int smt_colblock_gather(const void* x, int64_t ld_x, int64_t T, const int32_t* col_blocks_dev, int32_t n_cb,
                        void* out, hipStream_t stream);

/*
 * Wt[c*256 + j, r*256 + k] = tiles[flat_offset + k*256 + j] for each descriptor (weight = the bf16
 * transposed copy W^T of a W, row_block / col_block = the tile's (r, c) in W); NULL weight: skipped.
 */
int smt_tile_scatter_t(const smt_tile_desc* descs_dev, int32_t n_tiles, const void* tiles, hipStream_t stream);

/* tiles[i] = W[r_i*256:+256, c_i*256:+256]; elem_bytes 2 or 4. */
int smt_tile_gather(const void* weight, int64_t ld_weight, int32_t elem_bytes,
                    const int32_t* tile_rc_dev, int32_t n_tiles,
                    void* tiles, hipStream_t stream);

/* W[r_i*256:+256, c_i*256:+256] = tiles[i]; elem_bytes 2 or 4. */
int smt_tile_scatter(void* weight, int64_t ld_weight, int32_t elem_bytes,
                     const int32_t* tile_rc_dev, int32_t n_tiles,
                     const void* tiles, hipStream_t stream);

/* Multi-tensor warm-up accumulation; entries_dev is a device array of n_entries. */
int smt_grad_accumulate(const smt_accum_entry* entries_dev, int32_t n_entries,
                        int64_t total_chunks, hipStream_t stream);

/*
 * Multi-tensor block scoring. Per 256x256 block, out[2k] = fp64 sum of the strategy's terms and
 * out[2k+1] = fp64 sum of their magnitudes (equal unless MEAN_ABS). Deterministic order.
 */
int smt_block_score(const smt_score_entry* entries_dev, int32_t n_entries,
                    int64_t total_blocks, hipStream_t stream);

/* out_dev[0] = sum x[i]^2 in fp64 (deterministic two-pass); partials_dev holds n_partials doubles. */
int smt_sq_norm(const float* x, int64_t n, double* partials_dev, int32_t n_partials,
                double* out_dev, hipStream_t stream);

/*
 * Fused clip + AdamW + cast to args->param_dtype (+ scatter into W) over flat tile-major buffers of
 * n_tiles*65536 elements (tiles_dev != NULL) or n_elems plain elements (tiles_dev == NULL).
 * grad_sq_norm_dev: device fp64 squared global norm of the effective gradient (grad * grad_scale,
 * over every parameter the clip covers), or NULL for no clipping.
 */
int smt_adamw_step(const void* grad, float* master, float* exp_avg, float* exp_avg_sq,
                   void* param, const smt_tile_desc* tiles_dev, int32_t n_tiles,
                   int64_t n_elems, const double* grad_sq_norm_dev,
                   const smt_adamw_args* args, hipStream_t stream);

/*
 * Multi-tensor form of the flat step (ABI v5): one launch over n_tensors independent parameters
 * sharing the same args (DeepSpeed FusedAdam's multi_tensor_apply over a param group,
 * fine_tune.py:352-363). tensors_dev: device table; block_start_dev: device int64[n_tensors + 1],
 * block_start[t] = sum over u < t of ceil(n_u / 2048), n_blocks = block_start[n_tensors].
 */
int smt_adamw_multi(const smt_adamw_tensor* tensors_dev, const int64_t* block_start_dev, int32_t n_tensors,
                    int64_t n_blocks, const double* grad_sq_norm_dev, const smt_adamw_args* args,
                    hipStream_t stream);

/* ---- MX-fp8 tile weight gradient (ABI v5; BASELINE config 5) -------------
 * No reference counterpart (the reference has no fp8, deepspeed/fine_tune.py:955-959): the bf16
 * smt_tile_wgrad (smt.py:397-404) is the bar. "MX column blocks" of a bf16 [T, C] matrix, for a list
 * of n_blocks 256-column blocks, with ldq = T rounded up to a multiple of 64:
 *   q       e4m3 (OCP) [n_blocks][ldq/64][256][64]   K-major in 64-token panels: q[b][t/64][f][t%64]
 *           is column f of block b at row t (zero past T); one panel (16 KiB) is one wgrad stage
 *   scales  e8m0 [n_blocks][ldq/32][256]      exponent e + 127 of each 32-row group of each column
 * with e the smallest integer such that the group's max |x| <= 448 * 2^e (-127 for an all-zero
 * group) and q = e4m3_rne(x * 2^-e), so value = e4m3(q) * 2^e exactly reproduces the quantised x.
 */
int smt_mx_quant_cols(const void* x, int64_t ld_x, int64_t T, const int32_t* blocks_dev, int32_t n_blocks,
                      int64_t ldq, void* q, void* scales, hipStream_t stream);

/* fp32 split-K workspace bytes smt_tile_wgrad_mx needs (0 when the tiles are written directly). */
size_t smt_wgrad_mx_workspace_bytes(int64_t ldq, int32_t n_tiles);

/*
 * grad_tiles[i] (+)= A_i^T B_i for tile i, where A_i / B_i are the MX column blocks
 * tile_rc_dev[i] = (index into qg/sg, index into qx/sx) of the output gradient g and the input x
 * (v_mfma_scale_f32_32x32x64_f8f6f4, fp32 accumulation, one rounding to out_dtype). order_dev: the
 * schedule as for smt_tile_wgrad, or NULL.
 */
int smt_tile_wgrad_mx(const void* qg, const void* sg, const void* qx, const void* sx, int64_t ldq,
                      const int32_t* tile_rc_dev, const int32_t* order_dev, int32_t n_tiles, void* grad_tiles,
                      int32_t out_dtype, int32_t accumulate, void* workspace, size_t workspace_bytes,
                      hipStream_t stream);

/* One module of a batched MX tile wgrad: its MX blocks of g and x and its output. */
typedef struct smt_wgrad_mx_module {
    const void* qg;                 /* MX row blocks of the output gradient (e4m3 panels)          */
    const void* sg;                 /* their e8m0 exponents                                         */
    const void* qx;                 /* MX column blocks of the input                                */
    const void* sx;
    void* grad_tiles;               /* this module's [n_m*256, 256] output of out_dtype            */
    int32_t accumulate;
    int32_t reserved;
} smt_wgrad_mx_module;              /* 48 bytes                                                     */

/*
 * smt_tile_wgrad_mx over up to SMT_WGRAD_MAX_MODULES modules sharing ldq in one launch (as
 * smt_tile_wgrad_batch: HOST module array, device int32 [n_tiles][4] table of (module, index into
 * the module's g blocks, index into its x blocks, tile index in its output)). Workspace:
 * smt_wgrad_mx_workspace_bytes(ldq, n_tiles) over all tiles.
 */
int smt_tile_wgrad_mx_batch(const smt_wgrad_mx_module* modules, int32_t n_modules, int64_t ldq,
                            const int32_t* tile_tab_dev, const int32_t* order_dev, int32_t n_tiles,
                            int32_t out_dtype, void* workspace, size_t workspace_bytes, hipStream_t stream);

/* ---- channel path (ABI v3) ------------------------------------------------------------------- */

/* rows[i, 0:n_cols] = W[rows_dev[i], 0:n_cols]; elem_bytes 2 or 4; rows 16-byte aligned. */
int smt_row_gather(const void* weight, int64_t ld_weight, int32_t elem_bytes, int64_t n_cols,
                   const int32_t* rows_dev, int32_t n_rows, void* rows, int64_t ld_rows, hipStream_t stream);

/* W[rows_dev[i], 0:n_cols] = rows[i, 0:n_cols]; rows_dev must not repeat an index. */
int smt_row_scatter(void* weight, int64_t ld_weight, int32_t elem_bytes, int64_t n_cols,
                    const int32_t* rows_dev, int32_t n_rows, const void* rows, int64_t ld_rows, hipStream_t stream);

/*
 * out[t, j] = x[t, cols_dev[j]] for j < n_cols and 0 for n_cols <= j < ld_out (bf16/fp16 bits,
 * 2-byte elements); x [T, ld_x] with every cols_dev[j] < n_in <= ld_x (n_in <= 32768: rows are
 * staged in LDS), out [T, ld_out] row-major; ld_x, ld_out % 8 == 0; cols_dev 16-byte aligned.
 * (ABI v5: n_in added.)
 */
int smt_column_gather(const void* x, int64_t ld_x, int64_t n_in, int64_t T, const int32_t* cols_dev, int32_t n_cols,
                      void* out, int64_t ld_out, hipStream_t stream);

/*
 * acc[b, s, c] = (assign ? 0 : acc[b, s, c]) + float(|x[b, s, c]|), one fp32 add per element (the
 * reference's CPU `+=`, bit for bit). x: element (b, s, c) at x + b*batch_stride + s*ld_x + c (dtype
 * x_dtype); acc: contiguous fp32 [B, S, n_cols]; n_cols % 8 == 0. (ABI v4: was an fp64 [S, n_cols]
 * batch sum.)
 */
int smt_act_accumulate(const void* x, int32_t x_dtype, int64_t ld_x, int64_t batch_stride, int32_t B, int32_t S,
                       int32_t n_cols, float* acc, int32_t assign, hipStream_t stream);

/*
 * out[c] = sum_{s<S} A_s (strategy MEAN_ABS, ABS_MEAN, L1) or sum_{s<S} A_s^2 (L2) in fp64, with
 * A_s = sum_{b<B} |acc[b, s, c]| and acc a contiguous fp32 [B, S, n_cols] accumulator; summed as
 * 32-row partials (s ascending inside each) added in ascending order. partials: caller workspace of
 * smt_channel_score_workspace_bytes(S, n_cols) bytes (ABI v5). The caller divides by S (means) or
 * takes the square root (L2) and rounds to fp32 once.
 */
size_t smt_channel_score_workspace_bytes(int32_t S, int32_t n_cols);
int smt_channel_score(const float* acc, int32_t B, int32_t S, int32_t n_cols, int32_t strategy, double* partials,
                      size_t partial_bytes, double* out, hipStream_t stream);

/*
 * The mean_abs / abs_mean channel statistic of smt_helper.py:167-176 with the reference's own fp32
 * rounding: out[c] = torch.mean(torch.sum(act.abs(), dim=0).abs(), dim=0)[c] as ATen's CPU kernels
 * compute it (cascade_sum: 4 accumulator levels of 2^p rows, p = max(4, ceil_log2(n)/4), per output
 * column; then div_ by S), for a contiguous fp32 [B, S, n_cols] accumulator (ABI v6). The caller
 * confirms it against the reference expression on the host once per shape. Workspace:
 * smt_channel_mean_aten_workspace_bytes(S, n_cols) bytes of fp32 chunk sums.
 */
size_t smt_channel_mean_aten_workspace_bytes(int32_t S, int32_t n_cols);
int smt_channel_mean_aten(const float* acc, int32_t B, int32_t S, int32_t n_cols, float* workspace,
                          size_t workspace_bytes, float* out, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SMT_HIP_H */
