// Causal grouped-query flash attention for gfx950 (CDNA4), head_dim 128, bf16 or fp16 I/O (the model's
// dtype, smt_attn_shape.dtype; ABI v13), fp32 softmax.
// C ABI: include/smt_attention.h. Replaces transformers' sdpa attention (aotriton on this torch
// build) in the LLaMA decoder that carries the SMT modules.
//
// MFMA v_mfma_f32_32x32x16_bf16 lane maps (verified on gfx950):
//   A[m][k]: lane l holds m = l&31, k = 8*(l>>5) + j (j = 0..7)     B[k][n]: n = l&31, same k
//   C[m][n]: lane l holds n = l&31, m = (i&3) + 8*(i>>2) + 4*(l>>5) (i = 0..15)
// All products are arranged so that a softmax row lives on ONE lane pair (l, l^32):
//   forward   S^T[key][q] = K Q^T,  O^T[d][q] += V^T P^T          (q on the lane)
//   dQ        S^T, dP^T = V dO^T,   dQ^T[d][q] += K^T dS^T          (q on the lane)
//   dK, dV    S[q][key] = Q K^T, dP = dO V^T, dV^T += dO^T P, dK^T += Q^T dS   (key on the lane)
// so row statistics are per-lane scalars and the probability tile, packed to bf16 and exchanged
// once between the two wave halves (v_permlane32_swap), IS the next product's B operand.
// LDS images are [row][128 d] bf16 rows of 256 B, swizzled by 16-B chunk:
//   chunk' = chunk ^ (((row & 3) << 2) | ((row >> 2) & 3))
// which is conflict-free both for ds_read_b128 row reads (16 consecutive rows, same chunk) and for
// ds_read_b64_tr_b16 transposed reads (4 consecutive rows land in 4 different 64-B quarters).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <utility>

#include "smt_attention.h"
#include "smt_hip.h"

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

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

constexpr int kD = 128;
constexpr int kRowB = 256;                 // one [d] row in LDS
constexpr float kNegInf = -__builtin_huge_valf();

struct Tns {
    const uint16_t* p;
    int64_t sb, sh, ss;
};

__device__ __forceinline__ uint32_t swz(uint32_t row) { return ((row & 3u) << 2) | ((row >> 2) & 3u); }
__device__ __forceinline__ uint32_t lds_off(uint32_t row, uint32_t byte) { return row * kRowB + (byte ^ (swz(row) << 4)); }

// 8 consecutive d of one row (ds_read_b128): A[m=row][k] or B[k][n=row] fragments of row-major data.
__device__ __forceinline__ bf16x8_t row_frag(const uint8_t* img, uint32_t row, uint32_t byte) {
    return *reinterpret_cast<const bf16x8_t*>(img + lds_off(row, byte));
}

// Transposed fragment (two ds_read_b64_tr_b16): lane l gets column (col0 + l&31) at rows
// row0 + 8*(l>>5) + 0..7, i.e. the A[m=col][k=row] operand of row-major data.
struct TrLane {
    uint32_t krow, feat_byte;
};
__device__ __forceinline__ TrLane tr_lane(int lane) {
    const int gi = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    return TrLane{8u * (gi >> 1) + q, 2u * (16u * (gi & 1) + 4u * p)};
}
__device__ __forceinline__ bf16x8_t tr_frag(const uint8_t* img, TrLane tl, uint32_t row0, uint32_t col0) {
    const uint32_t r = row0 + tl.krow, byte = 2u * col0 + tl.feat_byte;
    s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(img + lds_off(r, byte)));
    s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(img + lds_off(r + 4, byte)));
    const s16x8_t both = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8_t, both);
}

// Fragments travel as bf16x8_t bit containers whatever the format; F = SMT_DTYPE_BF16 (0) or
// SMT_DTYPE_FP16 (2) picks the MFMA (v_mfma_f32_32x32x16_bf16 / _f16, the same lane maps) and the
// roundings of P, dS and the outputs.
template <int F>
__device__ __forceinline__ f32x16_t mfma(bf16x8_t a, bf16x8_t b, f32x16_t c) {
    if constexpr (F == SMT_DTYPE_FP16)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c,
                                                      0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Two-lane fp32 arithmetic of the softmax. PK: packed (v_pk_fma_f32 / v_pk_add_f32 / v_pk_mul_f32,
// one issue per pair); otherwise two scalar VALU ops per pair (the packed forms cost more than two
// scalar ones when issued beside MFMAs, MI355X_MICROARCH issue-cost table). Results are bit-identical
// either way (the same IEEE operations). The forward measured faster scalar, dQ and dK/dV packed
// (profiles/r04_e_attn_pk_ab.jsonl).
constexpr bool kPkFwd = false, kPkDq = true, kPkDkv = true;
template <bool PK>
__device__ __forceinline__ f32x2_t fma2(f32x2_t a, f32x2_t b, f32x2_t c) {
    if (PK) return __builtin_elementwise_fma(a, b, c);
    return f32x2_t{__builtin_fmaf(a.x, b.x, c.x), __builtin_fmaf(a.y, b.y, c.y)};
}
template <bool PK>
__device__ __forceinline__ f32x2_t submul2(f32x2_t a, f32x2_t d, f32x2_t p) {     // (a - d) * p
    if (PK) return (a - d) * p;
    return f32x2_t{(a.x - d.x) * p.x, (a.y - d.y) * p.y};
}
template <bool PK>
__device__ __forceinline__ f32x2_t add2(f32x2_t a, f32x2_t b) {
    if (PK) return a + b;
    return f32x2_t{a.x + b.x, a.y + b.y};
}

template <int F>
__device__ __forceinline__ uint32_t pk16(float a, float b) {        // two fp32 -> two 16-bit values (RNE)
    f32x2_t v = {a, b};
    if constexpr (F == SMT_DTYPE_FP16) return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2_t));
    else return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}
template <int F>
__device__ __forceinline__ float lo16(uint32_t w) {                  // the low / high 16-bit value of a word
    if constexpr (F == SMT_DTYPE_FP16) return (float)__builtin_bit_cast(_Float16, (uint16_t)(w & 0xffffu));
    else return __uint_as_float(w << 16);
}
template <int F>
__device__ __forceinline__ float hi16(uint32_t w) {
    if constexpr (F == SMT_DTYPE_FP16) return (float)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16));
    else return __uint_as_float(w & 0xffff0000u);
}

__device__ __forceinline__ float other_half_max(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float halves_sum(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// C-layout probabilities of one 32-column tile (16 fp32 per lane: column = lane's n, rows
// (i&3)+8(i>>2)+4hi) -> two B fragments for k-steps of 16 rows, rows 8hi..8hi+7 per lane.
template <int F>
__device__ __forceinline__ void pack_b_frags(const float (&p)[16], bf16x8_t& f0, bf16x8_t& f1) {
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = pk16<F>(p[2 * i], p[2 * i + 1]);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        auto a = __builtin_amdgcn_permlane32_swap(w[4 * h + 0], w[4 * h + 2], false, false);
        auto b = __builtin_amdgcn_permlane32_swap(w[4 * h + 1], w[4 * h + 3], false, false);
        u32x4_t v = {a[0], b[0], a[1], b[1]};
        if (h == 0) f0 = __builtin_bit_cast(bf16x8_t, v);
        else f1 = __builtin_bit_cast(bf16x8_t, v);
    }
}

// XCD-aware bijective remap (workgroups are dealt round-robin over the 8 XCDs): consecutive logical
// ids run on one XCD, so workgroups that share K/V (or Q/dO) share that XCD's L2.
__device__ __forceinline__ int xcd_logical(int bid, int total) {
    const int q8 = total >> 3, r8 = total & 7, xcd = bid & 7;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
}

// Explicit LDS addressing for compile-time image offsets. A swizzled row read (lds_off) of row r,
// 16-B chunk (ks, hi) is (r*256 + (16hi ^ swz(r)<<4)) ^ (ks<<5), and a transposed read at rows
// 16kq + krow (+4) and column block dt is 4096kq + ((r*256 + (feat_byte ^ swz<<4)) ^ (dt<<6)): one
// lane constant per read family, one v_xor per read, the image base in the instruction's offset.
// The lane constants are re-materialised per slice (an opaque copy), so hipcc cannot hoist the 8-16
// derived addresses out of the loop and spill them.
__device__ __forceinline__ uint32_t opaque(uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
}
template <int IMG>
__device__ __forceinline__ bf16x8_t rowx(const uint8_t* lds, uint32_t lo, int ks) {
    return *reinterpret_cast<const bf16x8_t*>(lds + IMG + (lo ^ (uint32_t)(ks << 5)));
}
template <int IMG>
__device__ __forceinline__ bf16x8_t trx(const uint8_t* lds, uint32_t t0, uint32_t t4, int kq, int dt) {
    const uint32_t x = (uint32_t)(dt << 6);
    s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(lds + IMG + 4096 * kq + (t0 ^ x)));
    s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(lds + IMG + 4096 * kq + (t4 ^ x)));
    const s16x8_t both = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8_t, both);
}

// LDS-DMA: lane l's 16 B from rsrc + voff land at LDS byte lds_base + 16*l (buffer_load ... lds).
// Inline asm so that hipcc does not treat it as an LDS write aliasing every ds_read (it then drains
// vmcnt before each read); completion is waited for explicitly (s_waitcnt vmcnt(0) + barrier).
// M0 is saved / restored inside the statement. Out-of-range offsets read as zeros.
typedef __attribute__((address_space(3))) uint8_t lds_u8_t;
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, uint32_t lds_base, int voff) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(lds_base) : "memory");
}
__device__ __forceinline__ uint32_t lds_addr(const uint8_t* p) { return (uint32_t)(uintptr_t)(const lds_u8_t*)p; }
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base, int64_t bytes) {
    const uint64_t a = (uint64_t)(uintptr_t)base;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const int n = __builtin_amdgcn_readfirstlane((int)bytes);
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}
__device__ __forceinline__ void vm_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// The same wait as a builtin the compiler's waitcnt pass understands: after it, the pass knows that
// the register loads issued before the loop (Q / dO / K fragments) have landed. Without it the pass
// still counts them as pending at the loop header and puts a vmcnt(0) in front of their first use
// INSIDE the loop, which also waits for the next tile's LDS-DMA issued just before it (the prefetch
// then never overlaps compute). gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15.
__device__ __forceinline__ void vm_wait_all_known() { __builtin_amdgcn_s_waitcnt(0x0F70); }
// Wait until at most n (wave-uniform) of this wave's vector-memory operations are outstanding,
// rounded down to an encodable immediate (waiting for more than needed is always safe).
__device__ __forceinline__ void vm_wait_upto(int n) {
    if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n >= 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// One wave copies `pieces` x 4 rows [row0, row0 + 4*pieces) of a [rows][128] bf16 operand (row stride
// ss elements, rows counted from the rsrc base) into a swizzled LDS image at img (image row = row - img_row0).
__device__ __forceinline__ void dma_rows(__amdgpu_buffer_rsrc_t rsrc, int64_t ss, uint32_t img, int img_row0,
                                         int row0, int pieces, int lane) {
#pragma unroll 4
    for (int i = 0; i < pieces; ++i) {
        const int r = row0 + 4 * i + (lane >> 4);             // source row of this lane
        const uint32_t ir = (uint32_t)(r - img_row0);          // image row
        const uint32_t ch = (uint32_t)(lane & 15) ^ swz(ir);   // logical chunk stored at this lane's slot
        const uint32_t base = __builtin_amdgcn_readfirstlane(img + (uint32_t)(r - (lane >> 4) - img_row0) * kRowB);
        dma16(rsrc, base, (int)((int64_t)r * ss * 2 + ch * 16));
    }
}

// ------------------------------------------------------------------------------------------------
// Forward: a workgroup = 4 waves x 32 query rows of one (b, q head); K/V tiles of 64 keys staged
// through registers into a double-buffered LDS ring (issue-early / write-late), one barrier per tile.
// ------------------------------------------------------------------------------------------------
// Waves (x 32 query rows) per workgroup of the forward / dQ kernels: 4, two workgroups per CU. Every
// workgroup stages its own K/V tiles, so 8 waves (256 query rows, one workgroup per CU) would halve
// the LDS-fill bytes per MFMA; measured at B16 Hq32 Hkv8 S2048 (profiles/r02_attn_waves.jsonl) the
// 8-wave forward ran 7 % slower (0.89 vs 0.83 ms) and the 8-wave dQ the same: these loops are not
// bound by the K/V fill. The forward reads its K / V fragments two MFMAs ahead (FwdLean::compute:
// 0.80 -> 0.76 ms at the bench shape, profiles/r04_f_attn_pref_ab.jsonl); the same read-ahead in dQ
// measured no faster and is not used.
constexpr int kFwdQW = 32, kFwdWaves = 4, kFwdQB = kFwdQW * kFwdWaves, kKV = 64;
constexpr int kDqWaves = 4, kDqQB = kFwdQW * kDqWaves;
constexpr int kTileB = kKV * kRowB;        // 16 KiB per operand tile

// Key mask (optional, smt_attn_*_kmask): bit (j & 63) of kmask[b * kmask_ld + (j >> 6)] set = key j
// of batch b takes part (transformers' 2-D attention_mask of a padded batch, e.g. the reference's
// collator mask input_ids != pad, deepspeed/helpers/helper.py:194-204). A query row whose every
// visible key is masked gets a zero output, lse = +inf and zero gradients (torch's safe softmax).
__device__ __forceinline__ bool key_bit(uint64_t w, int key) { return (w >> (key & 63)) & 1ull; }

struct FwdArgs {
    Tns q, k, v;
    uint16_t* o;
    int64_t o_sb, o_sh, o_ss;
    float* lse;
    const uint64_t* kmask;
    int64_t kmask_ld;
    int B, Hq, Hkv, S;
    float sl2;                             // scale * log2(e)
};

// Causal balance: a workgroup takes the query blocks qb and nqb-1-qb (equal total work per workgroup).
struct PairTask {
    int b, hk, hh, blk[2], n;
};
__device__ __forceinline__ PairTask pair_task(int L, int nblk, int G, int Hkv) {
    const int npair = (nblk + 1) / 2;
    const int per_group = G * npair;
    const int grp = L / per_group;
    const int rem = L - grp * per_group;
    const int p = rem / G;
    PairTask t;
    t.b = grp / Hkv;
    t.hk = grp % Hkv;
    t.hh = rem % G;
    t.blk[0] = nblk - 1 - p;
    t.blk[1] = p;
    t.n = (t.blk[1] == t.blk[0]) ? 1 : 2;
    return t;
}

constexpr float kFwdThr = 8.f;


// v_max3_f32 as one instruction: fmaxf on MFMA results makes hipcc canonicalise both inputs first
// (an extra v_max per operand; cdna_hip_programming Appendix B, attention pitfalls)
__device__ __forceinline__ float max3f(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// ------------------------------------------------------------------------------------------------
// Forward (FwdLean): two workgroups per CU, i.e. two waves per SIMD whose MFMA and VALU phases
// overlap each other; Q in registers; a 2-slot K/V ring, one barrier per 64-key tile; the per-tile
// VALU cut to what the softmax needs: tiles in pairs so the LDS slot is a compile-time offset (no
// per-read address adds), the scores' first MFMA on a zero accumulator (no per-tile zeroing), the row
// max by v_max3 without canonicalisation, row max / sum as trees, a deferred running max (a row's max
// moves only when a tile's max exceeds it by more than kFwdThr, log2 units, so P <= 2^kFwdThr and the
// O rescale is rare; cdna_hip_programming T13) and the causal mask only on the wave's diagonal tile.
// Measured and removed (git history): a software-pipelined one-workgroup-per-CU forward,
// one wave per SIMD over 64 rows (two builds), all slower.
// ------------------------------------------------------------------------------------------------

template <bool KMASK, int F>
struct FwdLean {
    const FwdArgs& a;
    uint8_t* lds;
    __amdgpu_buffer_rsrc_t rk, rv;
    uint32_t lds0;
    const uint64_t* km;
    bf16x8_t qf[8];
    f32x16_t o[4];
    float m_run, l_run;
    int qw, qrow, hi, l32, wave, lane, nt, last;
    TrLane tl;

    __device__ __forceinline__ FwdLean(const FwdArgs& a_, uint8_t* lds_) : a(a_), lds(lds_) {}

    __device__ __forceinline__ void issue(int t) {            // K(t), V(t) into slot t & 1
        const uint32_t slot = lds0 + (uint32_t)((t & 1) * 2 * kTileB);
        dma_rows(rk, a.k.ss, slot, t * kKV, t * kKV + 16 * wave, 4, lane);
        dma_rows(rv, a.v.ss, slot + kTileB, t * kKV, t * kKV + 16 * wave, 4, lane);
    }

    template <int SLOT, bool DIAG_>
    __device__ __forceinline__ void compute(int t, bool DIAG) {
        const uint8_t* K = lds + SLOT * 2 * kTileB;
        const uint8_t* V = K + kTileB;
        const int k0 = t * kKV;
        f32x16_t sc[2];
        // K fragments read two k-steps ahead of their MFMAs (a 3-deep register ring, fenced so hipcc
        // keeps the order): without it each MFMA waited lgkmcnt(0) on a read issued one MFMA earlier
        bf16x8_t kf[3][2];
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int j = 0; j < 2; ++j) kf[p][j] = row_frag(K, 32 * j + l32, 32 * p + 16 * hi);
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            if (ks + 2 < 8) {
#pragma unroll
                for (int j = 0; j < 2; ++j) kf[(ks + 2) % 3][j] = row_frag(K, 32 * j + l32, 32 * (ks + 2) + 16 * hi);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = 0; j < 2; ++j) sc[j] = mfma<F>(kf[ks % 3][j], qf[ks], ks ? sc[j] : f32x16_t{});
            __builtin_amdgcn_sched_barrier(0);
        }
        // the first two V fragments of the PV product, in flight during the softmax
        bf16x8_t vf[3];
        vf[0] = tr_frag(V, tl, 0, 0);
        vf[1] = tr_frag(V, tl, 16, 0);
        float x[32];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) x[16 * j + i] = sc[j][i];
        if (DIAG) {
#pragma unroll
            for (int i = 0; i < 32; ++i) {
                const int key = k0 + 32 * (i >> 4) + (i & 3) + 8 * ((i & 15) >> 2) + 4 * hi;
                if (key > qrow) x[i] = kNegInf;
            }
        }
        if (KMASK) {
            const uint64_t w = km[k0 >> 6];                    // workgroup-uniform
            if (~w != 0ull) {
#pragma unroll
                for (int i = 0; i < 32; ++i) {
                    const int key = k0 + 32 * (i >> 4) + (i & 3) + 8 * ((i & 15) >> 2) + 4 * hi;
                    if (!key_bit(w, key)) x[i] = kNegInf;
                }
            }
        }
        float mx[11];
#pragma unroll
        for (int i = 0; i < 10; ++i) mx[i] = max3f(x[3 * i], x[3 * i + 1], x[3 * i + 2]);
        mx[10] = max3f(x[30], x[31], mx[0]);
        mx[0] = max3f(mx[0], mx[1], mx[2]);
        mx[3] = max3f(mx[3], mx[4], mx[5]);
        mx[6] = max3f(mx[6], mx[7], mx[8]);
        mx[9] = max3f(mx[9], mx[10], mx[0]);
        const float m_tile = other_half_max(max3f(mx[3], mx[6], mx[9])) * a.sl2;
        const bool move = m_tile > m_run + kFwdThr;
        const float m_new = move ? m_tile : m_run;
        const float alpha = move ? __builtin_amdgcn_exp2f(m_run - m_new) : 1.f;
        const float m_use = (KMASK && m_new == kNegInf) ? 0.f : m_new;
        // packed fp32 (v_pk_fma_f32 / v_pk_add_f32: two lanes' worth per VALU issue)
        const f32x2_t sl2v = {a.sl2, a.sl2}, mv = {-m_use, -m_use};
        f32x2_t sm[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const f32x2_t e = fma2<kPkFwd>(f32x2_t{x[2 * i], x[2 * i + 1]}, sl2v, mv);
            x[2 * i] = __builtin_amdgcn_exp2f(e.x);
            x[2 * i + 1] = __builtin_amdgcn_exp2f(e.y);
            sm[i] = f32x2_t{x[2 * i], x[2 * i + 1]};
        }
#pragma unroll
        for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
            for (int i = 0; i < w; ++i) sm[i] = add2<kPkFwd>(sm[i], sm[i + w]);
        l_run = l_run * alpha + (sm[0].x + sm[0].y);
        m_run = m_new;
        if (__builtin_amdgcn_ballot_w64(move) != 0) {          // rare (deferred max)
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
        }
        bf16x8_t pf[4];
        pack_b_frags<F>(*reinterpret_cast<const float(*)[16]>(&x[0]), pf[0], pf[1]);
        pack_b_frags<F>(*reinterpret_cast<const float(*)[16]>(&x[16]), pf[2], pf[3]);
        // V^T fragments two MFMAs ahead (n = 4 dt + kst)
#pragma unroll
        for (int n = 0; n < 16; ++n) {
            if (n + 2 < 16) vf[(n + 2) % 3] = tr_frag(V, tl, 16 * ((n + 2) & 3), 32 * ((n + 2) >> 2));
            __builtin_amdgcn_sched_barrier(0);
            o[n >> 2] = mfma<F>(vf[n % 3], pf[n & 3], o[n >> 2]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }

    // tile t (t & 1 == SLOT): fetch tile t+1 into the other slot, compute, wait, barrier
    template <int SLOT>
    __device__ __forceinline__ void tile(int t) {
        if (t + 1 < nt) issue(t + 1);
        if (t <= last) compute<SLOT, true>(t, t == last);
        vm_wait_all();
        __syncthreads();
    }

    __device__ __forceinline__ void run(int b, int h, int hk, int qb) {
        const int tid = threadIdx.x;
        lane = tid & 63;
        wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        hi = lane >> 5;
        l32 = lane & 31;
        const int q0 = qb * kFwdQB;
        qw = q0 + wave * kFwdQW;
        qrow = qw + l32;
        const uint16_t* qp = a.q.p + b * a.q.sb + h * a.q.sh;
        const uint16_t* kp = a.k.p + b * a.k.sb + hk * a.k.sh;
        const uint16_t* vp = a.v.p + b * a.v.sb + hk * a.v.sh;
        km = KMASK ? a.kmask + (int64_t)b * a.kmask_ld : nullptr;
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            if (qrow < a.S) qf[ks] = *reinterpret_cast<const bf16x8_t*>(qp + qrow * a.q.ss + 16 * ks + 8 * hi);
            else qf[ks] = __builtin_bit_cast(bf16x8_t, u32x4_t{0u, 0u, 0u, 0u});
        }
        const int kv_end = min(a.S, q0 + kFwdQB);
        nt = (kv_end + kKV - 1) / kKV;
        last = min(nt - 1, qw / kKV);
        rk = uniform_rsrc(kp, (int64_t)a.S * a.k.ss * 2);
        rv = uniform_rsrc(vp, (int64_t)a.S * a.v.ss * 2);
        lds0 = lds_addr(lds);
        tl = tr_lane(lane);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int i = 0; i < 16; ++i) o[dt][i] = 0.f;
        m_run = kNegInf;
        l_run = 0.f;
        issue(0);
        vm_wait_all();
        vm_wait_all_known();                                   // the Q fragments too (compiler-visible)
        __syncthreads();
        for (int t = 0; t < nt; t += 2) {
            tile<0>(t);
            if (t + 1 < nt) tile<1>(t + 1);
        }
        const float l_tot = halves_sum(l_run);
        if (qrow < a.S) {
            const float inv = (KMASK && !(l_tot > 0.f)) ? 0.f : 1.f / l_tot;
            uint16_t* op = a.o + b * a.o_sb + h * a.o_sh + (int64_t)qrow * a.o_ss;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int d = 32 * dt + 8 * g + 4 * hi;
                    uint2 w;
                    w.x = pk16<F>(o[dt][4 * g] * inv, o[dt][4 * g + 1] * inv);
                    w.y = pk16<F>(o[dt][4 * g + 2] * inv, o[dt][4 * g + 3] * inv);
                    *reinterpret_cast<uint2*>(op + d) = w;
                }
            if (hi == 0)
                a.lse[((int64_t)b * a.Hq + h) * a.S + qrow] =
                    (KMASK && !(l_tot > 0.f)) ? __builtin_huge_valf() : m_run + __log2f(l_tot);
        }
    }
};

template <bool KMASK, int F>
__global__ __launch_bounds__(64 * kFwdWaves, 2)
void attn_fwd_kernel(FwdArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * 2 * kTileB];      // K/V ring: 2 x 32 KiB
    const int nqb = (a.S + kFwdQB - 1) / kFwdQB;
    const int G = a.Hq / a.Hkv;
    const int total = nqb * a.Hq * a.B;
    // consecutive ids: the G heads of one (b, kv head) at one q block, heaviest (longest causal row)
    // q blocks first (pairing q blocks measured 1-2 % slower here than this order)
    const int L = xcd_logical(blockIdx.x, total);
    const int per_group = G * nqb;
    const int grp = L / per_group;
    const int rem = L - grp * per_group;
    const int hk = grp % a.Hkv;
    FwdLean<KMASK, F> fl(a, lds);
    fl.run(grp / a.Hkv, hk * G + rem % G, hk, nqb - 1 - rem / G);
}

// ------------------------------------------------------------------------------------------------
// dQ: a workgroup = 4 waves x 32 query rows of one (b, q head), sweeping the K/V tiles up to the
// diagonal (staged as in the forward). Per tile: S^T = K Q^T, dP^T = V dO^T, P = exp2(S*c - lse),
// dS = P (dP - delta), dQ^T += K^T dS^T.
// ------------------------------------------------------------------------------------------------
// The dQ kernel also computes delta = rowsum(dO * O) of its own rows from the dO fragments it holds
// anyway (one O read) and writes it for the dK/dV kernel (no separate pass).

struct DqArgs {
    Tns q, k, v, dout, o;
    uint16_t* dq;
    int64_t dq_sb, dq_sh, dq_ss;
    const float* lse;
    float* delta;
    const uint64_t* kmask;
    int64_t kmask_ld;
    int B, Hq, Hkv, S;
    float sl2, scale;
};

// dQ (DqLean): a workgroup = 4 waves x 32 query rows of one (b, q head) sweeping the K/V tiles up to
// the diagonal; tiles in pairs (compile-time ring slot), explicit LDS addresses from two lane
// constants, S and dP from zero accumulators, p = exp2(c s - lse) and ds = p (dp - delta) in packed
// fp32, the causal test only on the wave's diagonal tile, scheduling fences that bound the fragment
// reads hoisted ahead. Measured and removed (git history): one wave per SIMD with AGPR
// accumulators, and dQ as a GEMM over a materialised dS, both slower.
template <bool KMASK, int F>
struct DqLean {
    const DqArgs& a;
    uint8_t* lds;
    bf16x8_t qf[8], df[8];
    f32x16_t dq[4];
    float lse, dlt;
    const uint64_t* km;
    __amdgpu_buffer_rsrc_t rk, rv;
    uint32_t lds0, lo_row, lo_t0, lo_t4;
    int lane, wave, hi, l32, qw, qrow, nt, last;

    __device__ __forceinline__ DqLean(const DqArgs& a_, uint8_t* lds_) : a(a_), lds(lds_) {}

    __device__ __forceinline__ void issue(int t) {            // K(t), V(t) into slot t & 1
        const uint32_t slot = lds0 + (uint32_t)((t & 1) * 2 * kTileB);
        constexpr int rows_w = kKV / kDqWaves;
        dma_rows(rk, a.k.ss, slot, t * kKV, t * kKV + rows_w * wave, rows_w / 4, lane);
        dma_rows(rv, a.v.ss, slot + kTileB, t * kKV, t * kKV + rows_w * wave, rows_w / 4, lane);
    }

    template <int SLOT>
    __device__ __forceinline__ void compute(int t, bool diag) {
        constexpr int KI = SLOT * 2 * kTileB, VI = KI + kTileB;
        const int k0 = t * kKV;
        const uint32_t lr = opaque(lo_row);
        constexpr int KH = KI + 32 * kRowB, VH = VI + 32 * kRowB;     // keys 32..63 of the tile
        f32x16_t s[2], dp[2];
        s[0] = mfma<F>(rowx<KI>(lds, lr, 0), qf[0], f32x16_t{});
        s[1] = mfma<F>(rowx<KH>(lds, lr, 0), qf[0], f32x16_t{});
        dp[0] = mfma<F>(rowx<VI>(lds, lr, 0), df[0], f32x16_t{});
        dp[1] = mfma<F>(rowx<VH>(lds, lr, 0), df[0], f32x16_t{});
#pragma unroll
        for (int ks = 1; ks < 8; ++ks) {
            s[0] = mfma<F>(rowx<KI>(lds, lr, ks), qf[ks], s[0]);
            s[1] = mfma<F>(rowx<KH>(lds, lr, ks), qf[ks], s[1]);
            dp[0] = mfma<F>(rowx<VI>(lds, lr, ks), df[ks], dp[0]);
            dp[1] = mfma<F>(rowx<VH>(lds, lr, ks), df[ks], dp[1]);
            if (ks & 1) __builtin_amdgcn_sched_barrier(0);
        }
        float pr[32];
        const f32x2_t sl2v = {a.sl2, a.sl2}, lv = {-lse, -lse}, dv = {dlt, dlt};
#pragma unroll
        for (int i = 0; i < 32; i += 2) {
            const int j = i >> 4, ii = i & 15;
            const f32x2_t e = fma2<kPkDq>(f32x2_t{s[j][ii], s[j][ii + 1]}, sl2v, lv);
            pr[i] = __builtin_amdgcn_exp2f(e.x);
            pr[i + 1] = __builtin_amdgcn_exp2f(e.y);
        }
        if (diag) {
#pragma unroll
            for (int i = 0; i < 32; ++i) {
                const int key = k0 + 32 * (i >> 4) + (i & 3) + 8 * ((i & 15) >> 2) + 4 * hi;
                if (key > qrow) pr[i] = 0.f;
            }
        }
        if (KMASK) {
            const uint64_t w = km[k0 >> 6];                    // workgroup-uniform
            if (~w != 0ull) {
#pragma unroll
                for (int i = 0; i < 32; ++i) {
                    const int key = k0 + 32 * (i >> 4) + (i & 3) + 8 * ((i & 15) >> 2) + 4 * hi;
                    if (!key_bit(w, key)) pr[i] = 0.f;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 32; i += 2) {
            const int j = i >> 4, ii = i & 15;
            const f32x2_t r = submul2<kPkDq>(f32x2_t{dp[j][ii], dp[j][ii + 1]}, dv, f32x2_t{pr[i], pr[i + 1]});
            pr[i] = r.x;
            pr[i + 1] = r.y;
        }
        bf16x8_t sf[4];
        pack_b_frags<F>(*reinterpret_cast<const float(*)[16]>(&pr[0]), sf[0], sf[1]);
        pack_b_frags<F>(*reinterpret_cast<const float(*)[16]>(&pr[16]), sf[2], sf[3]);
        const uint32_t t0 = opaque(lo_t0), t4 = opaque(lo_t4);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
            for (int kst = 0; kst < 4; ++kst) dq[dt] = mfma<F>(trx<KI>(lds, t0, t4, kst, dt), sf[kst], dq[dt]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }

    template <int SLOT>
    __device__ __forceinline__ void tile(int t) {
        if (t + 1 < nt) issue(t + 1);
        if (t <= last) compute<SLOT>(t, t == last);
        vm_wait_all();
        __syncthreads();
    }

    __device__ __forceinline__ void run(int b, int h, int hk, int qb) {
        const int tid = threadIdx.x;
        lane = tid & 63;
        wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        hi = lane >> 5;
        l32 = lane & 31;
        const int q0 = qb * kDqQB;
        qw = q0 + wave * kFwdQW;
        qrow = qw + l32;
        const bool qvalid = qrow < a.S;
        const uint16_t* qp = a.q.p + b * a.q.sb + h * a.q.sh;
        const uint16_t* dop = a.dout.p + b * a.dout.sb + h * a.dout.sh;
        const uint16_t* kp = a.k.p + b * a.k.sb + hk * a.k.sh;
        const uint16_t* vp = a.v.p + b * a.v.sb + hk * a.v.sh;
        km = KMASK ? a.kmask + (int64_t)b * a.kmask_ld : nullptr;
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            if (qvalid) {
                qf[ks] = *reinterpret_cast<const bf16x8_t*>(qp + qrow * a.q.ss + 16 * ks + 8 * hi);
                df[ks] = *reinterpret_cast<const bf16x8_t*>(dop + qrow * a.dout.ss + 16 * ks + 8 * hi);
            } else {
                qf[ks] = __builtin_bit_cast(bf16x8_t, u32x4_t{0u, 0u, 0u, 0u});
                df[ks] = qf[ks];
            }
        }
        const int64_t srow = ((int64_t)b * a.Hq + h) * a.S + (qvalid ? qrow : 0);
        lse = qvalid ? a.lse[srow] : 0.f;
        {
            const uint16_t* op = a.o.p + b * a.o.sb + h * a.o.sh;
            float part = 0.f;
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) {
                const u32x4_t ov = qvalid ? *reinterpret_cast<const u32x4_t*>(op + qrow * a.o.ss + 16 * ks + 8 * hi)
                                          : u32x4_t{0u, 0u, 0u, 0u};
                const u32x4_t dv = __builtin_bit_cast(u32x4_t, df[ks]);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    part += lo16<F>(ov[j]) * lo16<F>(dv[j]);
                    part += hi16<F>(ov[j]) * hi16<F>(dv[j]);
                }
            }
            dlt = halves_sum(part);
            if (qvalid && hi == 0) a.delta[srow] = dlt;
        }
        const int kv_end = min(a.S, q0 + kDqQB);
        nt = (kv_end + kKV - 1) / kKV;
        last = min(nt - 1, qw / kKV);
        rk = uniform_rsrc(kp, (int64_t)a.S * a.k.ss * 2);
        rv = uniform_rsrc(vp, (int64_t)a.S * a.v.ss * 2);
        lds0 = lds_addr(lds);
        {
            const uint32_t r = (uint32_t)l32;
            lo_row = r * kRowB + ((16u * hi) ^ (swz(r) << 4));
            const TrLane tl = tr_lane(lane);
            lo_t0 = tl.krow * kRowB + (tl.feat_byte ^ (swz(tl.krow) << 4));
            lo_t4 = (tl.krow + 4) * kRowB + (tl.feat_byte ^ (swz(tl.krow + 4) << 4));
        }
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int i = 0; i < 16; ++i) dq[dt][i] = 0.f;
        if (nt > 0) issue(0);
        vm_wait_all();
        vm_wait_all_known();
        __syncthreads();
        for (int t = 0; t < nt; t += 2) {
            tile<0>(t);
            if (t + 1 < nt) tile<1>(t + 1);
        }
        if (qvalid) {
            uint16_t* out = a.dq + b * a.dq_sb + h * a.dq_sh + (int64_t)qrow * a.dq_ss;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int d = 32 * dt + 8 * g + 4 * hi;
                    uint2 w;
                    w.x = pk16<F>(dq[dt][4 * g] * a.scale, dq[dt][4 * g + 1] * a.scale);
                    w.y = pk16<F>(dq[dt][4 * g + 2] * a.scale, dq[dt][4 * g + 3] * a.scale);
                    *reinterpret_cast<uint2*>(out + d) = w;
                }
        }
    }
};

template <bool KMASK, int F>
__global__ __launch_bounds__(64 * kDqWaves, 8 / kDqWaves)
void attn_dq_kernel(DqArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * 2 * kTileB];      // 64 KiB
    const int nqb = (a.S + kDqQB - 1) / kDqQB;
    const int G = a.Hq / a.Hkv;
    const int total = nqb * a.Hq * a.B;
    // consecutive ids: the G heads of one (b, kv head) at one q block, heaviest (longest causal row)
    // q blocks first (pairing q blocks measured 1-2 % slower here than this order)
    const int L = xcd_logical(blockIdx.x, total);
    const int per_group = G * nqb;
    const int grp = L / per_group;
    const int rem = L - grp * per_group;
    const int hk = grp % a.Hkv;
    DqLean<KMASK, F> dl(a, lds);
    dl.run(grp / a.Hkv, hk * G + rem % G, hk, nqb - 1 - rem / G);
}

// ------------------------------------------------------------------------------------------------
// dK, dV: a workgroup = 8 waves x 32 keys (256 keys) of one (b, kv head); it sweeps the G query
// heads x 32-row query slices from the block's first key to S, so the G heads' contributions are
// summed in registers (no atomics). K fragments live in registers, V rows in LDS (64 KiB); the
// Q / dO slices (+ their lse / delta) arrive by LDS-DMA into a kDkvLeanRing-deep ring (slices it+1 ..
// it+kDkvLeanRing-1 in flight while slice it is computed; the end-of-slice wait is a counted vmcnt).
// Per slice and wave: S = Q K^T and dP = dO V^T with the row constants (-lse/c, -delta) as the
// initial accumulators, P = exp2(c S'), dS = P dP', dV^T += dO^T P, dK^T += Q^T dS.
// Measured alternatives (profiles/r01_attn_variants.jsonl): V fragments in registers instead of the
// LDS image, and one wave per SIMD with 64 keys per wave (AGPR accumulators), both ran slower: at
// 256 VGPRs the kernel already spills ~30 registers, and every extra live value adds scratch reloads
// (each one a vmcnt wait) to the loop.
// ------------------------------------------------------------------------------------------------
// 256 keys per dK/dV workgroup (8 waves); 128-key workgroups of 4 waves (two per CU, independent
// barriers) measured the same (profiles/r03_attn_dkv128_ab.jsonl)
constexpr int kKB = 256, kKW = 32, kDkvWaves = kKB / kKW, kSlice = 32;
constexpr int kSliceB = kSlice * kRowB;            // 8 KiB per operand slice
constexpr int kSliceBuf = 2 * kSliceB + 256;       // Q, dO, 32 lse + 32 delta
constexpr int kVImg = kKB * kRowB;                 // 64 KiB

struct DkvArgs {
    Tns q, k, v, dout;
    uint16_t* dk;
    int64_t dk_sb, dk_sh, dk_ss;
    uint16_t* dv;
    int64_t dv_sb, dv_sh, dv_ss;
    const float* lse;
    const float* delta;
    const uint64_t* kmask;
    int64_t kmask_ld;
    int B, Hq, Hkv, S;
    float sl2, scale;
};

// dK / dV (DkvLean): the slice loop unrolled by two so that the ring slot is a compile-time LDS offset (the ring now sits in front of the V
// image, within the ds_read immediate range), S and dP started from zero accumulators and the row
// constants applied afterwards in packed fp32 (p = exp2(c s - lse), ds = p (dp - delta): v_pk_fma /
// v_pk_add / v_pk_mul), the causal test only on diagonal slices. Round 2's loop spilled ~30 VGPRs
// (the per-lane addresses of the runtime slot), and each scratch reload inside the loop carried a
// vmcnt wait that also drained the slice prefetch.
// Measured and removed (git history): one wave per SIMD x 64 keys with the accumulators in
// AGPRs (two builds), slower.
// slices in the ring (slices it+1 .. it+R-1 in flight while slice it is computed; rings of 2, 3 and 4
// measured 2.17, 2.21, 2.21 ms for the whole backward: profiles/r03_attn_bwd_variants.jsonl)
constexpr int kDkvLeanRing = 2;
static_assert(kDkvLeanRing >= 2 && kDkvLeanRing * kSliceBuf + kVImg <= 160 * 1024, "dK/dV lean ring");
template <bool KMASK, int F>
struct DkvLean {
    const DkvArgs& a;
    uint8_t* lds;
    bf16x8_t kf[8];
    f32x16_t dvt[4], dkt[4];
    int G, lane, wave, hi, l32, k0, kw, key, n_sl, n_it, b, hk, per_slice;
    bool kvalid;
    uint32_t lds0;
    uint32_t lo_row, lo_v, lo_t0, lo_t4;      // lane constants of the row / V-row / transposed reads

    __device__ __forceinline__ DkvLean(const DkvArgs& a_, uint8_t* lds_) : a(a_), lds(lds_) {}

    __device__ __forceinline__ void issue(int it) {
        const int hh = it / n_sl, sl = n_sl - 1 - (it - hh * n_sl);
        const int h = hk * G + hh;
        const int s0 = k0 + sl * kSlice;
        const uint32_t buf = lds0 + (uint32_t)((it % kDkvLeanRing) * kSliceBuf);
        if (kDkvWaves == 8) {                              // waves 0-3: Q rows 8w.., waves 4-7: dO rows
            const bool is_q = wave < 4;
            const Tns& src = is_q ? a.q : a.dout;
            const uint16_t* base = src.p + b * src.sb + h * src.sh;
            dma_rows(uniform_rsrc(base, (int64_t)a.S * src.ss * 2), src.ss, buf + (is_q ? 0u : (uint32_t)kSliceB), s0,
                     s0 + 8 * (wave & 3), 2, lane);
        } else {                                           // 4 waves: Q and dO rows 8w .. 8w+7 each
            const uint16_t* qb = a.q.p + b * a.q.sb + h * a.q.sh;
            const uint16_t* db = a.dout.p + b * a.dout.sb + h * a.dout.sh;
            dma_rows(uniform_rsrc(qb, (int64_t)a.S * a.q.ss * 2), a.q.ss, buf, s0, s0 + 8 * wave, 2, lane);
            dma_rows(uniform_rsrc(db, (int64_t)a.S * a.dout.ss * 2), a.dout.ss, buf + (uint32_t)kSliceB, s0,
                     s0 + 8 * wave, 2, lane);
        }
        if (wave < 2 && lane < 8) {
            const float* row = (wave == 0 ? a.lse : a.delta) + ((int64_t)b * a.Hq + h) * a.S;
            dma16(uniform_rsrc(row, (int64_t)a.S * 4), __builtin_amdgcn_readfirstlane(buf + 2 * kSliceB + 128 * wave),
                  (s0 + 4 * lane) * 4);
        }
    }

    // the slice's s0, or -1 when no q of the slice sees a key of the wave (both phases skip it)
    __device__ __forceinline__ int slice_s0(int it) const {
        const int sl = n_sl - 1 - it % n_sl;               // descending q: the longest causal rows first
        const int s0 = k0 + sl * kSlice;
        return (s0 + kSlice - 1 < kw) ? -1 : s0;
    }

    // phase 1 of a slice (ring slot SLOT): S = Q K^T and dP = dO V^T
    template <int SLOT>
    __device__ __forceinline__ void qk(f32x16_t& s, f32x16_t& dp) {
        // ring slot SLOT at [SLOT * kSliceBuf, ...): Q rows, dO rows, lse[32], delta[32]; V image after the ring
        constexpr int QI = SLOT * kSliceBuf, DI = QI + kSliceB;
        const uint32_t lr = opaque(lo_row), lv = opaque(lo_v);
        s = mfma<F>(rowx<QI>(lds, lr, 0), kf[0], f32x16_t{});
        dp = mfma<F>(rowx<DI>(lds, lr, 0), rowx<0>(lds, lv, 0), f32x16_t{});
#pragma unroll
        for (int ks = 1; ks < 8; ++ks) {
            s = mfma<F>(rowx<QI>(lds, lr, ks), kf[ks], s);
            dp = mfma<F>(rowx<DI>(lds, lr, ks), rowx<0>(lds, lv, ks), dp);
            if (ks & 1) __builtin_amdgcn_sched_barrier(0);    // bound the reads hoisted ahead (VGPRs)
        }
    }

    // phase 2: P, dS, dV^T += dO^T P, dK^T += Q^T dS
    template <int SLOT>
    __device__ __forceinline__ void pv(int s0, const f32x16_t& s, const f32x16_t& dp) {
        constexpr int QI = SLOT * kSliceBuf, DI = QI + kSliceB;
        const float* cst = reinterpret_cast<const float*>(lds + QI + 2 * kSliceB);
        // rows q = s0 + (i&3) + 8(i>>2) + 4hi of register i; their constants are cst[8(i>>2) + 4hi + (i&3)]
        float pr[16], dsv[16];
        const f32x2_t sl2v = {a.sl2, a.sl2};
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 lz = *reinterpret_cast<const float4*>(cst + 8 * g + 4 * hi);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = 4 * g + 2 * h;
                const f32x2_t l2 = h ? f32x2_t{lz.z, lz.w} : f32x2_t{lz.x, lz.y};
                const f32x2_t e = fma2<kPkDkv>(f32x2_t{s[i], s[i + 1]}, sl2v, -l2);
                pr[i] = __builtin_amdgcn_exp2f(e.x);
                pr[i + 1] = __builtin_amdgcn_exp2f(e.y);
            }
        }
        if (s0 < kw + kKW - 1) {                           // the slice crosses this wave's diagonal
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int q = s0 + (i & 3) + 8 * (i >> 2) + 4 * hi;
                if (key > q) pr[i] = 0.f;
            }
        }
        if (KMASK && !kvalid) {
#pragma unroll
            for (int i = 0; i < 16; ++i) pr[i] = 0.f;
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 dz = *reinterpret_cast<const float4*>(cst + 32 + 8 * g + 4 * hi);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = 4 * g + 2 * h;
                const f32x2_t d2 = h ? f32x2_t{dz.z, dz.w} : f32x2_t{dz.x, dz.y};
                const f32x2_t r = submul2<kPkDkv>(f32x2_t{dp[i], dp[i + 1]}, d2, f32x2_t{pr[i], pr[i + 1]});
                dsv[i] = r.x;
                dsv[i + 1] = r.y;
            }
        }
        bf16x8_t pf[2], sf[2];
        pack_b_frags<F>(pr, pf[0], pf[1]);
        pack_b_frags<F>(dsv, sf[0], sf[1]);
        const uint32_t t0 = opaque(lo_t0), t4 = opaque(lo_t4);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int kq = 0; kq < 2; ++kq) {
                dvt[dt] = mfma<F>(trx<DI>(lds, t0, t4, kq, dt), pf[kq], dvt[dt]);
                dkt[dt] = mfma<F>(trx<QI>(lds, t0, t4, kq, dt), sf[kq], dkt[dt]);
                if (kq) __builtin_amdgcn_sched_barrier(0);
            }
    }

    // Both phases of slice it in one barrier interval. (Tried: waves 4-7 lagging half a slice behind
    // their SIMD partners - phase 2 of slice it-1, then phase 1 of slice it - so that one wave's MFMA
    // chain meets its partner's softmax VALU: S / dP then stay live across the barrier, and at 256
    // VGPRs per wave hipcc spilled ~90 registers inside the loop.)
    template <int SLOT>
    __device__ __forceinline__ void step(int it) {
        constexpr int R = kDkvLeanRing;
        if (it + R - 1 < n_it) issue(it + R - 1);          // into the slot slice it-1 used
        const int s0 = slice_s0(it);
        if (s0 >= 0) {
            f32x16_t s, dp;
            qk<SLOT>(s, dp);
            pv<SLOT>(s0, s, dp);
        }
        // slice it+1 landed; it+2 .. it+R-1 (those issued) may stay in flight
        vm_wait_upto(per_slice * max(0, min(R - 2, n_it - 2 - it)));
        __syncthreads();
    }

    template <int SLOT>
    __device__ __forceinline__ void steps(int it0) {       // slices it0 .. it0+R-1, slot = compile-time
        if (it0 + SLOT < n_it) {
            step<SLOT>(it0 + SLOT);
            if constexpr (SLOT + 1 < kDkvLeanRing) steps<SLOT + 1>(it0);
        }
    }

    __device__ __forceinline__ void run(int b_, int hk_, int kb) {
        b = b_;
        hk = hk_;
        G = a.Hq / a.Hkv;
        const int tid = threadIdx.x;
        lane = tid & 63;
        wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        hi = lane >> 5;
        l32 = lane & 31;
        k0 = kb * kKB;
        kw = k0 + wave * kKW;
        key = kw + l32;
        kvalid = !KMASK || (key < a.S && key_bit(a.kmask[(int64_t)b * a.kmask_ld + (key >> 6)], key));
        const uint16_t* kp = a.k.p + b * a.k.sb + hk * a.k.sh;
        const uint16_t* vp = a.v.p + b * a.v.sb + hk * a.v.sh;
        lds0 = lds_addr(lds);
        dma_rows(uniform_rsrc(vp, (int64_t)a.S * a.v.ss * 2), a.v.ss, lds0 + kDkvLeanRing * kSliceBuf, k0, kw, kKW / 4, lane);
        {
            const uint32_t r = (uint32_t)l32;
            lo_row = r * kRowB + ((16u * hi) ^ (swz(r) << 4));
            // V rows wave*32 + l32 (same swizzle as row l32), image after the ring (past the ds offset range)
            lo_v = lo_row + (uint32_t)(kDkvLeanRing * kSliceBuf + wave * kKW * kRowB);
            const TrLane tl = tr_lane(lane);
            lo_t0 = tl.krow * kRowB + (tl.feat_byte ^ (swz(tl.krow) << 4));
            lo_t4 = (tl.krow + 4) * kRowB + (tl.feat_byte ^ (swz(tl.krow + 4) << 4));
        }
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            if (key < a.S) kf[ks] = *reinterpret_cast<const bf16x8_t*>(kp + (int64_t)key * a.k.ss + 16 * ks + 8 * hi);
            else kf[ks] = __builtin_bit_cast(bf16x8_t, u32x4_t{0u, 0u, 0u, 0u});
        }
        n_sl = (a.S - k0 + kSlice - 1) / kSlice;
        n_it = G * n_sl;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int i = 0; i < 16; ++i) { dvt[dt][i] = 0.f; dkt[dt][i] = 0.f; }
        per_slice = (kDkvWaves == 8 ? 2 : 4) + (wave < 2 ? 1 : 0);   // DMA instructions per slice (+ lse / delta)
#pragma unroll
        for (int i = 0; i < kDkvLeanRing - 1; ++i)
            if (i < n_it) issue(i);
        vm_wait_all();
        vm_wait_all_known();                               // the K fragments too (compiler-visible)
        __syncthreads();
        for (int it = 0; it < n_it; it += kDkvLeanRing) steps<0>(it);
        if (key < a.S) {
            uint16_t* dkr = a.dk + b * a.dk_sb + hk * a.dk_sh + (int64_t)key * a.dk_ss;
            uint16_t* dvr = a.dv + b * a.dv_sb + hk * a.dv_sh + (int64_t)key * a.dv_ss;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int d = 32 * dt + 8 * g + 4 * hi;
                    uint2 w;
                    w.x = pk16<F>(dkt[dt][4 * g] * a.scale, dkt[dt][4 * g + 1] * a.scale);
                    w.y = pk16<F>(dkt[dt][4 * g + 2] * a.scale, dkt[dt][4 * g + 3] * a.scale);
                    *reinterpret_cast<uint2*>(dkr + d) = w;
                    w.x = pk16<F>(dvt[dt][4 * g], dvt[dt][4 * g + 1]);
                    w.y = pk16<F>(dvt[dt][4 * g + 2], dvt[dt][4 * g + 3]);
                    *reinterpret_cast<uint2*>(dvr + d) = w;
                }
        }
    }
};

template <bool KMASK, int F>
__global__ __launch_bounds__(kDkvWaves * 64, 2)
void attn_dkdv_kernel(DkvArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kVImg + kDkvLeanRing * kSliceBuf];
    const int nkb = (a.S + kKB - 1) / kKB;
    const int total = ((nkb + 1) / 2) * a.Hkv * a.B;
    // key blocks kb (long causal sweep) and nkb-1-kb (short) in one workgroup: equal work per
    // workgroup (1594 vs 1946 us unpaired at B16 Hq32 Hkv8 S2048)
    const PairTask t = pair_task(xcd_logical(blockIdx.x, total), nkb, 1, a.Hkv);
#pragma nounroll
    for (int i = 0; i < t.n; ++i) {
        if (i) __syncthreads();
        DkvLean<KMASK, F> dl(a, lds);
        dl.run(t.b, t.hk, t.blk[1 - i]);
    }
}

inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

int check_tensor(const smt_attn_tensor* t, const char* what, const char* fn) {
    if (!t || !t->ptr) return fail(-1, "%s: null %s", fn, what);
    if (!al16(t->ptr) || (t->sb & 7) || (t->sh & 7) || (t->ss & 7))
        return fail(-2, "%s: %s needs 16-byte aligned rows (strides %% 8 == 0)", fn, what);
    return 0;
}

int check_shape(const smt_attn_shape* s, const char* fn) {
    if (!s) return fail(-1, "%s: null shape", fn);
    if (s->B <= 0 || s->Hq <= 0 || s->Hkv <= 0 || s->S <= 0 || s->Hq % s->Hkv)
        return fail(-1, "%s: bad shape B=%d Hq=%d Hkv=%d S=%d", fn, s->B, s->Hq, s->Hkv, s->S);
    if (!(s->scale > 0.f)) return fail(-1, "%s: scale must be > 0", fn);
    if (s->dtype != SMT_DTYPE_BF16 && s->dtype != SMT_DTYPE_FP16)
        return fail(-1, "%s: dtype %d is not a 16-bit format (SMT_DTYPE_BF16 / SMT_DTYPE_FP16)", fn, (int)s->dtype);
    return 0;
}

// the (key mask, format) instance of a kernel template
#define SMT_ATTN_LAUNCH(kernel, kmask, dtype, grid, block, stream, args)                                         \
    do {                                                                                                      \
        if ((dtype) == SMT_DTYPE_FP16) {                                                                      \
            if (kmask) hipLaunchKernelGGL((kernel<true, SMT_DTYPE_FP16>), grid, block, 0, stream, args);     \
            else hipLaunchKernelGGL((kernel<false, SMT_DTYPE_FP16>), grid, block, 0, stream, args);          \
        } else {                                                                                              \
            if (kmask) hipLaunchKernelGGL((kernel<true, SMT_DTYPE_BF16>), grid, block, 0, stream, args);     \
            else hipLaunchKernelGGL((kernel<false, SMT_DTYPE_BF16>), grid, block, 0, stream, args);          \
        }                                                                                                     \
    } while (0)

Tns tns(const smt_attn_tensor* t) { return Tns{static_cast<const uint16_t*>(t->ptr), t->sb, t->sh, t->ss}; }

}  // namespace

extern "C" {

const char* smt_attn_last_error(void) { return g_err; }


int smt_attn_fwd_kmask(const smt_attn_tensor* q, const smt_attn_tensor* k, const smt_attn_tensor* v,
                       const smt_attn_tensor* o, float* lse, const uint64_t* key_mask, int64_t key_mask_ld,
                       const smt_attn_shape* shape, hipStream_t stream) {
    int rc;
    const char* fn = key_mask ? "smt_attn_fwd_kmask" : "smt_attn_fwd";
    if ((rc = check_shape(shape, fn)) || (rc = check_tensor(q, "q", fn)) || (rc = check_tensor(k, "k", fn)) ||
        (rc = check_tensor(v, "v", fn)) || (rc = check_tensor(o, "o", fn)))
        return rc;
    if (!lse) return fail(-1, "%s: null lse", fn);
    if (key_mask && key_mask_ld < (shape->S + 63) / 64)
        return fail(-1, "%s: key_mask_ld %lld < ceil(S / 64)", fn, (long long)key_mask_ld);
    FwdArgs a;
    a.q = tns(q); a.k = tns(k); a.v = tns(v);
    a.o = static_cast<uint16_t*>(o->ptr); a.o_sb = o->sb; a.o_sh = o->sh; a.o_ss = o->ss;
    a.lse = lse;
    a.kmask = key_mask; a.kmask_ld = key_mask_ld;
    a.B = shape->B; a.Hq = shape->Hq; a.Hkv = shape->Hkv; a.S = shape->S;
    a.sl2 = shape->scale * 1.4426950408889634f;
    const int64_t nqb = (shape->S + kFwdQB - 1) / kFwdQB;
    const int64_t blocks = nqb * shape->Hq * shape->B;
    if (blocks > 0x7fffffffLL) return fail(-1, "%s: too many blocks", fn);
    SMT_ATTN_LAUNCH(attn_fwd_kernel, key_mask, shape->dtype, dim3((unsigned)blocks), dim3(64 * kFwdWaves), stream, a);
    return check_launch("attn_fwd_kernel");
}

int smt_attn_fwd(const smt_attn_tensor* q, const smt_attn_tensor* k, const smt_attn_tensor* v,
                 const smt_attn_tensor* o, float* lse, const smt_attn_shape* shape, hipStream_t stream) {
    return smt_attn_fwd_kmask(q, k, v, o, lse, nullptr, 0, shape, stream);
}

int smt_attn_bwd_kmask(const smt_attn_tensor* q, const smt_attn_tensor* k, const smt_attn_tensor* v,
                       const smt_attn_tensor* o, const smt_attn_tensor* d_o, const float* lse, float* delta_ws,
                       const smt_attn_tensor* dq, const smt_attn_tensor* dk, const smt_attn_tensor* dv,
                       const uint64_t* key_mask, int64_t key_mask_ld, const smt_attn_shape* shape,
                       hipStream_t stream) {
    int rc;
    const char* fn = key_mask ? "smt_attn_bwd_kmask" : "smt_attn_bwd";
    if ((rc = check_shape(shape, fn)) || (rc = check_tensor(q, "q", fn)) || (rc = check_tensor(k, "k", fn)) ||
        (rc = check_tensor(v, "v", fn)) || (rc = check_tensor(o, "o", fn)) || (rc = check_tensor(d_o, "do", fn)) ||
        (rc = check_tensor(dq, "dq", fn)) || (rc = check_tensor(dk, "dk", fn)) || (rc = check_tensor(dv, "dv", fn)))
        return rc;
    if (!lse || !delta_ws) return fail(-1, "%s: null lse / delta workspace", fn);
    if (!al16(lse) || !al16(delta_ws) || (shape->S & 3)) return fail(-2, "%s: lse / delta need 16-byte rows (S %% 4 == 0)", fn);
    if (key_mask && key_mask_ld < (shape->S + 63) / 64)
        return fail(-1, "%s: key_mask_ld %lld < ceil(S / 64)", fn, (long long)key_mask_ld);
    const int B = shape->B, Hq = shape->Hq, Hkv = shape->Hkv, S = shape->S;
    const float sl2 = shape->scale * 1.4426950408889634f;

    DqArgs qa;
    qa.q = tns(q); qa.k = tns(k); qa.v = tns(v); qa.dout = tns(d_o); qa.o = tns(o);
    qa.dq = static_cast<uint16_t*>(dq->ptr); qa.dq_sb = dq->sb; qa.dq_sh = dq->sh; qa.dq_ss = dq->ss;
    qa.lse = lse; qa.delta = delta_ws;
    qa.kmask = key_mask; qa.kmask_ld = key_mask_ld;
    qa.B = B; qa.Hq = Hq; qa.Hkv = Hkv; qa.S = S; qa.sl2 = sl2; qa.scale = shape->scale;
    const int64_t nqb = (S + kDqQB - 1) / kDqQB;
    const dim3 qgrid((unsigned)(nqb * Hq * B)), qblock(64 * kDqWaves);
    SMT_ATTN_LAUNCH(attn_dq_kernel, key_mask, shape->dtype, qgrid, qblock, stream, qa);
    if ((rc = check_launch("attn_dq_kernel"))) return rc;

    DkvArgs ka;
    ka.q = tns(q); ka.k = tns(k); ka.v = tns(v); ka.dout = tns(d_o);
    ka.dk = static_cast<uint16_t*>(dk->ptr); ka.dk_sb = dk->sb; ka.dk_sh = dk->sh; ka.dk_ss = dk->ss;
    ka.dv = static_cast<uint16_t*>(dv->ptr); ka.dv_sb = dv->sb; ka.dv_sh = dv->sh; ka.dv_ss = dv->ss;
    ka.lse = lse; ka.delta = delta_ws;
    ka.kmask = key_mask; ka.kmask_ld = key_mask_ld;
    ka.B = B; ka.Hq = Hq; ka.Hkv = Hkv; ka.S = S; ka.sl2 = sl2; ka.scale = shape->scale;
    const int64_t nkb = (S + kKB - 1) / kKB;
    const dim3 grid((unsigned)(((nkb + 1) / 2) * Hkv * B));
    SMT_ATTN_LAUNCH(attn_dkdv_kernel, key_mask, shape->dtype, grid, dim3(kDkvWaves * 64), stream, ka);
    return check_launch("attn_dkdv_kernel");
}

int smt_attn_bwd(const smt_attn_tensor* q, const smt_attn_tensor* k, const smt_attn_tensor* v,
                 const smt_attn_tensor* o, const smt_attn_tensor* d_o, const float* lse, float* delta_ws,
                 const smt_attn_tensor* dq, const smt_attn_tensor* dk, const smt_attn_tensor* dv,
                 const smt_attn_shape* shape, hipStream_t stream) {
    return smt_attn_bwd_kmask(q, k, v, o, d_o, lse, delta_ws, dq, dk, dv, nullptr, 0, shape, stream);
}

}  // extern "C"
