// Causal grouped-query flash attention for gfx950 (CDNA4), head_dim 128, bf16 I/O, fp32 softmax.
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

__device__ __forceinline__ f32x16_t mfma(bf16x8_t a, bf16x8_t b, f32x16_t c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Two-lane fp32 arithmetic of the lean kernels' softmax. PK: packed (v_pk_fma_f32 / v_pk_add_f32 /
// v_pk_mul_f32, one issue per pair); otherwise two scalar VALU ops per pair (the packed forms cost
// more than two scalar ones when issued beside MFMAs, MI355X_MICROARCH issue-cost table). Results are
// bit-identical either way (the same IEEE operations). Per kernel: SMT_ATTN_PK_FWD / _DQ / _DKV.
#ifndef SMT_ATTN_PK_FWD
#define SMT_ATTN_PK_FWD 0
#endif
#ifndef SMT_ATTN_PK_DQ
#define SMT_ATTN_PK_DQ 1
#endif
#ifndef SMT_ATTN_PK_DKV
#define SMT_ATTN_PK_DKV 1
#endif
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

__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
    f32x2_t v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
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
__device__ __forceinline__ void pack_b_frags(const float (&p)[16], bf16x8_t& f0, bf16x8_t& f1) {
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = pk_bf16(p[2 * i], p[2 * i + 1]);
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
// SMT_ATTN_FASTSM: forward softmax with the scale folded into the exponent's FMA and the O / l
// rescale skipped when no row's running max changed in the tile (exact: alpha = 1 then)
#ifndef SMT_ATTN_FASTSM
#define SMT_ATTN_FASTSM 1
#endif
#ifndef SMT_ATTN_KNOWN_WAIT
#define SMT_ATTN_KNOWN_WAIT 1
#endif
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
// SMT_FWD_WAVES / SMT_DQ_WAVES: waves (x 32 query rows) per workgroup of the forward / dQ kernels.
// Every workgroup stages its own K/V tiles, so 8 waves (256 query rows, one workgroup per CU) halve
// the LDS-fill bytes per MFMA; measured at B16 Hq32 Hkv8 S2048 (profiles/r02_attn_waves.jsonl) the
// 8-wave forward ran 7 % slower (0.89 vs 0.83 ms) and the 8-wave dQ the same: these loops are not
// bound by the K/V fill, so 4 stays the default.
#ifndef SMT_FWD_WAVES
#define SMT_FWD_WAVES 4
#endif
#ifndef SMT_DQ_WAVES
#define SMT_DQ_WAVES 4
#endif
// SMT_FWD_PREF=1 (default): the lean forward reads its K / V fragments two MFMAs ahead
// (FwdLean::compute); with SMT_ATTN_PK_FWD=0 the forward 0.80 -> 0.76 ms at the bench shape
// (profiles/r04_f_attn_pref_ab.jsonl, 3 interleaved rounds)
#ifndef SMT_FWD_PREF
#define SMT_FWD_PREF 1
#endif
// SMT_DQ_PREF=1: the same for the lean dQ kernel (DqLean::compute): measured no faster (the dQ loop
// is not waiting on these reads at two waves per SIMD), and its key-mask build spills more
#ifndef SMT_DQ_PREF
#define SMT_DQ_PREF 0
#endif
constexpr int kFwdQW = 32, kFwdWaves = SMT_FWD_WAVES, kFwdQB = kFwdQW * kFwdWaves, kKV = 64;
constexpr int kDqWaves = SMT_DQ_WAVES, kDqQB = kFwdQW * kDqWaves;
static_assert(kFwdWaves == 4 || kFwdWaves == 8, "forward: 4 or 8 waves");
static_assert(kDqWaves == 4 || kDqWaves == 8, "dQ: 4 or 8 waves");
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

// Forward K/V staging: tiles of SMT_FWD_KV keys (64 or 32) in a SMT_FWD_RING-deep LDS ring;
// 64 x 2 = 32 x 4 = 64 KiB per workgroup (two workgroups per CU). 32-key tiles in a 3- or 4-deep
// ring measured 8-12 % slower than 64 x 2 (profiles/r01_attn_variants.jsonl): the forward is not
// bound by the K/V DMA latency once the prologue wait is compiler-visible.
#ifndef SMT_FWD_KV
#define SMT_FWD_KV 64
#endif
#ifndef SMT_FWD_RING
#define SMT_FWD_RING 2
#endif
constexpr int kFKV = SMT_FWD_KV, kFRing = SMT_FWD_RING, kFTileB = kFKV * kRowB, kFS = kFKV / 32;

template <bool KMASK>
__device__ __forceinline__ void fwd_block(const FwdArgs& a, uint8_t* lds, int b, int h, int hk, int qb) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hi = lane >> 5, l32 = lane & 31;
    const int q0 = qb * kFwdQB, qw = q0 + wave * kFwdQW;
    const uint16_t* qp = a.q.p + b * a.q.sb + h * a.q.sh;
    const uint16_t* kp = a.k.p + b * a.k.sb + hk * a.k.sh;
    const uint16_t* vp = a.v.p + b * a.v.sb + hk * a.v.sh;
    const uint64_t* km = KMASK ? a.kmask + (int64_t)b * a.kmask_ld : nullptr;

    const int qrow = qw + l32;
    bf16x8_t qf[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
        if (qrow < a.S) qf[ks] = *reinterpret_cast<const bf16x8_t*>(qp + qrow * a.q.ss + 16 * ks + 8 * hi);
        else qf[ks] = __builtin_bit_cast(bf16x8_t, u32x4_t{0u, 0u, 0u, 0u});
    }

    const int kv_end = min(a.S, q0 + kFwdQB);
    const int nt = (kv_end + kFKV - 1) / kFKV;
    const __amdgpu_buffer_rsrc_t rk = uniform_rsrc(kp, (int64_t)a.S * a.k.ss * 2);
    const __amdgpu_buffer_rsrc_t rv = uniform_rsrc(vp, (int64_t)a.S * a.v.ss * 2);
    const uint32_t lds0 = lds_addr(lds);
    constexpr int kRowsW = kFKV / kFwdWaves;             // rows of each operand tile one wave brings
    constexpr int per_tile = 2 * (kRowsW / 4);           // its DMA instructions per tile (K + V)
    auto issue = [&](int t) {
        const uint32_t slot = lds0 + (uint32_t)((t % kFRing) * 2 * kFTileB);
        dma_rows(rk, a.k.ss, slot, t * kFKV, t * kFKV + kRowsW * wave, kRowsW / 4, lane);
        dma_rows(rv, a.v.ss, slot + kFTileB, t * kFKV, t * kFKV + kRowsW * wave, kRowsW / 4, lane);
    };

    const TrLane tl = tr_lane(lane);
    f32x16_t o[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[dt][i] = 0.f;
    float m_run = kNegInf, l_run = 0.f;

    if (kFRing > 2 && SMT_ATTN_KNOWN_WAIT) vm_wait_all_known();    // Q fragments landed (compiler-visible)
#pragma unroll
    for (int i = 0; i < kFRing - 1; ++i)
        if (i < nt) issue(i);
    vm_wait_upto(per_tile * min(kFRing - 2, nt - 1));                // tile 0 landed
    if (kFRing == 2 && SMT_ATTN_KNOWN_WAIT) vm_wait_all_known();
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
        if (t + kFRing - 1 < nt) issue(t + kFRing - 1);               // into the buffer tile t-1 used
        const uint8_t* K = lds + (t % kFRing) * 2 * kFTileB;
        const uint8_t* V = K + kFTileB;
        const int k0 = t * kFKV;
        if (k0 <= qw + kFwdQW - 1) {
            f32x16_t sc[kFS];
#pragma unroll
            for (int j = 0; j < kFS; ++j)
#pragma unroll
                for (int i = 0; i < 16; ++i) sc[j][i] = 0.f;
#pragma unroll
            for (int ks = 0; ks < 8; ++ks)
#pragma unroll
                for (int j = 0; j < kFS; ++j) sc[j] = mfma(row_frag(K, 32 * j + l32, 32 * ks + 16 * hi), qf[ks], sc[j]);
#if SMT_ATTN_FASTSM
            // raw scores; the log2-domain scale is folded into the exponent's FMA, and the row max is
            // taken on the raw scores (scale > 0: max commutes with the monotone rounding of s * c)
            float x[16 * kFS];
#pragma unroll
            for (int j = 0; j < kFS; ++j)
#pragma unroll
                for (int i = 0; i < 16; ++i) x[16 * j + i] = sc[j][i];
#else
            float x[16 * kFS];
#pragma unroll
            for (int j = 0; j < kFS; ++j)
#pragma unroll
                for (int i = 0; i < 16; ++i) x[16 * j + i] = sc[j][i] * a.sl2;
#endif
            if (k0 + kFKV - 1 > qw) {                              // tile crosses this wave's diagonal
#pragma unroll
                for (int i = 0; i < 16 * kFS; ++i) {
                    const int key = k0 + 32 * (i >> 4) + (i & 3) + 8 * ((i & 15) >> 2) + 4 * hi;
                    if (key > qrow) x[i] = kNegInf;
                }
            }
            if (KMASK) {
                const uint64_t w = km[k0 >> 6];                    // workgroup-uniform
                if (~w != 0ull) {
#pragma unroll
                    for (int i = 0; i < 16 * kFS; ++i) {
                        const int key = k0 + 32 * (i >> 4) + (i & 3) + 8 * ((i & 15) >> 2) + 4 * hi;
                        if (!key_bit(w, key)) x[i] = kNegInf;
                    }
                }
            }
            float mloc = x[0];
#pragma unroll
            for (int i = 1; i < 16 * kFS; ++i) mloc = fmaxf(mloc, x[i]);
#if SMT_ATTN_FASTSM
            const float m_new = fmaxf(m_run, other_half_max(mloc) * a.sl2);
#else
            const float m_new = fmaxf(m_run, other_half_max(mloc));
#endif
            // a row with no visible key so far (key mask only) keeps m = -inf: exponentiate against 0
            const float m_use = (KMASK && m_new == kNegInf) ? 0.f : m_new;
            float p[16 * kFS];
            float sum = 0.f;
#pragma unroll
            for (int i = 0; i < 16 * kFS; ++i) {
#if SMT_ATTN_FASTSM
                p[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(x[i], a.sl2, -m_use));
#else
                p[i] = __builtin_amdgcn_exp2f(x[i] - m_use);
#endif
                sum += p[i];
            }
            // rescale only when some row's max grew (alpha = 1 exactly otherwise: skipping is exact)
            if (!SMT_ATTN_FASTSM || __builtin_amdgcn_ballot_w64(m_new != m_run) != 0) {   // wave-uniform
                const float alpha = __builtin_amdgcn_exp2f(m_run - m_use);
                l_run *= alpha;
#pragma unroll
                for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                    for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
            }
            l_run += sum;
            m_run = m_new;
            bf16x8_t pf[2 * kFS];
#pragma unroll
            for (int j = 0; j < kFS; ++j)
                pack_b_frags(*reinterpret_cast<const float(*)[16]>(&p[16 * j]), pf[2 * j], pf[2 * j + 1]);
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int kst = 0; kst < 2 * kFS; ++kst) o[dt] = mfma(tr_frag(V, tl, 16 * kst, 32 * dt), pf[kst], o[dt]);
        }
        vm_wait_upto(per_tile * max(0, min(kFRing - 2, nt - 2 - t)));   // tile t+1 landed
        __syncthreads();
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
                w.x = pk_bf16(o[dt][4 * g] * inv, o[dt][4 * g + 1] * inv);
                w.y = pk_bf16(o[dt][4 * g + 2] * inv, o[dt][4 * g + 3] * inv);
                *reinterpret_cast<uint2*>(op + d) = w;
            }
        if (hi == 0)
            a.lse[((int64_t)b * a.Hq + h) * a.S + qrow] =
                (KMASK && !(l_tot > 0.f)) ? __builtin_huge_valf() : m_run + __log2f(l_tot);
    }
}

// ------------------------------------------------------------------------------------------------
// Forward, software-pipelined (SMT_ATTN_FWD_PIPE, default). Same workgroup geometry, K/V tiles and
// LDS ring as fwd_block; the loop is restructured after the PMC capture of round 3
// (profiles/r03_attn_pmc.json: 8.1 VALU instructions per MFMA, MFMA busy 0.39 -- the softmax VALU
// of a tile sat between that tile's QK^T and PV MFMAs, and the diagonal masking and O rescale were
// branches inside the loop body). Step t of a wave runs three independent pieces of work:
//   QK^T of tile t+1 (16 MFMA, K rows by ds_read_b128)       -> scores S(t+1)
//   softmax of tile t  (VALU: max, exp2, sum, bf16 pack)     -> P(t)
//   PV of tile t-1     (16 MFMA, V by ds_read_b64_tr_b16)    -> O += P(t-1) V(t-1)
// in one branch-free basic block, so the scheduler interleaves the VALU with the 32 MFMAs. K(t+1)
// and V(t-1) are read in step t, K(t+2) and V(t) are written: both live in LDS slot t%2 / (t+1)%2,
// one barrier per step. The running max is deferred (cdna_hip_programming T13): a row's max moves
// only when a tile's max exceeds it by more than kFwdThr (log2 units), so P <= 2^kFwdThr and the O
// rescale (a branch after the step's PV) is rare; P = exp2(s*c - m) keeps bf16's relative precision.
// The only masked tile of a wave (the causal diagonal) is its last one, handled by a step variant.
// ------------------------------------------------------------------------------------------------
// SMT_ATTN_FWD_IMPL: 0 fwd_block, 1 FwdPipe (one workgroup per CU), 2 FwdLean (two per CU),
// 3 FwdDual (one wave per SIMD, 64 rows per wave; attn_fwd_dual_kernel)
#ifndef SMT_ATTN_FWD_IMPL
#define SMT_ATTN_FWD_IMPL 2
#endif
#define SMT_ATTN_FWD_PIPE (SMT_ATTN_FWD_IMPL == 1)
constexpr float kFwdThr = 8.f;
constexpr int kFwdSlots = 3;
// SMT_ATTN_FWD_AHEAD: LDS fragment reads issued this many MFMAs ahead of their use
#ifndef SMT_ATTN_FWD_AHEAD
#define SMT_ATTN_FWD_AHEAD 2
#endif
constexpr int kFwdAhead = SMT_ATTN_FWD_AHEAD;


// v_max3_f32 as one instruction: fmaxf on MFMA results makes hipcc canonicalise both inputs first
// (an extra v_max per operand; cdna_hip_programming Appendix B, attention pitfalls)
__device__ __forceinline__ float max3f(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

template <bool KMASK>
struct FwdPipe {
    const FwdArgs& a;
    uint8_t* lds;
    uint32_t lds0;
    __amdgpu_buffer_rsrc_t rk, rv;
    const uint64_t* km;
    const uint8_t* qimg;        // this wave's 32 Q rows in LDS (read per MFMA: frees 32 VGPRs)
    f32x16_t o[4];
    f32x16_t sc[2][2];          // scores of two tiles (step parity)
    bf16x8_t pf[2][4];          // packed P of two tiles (step parity)
    float m_run, l_run;
    int qw, qrow, hi, l32, wave, lane, nt, last;
    TrLane tl;

    __device__ __forceinline__ FwdPipe(const FwdArgs& a_, uint8_t* lds_) : a(a_), lds(lds_) {}

    // LDS ring of 3 slots of {K tile, V tile}: tile t lives in slot t % 3 (K(t+3) and V(t+1) are
    // fetched in step t, two steps before they are read, so an HBM fetch has a whole step to land)
    __device__ __forceinline__ uint8_t* slot(int t) { return lds + (t % kFwdSlots) * 2 * kTileB; }

    __device__ __forceinline__ void issue_k(int t) {
        dma_rows(rk, a.k.ss, lds0 + (uint32_t)((t % kFwdSlots) * 2 * kTileB), t * kKV, t * kKV + 16 * wave, 4, lane);
    }
    __device__ __forceinline__ void issue_v(int t) {
        dma_rows(rv, a.v.ss, lds0 + (uint32_t)((t % kFwdSlots) * 2 * kTileB + kTileB), t * kKV, t * kKV + 16 * wave, 4,
                 lane);
    }

    template <int P>
    __device__ __forceinline__ void qk(int t) {               // S(t) = K(t) Q^T  -> sc[P]
        const uint8_t* K = slot(t);
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            const bf16x8_t qf = row_frag(qimg, l32, 32 * ks + 16 * hi);
#pragma unroll
            for (int j = 0; j < 2; ++j)
                sc[P][j] = mfma(row_frag(K, 32 * j + l32, 32 * ks + 16 * hi), qf, ks == 0 ? f32x16_t{} : sc[P][j]);
        }
    }

    template <int P>
    __device__ __forceinline__ void pv(int t) {               // O += P(t) V(t)  (pf[P])
        const uint8_t* V = slot(t) + kTileB;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int kst = 0; kst < 4; ++kst) o[dt] = mfma(tr_frag(V, tl, 16 * kst, 32 * dt), pf[P][kst], o[dt]);
    }

    // softmax of tile t (scores sc[P]) -> pf[P]; returns this lane's rescale factor (1: none).
    // Used by the first / last steps of a wave (and the diagonal tile, DIAG).
    template <int P, bool DIAG>
    __device__ __forceinline__ float softmax(int t) {
        const int k0 = t * kKV;
        float x[32];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) x[16 * j + i] = sc[P][j][i];
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
        const bool move = m_tile > m_run + kFwdThr;           // -inf + thr = -inf: the first tile moves
        const float m_new = move ? m_tile : m_run;
        const float alpha = move ? __builtin_amdgcn_exp2f(m_run - m_new) : 1.f;
        const float m_use = (KMASK && m_new == kNegInf) ? 0.f : m_new;
#pragma unroll
        for (int i = 0; i < 32; ++i) x[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(x[i], a.sl2, -m_use));
        float sm[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) sm[i] = x[i] + x[i + 16];
#pragma unroll
        for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
            for (int i = 0; i < w; ++i) sm[i] += sm[i + w];
        l_run = l_run * alpha + sm[0];
        m_run = m_new;
        pack_b_frags(*reinterpret_cast<const float(*)[16]>(&x[0]), pf[P][0], pf[P][1]);
        pack_b_frags(*reinterpret_cast<const float(*)[16]>(&x[16]), pf[P][2], pf[P][3]);
        return alpha;
    }

    __device__ __forceinline__ void rescale(float alpha) {
        if (__builtin_amdgcn_ballot_w64(alpha != 1.f) != 0) {      // rare (deferred max)
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
        }
    }

    // The steady-state step (1 <= t < last), hand-interleaved: 32 chunks, each one MFMA (16 of
    // QK(t+1), then 16 of PV(t-1)) with the LDS reads of the MFMA two chunks ahead and a slice of the
    // softmax of tile t (chunks 0-7 row max, 8 the deferred-max decision, 9-24 exp2, 25-27 row sum,
    // 28-31 bf16 pack of P(t) into pf[P]), fenced by sched_barrier so that every MFMA gap carries
    // about 24 cycles of VALU issue (MI355X_MICROARCH "vector-instruction ISSUE cost";
    // cdna_hip_programming Appendix B). The empty asm statements pin each slice's results to its chunk
    // (the SelectionDAG otherwise emits pure arithmetic next to its first use, e.g. the row sum at the
    // next step's head).
    // per-step state of the chunked softmax
    struct Chunks {
        const uint8_t* K;
        const uint8_t* V;
        float x[32], mx[1], sm[16];
        bf16x8_t fr[kFwdAhead + 1], qr[2];
        float m_new, alpha, m_use;
        int k0;
        uint64_t kw;                                             // key-mask word of tile t (KMASK)
    };

    __device__ __forceinline__ bf16x8_t frag(const Chunks& st, int c) {   // operand A of MFMA c
        if (c < 16) return row_frag(st.K, 32 * (c & 1) + l32, 32 * (c >> 1) + 16 * hi);
        const int cc = c - 16;                                   // PV: key step cc >> 2, d tile cc & 3
        return tr_frag(st.V, tl, 16 * (cc >> 2), 32 * (cc & 3));
    }

    template <int P, int C>
    __device__ __forceinline__ void chunk(Chunks& st) {
        constexpr int A = kFwdAhead;
        if constexpr (C + A < 32) st.fr[(C + A) % (A + 1)] = frag(st, C + A);
        // Q fragment ks is read two chunks before its first MFMA (chunk 2 ks) and used twice
        if constexpr (C + 2 < 16 && ((C + 2) & 1) == 0) st.qr[((C + 2) >> 1) & 1] = row_frag(qimg, l32, 32 * ((C + 2) >> 1) + 16 * hi);
        if constexpr (C < 16) {
            constexpr int ks = C >> 1, j = C & 1;
            sc[P ^ 1][j] = mfma(st.fr[C % (A + 1)], st.qr[ks & 1], ks == 0 ? f32x16_t{} : sc[P ^ 1][j]);
        } else {
            constexpr int cc = C - 16;
            o[cc & 3] = mfma(st.fr[C % (A + 1)], pf[P ^ 1][cc >> 2], o[cc & 3]);
        }
        float* x = st.x;
        float* sm = st.sm;
        // ---- softmax slice C of tile t ----
        if constexpr (C < 8) {                                   // row max over x[4C .. 4C+3]
            float v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = sc[P][C >> 2][4 * (C & 3) + i];
            if (KMASK) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int idx = 4 * C + i;
                    const int key = st.k0 + 32 * (idx >> 4) + (idx & 3) + 8 * ((idx & 15) >> 2) + 4 * hi;
                    if (!key_bit(st.kw, key)) v[i] = kNegInf;
                }
            }
            const float m0 = C == 0 ? v[0] : st.mx[0];
            st.mx[0] = max3f(max3f(m0, v[0], v[1]), v[2], v[3]);
#pragma unroll
            for (int i = 0; i < 4; ++i) x[4 * C + i] = v[i];
            asm volatile("" ::"v"(st.mx[0]));
        } else if constexpr (C == 8) {
            const float m_tile = other_half_max(st.mx[0]) * a.sl2;
            const bool move = m_tile > m_run + kFwdThr;          // -inf + thr = -inf: the first tile moves
            st.m_new = move ? m_tile : m_run;
            st.alpha = move ? __builtin_amdgcn_exp2f(m_run - st.m_new) : 1.f;
            st.m_use = (KMASK && st.m_new == kNegInf) ? 0.f : st.m_new;
            asm volatile("" ::"v"(st.m_use), "v"(st.alpha));
        } else if constexpr (C < 25) {                           // 2 x exp2(s*c - m)
            constexpr int i = 2 * (C - 9);
            x[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(x[i], a.sl2, -st.m_use));
            x[i + 1] = __builtin_amdgcn_exp2f(__builtin_fmaf(x[i + 1], a.sl2, -st.m_use));
            asm volatile("" ::"v"(x[i]), "v"(x[i + 1]));
        } else if constexpr (C == 25) {                          // row sum (tree)
#pragma unroll
            for (int i = 0; i < 11; ++i) sm[i] = x[i] + x[i + 16];
            asm volatile("" ::"v"(sm[0]), "v"(sm[1]), "v"(sm[2]), "v"(sm[3]), "v"(sm[4]), "v"(sm[5]), "v"(sm[6]),
                         "v"(sm[7]), "v"(sm[8]), "v"(sm[9]), "v"(sm[10]));
        } else if constexpr (C == 26) {
#pragma unroll
            for (int i = 11; i < 16; ++i) sm[i] = x[i] + x[i + 16];
#pragma unroll
            for (int i = 0; i < 5; ++i) sm[i] += sm[i + 8];
            asm volatile("" ::"v"(sm[0]), "v"(sm[1]), "v"(sm[2]), "v"(sm[3]), "v"(sm[4]), "v"(sm[5]), "v"(sm[6]),
                         "v"(sm[7]), "v"(sm[13]), "v"(sm[14]), "v"(sm[15]));
        } else if constexpr (C == 27) {
#pragma unroll
            for (int i = 5; i < 8; ++i) sm[i] += sm[i + 8];
#pragma unroll
            for (int i = 0; i < 4; ++i) sm[i] += sm[i + 4];
            sm[0] += sm[2];
            sm[1] += sm[3];
            l_run = l_run * st.alpha + (sm[0] + sm[1]);
            m_run = st.m_new;
            asm volatile("" ::"v"(l_run), "v"(m_run));
        } else {                                                 // 28..31: bf16 pack of P(t) into pf[P]
            constexpr int h = (C - 28) >> 1, g = (C - 28) & 1;   // P[16h + 8g .. 16h + 8g + 7]
            uint32_t w[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) w[i] = pk_bf16(x[16 * h + 8 * g + 2 * i], x[16 * h + 8 * g + 2 * i + 1]);
            // pack_b_frags for half h: words 4g'..4g'+3 of that half; chunk g = 0 holds words 0-3, g = 1 words 4-7
            auto p0 = __builtin_amdgcn_permlane32_swap(w[0], w[2], false, false);
            auto p1 = __builtin_amdgcn_permlane32_swap(w[1], w[3], false, false);
            u32x4_t v = {p0[0], p1[0], p0[1], p1[1]};
            pf[P][2 * h + g] = __builtin_bit_cast(bf16x8_t, v);
        }
        __builtin_amdgcn_sched_barrier(0);
    }

    template <int P, int... C>
    __device__ __forceinline__ void chunks(Chunks& st, std::integer_sequence<int, C...>) {
        (chunk<P, C>(st), ...);
    }

    // The steady-state step (1 <= t < last), hand-interleaved: 32 chunks, each one MFMA (16 of
    // QK(t+1), then 16 of PV(t-1)) with the LDS reads of the MFMA two chunks ahead and a slice of the
    // softmax of tile t (chunks 0-7 row max, 8 the deferred-max decision, 9-24 exp2, 25-27 row sum,
    // 28-31 bf16 pack of P(t) into pf[P]), fenced by sched_barrier so that every MFMA gap carries
    // about 24 cycles of VALU issue (MI355X_MICROARCH "vector-instruction ISSUE cost";
    // cdna_hip_programming Appendix B). The empty asm statements pin each slice's results to its chunk
    // (the SelectionDAG otherwise emits pure arithmetic next to its first use, e.g. the row sum at the
    // next step's head).
    template <int P, int R>
    __device__ __forceinline__ float steady(int t) {
        Chunks st;
        // P == t & 1, R == t % 3: K(t+1) in slot (R+1) % 3, V(t-1) in slot (R+2) % 3, compile-time LDS
        // offsets, so the per-lane fragment addresses are loop-invariant and the slot an immediate
        st.K = lds + ((R + 1) % kFwdSlots) * 2 * kTileB;
        st.V = lds + ((R + 2) % kFwdSlots) * 2 * kTileB + kTileB;
        st.k0 = t * kKV;
        st.kw = KMASK ? km[st.k0 >> 6] : ~0ull;
#pragma unroll
        for (int i = 0; i < kFwdAhead; ++i) st.fr[i] = frag(st, i);
        st.qr[0] = row_frag(qimg, l32, 16 * hi);
        st.m_new = 0.f;
        st.alpha = 1.f;
        st.m_use = 0.f;
        chunks<P>(st, std::make_integer_sequence<int, 32>{});
        return st.alpha;
    }

    // Step t with P = t & 1: DMA K(t+3) and V(t+1); QK(t+1) -> sc[P^1]; softmax(t): sc[P] -> pf[P];
    // PV(t-1) with pf[P^1]; then wait for the DMAs of the previous step (K(t+2), V(t)) and the
    // barrier. Every wave runs steps 0..nt (one barrier each): its steady steps 1..last-1 in a loop
    // of their own (so the O accumulators stay in one register set across the loop), the first,
    // diagonal, drain and idle steps through gen_step.
    __device__ __forceinline__ int issue(int t) {           // returns the DMA instructions issued
        int n = 0;
        if (t + 3 < nt) { issue_k(t + 3); n += 4; }
        if (t + 1 < nt) { issue_v(t + 1); n += 4; }
        return n;
    }

    template <int P, int R>
    __device__ __forceinline__ void steady_step(int t) {
        const int n = issue(t);
        rescale(steady<P, R>(t));
        vm_wait_upto(n);                                       // this step's DMAs may stay in flight
        __syncthreads();
    }

    template <int P>
    __device__ __forceinline__ void gen_step(int t) {
        const int n = issue(t);
        if (t <= last + 1) {
            float alpha = 1.f;
            if (t + 1 <= last) qk<P ^ 1>(t + 1);
            if (t == last) alpha = softmax<P, true>(t);
            else if (t < last) alpha = softmax<P, false>(t);
            if (t >= 1) pv<P ^ 1>(t - 1);
            rescale(alpha);
        }
        vm_wait_upto(n);
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
        const int kv_end = min(a.S, q0 + kFwdQB);
        nt = (kv_end + kKV - 1) / kKV;
        last = min(nt - 1, qw / kKV);                          // this wave's diagonal tile
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

        // LDS: K/V ring (3 slots x 32 KiB), then the 4 waves' Q rows (4 x 8 KiB)
        constexpr int kRingB = kFwdSlots * 2 * kTileB;
        qimg = lds + kRingB + wave * (kFwdQW * kRowB);
        dma_rows(uniform_rsrc(qp, (int64_t)a.S * a.q.ss * 2), a.q.ss, lds0 + kRingB + wave * (kFwdQW * kRowB),
                 qw, qw, kFwdQW / 4, lane);
        for (int i = 0; i < 3; ++i)
            if (i < nt) issue_k(i);
        issue_v(0);
        vm_wait_all();
        __syncthreads();
        qk<0>(0);
        __syncthreads();                                       // K(0)'s slot is rewritten in step 0
        gen_step<0>(0);
        int t = 1;
        // the steady steps, six per trip (t % 2 and t % 3 compile-time; t % 6 == 1 at entry), leaving
        // after any step
        while (t < last) {
            steady_step<1, 1>(t++);
            if (t >= last) break;
            steady_step<0, 2>(t++);
            if (t >= last) break;
            steady_step<1, 0>(t++);
            if (t >= last) break;
            steady_step<0, 1>(t++);
            if (t >= last) break;
            steady_step<1, 2>(t++);
            if (t >= last) break;
            steady_step<0, 0>(t++);
        }
        for (; t <= nt; ++t) {
            if (t & 1) gen_step<1>(t);
            else gen_step<0>(t);
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
                    w.x = pk_bf16(o[dt][4 * g] * inv, o[dt][4 * g + 1] * inv);
                    w.y = pk_bf16(o[dt][4 * g + 2] * inv, o[dt][4 * g + 3] * inv);
                    *reinterpret_cast<uint2*>(op + d) = w;
                }
            if (hi == 0)
                a.lse[((int64_t)b * a.Hq + h) * a.S + qrow] =
                    (KMASK && !(l_tot > 0.f)) ? __builtin_huge_valf() : m_run + __log2f(l_tot);
        }
    }
};

// ------------------------------------------------------------------------------------------------
// Forward, lean (SMT_ATTN_FWD_IMPL 2): fwd_block's structure (two workgroups per CU, i.e. two waves
// per SIMD whose MFMA and VALU phases overlap each other; Q in registers; a 2-slot K/V ring, one
// barrier per 64-key tile) with the per-tile VALU cut to what the softmax needs: tiles in pairs so the
// LDS slot is a compile-time offset (no per-read address adds), the scores' first MFMA on a zero
// accumulator (no per-tile zeroing), the row max by v_max3 without canonicalisation, row max / sum
// as trees, the deferred max of FwdPipe (no per-tile O rescale) and the causal mask only on the
// wave's diagonal tile.
// ------------------------------------------------------------------------------------------------
// SMT_ATTN_STAMPS (diagnostic builds only): every 64th forward workgroup's waves record, per K/V
// tile, the shader clock (s_memtime) at the tile start, after its compute, after the DMA wait and
// after the barrier; read back with smt_attn_debug_fwd_stamps (scripts/diag/attn_stamps.py)
#ifndef SMT_ATTN_STAMPS
#define SMT_ATTN_STAMPS 0
#endif
constexpr int kStampEvery = 64, kStampBlocks = 256, kStampTiles = 32;
#if SMT_ATTN_STAMPS
__device__ uint64_t g_fwd_stamps[kStampBlocks][4][kStampTiles][4];
// dK/dV: every 64th workgroup's 8 waves, the first 64 query slices: start, after S / dP, after the
// dV / dK products, after the DMA wait, after the barrier
constexpr int kDkvStampSlices = 64;
__device__ uint64_t g_dkv_stamps[kStampBlocks][8][kDkvStampSlices][5];
#endif

template <bool KMASK>
struct FwdLean {
    const FwdArgs& a;
    uint8_t* lds;
    uint64_t* stamps = nullptr;   // SMT_ATTN_STAMPS: this wave's [kStampTiles][4] record, or null
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
#if SMT_FWD_PREF
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
            for (int j = 0; j < 2; ++j) sc[j] = mfma(kf[ks % 3][j], qf[ks], ks ? sc[j] : f32x16_t{});
            __builtin_amdgcn_sched_barrier(0);
        }
        // the first two V fragments of the PV product, in flight during the softmax
        bf16x8_t vf[3];
        vf[0] = tr_frag(V, tl, 0, 0);
        vf[1] = tr_frag(V, tl, 16, 0);
#else
#pragma unroll
        for (int j = 0; j < 2; ++j) sc[j] = mfma(row_frag(K, 32 * j + l32, 16 * hi), qf[0], f32x16_t{});
#pragma unroll
        for (int ks = 1; ks < 8; ++ks)
#pragma unroll
            for (int j = 0; j < 2; ++j) sc[j] = mfma(row_frag(K, 32 * j + l32, 32 * ks + 16 * hi), qf[ks], sc[j]);
#endif
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
            const f32x2_t e = fma2<SMT_ATTN_PK_FWD != 0>(f32x2_t{x[2 * i], x[2 * i + 1]}, sl2v, mv);
            x[2 * i] = __builtin_amdgcn_exp2f(e.x);
            x[2 * i + 1] = __builtin_amdgcn_exp2f(e.y);
            sm[i] = f32x2_t{x[2 * i], x[2 * i + 1]};
        }
#pragma unroll
        for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
            for (int i = 0; i < w; ++i) sm[i] = add2<SMT_ATTN_PK_FWD != 0>(sm[i], sm[i + w]);
        l_run = l_run * alpha + (sm[0].x + sm[0].y);
        m_run = m_new;
        if (__builtin_amdgcn_ballot_w64(move) != 0) {          // rare (deferred max)
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
        }
        bf16x8_t pf[4];
        pack_b_frags(*reinterpret_cast<const float(*)[16]>(&x[0]), pf[0], pf[1]);
        pack_b_frags(*reinterpret_cast<const float(*)[16]>(&x[16]), pf[2], pf[3]);
#if SMT_FWD_PREF
        // V^T fragments two MFMAs ahead (n = 4 dt + kst)
#pragma unroll
        for (int n = 0; n < 16; ++n) {
            if (n + 2 < 16) vf[(n + 2) % 3] = tr_frag(V, tl, 16 * ((n + 2) & 3), 32 * ((n + 2) >> 2));
            __builtin_amdgcn_sched_barrier(0);
            o[n >> 2] = mfma(vf[n % 3], pf[n & 3], o[n >> 2]);
            __builtin_amdgcn_sched_barrier(0);
        }
#else
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int kst = 0; kst < 4; ++kst) o[dt] = mfma(tr_frag(V, tl, 16 * kst, 32 * dt), pf[kst], o[dt]);
#endif
    }

    // tile t (t & 1 == SLOT): fetch tile t+1 into the other slot, compute, wait, barrier
    template <int SLOT>
    __device__ __forceinline__ void tile(int t) {
#if SMT_ATTN_STAMPS
        const uint64_t s0 = __builtin_amdgcn_s_memtime();
#endif
        if (t + 1 < nt) issue(t + 1);
        if (t <= last) compute<SLOT, true>(t, t == last);
#if SMT_ATTN_STAMPS
        const uint64_t s1 = __builtin_amdgcn_s_memtime();
#endif
        vm_wait_all();
#if SMT_ATTN_STAMPS
        const uint64_t s2 = __builtin_amdgcn_s_memtime();
#endif
        __syncthreads();
#if SMT_ATTN_STAMPS
        const uint64_t s3 = __builtin_amdgcn_s_memtime();
        if (stamps != nullptr && lane == 0 && t < kStampTiles) {
            stamps[4 * t] = s0; stamps[4 * t + 1] = s1; stamps[4 * t + 2] = s2; stamps[4 * t + 3] = s3;
        }
#endif
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
                    w.x = pk_bf16(o[dt][4 * g] * inv, o[dt][4 * g + 1] * inv);
                    w.y = pk_bf16(o[dt][4 * g + 2] * inv, o[dt][4 * g + 3] * inv);
                    *reinterpret_cast<uint2*>(op + d) = w;
                }
            if (hi == 0)
                a.lse[((int64_t)b * a.Hq + h) * a.S + qrow] =
                    (KMASK && !(l_tot > 0.f)) ? __builtin_huge_valf() : m_run + __log2f(l_tot);
        }
    }
};

// ------------------------------------------------------------------------------------------------
// Forward, one wave per SIMD (SMT_ATTN_FWD_IMPL 3): a workgroup = 4 waves x 64 query rows (two 32-row
// blocks A, B per wave) = 256 rows of one (b, q head); 64-key K/V tiles in a kDualRing-deep LDS-DMA
// ring shared by the 4 waves. Each wave reads a tile's K and V fragments from LDS ONCE for both of
// its row blocks (half the LDS bytes per MFMA of the 32-row kernels, whose LDS traffic was ~3/4 of
// their MFMA time) and, with the whole 512-register file, holds both blocks' O (AGPRs), Q and scores.
// Per tile the two blocks are offset by one phase so that one block's softmax VALU overlaps the
// other block's MFMA chain inside the wave: QK(A); QK(B) || softmax(A); PV(A) || softmax(B); PV(B).
// ------------------------------------------------------------------------------------------------
#ifndef SMT_ATTN_DUAL_RING
#define SMT_ATTN_DUAL_RING 3
#endif
constexpr int kDualRing = SMT_ATTN_DUAL_RING, kDualQB = 256;
// SMT_ATTN_DUAL_OVERLAP=1: interior tiles run the two blocks offset by one phase (softmax chunks pinned
// beside the other block's MFMAs by scheduling fences). hipcc's register allocation of that body
// (O in AGPRs, Q / scores / probabilities / fragments in VGPRs) produced ~300 spill slots and ~2400
// AGPR<->VGPR moves, so it is off; the guide's one-wave-per-SIMD kernel owns its registers in asm.
#ifndef SMT_ATTN_DUAL_OVERLAP
#define SMT_ATTN_DUAL_OVERLAP 0
#endif

template <bool KMASK>
struct FwdDual {
    const FwdArgs& a;
    uint8_t* lds;
    bf16x8_t qa[8], qb[8];
    f32x16_t oa[4], ob[4];
    float ma, mb, la, lb;
    const uint64_t* km;
    __amdgpu_buffer_rsrc_t rk, rv;
    uint32_t lds0, lo_row, lo_t0, lo_t4;
    int lane, wave, hi, l32, qw, nt, last;

    __device__ __forceinline__ FwdDual(const FwdArgs& a_, uint8_t* lds_) : a(a_), lds(lds_) {}

    __device__ __forceinline__ void issue(int t) {            // K(t), V(t): 16 rows of each per wave
        const uint32_t slot = lds0 + (uint32_t)((t % kDualRing) * 2 * kTileB);
        dma_rows(rk, a.k.ss, slot, t * kKV, t * kKV + 16 * wave, 4, lane);
        dma_rows(rv, a.v.ss, slot + kTileB, t * kKV, t * kKV + 16 * wave, 4, lane);
    }

    __device__ __forceinline__ static void rescale(f32x16_t (&o)[4], float alpha) {
        if (__builtin_amdgcn_ballot_w64(alpha != 1.f) != 0) {     // rare (deferred max)
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
        }
    }

    // scores of one 32-row block against the tile's 64 keys (two 32-key halves) -> probabilities packed
    // as the PV B operand; the block's running max / sum and O updated (deferred max, T13)
    __device__ __forceinline__ void softmax(const f32x16_t (&sc)[2], int qrow, int k0, bool DIAG, float& m_run,
                                            float& l_run, f32x16_t (&o)[4], bf16x8_t (&pf)[4]) {
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
            const uint64_t w = km[k0 >> 6];
#pragma unroll
            for (int i = 0; i < 32; ++i) {
                const int key = k0 + 32 * (i >> 4) + (i & 3) + 8 * ((i & 15) >> 2) + 4 * hi;
                if (!key_bit(w, key)) x[i] = kNegInf;
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
        const f32x2_t sl2v = {a.sl2, a.sl2}, mv = {-m_use, -m_use};
        f32x2_t sm[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const f32x2_t e = __builtin_elementwise_fma(f32x2_t{x[2 * i], x[2 * i + 1]}, sl2v, mv);
            x[2 * i] = __builtin_amdgcn_exp2f(e.x);
            x[2 * i + 1] = __builtin_amdgcn_exp2f(e.y);
            sm[i] = f32x2_t{x[2 * i], x[2 * i + 1]};
        }
#pragma unroll
        for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
            for (int i = 0; i < w; ++i) sm[i] += sm[i + w];
        l_run = l_run * alpha + (sm[0].x + sm[0].y);
        m_run = m_new;
        rescale(o, alpha);
        pack_b_frags(*reinterpret_cast<const float(*)[16]>(&x[0]), pf[0], pf[1]);
        pack_b_frags(*reinterpret_cast<const float(*)[16]>(&x[16]), pf[2], pf[3]);
    }

    template <int SLOT>
    __device__ __forceinline__ void compute(int t, bool diag) {
        constexpr int KI = SLOT * 2 * kTileB, KH = KI + 32 * kRowB, VI = KI + kTileB;
        const int k0 = t * kKV;
        const uint32_t lr = opaque(lo_row);
        bf16x8_t kr[16];                                       // the tile's K fragments, read once
        f32x16_t sa[2], sb[2];
        kr[0] = rowx<KI>(lds, lr, 0);
        kr[1] = rowx<KH>(lds, lr, 0);
        sa[0] = mfma(kr[0], qa[0], f32x16_t{});
        sa[1] = mfma(kr[1], qa[0], f32x16_t{});
#pragma unroll
        for (int ks = 1; ks < 8; ++ks) {
            kr[2 * ks] = rowx<KI>(lds, lr, ks);
            kr[2 * ks + 1] = rowx<KH>(lds, lr, ks);
            sa[0] = mfma(kr[2 * ks], qa[ks], sa[0]);
            sa[1] = mfma(kr[2 * ks + 1], qa[ks], sa[1]);
        }
        // QK(B) || softmax(A)
        sb[0] = mfma(kr[0], qb[0], f32x16_t{});
        sb[1] = mfma(kr[1], qb[0], f32x16_t{});
#pragma unroll
        for (int ks = 1; ks < 8; ++ks) {
            sb[0] = mfma(kr[2 * ks], qb[ks], sb[0]);
            sb[1] = mfma(kr[2 * ks + 1], qb[ks], sb[1]);
        }
        bf16x8_t pa[4], pb[4];
        softmax(sa, qw + l32, k0, diag, ma, la, oa, pa);
        // PV(A) || softmax(B)
        const uint32_t t0 = opaque(lo_t0), t4 = opaque(lo_t4);
        bf16x8_t vr[16];
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int kst = 0; kst < 4; ++kst) {
                vr[4 * dt + kst] = trx<VI>(lds, t0, t4, kst, dt);
                oa[dt] = mfma(vr[4 * dt + kst], pa[kst], oa[dt]);
            }
        softmax(sb, qw + 32 + l32, k0, diag, mb, lb, ob, pb);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int kst = 0; kst < 4; ++kst) ob[dt] = mfma(vr[4 * dt + kst], pb[kst], ob[dt]);
    }

    // ---- the overlapped tile (interior tiles, no key mask): one block's softmax in 8 chunks, each
    // pinned beside two MFMAs of the other block's chain by scheduling fences ----
    struct Sm {
        float x[32];
        float mx;
        f32x2_t acc[4];
        float m_new, alpha, m_use;
    };

    template <int C>
    __device__ __forceinline__ void sm_chunk(Sm& st, const f32x16_t (&sc)[2], float& m_run, float& l_run,
                                             bf16x8_t (&pf)[4]) {
        float* x = st.x;
        if constexpr (C == 0 || C == 1) {                      // copy + row max over 16 scores
#pragma unroll
            for (int i = 0; i < 16; ++i) x[16 * C + i] = sc[C][i];
            const float* v = x + 16 * C;
            float m = max3f(v[0], v[1], v[2]);
            m = max3f(m, v[3], v[4]);
            m = max3f(m, v[5], v[6]);
            m = max3f(m, v[7], v[8]);
            m = max3f(m, v[9], v[10]);
            m = max3f(m, v[11], v[12]);
            m = max3f(m, v[13], v[14]);
            if constexpr (C == 0) {
                st.mx = fmaxf(m, v[15]);
            } else {
                m = max3f(m, v[15], st.mx);
                const float m_tile = other_half_max(m) * a.sl2;
                const bool move = m_tile > m_run + kFwdThr;
                st.m_new = move ? m_tile : m_run;
                st.alpha = move ? __builtin_amdgcn_exp2f(m_run - st.m_new) : 1.f;
                st.m_use = st.m_new;
            }
        } else if constexpr (C >= 2 && C <= 5) {               // 8 exponentials, packed scale-subtract
            constexpr int e0 = 8 * (C - 2);
            const f32x2_t sl2v = {a.sl2, a.sl2}, mv = {-st.m_use, -st.m_use};
            f32x2_t part = {0.f, 0.f};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const f32x2_t e = __builtin_elementwise_fma(f32x2_t{x[e0 + 2 * i], x[e0 + 2 * i + 1]}, sl2v, mv);
                x[e0 + 2 * i] = __builtin_amdgcn_exp2f(e.x);
                x[e0 + 2 * i + 1] = __builtin_amdgcn_exp2f(e.y);
                part = i ? part + f32x2_t{x[e0 + 2 * i], x[e0 + 2 * i + 1]} : f32x2_t{x[e0], x[e0 + 1]};
            }
            st.acc[C - 2] = part;
        } else if constexpr (C == 6) {                         // row sum, running max / sum
            const f32x2_t s2 = (st.acc[0] + st.acc[1]) + (st.acc[2] + st.acc[3]);
            l_run = l_run * st.alpha + (s2.x + s2.y);
            m_run = st.m_new;
            pack_b_frags(*reinterpret_cast<const float(*)[16]>(&x[0]), pf[0], pf[1]);
        } else {
            pack_b_frags(*reinterpret_cast<const float(*)[16]>(&x[16]), pf[2], pf[3]);
        }
    }

    // QK(B) re-reads the K fragments (16 KiB more LDS per tile) rather than keep 64 VGPRs of them
    template <int KI, int KH, int C>
    __device__ __forceinline__ void qk_b_step(uint32_t lr, f32x16_t (&sb)[2], Sm& st, const f32x16_t (&sa)[2],
                                              bf16x8_t (&pa)[4]) {
        sb[0] = mfma(rowx<KI>(lds, lr, C), qb[C], C == 0 ? f32x16_t{} : sb[0]);
        sb[1] = mfma(rowx<KH>(lds, lr, C), qb[C], C == 0 ? f32x16_t{} : sb[1]);
        sm_chunk<C>(st, sa, ma, la, pa);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (C + 1 < 8) qk_b_step<KI, KH, C + 1>(lr, sb, st, sa, pa);
    }

    template <int VI, int C>
    __device__ __forceinline__ void pv_a_step(uint32_t t0, uint32_t t4, bf16x8_t (&vr)[16], const bf16x8_t (&pa)[4],
                                              Sm& st, const f32x16_t (&sb)[2], bf16x8_t (&pb)[4]) {
        constexpr int dt = C >> 1, k0 = 2 * (C & 1);
        vr[4 * dt + k0] = trx<VI>(lds, t0, t4, k0, dt);
        vr[4 * dt + k0 + 1] = trx<VI>(lds, t0, t4, k0 + 1, dt);
        oa[dt] = mfma(vr[4 * dt + k0], pa[k0], oa[dt]);
        oa[dt] = mfma(vr[4 * dt + k0 + 1], pa[k0 + 1], oa[dt]);
        sm_chunk<C>(st, sb, mb, lb, pb);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (C + 1 < 8) pv_a_step<VI, C + 1>(t0, t4, vr, pa, st, sb, pb);
    }

    template <int SLOT>
    __device__ __forceinline__ void compute_overlap(int t) {
        constexpr int KI = SLOT * 2 * kTileB, KH = KI + 32 * kRowB, VI = KI + kTileB;
        const uint32_t lr = opaque(lo_row);
        f32x16_t sa[2], sb[2];
        sa[0] = mfma(rowx<KI>(lds, lr, 0), qa[0], f32x16_t{});
        sa[1] = mfma(rowx<KH>(lds, lr, 0), qa[0], f32x16_t{});
#pragma unroll
        for (int ks = 1; ks < 8; ++ks) {
            sa[0] = mfma(rowx<KI>(lds, lr, ks), qa[ks], sa[0]);
            sa[1] = mfma(rowx<KH>(lds, lr, ks), qa[ks], sa[1]);
            if (ks & 1) __builtin_amdgcn_sched_barrier(0);
        }
        Sm st;
        bf16x8_t pa[4], pb[4];
        const uint32_t lr2 = opaque(lo_row);
        qk_b_step<KI, KH, 0>(lr2, sb, st, sa, pa);             // QK(B) || softmax(A)
        rescale(oa, st.alpha);
        const uint32_t t0 = opaque(lo_t0), t4 = opaque(lo_t4);
        bf16x8_t vr[16];
        Sm st2;
        pv_a_step<VI, 0>(t0, t4, vr, pa, st2, sb, pb);         // PV(A) || softmax(B)
        rescale(ob, st2.alpha);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int kst = 0; kst < 4; ++kst) ob[dt] = mfma(vr[4 * dt + kst], pb[kst], ob[dt]);
    }

    template <int SLOT>
    __device__ __forceinline__ void tile(int t) {
        if (t + kDualRing - 1 < nt) issue(t + kDualRing - 1);  // into the slot tile t-1 used
        if (!KMASK && SMT_ATTN_DUAL_OVERLAP && t < last) compute_overlap<SLOT>(t);
        else if (t <= last) compute<SLOT>(t, t == last);
        vm_wait_upto(8 * max(0, min(kDualRing - 2, nt - 2 - t)));   // tile t+1 landed
        __syncthreads();
    }

    template <int SLOT>
    __device__ __forceinline__ void tiles(int t0) {            // tiles t0 .. t0+R-1, slot = compile-time
        if (t0 + SLOT < nt) {
            tile<SLOT>(t0 + SLOT);
            if constexpr (SLOT + 1 < kDualRing) tiles<SLOT + 1>(t0);
        }
    }

    __device__ __forceinline__ void store(const f32x16_t (&o)[4], float m_run, float l_run, int qrow, int b, int h) {
        const float l_tot = halves_sum(l_run);
        if (qrow >= a.S) return;
        const float inv = (KMASK && !(l_tot > 0.f)) ? 0.f : 1.f / l_tot;
        uint16_t* op = a.o + b * a.o_sb + h * a.o_sh + (int64_t)qrow * a.o_ss;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d = 32 * dt + 8 * g + 4 * hi;
                uint2 w;
                w.x = pk_bf16(o[dt][4 * g] * inv, o[dt][4 * g + 1] * inv);
                w.y = pk_bf16(o[dt][4 * g + 2] * inv, o[dt][4 * g + 3] * inv);
                *reinterpret_cast<uint2*>(op + d) = w;
            }
        if (hi == 0)
            a.lse[((int64_t)b * a.Hq + h) * a.S + qrow] =
                (KMASK && !(l_tot > 0.f)) ? __builtin_huge_valf() : m_run + __log2f(l_tot);
    }

    __device__ __forceinline__ void run(int b, int h, int hk, int qblk) {
        const int tid = threadIdx.x;
        lane = tid & 63;
        wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        hi = lane >> 5;
        l32 = lane & 31;
        const int q0 = qblk * kDualQB;
        qw = q0 + wave * 64;
        const uint16_t* qp = a.q.p + b * a.q.sb + h * a.q.sh;
        const uint16_t* kp = a.k.p + b * a.k.sb + hk * a.k.sh;
        const uint16_t* vp = a.v.p + b * a.v.sb + hk * a.v.sh;
        km = KMASK ? a.kmask + (int64_t)b * a.kmask_ld : nullptr;
        const int ra = qw + l32, rb = qw + 32 + l32;
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            qa[ks] = ra < a.S ? *reinterpret_cast<const bf16x8_t*>(qp + ra * a.q.ss + 16 * ks + 8 * hi)
                              : __builtin_bit_cast(bf16x8_t, u32x4_t{0u, 0u, 0u, 0u});
            qb[ks] = rb < a.S ? *reinterpret_cast<const bf16x8_t*>(qp + rb * a.q.ss + 16 * ks + 8 * hi)
                              : __builtin_bit_cast(bf16x8_t, u32x4_t{0u, 0u, 0u, 0u});
        }
        const int kv_end = min(a.S, q0 + kDualQB);
        nt = (kv_end + kKV - 1) / kKV;
        last = min(nt - 1, qw / kKV);                          // both blocks' diagonal tile (qw % 64 == 0)
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
            for (int i = 0; i < 16; ++i) { oa[dt][i] = 0.f; ob[dt][i] = 0.f; }
        ma = mb = kNegInf;
        la = lb = 0.f;
#pragma unroll
        for (int i = 0; i < kDualRing - 1; ++i)
            if (i < nt) issue(i);
        vm_wait_all();
        vm_wait_all_known();                                   // the Q fragments too (compiler-visible)
        __syncthreads();
        for (int t = 0; t < nt; t += kDualRing) tiles<0>(t);
        store(oa, ma, la, ra, b, h);
        store(ob, mb, lb, rb, b, h);
    }
};

template <bool KMASK>
__global__ __launch_bounds__(256, 1)
void attn_fwd_dual_kernel(FwdArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kDualRing * 2 * kTileB];
    const int nqb = (a.S + kDualQB - 1) / kDualQB;
    const int G = a.Hq / a.Hkv;
    const int total = nqb * a.Hq * a.B;
    const int L = xcd_logical(blockIdx.x, total);              // as attn_fwd_kernel: heaviest q blocks first
    const int per_group = G * nqb;
    const int grp = L / per_group;
    const int rem = L - grp * per_group;
    const int hk = grp % a.Hkv;
    FwdDual<KMASK> fd(a, lds);
    fd.run(grp / a.Hkv, hk * G + rem % G, hk, nqb - 1 - rem / G);
}

// SMT_ATTN_FWD_OCC: workgroups per CU of the forward (2: 256 VGPRs per wave; 1: 512)
#ifndef SMT_ATTN_FWD_OCC
#define SMT_ATTN_FWD_OCC 1
#endif
template <bool KMASK>
__global__ __launch_bounds__(64 * kFwdWaves, (SMT_ATTN_FWD_IMPL == 1 ? SMT_ATTN_FWD_OCC * 4 : 8) / kFwdWaves)
void attn_fwd_kernel(FwdArgs a) {
    // K/V ring: 2 x 32 KiB (fwd_block) or 3 x 32 KiB + 32 KiB of Q rows (the pipelined forward)
    __shared__ __attribute__((aligned(16))) uint8_t lds[SMT_ATTN_FWD_PIPE ? kFwdSlots * 2 * kTileB + kFwdQB * kRowB
                                                                          : kFRing * 2 * kFTileB];
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
    if (SMT_ATTN_FWD_IMPL == 1 && kFwdWaves == 4 && kFKV == kKV && kFRing == 2) {
        FwdPipe<KMASK> fp(a, lds);
        fp.run(grp / a.Hkv, hk * G + rem % G, hk, nqb - 1 - rem / G);
    } else if (SMT_ATTN_FWD_IMPL == 2 && kFwdWaves == 4 && kFKV == kKV && kFRing == 2) {
        FwdLean<KMASK> fl(a, lds);
#if SMT_ATTN_STAMPS
        if (L % kStampEvery == 0 && L / kStampEvery < kStampBlocks)
            fl.stamps = &g_fwd_stamps[L / kStampEvery][__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)][0][0];
#endif
        fl.run(grp / a.Hkv, hk * G + rem % G, hk, nqb - 1 - rem / G);
    } else {
        fwd_block<KMASK>(a, lds, grp / a.Hkv, hk * G + rem % G, hk, nqb - 1 - rem / G);
    }
}

// ------------------------------------------------------------------------------------------------
// Backward preprocess: delta[b, h, q] = sum_d dO * O (fp32 of the bf16 values). 16 lanes per row.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256)
void attn_delta_kernel(Tns o, Tns dout, float* __restrict__ delta, int Hq, int S, int64_t rows) {
    const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;
    const int part = threadIdx.x & 15;
    float acc = 0.f;
    if (row < rows) {
        const int64_t s = row % S;
        const int64_t bh = row / S;
        const int64_t h = bh % Hq, b = bh / Hq;
        const uint4 x = *reinterpret_cast<const uint4*>(o.p + b * o.sb + h * o.sh + s * o.ss + part * 8);
        const uint4 y = *reinterpret_cast<const uint4*>(dout.p + b * dout.sb + h * dout.sh + s * dout.ss + part * 8);
        const uint32_t xa[4] = {x.x, x.y, x.z, x.w}, ya[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            acc += __uint_as_float(xa[j] << 16) * __uint_as_float(ya[j] << 16);
            acc += __uint_as_float(xa[j] & 0xffff0000u) * __uint_as_float(ya[j] & 0xffff0000u);
        }
    }
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 16);
    if (row < rows && part == 0) delta[row] = acc;
}

// ------------------------------------------------------------------------------------------------
// dQ: a workgroup = 4 waves x 32 query rows of one (b, q head), sweeping the K/V tiles up to the
// diagonal (staged as in the forward). Per tile: S^T = K Q^T, dP^T = V dO^T, P = exp2(S*c - lse),
// dS = P (dP - delta), dQ^T += K^T dS^T.
// ------------------------------------------------------------------------------------------------
// SMT_DQ_DELTA: the dQ kernel computes delta = rowsum(dO * O) of its own rows from the dO fragments
// it holds anyway (one O read) and writes it for the dK/dV kernel, instead of a separate pass
#ifndef SMT_DQ_DELTA
#define SMT_DQ_DELTA 1
#endif

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

template <bool KMASK>
__device__ __forceinline__ void dq_block(const DqArgs& a, uint8_t* lds, int b, int h, int hk, int qb) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hi = lane >> 5, l32 = lane & 31;
    const int q0 = qb * kDqQB, qw = q0 + wave * kFwdQW;
    const uint16_t* qp = a.q.p + b * a.q.sb + h * a.q.sh;
    const uint16_t* dop = a.dout.p + b * a.dout.sb + h * a.dout.sh;
    const uint16_t* kp = a.k.p + b * a.k.sb + hk * a.k.sh;
    const uint16_t* vp = a.v.p + b * a.v.sb + hk * a.v.sh;
    const uint64_t* km = KMASK ? a.kmask + (int64_t)b * a.kmask_ld : nullptr;

    const int qrow = qw + l32;
    const bool qvalid = qrow < a.S;
    bf16x8_t qf[8], df[8];
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
    const float lse = qvalid ? a.lse[srow] : 0.f;
    float dlt;
    if (SMT_DQ_DELTA) {
        // delta of this row: the lane pair (l, l^32) holds all 128 d of dO; O read at the same places
        const uint16_t* op = a.o.p + b * a.o.sb + h * a.o.sh;
        float part = 0.f;
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            const u32x4_t ov = qvalid ? *reinterpret_cast<const u32x4_t*>(op + qrow * a.o.ss + 16 * ks + 8 * hi)
                                      : u32x4_t{0u, 0u, 0u, 0u};
            const u32x4_t dv = __builtin_bit_cast(u32x4_t, df[ks]);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                part += __uint_as_float(ov[j] << 16) * __uint_as_float(dv[j] << 16);
                part += __uint_as_float(ov[j] & 0xffff0000u) * __uint_as_float(dv[j] & 0xffff0000u);
            }
        }
        dlt = halves_sum(part);
        if (qvalid && hi == 0) a.delta[srow] = dlt;
    } else {
        dlt = qvalid ? a.delta[srow] : 0.f;
    }

    const int kv_end = min(a.S, q0 + kDqQB);
    const int nt = (kv_end + kKV - 1) / kKV;
    const __amdgpu_buffer_rsrc_t rk = uniform_rsrc(kp, (int64_t)a.S * a.k.ss * 2);
    const __amdgpu_buffer_rsrc_t rv = uniform_rsrc(vp, (int64_t)a.S * a.v.ss * 2);
    const uint32_t lds0 = lds_addr(lds);
    auto issue = [&](int t) {
        const uint32_t slot = lds0 + (uint32_t)((t & 1) * 2 * kTileB);
        constexpr int rows_w = kKV / kDqWaves;                 // rows of each operand tile one wave brings
        dma_rows(rk, a.k.ss, slot, t * kKV, t * kKV + rows_w * wave, rows_w / 4, lane);
        dma_rows(rv, a.v.ss, slot + kTileB, t * kKV, t * kKV + rows_w * wave, rows_w / 4, lane);
    };

    const TrLane tl = tr_lane(lane);
    f32x16_t dq[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) dq[dt][i] = 0.f;

    if (nt > 0) issue(0);
    vm_wait_all();
    if (SMT_ATTN_KNOWN_WAIT) vm_wait_all_known();
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
        if (t + 1 < nt) issue(t + 1);
        const uint8_t* K = lds + (t & 1) * 2 * kTileB;
        const uint8_t* V = K + kTileB;
        const int k0 = t * kKV;
        if (k0 <= qw + kFwdQW - 1) {
            f32x16_t s[2], dp[2];
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int i = 0; i < 16; ++i) { s[j][i] = 0.f; dp[j][i] = 0.f; }
#pragma unroll
            for (int ks = 0; ks < 8; ++ks)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    s[j] = mfma(row_frag(K, 32 * j + l32, 32 * ks + 16 * hi), qf[ks], s[j]);
                    dp[j] = mfma(row_frag(V, 32 * j + l32, 32 * ks + 16 * hi), df[ks], dp[j]);
                }
            const bool diag = k0 + kKV - 1 > qw;
            const uint64_t kw64 = KMASK ? km[k0 >> 6] : ~0ull;    // workgroup-uniform
            float ds[32];
#pragma unroll
            for (int i = 0; i < 32; ++i) {
                const int j = i >> 4, ii = i & 15;
                float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(s[j][ii], a.sl2, -lse));
                const int key = k0 + 32 * j + (ii & 3) + 8 * (ii >> 2) + 4 * hi;
                if (diag && key > qrow) pv = 0.f;
                if (KMASK && !key_bit(kw64, key)) pv = 0.f;
                ds[i] = pv * (dp[j][ii] - dlt);
            }
            bf16x8_t sf[4];
            pack_b_frags(*reinterpret_cast<const float(*)[16]>(&ds[0]), sf[0], sf[1]);
            pack_b_frags(*reinterpret_cast<const float(*)[16]>(&ds[16]), sf[2], sf[3]);
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int kst = 0; kst < 4; ++kst) dq[dt] = mfma(tr_frag(K, tl, 16 * kst, 32 * dt), sf[kst], dq[dt]);
        }
        vm_wait_all();
        __syncthreads();
    }

    if (qvalid) {
        uint16_t* out = a.dq + b * a.dq_sb + h * a.dq_sh + (int64_t)qrow * a.dq_ss;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d = 32 * dt + 8 * g + 4 * hi;
                uint2 w;
                w.x = pk_bf16(dq[dt][4 * g] * a.scale, dq[dt][4 * g + 1] * a.scale);
                w.y = pk_bf16(dq[dt][4 * g + 2] * a.scale, dq[dt][4 * g + 3] * a.scale);
                *reinterpret_cast<uint2*>(out + d) = w;
            }
    }
}

// dQ, lean (SMT_ATTN_DQ_IMPL 1, default): dq_block's algorithm with DkvLean's loop treatment: tiles
// in pairs (compile-time ring slot), explicit LDS addresses from two lane constants, S and dP from
// zero accumulators, p = exp2(c s - lse) and ds = p (dp - delta) in packed fp32, the causal test only
// on the wave's diagonal tile, scheduling fences that bound the fragment reads hoisted ahead.
#ifndef SMT_ATTN_DQ_IMPL
#define SMT_ATTN_DQ_IMPL 1
#endif
template <bool KMASK>
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
#if SMT_DQ_PREF
        // the K / V row fragments of k-step ks+1 are read while k-step ks's MFMAs run (a fenced
        // 2-deep register ring: without it most MFMAs waited on a read issued just before them)
        bf16x8_t f[2][4];
        f[0][0] = rowx<KI>(lds, lr, 0); f[0][1] = rowx<KH>(lds, lr, 0);
        f[0][2] = rowx<VI>(lds, lr, 0); f[0][3] = rowx<VH>(lds, lr, 0);
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            if (ks + 1 < 8) {
                bf16x8_t (&n)[4] = f[(ks + 1) & 1];
                n[0] = rowx<KI>(lds, lr, ks + 1); n[1] = rowx<KH>(lds, lr, ks + 1);
                n[2] = rowx<VI>(lds, lr, ks + 1); n[3] = rowx<VH>(lds, lr, ks + 1);
            }
            __builtin_amdgcn_sched_barrier(0);
            const bf16x8_t (&c)[4] = f[ks & 1];
            s[0] = mfma(c[0], qf[ks], ks ? s[0] : f32x16_t{});
            s[1] = mfma(c[1], qf[ks], ks ? s[1] : f32x16_t{});
            dp[0] = mfma(c[2], df[ks], ks ? dp[0] : f32x16_t{});
            dp[1] = mfma(c[3], df[ks], ks ? dp[1] : f32x16_t{});
            __builtin_amdgcn_sched_barrier(0);
        }
        const uint32_t t0 = opaque(lo_t0), t4 = opaque(lo_t4);
        bf16x8_t tf[3];                                    // dQ operands n = 0, 1 in flight during the softmax
        tf[0] = trx<KI>(lds, t0, t4, 0, 0);
        tf[1] = trx<KI>(lds, t0, t4, 1, 0);
#else
        s[0] = mfma(rowx<KI>(lds, lr, 0), qf[0], f32x16_t{});
        s[1] = mfma(rowx<KH>(lds, lr, 0), qf[0], f32x16_t{});
        dp[0] = mfma(rowx<VI>(lds, lr, 0), df[0], f32x16_t{});
        dp[1] = mfma(rowx<VH>(lds, lr, 0), df[0], f32x16_t{});
#pragma unroll
        for (int ks = 1; ks < 8; ++ks) {
            s[0] = mfma(rowx<KI>(lds, lr, ks), qf[ks], s[0]);
            s[1] = mfma(rowx<KH>(lds, lr, ks), qf[ks], s[1]);
            dp[0] = mfma(rowx<VI>(lds, lr, ks), df[ks], dp[0]);
            dp[1] = mfma(rowx<VH>(lds, lr, ks), df[ks], dp[1]);
            if (ks & 1) __builtin_amdgcn_sched_barrier(0);
        }
#endif
        float pr[32];
        const f32x2_t sl2v = {a.sl2, a.sl2}, lv = {-lse, -lse}, dv = {dlt, dlt};
#pragma unroll
        for (int i = 0; i < 32; i += 2) {
            const int j = i >> 4, ii = i & 15;
            const f32x2_t e = fma2<SMT_ATTN_PK_DQ != 0>(f32x2_t{s[j][ii], s[j][ii + 1]}, sl2v, lv);
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
            const f32x2_t r = submul2<SMT_ATTN_PK_DQ != 0>(f32x2_t{dp[j][ii], dp[j][ii + 1]}, dv, f32x2_t{pr[i], pr[i + 1]});
            pr[i] = r.x;
            pr[i + 1] = r.y;
        }
        bf16x8_t sf[4];
        pack_b_frags(*reinterpret_cast<const float(*)[16]>(&pr[0]), sf[0], sf[1]);
        pack_b_frags(*reinterpret_cast<const float(*)[16]>(&pr[16]), sf[2], sf[3]);
#if SMT_DQ_PREF
#pragma unroll
        for (int n = 0; n < 16; ++n) {                     // n = 4 dt + kst, operands two MFMAs ahead
            if (n + 2 < 16) tf[(n + 2) % 3] = trx<KI>(lds, t0, t4, (n + 2) & 3, (n + 2) >> 2);
            __builtin_amdgcn_sched_barrier(0);
            dq[n >> 2] = mfma(tf[n % 3], sf[n & 3], dq[n >> 2]);
            __builtin_amdgcn_sched_barrier(0);
        }
#else
        const uint32_t t0 = opaque(lo_t0), t4 = opaque(lo_t4);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
#pragma unroll
            for (int kst = 0; kst < 4; ++kst) dq[dt] = mfma(trx<KI>(lds, t0, t4, kst, dt), sf[kst], dq[dt]);
            __builtin_amdgcn_sched_barrier(0);
        }
#endif
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
        if (SMT_DQ_DELTA) {
            const uint16_t* op = a.o.p + b * a.o.sb + h * a.o.sh;
            float part = 0.f;
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) {
                const u32x4_t ov = qvalid ? *reinterpret_cast<const u32x4_t*>(op + qrow * a.o.ss + 16 * ks + 8 * hi)
                                          : u32x4_t{0u, 0u, 0u, 0u};
                const u32x4_t dv = __builtin_bit_cast(u32x4_t, df[ks]);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    part += __uint_as_float(ov[j] << 16) * __uint_as_float(dv[j] << 16);
                    part += __uint_as_float(ov[j] & 0xffff0000u) * __uint_as_float(dv[j] & 0xffff0000u);
                }
            }
            dlt = halves_sum(part);
            if (qvalid && hi == 0) a.delta[srow] = dlt;
        } else {
            dlt = qvalid ? a.delta[srow] : 0.f;
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
                    w.x = pk_bf16(dq[dt][4 * g] * a.scale, dq[dt][4 * g + 1] * a.scale);
                    w.y = pk_bf16(dq[dt][4 * g + 2] * a.scale, dq[dt][4 * g + 3] * a.scale);
                    *reinterpret_cast<uint2*>(out + d) = w;
                }
        }
    }
};

template <bool KMASK>
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
    if (SMT_ATTN_DQ_IMPL == 1 && kDqWaves == 4) {
        DqLean<KMASK> dl(a, lds);
        dl.run(grp / a.Hkv, hk * G + rem % G, hk, nqb - 1 - rem / G);
    } else {
        dq_block<KMASK>(a, lds, grp / a.Hkv, hk * G + rem % G, hk, nqb - 1 - rem / G);
    }
}

// ------------------------------------------------------------------------------------------------
// dK, dV: a workgroup = 8 waves x 32 keys (256 keys) of one (b, kv head); it sweeps the G query
// heads x 32-row query slices from the block's first key to S, so the G heads' contributions are
// summed in registers (no atomics). K fragments live in registers, V rows in LDS (64 KiB); the
// Q / dO slices (+ their lse / delta) arrive by LDS-DMA into a kDkvRing-deep ring (slices it+1 ..
// it+kDkvRing-1 in flight while slice it is computed; the end-of-slice wait is a counted vmcnt).
// Per slice and wave: S = Q K^T and dP = dO V^T with the row constants (-lse/c, -delta) as the
// initial accumulators, P = exp2(c S'), dS = P dP', dV^T += dO^T P, dK^T += Q^T dS.
// Measured alternatives (profiles/r01_attn_variants.jsonl): V fragments in registers instead of the
// LDS image, and one wave per SIMD with 64 keys per wave (AGPR accumulators), both ran slower: at
// 256 VGPRs the kernel already spills ~30 registers, and every extra live value adds scratch reloads
// (each one a vmcnt wait) to the loop.
// ------------------------------------------------------------------------------------------------
// SMT_DKV_KB: keys per dK/dV workgroup (256: 8 waves, one workgroup per CU; 128: 4 waves, two
// workgroups per CU, whose barriers are independent)
#ifndef SMT_DKV_KB
#define SMT_DKV_KB 256
#endif
constexpr int kKB = SMT_DKV_KB, kKW = 32, kDkvWaves = kKB / kKW, kSlice = 32;
static_assert(kKB == 128 || kKB == 256, "dK/dV key block");
constexpr int kSliceB = kSlice * kRowB;            // 8 KiB per operand slice
constexpr int kSliceBuf = 2 * kSliceB + 256;       // Q, dO, 32 lse + 32 delta
constexpr int kVImg = kKB * kRowB;                 // 64 KiB
#ifndef SMT_DKV_RING
#define SMT_DKV_RING 2
#endif
constexpr int kDkvRing = SMT_DKV_RING;             // 2; a 4-deep ring measured no faster (the loop is not DMA-bound)

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

template <bool KMASK>
__device__ __forceinline__ void dkdv_block(const DkvArgs& a, uint8_t* lds, int b, int hk, int kb) {
    const int G = a.Hq / a.Hkv;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hi = lane >> 5, l32 = lane & 31;
    const int k0 = kb * kKB, kw = k0 + wave * kKW;
    const int key = kw + l32;
    // a masked key (key mask) has P = 0 for every query: zero dK / dV
    const bool kvalid = !KMASK || (key < a.S && key_bit(a.kmask[(int64_t)b * a.kmask_ld + (key >> 6)], key));
    const uint16_t* kp = a.k.p + b * a.k.sb + hk * a.k.sh;
    const uint16_t* vp = a.v.p + b * a.v.sb + hk * a.v.sh;
    const uint32_t lds0 = lds_addr(lds);

    // V image of the block's 256 keys (each wave its own 32 rows), by DMA
    dma_rows(uniform_rsrc(vp, (int64_t)a.S * a.v.ss * 2), a.v.ss, lds0, k0, kw, kKW / 4, lane);

    // K fragments (B operand of S = Q K^T): key = kw + l32, d = 16ks + 8hi
    bf16x8_t kf[8];
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
        if (key < a.S) kf[ks] = *reinterpret_cast<const bf16x8_t*>(kp + (int64_t)key * a.k.ss + 16 * ks + 8 * hi);
        else kf[ks] = __builtin_bit_cast(bf16x8_t, u32x4_t{0u, 0u, 0u, 0u});
    }

    const int n_sl = (a.S - k0 + kSlice - 1) / kSlice;     // query slices per head, from q = k0
    const int n_it = G * n_sl;
    // Slice staging by DMA: waves 0-3 bring Q rows 8w..8w+7, waves 4-7 dO rows; waves 0 / 1 also
    // the slice's 32 lse / 32 delta values (8 lanes x 16 B).
    auto issue = [&](int it) {
        const int hh = it / n_sl, sl = n_sl - 1 - (it - hh * n_sl);
        const int h = hk * G + hh;
        const int s0 = k0 + sl * kSlice;
        const uint32_t buf = lds0 + kVImg + (uint32_t)((it % kDkvRing) * kSliceBuf);
        const bool is_q = wave < 4;
        const Tns& src = is_q ? a.q : a.dout;
        const uint16_t* base = src.p + b * src.sb + h * src.sh;
        dma_rows(uniform_rsrc(base, (int64_t)a.S * src.ss * 2), src.ss, buf + (is_q ? 0u : (uint32_t)kSliceB), s0,
                 s0 + 8 * (wave & 3), 2, lane);
        if (wave < 2 && lane < 8) {
            const float* row = (wave == 0 ? a.lse : a.delta) + ((int64_t)b * a.Hq + h) * a.S;
            dma16(uniform_rsrc(row, (int64_t)a.S * 4), __builtin_amdgcn_readfirstlane(buf + 2 * kSliceB + 128 * wave),
                  (s0 + 4 * lane) * 4);
        }
    };

    const TrLane tl = tr_lane(lane);
    f32x16_t dvt[4], dkt[4];
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) { dvt[dt][i] = 0.f; dkt[dt][i] = 0.f; }
    const float inv_sl2 = 1.f / a.sl2;

    // DMA instructions one wave issues per slice (Q or dO rows: 2; waves 0 / 1 also lse / delta)
    const int per_slice = wave < 2 ? 3 : 2;
#pragma unroll
    for (int i = 0; i < kDkvRing - 1; ++i)
        if (i < n_it) issue(i);
    vm_wait_upto(per_slice * min(kDkvRing - 2, n_it - 1));     // slice 0 (and V, K) landed
    if (SMT_ATTN_KNOWN_WAIT) vm_wait_all_known();               // K fragments: see vm_wait_all_known
    __syncthreads();
    for (int it = 0; it < n_it; ++it) {
        if (it + kDkvRing - 1 < n_it) issue(it + kDkvRing - 1);   // into the buffer slice it-1 used
        const uint8_t* Qs = lds + kVImg + (it % kDkvRing) * kSliceBuf;
        const uint8_t* Ds = Qs + kSliceB;
        const float* cst = reinterpret_cast<const float*>(Qs + 2 * kSliceB);     // lse[32], delta[32]
        const int sl = n_sl - 1 - it % n_sl;               // descending q: the group's key blocks read
        const int s0 = k0 + sl * kSlice;                   // the same slices at the same time (L2)
        if (s0 + kSlice - 1 >= kw) {                        // some q of the slice sees some key of the wave
            // row constants as initial accumulators: rows q = (i&3) + 8(i>>2) + 4hi
            f32x16_t s, dp;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const float4 lz = *reinterpret_cast<const float4*>(cst + 8 * g + 4 * hi);
                const float4 dz = *reinterpret_cast<const float4*>(cst + 32 + 8 * g + 4 * hi);
                s[4 * g] = -lz.x * inv_sl2; s[4 * g + 1] = -lz.y * inv_sl2;
                s[4 * g + 2] = -lz.z * inv_sl2; s[4 * g + 3] = -lz.w * inv_sl2;
                dp[4 * g] = -dz.x; dp[4 * g + 1] = -dz.y; dp[4 * g + 2] = -dz.z; dp[4 * g + 3] = -dz.w;
            }
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) {
                s = mfma(row_frag(Qs, l32, 32 * ks + 16 * hi), kf[ks], s);
                dp = mfma(row_frag(Ds, l32, 32 * ks + 16 * hi), row_frag(lds, wave * kKW + l32, 32 * ks + 16 * hi), dp);
            }
            const bool diag = s0 < kw + kKW - 1;
            float pr[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                float pv = __builtin_amdgcn_exp2f(s[i] * a.sl2);
                if (diag) {
                    const int q = s0 + (i & 3) + 8 * (i >> 2) + 4 * hi;
                    if (key > q) pv = 0.f;
                }
                if (KMASK && !kvalid) pv = 0.f;
                pr[i] = pv;
            }
            bf16x8_t pf[2], sf[2];
            pack_b_frags(pr, pf[0], pf[1]);
#pragma unroll
            for (int i = 0; i < 16; ++i) pr[i] *= dp[i];
            pack_b_frags(pr, sf[0], sf[1]);
#pragma unroll
            for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                for (int kq = 0; kq < 2; ++kq) {
                    dvt[dt] = mfma(tr_frag(Ds, tl, 16 * kq, 32 * dt), pf[kq], dvt[dt]);
                    dkt[dt] = mfma(tr_frag(Qs, tl, 16 * kq, 32 * dt), sf[kq], dkt[dt]);
                }
        }
        // slice it+1 must have landed; it+2 .. it+kDkvRing-1 (those issued) may stay in flight
        vm_wait_upto(per_slice * max(0, min(kDkvRing - 2, n_it - 2 - it)));
        __syncthreads();
    }

    // dK = scale * (dK^T)^T, dV = (dV^T)^T: the lane's key row, 4 consecutive d per register group
    if (key < a.S) {
        uint16_t* dkr = a.dk + b * a.dk_sb + hk * a.dk_sh + (int64_t)key * a.dk_ss;
        uint16_t* dvr = a.dv + b * a.dv_sb + hk * a.dv_sh + (int64_t)key * a.dv_ss;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d = 32 * dt + 8 * g + 4 * hi;
                uint2 w;
                w.x = pk_bf16(dkt[dt][4 * g] * a.scale, dkt[dt][4 * g + 1] * a.scale);
                w.y = pk_bf16(dkt[dt][4 * g + 2] * a.scale, dkt[dt][4 * g + 3] * a.scale);
                *reinterpret_cast<uint2*>(dkr + d) = w;
                w.x = pk_bf16(dvt[dt][4 * g], dvt[dt][4 * g + 1]);
                w.y = pk_bf16(dvt[dt][4 * g + 2], dvt[dt][4 * g + 3]);
                *reinterpret_cast<uint2*>(dvr + d) = w;
            }
    }
}

// dK / dV, lean (SMT_ATTN_DKV_IMPL 1, default): dkdv_block's algorithm with the slice loop unrolled
// by two so that the ring slot is a compile-time LDS offset (the ring now sits in front of the V
// image, within the ds_read immediate range), S and dP started from zero accumulators and the row
// constants applied afterwards in packed fp32 (p = exp2(c s - lse), ds = p (dp - delta): v_pk_fma /
// v_pk_add / v_pk_mul), the causal test only on diagonal slices. Round 2's loop spilled ~30 VGPRs
// (the per-lane addresses of the runtime slot), and each scratch reload inside the loop carried a
// vmcnt wait that also drained the slice prefetch.
#ifndef SMT_ATTN_DKV_IMPL
#define SMT_ATTN_DKV_IMPL 1
#endif
// slices in the lean loop's ring (slices it+1 .. it+R-1 in flight while slice it is computed; rings
// of 2, 3 and 4 measured 2.17, 2.21, 2.21 ms for the whole backward: profiles/r03_attn_bwd_variants.jsonl)
#ifndef SMT_DKV_LEAN_RING
#define SMT_DKV_LEAN_RING 2
#endif
constexpr int kDkvLeanRing = SMT_DKV_LEAN_RING;
static_assert(kDkvLeanRing >= 2 && kDkvLeanRing * kSliceBuf + kVImg <= 160 * 1024, "dK/dV lean ring");
template <bool KMASK>
struct DkvLean {
    const DkvArgs& a;
    uint8_t* lds;
    uint64_t* stamps = nullptr;   // SMT_ATTN_STAMPS: this wave's [kDkvStampSlices][5] record, or null
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
        const int sl = n_sl - 1 - it % n_sl;               // descending q (see dkdv_block)
        const int s0 = k0 + sl * kSlice;
        return (s0 + kSlice - 1 < kw) ? -1 : s0;
    }

    // phase 1 of a slice (ring slot SLOT): S = Q K^T and dP = dO V^T
    template <int SLOT>
    __device__ __forceinline__ void qk(f32x16_t& s, f32x16_t& dp) {
        // ring slot SLOT at [SLOT * kSliceBuf, ...): Q rows, dO rows, lse[32], delta[32]; V image after the ring
        constexpr int QI = SLOT * kSliceBuf, DI = QI + kSliceB;
        const uint32_t lr = opaque(lo_row), lv = opaque(lo_v);
        s = mfma(rowx<QI>(lds, lr, 0), kf[0], f32x16_t{});
        dp = mfma(rowx<DI>(lds, lr, 0), rowx<0>(lds, lv, 0), f32x16_t{});
#pragma unroll
        for (int ks = 1; ks < 8; ++ks) {
            s = mfma(rowx<QI>(lds, lr, ks), kf[ks], s);
            dp = mfma(rowx<DI>(lds, lr, ks), rowx<0>(lds, lv, ks), dp);
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
                const f32x2_t e = fma2<SMT_ATTN_PK_DKV != 0>(f32x2_t{s[i], s[i + 1]}, sl2v, -l2);
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
                const f32x2_t r = submul2<SMT_ATTN_PK_DKV != 0>(f32x2_t{dp[i], dp[i + 1]}, d2, f32x2_t{pr[i], pr[i + 1]});
                dsv[i] = r.x;
                dsv[i + 1] = r.y;
            }
        }
        bf16x8_t pf[2], sf[2];
        pack_b_frags(pr, pf[0], pf[1]);
        pack_b_frags(dsv, sf[0], sf[1]);
        const uint32_t t0 = opaque(lo_t0), t4 = opaque(lo_t4);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int kq = 0; kq < 2; ++kq) {
                dvt[dt] = mfma(trx<DI>(lds, t0, t4, kq, dt), pf[kq], dvt[dt]);
                dkt[dt] = mfma(trx<QI>(lds, t0, t4, kq, dt), sf[kq], dkt[dt]);
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
#if SMT_ATTN_STAMPS
        uint64_t st[5];
        st[0] = __builtin_amdgcn_s_memtime();
        st[1] = st[0];
#endif
        if (it + R - 1 < n_it) issue(it + R - 1);          // into the slot slice it-1 used
        const int s0 = slice_s0(it);
        if (s0 >= 0) {
            f32x16_t s, dp;
            qk<SLOT>(s, dp);
#if SMT_ATTN_STAMPS
            st[1] = __builtin_amdgcn_s_memtime();
#endif
            pv<SLOT>(s0, s, dp);
        }
#if SMT_ATTN_STAMPS
        st[2] = __builtin_amdgcn_s_memtime();
#endif
        // slice it+1 landed; it+2 .. it+R-1 (those issued) may stay in flight
        vm_wait_upto(per_slice * max(0, min(R - 2, n_it - 2 - it)));
#if SMT_ATTN_STAMPS
        st[3] = __builtin_amdgcn_s_memtime();
#endif
        __syncthreads();
#if SMT_ATTN_STAMPS
        st[4] = __builtin_amdgcn_s_memtime();
        if (stamps != nullptr && lane == 0 && it < kDkvStampSlices)
            for (int j = 0; j < 5; ++j) stamps[5 * it + j] = st[j];
#endif
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
                    w.x = pk_bf16(dkt[dt][4 * g] * a.scale, dkt[dt][4 * g + 1] * a.scale);
                    w.y = pk_bf16(dkt[dt][4 * g + 2] * a.scale, dkt[dt][4 * g + 3] * a.scale);
                    *reinterpret_cast<uint2*>(dkr + d) = w;
                    w.x = pk_bf16(dvt[dt][4 * g], dvt[dt][4 * g + 1]);
                    w.y = pk_bf16(dvt[dt][4 * g + 2], dvt[dt][4 * g + 3]);
                    *reinterpret_cast<uint2*>(dvr + d) = w;
                }
        }
    }
};

template <bool KMASK>
__global__ __launch_bounds__(kDkvWaves * 64, 2)
void attn_dkdv_kernel(DkvArgs a) {
    static_assert(kDkvWaves == 8 || (SMT_ATTN_DKV_IMPL == 1 && kDkvRing == 2), "4-wave dK/dV: lean loop only");
    constexpr int kLdsBytes = (SMT_ATTN_DKV_IMPL == 1 && kDkvRing == 2) ? kVImg + kDkvLeanRing * kSliceBuf
                                                                         : kVImg + kDkvRing * kSliceBuf;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
    const int nkb = (a.S + kKB - 1) / kKB;
    const int total = ((nkb + 1) / 2) * a.Hkv * a.B;
    // key blocks kb (long causal sweep) and nkb-1-kb (short) in one workgroup: equal work per
    // workgroup (1594 vs 1946 us unpaired at B16 Hq32 Hkv8 S2048)
    const PairTask t = pair_task(xcd_logical(blockIdx.x, total), nkb, 1, a.Hkv);
#pragma nounroll
    for (int i = 0; i < t.n; ++i) {
        if (i) __syncthreads();
        if (SMT_ATTN_DKV_IMPL == 1 && kDkvRing == 2) {
            DkvLean<KMASK> dl(a, lds);
#if SMT_ATTN_STAMPS
            const int L = xcd_logical(blockIdx.x, total);
            if (i == 0 && L % kStampEvery == 0 && L / kStampEvery < kStampBlocks)
                dl.stamps = &g_dkv_stamps[L / kStampEvery][__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) & 7][0][0];
#endif
            dl.run(t.b, t.hk, t.blk[1 - i]);
        } else {
            dkdv_block<KMASK>(a, lds, t.b, t.hk, t.blk[1 - i]);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// asm MFMA helpers of the one-wave-per-SIMD kernels (DqDual, DkvDual)
// ------------------------------------------------------------------------------------------------
// The 256 dK^T / dV^T accumulator registers are pinned to the accumulation registers (AGPRs) by
// issuing their MFMAs from inline asm with "+a" operands: left to itself, hipcc put the S / dP chains
// (64 registers, read by the softmax VALU) into AGPRs and spilled four accumulator tiles per slice.
// The asm MFMAs are invisible to the compiler's hazard tracking, so each group starts with an s_nop
// (VALU-written B operands), and the accumulators are read out only after a 24-wait-state pad.
__device__ __forceinline__ void mfma4_agpr(f32x16_t& c0, f32x16_t& c1, f32x16_t& c2, f32x16_t& c3, bf16x8_t a01,
                                           bf16x8_t b0, bf16x8_t b1, bf16x8_t a23, bf16x8_t b2, bf16x8_t b3) {
    asm("s_nop 2\n\t"
        "v_mfma_f32_32x32x16_bf16 %0, %4, %5, %0\n\t"
        "v_mfma_f32_32x32x16_bf16 %1, %4, %6, %1\n\t"
        "v_mfma_f32_32x32x16_bf16 %2, %7, %8, %2\n\t"
        "v_mfma_f32_32x32x16_bf16 %3, %7, %9, %3"
        : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3)
        : "v"(a01), "v"(b0), "v"(b1), "v"(a23), "v"(b2), "v"(b3));
}
// zero accumulators born in AGPRs (a zero-operand MFMA): a C++ zero would be materialised in VGPRs
// for all 256 registers at once and copied over, spilling whatever else is live at that point.
// The zero operand is a VGPR hipcc has just written (v_mov): without the pad the MFMA read it before
// the write landed and the "zero" accumulator of the first tile came out as garbage x garbage.
__device__ __forceinline__ void zero_agpr(f32x16_t& c) {
    const bf16x8_t z = __builtin_bit_cast(bf16x8_t, u32x4_t{0u, 0u, 0u, 0u});
    asm volatile("s_nop 2\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %1, 0" : "=a"(c) : "v"(z));
}
// S / dP (read by VALU) in arch VGPRs, the same way: C = 0 for the first k-step
__device__ __forceinline__ void mfma4_vgpr0(f32x16_t& c0, f32x16_t& c1, f32x16_t& c2, f32x16_t& c3, bf16x8_t a01,
                                            bf16x8_t b0, bf16x8_t b1, bf16x8_t a23, bf16x8_t b2, bf16x8_t b3) {
    asm("v_mfma_f32_32x32x16_bf16 %0, %4, %5, 0\n\t"
        "v_mfma_f32_32x32x16_bf16 %1, %4, %6, 0\n\t"
        "v_mfma_f32_32x32x16_bf16 %2, %7, %8, 0\n\t"
        "v_mfma_f32_32x32x16_bf16 %3, %7, %9, 0"
        : "=&v"(c0), "=&v"(c1), "=&v"(c2), "=&v"(c3)
        : "v"(a01), "v"(b0), "v"(b1), "v"(a23), "v"(b2), "v"(b3));
}
__device__ __forceinline__ void mfma4_vgpr(f32x16_t& c0, f32x16_t& c1, f32x16_t& c2, f32x16_t& c3, bf16x8_t a01,
                                           bf16x8_t b0, bf16x8_t b1, bf16x8_t a23, bf16x8_t b2, bf16x8_t b3) {
    asm("v_mfma_f32_32x32x16_bf16 %0, %4, %5, %0\n\t"
        "v_mfma_f32_32x32x16_bf16 %1, %4, %6, %1\n\t"
        "v_mfma_f32_32x32x16_bf16 %2, %7, %8, %2\n\t"
        "v_mfma_f32_32x32x16_bf16 %3, %7, %9, %3"
        : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3)
        : "v"(a01), "v"(b0), "v"(b1), "v"(a23), "v"(b2), "v"(b3));
}
// two-MFMA groups of the interleaved dual loop (one MFMA gap pair per softmax chunk)
__device__ __forceinline__ void mfma2_vgpr0(f32x16_t& c0, f32x16_t& c1, bf16x8_t a0, bf16x8_t b0, bf16x8_t a1,
                                            bf16x8_t b1) {
    asm("v_mfma_f32_32x32x16_bf16 %0, %2, %3, 0\n\t"
        "v_mfma_f32_32x32x16_bf16 %1, %4, %5, 0"
        : "=&v"(c0), "=&v"(c1) : "v"(a0), "v"(b0), "v"(a1), "v"(b1));
}
__device__ __forceinline__ void mfma2_vgpr(f32x16_t& c0, f32x16_t& c1, bf16x8_t a0, bf16x8_t b0, bf16x8_t a1,
                                           bf16x8_t b1) {
    asm("v_mfma_f32_32x32x16_bf16 %0, %2, %3, %0\n\t"
        "v_mfma_f32_32x32x16_bf16 %1, %4, %5, %1"
        : "+v"(c0), "+v"(c1) : "v"(a0), "v"(b0), "v"(a1), "v"(b1));
}
__device__ __forceinline__ void mfma2_agpr(f32x16_t& c0, f32x16_t& c1, bf16x8_t a0, bf16x8_t b0, bf16x8_t a1,
                                           bf16x8_t b1) {
    asm("s_nop 2\n\t"
        "v_mfma_f32_32x32x16_bf16 %0, %2, %3, %0\n\t"
        "v_mfma_f32_32x32x16_bf16 %1, %4, %5, %1"
        : "+a"(c0), "+a"(c1) : "v"(a0), "v"(b0), "v"(a1), "v"(b1));
}
__device__ __forceinline__ void mfma_drain2(f32x16_t& c0, f32x16_t& c1) {
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(c0), "+v"(c1));
}
// 24 wait states between the last asm MFMA writing these registers and any other reader (the tie
// keeps the pad between them)
__device__ __forceinline__ void mfma_drain4(f32x16_t& c0, f32x16_t& c1, f32x16_t& c2, f32x16_t& c3) {
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3));
}
__device__ __forceinline__ void mfma_drain_agpr(f32x16_t (&d)[2][4], f32x16_t (&k)[2][4]) {
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"
                 : "+a"(d[0][0]), "+a"(d[0][1]), "+a"(d[0][2]), "+a"(d[0][3]), "+a"(d[1][0]), "+a"(d[1][1]),
                   "+a"(d[1][2]), "+a"(d[1][3]), "+a"(k[0][0]), "+a"(k[0][1]), "+a"(k[0][2]), "+a"(k[0][3]),
                   "+a"(k[1][0]), "+a"(k[1][1]), "+a"(k[1][2]), "+a"(k[1][3]));
}

// ------------------------------------------------------------------------------------------------
// dQ, one wave per SIMD (runtime SMT_ATTN_DQ=2): a workgroup = 4 waves x 64 query rows (two 32-row
// blocks per wave) of one (b, q head); 64-key K / V tiles through the same LDS-DMA ring as DqLean.
// Per wave the Q and dO fragments of both blocks (128 registers) and the dQ^T accumulators of both
// (128) sit in the 256 AGPRs (the asm MFMAs read them from there); every K / V fragment read from LDS
// feeds both blocks (0.5 KiB of reads per MFMA instead of 1). Each tile is two halves of 32 keys, and
// one half's softmax runs in the MFMA gaps of the next product: S/dP(h0); S/dP(h1) || softmax(h0);
// dQ(h0) || softmax(h1); dQ(h1).
// ------------------------------------------------------------------------------------------------
constexpr int kDqDualQB = 256;

// S^T / dP^T of both query blocks for one key k-step: A = the K / V row fragment (VGPRs), B = the
// blocks' Q / dO fragments (AGPRs); accumulators in VGPRs (read by the softmax). FIRST: C = 0.
template <bool FIRST>
__device__ __forceinline__ void mfma4_qd(f32x16_t& sA, f32x16_t& sB, f32x16_t& dA, f32x16_t& dB, bf16x8_t kr,
                                         bf16x8_t vr, bf16x8_t qa, bf16x8_t qb, bf16x8_t da, bf16x8_t db) {
    if (FIRST)
        asm("s_nop 4\n\t"
            "v_mfma_f32_32x32x16_bf16 %0, %4, %6, 0\n\t"
            "v_mfma_f32_32x32x16_bf16 %1, %4, %7, 0\n\t"
            "v_mfma_f32_32x32x16_bf16 %2, %5, %8, 0\n\t"
            "v_mfma_f32_32x32x16_bf16 %3, %5, %9, 0"
            : "=&v"(sA), "=&v"(sB), "=&v"(dA), "=&v"(dB)
            : "v"(kr), "v"(vr), "a"(qa), "a"(qb), "a"(da), "a"(db));
    else
        asm("v_mfma_f32_32x32x16_bf16 %0, %4, %6, %0\n\t"
            "v_mfma_f32_32x32x16_bf16 %1, %4, %7, %1\n\t"
            "v_mfma_f32_32x32x16_bf16 %2, %5, %8, %2\n\t"
            "v_mfma_f32_32x32x16_bf16 %3, %5, %9, %3"
            : "+v"(sA), "+v"(sB), "+v"(dA), "+v"(dB)
            : "v"(kr), "v"(vr), "a"(qa), "a"(qb), "a"(da), "a"(db));
}

template <bool KMASK>
struct DqDual {
    const DqArgs& a;
    uint8_t* lds;
    bf16x8_t qf[2][8], df[2][8];
    f32x16_t dq[2][4];
    float lse[2], dlt[2];
    int qlim[2];                                           // causal limit of the tile: qrow, or INT_MAX off the diagonal
    const uint64_t* km;
    __amdgpu_buffer_rsrc_t rk, rv;
    uint32_t lds0, lo_row, lo_t0, lo_t4;
    int lane, wave, hi, l32, qw, qrow[2], nt, last;

    __device__ __forceinline__ DqDual(const DqArgs& a_, uint8_t* lds_) : a(a_), lds(lds_) {}

    __device__ __forceinline__ void issue(int t) {            // K(t), V(t) into slot t & 1: 16 rows per wave
        const uint32_t slot = lds0 + (uint32_t)((t & 1) * 2 * kTileB);
        dma_rows(rk, a.k.ss, slot, t * kKV, t * kKV + 16 * wave, 4, lane);
        dma_rows(rv, a.v.ss, slot + kTileB, t * kKV, t * kKV + 16 * wave, 4, lane);
    }

    // one eighth of the softmax of both query blocks over one 32-key half (chunk C, compile-time):
    // C 0-3 the probabilities of registers 4C..4C+3 (in place of S), C 4-7 dS (in place of dP), C 7 packs
    template <bool DIAG, int C>
    __device__ __forceinline__ void soft_chunk(int k0h, f32x16_t (&s)[2], f32x16_t (&dp)[2], bf16x8_t (&sf)[2][2]) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if constexpr (C < 4) {
                const f32x2_t sl2v = {a.sl2, a.sl2}, lv = {-lse[j], -lse[j]};
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int i = 4 * C + 2 * h;
                    const f32x2_t e = __builtin_elementwise_fma(f32x2_t{s[j][i], s[j][i + 1]}, sl2v, lv);
                    float p0 = __builtin_amdgcn_exp2f(e.x), p1 = __builtin_amdgcn_exp2f(e.y);
                    const int key = k0h + (i & 3) + 8 * (i >> 2) + 4 * hi;
                    // branch-free causal mask (qlim = INT_MAX off the diagonal): one code path for every
                    // tile, so the accumulators never take a second register assignment
                    p0 = key > qlim[j] ? 0.f : p0;
                    p1 = key + 1 > qlim[j] ? 0.f : p1;
                    if (KMASK) {
                        const uint64_t w = km[key >> 6];
                        p0 = key_bit(w, key) ? p0 : 0.f;
                        p1 = key_bit(w, key + 1) ? p1 : 0.f;
                    }
                    s[j][i] = p0;
                    s[j][i + 1] = p1;
                }
            } else {
                const f32x2_t dv = {dlt[j], dlt[j]};
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int i = 4 * (C - 4) + 2 * h;
                    const f32x2_t r = (f32x2_t{dp[j][i], dp[j][i + 1]} - dv) * f32x2_t{s[j][i], s[j][i + 1]};
                    dp[j][i] = r.x;
                    dp[j][i + 1] = r.y;
                }
                if constexpr (C == 7) {
                    float ds[16];
#pragma unroll
                    for (int i = 0; i < 16; ++i) ds[i] = dp[j][i];
                    pack_b_frags(ds, sf[j][0], sf[j][1]);
                }
            }
        }
    }
    template <bool DIAG, int C>
    __device__ __forceinline__ void soft_chunks_from(int c, int k0h, f32x16_t (&s)[2], f32x16_t (&dp)[2],
                                                     bf16x8_t (&sf)[2][2]) {
        if (c == C) soft_chunk<DIAG, C>(k0h, s, dp, sf);
        if constexpr (C + 1 < 8) soft_chunks_from<DIAG, C + 1>(c, k0h, s, dp, sf);
    }

    // S^T, dP^T of key half H into s / dp; with SOFT, the other half's softmax chunk per k-step
    template <int SLOT, int H, bool SOFT, bool DIAG>
    __device__ __forceinline__ void qk(f32x16_t (&s)[2], f32x16_t (&dp)[2], int k0o, f32x16_t (&so)[2],
                                       f32x16_t (&dpo)[2], bf16x8_t (&sfo)[2][2]) {
        constexpr int KI = SLOT * 2 * kTileB + H * 32 * kRowB, VI = KI + kTileB;
        const uint32_t lr = opaque(lo_row);
        bf16x8_t f[2][2];
        f[0][0] = rowx<KI>(lds, lr, 0);
        f[0][1] = rowx<VI>(lds, lr, 0);
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            if (ks < 7) {
                f[(ks + 1) & 1][0] = rowx<KI>(lds, lr, ks + 1);
                f[(ks + 1) & 1][1] = rowx<VI>(lds, lr, ks + 1);
            }
            if (ks == 0) mfma4_qd<true>(s[0], s[1], dp[0], dp[1], f[0][0], f[0][1], qf[0][0], qf[1][0], df[0][0], df[1][0]);
            else mfma4_qd<false>(s[0], s[1], dp[0], dp[1], f[ks & 1][0], f[ks & 1][1], qf[0][ks], qf[1][ks], df[0][ks],
                                 df[1][ks]);
            if (SOFT) {
                if (ks == 0) { mfma_drain2(so[0], so[1]); mfma_drain2(dpo[0], dpo[1]); }
                soft_chunks_from<DIAG, 0>(ks, k0o, so, dpo, sfo);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }

    // dQ^T += K^T dS^T over key half H; with SOFT, the other half's softmax chunk per step
    template <int SLOT, int H, bool SOFT, bool DIAG>
    __device__ __forceinline__ void dqp(const bf16x8_t (&sf)[2][2], int k0o, f32x16_t (&so)[2], f32x16_t (&dpo)[2],
                                        bf16x8_t (&sfo)[2][2]) {
        constexpr int KI = SLOT * 2 * kTileB;
        const uint32_t t0 = opaque(lo_t0), t4 = opaque(lo_t4);
        bf16x8_t tf[2];
        tf[0] = trx<KI>(lds, t0, t4, 2 * H, 0);
#pragma unroll
        for (int n = 0; n < 8; ++n) {
            const int dt = n >> 1, kst = n & 1;
            if (n < 7) tf[(n + 1) & 1] = trx<KI>(lds, t0, t4, 2 * H + ((n + 1) & 1), (n + 1) >> 1);
            mfma2_agpr(dq[0][dt], dq[1][dt], tf[n & 1], sf[0][kst], tf[n & 1], sf[1][kst]);
            if (SOFT) {
                if (n == 0) { mfma_drain2(so[0], so[1]); mfma_drain2(dpo[0], dpo[1]); }
                soft_chunks_from<DIAG, 0>(n, k0o, so, dpo, sfo);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }

    template <int SLOT, bool DIAG>
    __device__ __forceinline__ void compute(int t) {
        const int k0 = t * kKV;
        f32x16_t s0[2], dp0[2], s1[2], dp1[2];
        bf16x8_t sf0[2][2], sf1[2][2];
        qk<SLOT, 0, false, DIAG>(s0, dp0, 0, s1, dp1, sf1);              // (no softmax beside it)
        qk<SLOT, 1, true, DIAG>(s1, dp1, k0, s0, dp0, sf0);              // || softmax of half 0
        dqp<SLOT, 0, true, DIAG>(sf0, k0 + 32, s1, dp1, sf1);            // || softmax of half 1
        dqp<SLOT, 1, false, DIAG>(sf1, 0, s1, dp1, sf1);
    }

    template <int SLOT>
    __device__ __forceinline__ void tile(int t) {
        if (t + 1 < nt) issue(t + 1);
        if (t <= last) {
            qlim[0] = t == last ? qrow[0] : 0x7fffffff;
            qlim[1] = t == last ? qrow[1] : 0x7fffffff;
            compute<SLOT, false>(t);
        }
        vm_wait_all();
        __syncthreads();
    }

    __device__ __forceinline__ void run(int b, int h, int hk, int qb) {
        const int tid = threadIdx.x;
        lane = tid & 63;
        wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        hi = lane >> 5;
        l32 = lane & 31;
        const int q0 = qb * kDqDualQB;
        qw = q0 + wave * 64;
        const uint16_t* qp = a.q.p + b * a.q.sb + h * a.q.sh;
        const uint16_t* dop = a.dout.p + b * a.dout.sb + h * a.dout.sh;
        const uint16_t* op = a.o.p + b * a.o.sb + h * a.o.sh;
        const uint16_t* kp = a.k.p + b * a.k.sb + hk * a.k.sh;
        const uint16_t* vp = a.v.p + b * a.v.sb + hk * a.v.sh;
        km = KMASK ? a.kmask + (int64_t)b * a.kmask_ld : nullptr;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            qrow[j] = qw + 32 * j + l32;
            const bool qvalid = qrow[j] < a.S;
            // Q / dO fragments straight into AGPRs (a load the compiler would otherwise keep in VGPRs and
            // copy into AGPRs every tile). Rows past S read row S-1: their S^T / dS^T columns only reach
            // their own dQ^T column, which is never stored.
            const int64_t rr = qvalid ? qrow[j] : a.S - 1;
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) {
                const uint16_t* qa = qp + rr * a.q.ss + 16 * ks + 8 * hi;
                const uint16_t* da = dop + rr * a.dout.ss + 16 * ks + 8 * hi;
                asm volatile("global_load_dwordx4 %0, %1, off" : "=a"(qf[j][ks]) : "v"(qa) : "memory");
                asm volatile("global_load_dwordx4 %0, %1, off" : "=a"(df[j][ks]) : "v"(da) : "memory");
            }
            float part = 0.f;
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) {
                // delta = rowsum(dO * O) of this row (SMT_DQ_DELTA, as DqLean), from a second (VGPR) read of dO
                const u32x4_t ov = qvalid ? *reinterpret_cast<const u32x4_t*>(op + qrow[j] * a.o.ss + 16 * ks + 8 * hi)
                                          : u32x4_t{0u, 0u, 0u, 0u};
                const u32x4_t dv = qvalid ? *reinterpret_cast<const u32x4_t*>(dop + qrow[j] * a.dout.ss + 16 * ks + 8 * hi)
                                          : u32x4_t{0u, 0u, 0u, 0u};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    part += __uint_as_float(ov[e] << 16) * __uint_as_float(dv[e] << 16);
                    part += __uint_as_float(ov[e] & 0xffff0000u) * __uint_as_float(dv[e] & 0xffff0000u);
                }
            }
            const int64_t srow = ((int64_t)b * a.Hq + h) * a.S + (qvalid ? qrow[j] : 0);
            lse[j] = qvalid ? a.lse[srow] : 0.f;
            dlt[j] = halves_sum(part);
            if (qvalid && hi == 0) a.delta[srow] = dlt[j];
        }
        const int kv_end = min(a.S, q0 + kDqDualQB);
        nt = (kv_end + kKV - 1) / kKV;
        last = min(nt - 1, qw / kKV);                      // both blocks' diagonal: tile qw / 64
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
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) zero_agpr(dq[j][dt]);
        if (nt > 0) issue(0);
        vm_wait_all();
        vm_wait_all_known();
        __syncthreads();
        for (int t = 0; t < nt; t += 2) {
            tile<0>(t);
            if (t + 1 < nt) tile<1>(t + 1);
        }
        f32x16_t (&dqa)[2][4] = dq;
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"
                     : "+a"(dqa[0][0]), "+a"(dqa[0][1]), "+a"(dqa[0][2]), "+a"(dqa[0][3]), "+a"(dqa[1][0]),
                       "+a"(dqa[1][1]), "+a"(dqa[1][2]), "+a"(dqa[1][3]));
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (qrow[j] < a.S) {
                uint16_t* out = a.dq + b * a.dq_sb + h * a.dq_sh + (int64_t)qrow[j] * a.dq_ss;
#pragma unroll
                for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const int d = 32 * dt + 8 * g + 4 * hi;
                        uint2 w;
                        w.x = pk_bf16(dq[j][dt][4 * g] * a.scale, dq[j][dt][4 * g + 1] * a.scale);
                        w.y = pk_bf16(dq[j][dt][4 * g + 2] * a.scale, dq[j][dt][4 * g + 3] * a.scale);
                        *reinterpret_cast<uint2*>(out + d) = w;
                    }
            }
        }
    }
};

template <bool KMASK>
__global__ __launch_bounds__(256, 1)
void attn_dq_dual_kernel(DqArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * 2 * kTileB];      // 64 KiB
    const int nqb = (a.S + kDqDualQB - 1) / kDqDualQB;
    const int G = a.Hq / a.Hkv;
    const int total = nqb * a.Hq * a.B;
    const int L = xcd_logical(blockIdx.x, total);
    const int per_group = G * nqb;
    const int grp = L / per_group;
    const int rem = L - grp * per_group;
    const int hk = grp % a.Hkv;
    DqDual<KMASK> d(a, lds);
    d.run(grp / a.Hkv, hk * G + rem % G, hk, nqb - 1 - rem / G);
}

int dq_impl() {
    static const int v = [] { const char* e = getenv("SMT_ATTN_DQ"); return (e && atoi(e) == 2) ? 2 : 1; }();
    return v;
}

// ------------------------------------------------------------------------------------------------
// Forward, one wave per SIMD, software-pipelined across key tiles (runtime SMT_ATTN_FWD=4; no key
// mask). A workgroup = 4 waves x 64 query rows (row blocks 0 / 1 of 32 per wave) of one (b, q head);
// Q fragments (both blocks) and the O^T accumulators live in the 256 AGPRs (asm loads / asm MFMAs);
// 64-key K / V tiles in a 4-slot LDS-DMA ring, tile k+2 in flight while k and k-1 are read. Each key
// tile is two 32-key halves, and every MFMA phase of a step carries one half of a softmax, so the
// VALU work is spread over all MFMA gaps (at most ~5 single-issue instructions hide per gap):
//   P1: S(h0, k)           || softmax b-part of (h1, k-1)   (exponentials, sums, P packing)
//   P2: O += V(h0) P(h0, k-1) || softmax a-part of (h0, k)   (causal mask, row max, exponentials)
//   P3: S(h1, k)           || softmax b-part of (h0, k)
//   P4: O += V(h1) P(h1, k-1) || softmax a-part of (h1, k)
// There is no O rescale in the loop (hipcc cannot keep 128 AGPR accumulators in place through a
// read-modify-write: it spilled). Instead each row's exponent base is its first half-tile's max and
// stays there: P = 2^(s - m) may exceed 1, which bf16 and fp32 carry exactly as far as 2^127 (a power
// of two shifts no rounding). Should a later score exceed the base by more than kPwThr (2^64 headroom
// left), the workgroup runs the tiles a second time from the rows' true maxima, tracked in pass one.
// ------------------------------------------------------------------------------------------------
constexpr int kPwQB = 256, kPwRing = 4;
constexpr float kPwThr = 64.f;

// S^T of both row blocks for one k-step of a 32-key half: A = the K row fragment, B = the blocks'
// Q fragments (AGPRs); accumulators in VGPRs (read by the softmax). FIRST: C = 0.
template <bool FIRST>
__device__ __forceinline__ void mfma2_qs(f32x16_t& sA, f32x16_t& sB, bf16x8_t kr, bf16x8_t qa, bf16x8_t qb) {
    if (FIRST)
        asm("s_nop 1\n\t"
            "v_mfma_f32_32x32x16_bf16 %0, %2, %3, 0\n\t"
            "v_mfma_f32_32x32x16_bf16 %1, %2, %4, 0"
            : "=&v"(sA), "=&v"(sB) : "v"(kr), "a"(qa), "a"(qb));
    else
        asm("v_mfma_f32_32x32x16_bf16 %0, %2, %3, %0\n\t"
            "v_mfma_f32_32x32x16_bf16 %1, %2, %4, %1"
            : "+v"(sA), "+v"(sB) : "v"(kr), "a"(qa), "a"(qb));
}

// mfma2_agpr without the leading pad: the forward's P operands are packed a whole phase earlier and
// its V^T fragments come from LDS, so no VALU write is within reach of these MFMAs
__device__ __forceinline__ void mfma2_agpr_np(f32x16_t& c0, f32x16_t& c1, bf16x8_t a0, bf16x8_t b0, bf16x8_t a1,
                                              bf16x8_t b1) {
    asm("v_mfma_f32_32x32x16_bf16 %0, %2, %3, %0\n\t"
        "v_mfma_f32_32x32x16_bf16 %1, %4, %5, %1"
        : "+a"(c0), "+a"(c1) : "v"(a0), "v"(b0), "v"(a1), "v"(b1));
}

struct FwdPw {
    const FwdArgs& a;
    uint8_t* lds;
    bf16x8_t qf[2][8];                 // [block][k-step], AGPRs
    f32x16_t o[2][4];                  // O^T [block][32-feature tile], AGPRs
    f32x16_t s[2][2];                  // [half][block]: scores, then probabilities in place
    bf16x8_t pf[2][2][2];              // [half][block][16-key step]: P^T packed as the PV B operand
    float m[2], l[2], mx[2], mt[2], ps[2], mq[2][3];
    int bad;                           // a score beyond the exponent base's headroom (second pass)
    __amdgpu_buffer_rsrc_t rk, rv;
    uint32_t lds0, lo_row, lo_t0, lo_t4;
    int lane, wave, hi, l32, qw, qrow[2], nt, last;

    __device__ __forceinline__ FwdPw(const FwdArgs& a_, uint8_t* lds_) : a(a_), lds(lds_) {}

    __device__ __forceinline__ uint32_t slot_off(int t) const { return (uint32_t)((t & (kPwRing - 1)) * 2 * kTileB); }

    __device__ __forceinline__ void issue(int t) {            // K(t), V(t): 16 rows of each per wave
        const uint32_t slot = lds0 + slot_off(t);
        dma_rows(rk, a.k.ss, slot, t * kKV, t * kKV + 16 * wave, 4, lane);
        dma_rows(rv, a.v.ss, slot + kTileB, t * kKV, t * kKV + 16 * wave, 4, lane);
    }

    // one sixteenth of the softmax of half H (both blocks), chunk C compile-time; keys k0h .. k0h+31
    // The softmax of one half (both blocks) in 16 chunks, each beside one MFMA pair. With one wave per
    // SIMD nothing else fills the gap while a VALU result is awaited, so a chunk holds independent
    // operations only: the max trees are split into independent triples, and the 8 groups of 4
    // scores (g = 4j + i/4) run as a pipeline (chunk 5 + n: fma of group n, exp of group n-1, sums
    // of group n-2).
    template <int G>
    __device__ __forceinline__ void grp_fma(int H) {
        if constexpr (G >= 0 && G < 8) {
            constexpr int j = G / 4, i0 = 4 * (G % 4);
            f32x16_t& x = s[H][j];
            const float nm = -m[j];
#pragma unroll
            for (int i = i0; i < i0 + 4; ++i) x[i] = __builtin_fmaf(x[i], a.sl2, nm);
        }
    }
    template <int G>
    __device__ __forceinline__ void grp_exp(int H) {
        if constexpr (G >= 0 && G < 8) {
            constexpr int j = G / 4, i0 = 4 * (G % 4);
            f32x16_t& x = s[H][j];
#pragma unroll
            for (int i = i0; i < i0 + 4; ++i) x[i] = __builtin_amdgcn_exp2f(x[i]);
        }
    }
    template <int G>
    __device__ __forceinline__ void grp_sum(int H) {
        if constexpr (G >= 0 && G < 8) {
            constexpr int j = G / 4, i0 = 4 * (G % 4);
            const f32x16_t& x = s[H][j];
            const float q = (x[i0] + x[i0 + 1]) + (x[i0 + 2] + x[i0 + 3]);
            ps[j] = i0 == 0 ? q : ps[j] + q;
        }
    }
    template <bool DIAG, int H, int C>
    __device__ __forceinline__ void chunk(int k0h) {
        if constexpr (C == 0 || C == 2) {                      // causal mask (diagonal tile) + 3 triples
            constexpr int j = C / 2;
            f32x16_t& x = s[H][j];
            if (DIAG) {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const int key = k0h + (i & 3) + 8 * (i >> 2) + 4 * hi;
                    x[i] = key > qrow[j] ? kNegInf : x[i];
                }
            }
            mq[j][0] = max3f(x[0], x[1], x[2]);
            mq[j][1] = max3f(x[3], x[4], x[5]);
            mq[j][2] = max3f(x[6], x[7], x[8]);
        } else if constexpr (C == 1 || C == 3) {               // 2 more triples, then the tree
            constexpr int j = C / 2;
            const f32x16_t& x = s[H][j];
            const float t3 = max3f(x[9], x[10], x[11]);
            const float t4 = max3f(x[12], x[13], x[14]);
            const float u = max3f(mq[j][0], mq[j][1], mq[j][2]);
            mt[j] = max3f(u, max3f(t3, t4, x[15]), u);
        } else if constexpr (C == 4) {                         // row max over the half; the base fixed
            float mtile[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) mtile[j] = other_half_max(mt[j]) * a.sl2;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                mx[j] = fmaxf(mx[j], mtile[j]);
                const bool first = m[j] == kNegInf;            // the row's first half-tile sets the base
                bad |= (int)(!first && mtile[j] > m[j] + kPwThr);
                m[j] = first ? mtile[j] : m[j];
            }
        } else if constexpr (C >= 5 && C <= 14) {              // the group pipeline
            constexpr int n = C - 5;
            grp_fma<n>(H);
            grp_exp<n - 1>(H);
            grp_sum<n - 2>(H);
            if constexpr (n == 5) l[0] += ps[0];               // block 0's groups 0-3 summed at n = 5
            if constexpr (n == 6) {
                float p[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) p[i] = s[H][0][i];
                pack_b_frags(p, pf[H][0][0], pf[H][0][1]);
            }
            if constexpr (n == 9) l[1] += ps[1];
        } else {                                               // C == 15: block 1 packed
            float p[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) p[i] = s[H][1][i];
            pack_b_frags(p, pf[H][1][0], pf[H][1][1]);
        }
    }
    template <bool DIAG, int H, int C>
    __device__ __forceinline__ void chunks_from(int c, int k0h) {
#ifdef SMT_PW_DIAG_NO_SOFTMAX
        return;                                            // diagnostic build: the loop skeleton alone
#endif
        if (c == C) chunk<DIAG, H, C>(k0h);
        if constexpr (C + 1 < 16) chunks_from<DIAG, H, C + 1>(c, k0h);
    }

    // S(H) over the K tile at slot offset sk, with softmax chunks C0 .. C0+7 of half SH beside it
    template <int H, bool SM, bool DIAG, int SH, int C0>
    __device__ __forceinline__ void qk(uint32_t sk, int k0s) {
        constexpr int KI = H * 32 * kRowB;
        const uint32_t lr = opaque(lo_row) + sk;
        bf16x8_t f[3];                                     // K fragments two k-steps ahead (fenced)
        f[0] = rowx<KI>(lds, lr, 0);
        f[1] = rowx<KI>(lds, lr, 1);
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
#ifndef SMT_PW_DIAG_NO_LDS
            if (ks + 2 < 8) f[(ks + 2) % 3] = rowx<KI>(lds, lr, ks + 2);
#endif
            __builtin_amdgcn_sched_barrier(0);
            if (ks == 0) mfma2_qs<true>(s[H][0], s[H][1], f[0], qf[0][0], qf[1][0]);
            else mfma2_qs<false>(s[H][0], s[H][1], f[ks % 3], qf[0][ks], qf[1][ks]);
            if (SM) chunks_from<DIAG, SH, C0>(C0 + ks, k0s);
            __builtin_amdgcn_sched_barrier(0);
        }
    }

    // O^T += V^T(H) P^T(H) over the V tile at slot offset sv, with softmax chunks beside it. DRAIN:
    // the softmax half's scores were just written by MFMAs (24 wait states before its first read)
    template <int H, bool SM, bool DIAG, int SH, int C0, bool DRAIN>
    __device__ __forceinline__ void pv(uint32_t sv, int k0s) {
        constexpr int VI = kTileB;
        const uint32_t t0 = opaque(lo_t0) + sv, t4 = opaque(lo_t4) + sv;
        bf16x8_t tf[3];                                    // V^T fragments two steps ahead (fenced)
        tf[0] = trx<VI>(lds, t0, t4, 2 * H, 0);
        tf[1] = trx<VI>(lds, t0, t4, 2 * H + 1, 0);
#pragma unroll
        for (int n = 0; n < 8; ++n) {
            const int dt = n >> 1, kst = n & 1;
#ifndef SMT_PW_DIAG_NO_LDS
            if (n + 2 < 8) tf[(n + 2) % 3] = trx<VI>(lds, t0, t4, 2 * H + ((n + 2) & 1), (n + 2) >> 1);
#endif
            __builtin_amdgcn_sched_barrier(0);
            mfma2_agpr_np(o[0][dt], o[1][dt], tf[n % 3], pf[H][0][kst], tf[n % 3], pf[H][1][kst]);
            if (SM) {
                if (DRAIN && n == 0) mfma_drain2(s[SH][0], s[SH][1]);
                chunks_from<DIAG, SH, C0>(C0 + n, k0s);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    // the softmax chunks alone (no product beside them: the first and the drain steps)
    template <bool DIAG, int SH, int C0, bool DRAIN>
    __device__ __forceinline__ void sm_only(int k0s) {
        if (DRAIN) mfma_drain2(s[SH][0], s[SH][1]);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            chunks_from<DIAG, SH, C0>(C0 + c, k0s);
            __builtin_amdgcn_sched_barrier(0);
        }
    }

    // step k: S(k) and the softmax of tile k's halves; O += V(k-1) P(k-1). QK: tile k exists for this
    // wave (k <= last); PV: k >= 1; DIAG: k == last
    template <bool QK, bool PV, bool DIAG>
    __device__ __forceinline__ void step(int k) {
        const uint32_t sk = slot_off(k), sv = slot_off(k - 1);
        const int k0 = k * kKV, kp = (k - 1) * kKV;
        // P1: S(h0, k) || b-part of the previous tile's h1 softmax
        if (QK && PV) qk<0, true, false, 1, 8>(sk, kp + 32);
        else if (QK) qk<0, false, false, 1, 8>(sk, 0);
        else if (PV) sm_only<false, 1, 8, false>(kp + 32);
        // P2: O += V(h0, k-1) P(h0, k-1) || a-part of (h0, k)
        if (PV && QK) pv<0, true, DIAG, 0, 0, true>(sv, k0);
        else if (PV) pv<0, false, false, 0, 0, false>(sv, 0);
        else sm_only<DIAG, 0, 0, true>(k0);
        // P3: S(h1, k) || b-part of (h0, k)
        if (QK) qk<1, true, DIAG, 0, 8>(sk, k0);
        // P4: O += V(h1, k-1) P(h1, k-1) || a-part of (h1, k)
        if (PV && QK) pv<1, true, DIAG, 1, 0, true>(sv, k0 + 32);
        else if (PV) pv<1, false, false, 1, 0, false>(sv, 0);
        else if (QK) sm_only<DIAG, 1, 0, true>(k0 + 32);
    }

    // ring bookkeeping of step k (every wave, the same count of barriers): tile k+2 into the slot
    // tile k-2 used, then tile k+1 landed, barrier
    __device__ __forceinline__ void ring_pre(int k) {
#ifndef SMT_PW_DIAG_NO_DMA
        if (k + 2 < nt) issue(k + 2);
#endif
    }
    __device__ __forceinline__ void ring_post(int k) {
#ifndef SMT_PW_DIAG_NO_DMA
        if (k + 2 < nt) vm_wait_upto(8);
        else vm_wait_all();
#endif
#ifndef SMT_PW_DIAG_NO_BARRIER
        __syncthreads();
#endif
    }

    template <int j>
    __device__ __forceinline__ void store(int b, int h) {
        const float l_tot = halves_sum(l[j]);
        if (qrow[j] >= a.S) return;
        const float inv = 1.f / l_tot;
        uint16_t* op = a.o + b * a.o_sb + h * a.o_sh + (int64_t)qrow[j] * a.o_ss;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int d = 32 * dt + 8 * g + 4 * hi;
                uint2 w;
                w.x = pk_bf16(o[j][dt][4 * g] * inv, o[j][dt][4 * g + 1] * inv);
                w.y = pk_bf16(o[j][dt][4 * g + 2] * inv, o[j][dt][4 * g + 3] * inv);
                *reinterpret_cast<uint2*>(op + d) = w;
            }
        if (hi == 0) a.lse[((int64_t)b * a.Hq + h) * a.S + qrow[j]] = m[j] + __log2f(l_tot);
    }

    __device__ __forceinline__ void run(int b, int h, int hk, int qb) {
        const int tid = threadIdx.x;
        lane = tid & 63;
        wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        hi = lane >> 5;
        l32 = lane & 31;
        const int q0 = qb * kPwQB;
        qw = q0 + wave * 64;
        const uint16_t* qp = a.q.p + b * a.q.sb + h * a.q.sh;
        const uint16_t* kp = a.k.p + b * a.k.sb + hk * a.k.sh;
        const uint16_t* vp = a.v.p + b * a.v.sb + hk * a.v.sh;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            qrow[j] = qw + 32 * j + l32;
            // rows past S read row S-1: their scores only reach their own O column, never stored
            const int64_t rr = qrow[j] < a.S ? qrow[j] : a.S - 1;
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) {
                const uint16_t* qa = qp + rr * a.q.ss + 16 * ks + 8 * hi;
                asm volatile("global_load_dwordx4 %0, %1, off" : "=a"(qf[j][ks]) : "v"(qa) : "memory");
            }
            m[j] = kNegInf;
            mx[j] = kNegInf;
        }
        const int kv_end = min(a.S, q0 + kPwQB);
        nt = (kv_end + kKV - 1) / kKV;
        last = min(nt - 1, qw / kKV);                      // both blocks' diagonal tile (qw % 64 == 0)
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
        for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            l[j] = 0.f;
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) zero_agpr(o[j][dt]);
        }
        bad = 0;
        issue(0);
        if (nt > 1) issue(1);
        vm_wait_all();
        __syncthreads();
        // this wave's steps 0 .. last+1; the workgroup's ring runs steps 0 .. nt (the last wave's)
        int k = 0;
        ring_pre(0);
        if (last == 0) step<true, false, true>(0);
        else step<true, false, false>(0);
        ring_post(0);
        for (k = 1; k < last; ++k) {
            ring_pre(k);
            step<true, true, false>(k);
            ring_post(k);
        }
        if (last > 0) {
            ring_pre(last);
            step<true, true, true>(last);
            ring_post(last);
        }
        k = last + 1;
        ring_pre(k);
        step<false, true, false>(k);
        if (k < nt) ring_post(k);
        for (++k; k <= nt; ++k) {                          // ring duty only
            ring_pre(k);
            if (k < nt) ring_post(k);
        }
        // every wave's steps are done (the last barrier of the ring, or this one) before a second pass
        // re-fills the ring from tile 0
        if (!__syncthreads_or(bad)) break;
        m[0] = mx[0];
        m[1] = mx[1];
        }
        mfma_drain_agpr(o, o);
        store<0>(b, h);
        store<1>(b, h);
    }
};

__global__ __launch_bounds__(256, 1)
void attn_fwd_pw_kernel(FwdArgs a) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kPwRing * 2 * kTileB];         // 128 KiB
    const int nqb = (a.S + kPwQB - 1) / kPwQB;
    const int G = a.Hq / a.Hkv;
    const int total = nqb * a.Hq * a.B;
    const int L = xcd_logical(blockIdx.x, total);
    const int per_group = G * nqb;
    const int grp = L / per_group;
    const int rem = L - grp * per_group;
    const int hk = grp % a.Hkv;
    FwdPw f(a, lds);
    f.run(grp / a.Hkv, hk * G + rem % G, hk, nqb - 1 - rem / G);
}

// SMT_ATTN_FWD (runtime): 4 = attn_fwd_pw_kernel for unmasked batches; otherwise attn_fwd_kernel
int fwd_impl() {
    static const int v = [] { const char* e = getenv("SMT_ATTN_FWD"); return (e && atoi(e) == 4) ? 4 : 0; }();
    return v;
}

// ------------------------------------------------------------------------------------------------
// dK / dV, one wave per SIMD (runtime SMT_ATTN_DKV=2): the same 256-key block per workgroup, as 4
// waves x 64 keys. Each wave holds dK^T and dV^T of its two 32-key blocks (4 x 64 fp32 accumulators:
// 256 registers, MFMA-only, so they can live in the accumulation registers of the 512-register
// file) and the K fragments of both blocks. Every Q / dO fragment read from LDS -- rows for S / dP,
// transposed for dV / dK -- feeds the MFMAs of both key blocks, so a slice costs half the LDS-read
// bytes per MFMA of DkvLean (whose 8 waves x 32 keys read every fragment once per 32 keys), and one
// wave per SIMD has no partner wave to wait for at the barrier (MI355X_MICROARCH "Two waves per
// SIMD"; cdna_hip_programming "Attention backward": 4 waves x 64 keys, 256 accumulator registers).
// ------------------------------------------------------------------------------------------------
constexpr int kDualKW = 64, kDualKWaves = kKB / kDualKW;
#ifndef SMT_DKV_DUAL_ATTR
#define SMT_DKV_DUAL_ATTR
#endif
// SMT_DKV_DUAL_FENCE: a scheduling fence after every k-step (1) or every second one (0)
#ifndef SMT_DKV_DUAL_FENCE
#define SMT_DKV_DUAL_FENCE 1
#endif
#ifndef SMT_DKV_DUAL_RING
#define SMT_DKV_DUAL_RING 2
#endif
constexpr int kDkvDualRing = SMT_DKV_DUAL_RING;
// LDS: the slice ring, the V image of the 256 keys, and the K rows of every wave's second key block
// (its first block's K fragments stay in registers: 512 registers hold 256 accumulators + one block)
constexpr int kKbImg = kDualKWaves * kKW * kRowB;        // 32 KiB
static_assert(kDkvDualRing >= 2 && kDkvDualRing * kSliceBuf + kVImg + kKbImg <= 160 * 1024, "dK/dV dual ring");

// V (SMT_ATTN_DKV 2 / 3): 2 = both key blocks' S / dP, then both softmaxes, then the dV / dK products
// sharing every fragment read; 3 = the softmax of one block placed in the MFMA gaps of the other's
// products (S1/dP1 beside softmax 0, dV0/dK0 beside softmax 1): one wave per SIMD has no partner wave
// to hide the softmax behind, so the block pairs overlap inside the wave, at the price of reading the
// Q / dO fragments once per block (1.4 instead of 0.9 KiB of LDS reads per MFMA)
template <bool KMASK, int V = 2>
struct DkvDual {
    const DkvArgs& a;
    uint8_t* lds;
    bf16x8_t kf[8];                                        // K fragments of key block 0
    f32x16_t dvt[2][4], dkt[2][4];
    int G, lane, wave, hi, l32, k0, kw, n_sl, n_it, b, hk, per_slice;
    int key[2];
    bool kvalid[2];
    uint32_t lds0;
    uint32_t lo_row, lo_v0, lo_v1, lo_k1, lo_t0, lo_t4;

    __device__ __forceinline__ DkvDual(const DkvArgs& a_, uint8_t* lds_) : a(a_), lds(lds_) {}

    __device__ __forceinline__ void issue(int it) {            // Q and dO rows 8w .. 8w+7 of slice it
        const int hh = it / n_sl, sl = n_sl - 1 - (it - hh * n_sl);
        const int h = hk * G + hh;
        const int s0 = k0 + sl * kSlice;
        const uint32_t buf = lds0 + (uint32_t)((it % kDkvDualRing) * kSliceBuf);
        const uint16_t* qb = a.q.p + b * a.q.sb + h * a.q.sh;
        const uint16_t* db = a.dout.p + b * a.dout.sb + h * a.dout.sh;
        dma_rows(uniform_rsrc(qb, (int64_t)a.S * a.q.ss * 2), a.q.ss, buf, s0, s0 + 8 * wave, 2, lane);
        dma_rows(uniform_rsrc(db, (int64_t)a.S * a.dout.ss * 2), a.dout.ss, buf + (uint32_t)kSliceB, s0,
                 s0 + 8 * wave, 2, lane);
        if (wave < 2 && lane < 8) {
            const float* row = (wave == 0 ? a.lse : a.delta) + ((int64_t)b * a.Hq + h) * a.S;
            dma16(uniform_rsrc(row, (int64_t)a.S * 4), __builtin_amdgcn_readfirstlane(buf + 2 * kSliceB + 128 * wave),
                  (s0 + 4 * lane) * 4);
        }
    }

    // the slice's s0, or -1 when no q of the slice sees a key of the wave (both blocks skip it)
    __device__ __forceinline__ int slice_s0(int it) const {
        const int sl = n_sl - 1 - it % n_sl;               // descending q (see dkdv_block)
        const int s0 = k0 + sl * kSlice;
        return (s0 + kSlice - 1 < kw) ? -1 : s0;
    }

    // phase 1: S = Q K^T and dP = dO V^T of both key blocks; each Q / dO row fragment read once
    template <int SLOT>
    __device__ __forceinline__ void qk(f32x16_t (&s)[2], f32x16_t (&dp)[2]) {
        constexpr int QI = SLOT * kSliceBuf, DI = QI + kSliceB;
        const uint32_t lr = opaque(lo_row), lv0 = opaque(lo_v0), lv1 = opaque(lo_v1), lk1 = opaque(lo_k1);
        // k-step ks's five fragments (Q row, dO row, K row of block 1, V rows of blocks 0 / 1) are read
        // while k-step ks-1's four MFMAs run: one fence per k-step keeps that order
        bf16x8_t f[2][5];
        auto ld = [&](int ks, bf16x8_t (&g)[5]) {
            g[0] = rowx<QI>(lds, lr, ks);
            g[1] = rowx<DI>(lds, lr, ks);
            g[2] = rowx<0>(lds, lk1, ks);
            g[3] = rowx<0>(lds, lv0, ks);
            g[4] = rowx<0>(lds, lv1, ks);
        };
        ld(0, f[0]);
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            if (ks < 7) ld(ks + 1, f[(ks + 1) & 1]);
            const bf16x8_t(&c)[5] = f[ks & 1];
            if (ks == 0) mfma4_vgpr0(s[0], s[1], dp[0], dp[1], c[0], kf[ks], c[2], c[1], c[3], c[4]);
            else mfma4_vgpr(s[0], s[1], dp[0], dp[1], c[0], kf[ks], c[2], c[1], c[3], c[4]);
            __builtin_amdgcn_sched_barrier(0);
        }
        mfma_drain4(s[0], s[1], dp[0], dp[1]);
    }

    // P and dS of key block j (rows q = s0 + (i&3) + 8(i>>2) + 4hi of register i), packed to the B
    // fragments of the dV^T / dK^T products
    __device__ __forceinline__ void probs(int j, int s0, const float* cst, const f32x16_t& s, const f32x16_t& dp,
                                         bf16x8_t (&pf)[2], bf16x8_t (&sf)[2]) {
        float pr[16], dsv[16];
        const f32x2_t sl2v = {a.sl2, a.sl2};
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float4 lz = *reinterpret_cast<const float4*>(cst + 8 * g + 4 * hi);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = 4 * g + 2 * h;
                const f32x2_t l2 = h ? f32x2_t{lz.z, lz.w} : f32x2_t{lz.x, lz.y};
                const f32x2_t e = __builtin_elementwise_fma(f32x2_t{s[i], s[i + 1]}, sl2v, -l2);
                pr[i] = __builtin_amdgcn_exp2f(e.x);
                pr[i + 1] = __builtin_amdgcn_exp2f(e.y);
            }
        }
        const int kj = key[j];
        if (s0 < kj - l32 + kKW - 1) {                     // the slice crosses this block's diagonal
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int q = s0 + (i & 3) + 8 * (i >> 2) + 4 * hi;
                if (kj > q) pr[i] = 0.f;
            }
        }
        if (KMASK && !kvalid[j]) {
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
                const f32x2_t r = (f32x2_t{dp[i], dp[i + 1]} - d2) * f32x2_t{pr[i], pr[i + 1]};
                dsv[i] = r.x;
                dsv[i + 1] = r.y;
            }
        }
        pack_b_frags(pr, pf[0], pf[1]);
        pack_b_frags(dsv, sf[0], sf[1]);
    }

    // phase 2: dV^T += dO^T P and dK^T += Q^T dS of both blocks; each transposed fragment read once
    template <int SLOT>
    __device__ __forceinline__ void pv(int s0, const f32x16_t (&s)[2], const f32x16_t (&dp)[2]) {
        constexpr int QI = SLOT * kSliceBuf, DI = QI + kSliceB;
        const float* cst = reinterpret_cast<const float*>(lds + QI + 2 * kSliceB);
        bf16x8_t pf[2][2], sf[2][2];
        probs(0, s0, cst, s[0], dp[0], pf[0], sf[0]);
        probs(1, s0, cst, s[1], dp[1], pf[1], sf[1]);
        const uint32_t t0 = opaque(lo_t0), t4 = opaque(lo_t4);
        // the transposed dO / Q fragments of step n+1 are read while step n's MFMAs run
        bf16x8_t tf[2][2];
        tf[0][0] = trx<DI>(lds, t0, t4, 0, 0);
        tf[0][1] = trx<QI>(lds, t0, t4, 0, 0);
#pragma unroll
        for (int n = 0; n < 8; ++n) {
            const int dt = n >> 1, kq = n & 1;
            if (n < 7) {
                tf[(n + 1) & 1][0] = trx<DI>(lds, t0, t4, (n + 1) & 1, (n + 1) >> 1);
                tf[(n + 1) & 1][1] = trx<QI>(lds, t0, t4, (n + 1) & 1, (n + 1) >> 1);
            }
            mfma4_agpr(dvt[0][dt], dvt[1][dt], dkt[0][dt], dkt[1][dt], tf[n & 1][0], pf[0][kq], pf[1][kq], tf[n & 1][1],
                       sf[0][kq], sf[1][kq]);
            __builtin_amdgcn_sched_barrier(0);
        }
    }

    // one eighth of key block j's softmax (chunk c, compile-time): c 0-3: p of registers 4c..4c+3 (with
    // the causal mask when DIAG); c 4-7: ds of registers 4(c-4)..; c 5 / 7 also pack P / dS
    template <bool DIAG, int C>
    __device__ __forceinline__ void soft_chunk(int j, int s0, const float4 (&lz)[4], const float4 (&dz)[4],
                                               f32x16_t& s, f32x16_t& dp, bf16x8_t (&pf)[2], bf16x8_t (&sf)[2]) {
        if constexpr (C < 4) {
            const f32x2_t sl2v = {a.sl2, a.sl2};
            const float4 l = lz[C];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = 4 * C + 2 * h;
                const f32x2_t l2 = h ? f32x2_t{l.z, l.w} : f32x2_t{l.x, l.y};
                const f32x2_t e = __builtin_elementwise_fma(f32x2_t{s[i], s[i + 1]}, sl2v, -l2);
                float p0 = __builtin_amdgcn_exp2f(e.x), p1 = __builtin_amdgcn_exp2f(e.y);
                if (DIAG) {
                    const int q = s0 + (i & 3) + 8 * (i >> 2) + 4 * hi;
                    p0 = key[j] > q ? 0.f : p0;
                    p1 = key[j] > q + 1 ? 0.f : p1;
                }
                if (KMASK) {
                    p0 = kvalid[j] ? p0 : 0.f;
                    p1 = kvalid[j] ? p1 : 0.f;
                }
                s[i] = p0;                                 // P replaces S in place
                s[i + 1] = p1;
            }
        } else {
            const float4 d = dz[C - 4];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = 4 * (C - 4) + 2 * h;
                const f32x2_t d2 = h ? f32x2_t{d.z, d.w} : f32x2_t{d.x, d.y};
                const f32x2_t r = (f32x2_t{dp[i], dp[i + 1]} - d2) * f32x2_t{s[i], s[i + 1]};
                dp[i] = r.x;                               // dS replaces dP in place
                dp[i + 1] = r.y;
            }
            if constexpr (C == 5) {
                float pr[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) pr[i] = s[i];
                pack_b_frags(pr, pf[0], pf[1]);
            }
            if constexpr (C == 7) {
                float dsv[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) dsv[i] = dp[i];
                pack_b_frags(dsv, sf[0], sf[1]);
            }
        }
    }

    template <bool DIAG, int C>
    __device__ __forceinline__ void soft_chunks_from(int j, int s0, const float4 (&lz)[4], const float4 (&dz)[4],
                                                     f32x16_t& s, f32x16_t& dp, bf16x8_t (&pf)[2], bf16x8_t (&sf)[2],
                                                     int c) {
        // (dispatch on the unrolled loop index)
        if (c == C) soft_chunk<DIAG, C>(j, s0, lz, dz, s, dp, pf, sf);
        if constexpr (C + 1 < 8) soft_chunks_from<DIAG, C + 1>(j, s0, lz, dz, s, dp, pf, sf, c);
    }

    // V = 3: S0/dP0; S1/dP1 || softmax 0; dV0/dK0 || softmax 1; dV1/dK1 (2 MFMAs per group)
    template <int SLOT, bool DIAG>
    __device__ __forceinline__ void slice3(int s0) {
        constexpr int QI = SLOT * kSliceBuf, DI = QI + kSliceB;
        const uint32_t lr = opaque(lo_row), lv0 = opaque(lo_v0), lv1 = opaque(lo_v1), lk1 = opaque(lo_k1);
        const float* cst = reinterpret_cast<const float*>(lds + QI + 2 * kSliceB);
        float4 lz[4], dz[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            lz[g] = *reinterpret_cast<const float4*>(cst + 8 * g + 4 * hi);
            dz[g] = *reinterpret_cast<const float4*>(cst + 32 + 8 * g + 4 * hi);
        }
        f32x16_t s[2], dp[2];
        bf16x8_t pf[2][2], sf[2][2];
        // S0, dP0 (Q / dO rows, K0 in registers, V0 rows)
        {
            bf16x8_t f[2][3];
            auto ld = [&](int ks, bf16x8_t (&g)[3]) {
                g[0] = rowx<QI>(lds, lr, ks);
                g[1] = rowx<DI>(lds, lr, ks);
                g[2] = rowx<0>(lds, lv0, ks);
            };
            ld(0, f[0]);
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) {
                if (ks < 7) ld(ks + 1, f[(ks + 1) & 1]);
                const bf16x8_t(&c)[3] = f[ks & 1];
                if (ks == 0) mfma2_vgpr0(s[0], dp[0], c[0], kf[ks], c[1], c[2]);
                else mfma2_vgpr(s[0], dp[0], c[0], kf[ks], c[1], c[2]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // S1, dP1 (Q / dO rows again, K1 / V1 rows), softmax 0 in the gaps
        {
            bf16x8_t f[2][4];
            auto ld = [&](int ks, bf16x8_t (&g)[4]) {
                g[0] = rowx<QI>(lds, lr, ks);
                g[1] = rowx<DI>(lds, lr, ks);
                g[2] = rowx<0>(lds, lk1, ks);
                g[3] = rowx<0>(lds, lv1, ks);
            };
            ld(0, f[0]);
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) {
                if (ks < 7) ld(ks + 1, f[(ks + 1) & 1]);
                const bf16x8_t(&c)[4] = f[ks & 1];
                if (ks == 0) mfma2_vgpr0(s[1], dp[1], c[0], c[2], c[1], c[3]);
                else mfma2_vgpr(s[1], dp[1], c[0], c[2], c[1], c[3]);
                if (ks == 0) mfma_drain2(s[0], dp[0]);     // S0 / dP0 final before the softmax reads them
                soft_chunks_from<DIAG, 0>(0, s0, lz, dz, s[0], dp[0], pf[0], sf[0], ks);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        const uint32_t t0 = opaque(lo_t0), t4 = opaque(lo_t4);
        // dV0, dK0 (transposed dO / Q), softmax 1 in the gaps
        {
            bf16x8_t tf[2][2];
            tf[0][0] = trx<DI>(lds, t0, t4, 0, 0);
            tf[0][1] = trx<QI>(lds, t0, t4, 0, 0);
#pragma unroll
            for (int n = 0; n < 8; ++n) {
                const int dt = n >> 1, kq = n & 1;
                if (n < 7) {
                    tf[(n + 1) & 1][0] = trx<DI>(lds, t0, t4, (n + 1) & 1, (n + 1) >> 1);
                    tf[(n + 1) & 1][1] = trx<QI>(lds, t0, t4, (n + 1) & 1, (n + 1) >> 1);
                }
                mfma2_agpr(dvt[0][dt], dkt[0][dt], tf[n & 1][0], pf[0][kq], tf[n & 1][1], sf[0][kq]);
                if (n == 0) mfma_drain2(s[1], dp[1]);
                soft_chunks_from<DIAG, 0>(1, s0, lz, dz, s[1], dp[1], pf[1], sf[1], n);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // dV1, dK1 (the transposed fragments read again)
        {
            bf16x8_t tf[2][2];
            tf[0][0] = trx<DI>(lds, t0, t4, 0, 0);
            tf[0][1] = trx<QI>(lds, t0, t4, 0, 0);
#pragma unroll
            for (int n = 0; n < 8; ++n) {
                const int dt = n >> 1, kq = n & 1;
                if (n < 7) {
                    tf[(n + 1) & 1][0] = trx<DI>(lds, t0, t4, (n + 1) & 1, (n + 1) >> 1);
                    tf[(n + 1) & 1][1] = trx<QI>(lds, t0, t4, (n + 1) & 1, (n + 1) >> 1);
                }
                mfma2_agpr(dvt[1][dt], dkt[1][dt], tf[n & 1][0], pf[1][kq], tf[n & 1][1], sf[1][kq]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }

    template <int SLOT>
    __device__ __forceinline__ void step(int it) {
        constexpr int R = kDkvDualRing;
        if (it + R - 1 < n_it) issue(it + R - 1);          // into the slot slice it-1 used
        const int s0 = slice_s0(it);
        if (V == 3 && s0 >= 0) {
            // wave-uniform: the slice reaches below the diagonal of the wave's second block
            if (s0 < kw + 2 * kKW - 1) slice3<SLOT, true>(s0);
            else slice3<SLOT, false>(s0);
        } else if (s0 >= 0) {
            f32x16_t s[2], dp[2];
            qk<SLOT>(s, dp);
            pv<SLOT>(s0, s, dp);
        }
        vm_wait_upto(per_slice * max(0, min(R - 2, n_it - 2 - it)));   // slice it+1 landed
        __syncthreads();
    }

    template <int SLOT>
    __device__ __forceinline__ void steps(int it0) {       // slices it0 .. it0+R-1, slot = compile-time
        if (it0 + SLOT < n_it) {
            step<SLOT>(it0 + SLOT);
            if constexpr (SLOT + 1 < kDkvDualRing) steps<SLOT + 1>(it0);
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
        kw = k0 + wave * kDualKW;
        const uint16_t* kp = a.k.p + b * a.k.sb + hk * a.k.sh;
        const uint16_t* vp = a.v.p + b * a.v.sb + hk * a.v.sh;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            key[j] = kw + kKW * j + l32;
            kvalid[j] = !KMASK || (key[j] < a.S && key_bit(a.kmask[(int64_t)b * a.kmask_ld + (key[j] >> 6)], key[j]));
        }
        lds0 = lds_addr(lds);
        // V rows of the wave's 64 keys into the image after the ring; K rows of its second key block
        // into rows 32w .. 32w+31 of the K image after that
        dma_rows(uniform_rsrc(vp, (int64_t)a.S * a.v.ss * 2), a.v.ss, lds0 + kDkvDualRing * kSliceBuf, k0, kw,
                 kDualKW / 4, lane);
        dma_rows(uniform_rsrc(kp, (int64_t)a.S * a.k.ss * 2), a.k.ss, lds0 + kDkvDualRing * kSliceBuf + kVImg,
                 kw + kKW - kKW * wave, kw + kKW, kKW / 4, lane);
        {
            const uint32_t r = (uint32_t)l32;
            lo_row = r * kRowB + ((16u * hi) ^ (swz(r) << 4));
            // V rows wave*64 + 32j + l32 share row l32's swizzle (a multiple of 16 apart)
            lo_v0 = lo_row + (uint32_t)(kDkvDualRing * kSliceBuf + wave * kDualKW * kRowB);
            lo_v1 = lo_v0 + (uint32_t)(kKW * kRowB);
            lo_k1 = lo_row + (uint32_t)(kDkvDualRing * kSliceBuf + kVImg + wave * kKW * kRowB);
            const TrLane tl = tr_lane(lane);
            lo_t0 = tl.krow * kRowB + (tl.feat_byte ^ (swz(tl.krow) << 4));
            lo_t4 = (tl.krow + 4) * kRowB + (tl.feat_byte ^ (swz(tl.krow + 4) << 4));
        }
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
            if (key[0] < a.S)
                kf[ks] = *reinterpret_cast<const bf16x8_t*>(kp + (int64_t)key[0] * a.k.ss + 16 * ks + 8 * hi);
            else
                kf[ks] = __builtin_bit_cast(bf16x8_t, u32x4_t{0u, 0u, 0u, 0u});
        }
        n_sl = (a.S - k0 + kSlice - 1) / kSlice;
        n_it = G * n_sl;
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int dt = 0; dt < 4; ++dt) {
                zero_agpr(dvt[j][dt]);
                zero_agpr(dkt[j][dt]);
            }
        per_slice = 4 + (wave < 2 ? 1 : 0);                // DMA instructions per slice (+ lse / delta)
#pragma unroll
        for (int i = 0; i < kDkvDualRing - 1; ++i)
            if (i < n_it) issue(i);
        vm_wait_all();
        vm_wait_all_known();                               // the K fragments too (compiler-visible)
        __syncthreads();
        for (int it = 0; it < n_it; it += kDkvDualRing) steps<0>(it);
        mfma_drain_agpr(dvt, dkt);                         // the asm MFMAs' results, before any read
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (key[j] < a.S) {
                uint16_t* dkr = a.dk + b * a.dk_sb + hk * a.dk_sh + (int64_t)key[j] * a.dk_ss;
                uint16_t* dvr = a.dv + b * a.dv_sb + hk * a.dv_sh + (int64_t)key[j] * a.dv_ss;
#pragma unroll
                for (int dt = 0; dt < 4; ++dt)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const int d = 32 * dt + 8 * g + 4 * hi;
                        uint2 w;
                        w.x = pk_bf16(dkt[j][dt][4 * g] * a.scale, dkt[j][dt][4 * g + 1] * a.scale);
                        w.y = pk_bf16(dkt[j][dt][4 * g + 2] * a.scale, dkt[j][dt][4 * g + 3] * a.scale);
                        *reinterpret_cast<uint2*>(dkr + d) = w;
                        w.x = pk_bf16(dvt[j][dt][4 * g], dvt[j][dt][4 * g + 1]);
                        w.y = pk_bf16(dvt[j][dt][4 * g + 2], dvt[j][dt][4 * g + 3]);
                        *reinterpret_cast<uint2*>(dvr + d) = w;
                    }
            }
        }
    }
};

template <bool KMASK, int V>
__global__ __launch_bounds__(kDualKWaves * 64, 1) SMT_DKV_DUAL_ATTR
void attn_dkdv_dual_kernel(DkvArgs a) {
    static_assert(kKB == 256 && kDualKWaves == 4, "dual dK/dV: 256-key blocks of 4 waves");
    __shared__ __attribute__((aligned(16))) uint8_t lds[kDkvDualRing * kSliceBuf + kVImg + kKbImg];
    const int nkb = (a.S + kKB - 1) / kKB;
    const int total = ((nkb + 1) / 2) * a.Hkv * a.B;
    const PairTask t = pair_task(xcd_logical(blockIdx.x, total), nkb, 1, a.Hkv);
#pragma nounroll
    for (int i = 0; i < t.n; ++i) {
        if (i) __syncthreads();
        DkvDual<KMASK, V> d(a, lds);
        d.run(t.b, t.hk, t.blk[1 - i]);
    }
}

// SMT_ATTN_DKV (runtime): 1 = attn_dkdv_kernel (DkvLean, 8 waves x 32 keys, default), 2 / 3 = the
// one-wave-per-SIMD attn_dkdv_dual_kernel (DkvDual V = 2 / 3)
int dkv_impl() {
    static const int v = [] {
        const char* e = getenv("SMT_ATTN_DKV");
        const int x = e ? atoi(e) : 1;
        return (x == 2 || x == 3) ? x : 1;
    }();
    return v;
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
    return 0;
}

Tns tns(const smt_attn_tensor* t) { return Tns{static_cast<const uint16_t*>(t->ptr), t->sb, t->sh, t->ss}; }

}  // namespace

extern "C" {

const char* smt_attn_last_error(void) { return g_err; }

#if SMT_ATTN_STAMPS
// diagnostic builds only: copy the forward's tile stamps (uint64 [256][4][32][4]) to host memory
int smt_attn_debug_fwd_stamps(void* host, size_t bytes) {
    if (bytes < sizeof(g_fwd_stamps)) return fail(-1, "smt_attn_debug_fwd_stamps: %zu < %zu bytes", bytes, sizeof(g_fwd_stamps));
    hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fwd_stamps), sizeof(g_fwd_stamps), 0, hipMemcpyDeviceToHost);
    return e == hipSuccess ? 0 : fail(-4, "smt_attn_debug_fwd_stamps: %s", hipGetErrorString(e));
}
// the dK/dV kernel's slice stamps (uint64 [256][8][64][5])
int smt_attn_debug_dkv_stamps(void* host, size_t bytes) {
    if (bytes < sizeof(g_dkv_stamps)) return fail(-1, "smt_attn_debug_dkv_stamps: %zu < %zu bytes", bytes, sizeof(g_dkv_stamps));
    hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_dkv_stamps), sizeof(g_dkv_stamps), 0, hipMemcpyDeviceToHost);
    return e == hipSuccess ? 0 : fail(-4, "smt_attn_debug_dkv_stamps: %s", hipGetErrorString(e));
}
#endif

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
    if (!key_mask && fwd_impl() == 4) {
        const int64_t nqb = (shape->S + kPwQB - 1) / kPwQB;
        const int64_t blocks = nqb * shape->Hq * shape->B;
        if (blocks > 0x7fffffffLL) return fail(-1, "%s: too many blocks", fn);
        hipLaunchKernelGGL(attn_fwd_pw_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, a);
        return check_launch("attn_fwd_pw_kernel");
    }
    if (SMT_ATTN_FWD_IMPL == 3) {
        const int64_t nqb = (shape->S + kDualQB - 1) / kDualQB;
        const int64_t blocks = nqb * shape->Hq * shape->B;
        if (blocks > 0x7fffffffLL) return fail(-1, "%s: too many blocks", fn);
        if (key_mask) hipLaunchKernelGGL(attn_fwd_dual_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, stream, a);
        else hipLaunchKernelGGL(attn_fwd_dual_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, stream, a);
        return check_launch("attn_fwd_dual_kernel");
    }
    const int64_t nqb = (shape->S + kFwdQB - 1) / kFwdQB;
    const int64_t blocks = nqb * shape->Hq * shape->B;
    if (blocks > 0x7fffffffLL) return fail(-1, "%s: too many blocks", fn);
    if (key_mask) hipLaunchKernelGGL(attn_fwd_kernel<true>, dim3((unsigned)blocks), dim3(64 * kFwdWaves), 0, stream, a);
    else hipLaunchKernelGGL(attn_fwd_kernel<false>, dim3((unsigned)blocks), dim3(64 * kFwdWaves), 0, stream, a);
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

    if (!SMT_DQ_DELTA) {
        const int64_t rows = (int64_t)B * Hq * S;
        hipLaunchKernelGGL(attn_delta_kernel, dim3((unsigned)((rows * 16 + 255) / 256)), dim3(256), 0, stream,
                           tns(o), tns(d_o), delta_ws, Hq, S, rows);
        if ((rc = check_launch("attn_delta_kernel"))) return rc;
    }

    DqArgs qa;
    qa.q = tns(q); qa.k = tns(k); qa.v = tns(v); qa.dout = tns(d_o); qa.o = tns(o);
    qa.dq = static_cast<uint16_t*>(dq->ptr); qa.dq_sb = dq->sb; qa.dq_sh = dq->sh; qa.dq_ss = dq->ss;
    qa.lse = lse; qa.delta = delta_ws;
    qa.kmask = key_mask; qa.kmask_ld = key_mask_ld;
    qa.B = B; qa.Hq = Hq; qa.Hkv = Hkv; qa.S = S; qa.sl2 = sl2; qa.scale = shape->scale;
    if (dq_impl() == 2 && SMT_DQ_DELTA) {
        const int64_t nqb2 = (S + kDqDualQB - 1) / kDqDualQB;
        const dim3 g2((unsigned)(nqb2 * Hq * B)), b2(256);
        if (key_mask) hipLaunchKernelGGL(attn_dq_dual_kernel<true>, g2, b2, 0, stream, qa);
        else hipLaunchKernelGGL(attn_dq_dual_kernel<false>, g2, b2, 0, stream, qa);
        if ((rc = check_launch("attn_dq_dual_kernel"))) return rc;
    } else {
        const int64_t nqb = (S + kDqQB - 1) / kDqQB;
        const dim3 qgrid((unsigned)(nqb * Hq * B)), qblock(64 * kDqWaves);
        if (key_mask) hipLaunchKernelGGL(attn_dq_kernel<true>, qgrid, qblock, 0, stream, qa);
        else hipLaunchKernelGGL(attn_dq_kernel<false>, qgrid, qblock, 0, stream, qa);
        if ((rc = check_launch("attn_dq_kernel"))) return rc;
    }

    DkvArgs ka;
    ka.q = tns(q); ka.k = tns(k); ka.v = tns(v); ka.dout = tns(d_o);
    ka.dk = static_cast<uint16_t*>(dk->ptr); ka.dk_sb = dk->sb; ka.dk_sh = dk->sh; ka.dk_ss = dk->ss;
    ka.dv = static_cast<uint16_t*>(dv->ptr); ka.dv_sb = dv->sb; ka.dv_sh = dv->sh; ka.dv_ss = dv->ss;
    ka.lse = lse; ka.delta = delta_ws;
    ka.kmask = key_mask; ka.kmask_ld = key_mask_ld;
    ka.B = B; ka.Hq = Hq; ka.Hkv = Hkv; ka.S = S; ka.sl2 = sl2; ka.scale = shape->scale;
    const int64_t nkb = (S + kKB - 1) / kKB;
    const dim3 grid((unsigned)(((nkb + 1) / 2) * Hkv * B));
    if (dkv_impl() == 2) {
        if (key_mask) hipLaunchKernelGGL((attn_dkdv_dual_kernel<true, 2>), grid, dim3(kDualKWaves * 64), 0, stream, ka);
        else hipLaunchKernelGGL((attn_dkdv_dual_kernel<false, 2>), grid, dim3(kDualKWaves * 64), 0, stream, ka);
        return check_launch("attn_dkdv_dual_kernel");
    }
    if (dkv_impl() == 3) {
        if (key_mask) hipLaunchKernelGGL((attn_dkdv_dual_kernel<true, 3>), grid, dim3(kDualKWaves * 64), 0, stream, ka);
        else hipLaunchKernelGGL((attn_dkdv_dual_kernel<false, 3>), grid, dim3(kDualKWaves * 64), 0, stream, ka);
        return check_launch("attn_dkdv_dual_kernel");
    }
    if (key_mask) hipLaunchKernelGGL(attn_dkdv_kernel<true>, grid, dim3(kDkvWaves * 64), 0, stream, ka);
    else hipLaunchKernelGGL(attn_dkdv_kernel<false>, grid, dim3(kDkvWaves * 64), 0, stream, ka);
    return check_launch("attn_dkdv_kernel");
}

int smt_attn_bwd(const smt_attn_tensor* q, const smt_attn_tensor* k, const smt_attn_tensor* v,
                 const smt_attn_tensor* o, const smt_attn_tensor* d_o, const float* lse, float* delta_ws,
                 const smt_attn_tensor* dq, const smt_attn_tensor* dk, const smt_attn_tensor* dv,
                 const smt_attn_shape* shape, hipStream_t stream) {
    return smt_attn_bwd_kmask(q, k, v, o, d_o, lse, delta_ws, dq, dk, dv, nullptr, 0, shape, stream);
}

}  // extern "C"
