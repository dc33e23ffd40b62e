#include <hip/hip_runtime.h>
#include <stdint.h>
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;
constexpr int kTile = 256; constexpr int kTileElems = 65536;
constexpr int kWgThreads = 512;
constexpr int kBK = 64;                        // T rows per stage
constexpr int kRowBytes = kTile * 2;           // 512
constexpr int kImgBytes = kBK * kRowBytes;     // 32 KiB per operand per stage
constexpr int kChunksPerThread = (kImgBytes / 16) / kWgThreads;   // 4 x 16 B per operand
static_assert(kChunksPerThread == 4, "staging geometry");

__device__ __forceinline__ uint32_t img_off(uint32_t k, uint32_t byte_in_row) {
    return k * kRowBytes + (byte_in_row ^ ((k & 3u) << 6));
}

__device__ __forceinline__ bf16x8_t tr_frag(const uint8_t* img, uint32_t k, uint32_t byte_in_row) {
    s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(img + img_off(k, byte_in_row)));
    s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(img + img_off(k + 4, byte_in_row)));
    // whole-vector bit casts: element-wise __bf16 bit_casts of vector lanes miscompile (all lanes
    // came back equal to element 0 on ROCm 7.2 / gfx950)
    const s16x8_t both = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8_t, both);
}

__global__ __launch_bounds__(kWgThreads, 2)
void wgrad_dbg_kernel(const uint16_t* __restrict__ g, int64_t ldg,
                          const uint16_t* __restrict__ x, int64_t ldx,
                          int64_t T, int64_t chunk, int S,
                          const int32_t* __restrict__ tile_rc,
                          float* __restrict__ slab, uint8_t* dump) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * 2 * kImgBytes];   // 128 KiB, one array

    const int wg = blockIdx.x;
    const int tile = wg / S;
    const int s = wg - tile * S;
    const int r = tile_rc[2 * tile];
    const int c = tile_rc[2 * tile + 1];
    const int64_t t_begin = (int64_t)s * chunk;
    const int64_t t_end = (t_begin + chunk < T) ? (t_begin + chunk) : T;
    const int nst = (t_end > t_begin) ? (int)((t_end - t_begin + kBK - 1) / kBK) : 0;

    const uint16_t* gb = g + (int64_t)r * kTile;
    const uint16_t* xb = x + (int64_t)c * kTile;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int wm = wave >> 2;          // 0..1 -> rows wm*128
    const int wn = wave & 3;           // 0..3 -> cols wn*64

    uint4 ra[kChunksPerThread], rb[kChunksPerThread];

    auto gload = [&](int st) {
        const int64_t t0 = t_begin + (int64_t)st * kBK;
        if (t0 + kBK <= t_end) {
#pragma unroll
            for (int i = 0; i < kChunksPerThread; ++i) {
                const int cid = tid + kWgThreads * i;
                const int64_t t = t0 + (cid >> 5);
                const int e = (cid & 31) * 8;
                ra[i] = *reinterpret_cast<const uint4*>(gb + t * ldg + e);
                rb[i] = *reinterpret_cast<const uint4*>(xb + t * ldx + e);
            }
        } else {
#pragma unroll
            for (int i = 0; i < kChunksPerThread; ++i) {
                const int cid = tid + kWgThreads * i;
                const int64_t t = t0 + (cid >> 5);
                const int e = (cid & 31) * 8;
                if (t < t_end) {
                    ra[i] = *reinterpret_cast<const uint4*>(gb + t * ldg + e);
                    rb[i] = *reinterpret_cast<const uint4*>(xb + t * ldx + e);
                } else {
                    ra[i] = make_uint4(0, 0, 0, 0);
                    rb[i] = make_uint4(0, 0, 0, 0);
                }
            }
        }
    };
    auto swrite = [&](int buf) {
        uint8_t* A = lds + buf * 2 * kImgBytes;
        uint8_t* B = A + kImgBytes;
#pragma unroll
        for (int i = 0; i < kChunksPerThread; ++i) {
            const int cid = tid + kWgThreads * i;
            const uint32_t off = img_off((uint32_t)(cid >> 5), (uint32_t)(cid & 31) * 16u);
            *reinterpret_cast<uint4*>(A + off) = ra[i];
            *reinterpret_cast<uint4*>(B + off) = rb[i];
        }
    };

    f32x16_t acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    // tr-read lane geometry: group gi = lane>>4 covers feature offset 16*(gi&1) and k offset
    // 8*(gi>>1); lane 4q+p of the group supplies row q, features 4p..4p+3 (T10).
    const int gi = lane >> 4;
    const int q = (lane >> 2) & 3;
    const int p = lane & 3;
    const uint32_t feat_byte = 2u * (16u * (gi & 1) + 4u * p);
    const uint32_t krow = 8u * (gi >> 1) + q;

    if (nst > 0) {
        gload(0);
        swrite(0);
    }
    __syncthreads();

    if (dump) {
        if (wave == 0) {
            bf16x8_t f0 = tr_frag(lds, krow, 2u * 0 + feat_byte);
            bf16x8_t f1 = tr_frag(lds, 16 + krow, 2u * 32 + feat_byte);
            for (int j = 0; j < 8; ++j) { ((short*)dump)[lane * 16 + j] = __builtin_bit_cast(short, f0[j]); ((short*)dump)[lane * 16 + 8 + j] = __builtin_bit_cast(short, f1[j]); }
            ((int*)dump)[4096 + lane] = (int)img_off(krow, feat_byte);
        }
        return;
    }
    for (int st = 0; st < nst; ++st) {
        const int buf = st & 1;
        if (st + 1 < nst) gload(st + 1);
        const uint8_t* A = lds + buf * 2 * kImgBytes;
        const uint8_t* B = A + kImgBytes;
#pragma unroll
        for (int ks = 0; ks < kBK / 16; ++ks) {
            bf16x8_t af[4], bfr[2];
#pragma unroll
            for (int mb = 0; mb < 4; ++mb)
                af[mb] = tr_frag(A, ks * 16 + krow, 2u * (wm * 128 + mb * 32) + feat_byte);
#pragma unroll
            for (int nb = 0; nb < 2; ++nb)
                bfr[nb] = tr_frag(B, ks * 16 + krow, 2u * (wn * 64 + nb * 32) + feat_byte);
#pragma unroll
            for (int mb = 0; mb < 4; ++mb)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb)
                    acc[mb][nb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mb], bfr[nb], acc[mb][nb], 0, 0, 0);
        }
        if (st + 1 < nst) swrite(buf ^ 1);
        __syncthreads();
    }

    // C/D map of 32x32x16: col = lane&31, row = (i&3) + 8*(i>>2) + 4*(lane>>5)
    float* out = slab + (int64_t)(tile * S + s) * kTileElems;
    const int col = lane & 31;
    const int h = lane >> 5;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int m = wm * 128 + mb * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
                const int n = wn * 64 + nb * 32 + col;
                out[m * kTile + n] = acc[mb][nb][i];
            }
}


extern "C" int run_dbg(const void* g, const void* x, long T, const int* rc, float* slab, uint8_t* dump) {
  hipLaunchKernelGGL(wgrad_dbg_kernel, dim3(1), dim3(512), 0, 0, (const uint16_t*)g, 256L, (const uint16_t*)x, 256L, T, 64L, 1, rc, slab, dump);
  return hipDeviceSynchronize();
}
