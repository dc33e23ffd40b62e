// Diagnostic probes of gfx950 lane maps (ds_read_b64_tr_b16, mfma 32x32x16 bf16).
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) s16x4_t lds_s16x4_t;

// LDS image [16 rows][64 cols] int16 with value row*64+col; lane l supplies address of
// row (l>>2)&3 + 4*(l>>4), cols 4*(l&3); out[l*4+e] = returned element e.
__global__ void tr_probe(short* out) {
  __shared__ __attribute__((aligned(16))) short lds[16 * 64];
  for (int i = threadIdx.x; i < 16 * 64; i += 64) lds[i] = (short)i;
  __syncthreads();
  int l = threadIdx.x;
  int row = ((l >> 2) & 3) + 4 * (l >> 4);
  int col = 4 * (l & 3);
  s16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(lds + row * 64 + col));
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}

// A[32][16] with A[i][k] = i*16+k (as bf16, exact), B = [16][32] with B[k][j] = (k==j%16 && j<16)
// lane l: A elems j: A[l&31][8*(l>>5)+j]; B elems: B[8*(l>>5)+j][l&31]. out = D[32][32] via claimed C map.
__global__ void mfma_probe(float* out, int mode) {
  int l = threadIdx.x;
  bf16x8_t a, b;
  for (int j = 0; j < 8; ++j) {
    int i = l & 31, k = 8 * (l >> 5) + j;
    float av = (float)((i * 16 + k) % 61);
    float bv = (mode == 0) ? ((k == (i % 16)) ? 1.f : 0.f) : (float)((k * 3 + i) % 7);
    a[j] = (__bf16)av;
    b[j] = (__bf16)bv;
  }
  f32x16_t c = {};
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) {
    int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    int col = l & 31;
    out[row * 32 + col] = c[r];
  }
}

extern "C" int run_probes(short* tr_out, float* mf0, float* mf1) {
  hipLaunchKernelGGL(tr_probe, dim3(1), dim3(64), 0, 0, tr_out);
  hipLaunchKernelGGL(mfma_probe, dim3(1), dim3(64), 0, 0, mf0, 0);
  hipLaunchKernelGGL(mfma_probe, dim3(1), dim3(64), 0, 0, mf1, 1);
  return hipDeviceSynchronize();
}

// image [16 k-rows][256 features] bf16 with value k*256+f stored at swizzled byte k*512 + ((2f) ^ ((k&3)<<6)) (SWZ=1) or plain.
template <int SWZ>
__global__ void tr_swz_probe(short* out) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[16 * 512];
  for (int i = threadIdx.x; i < 16 * 256; i += 64) {
    int k = i / 256, f = i % 256;
    unsigned off = k * 512 + (SWZ ? ((2u * f) ^ ((k & 3u) << 6)) : 2u * f);
    *(short*)(lds + off) = (short)(k * 256 + f);
  }
  __syncthreads();
  int lane = threadIdx.x;
  int gi = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  unsigned k = 8u * (gi >> 1) + q;
  unsigned b = 2u * (32 + 16u * (gi & 1) + 4u * p);   // m0 = 32
  unsigned off = k * 512 + (SWZ ? (b ^ ((k & 3u) << 6)) : b);
  s16x4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(lds + off));
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = v[e];
}

extern "C" int run_swz(short* o0, short* o1) {
  hipLaunchKernelGGL(tr_swz_probe<0>, dim3(1), dim3(64), 0, 0, o0);
  hipLaunchKernelGGL(tr_swz_probe<1>, dim3(1), dim3(64), 0, 0, o1);
  return hipDeviceSynchronize();
}
