// One-off probe of the v_mfma_scale_f32_32x32x64_f8f6f4 operand / scale lane maps (e4m3 x e4m3).
// Wave w runs one MFMA on A = a[w][64 lanes][32 B], B = b[w][...], per-lane scales sa/sb[w][64]
// (opsel 0), and writes its 16 accumulators per lane to d[w][64][16].
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef int i32x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
__global__ __launch_bounds__(64) void probe(const int* a, const int* b, const int* sa, const int* sb, float* d) {
    const int w = blockIdx.x, l = threadIdx.x;
    i32x8_t A, B;
    for (int i = 0; i < 8; ++i) { A[i] = a[(w * 64 + l) * 8 + i]; B[i] = b[(w * 64 + l) * 8 + i]; }
    f32x16_t c;
    for (int i = 0; i < 16; ++i) c[i] = 0.f;
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B, c, 0, 0, 0, sa[w * 64 + l], 0, sb[w * 64 + l]);
    for (int i = 0; i < 16; ++i) d[(w * 64 + l) * 16 + i] = c[i];
}
extern "C" int run_probe(const int* a, const int* b, const int* sa, const int* sb, float* d, int waves) {
    hipLaunchKernelGGL(probe, dim3(waves), dim3(64), 0, 0, a, b, sa, sb, d);
    return (int)hipDeviceSynchronize();
}
