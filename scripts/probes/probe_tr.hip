// Probe: semantics of ds_read_b64_tr_b16 and the 16x16x32 bf16 MFMA layout on gfx950.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

// LDS [32 rows][16 cols] of shorts = row*100+col; lane 4q+p reads row (q + 4*(lane>>4)) cols 4p..
__global__ void k_tr(int* out) {
  __shared__ __attribute__((aligned(16))) short lds[32 * 16];
  for (int i = threadIdx.x; i < 32 * 16; i += 64) lds[i] = (short)((i / 16) * 100 + (i % 16));
  __syncthreads();
  int lane = threadIdx.x;
  int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  short* a = lds + (4 * g + q) * 16 + 4 * p;
  v4s r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(a));
  for (int e = 0; e < 4; ++e) out[lane * 4 + e] = r[e];
}

// MFMA: A[i][k] = i + 100*k (as small ints in bf16), B[k][j] = (k==j%32) ? 1 : 0 ... use plain map
__global__ void k_mfma(const float* A, const float* B, float* C) {
  int l = threadIdx.x;
  v8bf a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)A[(l & 15) * 32 + 8 * (l >> 4) + j];   // A[row][k], 16x32
    b[j] = (__bf16)B[(8 * (l >> 4) + j) * 16 + (l & 15)];  // B[k][col], 32x16
  }
  v4f c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) C[((l >> 4) * 4 + r) * 16 + (l & 15)] = c[r];
}

extern "C" int probe_tr(int* out_dev) { hipLaunchKernelGGL(k_tr, 1, 64, 0, 0, out_dev); return hipDeviceSynchronize(); }
extern "C" int probe_mfma(const float* A, const float* B, float* C) { hipLaunchKernelGGL(k_mfma, 1, 64, 0, 0, A, B, C); return hipDeviceSynchronize(); }
