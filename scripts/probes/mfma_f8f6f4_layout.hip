// Probe: A/B operand lane map of v_mfma_scale_f32_16x16x128_f8f6f4 (fp8 e4m3,
// unit scales) on gfx950. One wave computes C = A(16x128) * B(128x16) with
// small exact integers; two candidate lane maps are tried and compared with
// the host result.  hipcc --offload-arch=gfx950 -O2 mfma_f8f6f4_layout.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ uint8_t e4m3(float f) { return __builtin_amdgcn_cvt_pk_fp8_f32(f, f, 0, false) & 0xff; }

// map 0: lane l holds row l&15, k = 32*(l>>4) + j (j = 0..31)
// map 1: lane l holds row l&15, k = 16*(l>>4) + j (j<16), 64 + 16*(l>>4) + (j-16) (j>=16)
__global__ void probe(const float* A, const float* B, float* C, int map) {
  int l = threadIdx.x;
  uint8_t a[32], b[32];
  for (int j = 0; j < 32; ++j) {
    int k = map == 0 ? 32 * (l >> 4) + j : (j < 16 ? 16 * (l >> 4) + j : 64 + 16 * (l >> 4) + (j - 16));
    a[j] = e4m3(A[(l & 15) * 128 + k]);
    b[j] = e4m3(B[k * 16 + (l & 15)]);
  }
  i32x8 av, bv;
  for (int i = 0; i < 8; ++i) {
    av[i] = a[4 * i] | a[4 * i + 1] << 8 | a[4 * i + 2] << 16 | a[4 * i + 3] << 24;
    bv[i] = b[4 * i] | b[4 * i + 1] << 8 | b[4 * i + 2] << 16 | b[4 * i + 3] << 24;
  }
  f32x4 c = {0, 0, 0, 0};
  // cbsz = blgp = 0 (fp8 e4m3), opsel 0, scales 127 = 2^0
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, 127, 0, 127);
  for (int r = 0; r < 4; ++r) C[((l >> 4) * 4 + r) * 16 + (l & 15)] = c[r];
}

int main() {
  float hA[16 * 128], hB[128 * 16], ref[256];
  for (int i = 0; i < 16 * 128; ++i) hA[i] = (float)((i * 7 + 3) % 5 - 2);
  for (int i = 0; i < 128 * 16; ++i) hB[i] = (float)((i * 11 + 1) % 7 - 3);
  for (int m = 0; m < 16; ++m)
    for (int n = 0; n < 16; ++n) {
      float s = 0;
      for (int k = 0; k < 128; ++k) s += hA[m * 128 + k] * hB[k * 16 + n];
      ref[m * 16 + n] = s;
    }
  float *dA, *dB, *dC, hC[256];
  hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dC, sizeof hC);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  for (int map = 0; map < 2; ++map) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, map);
    hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += std::fabs(hC[i] - ref[i]) > 1e-3f;
    std::printf("{\"probe\":\"mfma_scale_16x16x128_f8f6f4\",\"map\":%d,\"mismatches\":%d,\"c00\":%g,\"ref00\":%g}\n", map, bad, hC[0], ref[0]);
  }
  return 0;
}
