// Probe: v_mfma_f32_16x16x4_f32 chains vs fmaf chains (k = 16 t + 4 g + c order) on network-like data:
// A = weights ~ N(0, 1/256), B = ReLU(N(0, 1)) (half exact zeros), C = small biases; 4096 chains per
// launch x 64 launches of different seeds. Prints the mismatch count and the first few mismatches.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int K = 256, NW = 16;  // waves per launch; each wave: 16 x 16 outputs

__global__ void k_mfma(const float* A, const float* B, const float* C, float* out) {
  const int w = blockIdx.x, l = threadIdx.x, j = l & 15, g = l >> 4;
  const float* Aw = A + (size_t)w * 16 * K;
  const float* Bw = B + (size_t)w * K * 16;
  f4 acc;
  for (int r = 0; r < 4; ++r) acc[r] = C[w * 256 + (4 * g + r) * 16 + j];
  for (int t = 0; t < K / 16; ++t)
    for (int c = 0; c < 4; ++c) {
      const int k = 16 * t + 4 * g + c;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(Aw[j * K + k], Bw[k * 16 + j], acc, 0, 0, 0);
    }
  for (int r = 0; r < 4; ++r) out[w * 256 + (4 * g + r) * 16 + j] = acc[r];
}
__global__ void k_fma(const float* A, const float* B, const float* C, float* out) {
  const int w = blockIdx.x, o = threadIdx.x, i = o >> 4, j = o & 15;
  const float* Aw = A + (size_t)w * 16 * K;
  const float* Bw = B + (size_t)w * K * 16;
  float acc = C[w * 256 + i * 16 + j];
  for (int t = 0; t < K / 16; ++t)
    for (int c = 0; c < 4; ++c)
      for (int g = 0; g < 4; ++g) {
        const int k = 16 * t + 4 * g + c;
        acc = __builtin_fmaf(Aw[i * K + k], Bw[k * 16 + j], acc);
      }
  out[w * 256 + o] = acc;
}

int main() {
  std::mt19937 rng(123);
  std::normal_distribution<float> nd(0.f, 1.f);
  const int NB = 256;  // waves per launch
  std::vector<float> A((size_t)NB * 16 * K), B((size_t)NB * K * 16), C(NB * 256);
  float *dA, *dB, *dC, *d1, *d2;
  (void)hipMalloc(&dA, A.size() * 4); (void)hipMalloc(&dB, B.size() * 4); (void)hipMalloc(&dC, C.size() * 4);
  (void)hipMalloc(&d1, C.size() * 4); (void)hipMalloc(&d2, C.size() * 4);
  std::vector<float> o1(C.size()), o2(C.size());
  long bad = 0, total = 0, zero_sign = 0;
  for (int rep = 0; rep < 16; ++rep) {
    for (auto& x : A) x = nd(rng) * 0.0625f;
    for (auto& x : B) { const float v = nd(rng); x = v > 0 ? v : 0.f; }
    for (auto& x : C) x = nd(rng) * 0.05f;
    (void)hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_mfma, dim3(NB), dim3(64), 0, 0, dA, dB, dC, d1);
    hipLaunchKernelGGL(k_fma, dim3(NB), dim3(256), 0, 0, dA, dB, dC, d2);
    (void)hipMemcpy(o1.data(), d1, o1.size() * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(o2.data(), d2, o2.size() * 4, hipMemcpyDeviceToHost);
    for (size_t i = 0; i < o1.size(); ++i) {
      ++total;
      if (memcmp(&o1[i], &o2[i], 4)) {
        if (o1[i] == o2[i]) ++zero_sign;
        else if (bad++ < 5) printf("{\"mismatch\": %zu, \"mfma\": %.9g, \"fma\": %.9g}\n", i, o1[i], o2[i]);
      }
    }
  }
  printf("{\"probe\": \"fma_chain_big\", \"chains\": %ld, \"mismatches\": %ld, \"signed_zero_only\": %ld}\n", total, bad,
         zero_sign);
  return 0;
}
