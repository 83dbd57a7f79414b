// Probe: v_mfma_f32_4x4x1_16b_f32 (16 blocks of 4x4, K = 1) on gfx950 —
//  (1) its operand / result lane map (hypothesis: lane l: block b = l >> 2; A[b][i = l & 3][0],
//      B[b][0][j = l & 3], result register r = row i of column j = l & 3);
//  (2) whether a chain of it over k is bitwise the fmaf chain in k order (as the 16x16x4 form is);
//  (3) cycles per instruction with 1, 2 and 4 independent accumulators (one wave on the SIMD).
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off scripts/probe/mfma4x4_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int K = 256;

// A [16 blocks][4][K], B [16][K][4] -> out [16][4][4]
__global__ void k_chain(const float* A, const float* B, float* out) {
  const int l = threadIdx.x, b = l >> 2, q = l & 3;
  f4 acc = f4{0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < K; ++k)
    acc = __builtin_amdgcn_mfma_f32_4x4x1f32(A[(b * 4 + q) * K + k], B[(b * K + k) * 4 + q], acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[(b * 4 + r) * 4 + q] = acc[r];  // hypothesis: reg r = row, lane q = column
}

__global__ void k_ref(const float* A, const float* B, float* out) {
  const int t = threadIdx.x, b = t >> 4, i = (t >> 2) & 3, j = t & 3;
  float acc = 0.f;
  for (int k = 0; k < K; ++k) acc = __builtin_fmaf(A[(b * 4 + i) * K + k], B[(b * K + k) * 4 + j], acc);
  out[(b * 4 + i) * 4 + j] = acc;
}

template <int NACC>
__global__ void k_time(float a, float bb, int n, float* out, long long* cyc) {
  f4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < n; ++it)
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, bb, acc[i], 0, 0, 0);
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += acc[i][0];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  srand(11);
  std::vector<float> A(16 * 4 * K), B(16 * K * 4);
  for (auto& x : A) x = ((float)rand() / RAND_MAX * 2.f - 1.f) * (rand() % 4 == 0 ? 50.f : 1.f);
  for (auto& x : B) x = ((float)rand() / RAND_MAX * 2.f - 1.f);
  float *dA, *dB, *dO, *dR;
  long long* dc;
  hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4); hipMalloc(&dO, 256 * 4); hipMalloc(&dR, 256 * 4);
  hipMalloc(&dc, 8);
  hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_chain, dim3(1), dim3(64), 0, 0, dA, dB, dO);
  hipLaunchKernelGGL(k_ref, dim3(1), dim3(256), 0, 0, dA, dB, dR);
  std::vector<float> o(256), r(256);
  hipMemcpy(o.data(), dO, 1024, hipMemcpyDeviceToHost);
  hipMemcpy(r.data(), dR, 1024, hipMemcpyDeviceToHost);
  int bad = 0, close = 0;
  for (int i = 0; i < 256; ++i) {
    bad += memcmp(&o[i], &r[i], 4) != 0;
    close += fabsf(o[i] - r[i]) <= 1e-4f * (1.f + fabsf(r[i]));
  }
  printf("{\"probe\": \"mfma4x4\", \"layout_close\": %d, \"bitwise_mismatches\": %d, \"of\": 256}\n", close, bad);
  long long c;
  const int n = 4096;
  hipLaunchKernelGGL(k_time<1>, dim3(1), dim3(64), 0, 0, 1.0f, 1e-6f, n, dO, dc);
  hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
  printf("{\"probe\": \"mfma4x4\", \"accumulators\": 1, \"cycles_per_mfma\": %.2f}\n", (double)c / n);
  hipLaunchKernelGGL(k_time<2>, dim3(1), dim3(64), 0, 0, 1.0f, 1e-6f, n, dO, dc);
  hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
  printf("{\"probe\": \"mfma4x4\", \"accumulators\": 2, \"cycles_per_mfma\": %.2f}\n", (double)c / (2.0 * n));
  hipLaunchKernelGGL(k_time<4>, dim3(1), dim3(64), 0, 0, 1.0f, 1e-6f, n, dO, dc);
  hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
  printf("{\"probe\": \"mfma4x4\", \"accumulators\": 4, \"cycles_per_mfma\": %.2f}\n", (double)c / (4.0 * n));
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
