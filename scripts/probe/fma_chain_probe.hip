// Probe: is one v_mfma_f32_16x16x4_f32 chain (the act / rollout layer chains: k-block t, k-step c,
// lane group g covering k = 16 t + 4 g + c) bitwise equal to a VALU fmaf chain over the same k
// order? If so, a VALU (v_pk_fma_f32) formulation of a layer with fewer rows per workgroup produces
// the MFMA path's results bit for bit. One wave; random operands incl. cancellation; prints the
// number of mismatching outputs for the MFMA chain against (a) the g-major fmaf chain
// k = 16 t + 4 g + c (g inner), (b) the c-major chain (c inner), (c) the natural order k = 0 .. K-1.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off scripts/probe/fma_chain_probe.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int K = 256, NKB = K / 16;

// D[i][j] = C[i][j] + sum_k A[i][k] B[k][j]; A [16][K], B [K][16] row-major; out [16][16]
__global__ void k_mfma(const float* A, const float* B, const float* C, float* out) {
  const int l = threadIdx.x, j = l & 15, g = l >> 4;
  f4 acc;
  for (int r = 0; r < 4; ++r) acc[r] = C[(4 * g + r) * 16 + j];
  for (int t = 0; t < NKB; ++t)
    for (int c = 0; c < 4; ++c) {
      const int k = 16 * t + 4 * g + c;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[j * K + k], B[k * 16 + j], acc, 0, 0, 0);
    }
  for (int r = 0; r < 4; ++r) out[(4 * g + r) * 16 + j] = acc[r];
}

// fmaf chains, one output per lane (256 lanes), three k orders
__global__ void k_fma(const float* A, const float* B, const float* C, float* out, int order) {
  const int o = threadIdx.x, i = o >> 4, j = o & 15;
  float acc = C[i * 16 + j];
  for (int t = 0; t < NKB; ++t)
    for (int p = 0; p < 4; ++p)
      for (int q = 0; q < 4; ++q) {
        int k;
        if (order == 0) k = 16 * t + 4 * q + p;       // c = p outer, g = q inner (MFMA lane-group order)
        else if (order == 1) k = 16 * t + 4 * p + q;  // g outer, c inner
        else k = 16 * t + 4 * p + q;                  // natural order == (1) for this decomposition
        acc = __builtin_fmaf(A[i * K + k], B[k * 16 + j], acc);
      }
  out[o] = acc;
}

// the same chain as packed fp32 FMAs over two rows (v_pk_fma_f32): out[i][2 jj .. 2 jj + 1]
__global__ void k_pkfma(const float* A, const float* B, const float* C, float* out) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const int o = threadIdx.x, i = o >> 3, jj = o & 7;  // 128 lanes
  f2 acc = f2{C[i * 16 + 2 * jj], C[i * 16 + 2 * jj + 1]};
  for (int t = 0; t < NKB; ++t)
    for (int p = 0; p < 4; ++p)
      for (int q = 0; q < 4; ++q) {
        const int k = 16 * t + 4 * q + p;
        const f2 a = f2{A[i * K + k], A[i * K + k]};
        const f2 b = f2{B[k * 16 + 2 * jj], B[k * 16 + 2 * jj + 1]};
        acc = __builtin_elementwise_fma(a, b, acc);
      }
  out[i * 16 + 2 * jj] = acc.x;
  out[i * 16 + 2 * jj + 1] = acc.y;
}

int main() {
  srand(7);
  std::vector<float> A(16 * K), B(K * 16), C(256);
  auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
  for (auto& x : A) x = rnd() * (rand() % 4 == 0 ? 100.f : 1.f);
  for (auto& x : B) x = rnd() * (rand() % 5 == 0 ? 1e-3f : 1.f);
  for (auto& x : C) x = rnd();
  float *dA, *dB, *dC, *dO;
  hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4); hipMalloc(&dC, 1024); hipMalloc(&dO, 1024);
  hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dC, C.data(), 1024, hipMemcpyHostToDevice);
  std::vector<float> m(256), f(256);
  hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, dA, dB, dC, dO);
  hipMemcpy(m.data(), dO, 1024, hipMemcpyDeviceToHost);
  const char* names[] = {"c-outer/g-inner (lane-group order)", "g-outer/c-inner", "natural"};
  for (int order = 0; order < 3; ++order) {
    hipLaunchKernelGGL(k_fma, dim3(1), dim3(256), 0, 0, dA, dB, dC, dO, order);
    hipMemcpy(f.data(), dO, 1024, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; ++i) bad += memcmp(&m[i], &f[i], 4) != 0;
    printf("{\"probe\": \"fma_chain\", \"order\": \"%s\", \"mismatches\": %d}\n", names[order], bad);
  }
  hipLaunchKernelGGL(k_pkfma, dim3(1), dim3(128), 0, 0, dA, dB, dC, dO);
  hipMemcpy(f.data(), dO, 1024, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 256; ++i) bad += memcmp(&m[i], &f[i], 4) != 0;
  printf("{\"probe\": \"fma_chain\", \"order\": \"pk_fma c-outer/g-inner\", \"mismatches\": %d}\n", bad);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
