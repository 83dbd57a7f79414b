// Probe: how much VALU issue one wave gets on a SIMD while another wave on the SAME SIMD streams
// fp32 MFMAs (v_mfma_f32_16x16x4_f32 or v_mfma_f32_32x32x2_f32, independent accumulators). One
// workgroup of 8 waves on one CU: waves w and w + 4 share a SIMD; waves 0-3 run the MFMA stream,
// waves 4-7 the VALU stream (16 independent v_fma_f32 chains). Host program; prints per case the
// cycles per MFMA and per VALU instruction, each alone and co-running.
// Build: hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 (scalar v_fma_f32, not v_pk_fma_f32)
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

template <int SHAPE>  // 0: 16x16x4 (8 accumulators), 1: 32x32x2 (4 accumulators)
__global__ __launch_bounds__(512) void k_probe(int n_mfma, int n_valu, float* out, long long* cyc) {
  const int wave = threadIdx.x >> 6;
  const float a = out[threadIdx.x & 7] + 1.0f, b = out[8 + (threadIdx.x & 7)] + 2.0f;
  float res = 0.f;
  __builtin_amdgcn_s_barrier();
  const long long t0 = __builtin_amdgcn_s_memtime();
  if (wave < 4) {
    if (SHAPE == 0) {
      f4 acc[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
      for (int it = 0; it < n_mfma; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 8; ++i) res += acc[i][0];
    } else {
      f16v acc[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
      for (int it = 0; it < n_mfma; ++it)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i) res += acc[i][0];
    }
  } else {
    float x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = a + i;
    for (int it = 0; it < n_valu; ++it)
#pragma unroll
      for (int i = 0; i < 16; ++i) x[i] = __builtin_fmaf(x[i], a, b);
#pragma unroll
    for (int i = 0; i < 16; ++i) res += x[i];
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[64 + threadIdx.x] = res;
  if ((threadIdx.x & 63) == 0) cyc[wave] = t1 - t0;
}

template <int SHAPE>
static void run(float* out, long long* cyc, int nm, int nv, const char* tag) {
  hipLaunchKernelGGL(k_probe<SHAPE>, dim3(1), dim3(512), 0, 0, nm, nv, out, cyc);
  hipDeviceSynchronize();
  long long h[8];
  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  const int per = SHAPE == 0 ? 8 : 4;
  double cm = 0, cv = 0;
  for (int w = 0; w < 4; ++w) { cm += h[w]; cv += h[4 + w]; }
  cm /= 4;
  cv /= 4;
  printf("{\"case\": \"%s\", \"mfma\": \"%s\", \"n_mfma\": %d, \"n_valu\": %d, \"mfma_wave_cycles\": %.0f, "
         "\"cyc_per_mfma\": %.2f, \"valu_wave_cycles\": %.0f, \"cyc_per_valu\": %.2f}\n",
         tag, SHAPE == 0 ? "16x16x4f32" : "32x32x2f32", nm * per, nv * 16, cm, nm ? cm / (nm * per) : 0.0, cv,
         nv ? cv / (nv * 16) : 0.0);
}

int main() {
  float* out;
  long long* cyc;
  hipMalloc(&out, 1024 * 4);
  hipMemset(out, 0, 1024 * 4);
  hipMalloc(&cyc, 8 * 8);
  for (int rep = 0; rep < 2; ++rep) {
    run<0>(out, cyc, 2000, 0, "mfma_alone");
    run<0>(out, cyc, 0, 4000, "valu_alone");
    run<0>(out, cyc, 2000, 4000, "corun");
    run<1>(out, cyc, 2000, 0, "mfma_alone");
    run<1>(out, cyc, 2000, 8000, "corun");
  }
  return 0;
}
