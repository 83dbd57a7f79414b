// Probe: per-CU fetch rate of an L2-resident 256 KB weight matrix ([256][256] fp32) with
// buffer_load_dwordx4, in the A-operand pattern of the MFMA kernels (lane (j, g) of a wave reads
// row 16 ft + j, columns 16 kb + 4 g: 16 rows x 64 B per instruction) against a contiguous pattern
// (1 KB per instruction) and a pre-swizzled layout. Host program; prints one line per case:
// bytes per CU clock (in-kernel s_memtime cycles) and the clock (s_memtime / s_memrealtime).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 ld(__amdgpu_buffer_rsrc_t r, int off_floats) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, off_floats * 4, 0, 0));
}

// PAT 0: MFMA A-operand rows (strided); PAT 1: contiguous 1 KB per wave-instruction
template <int PAT>
__global__ __launch_bounds__(256) void k_fetch(const float* w, int iters, int mask, float* out, unsigned long long* clk) {
  // mask is 0 at run time: every iteration re-reads the same 256 KB, but the compiler cannot hoist the loads
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)w, (short)0, 2 * 65536 * 4, 0x00020000);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, j = lane & 15, g = lane >> 4;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int ft = 0; ft < 4; ++ft) {
      f4 v[16];
#pragma unroll
      for (int kb = 0; kb < 16; ++kb) {
        const int off = (it & mask) * 65536 + (PAT == 0 ? (wave * 64 + 16 * ft + j) * 256 + 16 * kb + 4 * g
                                 : ((wave * 4 + ft) * 16 + kb) * 256 + 4 * lane);
        v[kb] = ld(r, off);
      }
#pragma unroll
      for (int kb = 0; kb < 16; ++kb) acc += v[kb];
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
  if (threadIdx.x == 0) {
    clk[blockIdx.x * 2] = t1 - t0;
    clk[blockIdx.x * 2 + 1] = r1 - r0;
  }
}

template <int PAT>
static void run(const float* w, float* out, unsigned long long* clk, int nblk, int iters) {
  hipLaunchKernelGGL(k_fetch<PAT>, dim3(nblk), dim3(256), 0, 0, w, 2, 0, out, clk);  // warm L2
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(k_fetch<PAT>, dim3(nblk), dim3(256), 0, 0, w, iters, 0, out, clk);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(2 * nblk);
  hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost);
  double cyc = 0, rt = 0;
  for (int b = 0; b < nblk; ++b) { cyc += h[2 * b]; rt += h[2 * b + 1]; }
  cyc /= nblk;
  rt /= nblk;
  const double bytes_wg = 256.0 * 1024 * iters;
  const double wg_per_cu = nblk / 256.0;
  printf("{\"pattern\": \"%s\", \"workgroups\": %d, \"wg_per_cu\": %.0f, \"B_per_clk_per_CU\": %.1f, \"GHz\": %.3f, "
         "\"kernel_ms\": %.3f, \"TB_per_s_total\": %.2f}\n",
         PAT == 0 ? "mfma_rows_strided" : "contiguous_1KB", nblk, wg_per_cu, bytes_wg * wg_per_cu / cyc,
         cyc / (rt * 10.0), ms, bytes_wg * nblk / (ms * 1e-3) / 1e12);
}

int main() {
  float *w, *out;
  unsigned long long* clk;
  hipMalloc(&w, 2 * 65536 * 4);
  hipMemset(w, 0, 2 * 65536 * 4);
  hipMalloc(&out, 1024 * 256 * 4);
  hipMalloc(&clk, 1024 * 2 * 8);
  for (int nblk : {256, 512, 1024}) {
    run<0>(w, out, clk, nblk, 64);
    run<1>(w, out, clk, nblk, 64);
  }
  return 0;
}
