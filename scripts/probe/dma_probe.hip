// Probe of buffer_load ... lds (LDS DMA) semantics on gfx950: where each lane's bytes land in LDS
// and what an out-of-range offset writes. Host program; prints the LDS image for one wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef struct { __amdgpu_buffer_rsrc_t r; } Buf;

__global__ void probe(const float* src, int n, float* out, int size16) {
  __shared__ __attribute__((aligned(16))) float s[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) s[i] = -1.f;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, n * 4, 0x00020000);
  const int lane = threadIdx.x;
  // lane L loads element (L * 3) % 64 (unit for 16-byte), lanes >= 48 use an out-of-range offset
  const unsigned off = lane >= 48 ? 0xFFFFFFF0u : (unsigned)((lane * 3) % 64) * (size16 ? 16u : 4u);
  auto* l = (__attribute__((address_space(3))) void*)(s + 256);
  if (size16) __builtin_amdgcn_raw_ptr_buffer_load_lds(r, l, 16, off, 0, 0, 0);
  else __builtin_amdgcn_raw_ptr_buffer_load_lds(r, l, 4, off, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 1024; i += 64) out[i] = s[i];
}

int main() {
  std::vector<float> h(256);
  for (int i = 0; i < 256; ++i) h[i] = 1000.f + i;
  float *d, *o;
  hipMalloc(&d, 256 * 4);
  hipMalloc(&o, 1024 * 4);
  hipMemcpy(d, h.data(), 256 * 4, hipMemcpyHostToDevice);
  for (int s16 = 0; s16 < 2; ++s16) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, 256, o, s16);
    std::vector<float> r(1024);
    hipMemcpy(r.data(), o, 1024 * 4, hipMemcpyDeviceToHost);
    printf("size %d: LDS[256 ..]:", s16 ? 16 : 4);
    for (int i = 256; i < 256 + (s16 ? 256 : 64) + 8; ++i) printf(" %g", r[i]);
    printf("\n");
  }
  return 0;
}
