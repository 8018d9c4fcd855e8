// Micro: 16-byte global loads / stores at 4-byte-aligned (not 16-byte-aligned) addresses on gfx950
// (LLVM emits global_load/store_dwordx4 for a 4-byte-aligned 16-byte struct). Checks the copy
// bit for bit and times aligned vs shifted copies of a 256 MiB buffer with HIP events.
// build: hipcc --offload-arch=gfx950 -O3 tools/micro/unal_copy.hip -o tools/micro/unal_copy
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

struct __attribute__((packed, aligned(4))) F4u {
  float x, y, z, w;
};

__global__ void copy_k(const float* __restrict__ s, float* __restrict__ d, long n4) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
    *reinterpret_cast<F4u*>(d + 4 * i) = *reinterpret_cast<const F4u*>(s + 4 * i);
}

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                       \
    }                                                                 \
  } while (0)

int main() {
  const long n = 64l << 20;  // floats
  const long n4 = (n - 16) / 4;
  float *s, *d;
  CK(hipMalloc(&s, n * 4));
  CK(hipMalloc(&d, n * 4));
  std::vector<float> h(n);
  for (long i = 0; i < n; ++i) h[i] = (float)(i % 1000003) * 0.5f;
  CK(hipMemcpy(s, h.data(), n * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int bad_total = 0;
  for (int so = 0; so < 4; ++so)
    for (int dof = 0; dof < 4; ++dof) {
      CK(hipMemset(d, 0, n * 4));
      hipLaunchKernelGGL(copy_k, dim3(2048), dim3(256), 0, 0, s + so, d + dof, n4);
      CK(hipGetLastError());
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(copy_k, dim3(2048), dim3(256), 0, 0, s + so, d + dof, n4);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      std::vector<float> o(n);
      CK(hipMemcpy(o.data(), d, n * 4, hipMemcpyDeviceToHost));
      long bad = 0;
      for (long i = 0; i < 4 * n4; ++i) bad += o[dof + i] != h[so + i];
      bad_total += bad != 0;
      printf("src+%d dst+%d floats: %.1f GB/s, mismatches %ld\n", so, dof, 2.0 * 16 * n4 / (ms / 10 * 1e-3) / 1e9, bad);
    }
  printf(bad_total ? "FAIL\n" : "OK\n");
  return bad_total ? 1 : 0;
}
