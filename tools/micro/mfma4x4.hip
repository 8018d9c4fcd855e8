// Micro: layout and issue rate of v_mfma_f32_4x4x1_16b_f32 vs v_mfma_f32_16x16x4_f32 on gfx950.
// Build: hipcc -O3 --offload-arch=gfx950 tools/micro/mfma4x4.hip -o tools/micro/mfma4x4
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ void layout(float* out, const float* A, const float* B) {
  const int l = threadIdx.x;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_4x4x1f32(A[l], B[l], acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = acc[r];
}

template <int KIND, int NACC>
__global__ void rate(float* out, int iters) {
  const int l = threadIdx.x & 63;
  float a = 1e-3f * l, b = 2e-3f * l;
  floatx4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      if (KIND == 0)
        acc[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[i], 0, 0, 0);
      else
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int KIND, int NACC>
double time_rate(int waves_per_cu, int cus) {
  float* out;
  hipMalloc(&out, sizeof(float) * cus * 64 * waves_per_cu);
  const int iters = 4096;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  rate<KIND, NACC><<<cus, 64 * waves_per_cu>>>(out, 16);
  hipEventRecord(e0);
  rate<KIND, NACC><<<cus, 64 * waves_per_cu>>>(out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double flop_per = KIND == 0 ? 512.0 : 2048.0;
  const double flops = flop_per * 64.0 / 64.0 * iters * NACC * waves_per_cu * cus;  // per wave-instruction
  hipFree(out);
  return flops / (ms * 1e-3) / 1e12;
}

int main() {
  std::vector<float> A(64), B(64), O(256);
  for (int l = 0; l < 64; ++l) {
    A[l] = 1.f + l;          // distinct per lane
    B[l] = 1000.f * (l + 1);
  }
  float *dA, *dB, *dO;
  hipMalloc(&dA, 256);
  hipMalloc(&dB, 256);
  hipMalloc(&dO, 1024);
  hipMemcpy(dA, A.data(), 256, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), 256, hipMemcpyHostToDevice);
  layout<<<1, 64>>>(dO, dA, dB);
  hipMemcpy(O.data(), dO, 1024, hipMemcpyDeviceToHost);
  // decode each output as A[la] * B[lb] -> (la, lb)
  int ok = 1;
  printf("4x4x1_16b layout: lane l reg r = A[la]*B[lb]\n");
  for (int l = 0; l < 64; ++l) {
    for (int r = 0; r < 4; ++r) {
      const float v = O[l * 4 + r];
      int la = -1, lb = -1;
      for (int i = 0; i < 64 && la < 0; ++i)
        for (int j = 0; j < 64; ++j)
          if (A[i] * B[j] == v) { la = i; lb = j; break; }
      if (l < 8 || l >= 60) printf(" l%2d r%d: A[%2d] B[%2d]\n", l, r, la, lb);
      const int b = l / 4, col = l % 4;
      if (la != 4 * b + r || lb != 4 * b + col) ok = 0;
    }
  }
  printf("hypothesis D[block l/4][row r][col l%%4] = A[4b+r] * B[4b+col]: %s\n", ok ? "yes" : "NO");
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  printf("4x4x1_16b  1 acc, 4 w/CU: %.1f TF\n", time_rate<0, 1>(4, cus));
  printf("4x4x1_16b  2 acc, 4 w/CU: %.1f TF\n", time_rate<0, 2>(4, cus));
  printf("4x4x1_16b  4 acc, 4 w/CU: %.1f TF\n", time_rate<0, 4>(4, cus));
  printf("4x4x1_16b  2 acc, 8 w/CU: %.1f TF\n", time_rate<0, 2>(8, cus));
  printf("16x16x4    1 acc, 4 w/CU: %.1f TF\n", time_rate<1, 1>(4, cus));
  printf("16x16x4    2 acc, 4 w/CU: %.1f TF\n", time_rate<1, 2>(4, cus));
  printf("16x16x4    4 acc, 4 w/CU: %.1f TF\n", time_rate<1, 4>(4, cus));
  return 0;
}
