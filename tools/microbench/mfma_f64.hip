// Microbenchmark 3: issue rate of the fp64 matrix instruction on gfx950
// (v_mfma_f64_16x16x4_f64) against the f32-input form and fp64 VALU FMA,
// to price gridding a 16x16 cell block as a rank-4 update per instruction
// (DESIGN.md "Next"). Reports SIMD-cycles per instruction at 2.4 GHz and the
// chip-wide rate; also checks the C/D lane map with exact integers.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__);exit(1);}}while(0)

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void mfma64(int iters, double* out) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (d4){0, 0, 0, 0};
  double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 1234.5) out[0] = s;
}

template <int NACC>
__global__ __launch_bounds__(256) void mfma32(int iters, double* out) {
  f4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (f4){0, 0, 0, 0};
  float a = 1.0f + threadIdx.x * 1e-7f, b = 1.0f - threadIdx.x * 1e-7f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (s == 1234.5f) out[0] = s;
}

__global__ __launch_bounds__(256) void fma64(int iters, double* out) {
  double x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3 + i;
  const double m = 1.0000001, c = 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = fma(x[i], m, c);
  }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  if (s == 1234.5) out[0] = s;
}

// layout check: A[i][k] = i + 16k, B[k][j] = (k == 0) * (j + 1) + (k==1)*100
// -> C[i][j] = i * (j + 1) + 16 * 100 * ... computed on the host
__global__ void layout(double* out) {
  const int l = threadIdx.x;
  const int i = l & 15, k = l >> 4;
  const double a = (double)(i + 16 * k);
  const double b = (double)((k + 1) * 1000 + (l & 15));
  d4 acc = (d4){0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = acc[r];
}

int main() {
  double* o; CK(hipMalloc(&o, 64 * 4 * 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  // layout
  layout<<<1, 64>>>(o);
  double h[256]; CK(hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost));
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int r = 0; r < 4; ++r) {
      const int col = l & 15, row = (l >> 4) + 4 * r;
      double ref = 0;
      for (int k = 0; k < 4; ++k) ref += (double)(row + 16 * k) * (double)((k + 1) * 1000 + col);
      if (ref != h[l * 4 + r]) ++bad;
    }
  printf("f64 16x16x4 C/D map col=lane&15 row=(lane>>4)+4r: %s (%d mismatches)\n", bad ? "WRONG" : "ok", bad);
  const int nblk = 1024 * 4, iters = 2000;
  auto run = [&](const char* name, double ops_per_thread_iter, double flop_per_op, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); for (int r = 0; r < 3; ++r) launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 3;
    const double waves = nblk * 4.0;
    const double instr = waves * iters * ops_per_thread_iter;  // wave-instructions
    const double simd_cycles = ms * 1e-3 * 2.4e9 * 1024;        // 256 CUs x 4 SIMDs
    printf("%-36s %8.3f ms  %6.2f SIMD-cycles/instr  %7.1f TFLOP/s\n", name, ms, simd_cycles / instr,
           instr * flop_per_op / (ms * 1e-3) / 1e12);
  };
  run("mfma_f64_16x16x4 1 acc", 1, 2048, [&] { mfma64<1><<<nblk, 256>>>(iters, o); });
  run("mfma_f64_16x16x4 4 acc", 4, 2048, [&] { mfma64<4><<<nblk, 256>>>(iters, o); });
  run("mfma_f64_16x16x4 8 acc", 8, 2048, [&] { mfma64<8><<<nblk, 256>>>(iters, o); });
  run("mfma_f32_16x16x4 4 acc", 4, 2048, [&] { mfma32<4><<<nblk, 256>>>(iters, o); });
  run("v_fma_f64 x32", 32, 128, [&] { fma64<<<nblk, 256>>>(iters, o); });
  return 0;
}
