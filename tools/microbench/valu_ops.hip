// Microbenchmark 4: issue cost on gfx950 of the grouped scatter's per-tap
// operations (cip_group.hip): v_fma_f64, the 64-bit integer accumulate
// (v_lshl_add_u64, and the v_add_co_u32 + v_addc_co_u32 pair it replaces),
// v_permlane32_swap_b32, and the fp64-accumulate alternative (fma into the
// accumulator). 8 independent chains per lane, 1024 blocks x 256 threads.
// Reports SIMD-cycles per wave-instruction at the measured clock.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#define CK(x)                                                        \
  do {                                                               \
    hipError_t e = (x);                                              \
    if (e != hipSuccess) {                                           \
      printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);       \
      exit(1);                                                       \
    }                                                                \
  } while (0)

constexpr int kUnroll = 16;

__global__ __launch_bounds__(256) void k_fma64(int iters, double* out) {
  double x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x * 1e-3 + i;
  const double m = 1.0000001, c = 1e-9;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int r = 0; r < kUnroll; ++r)
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] = fma(x[i], m, c);
  double s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  if (s == 1234.5) out[0] = s;
}

// fma to the magic constant + 64-bit add of its bits (the grouped tap)
__global__ __launch_bounds__(256) void k_fixed_tap(int iters, double* out) {
  unsigned long long acc[8];
  double a[8];
  for (int i = 0; i < 8; ++i) {
    acc[i] = i;
    a[i] = threadIdx.x * 1e-3 + i;
  }
  const double kv = 0.37;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int r = 0; r < kUnroll; ++r)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc[i] += (unsigned long long)__double_as_longlong(fma(a[i], kv, 6755399441055744.0));
        a[i] = __longlong_as_double((long long)(acc[i] & 0x000fffffffffffffull) | 0x3ff0000000000000ll);
      }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += (double)acc[i];
  if (s == 1234.5) out[0] = s;
}

// 64-bit adds only: v_lshl_add_u64 chains
__global__ __launch_bounds__(256) void k_add64(int iters, unsigned long long* out) {
  unsigned long long acc[8], b[8];
  for (int i = 0; i < 8; ++i) {
    acc[i] = i;
    b[i] = threadIdx.x * 977ull + i;
  }
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int r = 0; r < kUnroll; ++r)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc[i] += b[i];
        asm volatile("" : "+v"(acc[i]));
      }
  unsigned long long s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i];
  if (s == 1234) out[0] = s;
}

// 32-bit pair: v_add_co_u32 + v_addc_co_u32
__global__ __launch_bounds__(256) void k_add32pair(int iters, unsigned long long* out) {
  unsigned lo[8], hi[8], b[8];
  for (int i = 0; i < 8; ++i) {
    lo[i] = i;
    hi[i] = 0;
    b[i] = threadIdx.x * 977u + i;
  }
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int r = 0; r < kUnroll; ++r)
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, 0, vcc"
                                               : "+v"(lo[i]), "+v"(hi[i]) : "v"(b[i]) : "vcc");
  unsigned long long s = 0;
  for (int i = 0; i < 8; ++i) s += lo[i] + ((unsigned long long)hi[i] << 32);
  if (s == 1234) out[0] = s;
}

__global__ __launch_bounds__(256) void k_permlane(int iters, unsigned* out) {
  unsigned x[8];
  for (int i = 0; i < 8; ++i) x[i] = threadIdx.x + i;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int r = 0; r < kUnroll; ++r)
#pragma unroll
      for (int i = 0; i < 8; i += 2) {
        auto p = __builtin_amdgcn_permlane32_swap(x[i], x[i + 1], false, false);
        x[i] = p[0] + 1u;
        x[i + 1] = p[1];
      }
  unsigned s = 0;
  for (int i = 0; i < 8; ++i) s += x[i];
  if (s == 1234u) out[0] = s;
}

int main() {
  int dev = 0, clk_khz = 0, ncu = 0;
  CK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  double* d;
  CK(hipMalloc(&d, 64));
  const int iters = 2000, blocks = ncu * 8;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch, double ops_per_iter_lane) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double waves = (double)blocks * 4;
    const double instr = waves * iters * ops_per_iter_lane;   // wave-instructions
    const double simd_cycles = ms * 1e-3 * 2.4e9 * ncu * 4;   // at 2.4 GHz
    printf("%-28s %8.3f ms  %6.2f SIMD-cycles / wave-instr (2.4 GHz)\n", name, ms, simd_cycles / instr);
  };
  run("v_fma_f64", [&] { k_fma64<<<blocks, 256>>>(iters, d); }, kUnroll * 8);
  run("fma->magic + 64b add (tap)", [&] { k_fixed_tap<<<blocks, 256>>>(iters, d); }, kUnroll * 8 * 4);
  run("v_lshl_add_u64", [&] { k_add64<<<blocks, 256>>>(iters, (unsigned long long*)d); }, kUnroll * 8);
  run("v_add_co + v_addc pair", [&] { k_add32pair<<<blocks, 256>>>(iters, (unsigned long long*)d); },
      kUnroll * 8 * 2);
  run("v_permlane32_swap (+add)", [&] { k_permlane<<<blocks, 256>>>(iters, (unsigned*)d); }, kUnroll * 4 * 2);
  printf("clock attr %d kHz, %d CUs\n", clk_khz, ncu);
  return 0;
}
