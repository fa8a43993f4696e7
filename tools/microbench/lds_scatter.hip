// Microbenchmark 3: the scatter's LDS inner loop in isolation (u64 fixed-point
// atomics into separate re/im planes of a 39x39 sub-grid), per visibility:
//  A) lane-per-vis, random footprint origins      (current scatter)
//  B) lane-per-vis, origins with distinct bank class per 32 lanes (ORDER ideal)
//  C) tap-owned: 64 lanes = 64 taps of one visibility, + 2 broadcast LDS reads
// Reports CU-cycles per visibility (2.4 GHz nominal).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__);exit(1);}}while(0)
constexpr int P = 39, NC = P * P;

__device__ __forceinline__ unsigned hsh(unsigned x) { x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15; return x; }

template <int MODE>
__global__ __launch_bounds__(256) void k(int iters, unsigned long long* out) {
  __shared__ unsigned long long sub[2 * NC];
  __shared__ double stage[64 * 24];
  for (int i = threadIdx.x; i < 2 * NC; i += 256) sub[i] = 0;
  for (int i = threadIdx.x; i < 64 * 24; i += 256) stage[i] = i * 1e-3;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  unsigned long long a = threadIdx.x + 1;
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0 || MODE == 1) {
      unsigned h = hsh(blockIdx.x * 7919u + threadIdx.x * 2654435761u + it * 40503u);
      int lx = h & 31, ly = (h >> 5) & 31;
      if (MODE == 1) {  // force distinct classes (7 lx + ly) mod 32 == lane mod 32
        int want = lane & 31;
        ly = ((want - 7 * lx) % 32 + 32) % 32;
      }
      unsigned long long* b = sub + lx * P + ly;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          atomicAdd(b + i * P + j, a);
          atomicAdd(b + NC + i * P + j, a);
        }
    } else {  // tap-owned: 64 vis per iteration per wave
      const int off = (lane >> 3) * P + (lane & 7);
      for (int v = 0; v < 64; ++v) {
        unsigned h = hsh(blockIdx.x * 7919u + (threadIdx.x >> 6) * 131u + v * 2654435761u + it * 40503u);
        int p = __builtin_amdgcn_readfirstlane((int)((h & 31) * P + ((h >> 5) & 31)));
        double ku = stage[v * 24 + (lane & 7)];
        double2 kw = ((double2*)stage)[v * 12 + 4 + (lane >> 3)];
        unsigned long long x = (unsigned long long)__double_as_longlong(fma(ku, kw.x, 1.0));
        unsigned long long y = (unsigned long long)__double_as_longlong(fma(ku, kw.y, 1.0));
        atomicAdd(sub + p + off, x);
        atomicAdd(sub + NC + p + off, y);
      }
    }
  }
  __syncthreads();
  unsigned long long s = 0;
  for (int i = threadIdx.x; i < 2 * NC; i += 256) s += sub[i];
  atomicAdd(out, s);
}

int main() {
  const int nblk = 2048, iters = 16;
  unsigned long long* o; CK(hipMalloc(&o, 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch, double nvis) {
    launch(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); for (int r = 0; r < 5; ++r) launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
    printf("%-40s %8.3f ms %8.2f CU-cycles/vis\n", name, ms, ms * 1e-3 * 2.4e9 * 256 / nvis);
  };
  double nv = double(nblk) * 256 * iters;
  run("A lane-per-vis random", [&] { k<0><<<nblk, 256>>>(iters, o); }, nv);
  run("B lane-per-vis distinct class", [&] { k<1><<<nblk, 256>>>(iters, o); }, nv);
  run("C tap-owned + 2 bcast reads", [&] { k<2><<<nblk, 256>>>(iters / 4, o); }, double(nblk) * 4 * 64 * (iters / 4));
  return 0;
}
