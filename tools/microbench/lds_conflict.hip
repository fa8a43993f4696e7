// Microbenchmark (round 5): what the SQ counters call a bank conflict for the
// scatter's 64-bit LDS atomics. Four address patterns of one wave-wide
// ds_add_u64 each, timed (CU-cycles per wave-instruction, s_memtime) and run
// once per pattern as its own kernel so that `rocprofv3 --pmc
// SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS` attributes the counters
// per pattern:
//   0 linear  - lane i -> cell base + i (64 consecutive 8-byte cells)
//   1 tap41   - lane (r, c) -> r * 41 + c, 8 x 8 taps (the round-1 microbench)
//   2 tap39   - lane (r, c) -> r * 39 + c (the W = 8 scatter's sub-grid pitch)
//   3 distinct - lane i -> cell (i mod 32) + 64 * (i / 32) * 17: every 32-lane
//                half on 32 distinct bank pairs (the bank-class order's goal)
//   4 random  - per-lane hashed cells in the sub-grid
// Build: hipcc -O3 --offload-arch=gfx950 lds_conflict.hip -o lds_conflict
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int NCELL = 39 * 39 * 2;
constexpr int ITERS = 256;

template <int PAT>
__global__ __launch_bounds__(256) void lds_pattern(unsigned long long* out, long long* cycles) {
  __shared__ unsigned long long sub[NCELL];
  for (int i = threadIdx.x; i < NCELL; i += 256) sub[i] = 0ull;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int cell;
  if constexpr (PAT == 0) cell = lane;
  if constexpr (PAT == 1) cell = (lane >> 3) * 41 + (lane & 7);
  if constexpr (PAT == 2) cell = (lane >> 3) * 39 + (lane & 7);
  if constexpr (PAT == 3) cell = (lane & 31) + (lane >> 5) * 64 * 17 % 1400;
  if constexpr (PAT == 4) {
    unsigned h = (unsigned)(blockIdx.x * 977 + threadIdx.x * 2654435761u);
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    cell = (int)(h % 1400u);
  }
  const long long t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    // 8 atomics per iteration, the base moving by whole multiples of 32 cells
    // (bank pairs unchanged), wave-uniform
    const int base = __builtin_amdgcn_readfirstlane((it * 7 + wave) % 4) * 32;
#pragma unroll
    for (int q = 0; q < 8; ++q) atomicAdd(&sub[base + q * 32 + cell], (unsigned long long)(it + q));
  }
  const long long t1 = clock64();
  __syncthreads();
  unsigned long long s = 0;
  for (int i = threadIdx.x; i < NCELL; i += 256) s += sub[i];
  atomicAdd(out, s);
  if (threadIdx.x == 0) atomicAdd((unsigned long long*)cycles, (unsigned long long)(t1 - t0));
}

int main() {
  const int nblk = 4096;
  unsigned long long* out;
  long long* cyc;
  CK(hipMalloc(&out, 8));
  CK(hipMalloc(&cyc, 8));
  const char* names[5] = {"linear", "tap41", "tap39", "distinct", "random"};
  for (int p = 0; p < 5; ++p) {
    CK(hipMemset(cyc, 0, 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    switch (p) {
      case 0: lds_pattern<0><<<nblk, 256>>>(out, cyc); break;
      case 1: lds_pattern<1><<<nblk, 256>>>(out, cyc); break;
      case 2: lds_pattern<2><<<nblk, 256>>>(out, cyc); break;
      case 3: lds_pattern<3><<<nblk, 256>>>(out, cyc); break;
      default: lds_pattern<4><<<nblk, 256>>>(out, cyc); break;
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    long long c = 0;
    CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
    const double winstr = (double)nblk * 4 * ITERS * 8;  // wave-level ds_add_u64
    // 256 CUs: CU-cycles per wave-instruction at the measured wall time (2.4 GHz)
    const double cu_cycles = ms * 1e-3 * 2.4e9 * 256 / winstr;
    printf("%-9s %8.3f ms  %6.2f CU-cycles per ds_add_u64 wave-instr (wall)  %8.1f clk64 per block-loop\n",
           names[p], ms, cu_cycles, (double)c / nblk);
  }
  return 0;
}
