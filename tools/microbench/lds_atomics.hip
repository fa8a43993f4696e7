// Microbenchmark: LDS fp64/fp32 atomic-add throughput on gfx950 for the two
// scatter layouts considered for the gridder (see DESIGN.md "Scatter kernel").
//  A) "lane-per-vis": every lane owns one visibility and walks the 8x8 taps;
//     lane addresses are scattered over a (T+W+1)^2 sub-grid.
//  B) "tap-owned": the 64 lanes of a wave are the 64 taps of ONE visibility;
//     addresses are an 8x8 block -> conflict-free with a pitch == 8 mod 32.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__);exit(1);}}while(0)

constexpr int PITCH = 41;          // sub-grid pitch in cells (T=32, W=8 -> 41)
constexpr int ROWS  = 41;
constexpr int NCELL = PITCH*ROWS;

template <typename T>
__global__ __launch_bounds__(256) void lane_per_vis(const int* __restrict__ pos, int npos, int iters, T* out) {
  __shared__ T re[NCELL];
  __shared__ T im[NCELL];
  for (int i = threadIdx.x; i < NCELL; i += 256) { re[i] = 0; im[i] = 0; }
  __syncthreads();
  T a = (T)threadIdx.x * (T)1e-3;
  for (int it = 0; it < iters; ++it) {
    unsigned hsh = (unsigned)(blockIdx.x * 977 + threadIdx.x * 2654435761u + it * 40503u);
    hsh ^= hsh >> 13; hsh *= 0x5bd1e995u; hsh ^= hsh >> 15;
    int p = (int)((hsh & 31) + ((hsh >> 5) % 33) * PITCH);  // base cell of footprint
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        atomicAdd(&re[p + j * PITCH + i], a);
        atomicAdd(&im[p + j * PITCH + i], a);
      }
  }
  __syncthreads();
  T s = 0;
  for (int i = threadIdx.x; i < NCELL; i += 256) s += re[i] + im[i];
  atomicAdd(out, s);
}

template <typename T>
__global__ __launch_bounds__(256) void tap_owned(const int* __restrict__ pos, int npos, int iters, T* out) {
  __shared__ T re[NCELL];
  __shared__ T im[NCELL];
  for (int i = threadIdx.x; i < NCELL; i += 256) { re[i] = 0; im[i] = 0; }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int off = (lane >> 3) * PITCH + (lane & 7);
  T a = (T)threadIdx.x * (T)1e-3;
  // each wave handles 64 "visibilities" per outer iteration (same LDS op count as lane_per_vis)
  for (int it = 0; it < iters; ++it) {
    for (int v = 0; v < 64; ++v) {
      unsigned hsh = (unsigned)(blockIdx.x * 977 + wave * 131 + v * 2654435761u + it * 40503u);
      hsh ^= hsh >> 13; hsh *= 0x5bd1e995u; hsh ^= hsh >> 15;
      int p = (int)((hsh & 31) + ((hsh >> 5) % 33) * PITCH);
      p = __builtin_amdgcn_readfirstlane(p);
      atomicAdd(&re[p + off], a);
      atomicAdd(&im[p + off], a);
    }
  }
  __syncthreads();
  T s = 0;
  for (int i = threadIdx.x; i < NCELL; i += 256) s += re[i] + im[i];
  atomicAdd(out, s);
}

__global__ __launch_bounds__(256) void fma64(int iters, double* out) {
  double a = threadIdx.x, b = 1.0000001, c0 = 0.1, c1 = 0.2, c2 = 0.3, c3 = 0.4;
  for (int i = 0; i < iters; ++i) {
    c0 = fma(a, b, c0); c1 = fma(a, b, c1); c2 = fma(a, b, c2); c3 = fma(a, b, c3);
    c0 = fma(c1, b, c0); c1 = fma(c2, b, c1); c2 = fma(c3, b, c2); c3 = fma(c0, b, c3);
  }
  if (c0 + c1 + c2 + c3 == 1.2345) out[0] = c0;
}

int main() {
  const int nblk = 2048, npos = 1 << 20;
  std::vector<int> h(npos);
  srand(1);
  for (auto& x : h) { int u = rand() % (PITCH - 8), v = rand() % (ROWS - 8); x = v * PITCH + u; }
  int* d; CK(hipMalloc(&d, npos * 4)); CK(hipMemcpy(d, h.data(), npos * 4, hipMemcpyHostToDevice));
  double* o; CK(hipMalloc(&o, 16));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch, double nvis) {
    launch(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); for (int r = 0; r < 5; ++r) launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
    printf("%-28s %8.3f ms  %8.2f Gvis/s (64 taps, re+im)  %8.1f CU-cycles/vis @2.4GHz\n", name, ms, nvis / ms / 1e6,
           ms * 1e-3 * 2.4e9 * 256 / nvis);
  };
  int iters = 16;
  double nvis = double(nblk) * 256 * iters;
  run("lane_per_vis f64", [&] { lane_per_vis<double><<<nblk, 256>>>(d, npos, iters, o); }, nvis);
  run("tap_owned    f64", [&] { tap_owned<double><<<nblk, 256>>>(d, npos, iters, o); }, nvis);
  run("lane_per_vis f32", [&] { lane_per_vis<float><<<nblk, 256>>>(d, npos, iters, (float*)o); }, nvis);
  run("tap_owned    f32", [&] { tap_owned<float><<<nblk, 256>>>(d, npos, iters, (float*)o); }, nvis);
  int fi = 4096;
  run("fma64 (vis:=8 fma/thread)", [&] { fma64<<<nblk, 256>>>(fi, o); }, double(nblk) * 256 * fi);
  return 0;
}
