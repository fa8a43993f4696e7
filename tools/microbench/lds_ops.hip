// Microbenchmark 2: per-wave-instruction cost of LDS operations relevant to the
// gridder scatter on gfx950: f64/u64/u32 atomics with k active lanes (tap-owned,
// conflict-free 8x8 addressing), broadcast reads (8 distinct addresses / wave),
// and wide writes. Reports CU-cycles per wave-instruction (4 waves/WG, 2048 WGs).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s @%d\n",hipGetErrorString(e),__LINE__);exit(1);}}while(0)
constexpr int PITCH = 41, ROWS = 41, NCELL = PITCH * ROWS;
constexpr int NV = 64;

template <int MODE, int ACTIVE>
__global__ __launch_bounds__(256) void k(const int* __restrict__ pos, int npos, int iters, double* out) {
  __shared__ double buf[2 * NCELL + 64];
  unsigned long long* ubuf = (unsigned long long*)buf;
  unsigned* u32 = (unsigned*)buf;
  for (int i = threadIdx.x; i < 2 * NCELL; i += 256) buf[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int off = (lane >> 3) * PITCH + (lane & 7);
  double a = threadIdx.x * 1e-3; double acc = 0;
  for (int it = 0; it < iters; ++it) {
    for (int v = 0; v < NV; ++v) {
      // register-only position hash (no memory latency in the loop)
      unsigned hsh = (unsigned)(blockIdx.x * 977 + wave * 131 + v * 2654435761u + it * 40503u);
      hsh ^= hsh >> 13; hsh *= 0x5bd1e995u; hsh ^= hsh >> 15;
      int p = (int)((hsh & 31) + ((hsh >> 5) % 33) * PITCH);
      p = __builtin_amdgcn_readfirstlane(p);
      if (lane < ACTIVE) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {   // 8 x 2 ops per hashed position: LDS-bound loop
          const int pq = p + q * 3;
          if constexpr (MODE == 0) { atomicAdd(&buf[pq + off], a); atomicAdd(&buf[NCELL + pq + off], a); }
          if constexpr (MODE == 1) { atomicAdd(&ubuf[pq + off], (unsigned long long)v); atomicAdd(&ubuf[NCELL + pq + off], (unsigned long long)v); }
          if constexpr (MODE == 2) { atomicAdd(&u32[pq + off], (unsigned)v); atomicAdd(&u32[2*NCELL + pq + off], (unsigned)v); }
          if constexpr (MODE == 3) { acc += buf[(pq & 1023) * 8 + (lane & 7)]; acc += buf[(pq & 1023) * 8 + 8 + (lane >> 3)]; }
          if constexpr (MODE == 4) { double2 t = ((double2*)buf)[(pq & 511) * 8 + (lane >> 3)]; acc += t.x; acc += t.y;
                                     double2 t2 = ((double2*)buf)[(pq & 511) * 8 + 64 + (lane & 7)]; acc += t2.x * t2.y; }
          if constexpr (MODE == 5) { buf[pq + off] = a + v; buf[NCELL + pq + off] = a - v; }
          if constexpr (MODE == 6) { ((double2*)buf)[(pq + off) % (NCELL - 64)] = make_double2(a + v, a - q); ((double2*)buf)[(pq + off + 41) % (NCELL - 64)] = make_double2(a - v, a + q); }
        }
      }
    }
  }
  __syncthreads();
  double s = acc;
  for (int i = threadIdx.x; i < 2 * NCELL; i += 256) s += buf[i];
  atomicAdd(out, s);
}

int main() {
  const int nblk = 2048, npos = 1 << 20, iters = 16;
  std::vector<int> h(npos); srand(1);
  for (auto& x : h) { int u = rand() % (PITCH - 8), v = rand() % (ROWS - 8); x = v * PITCH + u; }
  int* d; CK(hipMalloc(&d, npos * 4)); CK(hipMemcpy(d, h.data(), npos * 4, hipMemcpyHostToDevice));
  double* o; CK(hipMalloc(&o, 16));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  double ninstr = double(nblk) * 4 * iters * NV * 16;  // wave-instructions of the op under test
  auto run = [&](const char* name, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); for (int r = 0; r < 5; ++r) launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= 5;
    printf("%-34s %8.3f ms  %6.2f CU-cycles per wave-instr\n", name, ms, ms * 1e-3 * 2.4e9 * 256 / ninstr);
  };
#define R(M, A, N) run(N, [&] { k<M, A><<<nblk, 256>>>(d, npos, iters, o); })
  R(0, 64, "ds_add_f64 64 lanes"); R(0, 32, "ds_add_f64 32 lanes"); R(0, 16, "ds_add_f64 16 lanes"); R(0, 8, "ds_add_f64 8 lanes"); R(0, 1, "ds_add_f64 1 lane");
  R(1, 64, "ds_add_u64 64 lanes"); R(1, 8, "ds_add_u64 8 lanes");
  R(2, 64, "ds_add_u32 64 lanes");
  R(3, 64, "ds_read_b64 8-addr bcast x2");
  R(4, 64, "ds_read_b128 x2 8-addr bcast");
  R(5, 64, "ds_write_b64 x2");
  R(5, 8, "ds_write_b64 x2 8 lanes");
  R(6, 64, "ds_write_b128 x2");
  R(0, 64, "ds_add_f64 64 lanes (again)");
  return 0;
}
