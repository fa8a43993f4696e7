// EXPERIMENT (not part of libcip_hip.so): the time-track scatter of the
// round-3 verdict, Romein-style, for the 2-D W = 8 fp64
// class - built to measure it against the lane kernel (cip_scatter.h) on the
// bench's C3 data (tools/timetrack/run_timetrack.py).
//
// A (baseline, channel) track in MS time order moves its footprint origin by
// at most one cell per 8-s dump on C3, so the W x W = 64 lanes of a wave own
// the 64 cell residues (x mod 8, y mod 8) of one track segment (its samples
// inside one 32 x 32 tile): lane (a, b) owns the footprint cell with
// x = a, y = b (mod 8) and accumulates that cell's fixed-point contributions
// in registers; only when a sample's origin moves does the lane whose cell
// leaves the footprint add its sum to the LDS sub-grid (ds_add_u64). Kernel
// values: the samples of a segment are placed 8 at a time, lane (s, i)
// evaluating piece i of sample s on both axes with per-lane coefficients
// (no coefficient selection per sample), staged in the wave's LDS scratch;
// each lane then reads its two values per sample. The fixed-point integers
// are exactly the lane kernel's (same placement, products and roundings), so
// the grids agree to the fp64 flush order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cip_common.h"

using namespace cip;

namespace {

constexpr int W = 8;
constexpr int T = kTile;
constexpr int P = T + W - 1;
constexpr int HW = W / 2;
constexpr int D = CIP_ES_DEGREE_8;
static_assert(D % 2 == 1, "odd degree assumed (even part D - 1, odd part D)");
constexpr int NE = (D + 1) / 2;  // even coefficients c[0], c[2], .., c[D - 1]
constexpr int NO = (D + 1) / 2;  // odd coefficients c[1], .., c[D]
constexpr int kWaves = 4;
constexpr unsigned long long kMagicBits = 0x4338000000000000ull;

__constant__ double kCoef[W / 2][D + 1] = CIP_ES_COEFFS_8;

struct WaveScratch {
  double ku[8][8];  // [sample][piece]
  double kv[8][8];
  double vr[8], vi[8];
  int lx[8], ly[8];
};

__device__ __forceinline__ void flush_cell(unsigned long long* sub, int cell, unsigned long long ar,
                                           unsigned long long ai, unsigned cnt) {
  const unsigned long long off = (unsigned long long)cnt * kMagicBits;
  atomicAdd(sub + cell, ar - off);
  atomicAdd(sub + P * P + cell, ai - off);
}

__global__ __launch_bounds__(64 * kWaves) void timetrack_kernel(
    const double* __restrict__ uvw, const double* __restrict__ fx, const float2* __restrict__ vis,
    const float* __restrict__ wgt, int64_t nchan, int64_t nbl, const int32_t* __restrict__ seg_b,
    const int32_t* __restrict__ seg_c, const int32_t* __restrict__ seg_t0, const int32_t* __restrict__ seg_t1,
    const int64_t* __restrict__ unit_s0, const int64_t* __restrict__ unit_s1, const int32_t* __restrict__ unit_tx,
    const int32_t* __restrict__ unit_ty, int64_t nu, int64_t nv, double su, double sv, double fixed_scale,
    double* __restrict__ grid, unsigned* __restrict__ err) {
#pragma clang fp contract(off)
  __shared__ unsigned long long sub[2 * P * P];
  __shared__ WaveScratch scr[kWaves];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  WaveScratch& ws = scr[wv];
  const int64_t u = blockIdx.x;
  const int64_t X0 = (int64_t)unit_tx[u] * T, Y0 = (int64_t)unit_ty[u] * T;
  for (int i = threadIdx.x; i < 2 * P * P; i += 64 * kWaves) sub[i] = 0ull;
  // lane (s, i) of a placement batch: piece i (mirrored for i >= W / 2)
  const int s = lane >> 3, pi = lane & 7;
  const int pk = pi < HW ? pi : W - 1 - pi;
  const double psign = pi < HW ? 1.0 : -1.0;
  double ce[NE], co[NO];
#pragma unroll
  for (int k = 0; k < NE; ++k) ce[k] = kCoef[pk][2 * k];
#pragma unroll
  for (int k = 0; k < NO; ++k) co[k] = kCoef[pk][2 * k + 1];
  // residue lane (a, b): footprint cell x = a, y = b (mod 8)
  const int ra = lane >> 3, rb = lane & 7;
  __syncthreads();
  const int64_t s1 = unit_s1[u];
  for (int64_t sg = unit_s0[u] + wv; sg < s1; sg += kWaves) {
    const int64_t b = seg_b[sg], c = seg_c[sg];
    const int t0 = seg_t0[sg], n = seg_t1[sg] - t0;
    const double f = fx[c];
    int cur = -1;
    unsigned long long ar = 0ull, ai = 0ull;
    unsigned cnt = 0u;
    for (int base = 0; base < n; base += 8) {
      // place sample s of the batch and evaluate piece pi on both axes
      const int ts = t0 + base + (base + s < n ? s : 0);
      const int64_t r = (int64_t)ts * nbl + b;
      const double x = (uvw[3 * r] * f) * su + (double)(nu / 2);
      const double y = (uvw[3 * r + 1] * f) * sv + (double)(nv / 2);
      const double sx = x - (double)HW, sy = y - (double)HW;
      const double flx = floor(sx), fly = floor(sy);
      const double yu = 2.0 * (sx - flx) - 1.0, yv = 2.0 * (sy - fly) - 1.0;
      int ix0 = (int)flx + 1, iy0 = (int)fly + 1;
      ix0 += ix0 < 0 ? (int)nu : 0;
      ix0 -= ix0 >= (int)nu ? (int)nu : 0;
      iy0 += iy0 < 0 ? (int)nv : 0;
      iy0 -= iy0 >= (int)nv ? (int)nv : 0;
      const double zu = yu * yu, zv = yv * yv;
      double eu = ce[NE - 1], ou = co[NO - 1], ev = ce[NE - 1], ov = co[NO - 1];
#pragma unroll
      for (int k = NE - 2; k >= 0; --k) {
        eu = fma(eu, zu, ce[k]);
        ev = fma(ev, zv, ce[k]);
      }
#pragma unroll
      for (int k = NO - 2; k >= 0; --k) {
        ou = fma(ou, zu, co[k]);
        ov = fma(ov, zv, co[k]);
      }
      ws.ku[s][pi] = fma(psign * yu, ou, eu);
      ws.kv[s][pi] = fma(psign * yv, ov, ev);
      if (pi == 0) {
        const int64_t iv = r * nchan + c;
        const float2 vv = vis[iv];
        const double sc = (double)wgt[iv] * fixed_scale;
        ws.vr[s] = (double)vv.x * sc;
        ws.vi[s] = (double)vv.y * sc;
        const int lx = (int)(ix0 - X0), ly = (int)(iy0 - Y0);
        if (base + s < n && (lx < 0 || lx >= T || ly < 0 || ly >= T)) atomicOr(err, 1u);
        ws.lx[s] = lx;
        ws.ly[s] = ly;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int nb = n - base < 8 ? n - base : 8;
      for (int q = 0; q < nb; ++q) {
        const int lx = ws.lx[q], ly = ws.ly[q];
        if ((unsigned)lx >= (unsigned)T || (unsigned)ly >= (unsigned)T) continue;  // inconsistent plan
        const int du = (ra - lx) & 7, dv = (rb - ly) & 7;
        const int cell = (lx + du) * P + (ly + dv);
        if (cell != cur) {
          if (cur >= 0) flush_cell(sub, cur, ar, ai, cnt);
          cur = cell;
          ar = ai = 0ull;
          cnt = 0u;
        }
        const double ku = ws.ku[q][du], kv = ws.kv[q][dv];
        const double kr = kv * ws.vr[q], ki = kv * ws.vi[q];
        ar += (unsigned long long)__double_as_longlong(fma(ku, kr, kMagic));
        ai += (unsigned long long)__double_as_longlong(fma(ku, ki, kMagic));
        ++cnt;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (cur >= 0) flush_cell(sub, cur, ar, ai, cnt);
  }
  __syncthreads();
  // the lane kernel's flush: touched cells added to the fp64 grid (gT[y][x])
  const double inv_scale = 1.0 / fixed_scale;
  for (int cell = threadIdx.x; cell < P * P; cell += 64 * kWaves) {
    const int lcell = (cell % P) * P + cell / P;  // lanes walk x (the grid's contiguous axis)
    const long long re = (long long)sub[lcell], im = (long long)sub[P * P + lcell];
    if ((re | im) != 0) {
      int64_t gx = X0 + lcell / P, gy = Y0 + lcell % P;
      gx -= gx >= nu ? nu : 0;
      gy -= gy >= nv ? nv : 0;
      double* dst = grid + 2 * (gy * nu + gx);
      unsafeAtomicAdd(dst, (double)re * inv_scale);
      unsafeAtomicAdd(dst + 1, (double)im * inv_scale);
    }
  }
}

}  // namespace

extern "C" int tt_grid(const double* uvw, const double* fx, const void* vis, const float* wgt, int64_t nchan,
                       int64_t nbl, const int32_t* seg_b, const int32_t* seg_c, const int32_t* seg_t0,
                       const int32_t* seg_t1, const int64_t* unit_s0, const int64_t* unit_s1,
                       const int32_t* unit_tx, const int32_t* unit_ty, int64_t nunits, int64_t nu, int64_t nv,
                       double su, double sv, double fixed_scale, double* grid, unsigned* err, void* stream) {
  if (nunits <= 0) return 0;
  if (nu >= (1ll << 30) || nv >= (1ll << 30)) return 1;
  timetrack_kernel<<<dim3((unsigned)nunits), dim3(64 * kWaves), 0, (hipStream_t)stream>>>(
      uvw, fx, (const float2*)vis, wgt, nchan, nbl, seg_b, seg_c, seg_t0, seg_t1, unit_s0, unit_s1, unit_tx,
      unit_ty, nu, nv, su, sv, fixed_scale, grid, err);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
