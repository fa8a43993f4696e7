// cip_scatter_large.hip - the convolutional scatter for the large kernel
// supports W = 24, 32, 48, 64 (BASELINE.json configs[2], "support = 64, LDS-tile
// stress"): wave-per-visibility instead of the
// lane-per-visibility scatter of cip_scatter.h.
//
// Why a second design: with W^2 = 576..4096 taps per visibility a lane cannot
// hold its visibility's 2W kernel values and W^2 unrolled taps in registers,
// and the work per visibility is large enough to spread over a wave. A wave
// takes 64 consecutive stream positions, every lane places its own visibility
// (the same fp64 placement as the planner and cip_scatter.h), then the wave
// walks the valid ones: each lane owns footprint column j = lane % W (R = 64/W
// rows per instruction, R = 2 for W = 24 and 32), evaluates its kernel piece at
// the broadcast u and v offsets (the lane's piece coefficients stay in
// registers for the whole kernel), and adds rows i = 0..W-1 with ku[i] read
// from lane i (v_readlane: the row loop is wave-uniform). A row's 64 lanes
// touch consecutive LDS cells, so the ds_add_u64s are conflict-free by
// construction (no bank-class order needed) and the sub-grid is the same
// 64-bit fixed-point re/im pair of planes as the small scatter, (T + W - 1)^2
// cells (144 KiB at W = 64: one 1024-thread workgroup per CU). The flush is
// the small scatter's: non-zero cells added to the fp64 HBM grid with global
// atomics. Bound: LDS atomic bytes, 16 B per tap as for W <= 16.
//
// Compiled once per support with -DCIP_LARGE_W=W (Makefile), like
// cip_scatter_w.hip; launch_scatter_large (cip_grid.hip) dispatches on W.
#include "cip_scatter.h"

#ifndef CIP_LARGE_W
#error "compile with -DCIP_LARGE_W=<support>"
#endif

namespace cip {

constexpr int kLargeThreads = 1024;
constexpr int kLargeDeg = CIP_ES_DEGREE_64;  // every large support is fitted with this degree
static_assert(CIP_ES_DEGREE_24 == kLargeDeg && CIP_ES_DEGREE_32 == kLargeDeg && CIP_ES_DEGREE_48 == kLargeDeg,
              "large supports share one polynomial degree");

// coefficient d of piece k (k < W/2): a constexpr table indexed at run time
// (the lane's piece), which the compiler places in read-only global memory
template <int W>
struct LargeKernel;
#define CIP_LARGE_KERNEL(WW)                                                  \
  template <>                                                                 \
  struct LargeKernel<WW> {                                                    \
    __device__ static inline double coef(int k, int d) {                      \
      constexpr double c[WW / 2][kLargeDeg + 1] = CIP_ES_COEFFS_##WW;         \
      return c[k][d];                                                         \
    }                                                                         \
  };
CIP_LARGE_KERNEL(24)
CIP_LARGE_KERNEL(32)
CIP_LARGE_KERNEL(48)
CIP_LARGE_KERNEL(64)
#undef CIP_LARGE_KERNEL

__device__ __forceinline__ double lane_bcast(double x, int s) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)b, s);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), s);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

__device__ __forceinline__ double horner(const double* c, double y) {
  double r = c[kLargeDeg];
#pragma unroll
  for (int d = kLargeDeg - 1; d >= 0; --d) r = fma(r, y, c[d]);
  return r;
}

template <int W, typename VisT, int WK, bool WSTACK, bool PERM>
__global__ __launch_bounds__(kLargeThreads) void scatter_large_kernel(
    const double* __restrict__ uvw, const double* __restrict__ fx, const VisT* __restrict__ vis,
    const void* __restrict__ wgt, RowMap m, const uint64_t* __restrict__ runs, const int64_t* __restrict__ run_goff,
    const void* __restrict__ perm, const Chunk* __restrict__ chunks, int64_t chunk_begin, GridGeometry g,
    int64_t plane, double fixed_scale, double inv_scale, double* __restrict__ grid) {
  extern __shared__ unsigned long long sub[];  // re plane, then im plane: 2 P^2 cells
  constexpr int T = kTile;
  constexpr int R = 64 / W;  // footprint rows per wave instruction (2 for W = 24, 32; 1 for 48, 64)
  constexpr int P = T + W - 1, PP = P * P;
  const Chunk ch = chunks[chunk_begin + blockIdx.x];
  int64_t X0, Y0;
  tile_origin(ch.tile, g, &X0, &Y0);
  for (int i = threadIdx.x; i < 2 * PP; i += kLargeThreads) sub[i] = 0ull;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int tap = lane % W;  // footprint column of this lane
  const int ri = lane / W;   // row offset within an instruction's R rows
  const bool act = ri < R;
  const int piece = tap < W / 2 ? tap : W - 1 - tap;  // piece W-1-k (y) == piece k (-y)
  const double sgn = tap < W / 2 ? 1.0 : -1.0;
  double c[kLargeDeg + 1];
#pragma unroll
  for (int d = 0; d <= kLargeDeg; ++d) c[d] = LargeKernel<W>::coef(piece, d);
  __syncthreads();

  const bool unit_vis = vis == nullptr;
  const VisT* vis_ld = unit_vis ? (const VisT*)uvw : vis;
  for (int64_t q0 = ch.g0 + (int64_t)wave * 64; q0 < ch.g1; q0 += kLargeThreads) {
    const int64_t q = q0 + lane;
    const bool ok = q < ch.g1;
    uint64_t idx;  // ordered-stream entry (perm_encode form)
    if constexpr (PERM) {
      idx = perm_entry(perm, m, ok ? q : ch.g0);
    } else {
      // the chunk's row slices [first_run, last_run]: last slice starting at or before q
      const int64_t qq = ok ? q : ch.g0;
      int64_t lo = ch.first_run, hi = ch.last_run;
      while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (run_goff[mid] <= qq) lo = mid;
        else hi = mid - 1;
      }
      const uint64_t rec = runs[lo];
      idx = perm_encode(m, (int64_t)(rec >> 32), (int64_t)((rec >> 16) & 0xffff) + (qq - run_goff[lo]));
    }
    RawFetch<VisT, WK> raw;
    fetch_raw<VisT, WK>(idx, uvw, fx, vis_ld, unit_vis, wgt, m, raw);
    const VisFetch f = from_raw<VisT, WK>(raw, unit_vis);
    int64_t ix0, iy0, iw0;
    double yu, yv, yw;
    bool valid = place_vis(f.u, f.v, f.w, f.fx, g, &ix0, &yu, &iy0, &yv, &iw0, &yw);
    valid = valid && ok && f.wt != 0.0;
    const int64_t lx = ix0 - X0, ly = iy0 - Y0;
    valid = valid && lx >= 0 && lx < T && ly >= 0 && ly < T;  // always, for a consistent plan
    double sc = f.wt * fixed_scale;
    if constexpr (WSTACK) {
      const int64_t kw = plane - iw0;
      valid = valid && kw >= 0 && kw < W;
      const int kwc = valid ? (int)kw : 0;
      const int pw = kwc < W / 2 ? kwc : W - 1 - kwc;
      double cw[kLargeDeg + 1];
#pragma unroll
      for (int d = 0; d <= kLargeDeg; ++d) cw[d] = LargeKernel<W>::coef(pw, d);
      sc *= horner(cw, kwc < W / 2 ? yw : -yw);
    }
    const double vr = f.vr * sc, vi = f.vi * sc;
    const int lxi = (int)lx, lyi = (int)ly;
    uint64_t todo = __ballot(valid);
    while (todo) {
      const int s = __builtin_ctzll(todo);
      todo &= todo - 1;
      const int sx = __builtin_amdgcn_readlane(lxi, s), sy = __builtin_amdgcn_readlane(lyi, s);
      const double su = lane_bcast(yu, s), sv = lane_bcast(yv, s);
      const double svr = lane_bcast(vr, s), svi = lane_bcast(vi, s);
      const double ku = horner(c, sgn * su);  // lane `tap`: ku[tap]
      const double kv = horner(c, sgn * sv);  // kv[tap]
      const double kr = kv * svr, ki = kv * svi;
      unsigned long long* base = sub + ((sx + ri) * P + sy + tap);
      for (int i0 = 0; i0 < W; i0 += R) {
        double kui = lane_bcast(ku, i0);
        if constexpr (R == 2) {
          const double k1 = lane_bcast(ku, i0 + 1 < W ? i0 + 1 : i0);
          kui = ri ? k1 : kui;
        }
        if (act && i0 + ri < W) {
          const double qr = fma(kui, kr, kMagic);
          const double qi = fma(kui, ki, kMagic);
          atomicAdd(base + i0 * P, (unsigned long long)__double_as_longlong(qr) - 0x4338000000000000ull);
          atomicAdd(base + PP + i0 * P, (unsigned long long)__double_as_longlong(qi) - 0x4338000000000000ull);
        }
      }
    }
  }
  __shared__ unsigned s_wm;  // the tiles the flush writes (GridGeometry::wmask)
  if (threadIdx.x == 0) s_wm = 0u;
  __syncthreads();
  unsigned wm = 0u;
  for (int cell = threadIdx.x; cell < PP; cell += kLargeThreads) {
    const int lcell = g.transposed ? (cell % P) * P + cell / P : cell;  // lx * P + ly
    const long long re = (long long)sub[lcell];
    const long long im = (long long)sub[PP + lcell];
    if ((re | im) != 0) {
      int64_t gx = X0 + lcell / P, gy = Y0 + lcell % P;
      gx -= (gx >= g.nu) ? g.nu : 0;
      gy -= (gy >= g.nv) ? g.nv : 0;
      const int64_t off = grid_cell_offset(g, gx, gy);
      if (off < 0) {
        if (g.oob) atomicOr(g.oob, 1u);
        continue;
      }
      wm |= 1u << ((lcell / P / T) * 3 + (lcell % P) / T);
      double* dst = grid + 2 * off;
      unsafeAtomicAdd(dst, (double)re * inv_scale);
      unsafeAtomicAdd(dst + 1, (double)im * inv_scale);
    }
  }
  if (g.wmask) {
    if (wm) atomicOr(&s_wm, wm);
    __syncthreads();
    if (threadIdx.x == 0 && s_wm) wmask_report(g, plane, X0, Y0, s_wm);
  }
}

template <int W, typename VisT, int WK, bool WSTACK, bool PERM>
static hipError_t launch_large_one(dim3 gd, hipStream_t s, const double* uvw, const double* fx, const void* vis,
                                   const void* wgt, const RowMap& m, const uint64_t* runs, const int64_t* run_goff,
                                   const void* perm, const Chunk* chunks, int64_t cb, const GridGeometry& g,
                                   int64_t plane, double fs, double* grid) {
  constexpr int P = kTile + W - 1;
  constexpr size_t lds = (size_t)2 * P * P * sizeof(unsigned long long);
  static_assert(lds <= 160 * 1024, "sub-grid fits the CU's LDS");
  auto* fn = scatter_large_kernel<W, VisT, WK, WSTACK, PERM>;
  // more than the default 64 KiB of dynamic LDS (144 KiB at W = 64); set on
  // every launch (the attribute belongs to the current device's function, and
  // a host thread may drive several devices; a large-support launch runs for
  // milliseconds)
  const hipError_t e = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  fn<<<gd, dim3(kLargeThreads), lds, s>>>(uvw, fx, (const VisT*)vis, wgt, m, runs, run_goff, perm, chunks, cb, g,
                                          plane, fs, 1.0 / fs, grid);
  return hipGetLastError();
}

template <int W, typename VisT, int WK>
static hipError_t launch_large_vt(dim3 gd, hipStream_t s, const double* uvw, const double* fx, const void* vis,
                                  const void* wgt, const RowMap& m, const uint64_t* runs, const int64_t* run_goff,
                                  const void* perm, const Chunk* chunks, int64_t cb, const GridGeometry& g,
                                  int64_t plane, double fs, double* grid) {
#define ARGS gd, s, uvw, fx, vis, wgt, m, runs, run_goff, perm, chunks, cb, g, plane, fs, grid
  if (g.do_wstacking) {
    if (perm) return launch_large_one<W, VisT, WK, true, true>(ARGS);
    return launch_large_one<W, VisT, WK, true, false>(ARGS);
  }
  if (perm) return launch_large_one<W, VisT, WK, false, true>(ARGS);
  return launch_large_one<W, VisT, WK, false, false>(ARGS);
#undef ARGS
}

template <int W>
hipError_t launch_scatter_large_w(int vis_dtype, int wgt_dtype, dim3 gd, hipStream_t s, const double* uvw,
                                  const double* fx, const void* vis, const void* wgt, const RowMap& m,
                                  const uint64_t* runs, const int64_t* run_goff, const void* perm,
                                  const Chunk* chunks, int64_t cb, const GridGeometry& g, int64_t plane, double fs,
                                  double* grid) {
  if (g.support != W) return hipErrorInvalidValue;
#define ARGS gd, s, uvw, fx, vis, wgt, m, runs, run_goff, perm, chunks, cb, g, plane, fs, grid
  if (vis_dtype == CIP_POL4I) return launch_large_vt<W, Pol4, WK_POL4I>(ARGS);
  if (vis_dtype == CIP_C64) {
    if (wgt_dtype == CIP_F32) return launch_large_vt<W, float2, WK_F32>(ARGS);
    if (wgt_dtype == CIP_F64) return launch_large_vt<W, float2, WK_F64>(ARGS);
    return launch_large_vt<W, float2, WK_NONE>(ARGS);
  }
  if (wgt_dtype == CIP_F32) return launch_large_vt<W, double2, WK_F32>(ARGS);
  if (wgt_dtype == CIP_F64) return launch_large_vt<W, double2, WK_F64>(ARGS);
  return launch_large_vt<W, double2, WK_NONE>(ARGS);
#undef ARGS
}

template hipError_t launch_scatter_large_w<CIP_LARGE_W>(int, int, dim3, hipStream_t, const double*, const double*,
                                                        const void*, const void*, const RowMap&, const uint64_t*,
                                                        const int64_t*, const void*, const Chunk*, int64_t,
                                                        const GridGeometry&, int64_t, double, double*);

}  // namespace cip
