// cip_common.h - shared device/host definitions of libcip_hip.so (gfx950).
//
// Geometry conventions (identical in oracle/cip_oracle.c):
//   grid cell ix in [0, nu) <-> u = (ix - nu/2) du,  du = 1 / (nu * pixsize_x)
//   a visibility at u_lambda = u_m * f / c sits at x = u_lambda * nu * pixsize_x + nu/2
//   footprint ix0 = floor(x - W/2) + 1 .. ix0 + W - 1, kernel piece k at
//   y = 2 frac(x - W/2) - 1 (pieces k >= W/2 by symmetry: phi_{W-1-k}(y) = phi_k(-y)).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "es_kernels.h"

#define CIP_SPEED_OF_LIGHT 299792458.0

namespace cip {

// Fixed-point accumulation: contributions are scaled by 2^S so the largest
// |w * V| maps to <= 2^46, rounded to integers by adding 1.5 * 2^52 (one
// correctly-rounded fma) and accumulated with 64-bit integer LDS atomics
// (ds_add_u64: 8 CU-cycles/wave-instruction vs 16 for ds_add_f64 measured on
// gfx950, tools/microbench/lds_ops.hip). Integer sums are exact and
// order-independent; a chunk holds <= kChunkVis visibilities so a cell sum
// stays below 2^60.
constexpr double kMagic = 6755399441055744.0;  // 1.5 * 2^52
constexpr uint32_t kMagicHi = 0x43380000u;      // high word of kMagic
constexpr int kFixedBits = 46;
constexpr int64_t kChunkVis = 16384;  // 16384 vs 32768: 2 % less scatter tail at C3 (tools/sweep_cv.sh)

// Packed single-precision class (complex64 input, ducc0's float gridding):
// (re, im) of a cell share ONE 64-bit integer, re * 2^32 + im, so a
// visibility costs W^2 LDS atomics instead of 2 W^2. Both halves must stay
// within +-2^31 per chunk: a chunk of n <= kChunkVisPacked visibilities is
// scaled so its largest contribution maps to 2^(kPackedBits + lg(kChunkVisPacked)
// - ceil(lg n)) (<= 2^30 / n). Quantisation is <= 2^-19 of max|wV| per
// contribution, finer than the float32 grid of the reference's gridder.
constexpr int kPackedBits = 18;
constexpr int64_t kChunkVisPacked = 4096;
constexpr int kChunkVisPackedLog2 = 12;
// The packed class rounds each tap in fp32 (cip_scatter.h packed_tap): an fma
// against 1.5 * 2^23 is an exact integer rounding for |x| < 2^22, so a short
// chunk's gain over the base scale (contributions < 2^18) is capped at 2^3.
constexpr float kMagicF = 12582912.0f;  // 1.5 * 2^23
constexpr uint32_t kMagicFBits = 0x4B400000u;
constexpr int kPackedGainLog2Max = 3;

// Tile edge (grid cells) of the scatter work decomposition (CIP_TILE
// overrides it in experiment builds, tools/build_variant_full.sh).
#ifndef CIP_TILE
#define CIP_TILE 32
#endif
constexpr int kTile = CIP_TILE;

// Visibilities per bank-class ordering window (cip_grid.hip order_kernel);
// divides kChunkVis and kChunkVisPacked so, in 2-D mode, windows never
// straddle chunks (w-stacking work units start at the first layer of their
// merged range, not at a window boundary: there a chunk boundary may fall
// inside a window, which is harmless because perm maps every position to a
// visibility of the same uv tile, but the invariant does not hold).
#ifndef CIP_ORDER_WINDOW
#define CIP_ORDER_WINDOW 1024  // experiment builds: 2048 (tools/build_variant_all.sh)
#endif
constexpr int kOrderWindow = CIP_ORDER_WINDOW;

__host__ __device__ inline int64_t floor_div(int64_t a, int64_t b) {
  int64_t q = a / b;
  return (q * b > a) ? q - 1 : q;
}

// Horner evaluation of the even/odd halves of piece k at z = y^2.
template <int W>
struct EsKernel;

#define CIP_DEFINE_KERNEL(WW)                                                  \
  template <>                                                                  \
  struct EsKernel<WW> {                                                        \
    static constexpr int W = WW;                                               \
    static constexpr int D = CIP_ES_DEGREE_##WW;                               \
    __device__ static inline double coef(int k, int d) {                       \
      constexpr double c[WW / 2][CIP_ES_DEGREE_##WW + 1] = CIP_ES_COEFFS_##WW; \
      return c[k][d];                                                          \
    }                                                                          \
  };
CIP_DEFINE_KERNEL(4)
CIP_DEFINE_KERNEL(6)
CIP_DEFINE_KERNEL(8)
CIP_DEFINE_KERNEL(10)
CIP_DEFINE_KERNEL(12)
CIP_DEFINE_KERNEL(14)
CIP_DEFINE_KERNEL(16)
#undef CIP_DEFINE_KERNEL

// A kernel coefficient materialised in an SGPR pair at its point of use. The
// empty volatile asm stops the compiler from hoisting all (W/2)(D+1)
// coefficients out of the scatter loop, which needs more than the 102 SGPRs
// and spills them to VGPR lanes (v_readlane per use); two s_mov_b32 per use
// issue on the scalar pipe beside the VALU instead.
__device__ __forceinline__ double sgpr_const(double c) {
  asm volatile("" : "+s"(c));
  return c;
}

// All W kernel values at y in [-1, 1): out[k] = phi_k(y).
template <int W>
__device__ __forceinline__ void eval_kernel(double y, double* out) {
  using K = EsKernel<W>;
  const double z = y * y;
#pragma unroll
  for (int k = 0; k < W / 2; ++k) {
    // even part: sum_m c[2m] z^m ; odd part: sum_m c[2m+1] z^m
    constexpr int D = K::D;
    double e = sgpr_const(K::coef(k, (D & 1) ? D - 1 : D));
#pragma unroll
    for (int d = ((D & 1) ? D - 1 : D) - 2; d >= 0; d -= 2) e = fma(e, z, sgpr_const(K::coef(k, d)));
    double o = sgpr_const(K::coef(k, (D & 1) ? D : D - 1));
#pragma unroll
    for (int d = ((D & 1) ? D : D - 1) - 2; d >= 1; d -= 2) o = fma(o, z, sgpr_const(K::coef(k, d)));
    out[k] = fma(y, o, e);
    out[W - 1 - k] = fma(-y, o, e);
  }
}

// The mirrored pieces k and W - 1 - k at y (z = y^2): out[0] = phi_k(y),
// out[1] = phi_{W-1-k}(y) - eval_kernel's values, one pair at a time.
template <int W>
__device__ __forceinline__ void eval_piece_pair(int k, double y, double z, double* out) {
  using K = EsKernel<W>;
  constexpr int D = K::D;
  double e = sgpr_const(K::coef(k, (D & 1) ? D - 1 : D));
#pragma unroll
  for (int d = ((D & 1) ? D - 1 : D) - 2; d >= 0; d -= 2) e = fma(e, z, sgpr_const(K::coef(k, d)));
  double o = sgpr_const(K::coef(k, (D & 1) ? D : D - 1));
#pragma unroll
  for (int d = ((D & 1) ? D : D - 1) - 2; d >= 1; d -= 2) o = fma(o, z, sgpr_const(K::coef(k, d)));
  out[0] = fma(y, o, e);
  out[1] = fma(-y, o, e);
}

// All W kernel values at y in [-1, 1) in fp32 (the packed class): the same
// polynomial pieces, coefficients rounded to float.
__device__ __forceinline__ float sgpr_constf(float c) {
  asm volatile("" : "+s"(c));
  return c;
}
template <int W>
__device__ __forceinline__ void eval_kernel_f32(float y, float* out) {
  using K = EsKernel<W>;
  const float z = y * y;
#pragma unroll
  for (int k = 0; k < W / 2; ++k) {
    constexpr int D = K::D;
    float e = sgpr_constf((float)K::coef(k, (D & 1) ? D - 1 : D));
#pragma unroll
    for (int d = ((D & 1) ? D - 1 : D) - 2; d >= 0; d -= 2) e = fmaf(e, z, sgpr_constf((float)K::coef(k, d)));
    float o = sgpr_constf((float)K::coef(k, (D & 1) ? D : D - 1));
#pragma unroll
    for (int d = ((D & 1) ? D : D - 1) - 2; d >= 1; d -= 2) o = fmaf(o, z, sgpr_constf((float)K::coef(k, d)));
    out[k] = fmaf(y, o, e);
    out[W - 1 - k] = fmaf(-y, o, e);
  }
}

// The u and v kernels of one visibility at once (the packed class): both axes
// share the polynomial pieces, so each Horner step is one v_pk_fma_f32 on
// (u, v) against the broadcast coefficient - half the VALU issue of two
// eval_kernel_f32 calls, the same fp32 values.
typedef float cip_f32x2 __attribute__((ext_vector_type(2)));
template <int W>
__device__ __forceinline__ void eval_kernel_f32x2(cip_f32x2 y, cip_f32x2* out) {
  using K = EsKernel<W>;
  const cip_f32x2 z = y * y;
#pragma unroll
  for (int k = 0; k < W / 2; ++k) {
    constexpr int D = K::D;
    float c = sgpr_constf((float)K::coef(k, (D & 1) ? D - 1 : D));
    cip_f32x2 e{c, c};
#pragma unroll
    for (int d = ((D & 1) ? D - 1 : D) - 2; d >= 0; d -= 2) {
      c = sgpr_constf((float)K::coef(k, d));
      e = __builtin_elementwise_fma(e, z, cip_f32x2{c, c});
    }
    c = sgpr_constf((float)K::coef(k, (D & 1) ? D : D - 1));
    cip_f32x2 o{c, c};
#pragma unroll
    for (int d = ((D & 1) ? D : D - 1) - 2; d >= 1; d -= 2) {
      c = sgpr_constf((float)K::coef(k, d));
      o = __builtin_elementwise_fma(o, z, cip_f32x2{c, c});
    }
    out[k] = __builtin_elementwise_fma(y, o, e);
    out[W - 1 - k] = __builtin_elementwise_fma(-y, o, e);
  }
}

// Scale of a packed chunk of n visibilities relative to the launch's base
// scale (which assumes n = kChunkVisPacked): 2^min(12 - ceil(lg n), 3), exact
// (the cap keeps every contribution below 2^22, the fp32 rounding's range;
// sums stay below 2^30 either way).
__host__ __device__ inline double packed_chunk_gain(int64_t n) {
  int lg = 0;
  while (((int64_t)1 << lg) < n) ++lg;
  int e = kChunkVisPackedLog2 - (lg < kChunkVisPackedLog2 ? lg : kChunkVisPackedLog2);
  e = e < kPackedGainLog2Max ? e : kPackedGainLog2Max;
  return (double)((int64_t)1 << e);
}

// A gridding work unit: the flattened visibilities [g0, g1) of tile `tile`
// (global indices into the tile-sorted visibility stream).
struct Chunk {
  int64_t g0, g1;
  int64_t tile;
  int64_t first_run;  // first row slice of the tile overlapping [g0, g1)
  int64_t last_run;   // last row slice overlapping [g0, g1)
  int64_t sole;       // 1: the only work unit of its tile (and plane group) - its private cells
                      // have no other writer in the launch (scatter flush, cip_scatter.h)
};

// Everything the planner and the scatter need to place a visibility.
struct GridGeometry {
  int64_t nu, nv;
  int support;
  double scale_u, scale_v;  // nu * pixsize_x, nv * pixsize_y
  int do_wstacking;
  double w0, dw;
  double inv_dw;  // 1 / dw: the w coordinate (w f / c - w0) / dw as one multiply (planner, scatter, oracle alike)
  int64_t nplanes;
  int tile;                 // T
  int64_t ntx, nty, ntw;    // tiles per axis (ntw = nplanes - W + 1, or 1 in 2-D)
  int transposed;           // HBM grid stored as gT[y, x] (pruned FFT), else g[x, y]
  // row window of the HBM buffer (transposed layout; uv-strip ranks, DESIGN.md
  // 7): buffer row k holds grid row (row0 + k) mod nv, k < rows. The whole
  // grid: row0 = 0, rows = nv. A flushed cell outside the window is dropped
  // and sets *oob (if given) - a plan inconsistent with the strip.
  int64_t row0, rows;
  unsigned* oob;
  // w planes this call grids (w-stacking plane groups split over GPUs,
  // cip_ms2dirty_wplanes): [plane_lo, plane_hi); the whole stack by default.
  // The planner drops visibilities feeding no plane of the range.
  int64_t plane_lo, plane_hi;
  // HBM grid planes of complex64 (float re, im) instead of complex128: the
  // packed single class's own planes on the pruned-FFT path (cip_ms2dirty),
  // half the flush and pass-A bytes (ducc0's float class grids in float32)
  int grid_f32;
  // written-tile mask (optional, zeroed by the caller): the scatter's flush
  // sets bit tx % 32 of word [p][ty][tx / 32] for every 32 x 32 tile (tx, ty)
  // of plane p it writes a cell of - the exact dirty tiles of the gridded
  // planes (the uv-strip ranks' masked pass A, cip_grid_tiles_strip_mask)
  uint32_t* wmask;
};

// The flush's report to GridGeometry::wmask: `bits` = the tiles of one work
// unit's sub-grid its flush wrote, bit dx * 3 + dy for tile (X0 / T + dx,
// Y0 / T + dy) (wrapped; dx, dy <= 2: the sub-grid spans T + W - 1 <= 95
// cells), plane p. A handful of device atomics per work unit.
__device__ __forceinline__ void wmask_report(const GridGeometry& g, int64_t p, int64_t X0, int64_t Y0,
                                             unsigned bits) {
  const int64_t tx0 = X0 / kTile, ty0 = Y0 / kTile;
  const int64_t wpr = g.ntx / 32;
  uint32_t* m = g.wmask + p * g.nty * wpr;
  while (bits) {
    const int b = __builtin_ctz(bits);
    bits &= bits - 1u;
    int64_t tx = tx0 + b / 3, ty = ty0 + b % 3;
    tx -= tx >= g.ntx ? g.ntx : 0;
    ty -= ty >= g.nty ? g.nty : 0;
    atomicOr(m + ty * wpr + tx / 32, 1u << (unsigned)(tx % 32));
  }
}

// Buffer offset (complex cells) of grid cell (gx, gy) in wrapped coordinates,
// or -1 outside the buffer's row window.
__device__ __forceinline__ int64_t grid_cell_offset(const GridGeometry& g, int64_t gx, int64_t gy) {
  if (!g.transposed) return gx * g.nv + gy;
  int64_t k = gy - g.row0;
  k += (k < 0) ? g.nv : 0;
  return k < g.rows ? k * g.nu + gx : -1;
}

// Grid coordinate -> footprint origin and kernel variable.
__device__ __forceinline__ void footprint(double x, int half_w, int64_t* i0, double* y) {
  const double s = x - (double)half_w;
  const double fl = floor(s);
  *i0 = (int64_t)fl + 1;
  *y = 2.0 * (s - fl) - 1.0;
}

// i mod n in [0, n): one compare-and-add for |i| < 2n (all but absurd
// coordinates), the 64-bit remainder only beyond that.
__device__ __forceinline__ int64_t wrap_index(int64_t i, int64_t n) {
  if (i >= n) {
    i -= n;
    if (i >= n) i %= n;
  } else if (i < 0) {
    i += n;
    if (i < 0) i = ((i % n) + n) % n;
  }
  return i;
}

__device__ __forceinline__ int wrap_index32(int i, int n) {
  if (i >= n) {
    i -= n;
    if (i >= n) i %= n;
  } else if (i < 0) {
    i += n;
    if (i < 0) {
      i %= n;
      if (i < 0) i += n;
    }
  }
  return i;
}

// Footprint origins (ix0, iy0) of grid coordinates (x, y), wrapped into
// [0, nu) x [0, nv), and the kernel variables. 32-bit integer arithmetic (one
// v_cvt_i32_f64 per axis; the f64 -> i64 conversion and 64-bit wrap are a
// dozen VALU instructions each); a wave-uniform branch takes the 64-bit path
// when any active lane is 2^30 cells or more from the origin (or not finite).
// The same integers either way.
__device__ __forceinline__ void uv_origin(double x, double y, int hw, const GridGeometry& g, int64_t* ix0,
                                          double* yu, int64_t* iy0, double* yv) {
#pragma clang fp contract(off)
  const double sx = x - (double)hw, sy = y - (double)hw;
  const double flx = floor(sx), fly = floor(sy);
  *yu = 2.0 * (sx - flx) - 1.0;
  *yv = 2.0 * (sy - fly) - 1.0;
  const bool small = fabs(flx) < 1073741824.0 && fabs(fly) < 1073741824.0;
  if (__ballot(!small) == 0ull) {
    *ix0 = wrap_index32((int)flx + 1, (int)g.nu);
    *iy0 = wrap_index32((int)fly + 1, (int)g.nv);
  } else {
    *ix0 = wrap_index(small || isfinite(flx) ? (int64_t)flx + 1 : 0, g.nu);
    *iy0 = wrap_index(small || isfinite(fly) ? (int64_t)fly + 1 : 0, g.nv);
  }
}

// Place one visibility (metres, fx = f / c) on the grid. Returns false when the
// footprint leaves the grid (or the w-plane stack). The arithmetic order is
// pinned (no contraction) so the planner and the scatter agree bit for bit and
// oracle/cip_oracle.c reproduces it.
__device__ __forceinline__ bool place_vis(double u_m, double v_m, double w_m, double fx,
                                          const GridGeometry& g, int64_t* ix0, double* yu,
                                          int64_t* iy0, double* yv, int64_t* iw0, double* yw) {
#pragma clang fp contract(off)
  const int hw = g.support / 2;
  const double x = (u_m * fx) * g.scale_u + (double)(g.nu / 2);
  const double y = (v_m * fx) * g.scale_v + (double)(g.nv / 2);
  // The dirty image is sampled at l = k * pixsize, so it is periodic in u with
  // period 1 / pixsize = the grid extent: coordinates beyond the grid wrap
  // (exactly, as ducc0 does), and the footprint origin is taken modulo nu.
  uv_origin(x, y, hw, g, ix0, yu, iy0, yv);
  bool ok = true;
  if (g.do_wstacking) {
    const double xw = ((w_m * fx) - g.w0) * g.inv_dw;
    footprint(xw, hw, iw0, yw);
    ok = ok && (*iw0 >= 0) && (*iw0 + g.support <= g.nplanes);
  } else {
    *iw0 = 0;
    *yw = 0.0;
  }
  // non-finite coordinates are an error (the planner raises)
  ok = ok && isfinite(x) && isfinite(y) && fabs(x) < 9.0e15 && fabs(y) < 9.0e15;
  return ok;
}

// The planner's placement: the footprint origins place_vis computes (the same
// integers), without the kernel variables and without divergent branches in
// the common case - the origin inside the grid, no wrap (one unsigned compare
// per axis; |origin| < 2^30 first, so the conversion is exact); a wave with
// any other lane (off the grid by a period or more, not finite) takes
// place_vis itself (a wave-uniform branch). WS: w-stacking at compile time
// (0 / 1; -1: g.do_wstacking).
template <int WS = -1>
__device__ __forceinline__ bool place_origin(double u_m, double v_m, double w_m, double fx, const GridGeometry& g,
                                             int* ix0, int* iy0, int64_t* iw0) {
#pragma clang fp contract(off)
  const int hw = g.support / 2;
  const double x = (u_m * fx) * g.scale_u + (double)(g.nu / 2);
  const double y = (v_m * fx) * g.scale_v + (double)(g.nv / 2);
  const double flx = floor(x - (double)hw), fly = floor(y - (double)hw);
  const bool small = fabs(flx) < 1073741824.0 && fabs(fly) < 1073741824.0;
  const int ix = small ? (int)flx + 1 : -1, iy = small ? (int)fly + 1 : -1;
  const bool fits = ((unsigned)ix < (unsigned)g.nu) & ((unsigned)iy < (unsigned)g.nv);
  if (__ballot(!fits) != 0ull) {
    int64_t a, b, c;
    double ya, yb, yc;
    const bool ok = place_vis(u_m, v_m, w_m, fx, g, &a, &ya, &b, &yb, &c, &yc);
    *ix0 = (int)a;
    *iy0 = (int)b;
    *iw0 = c;
    return ok;
  }
  *ix0 = ix;
  *iy0 = iy;
  if (WS > 0 || (WS < 0 && g.do_wstacking)) {
    const double xw = ((w_m * fx) - g.w0) * g.inv_dw;
    double yw;
    footprint(xw, hw, iw0, &yw);
    // |x|, |y| < 2^30 + W here: finite and inside place_vis's bound
    return (*iw0 >= 0) & (*iw0 + g.support <= g.nplanes);
  }
  *iw0 = 0;
  return true;
}

// Flattened MS index i = row * nchan + c (< 2^52) -> (row, c): i * (1/nchan)
// in fp64 is within one of the quotient (one compare fixes it).
__device__ __forceinline__ void split_index64(int64_t i, int64_t nchan, double inv_nchan, int64_t* row,
                                             int64_t* c) {
  int64_t r = (int64_t)((double)i * inv_nchan);
  int64_t cc = i - r * nchan;
  if (cc < 0) {
    --r;
    cc += nchan;
  } else if (cc >= nchan) {
    ++r;
    cc -= nchan;
  }
  *row = r;
  *c = cc;
}

// Flattened MS index i = row * nchan + c (< 2^32) -> (row, c): one fp64
// multiply by 1/nchan (relative error <= 2^-52, so the quotient is off by at
// most one, fixed by one compare).
__device__ __forceinline__ void split_index(uint32_t i, int64_t nchan, double inv_nchan, int64_t* row,
                                           int64_t* c) {
  int64_t r = (int64_t)((double)i * inv_nchan);
  int64_t cc = (int64_t)i - r * nchan;
  if (cc < 0) {
    --r;
    cc += nchan;
  } else if (cc >= nchan) {
    ++r;
    cc -= nchan;
  }
  *row = r;
  *c = cc;
}

// How a (row, channel) pair maps to its visibility. Dense: the MS layout,
// row-major (nrow, nchan), index row * nchan + c. Ragged: row slices (the
// uvw_tiling Tile layout, reference uvw_tiling/tile.py:14-124): row r holds
// channels [c0_r, c1_r) at vis[off_r, off_r + c1_r - c0_r), so the index is
// delta[r] + c with delta[r] = off_r - c0_r; seg_row[k] is the row of
// visibility 64 k (the place pass's wave segments find their lanes' rows from
// it and the row starts off[], ragged_row_of below).
struct RowMap {
  int64_t nchan;            // channels (f/c entries)
  int64_t nvis;             // visibilities
  double inv_nchan;         // 1 / nchan
  const int64_t* delta;     // ragged: per-row index offset; NULL = dense
  const int64_t* off;       // ragged: row starts (nrow + 1 entries)
  const uint32_t* seg_row;  // ragged: row of each 64-visibility segment's first visibility
  int64_t nrow;             // ragged: rows (slices)
  const uint8_t* flags4;    // raw linear-feed input (WK_POL4I): (nvis, 4) flags, or NULL = none flagged
  // ragged ordered-stream entries packed as (index, row, channel) when their
  // bit widths fit 64 bits (cbits = channel bits, rbits = row bits; 0 = the
  // (row << 16) | channel form, index = delta[row] + channel)
  int pk_cbits, pk_rbits;
  // packed ragged runs (pk_cbits != 0, bank-class ordered plans of the lane
  // scatter, keys of <= 24 bits; make_plan): a run record is the ordered-stream
  // entry of its first visibility (position d of the run: entry + d (1 +
  // 2^(cbits + rbits))) and its length - 1 rides in bits 26-31 of its sort key,
  // above the radix digits - so the order pass needs no delta[row] gather
  int pk_runs = 0;
  // the plan's ordered-stream entries carry row phases (cip_grid.hip
  // order_kernel: bit 31 of dense entries, bit 63 of ragged ones), which the
  // scatter strips and applies (cip_scatter.h fetch_raw)
  int row_phase = 0;
};

constexpr int kRunLenShift = 26;  // RowMap::pk_runs: run length - 1 in sort-key bits 26-31
constexpr uint32_t kRunKeyMask = (1u << kRunLenShift) - 1u;

__device__ __forceinline__ int64_t vis_index(const RowMap& m, int64_t r, int64_t c) {
  return m.delta ? m.delta[r] + c : r * m.nchan + c;
}

// Ragged rows: the row of lane visibility i of a wave's 64-visibility segment
// (wave-uniform s = seg_row[seg], nx = off[s + 1], ilast = the segment's last
// visibility; lanes past the end pass any i of the segment). A segment that
// stays inside row s (rows longer than a wave: every segment of whole
// 256-channel rows) needs no more, else the row starts after s are loaded one
// per lane and each lane counts those <= i (sorted; empty rows repeat a start).
__device__ __forceinline__ int64_t ragged_row_of(const RowMap& m, int64_t s, int64_t nx, int64_t ilast, int64_t i) {
  const int lane = threadIdx.x & 63;
  if (nx > ilast) return s;  // uniform
  int64_t r = s;
  for (int64_t base = s + 1;; base += 64) {
    const int64_t q = base + lane;
    const int64_t o = q <= m.nrow ? m.off[q] : INT64_MAX;
    const unsigned long long in = __ballot(o <= ilast);  // a prefix of the lanes (sorted)
    const int nb = __popcll(in);
    for (int j = 0; j < nb; ++j) {
      const int64_t oj = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(o >> 32), j) << 32) |
                                   (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)o, j));
      r += i >= oj ? 1 : 0;
    }
    if (nb < 64) break;
  }
  return r;
}

// Entries of the bank-class ordered stream (perm, cip_grid.hip order_kernel):
// dense rows store the flattened MS index (u32; (row, channel) by one fp64
// multiply); ragged row slices store (index << (rbits + cbits)) | (row <<
// cbits) | channel (u64) when the three fit (pk_cbits != 0: C4's 1G
// visibilities over 3.9M rows x 256 channels take 30 + 22 + 8 bits), so the
// scatter needs neither a row lookup nor the delta[row] gather; else (row <<
// 16) | channel and index = delta[row] + channel.
__device__ __forceinline__ uint64_t perm_entry(const void* perm, const RowMap& m, int64_t q) {
  return m.delta ? ((const uint64_t*)perm)[q] : (uint64_t)((const uint32_t*)perm)[q];
}
// ragged entry of visibility il = delta[r] + c (row r, channel c)
__device__ __forceinline__ uint64_t perm_encode_wide(const RowMap& m, int64_t il, int64_t r, int64_t c) {
  if (m.pk_cbits)
    return ((uint64_t)il << (m.pk_cbits + m.pk_rbits)) | ((uint64_t)r << m.pk_cbits) | (uint64_t)c;
  return ((uint64_t)r << 16) | (uint64_t)c;
}
__device__ __forceinline__ void perm_decode_wide(uint64_t e, const RowMap& m, int64_t* il, int64_t* r, int64_t* c) {
  if (m.pk_cbits) {
    *c = (int64_t)(e & ((1ull << m.pk_cbits) - 1ull));
    *r = (int64_t)((e >> m.pk_cbits) & ((1ull << m.pk_rbits) - 1ull));
    *il = (int64_t)(e >> (m.pk_cbits + m.pk_rbits));
  } else {
    *r = (int64_t)(e >> 16);
    *c = (int64_t)(e & 0xffffu);
    *il = m.delta[*r] + *c;
  }
}
__device__ __forceinline__ uint64_t perm_encode(const RowMap& m, int64_t r, int64_t c) {
  return m.delta ? perm_encode_wide(m, m.delta[r] + c, r, c) : (uint64_t)(r * m.nchan + c);
}
__device__ __forceinline__ void perm_store(void* perm, const RowMap& m, int64_t pos, uint64_t e) {
  if (m.delta) ((uint64_t*)perm)[pos] = e;
  else ((uint32_t*)perm)[pos] = (uint32_t)e;
}
// compile-time forms (WIDE: ragged row slices) for the hot kernels
template <bool WIDE>
__device__ __forceinline__ uint64_t perm_entry_t(const void* perm, int64_t q) {
  if constexpr (WIDE) return ((const uint64_t*)perm)[q];
  return (uint64_t)((const uint32_t*)perm)[q];
}
template <bool WIDE>
__device__ __forceinline__ void perm_decode_t(uint64_t e, const RowMap& m, int64_t* il, int64_t* r, int64_t* c) {
  if constexpr (WIDE) {
    perm_decode_wide(e, m, il, r, c);
  } else {
    *il = (int64_t)e;
    split_index64((int64_t)e, m.nchan, m.inv_nchan, r, c);
  }
}
// -> (visibility index, row, channel)
__device__ __forceinline__ void perm_decode(uint64_t e, const RowMap& m, int64_t* il, int64_t* r, int64_t* c) {
  if (m.delta) {
    perm_decode_wide(e, m, il, r, c);
  } else {
    *il = (int64_t)e;
    split_index64((int64_t)e, m.nchan, m.inv_nchan, r, c);
  }
}

// Tile key of a footprint origin: tile-major, key = ((iy0 / T) ntx + ix0 / T)
// ntw + iw0, so the w layers of one uv tile are adjacent in the tile-sorted
// stream and a w-stacking plane's work units (layers p - W + 1 .. p of a tile)
// are contiguous ranges (2-D: ntw = 1, key = tile).
__device__ __forceinline__ int64_t tile_key(int64_t ix0, int64_t iy0, int64_t iw0, const GridGeometry& g) {
  // ix0, iy0 in [0, 2^31) after wrapping: unsigned division
  return ((int64_t)((uint32_t)iy0 / (uint32_t)kTile) * g.ntx + (int64_t)((uint32_t)ix0 / (uint32_t)kTile)) * g.ntw +
         iw0;
}

// Grid origin of a tile key's T x T tile.
__device__ __forceinline__ void tile_origin(int64_t key, const GridGeometry& g, int64_t* X0, int64_t* Y0) {
  const int64_t t = key / g.ntw;
  *X0 = (t % g.ntx) * kTile;
  *Y0 = ((t / g.ntx) % g.nty) * kTile;
}

// visibility / weight loads by dtype (CIP_C64 -> float2, CIP_C128 -> double2;
// raw linear-feed columns -> Pol4 + WK_POL4I, Stokes I formed on load)
enum { WK_NONE = 0, WK_F32 = 1, WK_F64 = 2, WK_POL4I = 3 };
// internal vis / wgt dtype code of the raw linear-feed input (not in cip.h:
// reached through cip_ms2dirty_stokes_i only)
constexpr int CIP_POL4I = 0x100;

// One visibility's linear-feed correlations (XX, XY, YX, YY) in complex64:
// the raw (nrow, nchan, 4) MS column (cip_ms2dirty_stokes_i).
struct Pol4 {
  float2 c[4];
};

// Stokes I of the raw columns in the reference's numpy float32 arithmetic
// (invert.py:86-116, :72-76; bit-identical to cip_stokes_i, cip_tiling.hip):
// V = 0.5 (XX + YY) in complex64; effective weight = !(F_XX | F_YY) *
// 4 / (1 / w_XX + 1 / w_YY) in float32 (a zero weight gives 4 / inf = 0).
__device__ __forceinline__ float2 stokes_i_vis(float2 a, float2 d) {
  return make_float2(0.5f * (a.x + d.x), 0.5f * (a.y + d.y));
}
__device__ __forceinline__ float stokes_i_weight(float wa, float wb, uint32_t flags_word) {
  const bool fl = (flags_word & 0xff0000ffu) != 0u;  // bytes 0 (XX) and 3 (YY)
  const float w = 4.0f / (1.0f / wa + 1.0f / wb);
  return (fl ? 0.0f : 1.0f) * w;
}

template <int WK>
__device__ __forceinline__ double load_weight(const void* __restrict__ w, const RowMap& m, int64_t i) {
  if constexpr (WK == WK_F32) return (double)((const float*)w)[i];
  if constexpr (WK == WK_F64) return ((const double*)w)[i];
  if constexpr (WK == WK_POL4I) {
    const float* w4 = (const float*)w + 4 * i;
    const uint32_t fw = m.flags4 ? ((const uint32_t*)m.flags4)[i] : 0u;
    return (double)stokes_i_weight(w4[0], w4[3], fw);
  }
  return 1.0;
}

// p == NULL: unit visibilities (the point-spread function, CIP_PSF)
__device__ __forceinline__ void load_vis(const float2* __restrict__ p, int64_t i, double& re, double& im) {
  if (p == nullptr) {
    re = 1.0;
    im = 0.0;
    return;
  }
  const float2 v = p[i];
  re = v.x;
  im = v.y;
}
__device__ __forceinline__ void load_vis(const double2* __restrict__ p, int64_t i, double& re, double& im) {
  const double2 v = p[i];
  re = v.x;
  im = v.y;
}
__device__ __forceinline__ void load_vis(const Pol4* __restrict__ p, int64_t i, double& re, double& im) {
  if (p == nullptr) {
    re = 1.0;
    im = 0.0;
    return;
  }
  const float2 v = stokes_i_vis(p[i].c[0], p[i].c[3]);
  re = v.x;
  im = v.y;
}

}  // namespace cip
