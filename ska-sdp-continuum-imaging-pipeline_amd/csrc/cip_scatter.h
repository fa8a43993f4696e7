// cip_scatter.h - the convolutional scatter of visibilities onto the uv grid
// (the hot loop of ducc0.wgridder.ms2dirty), as device
// templates. cip_scatter_w.hip instantiates launch_scatter_w<W> once per
// kernel support W (one translation unit each, compiled in parallel);
// launch_scatter (cip_grid.hip) dispatches on W.
//
// Scatter design (DESIGN.md "Scatter kernel"): one 256-thread workgroup per
// chunk (<= kChunkVis visibilities of one T x T grid tile, T = 32). The tile's
// (T+W-1)^2 sub-grid lives in LDS as 64-bit fixed-point re/im pairs. Each lane
// owns one visibility at a time (lane-per-visibility), evaluates the 2 x W
// piecewise-polynomial kernel values, and adds its W x W taps with no-return
// ds_add_u64. After the chunk the non-zero sub-grid cells are converted back
// to fp64 and added to the HBM grid with global fp64 atomics. No MFMA: this
// is a scatter.
#pragma once
#include <cstdlib>
#include <type_traits>

#include "cip_internal.h"

// the bits of fma(k, v, 1.5 2^52) are the integer plus this bias
constexpr unsigned long long kTapBias = 0x4338000000000000ull;

namespace cip {

// ------------------------------------------------------------ scatter ----
#ifndef CIP_SCATTER_WAVES
#define CIP_SCATTER_WAVES 4  // min waves per SIMD the scatter is compiled for (register budget)
#endif
#ifndef CIP_GROUP_THREADS
#define CIP_GROUP_THREADS 512  // threads of a plane-group (G > 1) unit
#endif
constexpr int kScatterThreads = 256;
constexpr int kRunBatch = 256;

// Everything one visibility needs, loaded one iteration ahead of its use so
// the global-memory latency overlaps the previous visibility's taps.
struct VisFetch {
  double u, v, w, fx, vr, vi, wt;
  uint32_t h;  // row phase (order_kernel): 1 = footprint rows in the order 1 .. W - 1, 0
};

// last staged run starting at or before flattened visibility q
__device__ __forceinline__ void locate_vis(int64_t q, const int64_t* s_voff, const uint64_t* s_run, int nst,
                                           int64_t* irow, int64_t* c) {
  int lo = 0, hi = nst - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (s_voff[mid] <= q) lo = mid;
    else hi = mid - 1;
  }
  const uint64_t rec = s_run[lo];
  *irow = (int64_t)(rec >> 32);
  *c = (int64_t)((rec >> 16) & 0xffff) + (q - s_voff[lo]);
}

template <typename VisT, int WK>
__device__ __forceinline__ void fetch_vis(int64_t q, const int64_t* s_voff, const uint64_t* s_run, int nst,
                                          const double* __restrict__ uvw, const double* __restrict__ fx,
                                          const VisT* __restrict__ vis, const void* __restrict__ wgt,
                                          const RowMap& m, VisFetch& f) {
  int64_t irow, c;
  locate_vis(q, s_voff, s_run, nst, &irow, &c);
  const int64_t idx = vis_index(m, irow, c);
  f.u = uvw[3 * irow];
  f.v = uvw[3 * irow + 1];
  f.w = uvw[3 * irow + 2];
  f.fx = fx[c];
  load_vis(vis, idx, f.vr, f.vi);
  f.wt = load_weight<WK>(wgt, m, idx);
  f.h = 0u;
}

// The same, as loaded (complex64 / float32 kept in their own types): the
// position-ordered path converts only at use, so nothing waits for a load
// next to it and the loads of position q + 256 stay in flight while q grids.
// Raw linear-feed input keeps the two correlations, weights and the flag word
// of Stokes I (formed at use).
template <typename VisT, int WK>
struct RawFetch {
  using WT = typename std::conditional<WK == WK_F64, double, float>::type;
  double u, v, w, fx;
  VisT vis;
  WT wt;
  uint32_t h;
};
template <>
struct RawFetch<Pol4, WK_POL4I> {
  double u, v, w, fx;
  float2 a, d;
  float wa, wb;
  uint32_t fw;
  uint32_t h;
};

// Branch-free loads of the visibility of ordered-stream entry e (callers pass
// a valid entry for every lane - out-of-range lanes repeat one - and mask the
// result; a PSF call, vis == NULL, reads its ignored visibility from
// uvw[0..1]).
// WIDE = 0 / 1: dense / ragged entries (compile time); -1: decided by m.delta
template <typename VisT, int WK, int WIDE = -1>
__device__ __forceinline__ void fetch_raw(uint64_t e, const double* __restrict__ uvw,
                                          const double* __restrict__ fx, const VisT* __restrict__ vis_ld,
                                          bool unit_vis, const void* __restrict__ wgt, const RowMap& m,
                                          RawFetch<VisT, WK>& f) {
  int64_t il, r, c;
  f.h = 0u;
  if (m.row_phase) {  // (uniform)
    if constexpr (WIDE == 0) {
      // dense entries: the row phase in bit 31 (order_kernel<0, true>)
      f.h = (uint32_t)(e >> 31) & 1u;
      e &= 0x7fffffffull;
    } else if constexpr (WIDE == 1) {
      // ragged entries: bit 63 (order_kernel<1 / 2, true>)
      f.h = (uint32_t)(e >> 63);
      e &= 0x7fffffffffffffffull;
    }
  }
  if constexpr (WIDE < 0) perm_decode(e, m, &il, &r, &c);
  else perm_decode_t<WIDE == 1>(e, m, &il, &r, &c);
  f.u = uvw[3 * r];
  f.v = uvw[3 * r + 1];
  f.w = uvw[3 * r + 2];
  f.fx = fx[c];
  if constexpr (WK == WK_POL4I) {
    const float2* p = (const float2*)vis_ld;
    f.a = p[unit_vis ? 0 : 4 * il];
    f.d = p[unit_vis ? 0 : 4 * il + 3];
    const float* w4 = (const float*)wgt + 4 * il;
    f.wa = w4[0];
    f.wb = w4[3];
    f.fw = m.flags4 ? ((const uint32_t*)m.flags4)[il] : 0u;
  } else {
    using WT = typename RawFetch<VisT, WK>::WT;
    f.vis = vis_ld[unit_vis ? 0 : il];
    if constexpr (WK != WK_NONE) f.wt = ((const WT*)wgt)[il];
  }
}

template <typename VisT, int WK>
__device__ __forceinline__ VisFetch from_raw(const RawFetch<VisT, WK>& r, bool unit_vis) {
  VisFetch f;
  f.u = r.u;
  f.v = r.v;
  f.w = r.w;
  f.fx = r.fx;
  f.h = r.h;
  if constexpr (WK == WK_POL4I) {
    const float2 s = stokes_i_vis(r.a, r.d);
    f.vr = unit_vis ? 1.0 : (double)s.x;
    f.vi = unit_vis ? 0.0 : (double)s.y;
    f.wt = (double)stokes_i_weight(r.wa, r.wb, r.fw);
  } else {
    f.vr = unit_vis ? 1.0 : (double)r.vis.x;
    f.vi = unit_vis ? 0.0 : (double)r.vis.y;
    f.wt = WK == WK_NONE ? 1.0 : (double)r.wt;
  }
  return f;
}

// One packed single-precision tap (CIP_ACC_SINGLE): the contributions
// ku * kr and ku * ki rounded to integers in fp32 by one packed fma against
// 1.5 * 2^23 (exact for |x| < 2^22, which packed_chunk_gain guarantees): the
// two results' bits, (M + im) in the low and (M + re) in the high word, are
// one 64-bit integer, and subtracting M * (2^32 + 1) leaves re * 2^32 + im in
// two's complement (the borrow of a negative im comes with the 64-bit
// subtraction) for ONE 64-bit LDS add. Two VALU instructions per tap
// (v_pk_fma_f32 + v_lshl_add_u64), against two fp64 fmas + a combine - the
// arithmetic class of ducc0's float32 gridding that the reference's
// complex64 call uses.
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr unsigned long long kMagicPair = ((unsigned long long)kMagicFBits << 32) | kMagicFBits;
__device__ __forceinline__ unsigned long long packed_tap(float ku, f32x2 k_ir) {
  const f32x2 q = __builtin_elementwise_fma(f32x2{ku, ku}, k_ir, f32x2{kMagicF, kMagicF});
  return __builtin_bit_cast(unsigned long long, q) - kMagicPair;
}

// A visibility of row phase h (order_kernel) adds its footprint rows in the
// order h, h + 1, .., (W - 1 + h) mod W: its kernel values rotated by h here,
// and the rows' LDS addresses rotated in row_ptr - the same taps into the same
// cells, but at each tap instruction its bank pair is shifted by P (the order
// pass balances the bank classes with it).
template <int W, typename T>
__device__ __forceinline__ void rotate_rows(T* k, uint32_t h) {
  const T k0 = k[0];
#pragma unroll
  for (int i = 0; i < W - 1; ++i) k[i] = h ? k[i + 1] : k[i];
  k[W - 1] = h ? k0 : k[W - 1];
}
// the LDS address of tap (i, 0) of a footprint at base, rows rotated by h:
// rows i < W - 1 from base + h P (one register), the last from base + (1 - h)
// (W - 1) P
template <int W, int P>
__device__ __forceinline__ unsigned long long* row_ptr(unsigned long long* b0, unsigned long long* bl, int i) {
  return i < W - 1 ? b0 + i * P : bl;
}

// The packed class's visibility: fp32 kernel values and tap products (the
// placement stays fp64, the planner's bit for bit). G > 1: the unit's G
// planes as in grid_fetched.
template <int W, bool WSTACK, int G>
__device__ __forceinline__ void grid_fetched_packed(const VisFetch& f, const GridGeometry& g, int64_t plane,
                                                    int64_t X0, int64_t Y0, double fixed_scale,
                                                    unsigned long long* sub) {
  constexpr int T = kTile;
  constexpr int P = T + W - 1;
  constexpr int S = P * P;
  if (f.wt == 0.0) return;
  int64_t ix0, iy0, iw0;
  double yu, yv, yw;
  if (!place_vis(f.u, f.v, f.w, f.fx, g, &ix0, &yu, &iy0, &yv, &iw0, &yw)) return;
  const int64_t lx = ix0 - X0, ly = iy0 - Y0;
  if (lx < 0 || lx >= T || ly < 0 || ly >= T) return;  // never for a consistent plan
  const double sc0 = f.wt * fixed_scale;
  const float vr0 = (float)(f.vr * sc0), vi0 = (float)(f.vi * sc0);
  float ku[W], kv[W];
  {
    f32x2 kuv[W];
    eval_kernel_f32x2<W>(f32x2{(float)yu, (float)yv}, kuv);
#pragma unroll
    for (int i = 0; i < W; ++i) {
      ku[i] = kuv[i].x;
      kv[i] = kuv[i].y;
    }
  }
  unsigned long long* base = sub + (lx * P + ly);
  rotate_rows<W>(ku, f.h);
  auto taps = [&](unsigned long long* bk, float vr, float vi) {
    f32x2 k_ir[W];  // (kv vi, kv vr): the low / high word of each tap
    const f32x2 v_ir{vi, vr};
#pragma unroll
    for (int j = 0; j < W; ++j) k_ir[j] = f32x2{kv[j], kv[j]} * v_ir;
    unsigned long long* b0 = bk + (f.h ? P : 0);
    unsigned long long* bl = bk + (f.h ? 0 : (W - 1) * P);
#pragma unroll
    for (int i = 0; i < W; ++i)
#pragma unroll
      for (int j = 0; j < W; ++j) atomicAdd(row_ptr<W, P>(b0, bl, i) + j, packed_tap(ku[i], k_ir[j]));
  };
  if constexpr (!WSTACK) {
    taps(base, vr0, vi0);
  } else {
    float kwv[W];
    eval_kernel_f32<W>((float)yw, kwv);
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const int64_t kw = plane + k - iw0;
      if (kw < 0 || kw >= W) continue;  // the visibility does not feed plane + k
      if (plane + k < g.plane_lo || plane + k >= g.plane_hi) continue;  // outside the call's plane range
      float sel = 0.0f;
#pragma unroll
      for (int q = 0; q < W; ++q) sel = (q == kw) ? kwv[q] : sel;
      taps(base + k * S, vr0 * sel, vi0 * sel);
    }
  }
}

// One visibility onto the unit's sub-grid(s). G > 1 (w-stacking): the unit
// grids planes plane .. plane + G - 1 at once (G sub-grids, S u64 apart), the
// visibility placed and its u, v, w kernels evaluated once for all of them.
template <int W, bool WSTACK, bool PACK, int G = 1>
__device__ __forceinline__ void grid_fetched(const VisFetch& f, const GridGeometry& g, int64_t plane, int64_t X0,
                                             int64_t Y0, double fixed_scale, unsigned long long* sub) {
  constexpr int T = kTile;
  constexpr int P = T + W - 1;
  if constexpr (PACK) {
    grid_fetched_packed<W, WSTACK, G>(f, g, plane, X0, Y0, fixed_scale, sub);
    return;
  }
  if (f.wt == 0.0) return;
  int64_t ix0, iy0, iw0;
  double yu, yv, yw;
  if (!place_vis(f.u, f.v, f.w, f.fx, g, &ix0, &yu, &iy0, &yv, &iw0, &yw)) return;
  const int64_t lx = ix0 - X0, ly = iy0 - Y0;
  if (lx < 0 || lx >= T || ly < 0 || ly >= T) return;  // never for a consistent plan
  if constexpr (G > 1) {
    constexpr int S = P * P * (PACK ? 1 : 2);
    double kwv[W], ku[W], kv[W];
    eval_kernel<W>(yw, kwv);
    eval_kernel<W>(yu, ku);
    eval_kernel<W>(yv, kv);
    rotate_rows<W>(ku, f.h);
    const double sc0 = f.wt * fixed_scale;
    unsigned long long* base = sub + (lx * P + ly);
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const int64_t kw = plane + k - iw0;
      if (kw < 0 || kw >= W) continue;  // the visibility does not feed plane + k
      if (plane + k < g.plane_lo || plane + k >= g.plane_hi) continue;  // outside the call's plane range
      double sel = 0.0;
#pragma unroll
      for (int q = 0; q < W; ++q) sel = (q == kw) ? kwv[q] : sel;
      const double sc = sc0 * sel;
      const double vr = f.vr * sc, vi = f.vi * sc;
      double kr[W], ki[W];
#pragma unroll
      for (int j = 0; j < W; ++j) {
        kr[j] = kv[j] * vr;
        ki[j] = kv[j] * vi;
      }
      unsigned long long* bk = base + k * S;
      unsigned long long* b0 = bk + (f.h ? P : 0);
      unsigned long long* bl = bk + (f.h ? 0 : (W - 1) * P);
#pragma unroll
      for (int i = 0; i < W; ++i) {
        unsigned long long* bi0 = row_ptr<W, P>(b0, bl, i);
#pragma unroll
        for (int j = 0; j < W; ++j) {
          const double qr = fma(ku[i], kr[j], kMagic);
          const double qi = fma(ku[i], ki[j], kMagic);
          const unsigned long long br = (unsigned long long)__double_as_longlong(qr);
          const unsigned long long bi = (unsigned long long)__double_as_longlong(qi);
          if constexpr (PACK) {
            unsigned hi;
            asm("v_add3_u32 %0, %1, %2, %3" : "=v"(hi) : "v"((unsigned)br), "v"((unsigned)(bi >> 32)),
                "s"(0u - kMagicHi));
            atomicAdd(bi0 + j, __builtin_bit_cast(unsigned long long, make_uint2((unsigned)bi, hi)));
          } else {
            atomicAdd(bi0 + j, br - kTapBias);
            atomicAdd(bi0 + P * P + j, bi - kTapBias);
          }
        }
      }
    }
    return;
  }
  double sc = f.wt * fixed_scale;
  if constexpr (WSTACK) {
    const int64_t kw = plane - iw0;
    if (kw < 0 || kw >= W) return;
    double kwv[W];
    eval_kernel<W>(yw, kwv);
    double sel = 0.0;
#pragma unroll
    for (int k = 0; k < W; ++k) sel = (k == kw) ? kwv[k] : sel;
    sc *= sel;
  }
  const double vr = f.vr * sc, vi = f.vi * sc;
  double ku[W], kv[W];
  eval_kernel<W>(yu, ku);
  eval_kernel<W>(yv, kv);
  rotate_rows<W>(ku, f.h);
  double kr[W], ki[W];
#pragma unroll
  for (int j = 0; j < W; ++j) {
    kr[j] = kv[j] * vr;
    ki[j] = kv[j] * vi;
  }
  // separate re / im planes: a lane-scattered 8-byte add touches 2 of the 64
  // LDS banks, so 8-byte cells spread a wave over twice the bank pairs that
  // interleaved 16-byte (re, im) cells would
  unsigned long long* base = sub + (lx * P + ly);
  unsigned long long* b0 = base + (f.h ? P : 0);
  unsigned long long* bl = base + (f.h ? 0 : (W - 1) * P);
#pragma unroll
  for (int i = 0; i < W; ++i) {
    unsigned long long* bi0 = row_ptr<W, P>(b0, bl, i);
#pragma unroll
    for (int j = 0; j < W; ++j) {
      const double qr = fma(ku[i], kr[j], kMagic);
      const double qi = fma(ku[i], ki[j], kMagic);
      const unsigned long long br = (unsigned long long)__double_as_longlong(qr);
      const unsigned long long bi = (unsigned long long)__double_as_longlong(qi);
      if constexpr (PACK) {
        // bits(kMagic + k) = 0x43380000'00000000 + k (two's complement), so
        // re * 2^32 + im = {lo32(br) + hi32(bi) - 0x43380000, lo32(bi)}
        unsigned hi;  // one v_add3_u32 (the compiler otherwise widens it to 64-bit adds)
        asm("v_add3_u32 %0, %1, %2, %3" : "=v"(hi) : "v"((unsigned)br), "v"((unsigned)(bi >> 32)),
            "s"(0u - kMagicHi));
        atomicAdd(bi0 + j, __builtin_bit_cast(unsigned long long, make_uint2((unsigned)bi, hi)));
      } else {
        atomicAdd(bi0 + j, br - kTapBias);
        atomicAdd(bi0 + P * P + j, bi - kTapBias);
      }
    }
  }
}

// Flush the touched cells of a work unit's sub-grid(s) to the HBM grid(s)
// (called after the unit's last LDS atomic and a barrier).
template <int W, bool PACK, int G, int NT>
__device__ __forceinline__ void flush_subgrid(const unsigned long long* sub, const GridGeometry& g, int64_t plane,
                                              int64_t X0, int64_t Y0, const Chunk& ch, int store_private,
                                              double inv_scale, double* __restrict__ grid) {
  constexpr int T = kTile;
  constexpr int P = T + W - 1;
  constexpr int S = P * P * (PACK ? 1 : 2);
  // flush the touched cells of the sub-grid(s) to the fp64 HBM grid(s)
  // (lanes walk the HBM grid's contiguous axis: y, or x when it is stored
  // transposed for the pruned FFT); plane group: plane + k -> grid + k planes.
  // A tile's cells [W - 1, T)^2 are written by its own units only (the
  // neighbours' sub-grids reach W - 1 cells into it): when this unit is the
  // tile's only one and the grid is zero (store_private: a cip_ms2dirty plane,
  // not an accumulating one; set on 16384^2+ planes), those cells are stored,
  // not added - one 16-B store instead of two read-modify-write fp64 atomics
  // at the L2 (C4's 16384^2 grid: the flush is ~1.1 of the 4.9 ms scatter,
  // 0.28 ms less with the stores; profiles/r03_ab_flush_store.txt)
  const bool own = store_private != 0 && ch.sole != 0;
  // packed class on complex64 planes (GridGeometry::grid_f32)
  const bool f32 = PACK && g.grid_f32 != 0;
  // the tiles this unit writes, per plane (GridGeometry::wmask; uniform branch)
  __shared__ unsigned s_wm[G];
  unsigned wm[G];
#pragma unroll
  for (int k = 0; k < G; ++k) wm[k] = 0u;
  if (g.wmask) {
    if (threadIdx.x < G) s_wm[threadIdx.x] = 0u;
    __syncthreads();
  }
  // one pass over the cells for all G planes: a cell's G sub-grid values are
  // read together and its HBM offset (the wrap, the strip's row map, the
  // transposed layout: ~45 VALU) is computed once, not once per plane - on the
  // reference call's G = 5 plane groups the per-plane form was ~1/3 of the
  // scatter's VALU instructions (7.25 -> 7.17 ms, profiles/r04_ab_flush_fused.txt)
  for (int cell = threadIdx.x; cell < P * P; cell += NT) {
    const int lcell = g.transposed ? (cell % P) * P + cell / P : cell;  // lx * P + ly
    unsigned long long sv[G];  // PACK: re * 2^32 + im
    unsigned long long si[G];  // !PACK: the im plane
    bool any = false;
#pragma unroll
    for (int k = 0; k < G; ++k) {
      sv[k] = 0ull;
      si[k] = 0ull;
      if (G > 1 && (plane + k >= g.nplanes || plane + k < g.plane_lo || plane + k >= g.plane_hi)) continue;
      sv[k] = sub[k * S + lcell];
      if constexpr (!PACK) si[k] = sub[k * S + P * P + lcell];
      any |= (sv[k] | si[k]) != 0ull;
    }
    if (!any) continue;
    // the sub-grid of an edge tile wraps around the periodic grid
    int64_t gx = X0 + lcell / P, gy = Y0 + lcell % P;
    gx -= (gx >= g.nu) ? g.nu : 0;
    gy -= (gy >= g.nv) ? g.nv : 0;
    const int64_t off = grid_cell_offset(g, gx, gy);
    if (off < 0) {
      if (g.oob) atomicOr(g.oob, 1u);
      continue;
    }
    const int lx = lcell / P, ly = lcell % P;
    const bool priv = own && lx >= W - 1 && lx < T && ly >= W - 1 && ly < T;
    const unsigned tbit = 1u << ((lx / T) * 3 + ly / T);
#pragma unroll
    for (int k = 0; k < G; ++k) {
      if ((sv[k] | si[k]) == 0ull) continue;  // (also every plane outside the call's range)
      wm[k] |= tbit;
      long long re, im;
      if constexpr (PACK) {
        im = (long long)(int)(unsigned)sv[k];
        re = (long long)(int)(unsigned)((sv[k] - (unsigned long long)im) >> 32);
      } else {
        re = (long long)sv[k];
        im = (long long)si[k];
      }
      // planes of g.rows rows (a uv strip's buffer holds its rows of every plane)
      const int64_t pk = (int64_t)k * 2 * g.nu * g.rows + 2 * off;
      if (f32) {
        float* dstf = (float*)grid + pk;
        if (priv) {
          *reinterpret_cast<float2*>(dstf) = make_float2((float)((double)re * inv_scale),
                                                         (float)((double)im * inv_scale));
        } else {
          unsafeAtomicAdd(dstf, (float)((double)re * inv_scale));
          unsafeAtomicAdd(dstf + 1, (float)((double)im * inv_scale));
        }
        continue;
      }
      double* dst = grid + pk;
      if (priv) {
        *reinterpret_cast<double2*>(dst) = make_double2((double)re * inv_scale, (double)im * inv_scale);
      } else {
        unsafeAtomicAdd(dst, (double)re * inv_scale);
        unsafeAtomicAdd(dst + 1, (double)im * inv_scale);
      }
    }
  }
  if (g.wmask) {
#pragma unroll
    for (int k = 0; k < G; ++k)
      if (wm[k]) atomicOr(&s_wm[k], wm[k]);
    __syncthreads();
    if (threadIdx.x < G && s_wm[threadIdx.x]) wmask_report(g, plane + threadIdx.x, X0, Y0, s_wm[threadIdx.x]);
  }
}

// PERM: 0 = tile order through the row slices, 1 / 2 = the bank-class ordered
// stream of dense (u32) / ragged (u64) entries. G: w planes per work unit
// (w-stacking plane groups; G > 1 runs 512-thread blocks holding G sub-grids).
template <int G>
constexpr int scatter_threads() {
  return G == 1 ? kScatterThreads : CIP_GROUP_THREADS;
}
template <int W, typename VisT, int WK, bool WSTACK, int PERM, bool PACK, int G = 1>
__global__ __launch_bounds__(scatter_threads<G>(), CIP_SCATTER_WAVES) void scatter_kernel(
    const double* __restrict__ uvw, const double* __restrict__ fx, const VisT* __restrict__ vis,
    const void* __restrict__ wgt, RowMap m, const uint64_t* __restrict__ runs,
    const int64_t* __restrict__ run_goff, const int64_t* __restrict__ tile_run_off,
    const void* __restrict__ perm, const Chunk* __restrict__ chunks, int64_t chunk_begin, GridGeometry g,
    int64_t plane, double fixed_scale, double inv_scale, double* __restrict__ grid, int store_private) {
  constexpr int T = kTile;
  constexpr int P = T + W - 1;
  constexpr int S = P * P * (PACK ? 1 : 2);
  constexpr int NT = scatter_threads<G>();
  __shared__ unsigned long long sub[G * S];
  __shared__ int64_t s_voff[PERM ? 1 : kRunBatch + 1];
  __shared__ uint64_t s_run[PERM ? 1 : kRunBatch];
  constexpr bool kWide = PERM == 2;

  const Chunk ch = chunks[chunk_begin + blockIdx.x];
  int64_t X0, Y0;
  tile_origin(ch.tile, g, &X0, &Y0);
  for (int i = threadIdx.x; i < G * S; i += NT) sub[i] = 0ull;
  if constexpr (PACK) {
    fixed_scale *= packed_chunk_gain(ch.g1 - ch.g0);
    inv_scale = 1.0 / fixed_scale;
  }
  if constexpr (PERM) {
    // bank-class ordered stream (order_kernel); software pipeline, two
    // deep: perm record of q + 512 and data of q + 256 in flight while q grids
    __syncthreads();
    const bool unit_vis = vis == nullptr;
    const VisT* vis_ld = unit_vis ? (const VisT*)uvw : vis;
    int64_t q = ch.g0 + threadIdx.x;
    bool have = q < ch.g1;
    RawFetch<VisT, WK> cur;
    int64_t qn = q + NT;
    bool hn = qn < ch.g1;
    uint64_t pn = 0;
    if (have) {
      fetch_raw<VisT, WK, kWide>(perm_entry_t<kWide>(perm, q), uvw, fx, vis_ld, unit_vis, wgt, m, cur);
      pn = perm_entry_t<kWide>(perm, hn ? qn : q);
    }
    while (have) {
      const int64_t qnn = qn + NT;
      const bool hnn = qnn < ch.g1;
      const uint64_t pnn = perm_entry_t<kWide>(perm, hnn ? qnn : q);
      RawFetch<VisT, WK> nxt;
      fetch_raw<VisT, WK, kWide>(pn, uvw, fx, vis_ld, unit_vis, wgt, m, nxt);
      grid_fetched<W, WSTACK, PACK, G>(from_raw<VisT, WK>(cur, unit_vis), g, plane, X0, Y0, fixed_scale, sub);
      cur = nxt;
      q = qn;
      have = hn;
      qn = qnn;
      hn = hnn;
      pn = pnn;
    }
  } else {
    const int64_t rb = ch.last_run + 1;  // (a w-stacking unit spans several tile keys)
    int64_t r = ch.first_run;
    int64_t v = ch.g0;
    while (v < ch.g1 && r < rb) {
      const int nst = (int)((rb - r) < kRunBatch ? (rb - r) : kRunBatch);
      __syncthreads();
      for (int k = threadIdx.x; k <= nst; k += NT) {
        s_voff[k] = run_goff[r + k];
        if (k < nst) s_run[k] = runs[r + k];
      }
      __syncthreads();
      const int64_t bend = ch.g1 < s_voff[nst] ? ch.g1 : s_voff[nst];
      // software pipeline: fetch visibility q + 256 while gridding q
      int64_t q = v + threadIdx.x;
      bool have = q < bend;
      VisFetch cur;
      if (have) fetch_vis<VisT, WK>(q, s_voff, s_run, nst, uvw, fx, vis, wgt, m, cur);
      while (have) {
        const int64_t qn = q + NT;
        const bool hn = qn < bend;
        VisFetch nxt;
        if (hn) fetch_vis<VisT, WK>(qn, s_voff, s_run, nst, uvw, fx, vis, wgt, m, nxt);
        grid_fetched<W, WSTACK, PACK, G>(cur, g, plane, X0, Y0, fixed_scale, sub);
        cur = nxt;
        q = qn;
        have = hn;
      }
      v = bend;
      r += nst;
    }
  }
  __syncthreads();
  flush_subgrid<W, PACK, G, NT>(sub, g, plane, X0, Y0, ch, store_private, inv_scale, grid);
}

template <int W, typename VisT, int WK>
inline hipError_t scatter_dispatch_ws(bool ws, int group, bool pack, unsigned lds_extra, int store_private,
                                      dim3 grid_dim, hipStream_t s,
                                      const double* uvw,
                                      const double* fx, const void* vis, const void* wgt, const RowMap& m,
                                      const uint64_t* runs, const int64_t* run_goff, const int64_t* tile_run_off,
                                      const void* perm, const Chunk* chunks, int64_t chunk_begin,
                                      const GridGeometry& g, int64_t plane, double fs, double* grid) {
#define LAUNCH(WSV, PRM, PK, GG)                                                                            \
  scatter_kernel<W, VisT, WK, WSV, PRM, PK, GG><<<grid_dim, dim3(scatter_threads<GG>()), lds_extra, s>>>(   \
      uvw, fx, (const VisT*)vis, wgt, m, runs, run_goff, tile_run_off, perm, chunks, chunk_begin, g, plane,    \
      fs, 1.0 / fs, grid, store_private)
#define LAUNCH_WS(PRM, PK)            \
  {                                   \
    if (ws && group == 3) {           \
      LAUNCH(true, PRM, PK, 3);       \
    } else if (ws && group == 2) {    \
      LAUNCH(true, PRM, PK, 2);       \
    } else if (ws) {                  \
      LAUNCH(true, PRM, PK, 1);       \
    } else {                          \
      LAUNCH(false, PRM, PK, 1);      \
    }                                 \
  }
  // the packed class's 8-byte cells fit larger plane groups (4, 5) in LDS
#define LAUNCH_WS_PACKED(PRM)                                \
  {                                                          \
    bool hit = false;                                        \
    if constexpr (kFitG7) {                                  \
      if (ws && group == 7) {                                \
        LAUNCH(true, PRM, true, 7);                          \
        hit = true;                                          \
      }                                                      \
    }                                                        \
    if constexpr (kFitG6) {                                  \
      if (!hit && ws && group == 6) {                        \
        LAUNCH(true, PRM, true, 6);                          \
        hit = true;                                          \
      }                                                      \
    }                                                        \
    if constexpr (kFitG5) {                                  \
      if (!hit && ws && group == 5) {                        \
        LAUNCH(true, PRM, true, 5);                          \
        hit = true;                                          \
      }                                                      \
    }                                                        \
    if constexpr (kFitG4) {                                  \
      if (!hit && ws && group == 4) {                        \
        LAUNCH(true, PRM, true, 4);                          \
        hit = true;                                          \
      }                                                      \
    }                                                        \
    if (!hit) LAUNCH_WS(PRM, true)                           \
  }
  // the packed single-precision class exists for complex64 input only (the
  // reference's configuration; raw linear-feed columns are complex64 too)
  // plane groups of 4 / 5 packed sub-grids while they fit 64 KB of static LDS
  constexpr int P2 = (kTile + W - 1) * (kTile + W - 1);
  constexpr bool kFitG5 = 5 * P2 * 8 + 4200 <= 65536;
  // 6 / 7: two blocks per CU in 160 KB
  constexpr bool kFitG7 = 7 * P2 * 8 + 4200 <= 81920;
  constexpr bool kFitG6 = 6 * P2 * 8 + 4200 <= 81920;
  constexpr bool kFitG4 = 4 * P2 * 8 + 4200 <= 65536;
  bool done = false;
  const bool wide = m.delta != nullptr;  // ragged row slices: u64 entries
  if constexpr (std::is_same<VisT, float2>::value || std::is_same<VisT, Pol4>::value) {
    if (pack) {
      if (perm && wide) {
        LAUNCH_WS_PACKED(2)
      } else if (perm) {
        LAUNCH_WS_PACKED(1)
      } else {
        LAUNCH_WS_PACKED(0)
      }
      done = true;
    }
  }
  if (!done) {
    if (perm && wide) {
      LAUNCH_WS(2, false)
    } else if (perm) {
      LAUNCH_WS(1, false)
    } else {
      LAUNCH_WS(0, false)
    }
  }
#undef LAUNCH_WS_PACKED
#undef LAUNCH_WS
#undef LAUNCH
  return hipGetLastError();
}

template <int W>
hipError_t launch_scatter_w(int vis_dtype, int wgt_dtype, bool pack, int group, unsigned lds_extra,
                            int store_private, dim3 gd, hipStream_t s,
                                     const double* uvw, const double* fx, const void* vis, const void* wgt,
                                     const RowMap& m, const uint64_t* runs, const int64_t* run_goff,
                                     const int64_t* tile_run_off, const void* perm, const Chunk* chunks,
                                     int64_t cb, const GridGeometry& g, int64_t plane, double fs, double* grid) {
  const bool ws = g.do_wstacking != 0;
#define ARGS \
  ws, group, pack, lds_extra, store_private, gd, s, uvw, fx, vis, wgt, m, runs, run_goff, tile_run_off, perm, \
      chunks, cb, g, plane, fs, grid
  if (vis_dtype == CIP_POL4I) return scatter_dispatch_ws<W, Pol4, WK_POL4I>(ARGS);
  if (vis_dtype == CIP_C64) {
    if (wgt_dtype == CIP_F32) return scatter_dispatch_ws<W, float2, WK_F32>(ARGS);
    if (wgt_dtype == CIP_F64) return scatter_dispatch_ws<W, float2, WK_F64>(ARGS);
    return scatter_dispatch_ws<W, float2, WK_NONE>(ARGS);
  }
  if (wgt_dtype == CIP_F32) return scatter_dispatch_ws<W, double2, WK_F32>(ARGS);
  if (wgt_dtype == CIP_F64) return scatter_dispatch_ws<W, double2, WK_F64>(ARGS);
  return scatter_dispatch_ws<W, double2, WK_NONE>(ARGS);
#undef ARGS
}

}  // namespace cip
