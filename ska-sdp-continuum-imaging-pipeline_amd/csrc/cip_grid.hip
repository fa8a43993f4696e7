// cip_grid.hip - the convolutional scatter of visibilities onto the uv grid
// (the hot loop of ducc0.wgridder.ms2dirty) and the
// post-FFT crop / grid-correction / w-screen kernels (a4.5, a4.6).
//
// Scatter design (DESIGN.md "Scatter kernel"): one 256-thread workgroup per
// chunk (<= kChunkVis visibilities of one T x T grid tile, T = 32). The tile's
// (T+W-1)^2 sub-grid lives in LDS as 64-bit fixed-point re/im pairs. Each lane
// owns one visibility at a time (lane-per-visibility), evaluates the 2 x W
// piecewise-polynomial kernel values, and adds its W x W taps with no-return
// ds_add_u64. After the chunk the non-zero sub-grid cells are converted back
// to fp64 and added to the HBM grid with global fp64 atomics. No MFMA: this
// is a scatter.
#include "cip_internal.h"
#include <type_traits>

// Experiment-only builds (tools/build_variant.sh): 1 = conflict-free LDS
// addresses, 2 = no LDS atomics, 3 = no kernel evaluation, 4 = no flush to
// HBM (timing only, wrong images). 0 in the library. Measured at C3
// (profiles/microbench_r01.txt): kernel evaluation ~0.2 ms, flush ~0.1 ms of
// the 3.1 ms scatter.
#ifndef CIP_ABLATE
#define CIP_ABLATE 0
#endif

namespace cip {

// ------------------------------------------------------ prep reduction ----
// Sum of weights (the reference's total_weight, invert.py:184) and max |w V|
// (sets the fixed-point scale): per-block partials come from the planner's
// place pass (cip_plan.hip); this reduces them in a fixed order.

// 1024 threads, 4 independent partial sums per thread (the loads of one
// thread are not serialised behind one accumulator); fixed order throughout.
__global__ __launch_bounds__(1024) void prep_final_kernel(const double* partial, int nblocks, double* out2) {
  double sum[4] = {0.0, 0.0, 0.0, 0.0}, mx = 0.0;
  for (int i0 = threadIdx.x; i0 < nblocks; i0 += 4 * 1024) {
    if (i0 + 3 * 1024 < nblocks) {
      // all 4 in range: the loads issue back to back (same order of sums)
      double2 p[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) p[k] = reinterpret_cast<const double2*>(partial)[i0 + k * 1024];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        sum[k] += p[k].x;
        mx = fmax(mx, p[k].y);
      }
      continue;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = i0 + k * 1024;
      if (i < nblocks) {
        const double2 p = reinterpret_cast<const double2*>(partial)[i];
        sum[k] += p.x;
        mx = fmax(mx, p.y);
      }
    }
  }
  double s = (sum[0] + sum[1]) + (sum[2] + sum[3]);
  for (int d = 32; d > 0; d >>= 1) {
    s += __shfl_xor(s, d, 64);
    mx = fmax(mx, __shfl_xor(mx, d, 64));
  }
  __shared__ double ss[16], sm[16];
  if ((threadIdx.x & 63) == 0) {
    ss[threadIdx.x >> 6] = s;
    sm[threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0, m = 0.0;
    for (int w = 0; w < 16; ++w) {
      t += ss[w];
      m = fmax(m, sm[w]);
    }
    out2[0] = t;
    out2[1] = m;
  }
}

hipError_t launch_prep_final(const double* partial, int nblocks, double* out2, hipStream_t s) {
  prep_final_kernel<<<dim3(1), dim3(1024), 0, s>>>(partial, nblocks, out2);
  return hipGetLastError();
}

// *dst += *src (one device scalar; the accumulating gridder's weight sum)
__global__ void add_scalar_kernel(const double* src, double* dst) {
  if (threadIdx.x == 0) *dst += *src;
}

hipError_t launch_add_scalar(const double* src, double* dst, hipStream_t s) {
  add_scalar_kernel<<<dim3(1), dim3(64), 0, s>>>(src, dst);
  return hipGetLastError();
}

// ------------------------------------------------------------ scatter ----
#ifndef CIP_SCATTER_WAVES
#define CIP_SCATTER_WAVES 4  // min waves per SIMD the scatter is compiled for (register budget)
#endif
constexpr int kScatterThreads = 256;
constexpr int kRunBatch = 256;

// Everything one visibility needs, loaded one iteration ahead of its use so
// the global-memory latency overlaps the previous visibility's taps.
struct VisFetch {
  double u, v, w, fx, vr, vi, wt;
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
__device__ __forceinline__ void fetch_at(int64_t irow, int64_t c, int64_t idx, const double* __restrict__ uvw,
                                         const double* __restrict__ fx, const VisT* __restrict__ vis,
                                         const void* __restrict__ wgt, VisFetch& f) {
  f.u = uvw[3 * irow];
  f.v = uvw[3 * irow + 1];
  f.w = uvw[3 * irow + 2];
  f.fx = fx[c];
  load_vis(vis, idx, f.vr, f.vi);
  f.wt = load_weight<WK>(wgt, idx);
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
  f.wt = load_weight<WK>(wgt, idx);
}

// The same, as loaded (complex64 / float32 kept in their own types): the
// position-ordered path converts only at use, so nothing waits for a load
// next to it and the loads of position q + 256 stay in flight while q grids.
template <typename VisT, int WK>
struct RawFetch {
  using WT = typename std::conditional<WK == WK_F64, double, float>::type;
  double u, v, w, fx;
  VisT vis;
  WT wt;
};

// Branch-free loads of MS visibility i (lanes with !ok load element 0; a PSF
// call, vis == NULL, reads its ignored visibility from uvw[0..1]).
template <typename VisT, int WK>
__device__ __forceinline__ void fetch_raw(int64_t i, bool ok, const double* __restrict__ uvw,
                                          const double* __restrict__ fx, const VisT* __restrict__ vis_ld,
                                          bool unit_vis, const void* __restrict__ wgt, const RowMap& m,
                                          RawFetch<VisT, WK>& f) {
  using WT = typename RawFetch<VisT, WK>::WT;
  const int64_t il = ok ? i : 0;
  int64_t r, c;
  vis_rowchan(m, il, &r, &c);
  f.u = uvw[3 * r];
  f.v = uvw[3 * r + 1];
  f.w = uvw[3 * r + 2];
  f.fx = fx[c];
  f.vis = vis_ld[unit_vis ? 0 : il];
  if constexpr (WK != WK_NONE) f.wt = ((const WT*)wgt)[il];
}

template <typename VisT, int WK>
__device__ __forceinline__ VisFetch from_raw(const RawFetch<VisT, WK>& r, bool unit_vis) {
  VisFetch f;
  f.u = r.u;
  f.v = r.v;
  f.w = r.w;
  f.fx = r.fx;
  f.vr = unit_vis ? 1.0 : (double)r.vis.x;
  f.vi = unit_vis ? 0.0 : (double)r.vis.y;
  f.wt = WK == WK_NONE ? 1.0 : (double)r.wt;
  return f;
}

template <int W, bool WSTACK, bool PACK>
__device__ __forceinline__ void grid_fetched(const VisFetch& f, const GridGeometry& g, int64_t plane, int64_t X0,
                                             int64_t Y0, double fixed_scale, unsigned long long* sub) {
  constexpr int T = kTile;
  constexpr int P = T + W - 1;
  if (f.wt == 0.0) return;
  int64_t ix0, iy0, iw0;
  double yu, yv, yw;
  if (!place_vis(f.u, f.v, f.w, f.fx, g, &ix0, &yu, &iy0, &yv, &iw0, &yw)) return;
  const int64_t lx = ix0 - X0, ly = iy0 - Y0;
  if (lx < 0 || lx >= T || ly < 0 || ly >= T) return;  // never for a consistent plan
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
#if CIP_ABLATE == 3
#pragma unroll
  for (int k = 0; k < W; ++k) {
    ku[k] = yu + (double)k;
    kv[k] = yv - (double)k;
  }
#else
  eval_kernel<W>(yu, ku);
  eval_kernel<W>(yv, kv);
#endif
  double kr[W], ki[W];
#pragma unroll
  for (int j = 0; j < W; ++j) {
    kr[j] = kv[j] * vr;
    ki[j] = kv[j] * vi;
  }
  // separate re / im planes: a lane-scattered 8-byte add touches 2 of the 64
  // LDS banks, so 8-byte cells spread a wave over twice the bank pairs that
  // interleaved 16-byte (re, im) cells would
#if CIP_ABLATE == 1
  unsigned long long* base = sub + ((threadIdx.x & 31) + ((threadIdx.x & 32) ? 8 * P : 0));
#else
  unsigned long long* base = sub + (lx * P + ly);
#endif
#if CIP_ABLATE == 2
  unsigned long long acc = 0;
#define atomicAdd(p, v) (acc += (v) ^ (unsigned long long)(p))
#endif
#pragma unroll
  for (int i = 0; i < W; ++i) {
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
#if CIP_ABLATE == 2
        hi = (unsigned)br + (unsigned)(bi >> 32) + (0u - kMagicHi);
#else
        asm("v_add3_u32 %0, %1, %2, %3" : "=v"(hi) : "v"((unsigned)br), "v"((unsigned)(bi >> 32)),
            "s"(0u - kMagicHi));
#endif
        atomicAdd(base + (i * P + j), __builtin_bit_cast(unsigned long long, make_uint2((unsigned)bi, hi)));
      } else {
        atomicAdd(base + (i * P + j), br - 0x4338000000000000ull);
        atomicAdd(base + P * P + (i * P + j), bi - 0x4338000000000000ull);
      }
    }
  }
#if CIP_ABLATE == 2
#undef atomicAdd
  if (acc == 0x123456789ull) sub[0] = acc;
#endif
}

// ------------------------------------------ bank-class visibility order ----
// A lane-scattered 8-byte LDS atomic hits bank pair (cell mod 32): 32 lanes
// whose footprints start on equal classes serialise (tools/microbench:
// 27 CU-cycles per visibility at random classes, 14 at distinct ones; the
// scatter with conflict-free addresses runs 1.7x faster, profiles/). The
// planner therefore stores, per chunk, the tile-order visibilities of each
// aligned window of kOrderBatch positions counting-sorted by class into
// level-major order (position = visibilities of lower rank in every class +
// lower classes of equal rank), so any 32 consecutive positions of a level
// have distinct classes and the scatter's waves (64 consecutive positions)
// issue conflict-free atomics. Level tables: S[r] = sum_c min(cnt[c], r),
// M[r] = {c : cnt[c] > r}. perm[g] = (row << 16) | channel. Atomic ranks make
// the order within a class run-to-run variable; the integer sums are not.
constexpr int kOrderThreads = 256;
constexpr int kOrderPer = 4;
constexpr int kOrderBatch = kOrderThreads * kOrderPer;
static_assert(kOrderBatch == kOrderWindow, "one order block per window");

// Bank class of a visibility's footprint origin in its tile's LDS sub-grid,
// recomputed from (u, v, f/c) with place_vis's arithmetic (fp contraction off,
// so it matches the scatter bit for bit; a mismatch would only cost a bank
// conflict, never a wrong sum).
__device__ __forceinline__ unsigned origin_class(double u_m, double v_m, double fx, const GridGeometry& g) {
#pragma clang fp contract(off)
  const int hw = g.support / 2;
  const int P = kTile + g.support - 1;
  const double x = (u_m * fx) * g.scale_u + (double)(g.nu / 2);
  const double y = (v_m * fx) * g.scale_v + (double)(g.nv / 2);
  int64_t ix0, iy0;
  double t0, t1;
  uv_origin(x, y, hw, g, &ix0, &t0, &iy0, &t1);
  return (unsigned)((((int)ix0 % kTile) * P + (int)iy0 % kTile) & 31);  // ix0, iy0 in [0, 2^31)
}

// One block per window (<= kOrderWindow consecutive tile-order positions).
// The window's row slices are staged in LDS with their rows' (u, v)
// (positions relative to the window start; the next window of the tile starts
// in its last slice), each thread finds the slice of its 4 positions by binary
// search, recomputes the bank class of each visibility (no per-visibility
// class array: a gathered byte per visibility cost more HBM lines than the
// whole perm stream) and the window is counting-sorted into level-major
// order: perm[g] = row * nchan + channel (32-bit flattened MS index).
template <bool GATHER>
__global__ __launch_bounds__(kOrderThreads, 8) void order_kernel(const double* __restrict__ uvw,
                                                              const double* __restrict__ fx,
                                                              const uint8_t* __restrict__ vis_class, GridGeometry g,
                                                              RowMap m, const uint64_t* __restrict__ runs,
                                                              const int64_t* __restrict__ run_goff,
                                                              const int64_t* __restrict__ tile_run_off,
                                                              const Chunk* __restrict__ windows, int64_t nwindows,
                                                              uint32_t* __restrict__ perm) {
  __shared__ __attribute__((aligned(16))) unsigned s_cnt[32];
  // the staged slices are dead once every position has its class: the level
  // tables reuse their space
  __shared__ union {
    struct {
      double2 uv[GATHER ? 1 : kOrderBatch];  // (u, v) of each slice's row (recompute only)
      uint64_t rec[kOrderBatch];
      int off[kOrderBatch + 1];  // slice starts relative to the window start
      uint16_t idx[kOrderBatch];  // slice of each position
    } a;
    struct {
      unsigned S[kOrderBatch], M[kOrderBatch];
    } b;
  } sh;
  double2* const s_uv = sh.a.uv;
  uint64_t* const s_rec = sh.a.rec;
  int* const s_off = sh.a.off;
  uint16_t* const s_idx = sh.a.idx;
  unsigned* const s_S = sh.b.S;
  unsigned* const s_M = sh.b.M;
  const Chunk ch = windows[blockIdx.x];
  const int64_t sb = ch.g0;
  const int nsb = (int)(ch.g1 - ch.g0);
  // the window's slices [first_run, last_run] (at most one per position)
  const int nst = (int)(ch.last_run - ch.first_run + 1);
  for (int k = threadIdx.x; k < nst; k += kOrderThreads) {
    s_off[k] = (int)(run_goff[ch.first_run + k] - sb);
    const uint64_t rec = runs[ch.first_run + k];
    s_rec[k] = rec;
    if constexpr (!GATHER) {
      const int64_t row = (int64_t)(rec >> 32);
      s_uv[k] = make_double2(uvw[3 * row], uvw[3 * row + 1]);
    }
  }
  if (threadIdx.x < 32) s_cnt[threadIdx.x] = 0u;
  __syncthreads();
  // expand: every position learns its slice (slices are <= 64 positions long)
  for (int k = threadIdx.x; k < nst; k += kOrderThreads) {
    const int a = s_off[k] > 0 ? s_off[k] : 0;
    const int b = k + 1 < nst ? s_off[k + 1] : nsb;
    for (int p = a; p < b; ++p) s_idx[p] = (uint16_t)k;
  }
  __syncthreads();
  uint32_t packed[kOrderPer];
  unsigned cls[kOrderPer], rk[kOrderPer];
  int slice[kOrderPer];
  int64_t chan[kOrderPer];
  // indices first, then the class loads back to back: one memory round trip
  // for the thread's positions instead of one each
#pragma unroll
  for (int k = 0; k < kOrderPer; ++k) {
    const int qi = threadIdx.x + k * kOrderThreads;
    if (qi < nsb) {
      const int lo = s_idx[qi];
      const uint64_t rec = s_rec[lo];
      const int64_t row = (int64_t)(rec >> 32);
      const int64_t c = (int64_t)((rec >> 16) & 0xffff) + (qi - s_off[lo]);
      packed[k] = (uint32_t)vis_index(m, row, c);
      slice[k] = lo;
      chan[k] = c;
    }
  }
#pragma unroll
  for (int k = 0; k < kOrderPer; ++k) {
    cls[k] = 32u;
    if (threadIdx.x + k * kOrderThreads < nsb) {
      if constexpr (GATHER) {
        cls[k] = vis_class[packed[k]];
      } else {
        const double2 uv = s_uv[slice[k]];
        cls[k] = origin_class(uv.x, uv.y, fx[chan[k]], g);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < kOrderPer; ++k)
    if (cls[k] < 32u) rk[k] = atomicAdd(&s_cnt[cls[k]], 1u);
  __syncthreads();
  unsigned maxcnt = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) maxcnt = s_cnt[i] > maxcnt ? s_cnt[i] : maxcnt;  // LDS broadcast reads
  for (unsigned r = threadIdx.x; r < maxcnt; r += kOrderThreads) {
    unsigned S = 0, M = 0;
#pragma unroll
    for (int c2 = 0; c2 < 32; ++c2) {
      const unsigned cnt = s_cnt[c2];
      S += cnt < r ? cnt : r;
      M |= (cnt > r ? 1u : 0u) << c2;
    }
    s_S[r] = S;
    s_M[r] = M;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kOrderPer; ++k)
    if (cls[k] < 32u) perm[sb + s_S[rk[k]] + __popc(s_M[rk[k]] & ((1u << cls[k]) - 1u))] = packed[k];
}

hipError_t launch_order(const double* uvw, const double* fx, const uint8_t* vis_class, const GridGeometry& g,
                        const RowMap& m, const uint64_t* runs, const int64_t* run_goff, const int64_t* tile_run_off,
                        const Chunk* windows, int64_t nwindows, uint32_t* perm, hipStream_t s) {
  if (nwindows <= 0) return hipSuccess;
  if (vis_class)
    order_kernel<true><<<dim3((unsigned)nwindows), dim3(kOrderThreads), 0, s>>>(
        uvw, fx, vis_class, g, m, runs, run_goff, tile_run_off, windows, nwindows, perm);
  else
    order_kernel<false><<<dim3((unsigned)nwindows), dim3(kOrderThreads), 0, s>>>(
        uvw, fx, vis_class, g, m, runs, run_goff, tile_run_off, windows, nwindows, perm);
  return hipGetLastError();
}

template <int W, typename VisT, int WK, bool WSTACK, bool PERM, bool PACK>
__global__ __launch_bounds__(kScatterThreads, CIP_SCATTER_WAVES) void scatter_kernel(
    const double* __restrict__ uvw, const double* __restrict__ fx, const VisT* __restrict__ vis,
    const void* __restrict__ wgt, RowMap m, const uint64_t* __restrict__ runs,
    const int64_t* __restrict__ run_goff, const int64_t* __restrict__ tile_run_off,
    const uint32_t* __restrict__ perm, const Chunk* __restrict__ chunks, int64_t chunk_begin, GridGeometry g,
    int64_t plane, double fixed_scale, double inv_scale, double* __restrict__ grid) {
  constexpr int T = kTile;
  constexpr int P = T + W - 1;
  __shared__ unsigned long long sub[P * P * (PACK ? 1 : 2)];
  __shared__ int64_t s_voff[PERM ? 1 : kRunBatch + 1];
  __shared__ uint64_t s_run[PERM ? 1 : kRunBatch];

  const Chunk ch = chunks[chunk_begin + blockIdx.x];
  const int64_t t = ch.tile;
  const int64_t X0 = (t % g.ntx) * T;
  const int64_t Y0 = ((t / g.ntx) % g.nty) * T;
  for (int i = threadIdx.x; i < P * P * (PACK ? 1 : 2); i += kScatterThreads) sub[i] = 0ull;
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
    int64_t qn = q + kScatterThreads;
    bool hn = qn < ch.g1;
    uint32_t pn = 0;
    if (have) {
      fetch_raw<VisT, WK>((int64_t)perm[q], true, uvw, fx, vis_ld, unit_vis, wgt, m, cur);
      pn = perm[hn ? qn : q];
    }
    while (have) {
      const int64_t qnn = qn + kScatterThreads;
      const bool hnn = qnn < ch.g1;
      const uint32_t pnn = perm[hnn ? qnn : q];
      RawFetch<VisT, WK> nxt;
      fetch_raw<VisT, WK>((int64_t)pn, hn, uvw, fx, vis_ld, unit_vis, wgt, m, nxt);
      grid_fetched<W, WSTACK, PACK>(from_raw<VisT, WK>(cur, unit_vis), g, plane, X0, Y0, fixed_scale, sub);
      cur = nxt;
      q = qn;
      have = hn;
      qn = qnn;
      hn = hnn;
      pn = pnn;
    }
  } else {
    const int64_t rb = tile_run_off[t + 1];
    int64_t r = ch.first_run;
    int64_t v = ch.g0;
    while (v < ch.g1 && r < rb) {
      const int nst = (int)((rb - r) < kRunBatch ? (rb - r) : kRunBatch);
      __syncthreads();
      for (int k = threadIdx.x; k <= nst; k += kScatterThreads) {
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
        const int64_t qn = q + kScatterThreads;
        const bool hn = qn < bend;
        VisFetch nxt;
        if (hn) fetch_vis<VisT, WK>(qn, s_voff, s_run, nst, uvw, fx, vis, wgt, m, nxt);
        grid_fetched<W, WSTACK, PACK>(cur, g, plane, X0, Y0, fixed_scale, sub);
        cur = nxt;
        q = qn;
        have = hn;
      }
      v = bend;
      r += nst;
    }
  }
  __syncthreads();
  // flush the touched cells of the sub-grid to the fp64 HBM grid
  // (lanes walk the HBM grid's contiguous axis: y, or x when it is stored
  // transposed for the pruned FFT)
  for (int cell = threadIdx.x; cell < P * P; cell += kScatterThreads) {
    const int lcell = g.transposed ? (cell % P) * P + cell / P : cell;  // lx * P + ly
    long long re, im;
    if constexpr (PACK) {
      const unsigned long long s = sub[lcell];
      im = (long long)(int)(unsigned)s;
      re = (long long)(int)(unsigned)((s - (unsigned long long)im) >> 32);
    } else {
      re = (long long)sub[lcell];
      im = (long long)sub[P * P + lcell];
    }
#if CIP_ABLATE == 4
    if (((re | im) != 0) && re == 0x123456789ll) {  // ablation: no flush (timing only)
#else
    if ((re | im) != 0) {
#endif
      // the sub-grid of an edge tile wraps around the periodic grid
      int64_t gx = X0 + lcell / P, gy = Y0 + lcell % P;
      gx -= (gx >= g.nu) ? g.nu : 0;
      gy -= (gy >= g.nv) ? g.nv : 0;
      double* dst = grid + 2 * (g.transposed ? gy * g.nu + gx : gx * g.nv + gy);
      unsafeAtomicAdd(dst, (double)re * inv_scale);
      unsafeAtomicAdd(dst + 1, (double)im * inv_scale);
    }
  }
}

template <int W, typename VisT, int WK>
static hipError_t scatter_dispatch_ws(bool ws, bool pack, dim3 grid_dim, hipStream_t s, const double* uvw,
                                      const double* fx, const void* vis, const void* wgt, const RowMap& m,
                                      const uint64_t* runs, const int64_t* run_goff, const int64_t* tile_run_off,
                                      const uint32_t* perm, const Chunk* chunks, int64_t chunk_begin,
                                      const GridGeometry& g, int64_t plane, double fs, double* grid) {
#define LAUNCH(WSV, PRM, PK)                                                                                   \
  scatter_kernel<W, VisT, WK, WSV, PRM, PK><<<grid_dim, dim3(kScatterThreads), 0, s>>>(                        \
      uvw, fx, (const VisT*)vis, wgt, m, runs, run_goff, tile_run_off, perm, chunks, chunk_begin, g, plane,     \
      fs, 1.0 / fs, grid)
#define LAUNCH_WS(PRM, PK)      \
  if (ws) LAUNCH(true, PRM, PK); \
  else LAUNCH(false, PRM, PK);
  // the packed single-precision class exists for complex64 input only (the
  // reference's configuration)
  bool done = false;
  if constexpr (std::is_same<VisT, float2>::value) {
    if (pack) {
      if (perm) {
        LAUNCH_WS(true, true)
      } else {
        LAUNCH_WS(false, true)
      }
      done = true;
    }
  }
  if (!done) {
    if (perm) {
      LAUNCH_WS(true, false)
    } else {
      LAUNCH_WS(false, false)
    }
  }
#undef LAUNCH_WS
#undef LAUNCH
  return hipGetLastError();
}

template <int W>
static hipError_t scatter_dispatch_w(int vis_dtype, int wgt_dtype, bool pack, dim3 gd, hipStream_t s,
                                     const double* uvw, const double* fx, const void* vis, const void* wgt,
                                     const RowMap& m, const uint64_t* runs, const int64_t* run_goff,
                                     const int64_t* tile_run_off, const uint32_t* perm, const Chunk* chunks,
                                     int64_t cb, const GridGeometry& g, int64_t plane, double fs, double* grid) {
  const bool ws = g.do_wstacking != 0;
#define ARGS \
  ws, pack, gd, s, uvw, fx, vis, wgt, m, runs, run_goff, tile_run_off, perm, chunks, cb, g, plane, fs, grid
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

hipError_t launch_scatter(int support, int vis_dtype, int wgt_dtype, bool packed, const double* uvw,
                          const double* fx, const void* vis, const void* wgt, const RowMap& m, const uint64_t* runs,
                          const int64_t* run_goff, const int64_t* tile_run_off, const uint32_t* perm,
                          const Chunk* chunks, int64_t chunk_begin, int64_t nchunks, const GridGeometry& g,
                          int64_t plane, double fixed_scale, double* grid, hipStream_t s) {
  if (nchunks <= 0) return hipSuccess;
  if (packed && vis_dtype != CIP_C64) return hipErrorInvalidValue;
  const dim3 gd((unsigned)nchunks);
#define CASE(WW)                                                                                             \
  case WW:                                                                                                   \
    return scatter_dispatch_w<WW>(vis_dtype, wgt_dtype, packed, gd, s, uvw, fx, vis, wgt, m, runs,           \
                                  run_goff, tile_run_off, perm, chunks, chunk_begin, g, plane, fixed_scale, grid);
  switch (support) {
    CASE(4)
    CASE(6)
    CASE(8)
    CASE(10)
    CASE(12)
    CASE(14)
    CASE(16)
    default:
      return hipErrorInvalidValue;
  }
#undef CASE
}

// ---------------------------------------------------- post-FFT kernels ----
// dirty[i, j] = (-1)^(p+q) Re G^[p mod nu, q mod nv] * cx[i] * cy[j],
// p = i - npix_x/2, q = j - npix_y/2; cx, cy = 1 / F(p/nu), 1 / F(q/nv).
__global__ void crop_correct_2d_kernel(const double2* __restrict__ grid, int64_t nu, int64_t nv, int64_t nx,
                                       int64_t ny, const double* __restrict__ cx, const double* __restrict__ cy,
                                       double* __restrict__ dirty) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = blockIdx.y;
  if (j >= ny) return;
  const int64_t p = i - nx / 2, q = j - ny / 2;
  const int64_t ip = (p + nu) % nu, iq = (q + nv) % nv;
  const double sgn = ((p + q) & 1) ? -1.0 : 1.0;
  dirty[i * ny + j] = sgn * grid[ip * nv + iq].x * cx[i] * cy[j];
}

hipError_t launch_crop_correct_2d(const double* grid, const GridGeometry& g, int64_t npix_x, int64_t npix_y,
                                  const double* cx, const double* cy, double* dirty, hipStream_t s) {
  crop_correct_2d_kernel<<<dim3((unsigned)((npix_y + 255) / 256), (unsigned)npix_x), dim3(256), 0, s>>>(
      (const double2*)grid, g.nu, g.nv, npix_x, npix_y, cx, cy, dirty);
  return hipGetLastError();
}

__device__ __forceinline__ double nm1_of(int64_t i, int64_t j, int64_t nx, int64_t ny, double px, double py) {
  const double l = (double)(i - nx / 2) * px;
  const double m = (double)(j - ny / 2) * py;
  const double e = l * l + m * m;
  return -e / (sqrt(1.0 - e) + 1.0);
}

// acc[i, j] (+)= (-1)^(p+q) Re(G^_p[..] exp(-2 pi i w_p (n - 1)))
__global__ void wplane_accumulate_kernel(const double2* __restrict__ grid, int64_t nu, int64_t nv, int64_t nx,
                                         int64_t ny, double px, double py, double w_plane, int first,
                                         double* __restrict__ acc) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = blockIdx.y;
  if (j >= ny) return;
  const int64_t p = i - nx / 2, q = j - ny / 2;
  const int64_t ip = (p + nu) % nu, iq = (q + nv) % nv;
  const double sgn = ((p + q) & 1) ? -1.0 : 1.0;
  const double nm1 = nm1_of(i, j, nx, ny, px, py);
  double sn, cs;
  sincospi(-2.0 * w_plane * nm1, &sn, &cs);
  const double2 gval = grid[ip * nv + iq];
  const double val = sgn * (gval.x * cs - gval.y * sn);
  if (first) acc[i * ny + j] = val;
  else acc[i * ny + j] += val;
}

hipError_t launch_wplane_accumulate(const double* grid, const GridGeometry& g, int64_t npix_x, int64_t npix_y,
                                    double pixsize_x, double pixsize_y, double w_plane, int first, double* acc,
                                    hipStream_t s) {
  wplane_accumulate_kernel<<<dim3((unsigned)((npix_y + 255) / 256), (unsigned)npix_x), dim3(256), 0, s>>>(
      (const double2*)grid, g.nu, g.nv, npix_x, npix_y, pixsize_x, pixsize_y, w_plane, first, acc);
  return hipGetLastError();
}

// acc *= cx[i] cy[j] / (F(dw |n-1|) n): F from a uniform table (cubic Lagrange).
__global__ void wfinal_correct_kernel(double* __restrict__ acc, int64_t nx, int64_t ny, double px, double py,
                                      const double* __restrict__ cx, const double* __restrict__ cy,
                                      const double* __restrict__ fw, int64_t fw_n, double fw_dnu, double dw) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = blockIdx.y;
  if (j >= ny) return;
  const double nm1 = nm1_of(i, j, nx, ny, px, py);
  const double t = fabs(dw * nm1) / fw_dnu;
  int64_t k = (int64_t)t;
  if (k < 1) k = 1;
  if (k > fw_n - 3) k = fw_n - 3;
  const double x = t - (double)k;  // in [-1, 2]
  const double f0 = fw[k - 1], f1 = fw[k], f2 = fw[k + 1], f3 = fw[k + 2];
  const double F = -x * (x - 1.0) * (x - 2.0) / 6.0 * f0 + (x + 1.0) * (x - 1.0) * (x - 2.0) / 2.0 * f1 -
                   (x + 1.0) * x * (x - 2.0) / 2.0 * f2 + (x + 1.0) * x * (x - 1.0) / 6.0 * f3;
  acc[i * ny + j] *= cx[i] * cy[j] / (F * (nm1 + 1.0));
}

hipError_t launch_wfinal_correct(double* acc, int64_t npix_x, int64_t npix_y, double pixsize_x, double pixsize_y,
                                 const double* cx, const double* cy, const double* fw_table, int64_t fw_n,
                                 double fw_dnu, double dw, hipStream_t s) {
  wfinal_correct_kernel<<<dim3((unsigned)((npix_y + 255) / 256), (unsigned)npix_x), dim3(256), 0, s>>>(
      acc, npix_x, npix_y, pixsize_x, pixsize_y, cx, cy, fw_table, fw_n, fw_dnu, dw);
  return hipGetLastError();
}

}  // namespace cip
