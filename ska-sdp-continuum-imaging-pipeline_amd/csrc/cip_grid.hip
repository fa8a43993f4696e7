// cip_grid.hip - the planner's order pass (bank-class order, SURVEY.md 8(a)
// a4.3), the support dispatch of the scatter (cip_scatter.h, a4.4) and the
// post-FFT crop / grid-correction / w-screen kernels (a4.5, a4.6).
#include <type_traits>

#include "cip_internal.h"

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
// M[r] = {c : cnt[c] > r}. perm[g] = the visibility's perm_encode entry
// (cip_common.h: flattened index, or (row << 16) | channel for ragged row
// slices). Atomic ranks make
// the order within a class run-to-run variable; the integer sums are not.
constexpr int kOrderThreads = 256;
constexpr int kOrderPer = kOrderWindow / kOrderThreads;
constexpr int kOrderBatch = kOrderThreads * kOrderPer;
static_assert(kOrderBatch == kOrderWindow, "one order block per window");

// One block per window (<= kOrderWindow consecutive tile-order positions).
// The window's row slices are staged in LDS (positions relative to the window
// start; the next window of the tile starts in its last slice), each thread
// finds the slice of its 4 positions, gathers the bank class the place pass
// stored for each visibility, and the window is counting-sorted into
// level-major order: perm[g] = perm_encode(row, channel). (Recomputing the
// classes here instead - from a uvw gather, or from fp32 (u, v) carried with
// each run through the radix sort - measured slower in rounds 2-5: the
// gathered class byte costs fewer lines than either.)
//
// Bank classes (round 6): 8-byte LDS atomics are banked like ds_write_b64 -
// four 16-lane groups, bank pair = element mod 16 (MI355X_MICROARCH.md, LDS) -
// so a class is the footprint origin's sub-grid element mod NC = 16 (32 in
// rounds 1-5; CIP_ORDER_CLASSES=32 for A/B).
// Row phases (PH: dense entries of < 2^31 visibilities, W <= 16): a
// visibility of phase 1 adds its footprint rows in the order 1, 2, .., W - 1,
// 0 instead of 0 .. W - 1 (cip_scatter.h rotate_rows / row_ptr), so at every
// tap but the last row's its bank pair is its class + dP (dP = P mod 16) - it
// behaves as class c + dP. The windows' class counts are skewed (the largest
// ~1.6x the mean), which leaves the level-major order's top levels with
// repeated classes in a 16-lane group; moving the excess of each class to its
// neighbour c + dP along the cycle c -> c + dP (a carry walk twice round, by
// wave 0 with a scalar carry) evens the
// effective counts. Host simulation of C3's windows under the 16-lane model
// (tools/sim_bank16.py): 1.74 LDS cycles per 16-lane tap for mod-32 classes,
// 1.58 mod 16, 1.27 mod 16 with phases. The phase rides in bit 31 of the entry.
template <int WIDE, bool PH, int NC = 16>
__global__ __launch_bounds__(kOrderThreads, 8) void order_kernel(const uint8_t* __restrict__ vis_class, RowMap m,
                                                                 const uint64_t* __restrict__ runs,
                                                                 const int64_t* __restrict__ run_goff,
                                                                 const Chunk* __restrict__ windows,
                                                                 void* __restrict__ perm, int dP) {
  __shared__ __attribute__((aligned(16))) unsigned s_cnt[32];
  __shared__ unsigned s_keep[PH ? NC : 1], s_eff[PH ? NC : 1];  // PH: phase-0 items / effective count per class
  // the staged slices are dead once every position has its class: the level
  // tables reuse their space
  __shared__ union {
    struct {
      uint64_t rec[kOrderBatch];
      int64_t delta[WIDE == 1 ? kOrderBatch : 1];  // ragged: delta[row] of each slice (index = delta + channel)
      int off[kOrderBatch + 1];  // slice starts relative to the window start
      uint16_t idx[kOrderBatch];  // slice of each position
    } a;
    struct {
      unsigned S[kOrderBatch], M[kOrderBatch];
    } b;
  } sh;
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
    if constexpr (WIDE == 2) {
      // packed ragged entries: the slice's first entry; position d of the
      // slice is that + d (index + d, channel + d); packed runs carry it
      if (m.pk_runs) {
        s_rec[k] = rec;
      } else {
        const int64_t row = (int64_t)(rec >> 32), c = (int64_t)((rec >> 16) & 0xffff);
        s_rec[k] = perm_encode_wide(m, m.delta[row] + c, row, c);
      }
    } else {
      s_rec[k] = rec;
    }
    if constexpr (WIDE == 1) sh.a.delta[k] = m.delta[(int64_t)(rec >> 32)];
  }
  if (threadIdx.x < NC) s_cnt[threadIdx.x] = 0u;
  __syncthreads();
  // expand: every position learns its slice (slices are <= 64 positions long)
  for (int k = threadIdx.x; k < nst; k += kOrderThreads) {
    const int a = s_off[k] > 0 ? s_off[k] : 0;
    const int b = k + 1 < nst ? s_off[k + 1] : nsb;
    for (int p = a; p < b; ++p) s_idx[p] = (uint16_t)k;
  }
  __syncthreads();
  using Entry = typename std::conditional<WIDE != 0, uint64_t, uint32_t>::type;
  const int pk_shift = m.pk_cbits + m.pk_rbits;  // WIDE == 2: entry = (index << pk_shift) | (row << cbits) | channel
  const uint64_t pk_step = WIDE == 2 ? (1ull << pk_shift) + 1ull : 0ull;
  Entry packed[kOrderPer];
  unsigned cls[kOrderPer], rk[kOrderPer];
  int slice[kOrderPer];
  int chan[kOrderPer];
  // indices first, then the class loads back to back: one memory round trip
  // for the thread's positions instead of one each
#pragma unroll
  for (int k = 0; k < kOrderPer; ++k) {
    const int qi = threadIdx.x + k * kOrderThreads;
    if (qi < nsb) {
      const int lo = s_idx[qi];
      const int d = qi - s_off[lo];
      if constexpr (WIDE == 2) {
        packed[k] = (Entry)(s_rec[lo] + (uint64_t)d * pk_step);
        chan[k] = (int)(packed[k] & ((1ull << m.pk_cbits) - 1ull));
      } else {
        const uint64_t rec = s_rec[lo];
        const int64_t row = (int64_t)(rec >> 32);
        const int64_t c = (int64_t)((rec >> 16) & 0xffff) + d;
        if constexpr (WIDE == 1) packed[k] = (Entry)perm_encode_wide(m, sh.a.delta[lo] + c, row, c);
        else packed[k] = (Entry)(row * m.nchan + c);
        chan[k] = (int)c;
      }
      slice[k] = lo;
    }
  }
#pragma unroll
  for (int k = 0; k < kOrderPer; ++k) {
    cls[k] = 32u;  // none (past the window)
    if (threadIdx.x + k * kOrderThreads < nsb)
      cls[k] = vis_class[WIDE == 2   ? (int64_t)((uint64_t)packed[k] >> pk_shift)
                         : WIDE == 1 ? sh.a.delta[slice[k]] + chan[k]
                                     : (int64_t)packed[k]] &
               (unsigned)(NC - 1);
  }
#pragma unroll
  for (int k = 0; k < kOrderPer; ++k)
    if (cls[k] < 32u) rk[k] = atomicAdd(&s_cnt[cls[k]], 1u);
  __syncthreads();
  const unsigned* cnt_of = s_cnt;  // the counts the level tables follow
  if constexpr (PH) {
    if (threadIdx.x < 64) {
      // wave 0: k_c = items of class c moved to c + dP, one carry walk along
      // the cycle c -> c + dP from class dP, twice round (where the walk
      // starts does not matter after two laps - host simulation), against the
      // mean count ceil(positions / NC); lane j < NC holds the j-th class of
      // the walk and its count
      const int lane = threadIdx.x;
      const unsigned mean = ((unsigned)nsb + (unsigned)NC - 1u) / (unsigned)NC;
      const int cw = ((lane + 1) * dP) & (NC - 1);
      const unsigned nw = lane < NC ? s_cnt[cw] : 0u;
      // the walk, unrolled over constant lanes (scalar carry; lap 2 final)
      unsigned kc = 0u, kw = 0u;
#pragma unroll
      for (int s2 = 0; s2 < 2 * NC; ++s2) {
        const unsigned n = (unsigned)__builtin_amdgcn_readlane((int)nw, s2 & (NC - 1));
        const unsigned e = n + kc;  // its own items and the carry from the class before
        kc = e > mean ? (e - mean < n ? e - mean : n) : 0u;
        if (s2 >= NC) kw = lane == (s2 & (NC - 1)) ? kc : kw;
      }
      // the carry into walk position j is position j - 1's
      const unsigned kin = (unsigned)__shfl((int)kw, (lane - 1) & (NC - 1), 64);
      if (lane < NC) {
        s_keep[cw] = nw - kw;
        s_eff[cw] = nw - kw + kin;
      }
    }
    __syncthreads();
    // each item's effective class and rank: the last k_c items of class c go
    // to c + dP after that class's own kept items
#pragma unroll
    for (int k = 0; k < kOrderPer; ++k)
      if (cls[k] < 32u) {
        const unsigned keep = s_keep[cls[k]];
        if (rk[k] >= keep) {
          const unsigned e = (cls[k] + (unsigned)dP) & (unsigned)(NC - 1);
          rk[k] = s_keep[e] + (rk[k] - keep);
          cls[k] = e;
          // the phase: bit 31 of a dense entry, bit 63 of a ragged one
          if constexpr (WIDE == 0) packed[k] = (Entry)((uint32_t)packed[k] | 0x80000000u);
          else packed[k] = (Entry)((uint64_t)packed[k] | 0x8000000000000000ull);
        }
      }
    cnt_of = s_eff;
  }
  unsigned maxcnt = 0;
#pragma unroll
  for (int i = 0; i < NC; ++i) maxcnt = cnt_of[i] > maxcnt ? cnt_of[i] : maxcnt;  // LDS broadcast reads
  for (unsigned r = threadIdx.x; r < maxcnt; r += kOrderThreads) {
    unsigned S = 0, M = 0;
#pragma unroll
    for (int c2 = 0; c2 < NC; ++c2) {
      const unsigned cnt = cnt_of[c2];
      S += cnt < r ? cnt : r;
      M |= (cnt > r ? 1u : 0u) << c2;
    }
    s_S[r] = S;
    s_M[r] = M;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kOrderPer; ++k)
    if (cls[k] < 32u) ((Entry*)perm)[sb + s_S[rk[k]] + __popc(s_M[rk[k]] & ((1u << cls[k]) - 1u))] = packed[k];
}

// CIP_ORDER_CLASSES=32: bank classes mod 32 (rounds 1-6) instead of mod 16 (A/B)
static bool order_classes32() {
  static const bool on = [] {
    const char* e = getenv("CIP_ORDER_CLASSES");
    return e && e[0] == '3';
  }();
  return on;
}

// Row phases apply when the entries have a bit to spare (bit 31 of dense
// entries, bit 63 of ragged ones - the packed (index, row, channel) form must
// leave it free) and the lane scatter's support gives a full cycle (dP = (T +
// W - 1) mod 16 odd)
bool order_phases_ok(const RowMap& m, int support) {
  auto bits = [](int64_t n) {
    int b = 1;
    while (b < 62 && ((int64_t)1 << b) < n) ++b;
    return b;
  };
  const int wide = m.delta == nullptr ? 0 : (m.pk_cbits ? 2 : 1);
  const bool spare = wide == 0 ? m.nvis < ((int64_t)1 << 31)
                               : (wide == 1 || m.pk_cbits + m.pk_rbits + bits(m.nvis) <= 63);
  const int nc = order_classes32() ? 32 : 16;
  const int dP = (kTile + support - 1) & (nc - 1);
  return spare && support >= 2 && support <= 16 && (dP & 1);
}

hipError_t launch_order(const uint8_t* vis_class, const RowMap& m, const uint64_t* runs, const int64_t* run_goff,
                        const Chunk* windows, int64_t nwindows, void* perm, hipStream_t s, int phase_support) {
  if (nwindows <= 0) return hipSuccess;
  if (!vis_class) return hipErrorInvalidValue;
#define ORDER(WI, PHV, NCV)                                                                                    \
  order_kernel<WI, PHV, NCV><<<dim3((unsigned)nwindows), dim3(kOrderThreads), 0, s>>>(vis_class, m, runs,     \
                                                                                      run_goff, windows, perm, dP)
  // ragged row slices: u64 entries (2: packed (index, row, channel))
  const int wide = m.delta == nullptr ? 0 : (m.pk_cbits ? 2 : 1);
  // 8-byte LDS atomics are banked like ds_write_b64 (MI355X_MICROARCH.md, LDS:
  // four 16-lane groups, bank pair = element mod 16), so the classes are the
  // footprint origin's element mod 16 (mod 32 before round 6)
  const bool c32 = order_classes32();
  const int nc = c32 ? 32 : 16;
  const int dP = (kTile + phase_support - 1) & (nc - 1);
  const bool ph = phase_support > 0 && order_phases_ok(m, phase_support);
  if (c32) {
    if (wide == 2 && ph) ORDER(2, true, 32);
    else if (wide == 2) ORDER(2, false, 32);
    else if (wide && ph) ORDER(1, true, 32);
    else if (wide) ORDER(1, false, 32);
    else if (ph) ORDER(0, true, 32);
    else ORDER(0, false, 32);
  } else {
    if (wide == 2 && ph) ORDER(2, true, 16);
    else if (wide == 2) ORDER(2, false, 16);
    else if (wide && ph) ORDER(1, true, 16);
    else if (wide) ORDER(1, false, 16);
    else if (ph) ORDER(0, true, 16);
    else ORDER(0, false, 16);
  }
#undef ORDER
  return hipGetLastError();
}

hipError_t launch_scatter(int support, int vis_dtype, int wgt_dtype, bool packed, int group, bool share_cus,
                          bool store_private, const double* uvw,
                          const double* fx, const void* vis, const void* wgt, const RowMap& m, const uint64_t* runs,
                          const int64_t* run_goff, const int64_t* tile_run_off, const void* perm,
                          const Chunk* chunks, int64_t chunk_begin, int64_t nchunks, const GridGeometry& g,
                          int64_t plane, double fixed_scale, double* grid, hipStream_t s) {
  if (nchunks <= 0) return hipSuccess;
  if (packed && vis_dtype != CIP_C64 && vis_dtype != CIP_POL4I) return hipErrorInvalidValue;
  const dim3 gd((unsigned)nchunks);
  // three blocks per CU: each needs > 160 KB / 4 of LDS (static sub-grid +
  // this pad); the 256-thread lane kernels only (plane groups run 512)
  unsigned pad = 0;
  if (share_cus && group == 1 && support <= 16) {
    const unsigned P = (unsigned)(kTile + support - 1);
    const unsigned stat = P * P * (packed ? 8u : 16u) + 64u;
    // 3 blocks per CU: the optimum of 2 / 3 / 4 (profiles/r03_ab_scatter_share.txt, r05z_ab_share_blocks.txt)
    const unsigned nb = 3u;
    const unsigned need = 160u * 1024u / (nb + 1u) + 256u;
    pad = stat < need ? need - stat : 0u;
  }
#define CASE(WW)                                                                                             \
  case WW:                                                                                                   \
    return launch_scatter_w<WW>(vis_dtype, wgt_dtype, packed, group, pad, store_private ? 1 : 0, gd, s, uvw, fx,  \
                                vis, wgt, m, runs, \
                                  run_goff, tile_run_off, perm, chunks, chunk_begin, g, plane, fixed_scale, grid);
  switch (support) {
    CASE(4)
    CASE(6)
    CASE(8)
    CASE(10)
    CASE(12)
    CASE(14)
    CASE(16)
#define LARGE(WW)                                                                                              \
  case WW:                                                                                                     \
    /* wave-per-visibility scatter (cip_scatter_large.hip); fp64 class, one plane per unit */                  \
    if (packed || group != 1) return hipErrorInvalidValue;                                                     \
    return launch_scatter_large_w<WW>(vis_dtype, wgt_dtype, gd, s, uvw, fx, vis, wgt, m, runs, run_goff, perm, \
                                      chunks, chunk_begin, g, plane, fixed_scale, grid);
    LARGE(24)
    LARGE(32)
    LARGE(48)
    LARGE(64)
#undef LARGE
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
// Image rows i0 + blockIdx.y (acc row blockIdx.y: a uv strip's image rows,
// DESIGN.md 7); norm (may be NULL): also / *norm (the weight sum).
// AT: the plane accumulator's type (double: in place, out == acc; float: the
// packed class's accumulator, corrected into the fp64 image `out`)
template <typename AT>
__global__ void wfinal_correct_kernel(const AT* __restrict__ acc, double* __restrict__ out, int64_t nx, int64_t ny,
                                      double px, double py, const double* __restrict__ cx,
                                      const double* __restrict__ cy, const double* __restrict__ fw, int64_t fw_n,
                                      double fw_dnu, double dw, int64_t i0, const double* __restrict__ norm) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = i0 + blockIdx.y;
  const AT* arow = acc + (int64_t)blockIdx.y * ny;
  double* row = out + (int64_t)blockIdx.y * ny;
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
  const double c = cx[i] * cy[j] / (F * (nm1 + 1.0));
  row[j] = (double)arow[j] * (norm ? c / *norm : c);
}

hipError_t launch_wfinal_correct(double* acc, int64_t npix_x, int64_t npix_y, double pixsize_x, double pixsize_y,
                                 const double* cx, const double* cy, const double* fw_table, int64_t fw_n,
                                 double fw_dnu, double dw, hipStream_t s, int64_t i0, int64_t nrows,
                                 const double* norm, const float* acc_f32) {
  if (nrows < 0) nrows = npix_x - i0;
  if (nrows <= 0) return hipSuccess;
  const dim3 gd((unsigned)((npix_y + 255) / 256), (unsigned)nrows);
  if (acc_f32)
    wfinal_correct_kernel<float><<<gd, dim3(256), 0, s>>>(acc_f32, acc, npix_x, npix_y, pixsize_x, pixsize_y, cx,
                                                          cy, fw_table, fw_n, fw_dnu, dw, i0, norm);
  else
    wfinal_correct_kernel<double><<<gd, dim3(256), 0, s>>>(acc, acc, npix_x, npix_y, pixsize_x, pixsize_y, cx, cy,
                                                           fw_table, fw_n, fw_dnu, dw, i0, norm);
  return hipGetLastError();
}

// ------------------------------------------- strip all-to-all packing ----
// The uv strips' sparse all-to-all moves pass-A rows in
// records: row y of block b of H (b, y, 4 columns) = `units` 16-byte units
// (4: complex128, 2: complex64). Pack: this rank's live rows, compacted
// (slot[y] >= 0: the row's place among them) - the send buffer, block-major,
// so each receiver's block range is contiguous. Unpack: a receiver's H from
// the received pieces, rec[y] = the record of row y's block 0 in recv (-1:
// no rank sent it, zeros), stride[y] = the records between its blocks (its
// source's live row count). One pass each, coalesced along the rows.
template <int UNITS>
__global__ __launch_bounds__(256) void strip_pack_kernel(const uint4* __restrict__ H, int64_t h,
                                                         const int64_t* __restrict__ slot, int64_t nlive,
                                                         uint4* __restrict__ out) {
  const int64_t b = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= h * UNITS) return;
  const int64_t y = i / UNITS, u = i % UNITS;  // UNITS: 2 or 4 (shifts)
  const int64_t k = slot[y];
  if (k >= 0) out[(b * nlive + k) * UNITS + u] = H[(b * h + y) * UNITS + u];
}

template <int UNITS>
__global__ __launch_bounds__(256) void strip_unpack_kernel(const uint4* __restrict__ recv, int64_t nv,
                                                           const int64_t* __restrict__ rec,
                                                           const int64_t* __restrict__ stride,
                                                           uint4* __restrict__ H) {
  const int64_t b = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nv * UNITS) return;
  const int64_t y = i / UNITS, u = i % UNITS;
  const int64_t r = rec[y];
  H[(b * nv + y) * UNITS + u] = r >= 0 ? recv[(r + b * stride[y]) * UNITS + u] : make_uint4(0u, 0u, 0u, 0u);
}

hipError_t launch_strip_pack(const void* H, int64_t nb, int64_t h, int units, const int64_t* slot, int64_t nlive,
                             void* out, hipStream_t s) {
  if (nb <= 0 || h <= 0 || nlive <= 0) return hipSuccess;
  const dim3 gd((unsigned)((h * units + 255) / 256), (unsigned)nb);
  if (units == 4)
    strip_pack_kernel<4><<<gd, dim3(256), 0, s>>>((const uint4*)H, h, slot, nlive, (uint4*)out);
  else
    strip_pack_kernel<2><<<gd, dim3(256), 0, s>>>((const uint4*)H, h, slot, nlive, (uint4*)out);
  return hipGetLastError();
}

hipError_t launch_strip_unpack(const void* recv, int64_t nb, int64_t nv, int units, const int64_t* rec,
                               const int64_t* stride, void* H, hipStream_t s) {
  if (nb <= 0 || nv <= 0) return hipSuccess;
  const dim3 gd((unsigned)((nv * units + 255) / 256), (unsigned)nb);
  if (units == 4)
    strip_unpack_kernel<4><<<gd, dim3(256), 0, s>>>((const uint4*)recv, nv, rec, stride, (uint4*)H);
  else
    strip_unpack_kernel<2><<<gd, dim3(256), 0, s>>>((const uint4*)recv, nv, rec, stride, (uint4*)H);
  return hipGetLastError();
}

}  // namespace cip
