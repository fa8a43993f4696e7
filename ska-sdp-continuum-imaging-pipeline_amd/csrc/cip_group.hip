// cip_group.hip - the grouped scatter: the visibilities of a work unit are
// grouped by the grid cell of their footprint origin and each group is
// accumulated in REGISTERS, so the LDS sub-grid sees one W x W flush per group
// instead of one per visibility (the hot loop of ducc0.wgridder.ms2dirty,
// SURVEY.md 8(a) a4.4, with its bucketing a4.3 fused in).
//
// Why: the lane-per-visibility scatter (cip_scatter.h) issues 2 W^2 64-bit LDS
// atomics per visibility and runs at ~90 % of the measured ds_add_u64 rate
// (DESIGN.md 5). In a 2048-position window of a 32 x 32 tile (C3) there are
// 0.31 distinct origin cells per visibility (short baselines' neighbouring
// channels and time steps pile onto the same cells), so grouping cuts the LDS
// atomics ~3x and the kernel moves to the vector ALU.
//
// One 256-thread workgroup per work unit (<= kChunkVis tile-order positions of
// one tile, the planner's chunk), processed in windows of <= 2048 positions
// and <= 512 row slices, everything in LDS:
//  1. stage the window's row slices (row, first channel, u, v) and map every
//     position to its slice;
//  2. place every position (the scatter's own fp64 arithmetic) -> origin cell;
//     its rank among the cell's positions in position order (wave w takes a
//     contiguous quarter of the window; ranks within a wave step by 10
//     ballots, a wave-private counter per cell, then a prefix over the waves):
//     deterministic;
//  3. items: a cell's n visibilities make n / kGroupCap full items and one
//     remainder item; items sorted by size, longest first (counting sort);
//     rounds of S items (S = 32 for W = 6, 8: two lanes per item; 64 for W = 4);
//     row t of a round holds the t-th visibility (rank order) of each slot's
//     item, padding past an item's end;
//  4. the waves walk their rounds (snake order over the longest-first table)
//     with one software pipeline (the global loads of step t + 1 in flight
//     while step t grids); a slot's lanes accumulate the item's W x W complex
//     footprint in fp64 registers (one fma per tap and component), and at the
//     round's end round each sum once to the 64-bit fixed-point quantum
//     (2^-46 of max |w V|, as the lane-per-visibility kernel's per-tap
//     rounding) and add it to the LDS sub-grid (ds_add_u64).
// After the unit the sub-grid goes to the fp64 HBM grid (global atomics), as
// in cip_scatter.h. Item composition and order follow the ranks, and the
// integer sums are order-independent: images are bit-reproducible.
//   W = 6, 8 (two lanes per item, slot s on lanes s and s + 32): lane h places
//   the visibility on axis h only (u or v), evaluates all W kernel pieces
//   there (coefficients in SGPRs), one v_permlane32_swap per dword gives every
//   lane both axes' values; lane h accumulates footprint rows hW/2 .. hW/2 + W/2 - 1.
//   W = 4 (one lane per item): all W rows.
#include "cip_internal.h"

namespace cip {

constexpr int kGThreads = 256;
constexpr int kGWaves = kGThreads / 64;
constexpr int kGWin = 2048;    // positions per window
constexpr int kGSlices = 512;  // row slices per window
constexpr int kGCells = kTile * kTile;
constexpr int kGPosWave = kGWin / kGWaves;
constexpr uint16_t kGEmpty = 0xffffu;
static_assert(kGWin / kGroupCap + kGCells <= 32 * kGroupMaxRounds, "round table");

// one grid axis: coordinate -> footprint origin (unwrapped, 32-bit: |origin|
// < 2^30 for every placed visibility, checked by the planner's place pass)
// and kernel variable, with place_vis's arithmetic (contraction off)
__device__ __forceinline__ void axis_place(double coord_m, double fx, double scale, int64_t n, int hw, int* o,
                                           double* y) {
#pragma clang fp contract(off)
  const double x = (coord_m * fx) * scale + (double)(n / 2);
  const double s = x - (double)hw;
  const double fl = floor(s);
  *y = 2.0 * (s - fl) - 1.0;
  *o = (int)fl + 1;
}

// element 0: the lower half-wave's value of this lane's slot, element 1: the upper's
__device__ __forceinline__ double swap_halves(double x, double* hi) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(x);
  const auto lo32 = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
  const auto hi32 = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
  *hi = __longlong_as_double((long long)(((unsigned long long)hi32[1] << 32) | lo32[1]));
  return __longlong_as_double((long long)(((unsigned long long)hi32[0] << 32) | lo32[0]));
}

// size of item idx (>= nfull): the remainder bins in descending size
__device__ __forceinline__ unsigned rem_item_size(unsigned idx, const unsigned* s_binoff, const unsigned* s_bin) {
  unsigned size = 0;
#pragma unroll
  for (int sz = 1; sz < kGroupCap; ++sz) size = (idx >= s_binoff[sz] && idx < s_binoff[sz] + s_bin[sz]) ? sz : size;
  return size;
}

// what one step of a slot needs from global memory
template <typename VisT, int WK>
struct GroupFetch {
  using WT = typename std::conditional<WK == WK_F64, double, float>::type;
  double fx;
  VisT vis;
  WT wt;
};

// A wave's position in its sequence of rounds (wave-uniform): round j of the
// wave (its table entry in lane j of `tab`), step t of the round's len steps.
struct RoundCursor {
  int j, t, len, row;
};

__device__ __forceinline__ void cursor_load(RoundCursor& c, uint32_t tab, int nr) {
  const uint32_t rec = c.j < nr ? (uint32_t)__builtin_amdgcn_readlane((int)tab, c.j) : 0u;
  c.len = (int)(rec & 255u);
  c.row = (int)(rec >> 8);
}

__device__ __forceinline__ void cursor_next(RoundCursor& c, uint32_t tab, int nr) {
  if (++c.t == c.len) {
    ++c.j;
    c.t = 0;
    cursor_load(c, tab, nr);
  }
}

template <int W, typename VisT, int WK>
__global__ __launch_bounds__(kGThreads, 2) void group_scatter_kernel(
    const double* __restrict__ uvw, const double* __restrict__ fx, const VisT* __restrict__ vis,
    const void* __restrict__ wgt, RowMap m, const uint64_t* __restrict__ runs, const int64_t* __restrict__ run_goff,
    const Chunk* __restrict__ chunks, int64_t chunk_begin, GridGeometry g, double fixed_scale, double inv_scale,
    double* __restrict__ grid) {
  using WT = typename GroupFetch<VisT, WK>::WT;
  constexpr int L = W >= 6 ? 2 : 1;  // lanes per item
  constexpr int S = 64 / L;          // items per round
  constexpr int R = W / L;           // footprint rows per lane
  constexpr int T = kTile;
  constexpr int P = T + W - 1;
  constexpr int ROWS = kGroupCap + kGWin / S;  // rows of a window's layout
  static_assert(W % L == 0 && W <= 8, "grouped scatter: W in {4, 6, 8}");
  __shared__ unsigned long long sub[2 * P * P];
  __shared__ double s_u[kGSlices], s_v[kGSlices];
  __shared__ uint32_t s_row[kGSlices];
  __shared__ int s_off[kGSlices];
  __shared__ uint16_t s_c0[kGSlices];
  __shared__ uint16_t s_idx[kGWin];   // slice of each position
  __shared__ uint16_t s_cell[kGWin];  // origin cell of each position
  __shared__ uint16_t s_rank[kGWin];  // rank among its cell's positions of its wave's quarter
  __shared__ uint16_t s_cntw[kGWaves][kGCells];  // per wave cell counts, then their prefix over waves
  __shared__ uint16_t s_n[kGCells], s_foff[kGCells], s_ridx[kGCells];
  __shared__ uint16_t s_lay[ROWS * S];
  __shared__ unsigned s_bin[kGroupCap], s_binoff[kGroupCap], s_bnext[kGroupCap];
  __shared__ unsigned s_nfull, s_fnext, s_nst;
  __shared__ int64_t s_wend, s_rnext;
  __shared__ uint32_t s_round[kGroupMaxRounds];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int slot = lane % S, h = lane / S;
  const int hw = W / 2;
  const int64_t ci = chunk_begin + blockIdx.x;
  const Chunk ch = chunks[ci];
  int64_t X0, Y0;
  tile_origin(ch.tile, g, &X0, &Y0);
  for (int i = tid; i < 2 * P * P; i += kGThreads) sub[i] = 0ull;
  const bool unit_vis = vis == nullptr;
  const VisT* vis_ld = unit_vis ? (const VisT*)uvw : vis;
  const double scale_h = h ? g.scale_v : g.scale_u;
  const int64_t n_h = h ? g.nv : g.nu;
  int64_t wstart = ch.g0, r0 = ch.first_run;
  while (wstart < ch.g1) {  // block-uniform
    __syncthreads();  // the previous window's LDS is free
    // ---- 1. the window's row slices
    const int nload = (int)((ch.last_run - r0 + 1) < kGSlices ? (ch.last_run - r0 + 1) : kGSlices);
    for (int k = tid; k < nload; k += kGThreads) {
      const int64_t go = run_goff[r0 + k] - wstart;
      s_off[k] = go < (int64_t)kGWin ? (int)go : kGWin;
      const uint64_t rec = runs[r0 + k];
      const int64_t row = (int64_t)(rec >> 32);
      s_row[k] = (uint32_t)row;
      s_c0[k] = (uint16_t)((rec >> 16) & 0xffff);
      s_u[k] = uvw[3 * row];
      s_v[k] = uvw[3 * row + 1];
    }
    for (int i = tid; i < kGWaves * kGCells / 2; i += kGThreads) ((unsigned*)&s_cntw[0][0])[i] = 0u;
    if (tid < kGroupCap) s_bin[tid] = s_bnext[tid] = 0u;
    if (tid == 0) {
      s_nfull = s_fnext = 0u;
      int64_t e = ch.g1 < wstart + kGWin ? ch.g1 : wstart + kGWin;
      if (r0 + kGSlices <= ch.last_run) {
        const int64_t lim = run_goff[r0 + kGSlices];
        e = lim < e ? lim : e;
      }
      s_wend = e;
    }
    __syncthreads();
    const int64_t wend = s_wend;
    const int npos = (int)(wend - wstart);
    if (tid == 0) {
      // slices starting before the window's end (offsets increase)
      int lo = 1, hi = nload;  // slice 0 holds position 0
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s_off[mid] < npos) lo = mid + 1;
        else hi = mid;
      }
      s_nst = (unsigned)lo;
      // the run holding wend starts the next window
      int64_t nx = r0 + lo - 1;
      if (r0 + lo <= ch.last_run && run_goff[r0 + lo] <= wend) nx = r0 + lo;
      s_rnext = nx;
    }
    __syncthreads();
    const int nst = (int)s_nst;
    for (int k = tid; k < nst; k += kGThreads) {
      const int lo = s_off[k] > 0 ? s_off[k] : 0;
      int hi = k + 1 < nst ? s_off[k + 1] : npos;
      hi = hi < npos ? hi : npos;
      for (int p = lo; p < hi; ++p) s_idx[p] = (uint16_t)k;
    }
    __syncthreads();
    // ---- 2. origin cells and stable ranks (wave w: positions [512 w, 512 w + 512))
    {
      constexpr int kSteps = kGPosWave / 64;
      double fxv[kSteps];
#pragma unroll
      for (int st = 0; st < kSteps; ++st) {  // the frequency loads back to back
        const int p = wave * kGPosWave + st * 64 + lane;
        fxv[st] = 0.0;
        if (p < npos) {
          const int k = s_idx[p];
          fxv[st] = fx[s_c0[k] + (p - s_off[k])];
        }
      }
#pragma unroll
      for (int st = 0; st < kSteps; ++st) {
        const int p = wave * kGPosWave + st * 64 + lane;
        const bool valid = p < npos;
        unsigned cell = 0u;
        if (valid) {
          const int k = s_idx[p];
          int ou, ov;
          double yu, yv;
          axis_place(s_u[k], fxv[st], g.scale_u, g.nu, hw, &ou, &yu);
          axis_place(s_v[k], fxv[st], g.scale_v, g.nv, hw, &ov, &yv);
          cell = (unsigned)(wrap_index32(ou, (int)g.nu) % kTile) * kTile + (unsigned)(wrap_index32(ov, (int)g.nv) % kTile);
        }
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 10; ++bit) {
          const bool on = (cell >> bit) & 1u;
          const unsigned long long mk = __ballot(on);
          peers &= on ? mk : ~mk;
        }
        if (valid) {
          const unsigned below = (unsigned)__popcll(peers & ((1ull << lane) - 1ull));
          const unsigned prior = s_cntw[wave][cell];
          if (below == 0u) s_cntw[wave][cell] = (uint16_t)(prior + (unsigned)__popcll(peers));
          s_cell[p] = (uint16_t)cell;
          s_rank[p] = (uint16_t)(prior + below);
        }
      }
    }
    __syncthreads();
    // ---- 3. items and rounds
    unsigned nf_t = 0;
    for (int c = tid; c < kGCells; c += kGThreads) {
      unsigned run = 0;
#pragma unroll
      for (int w = 0; w < kGWaves; ++w) {
        const unsigned a = s_cntw[w][c];
        s_cntw[w][c] = (uint16_t)run;
        run += a;
      }
      s_n[c] = (uint16_t)run;
      nf_t += run / kGroupCap;
      if (run % kGroupCap) atomicAdd(&s_bin[run % kGroupCap], 1u);
    }
    for (int d = 32; d > 0; d >>= 1) nf_t += __shfl_xor(nf_t, d, 64);
    if (lane == 0 && nf_t) atomicAdd(&s_nfull, nf_t);
    __syncthreads();
    if (tid == 0) {
      unsigned off = s_nfull;
      for (int sz = kGroupCap - 1; sz >= 1; --sz) {
        s_binoff[sz] = off;
        off += s_bin[sz];
      }
      s_binoff[0] = off;  // = number of items
    }
    __syncthreads();
    for (int c = tid; c < kGCells; c += kGThreads) {
      const unsigned n = s_n[c];
      const unsigned nf = n / kGroupCap, rem = n % kGroupCap;
      s_foff[c] = (uint16_t)(nf ? atomicAdd(&s_fnext, nf) : 0u);
      s_ridx[c] = (uint16_t)(rem ? s_binoff[rem] + atomicAdd(&s_bnext[rem], 1u) : 0u);
    }
    const unsigned nfull = s_nfull, nitems = s_binoff[0];
    const int nrounds = (int)((nitems + S - 1) / S);
    if (wave == 0) {
      unsigned len = 0;
      if (lane < nrounds) {
        const unsigned idx = (unsigned)lane * S;
        len = idx < nfull ? (unsigned)kGroupCap : rem_item_size(idx, s_binoff, s_bin);
      }
      unsigned incl = len;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const unsigned o = __shfl_up(incl, d, 64);
        if (lane >= d) incl += o;
      }
      if (lane < kGroupMaxRounds) s_round[lane] = ((incl - len) << 8) | len;
    }
    __syncthreads();
    // ---- layout: position -> (round, row, slot)
    for (int p = tid; p < npos; p += kGThreads) {
      const unsigned c = s_cell[p];
      const unsigned rank = (unsigned)s_cntw[p / kGPosWave][c] + s_rank[p];
      const unsigned piece = rank / kGroupCap, t = rank % kGroupCap;
      const unsigned idx = piece < (unsigned)s_n[c] / kGroupCap ? (unsigned)s_foff[c] + piece : (unsigned)s_ridx[c];
      s_lay[((s_round[idx / S] >> 8) + t) * S + idx % S] = (uint16_t)p;
    }
    for (int idx = tid; idx < nrounds * S; idx += kGThreads) {
      const unsigned size =
          (unsigned)idx < nfull ? (unsigned)kGroupCap : ((unsigned)idx < nitems ? rem_item_size(idx, s_binoff, s_bin) : 0u);
      const uint32_t rr = s_round[idx / S];
      for (unsigned t = size; t < (rr & 255u); ++t) s_lay[((rr >> 8) + t) * S + idx % S] = kGEmpty;
    }
    __syncthreads();
    // ---- 4. the rounds: wave's j-th is round 4j + wave (j even) or 4j + 3 - wave
    uint32_t tab = 0u;
    if (lane < kGroupMaxRounds / kGWaves) {
      const int k = kGWaves * lane + ((lane & 1) ? kGWaves - 1 - wave : wave);
      tab = k < nrounds ? s_round[k] : 0u;
    }
    const int nr = __popcll(__ballot((tab & 255u) != 0u));  // valid rounds are a prefix
    int total = (int)(tab & 255u);
    for (int d = 32; d > 0; d >>= 1) total += __shfl_xor(total, d, 64);
    total = __builtin_amdgcn_readfirstlane(total);
    double accr[R][W], acci[R][W];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < W; ++j) accr[i][j] = acci[i][j] = 0.0;
    unsigned item_cell = 0u;
    bool any = false;
    // the entry of a step and what it needs: its coordinate(s) from the staged
    // slice, the global loads
    auto entry = [&](const RoundCursor& c) -> unsigned {
      return c.j < nr ? (unsigned)s_lay[(c.row + c.t) * S + slot] : (unsigned)kGEmpty;
    };
    auto fetch = [&](unsigned e, double* ca, double* cb, GroupFetch<VisT, WK>& f) {
      const int p = e == kGEmpty ? 0 : (int)e;
      const int k = s_idx[p];
      const int64_t c = (int64_t)s_c0[k] + (p - s_off[k]);
      const int64_t i = e == kGEmpty ? 0 : vis_index(m, (int64_t)s_row[k], c);
      if constexpr (L == 2) {
        *ca = h ? s_v[k] : s_u[k];
      } else {
        *ca = s_u[k];
        *cb = s_v[k];
      }
      f.fx = fx[c];
      f.vis = vis_ld[unit_vis ? 0 : i];
      if constexpr (WK != WK_NONE) f.wt = ((const WT*)wgt)[i];
    };
    RoundCursor c0{0, 0, 0, 0};
    cursor_load(c0, tab, nr);
    RoundCursor c1 = c0;
    cursor_next(c1, tab, nr);
    // one step: issue step st + 1's loads into `nx`, then grid step st from
    // `cu` (loaded one step earlier: one step of compute hides the latency);
    // the loop is unrolled by two with the buffers swapped (no register copies,
    // which would make the compiler wait for the loads just issued)
    auto step = [&](unsigned& e_cu, GroupFetch<VisT, WK>& cu, double& a_cu, double& b_cu, unsigned& e_nx,
                    GroupFetch<VisT, WK>& nx, double& a_nx, double& b_nx) {
      e_nx = entry(c1);
      fetch(e_nx, &a_nx, &b_nx, nx);
      const bool ok = e_cu != kGEmpty;
      const double wt = WK == WK_NONE ? 1.0 : (double)cu.wt;
      const double sc = (ok && wt != 0.0) ? wt * fixed_scale : 0.0;
      const double vr = unit_vis ? 1.0 : (double)cu.vis.x, vi = unit_vis ? 0.0 : (double)cu.vis.y;
      const double ar = sc != 0.0 ? vr * sc : 0.0, ai = sc != 0.0 ? vi * sc : 0.0;
      item_cell = (ok && !any) ? (unsigned)s_cell[ok ? e_cu : 0u] : item_cell;
      any = any || ok;
      double ku[W], kv[W];
      if constexpr (L == 2) {
        int o;
        double y;
        axis_place(a_cu, cu.fx, scale_h, n_h, hw, &o, &y);
        double kk[W];
        eval_kernel<W>(ok ? y : 0.0, kk);
#pragma unroll
        for (int q = 0; q < W; ++q) ku[q] = swap_halves(kk[q], &kv[q]);
      } else {
        int o1, o2;
        double y1, y2;
        axis_place(a_cu, cu.fx, g.scale_u, g.nu, hw, &o1, &y1);
        axis_place(b_cu, cu.fx, g.scale_v, g.nv, hw, &o2, &y2);
        eval_kernel<W>(ok ? y1 : 0.0, ku);
        eval_kernel<W>(ok ? y2 : 0.0, kv);
      }
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const double kr = (L == 2 && h) ? ku[R + i] : ku[i];
        const double br = ar * kr, bi = ai * kr;
#pragma unroll
        for (int j = 0; j < W; ++j) {
          accr[i][j] = fma(br, kv[j], accr[i][j]);
          acci[i][j] = fma(bi, kv[j], acci[i][j]);
        }
      }
      if (c0.t == c0.len - 1) {  // wave-uniform: the round ends, its items go to the sub-grid
        if (any) {
          const int lx = (int)(item_cell / kTile), ly = (int)(item_cell % kTile);
          unsigned long long* base = sub + (lx + h * R) * P + ly;
#pragma unroll
          for (int i = 0; i < R; ++i)
#pragma unroll
            for (int j = 0; j < W; ++j) {
              // one rounding per item sum (|sum| < 2^51): + 1.5 * 2^52, the
              // integer is the low mantissa word; only the high word changes
              const unsigned long long br2 = (unsigned long long)__double_as_longlong(accr[i][j] + kMagic);
              const unsigned long long bi2 = (unsigned long long)__double_as_longlong(acci[i][j] + kMagic);
              atomicAdd(base + i * P + j, br2 - 0x4338000000000000ull);
              atomicAdd(base + P * P + i * P + j, bi2 - 0x4338000000000000ull);
            }
        }
#pragma unroll
        for (int i = 0; i < R; ++i)
#pragma unroll
          for (int j = 0; j < W; ++j) accr[i][j] = acci[i][j] = 0.0;
        any = false;
      }
      cursor_next(c0, tab, nr);
      cursor_next(c1, tab, nr);
    };
    unsigned eA = entry(c0), eB = kGEmpty;
    GroupFetch<VisT, WK> fA, fB;
    double aA = 0.0, bA = 0.0, aB = 0.0, bB = 0.0;
    fetch(eA, &aA, &bA, fA);
    for (int st = 0; st < total; st += 2) {
      step(eA, fA, aA, bA, eB, fB, aB, bB);
      if (st + 1 < total) step(eB, fB, aB, bB, eA, fA, aA, bA);
    }
    wstart = wend;
    r0 = s_rnext;
  }
  __syncthreads();
  // flush the touched cells of the sub-grid to the fp64 HBM grid (as
  // cip_scatter.h: lanes along the grid's contiguous axis)
  for (int cell = tid; cell < P * P; cell += kGThreads) {
    const int lcell = g.transposed ? (cell % P) * P + cell / P : cell;
    const long long re = (long long)sub[lcell], im = (long long)sub[P * P + lcell];
    if ((re | im) != 0) {
      int64_t gx = X0 + lcell / P, gy = Y0 + lcell % P;
      gx -= (gx >= g.nu) ? g.nu : 0;
      gy -= (gy >= g.nv) ? g.nv : 0;
      double* dst = grid + 2 * (g.transposed ? gy * g.nu + gx : gx * g.nv + gy);
      unsafeAtomicAdd(dst, (double)re * inv_scale);
      unsafeAtomicAdd(dst + 1, (double)im * inv_scale);
    }
  }
}

bool group_supported(int support) { return support == 4 || support == 6 || support == 8; }

template <int W>
static hipError_t group_scatter_w(int vis_dtype, int wgt_dtype, dim3 gd, hipStream_t s, const double* uvw,
                                  const double* fx, const void* vis, const void* wgt, const RowMap& m,
                                  const uint64_t* runs, const int64_t* run_goff, const Chunk* chunks, int64_t cb,
                                  const GridGeometry& g, double fs, double* grid) {
#define GLAUNCH(VT, WKV)                                                                                         \
  group_scatter_kernel<W, VT, WKV><<<gd, dim3(kGThreads), 0, s>>>(uvw, fx, (const VT*)vis, wgt, m, runs, run_goff, \
                                                                  chunks, cb, g, fs, 1.0 / fs, grid)
  if (vis_dtype == CIP_C64) {
    if (wgt_dtype == CIP_F32) GLAUNCH(float2, WK_F32);
    else if (wgt_dtype == CIP_F64) GLAUNCH(float2, WK_F64);
    else GLAUNCH(float2, WK_NONE);
  } else {
    if (wgt_dtype == CIP_F32) GLAUNCH(double2, WK_F32);
    else if (wgt_dtype == CIP_F64) GLAUNCH(double2, WK_F64);
    else GLAUNCH(double2, WK_NONE);
  }
#undef GLAUNCH
  return hipGetLastError();
}

hipError_t launch_group_scatter(int support, int vis_dtype, int wgt_dtype, const double* uvw, const double* fx,
                                const void* vis, const void* wgt, const RowMap& m, const uint64_t* runs,
                                const int64_t* run_goff, const Chunk* chunks, int64_t chunk_begin, int64_t nchunks,
                                const GridGeometry& g, double fixed_scale, double* grid, hipStream_t s) {
  if (nchunks <= 0) return hipSuccess;
  const dim3 gd((unsigned)nchunks);
#define GCASE(WW)                                                                                                 \
  case WW:                                                                                                        \
    return group_scatter_w<WW>(vis_dtype, wgt_dtype, gd, s, uvw, fx, vis, wgt, m, runs, run_goff, chunks,         \
                               chunk_begin, g, fixed_scale, grid);
  switch (support) {
    GCASE(4)
    GCASE(6)
    GCASE(8)
    default:
      return hipErrorInvalidValue;
  }
#undef GCASE
}

}  // namespace cip
