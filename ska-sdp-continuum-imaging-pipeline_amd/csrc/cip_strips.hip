// cip_strips.hip - the uv-strip split of the strong-scaling path (DESIGN.md 7,
// SURVEY.md 8(e) option 1) on the device: which grid rows each rank owns and
// which visibilities it grids. The reference's counterpart is its offline
// bucket step - uvw_tiling/tiling_plan.py:29-61 (tile keys and row runs) and
// reorder.py:19-111 (regrouping the visibilities by tile) - here cut by
// footprint-origin grid row instead of by uvw tile, so that a rank's share is
// a contiguous strip of grid rows.
//
// Three kernels, all of them one wave per MS row walking its channels 64 at a
// time (lane = channel), with the gridder's own fp64 placement (place_origin's
// operations and order, so a visibility lands in the strip its footprint
// starts in - bit for bit the planner's origin):
//  * strip_hist_kernel: per grid row, the visibilities whose footprint origin
//    lies in it and the row slices starting there (the cost model's inputs,
//    strips.row_costs); wave-segmented counts into a block-private LDS
//    histogram, per-block partials summed by strip_hist_reduce_kernel;
//  * strip_count_kernel: per MS row, the maximal channel runs whose origin row
//    lies in [y0, y1) and their visibilities (then two exclusive scans);
//  * strip_emit_kernel: the runs as Tile-layout row slices (uvw, channel
//    range, MS row) and the strip's visibilities and weights gathered into
//    slice order - the whole strip in one pass over the dense columns.
#include "cip_internal.h"

namespace cip {

// Footprint origin index along one axis: floor((c fx) s + n / 2 - W / 2) + 1
// wrapped into [0, n) (n a power of two), the gridder's placement arithmetic
// (cip_common.h place_origin / place_vis: the same fp64 operations, no
// contraction). Non-finite or huge coordinates give 0 (the planner rejects
// such visibilities when they are gridded).
__device__ __forceinline__ int64_t strip_origin(double c_m, double fx, double scale, int64_t n, int hw) {
#pragma clang fp contract(off)
  const double x = (c_m * fx) * scale + (double)(n / 2);
  const double fl = floor(x - (double)hw);
  const bool ok = fabs(fl) < 4.0e18;  // false for NaN / inf too
  const int64_t i = ok ? (int64_t)fl + 1 : 0;
  return i & (n - 1);
}

constexpr int kStripThreads = 1024;

// Block-private histograms (2 nv uint32 in dynamic LDS: visibilities, then
// slice starts, per footprint-origin grid row) over a grid-stride of MS rows,
// one wave per row. A slice starts at channel 0 and wherever the origin's
// 32-cell tile (iy / 32, ix / 32) changes along the channels (strips.py
// row_costs' key). Lanes of one wave with equal origin rows are counted by
// their segment head (consecutive channels mostly share a row), so the LDS
// atomics per 64 channels are the number of row changes, not 64.
__global__ __launch_bounds__(kStripThreads) void strip_hist_kernel(const double* __restrict__ uvw, int64_t nrow,
                                                                   const double* __restrict__ fx, int64_t nchan,
                                                                   int64_t nu, int64_t nv, double scale_u,
                                                                   double scale_v, int hw,
                                                                   uint32_t* __restrict__ partial) {
  extern __shared__ uint32_t s_h[];  // [0, nv): visibilities, [nv, 2 nv): slice starts
  for (int64_t k = threadIdx.x; k < 2 * nv; k += kStripThreads) s_h[k] = 0u;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * (kStripThreads / 64);
  const int64_t key_row = nu / 32 + 1;
  for (int64_t r = (int64_t)blockIdx.x * (kStripThreads / 64) + (threadIdx.x >> 6); r < nrow; r += waves) {
    const double u = uvw[3 * r], v = uvw[3 * r + 1];
    int64_t carry_key = -1;  // the previous chunk's last key (-1: row start)
    for (int64_t c0 = 0; c0 < nchan; c0 += 64) {
      const int64_t c = c0 + lane;
      const bool valid = c < nchan;
      const double f = fx[valid ? c : 0];
      const int64_t iy = strip_origin(v, f, scale_v, nv, hw);
      const int64_t ix = strip_origin(u, f, scale_u, nu, hw);
      const int64_t key = (iy >> 5) * key_row + (ix >> 5);
      int64_t prev = __shfl_up(key, 1, 64);
      if (lane == 0) prev = carry_key;
      const bool start = valid && (prev < 0 || key != prev);
      // segments of equal origin row: heads where the row differs from the
      // previous lane's (or lane 0); a head counts up to the next head
      const int64_t prev_iy = __shfl_up(iy, 1, 64);
      const bool head = valid && (lane == 0 || iy != prev_iy);
      const unsigned long long heads = __ballot(head);
      const unsigned long long starts = __ballot(start);
      const int nvalid = __popcll(__ballot(valid));
      if (head) {
        const unsigned long long above = heads & ~((2ull << lane) - 1ull);  // lane 63: 2 << 63 == 0
        const int next = above ? (__ffsll((long long)above) - 1) : nvalid;
        const unsigned long long seg = (next >= 64 ? ~0ull : ((1ull << next) - 1ull)) & ~((1ull << lane) - 1ull);
        atomicAdd(&s_h[iy], (uint32_t)(next - lane));
        const int ns = __popcll(starts & seg);
        if (ns) atomicAdd(&s_h[nv + iy], (uint32_t)ns);
      }
      carry_key = __shfl(key, 63, 64);
    }
  }
  __syncthreads();
  uint32_t* out = partial + (int64_t)blockIdx.x * 2 * nv;
  for (int64_t k = threadIdx.x; k < 2 * nv; k += kStripThreads) out[k] = s_h[k];
}

// hist[k] = sum over blocks of partial[b][k] (int64; k < 2 nv: the
// visibilities, then the slice starts, per grid row)
__global__ void strip_hist_reduce_kernel(const uint32_t* __restrict__ partial, int nblocks, int64_t n2,
                                         int64_t* __restrict__ hist) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n2) return;
  int64_t s = 0;
  for (int b = 0; b < nblocks; ++b) s += partial[(int64_t)b * n2 + k];
  hist[k] = s;
}

int strip_hist_blocks(int64_t nrow) {
  const int64_t b = (nrow + kStripThreads / 64 - 1) / (kStripThreads / 64);
  return (int)(b < 256 ? (b > 0 ? b : 1) : 256);
}

hipError_t launch_strip_hist(const double* uvw, int64_t nrow, const double* fx, int64_t nchan,
                             const GridGeometry& g, uint32_t* partial, int nblocks, int64_t* hist, hipStream_t s) {
  const size_t lds = sizeof(uint32_t) * 2 * (size_t)g.nv;
  if (lds > 160 * 1024 - 1024) return hipErrorInvalidValue;
  strip_hist_kernel<<<dim3(nblocks), dim3(kStripThreads), lds, s>>>(uvw, nrow, fx, nchan, g.nu, g.nv, g.scale_u,
                                                                    g.scale_v, g.support / 2, partial);
  const int64_t n2 = 2 * g.nv;
  strip_hist_reduce_kernel<<<dim3((unsigned)((n2 + 255) / 256)), dim3(256), 0, s>>>(partial, nblocks, n2, hist);
  return hipGetLastError();
}

// The runs of channels of row r whose origin row lies in [y0, y1), chunk by
// chunk: in = the channel's origin row inside the strip; a run starts where
// `in` rises and stops where it falls (or at the row's end).
struct StripWalk {
  int64_t runs = 0, vis = 0;  // before this chunk
  bool carry_in = false;      // the previous chunk's last channel was inside
};

__device__ __forceinline__ bool strip_in(double v, const double* __restrict__ fx, int64_t c, int64_t nchan,
                                         double scale_v, int64_t nv, int hw, int64_t y0, int64_t y1) {
  if (c >= nchan) return false;
  const int64_t iy = strip_origin(v, fx[c], scale_v, nv, hw);
  return iy >= y0 && iy < y1;
}

// row_runs[r] / row_vis[r]: the strip's runs and visibilities in MS row r
// (entry nrow: 0, so the exclusive scans' last entries are the totals)
__global__ __launch_bounds__(256) void strip_count_kernel(const double* __restrict__ uvw, int64_t nrow,
                                                          const double* __restrict__ fx, int64_t nchan, int64_t nv,
                                                          double scale_v, int hw, int64_t y0, int64_t y1,
                                                          int64_t* __restrict__ row_runs,
                                                          int64_t* __restrict__ row_vis) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r == nrow && lane == 0) {
    row_runs[nrow] = 0;
    row_vis[nrow] = 0;
  }
  if (r >= nrow) return;
  const double v = uvw[3 * r + 1];
  StripWalk w;
  for (int64_t c0 = 0; c0 < nchan; c0 += 64) {
    const bool in = strip_in(v, fx, c0 + lane, nchan, scale_v, nv, hw, y0, y1);
    const unsigned long long ins = __ballot(in);
    const unsigned long long rises = ins & ~((ins << 1) | (w.carry_in ? 1ull : 0ull));
    w.runs += __popcll(rises);
    w.vis += __popcll(ins);
    w.carry_in = (ins >> 63) & 1ull;
    if (c0 + 64 > nchan) w.carry_in = false;
  }
  if (lane == 0) {
    row_runs[r] = w.runs;
    row_vis[r] = w.vis;
  }
}

hipError_t launch_strip_count(const double* uvw, int64_t nrow, const double* fx, int64_t nchan,
                              const GridGeometry& g, int64_t y0, int64_t y1, int64_t* row_runs, int64_t* row_vis,
                              hipStream_t s) {
  strip_count_kernel<<<dim3((unsigned)(nrow / 4 + 1)), dim3(256), 0, s>>>(uvw, nrow, fx, nchan, g.nv, g.scale_v,
                                                                         g.support / 2, y0, y1, row_runs, row_vis);
  return hipGetLastError();
}

// The strip's row slices and its visibilities, from the scanned counts: slice
// k of row r (k-th rise of `in`) at run_off[r] + k with the row's uvw, the
// channel range and the MS row; its visibilities (and weights) copied to
// vis_off[r] + (the row's inside channels before them), in channel order -
// slices in (row, channel) order, the Tile layout of reference
// uvw_tiling/tile.py:14-124. VB / WB: bytes per visibility / weight (0: none).
template <int VB, int WB>
__global__ __launch_bounds__(256) void strip_emit_kernel(
    const double* __restrict__ uvw, int64_t nrow, const double* __restrict__ fx, int64_t nchan, int64_t nv,
    double scale_v, int hw, int64_t y0, int64_t y1, const int64_t* __restrict__ run_off,
    const int64_t* __restrict__ vis_off, const void* __restrict__ vis, const void* __restrict__ wgt,
    double* __restrict__ slice_uvw, int32_t* __restrict__ chan_start, int32_t* __restrict__ chan_stop,
    int64_t* __restrict__ slice_row, void* __restrict__ vis_out, void* __restrict__ wgt_out) {
  using VT = typename std::conditional<VB == 16, uint4, uint2>::type;
  using WT = typename std::conditional<WB == 8, uint64_t, uint32_t>::type;
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= nrow) return;
  const int64_t rb = run_off[r], vb = vis_off[r];
  if (run_off[r + 1] == rb) return;  // nothing of this row in the strip
  const double u = uvw[3 * r], v = uvw[3 * r + 1], w = uvw[3 * r + 2];
  StripWalk st;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int64_t c0 = 0; c0 < nchan; c0 += 64) {
    const int64_t c = c0 + lane;
    const bool in = strip_in(v, fx, c, nchan, scale_v, nv, hw, y0, y1);
    const unsigned long long ins = __ballot(in);
    const unsigned long long prev = (ins << 1) | (st.carry_in ? 1ull : 0ull);
    const unsigned long long rises = ins & ~prev;
    const unsigned long long falls = ~ins & prev;  // lane l: channel c0 + l is the first one outside
    if ((rises >> lane) & 1ull) {
      const int64_t k = rb + st.runs + __popcll(rises & below);
      slice_uvw[3 * k] = u;
      slice_uvw[3 * k + 1] = v;
      slice_uvw[3 * k + 2] = w;
      chan_start[k] = (int32_t)c;
      slice_row[k] = r;
    }
    if (((falls >> lane) & 1ull) && c <= nchan) {
      // the run that fell here is the last one started before this lane
      const int64_t k = rb + st.runs + __popcll(rises & below) - 1;
      chan_stop[k] = (int32_t)c;
    }
    if constexpr (VB > 0) {
      if (in) {
        const int64_t d = vb + st.vis + __popcll(ins & below);
        ((VT*)vis_out)[d] = ((const VT*)vis)[r * nchan + c];
        if constexpr (WB > 0) ((WT*)wgt_out)[d] = ((const WT*)wgt)[r * nchan + c];
      }
    }
    st.runs += __popcll(rises);
    st.vis += __popcll(ins);
    st.carry_in = (ins >> 63) & 1ull;
  }
  // a run still open at the row's end stops at nchan (when nchan is a
  // multiple of 64 no lane of the loop saw position nchan)
  if (nchan % 64 == 0 && st.carry_in && lane == 0) chan_stop[rb + st.runs - 1] = (int32_t)nchan;
}

hipError_t launch_strip_emit(const double* uvw, int64_t nrow, const double* fx, int64_t nchan, const GridGeometry& g,
                             int64_t y0, int64_t y1, const int64_t* run_off, const int64_t* vis_off, const void* vis,
                             int vis_bytes, const void* wgt, int wgt_bytes, double* slice_uvw, int32_t* chan_start,
                             int32_t* chan_stop, int64_t* slice_row, void* vis_out, void* wgt_out, hipStream_t s) {
  const dim3 gd((unsigned)((nrow + 3) / 4)), bd(256);
#define EMIT(VB, WB)                                                                                            \
  strip_emit_kernel<VB, WB><<<gd, bd, 0, s>>>(uvw, nrow, fx, nchan, g.nv, g.scale_v, g.support / 2, y0, y1,    \
                                              run_off, vis_off, vis, wgt, slice_uvw, chan_start, chan_stop,    \
                                              slice_row, vis_out, wgt_out)
  if (vis_bytes == 0) EMIT(0, 0);
  else if (vis_bytes == 8 && wgt_bytes == 0) EMIT(8, 0);
  else if (vis_bytes == 8 && wgt_bytes == 4) EMIT(8, 4);
  else if (vis_bytes == 8 && wgt_bytes == 8) EMIT(8, 8);
  else if (vis_bytes == 16 && wgt_bytes == 0) EMIT(16, 0);
  else if (vis_bytes == 16 && wgt_bytes == 4) EMIT(16, 4);
  else if (vis_bytes == 16 && wgt_bytes == 8) EMIT(16, 8);
  else return hipErrorInvalidValue;
#undef EMIT
  return hipGetLastError();
}

// A strip's dirty-tile bits for its masked pass A (cip_strip_rows_masked):
// the planner's own per-plane mask of the gridded strip (dirty_mask_kernel:
// every tile the scatter's flush may write), plus every tile of the tile rows
// holding buffer rows [0, halo) - grid rows row0 .. row0 + halo - 1 (mod nv),
// where the previous rank's halo is added after the gridding. dmask may be
// NULL (an empty strip). words = nty * (ntx / 32) per plane.
__global__ void strip_mask_kernel(const uint32_t* __restrict__ dmask, int64_t nplanes, int64_t nty, int64_t wpr,
                                  int64_t row0, int64_t halo, int64_t nv, uint32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nplanes * nty * wpr) return;
  const int64_t ty = (i / wpr) % nty;
  // tile rows of grid rows row0 .. row0 + halo - 1 (wrapping)
  const int64_t t0 = row0 / 32, t1 = (row0 + (halo > 0 ? halo : 1) - 1) / 32;  // unwrapped tile rows
  const int64_t nt = nv / 32;
  bool in_halo = false;
  for (int64_t t = t0; t <= t1; ++t) in_halo = in_halo || (t % nt) == ty;
  out[i] = (dmask ? dmask[i] : 0u) | (in_halo ? 0xffffffffu : 0u);
}

hipError_t launch_strip_mask(const uint32_t* dmask, const GridGeometry& g, int64_t row0, int64_t halo, uint32_t* out,
                             hipStream_t s) {
  const int64_t wpr = g.ntx / 32;
  const int64_t n = g.nplanes * g.nty * wpr;
  if (n <= 0) return hipSuccess;
  strip_mask_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s>>>(dmask, g.nplanes, g.nty, wpr, row0, halo,
                                                                          g.nv, out);
  return hipGetLastError();
}

}  // namespace cip
