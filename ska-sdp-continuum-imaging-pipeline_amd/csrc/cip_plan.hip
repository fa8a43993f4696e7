// cip_plan.hip - device tile bucket/sort for the gridder (SURVEY.md 8(a) a8/a9,
// 8(f)): per-row runs of constant grid tile, counting sort of the runs by tile
// (histogram -> exclusive scan -> scatter), and the chunk table that splits hot
// tiles into <= kChunkVis-visibility work units (the role of split_tile,
// reference uvw_tiling/tile.py:155-211, for the device gridder).
#include "cip_internal.h"

namespace cip {

// ---------------------------------------------------------------- scan ----
constexpr int kScanThreads = 1024;
constexpr int kScanItems = 4;
constexpr int64_t kScanBlock = (int64_t)kScanThreads * kScanItems;

__global__ __launch_bounds__(kScanThreads) void scan_local_kernel(int64_t* data, int64_t n, int64_t* block_sums) {
  __shared__ int64_t wave_tot[kScanThreads / 64];
  const int64_t base = (int64_t)blockIdx.x * kScanBlock + (int64_t)threadIdx.x * kScanItems;
  int64_t v[kScanItems];
  int64_t tsum = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    v[i] = (base + i < n) ? data[base + i] : 0;
    tsum += v[i];
  }
  // inclusive wave scan of the thread sums
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t incl = tsum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int64_t o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  if (lane == 63) wave_tot[wave] = incl;
  __syncthreads();
  if (wave == 0) {
    int64_t t = (lane < kScanThreads / 64) ? wave_tot[lane] : 0;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      int64_t o = __shfl_up(t, d, 64);
      if (lane >= d) t += o;
    }
    if (lane < kScanThreads / 64) wave_tot[lane] = t;  // inclusive over waves
  }
  __syncthreads();
  int64_t run = incl - tsum + (wave > 0 ? wave_tot[wave - 1] : 0);
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    if (base + i < n) data[base + i] = run;
    run += v[i];
  }
  if (threadIdx.x == kScanThreads - 1) block_sums[blockIdx.x] = run;
}

__global__ void scan_add_kernel(int64_t* data, int64_t n, const int64_t* offsets) {
  const int64_t i = (int64_t)blockIdx.x * kScanBlock + threadIdx.x;
  const int64_t off = offsets[blockIdx.x];
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int64_t j = i + (int64_t)k * kScanThreads;
    if (j < n) data[j] += off;
  }
}

int64_t scan_tmp_elems(int64_t n) {
  int64_t total = 0;
  while (n > 1) {
    const int64_t nb = (n + kScanBlock - 1) / kScanBlock;
    total += nb;
    n = nb;
  }
  return total + 1;
}

hipError_t exclusive_scan_i64(int64_t* data, int64_t n, int64_t* tmp, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t nb = (n + kScanBlock - 1) / kScanBlock;
  scan_local_kernel<<<dim3((unsigned)nb), dim3(kScanThreads), 0, s>>>(data, n, tmp);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || nb == 1) return e;
  e = exclusive_scan_i64(tmp, nb, tmp + nb, s);
  if (e != hipSuccess) return e;
  scan_add_kernel<<<dim3((unsigned)nb), dim3(kScanThreads), 0, s>>>(data, n, tmp);
  return hipGetLastError();
}

// ------------------------------------------------------------ helpers ----
__global__ void freq_scale_kernel(const double* freq, int64_t nchan, double* fx) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < nchan) fx[c] = freq[c] / CIP_SPEED_OF_LIGHT;
}

hipError_t launch_freq_scale(const double* freq, int64_t nchan, double* fx, hipStream_t s) {
  freq_scale_kernel<<<dim3((unsigned)((nchan + 255) / 256)), dim3(256), 0, s>>>(freq, nchan, fx);
  return hipGetLastError();
}

// min / max of w * fx over rows and the two extreme channels
__global__ __launch_bounds__(256) void w_range_kernel(const double* uvw, int64_t nrow, double fxmin, double fxmax,
                                                      double* partial) {
  double lo = INFINITY, hi = -INFINITY;
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < nrow; r += (int64_t)gridDim.x * 256) {
    const double w = uvw[3 * r + 2];
    const double a = w * fxmin, b = w * fxmax;
    lo = fmin(lo, fmin(a, b));
    hi = fmax(hi, fmax(a, b));
  }
  for (int d = 32; d > 0; d >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, d, 64));
    hi = fmax(hi, __shfl_xor(hi, d, 64));
  }
  __shared__ double sl[4], sh[4];
  if ((threadIdx.x & 63) == 0) { sl[threadIdx.x >> 6] = lo; sh[threadIdx.x >> 6] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; ++i) { lo = fmin(lo, sl[i]); hi = fmax(hi, sh[i]); }
    partial[2 * blockIdx.x] = lo;
    partial[2 * blockIdx.x + 1] = hi;
  }
}

hipError_t launch_w_range(const double* uvw, int64_t nrow, double fxmin, double fxmax, double* partial,
                          int nblocks, hipStream_t s) {
  w_range_kernel<<<dim3(nblocks), dim3(256), 0, s>>>(uvw, nrow, fxmin, fxmax, partial);
  return hipGetLastError();
}

// ---------------------------------------------------------- planner ----
// A run is a maximal range of consecutive channels of one row with constant
// tile key (cf. the reference's row slices, tiling_plan.py:150-181). Each
// wave takes 64 consecutive flattened (row, channel) visibilities, one per
// lane: a lane starts a run when its key differs from the previous channel's
// (or at a row start or the wave's first lane), and the run ends at the next
// start in the wave (ballot), so runs are split at 64-visibility segment
// boundaries. The place pass is the only one that places visibilities: it
// counts runs per tile (one global atomic per run), parks each run in its
// segment's slots of a scratch array and records every visibility's LDS bank
// class for the order pass; the distribute pass moves the parked runs into
// their tile buckets.
__global__ __launch_bounds__(256) void plan_place_kernel(const double* __restrict__ uvw, int64_t nrow,
                                                         const double* __restrict__ fx, int64_t nchan,
                                                         GridGeometry g, int64_t* tile_runs, unsigned* err_flag,
                                                         uint8_t* __restrict__ vis_class,
                                                         uint8_t* __restrict__ seg_nruns,
                                                         int64_t* __restrict__ park_key,
                                                         uint64_t* __restrict__ park_run) {
  const int lane = threadIdx.x & 63;
  const int64_t nvis = nrow * nchan;
  const int64_t nseg = (nvis + 63) / 64;
  const int P = kTile + g.support - 1;
  for (int64_t seg = ((int64_t)blockIdx.x * 256 + threadIdx.x) / 64; seg < nseg;
       seg += (int64_t)gridDim.x * 4) {
    const int64_t i = seg * 64 + lane;
    const bool valid = i < nvis;
    int64_t key = -1, r = 0, c = 0;
    bool bad = false;
    if (valid) {
      // i / nchan through fp64 (exact after one correction for i < 2^52)
      r = (int64_t)((double)i / (double)nchan);
      c = i - r * nchan;
      if (c < 0) {
        --r;
        c += nchan;
      } else if (c >= nchan) {
        ++r;
        c -= nchan;
      }
      int64_t ix0, iy0, iw0;
      double yu, yv, yw;
      if (place_vis(uvw[3 * r], uvw[3 * r + 1], uvw[3 * r + 2], fx[c], g, &ix0, &yu, &iy0, &yv, &iw0, &yw)) {
        key = tile_key(ix0, iy0, iw0, g);
        vis_class[i] = (uint8_t)((((int)(ix0 % kTile)) * P + (int)(iy0 % kTile)) & 31);
      } else {
        bad = true;
        vis_class[i] = 0;
      }
    }
    if (__ballot(bad) != 0ull && lane == 0) atomicOr(err_flag, 1u);
    const int64_t prev = __shfl_up(key, 1, 64);
    const bool start = valid && (lane == 0 || c == 0 || key != prev);
    const unsigned long long starts = __ballot(start);
    const bool emit = start && key >= 0;
    const unsigned long long emits = __ballot(emit);
    const int nvalid = __popcll(__ballot(valid));  // wave-uniform: outside the branch
    if (lane == 0) seg_nruns[seg] = (uint8_t)__popcll(emits);
    if (emit) {
      const unsigned long long above = starts & ~((2ull << lane) - 1ull);  // lane 63: 2 << 63 == 0
      const int next = above ? (__ffsll((long long)above) - 1) : nvalid;
      const int slot = __popcll(emits & ((1ull << lane) - 1ull));
      park_key[seg * 64 + slot] = key;
      park_run[seg * 64 + slot] = ((uint64_t)r << 32) | ((uint64_t)c << 16) | (uint64_t)(c + (next - lane));
      atomicAdd((unsigned long long*)&tile_runs[key], 1ull);
    }
  }
}

__global__ __launch_bounds__(256) void plan_distribute_kernel(int64_t nseg, const uint8_t* __restrict__ seg_nruns,
                                                              const int64_t* __restrict__ park_key,
                                                              const uint64_t* __restrict__ park_run,
                                                              const int64_t* __restrict__ tile_run_off,
                                                              int64_t* tile_cursor, uint64_t* __restrict__ runs) {
  const int lane = threadIdx.x & 63;
  for (int64_t seg = ((int64_t)blockIdx.x * 256 + threadIdx.x) / 64; seg < nseg;
       seg += (int64_t)gridDim.x * 4) {
    if (lane < (int)seg_nruns[seg]) {
      const int64_t key = park_key[seg * 64 + lane];
      const int64_t pos = tile_run_off[key] + atomicAdd((unsigned long long*)&tile_cursor[key], 1ull);
      runs[pos] = park_run[seg * 64 + lane];
    }
  }
}

static unsigned plan_blocks(int64_t nvis) {
  const int64_t segs = (nvis + 63) / 64;
  const int64_t b = (segs + 3) / 4;
  return (unsigned)(b < 16384 ? (b > 0 ? b : 1) : 16384);
}

hipError_t launch_plan_place(const double* uvw, int64_t nrow, const double* fx, int64_t nchan,
                             const GridGeometry& g, int64_t* tile_runs, unsigned* err_flag, uint8_t* vis_class,
                             uint8_t* seg_nruns, int64_t* park_key, uint64_t* park_run, hipStream_t s) {
  plan_place_kernel<<<dim3(plan_blocks(nrow * nchan)), dim3(256), 0, s>>>(uvw, nrow, fx, nchan, g, tile_runs, err_flag,
                                                                         vis_class, seg_nruns, park_key, park_run);
  return hipGetLastError();
}

hipError_t launch_plan_distribute(int64_t nvis, const uint8_t* seg_nruns, const int64_t* park_key,
                                  const uint64_t* park_run, const int64_t* tile_run_off, int64_t* tile_cursor,
                                  uint64_t* runs, hipStream_t s) {
  const int64_t nseg = (nvis + 63) / 64;
  plan_distribute_kernel<<<dim3(plan_blocks(nvis)), dim3(256), 0, s>>>(nseg, seg_nruns, park_key, park_run,
                                                                      tile_run_off, tile_cursor, runs);
  return hipGetLastError();
}

__global__ void run_lengths_kernel(const uint64_t* runs, int64_t nruns, int64_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nruns) {
    const uint64_t rec = runs[i];
    out[i] = (int64_t)(rec & 0xffff) - (int64_t)((rec >> 16) & 0xffff);
  } else if (i == nruns) {
    out[i] = 0;
  }
}

hipError_t launch_run_lengths(const uint64_t* runs, int64_t nruns, int64_t* out, hipStream_t s) {
  run_lengths_kernel<<<dim3((unsigned)((nruns + 256) / 256)), dim3(256), 0, s>>>(runs, nruns, out);
  return hipGetLastError();
}

// tile_vis_off[t] = run_goff[tile_run_off[t]], tile_vis[t] = its difference
__global__ void tile_vis_kernel(const int64_t* run_goff, const int64_t* tile_run_off, int64_t ntiles,
                                int64_t* tile_vis_off, int64_t* tile_vis) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t > ntiles) return;
  const int64_t a = run_goff[tile_run_off[t]];
  tile_vis_off[t] = a;
  if (t < ntiles) tile_vis[t] = run_goff[tile_run_off[t + 1]] - a;
}

hipError_t launch_tile_vis(const int64_t* run_goff, const int64_t* tile_run_off, int64_t ntiles,
                           int64_t* tile_vis_off, int64_t* tile_vis, hipStream_t s) {
  tile_vis_kernel<<<dim3((unsigned)((ntiles + 256) / 256)), dim3(256), 0, s>>>(run_goff, tile_run_off, ntiles,
                                                                               tile_vis_off, tile_vis);
  return hipGetLastError();
}

__global__ void chunk_counts_kernel(const int64_t* tile_vis, int64_t ntiles, int64_t cv, int64_t* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < ntiles) out[t] = (tile_vis[t] + cv - 1) / cv;
  else if (t == ntiles) out[t] = 0;
}

hipError_t launch_chunk_counts(const int64_t* tile_vis, int64_t ntiles, int64_t chunk_vis, int64_t* out,
                               hipStream_t s) {
  chunk_counts_kernel<<<dim3((unsigned)((ntiles + 256) / 256)), dim3(256), 0, s>>>(tile_vis, ntiles, chunk_vis,
                                                                                   out);
  return hipGetLastError();
}

__global__ void chunk_emit_kernel(const int64_t* tile_vis_off, const int64_t* tile_vis, const int64_t* chunk_off,
                                  const int64_t* run_goff, const int64_t* tile_run_off, int64_t ntiles, int64_t cv,
                                  Chunk* chunks) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  const int64_t nv = tile_vis[t];
  const int64_t b = chunk_off[t];
  const int64_t g = tile_vis_off[t];
  int64_t lo = tile_run_off[t];
  const int64_t rend = tile_run_off[t + 1];
  for (int64_t k = 0; k * cv < nv; ++k) {
    Chunk ch;
    ch.g0 = g + k * cv;
    ch.g1 = g + ((k + 1) * cv < nv ? (k + 1) * cv : nv);
    ch.tile = t;
    // first run whose end lies beyond g0 (runs of a tile are consecutive)
    int64_t hi = rend - 1;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (run_goff[mid + 1] > ch.g0) hi = mid;
      else lo = mid + 1;
    }
    ch.first_run = lo;
    chunks[b + k] = ch;
  }
}

hipError_t launch_chunk_emit(const int64_t* tile_vis_off, const int64_t* tile_vis, const int64_t* chunk_off,
                             const int64_t* run_goff, const int64_t* tile_run_off, int64_t ntiles,
                             int64_t chunk_vis, Chunk* chunks, hipStream_t s) {
  chunk_emit_kernel<<<dim3((unsigned)((ntiles + 255) / 256)), dim3(256), 0, s>>>(
      tile_vis_off, tile_vis, chunk_off, run_goff, tile_run_off, ntiles, chunk_vis, chunks);
  return hipGetLastError();
}

__global__ void gather_kernel(const int64_t* src, int64_t stride, int64_t count, int64_t* dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) dst[i] = src[i * stride];
}

hipError_t launch_gather_i64(const int64_t* src, int64_t stride, int64_t count, int64_t* dst, hipStream_t s) {
  gather_kernel<<<dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s>>>(src, stride, count, dst);
  return hipGetLastError();
}

}  // namespace cip
