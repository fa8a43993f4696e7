// cip_plan.hip - device tile bucket/sort for the gridder (SURVEY.md 8(a) a8/a9,
// 8(f)): per-row runs of constant grid tile, counting sort of the runs by tile
// (histogram -> exclusive scan -> scatter), and the chunk table that splits hot
// tiles into <= kChunkVis-visibility work units (the role of split_tile,
// reference uvw_tiling/tile.py:155-211, for the device gridder).
#include <type_traits>

#include "cip_internal.h"

namespace cip {

// ---------------------------------------------------------------- scan ----
constexpr int kScanThreads = 1024;
constexpr int kScanItems = 4;
constexpr int64_t kScanBlock = (int64_t)kScanThreads * kScanItems;

// RUNS: the input is the runs (n - 1 of them): item k is run k's length, item
// n - 1 is 0, and the scan goes to `data` (the fused run-length pass of the
// slice offsets); RUNS = 1: lengths from the run records (channel stop -
// start), 2: from the sort keys (RowMap::pk_runs: length - 1 in bits 26-31)
template <int RUNS>
__device__ __forceinline__ int64_t run_length_at(const void* __restrict__ src, int64_t k) {
  if constexpr (RUNS == 2) {
    return (int64_t)(((const uint32_t*)src)[k] >> kRunLenShift) + 1;
  } else {
    const uint64_t rec = ((const uint64_t*)src)[k];
    return (int64_t)(rec & 0xffff) - (int64_t)((rec >> 16) & 0xffff);
  }
}
template <int RUNS>
__global__ __launch_bounds__(kScanThreads) void scan_local_kernel(int64_t* data, int64_t n, int64_t* block_sums,
                                                                  const void* __restrict__ runs) {
  __shared__ int64_t wave_tot[kScanThreads / 64];
  const int64_t base = (int64_t)blockIdx.x * kScanBlock + (int64_t)threadIdx.x * kScanItems;
  int64_t v[kScanItems];
  int64_t tsum = 0;
  // threads with all their items in range load them unconditionally (the
  // loads issue back to back; a per-item branch waits for each in turn)
  if (base + kScanItems <= (RUNS ? n - 1 : n)) {
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
      if constexpr (RUNS) {
        v[i] = run_length_at<RUNS>(runs, base + i);
      } else {
        v[i] = data[base + i];
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < kScanItems; ++i) {
      if constexpr (RUNS) {
        v[i] = 0;
        if (base + i < n - 1) v[i] = run_length_at<RUNS>(runs, base + i);
      } else {
        v[i] = (base + i < n) ? data[base + i] : 0;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) tsum += v[i];
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
  if (i + (int64_t)(kScanItems - 1) * kScanThreads < n) {
    int64_t v[kScanItems];
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) v[k] = data[i + (int64_t)k * kScanThreads];
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) data[i + (int64_t)k * kScanThreads] = v[k] + off;
    return;
  }
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

static hipError_t scan_impl(int64_t* data, int64_t n, int64_t* tmp, const uint64_t* runs, hipStream_t s,
                            const uint32_t* run_keys = nullptr) {
  if (n <= 0) return hipSuccess;
  const int64_t nb = (n + kScanBlock - 1) / kScanBlock;
  if (run_keys)
    scan_local_kernel<2><<<dim3((unsigned)nb), dim3(kScanThreads), 0, s>>>(data, n, tmp, run_keys);
  else if (runs)
    scan_local_kernel<1><<<dim3((unsigned)nb), dim3(kScanThreads), 0, s>>>(data, n, tmp, runs);
  else
    scan_local_kernel<0><<<dim3((unsigned)nb), dim3(kScanThreads), 0, s>>>(data, n, tmp, nullptr);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || nb == 1) return e;
  e = scan_impl(tmp, nb, tmp + nb, nullptr, s);
  if (e != hipSuccess) return e;
  scan_add_kernel<<<dim3((unsigned)nb), dim3(kScanThreads), 0, s>>>(data, n, tmp);
  return hipGetLastError();
}

hipError_t exclusive_scan_i64(int64_t* data, int64_t n, int64_t* tmp, hipStream_t s) {
  return scan_impl(data, n, tmp, nullptr, s);
}

hipError_t scan_run_offsets(const uint64_t* runs, int64_t nruns, int64_t* run_goff, int64_t* tmp, hipStream_t s,
                            const uint32_t* run_keys) {
  return scan_impl(run_goff, nruns + 1, tmp, runs, s, run_keys);
}

// ------------------------------------------------------------ helpers ----
// fx = f / c; err bit 2 (value 4) when a frequency is not finite and positive
__global__ void freq_scale_kernel(const double* freq, int64_t nchan, double* fx, unsigned* err) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < nchan) {
    const double f = freq[c];
    fx[c] = f / CIP_SPEED_OF_LIGHT;
    if (err && !(f > 0.0 && isfinite(f))) atomicOr(err, 4u);
  }
}

hipError_t launch_freq_scale(const double* freq, int64_t nchan, double* fx, unsigned* err, hipStream_t s) {
  freq_scale_kernel<<<dim3((unsigned)((nchan + 255) / 256)), dim3(256), 0, s>>>(freq, nchan, fx, err);
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
// boundaries. The place pass parks each run with its tile key in its block's
// slots of a scratch array and counts the keys' low bytes (the histogram of
// radix pass 0, written digit-major). The runs are then bucketed by tile with a stable LSD radix sort (8-bit digits, no
// global atomics: scattered device-scope atomics execute at the memory side
// at ~10-25 G/s on MI355X, which made an atomic counting sort of the 13 M
// runs of C3 cost more than 1 ms).
constexpr int kPlaceSegs = 64;  // 64-visibility segments per place block (4096 visibilities)

// lane i <- lane i - 1 of the wave (lane 0 <- 0): one DPP move
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138 /* wave_shr:1 */, 0xf, 0xf, false);
}
constexpr uint32_t kNoKey = 0xffffffffu;  // visibility off the grid (tile keys are < 2^32 - 1)

// PLACE = false: only the fused reduction (sum of weights, max |w V|,
// non-finite check), in exactly the place pass's order - a call that reuses
// its predecessor's plan (CIP_REUSE_PLAN) gets the same sums bit for bit.
// blk / nblocks: this place block and their count.
// RM: the row map, at compile time (each mode's registers only): 0 dense MS
// rows, 1 dense rows of a multiple of 64 channels (every wave's 64
// visibilities are channels of ONE row: the row, its uvw and the run
// detection's row check are wave-uniform - scalar registers and loads), 2
// ragged row slices
template <typename VisT, int WK, bool PLACE, int RM>
__device__ __forceinline__ void place_body(const double* __restrict__ uvw, const double* __restrict__ fx,
                                           const RowMap& m, const VisT* __restrict__ vis,
                                           const void* __restrict__ wgt, const GridGeometry& g, unsigned* err_flag,
                                           uint8_t* __restrict__ vis_class, int64_t* __restrict__ blk_cnt,
                                           uint32_t* __restrict__ park_key, uint64_t* __restrict__ park_run,
                                           double* partial, int64_t* __restrict__ hist0, const int64_t blk,
                                           const int64_t nblocks) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  __shared__ unsigned s_nruns;
  __shared__ unsigned s_hist[256];
  if (threadIdx.x == 0) s_nruns = 0u;
  s_hist[threadIdx.x] = 0u;
  __syncthreads();
  // fused prep reduction (sum of weights, max |w V|), fixed order
  double wsum = 0.0, wvmax = 0.0;
  bool nonfinite = false;
  bool bad_any = false;  // a placement failed (reported once, after the loop)
  const int64_t nvis = m.nvis, nchan = m.nchan;
  constexpr bool ragged = RM == 2;
  constexpr bool rowwave = RM == 1;
  const int64_t nseg = (nvis + 63) / 64;
  const int P = kTile + g.support - 1;
  // block b owns segments [64 b, 64 b + 64): wave w takes every 4th
  const int64_t seg_end = (blk + 1) * kPlaceSegs < nseg ? (blk + 1) * kPlaceSegs : nseg;
  // (row, channel) of the lane's visibility, advanced by 256 visibilities per
  // step without a division
  // (ragged rows: from the segment's first row, ragged_row_of)
  int64_t r0 = 0, c0 = 0;
  if (rowwave) {
    // the wave's row and first channel (wave-uniform: the lane adds its own)
    const int64_t i0 = (blk * kPlaceSegs + wave) * 64;
    r0 = i0 / nchan;
    c0 = i0 - r0 * nchan;
  } else if (!ragged) {
    split_index64((blk * kPlaceSegs + wave) * 64 + lane, nchan, m.inv_nchan, &r0, &c0);
  }
  const int64_t step_r = 256 / nchan, step_c = 256 % nchan;
  // ragged rows: the first rows of the wave's kPlaceSegs / 4 segments and the
  // starts of the rows after them, loaded once (lane j: segment j), so the
  // loop's row lookup is a register read, not a chain of dependent loads
  static_assert(kPlaceSegs / 4 <= 64, "one lane per segment of the wave");
  int seg_s = 0;
  int64_t seg_nx = 0, seg_dl = 0;
  if (ragged) {
    const int64_t sj = blk * kPlaceSegs + wave + 4 * (int64_t)lane;
    if (lane < kPlaceSegs / 4 && sj < seg_end) {
      const uint32_t s0 = m.seg_row[sj];  // rows < 2^32
      seg_s = (int)s0;
      seg_nx = m.off[(int64_t)s0 + 1];
      seg_dl = m.delta[s0];
    }
  }
  int it = 0;
  for (int64_t seg = blk * kPlaceSegs + wave; seg < seg_end; seg += 4, ++it) {
    const int64_t i = seg * 64 + lane;
    // rowwave: nvis = nrow nchan is a multiple of 64, every segment is whole
    const bool valid = rowwave ? true : i < nvis;
    int64_t r = r0, c = rowwave ? c0 + lane : c0;
    // lanes past the end load index 0's data (no divergent branch around the
    // loads); their results are masked by `valid`
    const int64_t il = valid ? i : 0;
    if (ragged) {
      const int64_t s = (int64_t)(uint32_t)__builtin_amdgcn_readlane(seg_s, it);
      const int64_t nx = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(seg_nx >> 32), it) << 32) |
                                   (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)seg_nx, it));
      const int64_t ilast = seg * 64 + 63 < nvis ? seg * 64 + 63 : nvis - 1;
      if (nx > ilast) {  // the segment inside row s (uniform): its delta is prefetched too
        const int64_t dl = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(seg_dl >> 32), it) << 32) |
                                     (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)seg_dl, it));
        r = s;
        c = il - dl;
      } else {
        r = ragged_row_of(m, s, nx, ilast, i);
        c = il - m.delta[r];
      }
    } else {
      c0 += step_c;
      r0 += step_r;
      if (c0 >= nchan) {
        c0 -= nchan;
        ++r0;
      }
    }
    const int64_t rl = valid ? r : 0, cl = valid ? c : 0;
    // position loads first: the visibility load of a PSF call is a branch,
    // and the wait inside it then covers every load (one memory round trip)
    double u = 0.0, v = 0.0, w = 0.0, f = 0.0;
    if constexpr (PLACE) {
      u = uvw[3 * rl];
      v = uvw[3 * rl + 1];
      if (g.do_wstacking) w = uvw[3 * rl + 2];  // (uniform)
      f = fx[cl];
    }
    {
      const double wt = load_weight<WK>(wgt, m, il);
      double vr, vi;
      load_vis(vis, il, vr, vi);
      // zero-weight visibilities are skipped by the scatter, whatever they hold
      const bool counted = valid & (wt != 0.0);
      const double a = counted ? fabs(wt) * fmax(fabs(vr), fabs(vi)) : 0.0;
      nonfinite = nonfinite | (counted && !(isfinite(wt) && isfinite(vr) && isfinite(vi)));
      wsum = valid ? wsum + wt : wsum;
      wvmax = fmax(wvmax, a);
    }
    if constexpr (PLACE) {
      int ix0, iy0;
      int64_t iw0;
      const bool ok = place_origin(u, v, w, f, g, &ix0, &iy0, &iw0);
      // a w layer feeds planes [iw0, iw0 + W): dropped when none is in the
      // call's plane range (plane groups split over GPUs; 2-D: the one plane)
      bool feeds = true;
      if (g.do_wstacking) feeds = (iw0 + g.support > g.plane_lo) & (iw0 < g.plane_hi);
      // the tile key modulo 2^32 (keys are < 2^32 - 1)
      // tile_key(): tile-major, the w layers of a uv tile adjacent
      const uint32_t key = (valid & ok & feeds) ? ((((uint32_t)iy0 / (uint32_t)kTile) * (uint32_t)g.ntx +
                                            (uint32_t)ix0 / (uint32_t)kTile) *
                                               (uint32_t)g.ntw +
                                           (uint32_t)iw0)
                                        : kNoKey;
      bad_any = bad_any | (valid & !ok);
      // the bank class ((ix0 % T) P + iy0 % T) % 32 (T = 32)
      if (vis_class && valid)
        vis_class[i] = ok ? (uint8_t)(((unsigned)ix0 * (unsigned)P + (unsigned)iy0) & 31u) : (uint8_t)0;
      // the previous lane's key and row: DPP wave_shr:1 (a VALU move; __shfl_up
      // is an LDS ds_bpermute with its own latency); lane 0 is a start anyway
      const uint32_t prev = wave_shr1(key);
      bool start;
      if constexpr (rowwave) {
        start = lane == 0 || key != prev;  // one row per wave
      } else {
        const uint32_t prev_r = wave_shr1((uint32_t)r);  // rows < 2^32
        start = valid && (lane == 0 || (uint32_t)r != prev_r || key != prev);
      }
      const unsigned long long starts = __ballot(start);
      const bool emit = start && key != kNoKey;
      const unsigned long long emits = __ballot(emit);
      const int nvalid = __popcll(__ballot(valid));  // wave-uniform: outside the branch
      // the block's runs are parked densely from slot 64 * kPlaceSegs * b on
      unsigned wbase = 0;
      if (lane == 0 && emits) wbase = atomicAdd(&s_nruns, (unsigned)__popcll(emits));
      wbase = (unsigned)__builtin_amdgcn_readlane((int)wbase, 0);  // lane 0's slot base (scalar)
      if (emit) {
        const unsigned long long above = starts & ~((2ull << lane) - 1ull);  // lane 63: 2 << 63 == 0
        const int next = above ? (__ffsll((long long)above) - 1) : nvalid;
        const int64_t slot = blk * kPlaceSegs * 64 + wbase + __popcll(emits & ((1ull << lane) - 1ull));
        atomicAdd(&s_hist[key & 255u], 1u);
        if (ragged && m.pk_runs) {  // wave-uniform
          park_key[slot] = key | ((uint32_t)(next - lane - 1) << kRunLenShift);
          park_run[slot] = perm_encode_wide(m, i, r, c);
        } else {
          park_key[slot] = key;
          park_run[slot] = ((uint64_t)r << 32) | ((uint64_t)c << 16) | (uint64_t)(c + (next - lane));
        }
      }
    }
  }
  __shared__ double ss[4], sm[4];
  {
    if (nonfinite) atomicOr(err_flag, 2u);
    if (bad_any) atomicOr(err_flag, 1u);
    for (int d = 32; d > 0; d >>= 1) {
      wsum += __shfl_xor(wsum, d, 64);
      wvmax = fmax(wvmax, __shfl_xor(wvmax, d, 64));
    }
    if (lane == 0) {
      ss[threadIdx.x >> 6] = wsum;
      sm[threadIdx.x >> 6] = wvmax;
    }
  }
  __syncthreads();
  if constexpr (PLACE) hist0[(int64_t)threadIdx.x * nblocks + blk] = s_hist[threadIdx.x];
  if (threadIdx.x == 0) {
    {
      partial[2 * blk] = (ss[0] + ss[1]) + (ss[2] + ss[3]);
      partial[2 * blk + 1] = fmax(fmax(sm[0], sm[1]), fmax(sm[2], sm[3]));
    }
    if constexpr (PLACE) {
      blk_cnt[blk] = s_nruns;
      if (blk == 0) hist0[256 * nblocks] = 0;
    }
  }
}

// p in scalar registers: an opaque wave-uniform pointer, so p[lane] keeps the
// scalar-base load form (the compiler otherwise reassociates p + lane into a
// hoisted per-lane 64-bit pointer plus a VALU add per access)
template <typename T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
  return (T*)(((uint64_t)hi << 32) | lo);
}

// base[lane] / base[lane] = x with base wave-uniform: the global access's
// scalar-base form (base in scalar registers + the lane's 32-bit byte offset,
// laundered through an empty asm inside the loop so the offset's zero
// extension is not hoisted out of the loop body, where instruction selection
// would no longer see it)
template <typename T>
__device__ __forceinline__ T seg_ld(const T* base, int lane) {
  // loaded as a same-size integer (vector types have no constructor from an
  // address-space-qualified object)
  using U = typename std::conditional<sizeof(T) == 16, __uint128_t,
                                      typename std::conditional<sizeof(T) == 8, uint64_t, uint32_t>::type>::type;
  static_assert(sizeof(T) == sizeof(U), "4-, 8- or 16-byte elements");
  unsigned off = (unsigned)lane * (unsigned)sizeof(T);
  asm volatile("" : "+v"(off));
  const __attribute__((address_space(1))) char* b = (const __attribute__((address_space(1))) char*)uniform_ptr(base);
  return __builtin_bit_cast(T, *(const __attribute__((address_space(1))) U*)(b + off));
}
template <typename T>
__device__ __forceinline__ void seg_st(T* base, unsigned idx, T x) {
  unsigned off = idx * (unsigned)sizeof(T);
  asm volatile("" : "+v"(off));
  __attribute__((address_space(1))) char* b = (__attribute__((address_space(1))) char*)uniform_ptr(base);
  *(__attribute__((address_space(1))) T*)(b + off) = x;
}

// Lane loads of the dense-row place pass: a wave-uniform base (the segment's
// first visibility i0, scalar registers) plus the lane's 32-bit offset, so the
// loads take the scalar-base form with no per-lane 64-bit address arithmetic.
template <int WK>
__device__ __forceinline__ double seg_weight(const void* __restrict__ w, const RowMap& m, int64_t i0, int lane) {
  if constexpr (WK == WK_F32) return (double)seg_ld((const float*)w + i0, lane);
  if constexpr (WK == WK_F64) return seg_ld((const double*)w + i0, lane);
  if constexpr (WK == WK_POL4I) return load_weight<WK>(w, m, i0 + lane);
  return 1.0;
}
// max(|re|, |im|) of a visibility and whether both parts are finite: complex64
// in fp32 (the max of the exact fp32 magnitudes converts to the same double as
// the max of the converted parts; the finite test is the same too)
__device__ __forceinline__ double seg_vis_abs(const float2* __restrict__ p, int64_t i0, int lane, bool* finite) {
  if (p == nullptr) {  // PSF: the unit visibility
    *finite = true;
    return 1.0;
  }
  const float2 v = seg_ld(p + i0, lane);
  *finite = isfinite(v.x) && isfinite(v.y);
  return (double)fmaxf(fabsf(v.x), fabsf(v.y));
}
__device__ __forceinline__ double seg_vis_abs(const double2* __restrict__ p, int64_t i0, int lane, bool* finite) {
  const double2 v = seg_ld(p + i0, lane);
  *finite = isfinite(v.x) && isfinite(v.y);
  return fmax(fabs(v.x), fabs(v.y));
}
__device__ __forceinline__ double seg_vis_abs(const Pol4* __restrict__ p, int64_t i0, int lane, bool* finite) {
  double re, im;
  load_vis(p, i0 + lane, re, im);
  *finite = isfinite(re) && isfinite(im);
  return fmax(fabs(re), fabs(im));
}

// The place pass over dense rows of a multiple of 64 channels (RM = 1, the
// MS layout of the benchmark): every wave's 64 visibilities are channels
// c0 .. c0 + 63 of ONE row r, so the row, its uvw, the segment's load bases,
// the park slots' base and the run detection's row check are wave-uniform
// (scalar registers and loads), the key and class arithmetic is 32-bit, and
// the per-lane work is the placement, the run detection and the stores.
// Bit-identical to place_body<.., RM = 1>: the same sums in the same order,
// the same keys, classes and park records.
template <typename VisT, int WK, bool WS>
__device__ __forceinline__ void place_rows64_body(const double* __restrict__ uvw, const double* __restrict__ fx,
                                                  const RowMap& m, const VisT* __restrict__ vis,
                                                  const void* __restrict__ wgt, const GridGeometry& g,
                                                  unsigned* err_flag, uint8_t* __restrict__ vis_class,
                                                  int64_t* __restrict__ blk_cnt, uint32_t* __restrict__ park_key,
                                                  uint64_t* __restrict__ park_run, double* partial,
                                                  int64_t* __restrict__ hist0, const int64_t blk,
                                                  const int64_t nblocks) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  __shared__ unsigned s_nruns;
  __shared__ unsigned s_hist[256];
  if (threadIdx.x == 0) s_nruns = 0u;
  s_hist[threadIdx.x] = 0u;
  __syncthreads();
  double wsum = 0.0, wvmax = 0.0;
  // non-finite visibility / weight, failed placement: any lane, ever (scalar)
  unsigned long long nonfinite = 0ull, bad_any = 0ull;
  // 32-bit uniform row / channel / segment counters (launch_plan_place picks
  // this body for nrow < 2^31 and nvis < 2^37): scalar compares, so the row
  // and the loop stay in scalar registers
  const int nchan = (int)m.nchan;
  const int nseg = (int)(m.nvis / 64);  // nvis = nrow nchan: whole segments
  const int blk32 = (int)blk;
  const int seg_end = (blk32 + 1) * kPlaceSegs < nseg ? (blk32 + 1) * kPlaceSegs : nseg;
  const unsigned P = (unsigned)(kTile + g.support - 1);
  const uint32_t ntx = (uint32_t)g.ntx, ntw = (uint32_t)g.ntw;
  constexpr bool wstack = WS;
  // the wave's first segment: row r, channels c0 .. c0 + 63; then 256
  // visibilities per step
  const int64_t i00 = ((int64_t)blk32 * kPlaceSegs + wave) * 64;
  int r = (int)(i00 / nchan);
  int c0 = (int)(i00 - (int64_t)r * nchan);
  const int step_r = 256 / nchan, step_c = 256 % nchan;
  // this block's park region
  uint32_t* const pkey = park_key + blk * kPlaceSegs * 64;
  uint64_t* const prun = park_run + blk * kPlaceSegs * 64;
  const unsigned long long upto = (2ull << lane) - 1ull;   // lane 63: 2 << 63 == 0 - 1 = all
  for (int seg = blk32 * kPlaceSegs + wave; seg < seg_end; seg += 4) {
    // readfirstlane: an opaque uniform base, so the loads below keep the
    // scalar-base form (no per-lane pointer induction variables)
    const int64_t i0 = (int64_t)__builtin_amdgcn_readfirstlane(seg) * 64;
    const int64_t ru = (int64_t)__builtin_amdgcn_readfirstlane(r);
    // loads first (one memory round trip per iteration)
    const double u = uvw[3 * ru], v = uvw[3 * ru + 1];
    const double w = wstack ? uvw[3 * ru + 2] : 0.0;
    const double f = seg_ld(fx + c0, lane);
    const double wt = seg_weight<WK>(wgt, m, i0, lane);
    bool vfin;
    const double vabs = seg_vis_abs(vis, i0, lane, &vfin);
    // the fused reduction (place_body's order: every lane is valid here). A
    // zero weight adds 0 * |V| = 0 or NaN (|V| not finite) to the max, which
    // fmax ignores as it ignores place_body's 0 - the same max either way.
    const bool counted = wt != 0.0;
    nonfinite |= __ballot(counted && !(isfinite(wt) && vfin));
    wsum = wsum + wt;
    wvmax = fmax(wvmax, fabs(wt) * vabs);
    int ix0, iy0;
    int64_t iw0;
    const bool ok = place_origin<WS ? 1 : 0>(u, v, w, f, g, &ix0, &iy0, &iw0);
    bool feeds = true;
    if constexpr (WS) feeds = (iw0 + g.support > g.plane_lo) & (iw0 < g.plane_hi);
    const uint32_t tk = ((uint32_t)iy0 / (uint32_t)kTile) * ntx + (uint32_t)ix0 / (uint32_t)kTile;
    const uint32_t key = (ok & feeds) ? (WS ? tk * ntw + (uint32_t)iw0 : tk) : kNoKey;
    bad_any |= __ballot(!ok);
    if (vis_class)
      seg_st(vis_class + i0, (unsigned)lane, ok ? (uint8_t)(((unsigned)ix0 * P + (unsigned)iy0) & 31u) : (uint8_t)0);
    // runs: a lane starts one where its key differs from the previous lane's
    // (DPP shift; lane 0 always), and emits it unless off the grid (masks in
    // scalar registers: the ballots are the compares themselves)
    const uint32_t prev = wave_shr1(key);
    const unsigned long long starts = __ballot(key != prev) | 1ull;
    const bool emit = key != kNoKey && (key != prev || lane == 0);
    const unsigned long long emits = __ballot(emit);
    unsigned wbase = 0;
    if (lane == 0 && emits) wbase = atomicAdd(&s_nruns, (unsigned)__popcll(emits));
    wbase = (unsigned)__builtin_amdgcn_readlane((int)wbase, 0);
    if (emit) {
      const unsigned long long above = starts & ~upto;
      const int next = above ? (__ffsll((long long)above) - 1) : 64;
      const unsigned slot = wbase + __builtin_amdgcn_mbcnt_hi((unsigned)(emits >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((unsigned)emits, 0u));
      atomicAdd(&s_hist[key & 255u], 1u);
      seg_st(pkey, slot, key);
      const uint32_t c = (uint32_t)(c0 + lane);
      // (row << 32) | (c << 16) | channel stop, as two 32-bit words
      const uint32_t lo = (c << 16) | (uint32_t)(c0 + next);
      seg_st(prun, slot, ((uint64_t)(uint32_t)ru << 32) | (uint64_t)lo);
    }
    c0 += step_c;
    r += step_r;
    if (c0 >= nchan) {
      c0 -= nchan;
      ++r;
    }
  }
  __shared__ double ss[4], sm[4];
  if (lane == 0 && nonfinite) atomicOr(err_flag, 2u);
  if (lane == 0 && bad_any) atomicOr(err_flag, 1u);
  for (int d = 32; d > 0; d >>= 1) {
    wsum += __shfl_xor(wsum, d, 64);
    wvmax = fmax(wvmax, __shfl_xor(wvmax, d, 64));
  }
  if (lane == 0) {
    ss[threadIdx.x >> 6] = wsum;
    sm[threadIdx.x >> 6] = wvmax;
  }
  __syncthreads();
  hist0[(int64_t)threadIdx.x * nblocks + blk] = s_hist[threadIdx.x];
  if (threadIdx.x == 0) {
    partial[2 * blk] = (ss[0] + ss[1]) + (ss[2] + ss[3]);
    partial[2 * blk + 1] = fmax(fmax(sm[0], sm[1]), fmax(sm[2], sm[3]));
    blk_cnt[blk] = s_nruns;
    if (blk == 0) hist0[256 * nblocks] = 0;
  }
}

// CIP_PLACE_ROWS64=0: dense 64-channel rows through place_body (A/B)
static bool place_rows64() {
  static const bool on = [] {
    const char* e = getenv("CIP_PLACE_ROWS64");
    return !(e && e[0] == '0');
  }();
  return on;
}

// The place pass (reduction fused, the place block = this workgroup); PLACE =
// false: the reduction alone (CIP_REUSE_PLAN calls). RM = 3 / 4: dense rows of
// a multiple of 64 channels through place_rows64_body (2-D / w-stacking).
template <typename VisT, int WK, bool PLACE = true, int RM = 0>
__global__ __launch_bounds__(256) void plan_place_kernel(const double* __restrict__ uvw,
                                                         const double* __restrict__ fx, RowMap m,
                                                         const VisT* __restrict__ vis, const void* __restrict__ wgt,
                                                         GridGeometry g, unsigned* err_flag,
                                                         uint8_t* __restrict__ vis_class,
                                                         int64_t* __restrict__ blk_cnt,
                                                         uint32_t* __restrict__ park_key,
                                                         uint64_t* __restrict__ park_run, double* partial,
                                                         int64_t* __restrict__ hist0) {
  if constexpr (PLACE && (RM == 3 || RM == 4))
    place_rows64_body<VisT, WK, RM == 4>(uvw, fx, m, vis, wgt, g, err_flag, vis_class, blk_cnt, park_key, park_run, partial,
                                hist0, blockIdx.x, gridDim.x);
  else
    place_body<VisT, WK, PLACE, RM>(uvw, fx, m, vis, wgt, g, err_flag, vis_class, blk_cnt, park_key, park_run,
                                    partial, hist0, blockIdx.x, gridDim.x);
}

static unsigned plan_blocks(int64_t nvis) {
  const int64_t segs = (nvis + 63) / 64;
  const int64_t b = (segs + kPlaceSegs - 1) / kPlaceSegs;
  return (unsigned)(b > 0 ? b : 1);
}

int plan_place_blocks(int64_t nvis) { return (int)plan_blocks(nvis); }

hipError_t launch_prep_reduce(const RowMap& m, const void* vis, int vis_dtype, const void* wgt, int wgt_dtype,
                              const GridGeometry& g, unsigned* err_flag, double* partial, hipStream_t s) {
  const dim3 gd(plan_blocks(m.nvis));
#define REDUCE(VT, WKV)                                                                                      \
  plan_place_kernel<VT, WKV, false><<<gd, dim3(256), 0, s>>>(nullptr, nullptr, m, (const VT*)vis, wgt, g,    \
                                                            err_flag, nullptr, nullptr, nullptr, nullptr,   \
                                                            partial, nullptr)
  if (vis_dtype == CIP_POL4I) {
    REDUCE(Pol4, WK_POL4I);
  } else if (vis_dtype == CIP_C64) {
    if (wgt_dtype == CIP_F32) REDUCE(float2, WK_F32);
    else if (wgt_dtype == CIP_F64) REDUCE(float2, WK_F64);
    else REDUCE(float2, WK_NONE);
  } else {
    if (wgt_dtype == CIP_F32) REDUCE(double2, WK_F32);
    else if (wgt_dtype == CIP_F64) REDUCE(double2, WK_F64);
    else REDUCE(double2, WK_NONE);
  }
#undef REDUCE
  return hipGetLastError();
}

hipError_t launch_plan_place(const double* uvw, const double* fx, const RowMap& m,
                             const void* vis, int vis_dtype, const void* wgt, int wgt_dtype, const GridGeometry& g,
                             unsigned* err_flag, uint8_t* vis_class, int64_t* blk_cnt, uint32_t* park_key,
                             uint64_t* park_run, double* partial, int64_t* hist0, hipStream_t s) {
  const dim3 gd(plan_blocks(m.nvis));
  const bool rows64 = place_rows64() && m.nchan > 0 && m.nvis / m.nchan < ((int64_t)1 << 31) && m.nvis < ((int64_t)1 << 37);
  const int rm = m.delta != nullptr ? 2 : (m.nchan % 64 == 0 ? (rows64 ? (g.do_wstacking ? 4 : 3) : 1) : 0);
#define PLACE_RM(VT, WKV, RMV)                                                                                      \
  plan_place_kernel<VT, WKV, true, RMV><<<gd, dim3(256), 0, s>>>(uvw, fx, m, (const VT*)vis, wgt, g, err_flag,     \
                                                                 vis_class, blk_cnt, park_key, park_run, partial,   \
                                                                 hist0)
#define PLACE(VT, WKV)            \
  do {                            \
    if (rm == 4) {                \
      PLACE_RM(VT, WKV, 4);       \
    } else if (rm == 3) {         \
      PLACE_RM(VT, WKV, 3);       \
    } else if (rm == 2) {         \
      PLACE_RM(VT, WKV, 2);       \
    } else if (rm == 1) {         \
      PLACE_RM(VT, WKV, 1);       \
    } else {                      \
      PLACE_RM(VT, WKV, 0);       \
    }                             \
  } while (0)
  if (vis_dtype == CIP_POL4I) {
    PLACE(Pol4, WK_POL4I);
  } else if (vis_dtype == CIP_C64) {
    if (wgt_dtype == CIP_F32) PLACE(float2, WK_F32);
    else if (wgt_dtype == CIP_F64) PLACE(float2, WK_F64);
    else PLACE(float2, WK_NONE);
  } else {
    if (wgt_dtype == CIP_F32) PLACE(double2, WK_F32);
    else if (wgt_dtype == CIP_F64) PLACE(double2, WK_F64);
    else PLACE(double2, WK_NONE);
  }
#undef PLACE
#undef PLACE_RM
  return hipGetLastError();
}

// ------------------------------------------------------- ragged rows ----
__global__ void ragged_lengths_kernel(const int32_t* __restrict__ c0, const int32_t* __restrict__ c1, int64_t nrow,
                                      int64_t nchan, int64_t* __restrict__ out, unsigned* err) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < nrow) {
    const int32_t a = c0[r], b = c1[r];
    const bool ok = a >= 0 && a <= b && (int64_t)b <= nchan;
    if (!ok) atomicOr(err, 1u);
    out[r] = ok ? (int64_t)(b - a) : 0;
  } else if (r == nrow) {
    out[r] = 0;
  }
}

hipError_t launch_ragged_lengths(const int32_t* c0, const int32_t* c1, int64_t nrow, int64_t nchan, int64_t* out,
                                 unsigned* err, hipStream_t s) {
  ragged_lengths_kernel<<<dim3((unsigned)((nrow + 256) / 256)), dim3(256), 0, s>>>(c0, c1, nrow, nchan, out, err);
  return hipGetLastError();
}

// one thread per row: delta[r] = off[r] - chan_start[r], and the row of every
// 64-visibility segment that starts inside it (seg_row[k] = r for
// 64 k in [off[r], off[r + 1]); one entry per 64 visibilities, where a
// per-visibility row array cost 4 bytes per visibility written and read)
__global__ __launch_bounds__(256) void ragged_expand_kernel(const int64_t* __restrict__ off,
                                                            const int32_t* __restrict__ c0, int64_t nrow,
                                                            int64_t* __restrict__ delta,
                                                            uint32_t* __restrict__ seg_row) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrow) return;
  const int64_t a = off[r], b = off[r + 1];
  delta[r] = a - (int64_t)c0[r];
  for (int64_t k = (a + 63) >> 6; k * 64 < b; ++k) seg_row[k] = (uint32_t)r;
}

hipError_t launch_ragged_expand(const int64_t* off, const int32_t* c0, int64_t nrow, int64_t* delta,
                                uint32_t* seg_row, hipStream_t s) {
  if (nrow <= 0) return hipSuccess;
  ragged_expand_kernel<<<dim3((unsigned)((nrow + 255) / 256)), dim3(256), 0, s>>>(off, c0, nrow, delta, seg_row);
  return hipGetLastError();
}

// ---------------------------------------------------------- radix sort ----
// Stable LSD radix sort of (uint32 key, uint64 run) pairs, 8-bit digits.
// Items come in sub-blocks of <= 4096 slots: dense (slots [4096 b, 4096 b +
// 4096) of n), or the place pass's per-block runs (slots [4096 b, 4096 b +
// blk_cnt[b])). A workgroup takes a group of G consecutive sub-blocks in
// order; per sub-block, wave w ranks its contiguous quarter of the items in
// order, 64 at a time (8 ballots give each lane its digit's peer mask; a
// wave-private LDS counter per digit carries the rank across steps, read by
// every lane and then advanced by the digit's first lane - one wave's LDS ops
// execute in order, so no barrier is needed). A per-digit prefix over the 4
// waves and the group's running digit offsets place each item at its digit's
// next position: the order of a digit's items is the input order (stable).
// Global bases: the exclusive scan of the digit-major group histogram
// hist[d * ngroups + g] (+1 trailing entry: the item count). Grouping pass
// 0's place blocks (8 of ~500 runs) divides its histogram scan by 8 (C3:
// 6.2 M -> 0.78 M entries; the kernel's own time is unchanged, ~180 us,
// latency-bound, and staging a sub-block in LDS for line-coalesced stores did
// not change it either).
constexpr int kRadixThreads = 256;
constexpr int kRadixPer = 16;
constexpr int64_t kRadixBlock = (int64_t)kRadixThreads * kRadixPer;
static_assert(kRadixBlock == 64 * 64, "a radix sub-block covers one place block's park region");

__device__ __forceinline__ int64_t radix_count(int64_t b, int64_t n, const int64_t* __restrict__ blk_cnt) {
  if (blk_cnt) return blk_cnt[b];
  const int64_t rem = n - b * kRadixBlock;
  return rem < kRadixBlock ? rem : kRadixBlock;
}

__global__ __launch_bounds__(kRadixThreads) void radix_hist_kernel(const uint32_t* __restrict__ keys, int64_t n,
                                                                   const int64_t* __restrict__ blk_cnt, int64_t nsub,
                                                                   int G, int shift, int64_t ngroups,
                                                                   int64_t* __restrict__ hist) {
  __shared__ unsigned cnt[256];
  cnt[threadIdx.x] = 0u;
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * G;
  const int64_t b1 = b0 + G < nsub ? b0 + G : nsub;
  for (int64_t b = b0; b < b1; ++b) {
    const int64_t cnt_b = radix_count(b, n, blk_cnt);
    const uint32_t* kb = keys + b * kRadixBlock;
    if (cnt_b == kRadixBlock) {
      // full sub-block: the loads issue back to back (the loop below waits for each)
      uint32_t kk[kRadixPer];
#pragma unroll
      for (int k = 0; k < kRadixPer; ++k) kk[k] = kb[threadIdx.x + k * kRadixThreads];
#pragma unroll
      for (int k = 0; k < kRadixPer; ++k) atomicAdd(&cnt[(kk[k] >> shift) & 255u], 1u);
    } else {
      for (int64_t i = threadIdx.x; i < cnt_b; i += kRadixThreads) atomicAdd(&cnt[(kb[i] >> shift) & 255u], 1u);
    }
  }
  __syncthreads();
  hist[(int64_t)threadIdx.x * ngroups + blockIdx.x] = cnt[threadIdx.x];
  if (blockIdx.x == 0 && threadIdx.x == 0) hist[256 * ngroups] = 0;
}

// hg[d * ngroups + g] = sum of hist0[d * nsub + b] over the G sub-blocks of
// group g (the place pass's per-block histogram, summed per radix group)
__global__ void radix_group_hist_kernel(const int64_t* __restrict__ hist0, int64_t nsub, int G, int64_t ngroups,
                                        int64_t* __restrict__ hg) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0) hg[256 * ngroups] = 0;
  if (t >= 256 * ngroups) return;
  const int64_t d = t / ngroups, gi = t - d * ngroups;
  const int64_t b0 = gi * G, b1 = b0 + G < nsub ? b0 + G : nsub;
  int64_t sum = 0;
  for (int64_t b = b0; b < b1; ++b) sum += hist0[d * nsub + b];
  hg[t] = sum;
}

__global__ __launch_bounds__(kRadixThreads) void radix_scatter_kernel(
    const uint32_t* __restrict__ keys, const uint64_t* __restrict__ vals, int64_t n,
    const int64_t* __restrict__ blk_cnt, int64_t nsub, int G, int shift, int64_t ngroups,
    const int64_t* __restrict__ hist, uint32_t* __restrict__ keys_out, uint64_t* __restrict__ vals_out) {
  __shared__ unsigned wcnt[4][256];  // per-wave running digit counts
  __shared__ int64_t dnext[256];     // the group's next position per digit
  __shared__ int64_t woff[4][256];   // global position of each wave's first item per digit
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  dnext[threadIdx.x] = hist[(int64_t)threadIdx.x * ngroups + blockIdx.x];
  const int64_t b0 = (int64_t)blockIdx.x * G;
  const int64_t b1 = b0 + G < nsub ? b0 + G : nsub;
  for (int64_t b = b0; b < b1; ++b) {
    const int64_t cnt_b = radix_count(b, n, blk_cnt);
    // the sub-block's items are split into 4 contiguous, 64-aligned wave
    // ranges of q items (q = 1024 for a full sub-block; a parked block holds
    // ~500 runs, which would otherwise all fall to wave 0); wave ranges in
    // order keep it stable
    const int steps = (int)((cnt_b + 255) / 256);  // 64-item steps per wave
    const int q = 64 * steps;
    const int64_t i0 = b * kRadixBlock + wave * q + lane;
    const int64_t wlim = b * kRadixBlock + (int64_t)(wave + 1) * q;
    const int64_t blim = b * kRadixBlock + cnt_b;
    const int64_t lim = wlim < blim ? wlim : blim;
#pragma unroll
    for (int w = 0; w < 4; ++w) wcnt[w][threadIdx.x] = 0u;
    uint32_t key[kRadixPer];
    uint64_t val[kRadixPer];
#pragma unroll
    for (int k = 0; k < kRadixPer; ++k) {
      const int64_t i = i0 + k * 64;
      key[k] = (k < steps && i < lim) ? keys[i] : 0u;
      val[k] = (k < steps && i < lim) ? vals[i] : 0ull;
    }
    __syncthreads();
    unsigned rank[kRadixPer];
#pragma unroll
    for (int k = 0; k < kRadixPer; ++k) {
      if (k < steps) {  // block-uniform
        const bool valid = i0 + k * 64 < lim;
        const unsigned d = (key[k] >> shift) & 255u;
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
          const bool on = (d >> bit) & 1u;
          const unsigned long long m = __ballot(on);
          peers &= on ? m : ~m;
        }
        const unsigned prior = valid ? wcnt[wave][d] : 0u;
        rank[k] = prior + (unsigned)__popcll(peers & ((1ull << lane) - 1ull));
        if (valid && (peers & ((1ull << lane) - 1ull)) == 0ull) wcnt[wave][d] = prior + (unsigned)__popcll(peers);
      }
    }
    __syncthreads();
    {
      const int d = threadIdx.x;
      int64_t o = dnext[d];
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        woff[w][d] = o;
        o += wcnt[w][d];
      }
      dnext[d] = o;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kRadixPer; ++k)
      if (k < steps && i0 + k * 64 < lim) {
        const int64_t pos = woff[wave][(key[k] >> shift) & 255u] + rank[k];
        keys_out[pos] = key[k];
        vals_out[pos] = val[k];
      }
    __syncthreads();  // wcnt / woff are reused by the next sub-block
  }
}

// tile_run_off[t] = first sorted run with key >= t (t in [0, ntiles]; key
// bits outside kmask carry run lengths, RowMap::pk_runs)
__global__ void tile_offsets_kernel(const uint32_t* __restrict__ keys, int64_t nruns, int64_t ntiles,
                                    int64_t* __restrict__ tile_run_off, uint32_t kmask) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t > ntiles) return;
  int64_t lo = 0, hi = nruns;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)(keys[mid] & kmask) < t) lo = mid + 1;
    else hi = mid;
  }
  tile_run_off[t] = lo;
}

int64_t radix_blocks(int64_t n) { return (n + kRadixBlock - 1) / kRadixBlock; }

hipError_t launch_radix_hist(const uint32_t* keys, int64_t n, const int64_t* blk_cnt, int64_t nsub, int G, int shift,
                             int64_t* hist, hipStream_t s) {
  if (nsub == 0) return hipSuccess;
  const int64_t ngroups = (nsub + G - 1) / G;
  radix_hist_kernel<<<dim3((unsigned)ngroups), dim3(kRadixThreads), 0, s>>>(keys, n, blk_cnt, nsub, G, shift,
                                                                          ngroups, hist);
  return hipGetLastError();
}

hipError_t launch_radix_group_hist(const int64_t* hist0, int64_t nsub, int G, int64_t* hg, hipStream_t s) {
  const int64_t ngroups = (nsub + G - 1) / G;
  const int64_t nt = 256 * ngroups > 0 ? 256 * ngroups : 1;
  radix_group_hist_kernel<<<dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s>>>(hist0, nsub, G, ngroups, hg);
  return hipGetLastError();
}

hipError_t launch_radix_scatter(const uint32_t* keys, const uint64_t* vals, int64_t n, const int64_t* blk_cnt,
                                int64_t nsub, int G, int shift, const int64_t* hist, uint32_t* keys_out,
                                uint64_t* vals_out, hipStream_t s) {
  if (nsub == 0) return hipSuccess;
  const int64_t ngroups = (nsub + G - 1) / G;
  radix_scatter_kernel<<<dim3((unsigned)ngroups), dim3(kRadixThreads), 0, s>>>(
      keys, vals, n, blk_cnt, nsub, G, shift, ngroups, hist, keys_out, vals_out);
  return hipGetLastError();
}

hipError_t launch_tile_offsets(const uint32_t* keys, int64_t nruns, int64_t ntiles, int64_t* tile_run_off,
                               hipStream_t s, uint32_t kmask) {
  tile_offsets_kernel<<<dim3((unsigned)((ntiles + 256) / 256)), dim3(256), 0, s>>>(keys, nruns, ntiles, tile_run_off,
                                                                                 kmask);
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

// Dirty-tile masks of the HBM grid, one per grid plane (nplanes x ntx x nty
// bytes, zeroed by the caller): tile (tx, ty) of plane p is written by the
// scatter's flush when a visibility of a tile layer feeding p (w-stacking:
// layers p - W + 1 .. p; 2-D: the one layer) lands in it or, through the
// (T + W - 1)^2 sub-grid's halo, in one of its -x, -y or -x-y neighbours
// within the halo's reach (periodic grid).
__global__ void dirty_mask_kernel(const int64_t* __restrict__ tile_vis, int64_t ntx, int64_t nty, int64_t ntw,
                                  int support, int64_t nplanes, uint8_t* __restrict__ mask) {
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nt = ntx * nty;
  if (id >= nt * nplanes) return;
  const int64_t p = id / nt, t = id - p * nt;
  int64_t lo = 0, hi = 0;
  if (nplanes > 1) {
    lo = p - support + 1 > 0 ? p - support + 1 : 0;
    hi = p < ntw - 1 ? p : ntw - 1;
  }
  bool touched = false;
  for (int64_t w = lo; w <= hi && !touched; ++w) touched = tile_vis[t * ntw + w] > 0;  // tile-major keys
  if (!touched) return;
  const int64_t tx = t % ntx, ty = t / ntx;
  uint8_t* m = mask + p * nt;
  // the sub-grid's cells reach T + W - 2 past the tile origin: h more tiles
  // per axis (1 for W <= T + 1, 2 for the large supports up to 64)
  const int h = (kTile + support - 2) / kTile;
  for (int dy = 0; dy <= h; ++dy) {
    const int64_t yy = (ty + dy) % nty;
    for (int dx = 0; dx <= h; ++dx) m[yy * ntx + (tx + dx) % ntx] = 1;  // idempotent stores: no atomics needed
  }
}

// bit-pack the byte mask: bit tx % 32 of word ty * (ntx / 32) + tx / 32
__global__ void pack_mask_kernel(const uint8_t* __restrict__ mask, int64_t nwords, uint32_t* __restrict__ bits) {
  const int64_t wd = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (wd >= nwords) return;
  uint32_t b = 0u;
  for (int k = 0; k < 32; ++k) b |= (uint32_t)(mask[32 * wd + k] != 0) << k;
  bits[wd] = b;
}

// Tile-row bits of the packed mask (one per plane and tile row ty: any dirty
// tile in the row), nrw = ceil(nty / 32) words per plane. The pruned FFT skips
// the grid rows of clean tile rows in both passes: pass A neither transforms
// nor writes them, pass B reads them as zero (C3 w-stacking: 36 % of the
// rows over the 14 planes; 2-D: 14 %).
__global__ void row_bits_kernel(const uint32_t* __restrict__ bits, int64_t ntx, int64_t nty, int64_t nplanes,
                                uint32_t* __restrict__ rows) {
  const int64_t nrw = (nty + 31) / 32;
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= nrw * nplanes) return;
  const int64_t p = id / nrw, w = id - p * nrw;
  const int64_t wpr = ntx / 32;  // mask words per tile row
  const uint32_t* b = bits + p * (nty * wpr);
  uint32_t out = 0u;
  for (int k = 0; k < 32; ++k) {
    const int64_t ty = w * 32 + k;
    if (ty >= nty) break;
    uint32_t any = 0u;
    for (int64_t j = 0; j < wpr; ++j) any |= b[ty * wpr + j];
    out |= (any != 0u ? 1u : 0u) << k;
  }
  rows[id] = out;
}

hipError_t launch_dirty_mask(const int64_t* tile_vis, int64_t ntx, int64_t nty, int64_t ntw, int support,
                             int64_t nplanes, uint8_t* mask, uint32_t* bits, hipStream_t s) {
  const int64_t n = ntx * nty * nplanes;
  dirty_mask_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s>>>(tile_vis, ntx, nty, ntw, support,
                                                                           nplanes, mask);
  if (bits) {
    if (ntx % 32 != 0) return hipErrorInvalidValue;
    const int64_t nw = n / 32;
    pack_mask_kernel<<<dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, s>>>(mask, nw, bits);
    // the row bits follow the tile bits (dirty_bits_words())
    const int64_t nr = (nty + 31) / 32 * nplanes;
    row_bits_kernel<<<dim3((unsigned)((nr + 255) / 256)), dim3(256), 0, s>>>(bits, ntx, nty, nplanes, bits + nw);
  }
  return hipGetLastError();
}

hipError_t launch_tile_vis(const int64_t* run_goff, const int64_t* tile_run_off, int64_t ntiles,
                           int64_t* tile_vis_off, int64_t* tile_vis, hipStream_t s) {
  tile_vis_kernel<<<dim3((unsigned)((ntiles + 256) / 256)), dim3(256), 0, s>>>(run_goff, tile_run_off, ntiles,
                                                                               tile_vis_off, tile_vis);
  return hipGetLastError();
}

// Chunks per tile: out[t] = ceil(tile_vis[t] / cv), out[ntiles] = 0. With
// full_first (largest work units first: a 2-D scatter dispatch then ends on
// the small ones, not on a full chunk that started late), full and partial
// chunks are counted separately: out[t] = tile_vis[t] / cv, out[ntiles + t] =
// 1 if a partial remainder exists, out[2 ntiles] = 0 - the exclusive scan then
// places every full chunk before every partial one.
__global__ void chunk_counts_kernel(const int64_t* tile_vis, int64_t ntiles, int64_t cv, int full_first,
                                    int64_t* out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (!full_first) {
    if (t < ntiles) out[t] = (tile_vis[t] + cv - 1) / cv;
    else if (t == ntiles) out[t] = 0;
    return;
  }
  if (t < ntiles) {
    out[t] = tile_vis[t] / cv;
    out[ntiles + t] = (tile_vis[t] % cv) != 0 ? 1 : 0;
  } else if (t == ntiles) {
    out[2 * ntiles] = 0;
  }
}

hipError_t launch_chunk_counts(const int64_t* tile_vis, int64_t ntiles, int64_t chunk_vis, int full_first,
                               int64_t* out, hipStream_t s) {
  chunk_counts_kernel<<<dim3((unsigned)((ntiles + 256) / 256)), dim3(256), 0, s>>>(tile_vis, ntiles, chunk_vis,
                                                                                   full_first, out);
  return hipGetLastError();
}

// One thread per chunk j: its entry e is the last with chunk_off[e] <= j
// (entries without chunks repeat an offset); entry e < ntiles is tile e's
// chunk k = j - chunk_off[e], entry ntiles + t (full_first) tile t's partial
// chunk k = tile_vis[t] / cv. The chunk's first and last runs by binary search
// among the tile's runs.
__global__ void chunk_emit_kernel(const int64_t* __restrict__ tile_vis_off, const int64_t* __restrict__ tile_vis,
                                  const int64_t* __restrict__ chunk_off, const int64_t* __restrict__ run_goff,
                                  const int64_t* __restrict__ tile_run_off, int64_t ntiles, int64_t cv,
                                  int full_first, int64_t nchunks, Chunk* __restrict__ chunks) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nchunks) return;
  int64_t lo = 0, hi = (full_first ? 2 * ntiles : ntiles) - 1;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (chunk_off[mid] <= j) lo = mid;
    else hi = mid - 1;
  }
  const bool partial = lo >= ntiles;
  const int64_t t = partial ? lo - ntiles : lo;
  const int64_t k = partial ? tile_vis[t] / cv : j - chunk_off[lo];
  const int64_t g = tile_vis_off[t], nv = tile_vis[t];
  Chunk ch;
  ch.g0 = g + k * cv;
  ch.g1 = g + ((k + 1) * cv < nv ? (k + 1) * cv : nv);
  ch.tile = t;
  ch.sole = nv <= cv ? 1 : 0;
  // first run whose end lies beyond g0 (runs of a tile are consecutive)
  int64_t rl = tile_run_off[t], rh = tile_run_off[t + 1] - 1;
  while (rl < rh) {
    const int64_t mid = (rl + rh) >> 1;
    if (run_goff[mid + 1] > ch.g0) rh = mid;
    else rl = mid + 1;
  }
  ch.first_run = rl;
  // last run whose start lies before g1 (the one holding position g1 - 1)
  rh = tile_run_off[t + 1] - 1;
  while (rl < rh) {
    const int64_t mid = (rl + rh + 1) >> 1;
    if (run_goff[mid] < ch.g1) rl = mid;
    else rh = mid - 1;
  }
  ch.last_run = rl;
  chunks[j] = ch;
}

hipError_t launch_chunk_emit(const int64_t* tile_vis_off, const int64_t* tile_vis, const int64_t* chunk_off,
                             const int64_t* run_goff, const int64_t* tile_run_off, int64_t ntiles,
                             int64_t chunk_vis, int full_first, int64_t nchunks, Chunk* chunks, hipStream_t s) {
  if (nchunks <= 0) return hipSuccess;
  chunk_emit_kernel<<<dim3((unsigned)((nchunks + 255) / 256)), dim3(256), 0, s>>>(
      tile_vis_off, tile_vis, chunk_off, run_goff, tile_run_off, ntiles, chunk_vis, full_first, nchunks, chunks);
  return hipGetLastError();
}

// w-stacking work units. With tile-major keys the positions of uv tile t's
// layers feeding plane p (lo = max(p - W + 1, 0) .. hi = min(p, ntw - 1)) are
// one contiguous range, so a plane's work unit covers all of them: one LDS
// sub-grid zeroing and one flush per tile and plane instead of one per tile
// layer (C3, 16 planes: 291k instead of 665k work units). Entry p ntxy + t
// counts ceil(n / cv) units; out[nplanes ntxy] = 0.
// plane group q = planes [q G, q G + G): the layers feeding them are
// [q G - W + 1, q G + G - 1] (clipped to [0, ntw))
__global__ void plane_chunk_counts_kernel(const int64_t* __restrict__ tile_vis_off, int64_t ntxy, int64_t ntw,
                                          int64_t ngroups, int group, int support, int64_t cv,
                                          int64_t* __restrict__ out) {
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nent = ngroups * ntxy;
  if (id > nent) return;
  if (id == nent) {
    out[id] = 0;
    return;
  }
  const int64_t q = id / ntxy, t = id - q * ntxy;
  const int64_t p0 = q * group, p1 = p0 + group - 1;
  const int64_t lo = p0 - support + 1 > 0 ? p0 - support + 1 : 0, hi = p1 < ntw - 1 ? p1 : ntw - 1;
  const int64_t n = hi < lo ? 0 : tile_vis_off[t * ntw + hi + 1] - tile_vis_off[t * ntw + lo];
  out[id] = (n + cv - 1) / cv;
}

hipError_t launch_plane_chunk_counts(const int64_t* tile_vis_off, int64_t ntxy, int64_t ntw, int64_t ngroups,
                                     int group, int support, int64_t cv, int64_t* out, hipStream_t s) {
  const int64_t n = ngroups * ntxy + 1;
  plane_chunk_counts_kernel<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s>>>(tile_vis_off, ntxy, ntw, ngroups,
                                                                                    group, support, cv, out);
  return hipGetLastError();
}

// One thread per work unit j of the plane-major table (chunk_off: the
// exclusive scan of plane_chunk_counts): its entry (p, t), its range
// [g0, g1) of the tile's merged layer range, tile = the key of (t, lo) (its
// grid origin, tile_origin), first and last run by binary search.
__global__ void plane_chunk_emit_kernel(const int64_t* __restrict__ tile_vis_off, const int64_t* __restrict__ chunk_off,
                                        const int64_t* __restrict__ run_goff, const int64_t* __restrict__ tile_run_off,
                                        int64_t ntxy, int64_t ntw, int64_t ngroups, int group, int support,
                                        int64_t cv, int64_t nchunks, Chunk* __restrict__ chunks) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= nchunks) return;
  int64_t lo = 0, hi = ngroups * ntxy - 1;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (chunk_off[mid] <= j) lo = mid;
    else hi = mid - 1;
  }
  const int64_t e = lo;
  const int64_t q = e / ntxy, t = e - q * ntxy;
  const int64_t p0 = q * group, p1 = p0 + group - 1;
  const int64_t l0 = p0 - support + 1 > 0 ? p0 - support + 1 : 0, l1 = p1 < ntw - 1 ? p1 : ntw - 1;
  const int64_t k = j - chunk_off[e];
  const int64_t a = tile_vis_off[t * ntw + l0], b = tile_vis_off[t * ntw + l1 + 1];
  Chunk ch;
  ch.g0 = a + k * cv;
  ch.g1 = a + (k + 1) * cv < b ? a + (k + 1) * cv : b;
  ch.tile = t * ntw + l0;
  ch.sole = b - a <= cv ? 1 : 0;
  int64_t rl = tile_run_off[t * ntw + l0], rh = tile_run_off[t * ntw + l1 + 1] - 1;
  while (rl < rh) {
    const int64_t mid = (rl + rh) >> 1;
    if (run_goff[mid + 1] > ch.g0) rh = mid;
    else rl = mid + 1;
  }
  ch.first_run = rl;
  rh = tile_run_off[t * ntw + l1 + 1] - 1;
  while (rl < rh) {
    const int64_t mid = (rl + rh + 1) >> 1;
    if (run_goff[mid] < ch.g1) rl = mid;
    else rh = mid - 1;
  }
  ch.last_run = rl;
  chunks[j] = ch;
}

hipError_t launch_plane_chunk_emit(const int64_t* tile_vis_off, const int64_t* chunk_off, const int64_t* run_goff,
                                   const int64_t* tile_run_off, int64_t ntxy, int64_t ntw, int64_t ngroups,
                                   int group, int support, int64_t cv, int64_t nchunks, Chunk* chunks,
                                   hipStream_t s) {
  if (nchunks <= 0) return hipSuccess;
  plane_chunk_emit_kernel<<<dim3((unsigned)((nchunks + 255) / 256)), dim3(256), 0, s>>>(
      tile_vis_off, chunk_off, run_goff, tile_run_off, ntxy, ntw, ngroups, group, support, cv, nchunks, chunks);
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
