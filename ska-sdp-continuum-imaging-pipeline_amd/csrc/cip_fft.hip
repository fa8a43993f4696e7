// cip_fft.hip - the dirty image's 2-D FFT as two hand-written pruned passes
// (SURVEY.md 8(a) a4.5), for power-of-two grids of 1024..16384 cells per axis.
//
// The image keeps only nx x ny of the nu x nv frequencies (a quarter for
// sigma = 2). The scatter writes the grid transposed (gT[y, x]); pass A
// transforms each row of gT along u and keeps the nx frequencies i, written
// in 4-column blocks; pass B transforms each kept column i along v and writes
// image row i directly through the crop epilogue (grid correction, or the
// w-plane screen and accumulation). Each workgroup holds one N-point
// transform: N/16 threads x 16 complex values in registers, radix-16 (and a
// last radix-2/4/8) Stockham passes exchanged through one N-element LDS array
// (fp64: real parts, then imaginary parts, N doubles; fp32: whole complex
// values, N float2) - 64 KiB at N = 8192 (two workgroups per CU), 128 KiB at
// N = 16384 (one per CU). HBM bytes per plane: pass A 16 nu nv read +
// 16 nx nv written, pass B 16 nx nv read + 8 nx ny written (against 64 nu nv
// for hipFFT's in-place 2-D c2c plus the crop pass).
#include <type_traits>

#include "cip_internal.h"

namespace cip {

// exp(+2 pi i k / 16), k = 0..15
__device__ __constant__ const double kW16c[16] = {1.0,
                                                  0.92387953251128674,
                                                  0.70710678118654757,
                                                  0.38268343236508978,
                                                  0.0,
                                                  -0.38268343236508978,
                                                  -0.70710678118654757,
                                                  -0.92387953251128674,
                                                  -1.0,
                                                  -0.92387953251128674,
                                                  -0.70710678118654757,
                                                  -0.38268343236508978,
                                                  0.0,
                                                  0.38268343236508978,
                                                  0.70710678118654757,
                                                  0.92387953251128674};

// The transform's complex type CT: double2, or float2 for the packed class
// (complex64 planes, CIP_FFT_F32): the same passes on fp32 values. Both
// exchange N 8-byte elements through LDS (kXLen), so the fp32 form saves
// registers and HBM bytes, not LDS: two N = 8192 workgroups per CU either way
// (the register file allows no more: 90 VGPRs x 8 waves per SIMD).
template <typename CT>
struct Cx;
template <>
struct Cx<double2> {
  using R = double;
  __device__ static __forceinline__ double2 make(double x, double y) { return make_double2(x, y); }
};
template <>
struct Cx<float2> {
  using R = float;
  __device__ static __forceinline__ float2 make(float x, float y) { return make_float2(x, y); }
};
template <typename D, typename S>
__device__ __forceinline__ D ccast(S v) {
  using R = typename Cx<D>::R;
  return Cx<D>::make((R)v.x, (R)v.y);
}

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x));
}

// In-register DFT of size R (R | 16), natural order in and out, sign +.
// Radix-2 decimation in frequency, then the bit-reversed result re-indexed
// at compile time.
template <int R, typename CT>
__device__ __forceinline__ void dft(CT* v) {
  using RT = typename Cx<CT>::R;
#pragma unroll
  for (int span = R / 2; span >= 1; span >>= 1) {
#pragma unroll
    for (int b = 0; b < R; b += 2 * span) {
#pragma unroll
      for (int i = 0; i < span; ++i) {
        const CT a = v[b + i], c = v[b + i + span];
        v[b + i] = Cx<CT>::make(a.x + c.x, a.y + c.y);
        const CT d = Cx<CT>::make(a.x - c.x, a.y - c.y);
        // twiddle exp(+2 pi i i / (2 span)) = W16^(i * 16 / (2 span))
        switch (2 * span) {
          case 2: v[b + i + span] = d; break;
          case 4: v[b + i + span] = (i == 0) ? d : Cx<CT>::make(-d.y, d.x); break;
          default: {
            const int idx = (i * 16 / (2 * span)) & 15;
            const RT cc = (RT)kW16c[idx], ss = (RT)kW16c[(idx + 12) & 15];
            v[b + i + span] = (i == 0) ? d : Cx<CT>::make(fma(d.x, cc, -d.y * ss), fma(d.x, ss, d.y * cc));
          }
        }
      }
    }
  }
  CT t[R];
#pragma unroll
  for (int i = 0; i < R; ++i) t[i] = v[i];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    int rev = 0;
#pragma unroll
    for (int b = 1, rb = R / 2; b < R; b <<= 1, rb >>= 1)
      if (i & b) rev |= rb;
    v[rev] = t[i];
  }
}

// One Stockham pass of radix R over the thread's 16 values (16 / R
// butterflies j_m = t + m T), twiddles from the table tw[m] = exp(+2 pi i m / N).
// TWS: the table's stride (tw holds exp(+2 pi i m / (TWS N)): the even / odd
// halves of a 2N-point column transform their N points with the 2N table)
// LASTW: the last pass's twiddles (ns R = N: w = tw[t + m T]) as tw[t] W16^m,
// one table load per lane instead of one per butterfly (16 / R loads in
// flight at once: the registers the even / odd pass B needs)
template <int N, int R, typename CT, int TWS = 1, bool LASTW = false>
__device__ __forceinline__ void stockham_pass(CT* v, int t, int ns, const double2* __restrict__ tw) {
  constexpr int T = N / 16;
  const double2 wlast = (LASTW && ns * R == N) ? tw[t * TWS] : make_double2(1.0, 0.0);
#pragma unroll
  for (int m = 0; m < 16 / R; ++m) {
    const int j = t + m * T;
    const int k = j & (ns - 1);
    if (ns > 1) {
      // exp(+2 pi i r k / (ns R)) = w^r, w = tw[k N / (ns R)]: one table load
      // per butterfly (the loads were latency on the critical path), powers by
      // repeated products (error grows by ~1 ulp per power, R <= 16)
      CT w;
      if (LASTW && ns * R == N)
        w = ccast<CT>(m == 0 ? wlast : cmul(wlast, make_double2(kW16c[m & 15], kW16c[(m + 12) & 15])));
      else
        w = ccast<CT>(tw[((k * (N / (ns * R))) & (N - 1)) * TWS]);
      CT wr = w;
#pragma unroll
      for (int r = 1; r < R; ++r) {
        v[m * R + r] = cmul(v[m * R + r], wr);
        if (r + 1 < R) wr = cmul(wr, w);
      }
    }
    dft<R>(v + m * R);
  }
}

// LDS positions: output of a pass (idxD + r ns) and input of the next (j + r N / R')
template <int N, int R>
__device__ __forceinline__ int out_pos(int t, int m, int r, int ns) {
  constexpr int T = N / 16;
  const int j = t + m * T;
  const int k = j & (ns - 1);
  return (j - k) * R + k + r * ns;
}

template <int N, int R>
__device__ __forceinline__ int in_pos(int t, int m, int r) {
  constexpr int T = N / 16;
  return t + m * T + r * (N / R);
}

// Exchange layout (round 5): fp32 transforms move whole
// complex values (one ds_write_b64 / ds_read_b64 per element, one pass
// instead of real then imaginary b32 halves), fp64 ones their two halves; both
// at position p ^ ((p >> 4) & 15) (no padding). ds_read_b64 banks a wave's two
// 32-lane groups by element mod 32, ds_write_b64 its four 16-lane groups by
// element mod 16 (MI355X_MICROARCH.md, LDS): reads (32 consecutive, 32-aligned
// positions) keep their 16-element blocks; the first exchange's writes
// (positions 16 t + r) and the second's (256 (j >> 4) + 16 r + j % 16) land on
// 16 distinct elements mod 16 per group. The round-4 padded layout (p + p /
// 16, real / imaginary b32 halves) spanned 34 elements for 32 consecutive
// reads, a 2-way conflict on every read: 40 % of the LDS cycles of the
// refcall's fp32 transforms were conflict cycles (profiles/r05_sq_refcall.md),
// 0 with this one (profiles/r05aq_sq_refcall_xlds.md).
__device__ __forceinline__ int pad(int p) { return p ^ ((p >> 4) & 15); }

template <typename CT>
using XT = std::conditional_t<sizeof(CT) == 8, CT, typename Cx<CT>::R>;
template <int N>
constexpr int kXLen = N;
// every instantiated transform's exchange array (plus the small per-block
// tables) within the 160 KiB of LDS a CU has
static_assert(kXLen<16384> * 8 + 4096 <= 160 * 1024, "N = 16384 exchange must fit one CU's LDS");
static_assert(2 * (kXLen<8192> * 8 + 4096) <= 160 * 1024, "two N = 8192 transforms per CU");

template <int N, int R, int R2, typename CT>
__device__ __forceinline__ void exchange(CT* v, int t, int ns, XT<CT>* lds) {
  if constexpr (!std::is_same<XT<CT>, typename Cx<CT>::R>::value) {
#pragma unroll
    for (int m = 0; m < 16 / R; ++m)
#pragma unroll
      for (int r = 0; r < R; ++r) lds[pad(out_pos<N, R>(t, m, r, ns))] = v[m * R + r];
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 16 / R2; ++m)
#pragma unroll
      for (int r = 0; r < R2; ++r) v[m * R2 + r] = lds[pad(in_pos<N, R2>(t, m, r))];
    __syncthreads();
  } else {
    // real parts, then imaginary parts, through one N-double array
#pragma unroll
    for (int half = 0; half < 2; ++half) {
#pragma unroll
    for (int m = 0; m < 16 / R; ++m)
#pragma unroll
      for (int r = 0; r < R; ++r) lds[pad(out_pos<N, R>(t, m, r, ns))] = half ? v[m * R + r].y : v[m * R + r].x;
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 16 / R2; ++m)
#pragma unroll
      for (int r = 0; r < R2; ++r) {
        const auto x = lds[pad(in_pos<N, R2>(t, m, r))];
        if (half) v[m * R2 + r].y = x;
        else v[m * R2 + r].x = x;
      }
    __syncthreads();
    }
  }
}

// Pass A output block width (columns i per contiguous 16 CIP_FFT_COLBLOCK-byte
// row of a block). 4 and 8 tie at N = 8192; at N = 16384 (one block per CU)
// 4 is faster: FFT 3.50 -> 3.23 ms at C4, interleaved A/B
// (profiles/r02_ab_fft_colblock.txt).
#ifndef CIP_FFT_COLBLOCK
#define CIP_FFT_COLBLOCK 4
#endif
constexpr int kColBlock = CIP_FFT_COLBLOCK;
#ifndef CIP_SCREEN_F32
#define CIP_SCREEN_F32 1  // 0: fp64 w-screen sine / cosine on fp32 transforms too (A/B builds)
#endif
#ifndef CIP_FFT_EO
#define CIP_FFT_EO 1  // 0: 16384-point fp64 pass B as one transform per workgroup (A/B builds)
#endif
#ifndef CIP_FFT_ROWS_XCD
#define CIP_FFT_ROWS_XCD 1  // 0: pass A's workgroup b transforms row b (A/B builds)
#endif

// All passes of an N-point transform (log2 N = 4 P + B: P radix-16 passes,
// then one radix-2^B pass). On return v[m * RF + r] holds frequency
// out_pos<N, RF>(t, m, r, N / RF).
// min waves per SIMD the fp32 transforms are compiled for (A/B knob): 6 fits
// three N = 8192 workgroups per CU in 80 VGPRs but spills, and measured slower
// than the unconstrained 90-VGPR form (refcall FFT 5.32 vs 5.21 ms,
// profiles/r04_ab_fft_f32.txt)
#ifndef CIP_FFT_F32_WAVES
#define CIP_FFT_F32_WAVES 1
#endif
#ifndef CIP_FFT_F32_WAVES_ROWS
#define CIP_FFT_F32_WAVES_ROWS CIP_FFT_F32_WAVES  // pass A's own (A/B builds)
#endif
template <typename CT>
constexpr int fft_waves() {
  return sizeof(CT) == 8 ? CIP_FFT_F32_WAVES : 1;
}
template <typename CT>
constexpr int fft_waves_rows() {
  return sizeof(CT) == 8 ? CIP_FFT_F32_WAVES_ROWS : 1;
}

template <int N>
struct FftShape {
  static constexpr int T = N / 16;
  static constexpr int L = __builtin_ctz(N);
  static constexpr int P = L / 4, B = L % 4;
  static constexpr int RF = B ? (1 << B) : 16;  // radix of the final pass
};

template <int N, typename CT, int TWS = 1, bool LASTW = false>
__device__ __forceinline__ void fft_core(CT* v, int t, XT<CT>* lds, const double2* __restrict__ tw) {
  using S = FftShape<N>;
  int ns = 1;
  stockham_pass<N, 16, CT, TWS, LASTW>(v, t, ns, tw);
#pragma unroll
  for (int p = 1; p < S::P; ++p) {
    exchange<N, 16, 16>(v, t, ns, lds);
    ns *= 16;
    stockham_pass<N, 16, CT, TWS, LASTW>(v, t, ns, tw);
  }
  if constexpr (S::B != 0) {
    exchange<N, 16, S::RF>(v, t, ns, lds);
    ns *= 16;
    stockham_pass<N, S::RF, CT, TWS, LASTW>(v, t, ns, tw);
  }
}

// Pass A, along u: row y of the transposed grid gT (nv rows of nu = N cells)
// -> the nx kept frequencies, i = (k + nx/2) mod N < nx, stored in blocks of
// C = kColBlock columns: H[((i / C) nv + y) C + i % C] (16 C-byte rows per
// block, so pass B's C columns of a block read whole rows between them).
// MASKED: only the row's cells in dirty tiles (dmask, kTile-cell segments)
// are read - the rest of the grid is zero - and those are zeroed after the
// read, so the next scatter needs no memset of the whole grid. Rows
// y0 + blockIdx.x (a strip of the grid) go to H rows y - hy0 of
// an H with hrows rows per block (the whole grid: y0 = hy0 = 0, hrows = nv);
// ZERO (unmasked strips) zeroes every cell read.
// grid cells as stored (GT = double2, or float2 for the packed class's
// complex64 planes), widened to fp64 for the transform
// (ccast: widened to the transform's type CT, or kept)
// pass A's output as stored (HT = double2, or float2 beside complex64 planes:
// the packed class's precision, half the pass-A write and pass-B read bytes)

// EO (the whole grid, pass B by even / odd halves: fft_cols_eo_kernel): grid
// row y goes to H row (y mod 2) nv / 2 + y / 2, so each half's rows are
// contiguous.
template <int N, bool MASKED, bool ZERO = false, typename GT = double2, typename HT = double2,
          typename CT = double2, bool EO = false>
__global__ __launch_bounds__(N / 16, fft_waves_rows<CT>()) void fft_rows_kernel(GT* __restrict__ gT, int64_t hrows, int64_t nx,
                                                          const double2* __restrict__ tw, HT* __restrict__ H,
                                                          const uint32_t* __restrict__ dmask, int64_t ntx,
                                                          int64_t y0 = 0, int64_t hy0 = 0, bool skip_clean = false,
                                                          int64_t mrow0 = 0, int64_t mnv = 0,
                                                          const int64_t* __restrict__ row_slot = nullptr) {
  using S = FftShape<N>;
  __shared__ XT<CT> lds[kXLen<N>];
  const int t = threadIdx.x;
  // rows y .. y + kColBlock - 1 share their H lines (kColBlock-column rows of
  // 8 or 16 bytes): a group of 8 kColBlock consecutive workgroups (dispatched
  // round-robin over the 8 XCDs) is remapped so that each XCD transforms
  // kColBlock adjacent rows and their partial H lines meet in one L2
  int64_t yl = blockIdx.x;
#if CIP_FFT_ROWS_XCD
  if (gridDim.x % (8 * kColBlock) == 0) {
    const int64_t b = blockIdx.x;
    yl = (b / (8 * kColBlock)) * (8 * kColBlock) + (b % 8) * kColBlock + (b / 8) % kColBlock;
  }
#endif
  const int64_t y = y0 + yl;
  GT* row = gT + y * N;
  // row_slot (uv strips' packed pass A): the row's place among the live
  // rows - H holds those only, in order; a dead row (no dirty tile in its
  // tile row: nothing to read or zero) is skipped
  int64_t orow = y - hy0;
  if constexpr (EO) orow = (orow & 1) * (hrows >> 1) + (orow >> 1);
  if (row_slot) {
    orow = row_slot[y - hy0];
    if (orow < 0) return;
  }
  CT v[16];
  if constexpr (MASKED) {
    // the 32-tile word of element r is uniform over the block (T = N / 16
    // threads, t < T: (t + r T) / (32 kTile) = r T / 1024 for every t), so the
    // mask words are scalar loads and each lane tests one bit
    static_assert(kTile == 32 && 1024 % S::T == 0, "mask word per element uniform");
    // the mask's grid row: y itself, or (a uv strip's buffer row y) grid row
    // (mrow0 + y) mod mnv
    const int64_t my = mnv ? (mrow0 + y) % mnv : y;
    const uint32_t* mrow = dmask + (my / kTile) * (ntx / 32);
    uint32_t words[16];
    uint32_t any = 0u;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      words[r] = mrow[(r * S::T) >> 10];
      any |= words[r];
    }
    // a clean tile row (every word of it is read above): nothing to transform
    // or zero, and pass B reads its H rows as zero (row_bits_kernel)
    if (skip_clean && any == 0u) return;
    // cells as stored first, widened after every load is issued: a widen
    // inside the branch makes each branch wait for its own load (16
    // serialised loads for float2 cells, measured 381 vs 336 us a plane)
    GT raw[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int x = t + r * S::T;
      const uint32_t word = words[r];
      raw[r] = GT{0, 0};
      if ((word >> ((x >> 5) & 31)) & 1u) {
        raw[r] = row[x];
        row[x] = GT{0, 0};
      }
    }
    // (the empty asm pins the raw values past the branches: without it the
    // compiler sinks each widen back into its branch)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if constexpr (sizeof(GT) == 8) asm volatile("" : "+v"(raw[r].x), "+v"(raw[r].y));
      v[r] = ccast<CT>(raw[r]);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = ccast<CT>(row[t + r * S::T]);
    if constexpr (ZERO) {
#pragma unroll
      for (int r = 0; r < 16; ++r) row[t + r * S::T] = GT{0, 0};
    }
  }
  fft_core<N>(v, t, lds, tw);
#pragma unroll
  for (int m = 0; m < 16 / S::RF; ++m)
#pragma unroll
    for (int r = 0; r < S::RF; ++r) {
      const int k = out_pos<N, S::RF>(t, m, r, N / S::RF);
      const int64_t i = (int64_t)((k + (int)(nx / 2)) & (N - 1));
      if (i < nx) H[((i / kColBlock) * hrows + orow) * kColBlock + (i % kColBlock)] = ccast<HT>(v[m * S::RF + r]);
    }
}

// Pass B, along v, for image row i: column i of H (N = nv points) -> the ny
// kept frequencies j = (k + ny/2) mod N < ny, written straight into image row
// i with the crop epilogue:
//   MODE 0 (2-D):      dirty[i, j]  = (-1)^(p+q) Re(.) cx[i] cy[j]
//   MODE 1 (w plane):  acc[i, j] (+)= (-1)^(p+q) Re(. exp(-2 pi i w (n-1)))
// p = i - nx/2, q = j - ny/2. Blocks b, b+8, ... share an XCD (round-robin
// dispatch), so the kColBlock columns of one H block go to one XCD's L2 together.
struct ColEpilogue {
  double* out;
  const double* cx;
  const double* cy;
  double px, py, w_plane;
  int first;
  const double* norm;  // MODE 0: divide by *norm (the weight sum), NULL = no
};

// The packed class's w screen (fp32 transforms), round 6. Pass B of the
// reference call was VALU-bound on its epilogue (~130 instructions an image
// cell: fp64 sqrt with denormal scaling, an fp64 divide, ocml's general
// sincospif). Three cheaper steps with the same phase accuracy:
//  - n - 1 = sqrt(1 - e) - 1 directly: only its ABSOLUTE error enters the
//    phase (2 pi w (n - 1)), and that is one ulp of 1 (1.1e-16) whichever
//    form is used - the -e / (sqrt(1 - e) + 1) form only buys relative
//    accuracy for tiny e, which the phase does not need;
//  - sqrt(x), x = 1 - e in (0, 1]: hardware rsq_f64 and one Newton-Raphson
//    correction (no scaling: x is never denormal or huge);
//  - sin / cos (pi x) for the already-reduced |x| <= 1 (half turns): quadrant
//    n = rint(2 x), |y| = |x - n / 2| <= 1/4, Taylor polynomials of degree 9 /
//    10 (truncation < 2e-9), then the quadrant's swap and signs.
// The n - 1 and phase stay fp64 (|phase| reaches hundreds of half turns),
// only the reduced angle's sine and cosine are fp32, as before.
__device__ __forceinline__ double screen_nm1(double e) {
  const double x = 1.0 - e;
  const double y = __builtin_amdgcn_rsq(x);
  double s = x * y, h = 0.5 * y;
  const double r = fma(-h, s, 0.5);
  s = fma(s, r, s);
  h = fma(h, r, h);
  s = fma(fma(-s, s, x), h, s);
  return s - 1.0;
}

__device__ __forceinline__ void screen_sincospi(float x, float* sn, float* cs) {
  const float n = rintf(2.0f * x);
  const float y = fmaf(-0.5f, n, x);
  const float y2 = y * y;
  // pi^(2k+1) / (2k+1)! and pi^(2k) / (2k)!, alternating signs
  float ps = fmaf(y2, 0.0821458866111282f, -0.599264529320792f);
  ps = fmaf(y2, ps, 2.55016403987735f);
  ps = fmaf(y2, ps, -5.16771278004997f);
  ps = fmaf(y2, ps, 3.14159265358979f);
  float pc = fmaf(y2, -0.0258068913900140f, 0.235330630358893f);
  pc = fmaf(y2, pc, -1.33526276885459f);
  pc = fmaf(y2, pc, 4.05871212641677f);
  pc = fmaf(y2, pc, -4.93480220054468f);
  const float sv = y * ps, cv = fmaf(y2, pc, 1.0f);
  // sin / cos (pi y + n pi / 2): n mod 4 = 0 (s, c), 1 (c, -s), 2 (-s, -c), 3 (-c, s)
  const int q = (int)n & 3;
  const float a = (q & 1) ? cv : sv, b = (q & 1) ? sv : cv;
  *sn = (q & 2) ? -a : a;
  *cs = ((q + 1) & 2) ? -b : b;
}

// A strip of image rows [i0, i0 + gridDim.x): H holds the
// blocks from i0 / kColBlock on (i0 a multiple of kColBlock), and image row i
// goes to ep.out row i - i0. The whole image: i0 = 0.
// rowbits (may be NULL: every H row is read): bit ty of the plane's tile-row
// words - H rows y of clean tile rows (y / kTile) were not written by pass A
// and are zero.
// OT (MODE 1): the plane accumulator's type - double, or float for the packed
// class (its own precision; one rounding per plane: acc = (float)(acc + val))
template <int N, int MODE, typename HT = double2, typename CT = double2, typename OT = double>
__global__ __launch_bounds__(N / 16, fft_waves<CT>()) void fft_cols_kernel(const HT* __restrict__ H, int64_t nx, int64_t ny,
                                                          const double2* __restrict__ tw, ColEpilogue ep,
                                                          int64_t i0 = 0, const uint32_t* __restrict__ rowbits = nullptr) {
  using S = FftShape<N>;
  __shared__ XT<CT> lds[kXLen<N>];
  const int t = threadIdx.x;
  const int64_t b = blockIdx.x;
  const int64_t nrows = gridDim.x;
  int64_t il = b;
  // a group of 8 kColBlock consecutive blocks -> one column block per XCD
  if (nrows % (8 * kColBlock) == 0)
    il = (b / (8 * kColBlock)) * (8 * kColBlock) + (b % 8) * kColBlock + (b / 8) % kColBlock;
  const int64_t i = i0 + il;
  const HT* col = H + ((il / kColBlock) * N) * kColBlock + (il % kColBlock);
  CT v[16];
  HT raw[16];
  if (rowbits) {
    // the row-bit word of element r (rows t + r T, tile rows (t + r T) / 32)
    // is uniform over the block, as in pass A: scalar loads, one bit per lane
    static_assert(kTile == 32 && 1024 % S::T == 0, "row word per element uniform");
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int y = t + r * S::T;
      const uint32_t word = rowbits[(r * S::T) >> 10];
      raw[r] = HT{0, 0};
      if ((word >> ((y >> 5) & 31)) & 1u) raw[r] = col[(int64_t)y * kColBlock];
    }
  } else {
#pragma unroll
    for (int r = 0; r < 16; ++r) raw[r] = col[(int64_t)(t + r * S::T) * kColBlock];
  }
  // widened after every load is issued (as in pass A)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    if constexpr (sizeof(HT) == 8) asm volatile("" : "+v"(raw[r].x), "+v"(raw[r].y));
    v[r] = ccast<CT>(raw[r]);
  }
  fft_core<N>(v, t, lds, tw);
  // (nx, ny <= N <= 16384: the crop indices are 32-bit)
  const int p = (int)(i - nx / 2);
  const int nyi = (int)ny;
  OT* orow = reinterpret_cast<OT*>(ep.out) + il * ny;
  const double cxi = MODE == 0 ? (ep.norm ? ep.cx[i] / *ep.norm : ep.cx[i]) : 0.0;
  const double l = (double)p * ep.px;
  const double l2 = l * l;
  // MODE 1 accumulating into float planes: the accumulator's old values,
  // every load issued before the first is used (a load inside the loop below
  // is waited for before its own add, 8 serialised HBM round trips a lane);
  // the loads come before every store, so no aliasing holds them back. (fp64
  // planes load in the loop: 16 more doubles live would cost the fp64
  // transform its second workgroup per CU, 124 -> 154 VGPRs)
  constexpr bool kHoist = std::is_same<OT, float>::value;
  OT old[16];
  if (MODE == 1 && kHoist && !ep.first) {
#pragma unroll
    for (int m = 0; m < 16 / S::RF; ++m)
#pragma unroll
      for (int r = 0; r < S::RF; ++r) {
        const int j = (out_pos<N, S::RF>(t, m, r, N / S::RF) + nyi / 2) & (N - 1);
        old[m * S::RF + r] = j < nyi ? orow[j] : OT(0);
      }
  }
#pragma unroll
  for (int m = 0; m < 16 / S::RF; ++m)
#pragma unroll
    for (int r = 0; r < S::RF; ++r) {
      const int k = out_pos<N, S::RF>(t, m, r, N / S::RF);
      const int j = (k + nyi / 2) & (N - 1);
      if (j < nyi) {
        const int q = j - nyi / 2;
        const double sgn = ((p + q) & 1) ? -1.0 : 1.0;
        const double2 g = ccast<double2>(v[m * S::RF + r]);
        if constexpr (MODE == 0) {
          orow[j] = sgn * g.x * cxi * ep.cy[j];
        } else {
          const double mm = (double)q * ep.py;
          const double e = fma(mm, mm, l2);
          double sn, cs;
          if constexpr (sizeof(CT) == 8 && CIP_SCREEN_F32 == 1) {
            // fp32 transforms (the packed class): the phase / pi is reduced
            // exactly in fp64 to [-1, 1] (period 2) and only its sine and
            // cosine are fp32 - ~1e-7, the class's own rounding of the plane
            // values (screen_nm1 / screen_sincospi above)
            const double ph = -2.0 * ep.w_plane * screen_nm1(e);
            const float red = (float)(ph - 2.0 * rint(0.5 * ph));
            float sf, cf;
            screen_sincospi(red, &sf, &cf);
            sn = sf;
            cs = cf;
          } else if constexpr (sizeof(CT) == 8 && CIP_SCREEN_F32 == 2) {
            sn = 0.0 * e;  // ablation (timing only, wrong images)
            cs = 1.0;
          } else {
            const double nm1 = -e / (sqrt(1.0 - e) + 1.0);
            const double ph = -2.0 * ep.w_plane * nm1;  // the screen's phase / pi
            sincospi(ph, &sn, &cs);
          }
          // one rounding per plane for float planes: acc = (OT)((double)acc + val)
          const double val = sgn * (g.x * cs - g.y * sn);
          if (ep.first) orow[j] = (OT)val;
          else orow[j] = (OT)((double)(kHoist ? old[m * S::RF + r] : orow[j]) + val);
        }
      }
    }
}

// Pass B of the 2-D crop for fp64 columns of N = 2 NH points (C4's 16384;
// round 6) as their even and odd halves in one workgroup, one after the other:
//   X[k] = E[k'] + w^k' O[k'],  X[k + NH] = E[k'] - w^k' O[k'],  w = exp(2 pi i / N)
// (E, O: the NH-point transforms of the column's even / odd rows, which pass A
// wrote as the contiguous H halves: fft_rows_kernel EO). One N-point fp64
// transform is 256 KiB of registers and 128 KiB of LDS, so fft_cols_kernel
// runs ONE workgroup per CU, and a CU alternates between loading its column
// (HBM busy, ALUs idle) and transforming it (the reverse): pass B ran at ~33 %
// of the HBM roof. The NH-point halves need 64 KiB of LDS and <= 128 VGPRs:
// two workgroups per CU, one loading while the other transforms.
// With ny <= N / 2 (the host checks) at most one of k', k' + NH is kept. The
// even half stores Re E[k'] into its output cell, the odd half reads it back
// (the same lane: both halves use one output mapping) and finishes
//   dirty[i, j] = (-1)^(p+q) (Re E[k'] +- Re(w^k' O[k'])) cx[i] cy[j].
// Loads before stores, batches of 8 (see the MODE 1 epilogue).
template <int NH>
__global__ __launch_bounds__(NH / 16, 4) void fft_cols_eo_kernel(const double2* __restrict__ H, int64_t nx,
                                                              int64_t ny, const double2* __restrict__ tw,
                                                              ColEpilogue ep, const uint32_t* __restrict__ rowbits) {
  constexpr int N = 2 * NH;
  using S = FftShape<NH>;
  // k' = t + m T + r NH / 2 (out_pos with a final radix-2 pass)
  static_assert(S::RF == 2 && NH / 16 <= 1024 && kTile == 32, "even / odd pass B layout");
  __shared__ double lds[kXLen<NH>];
  const int64_t b = blockIdx.x;
  int64_t il = b;
  if (gridDim.x % (8 * kColBlock) == 0)
    il = (b / (8 * kColBlock)) * (8 * kColBlock) + (b % 8) * kColBlock + (b / 8) % kColBlock;
  const int64_t i = il;
  const double2* col = H + ((il / kColBlock) * N) * kColBlock + (il % kColBlock);
  const int p = (int)(i - nx / 2);
  const int nyi = (int)ny;
  double* orow = ep.out + il * ny;
  const double cxi = ep.norm ? ep.cx[i] / *ep.norm : ep.cx[i];
  // the output cell of element x (mod N: the kept one of k', k' + NH), or -1;
  // tt / nyy: t and ny re-issued after each transform (below), so the
  // compiler cannot compute the 16 cells ahead, inside the transform, where
  // their registers spill
  int tt = threadIdx.x, nyy = nyi;
  auto cell = [&](int x, bool* plus) {
    const int kp = out_pos<NH, 2>(tt, x / 2, x % 2, NH / 2);
    const int j0 = (kp + nyy / 2) & (N - 1), j1 = (kp + NH + nyy / 2) & (N - 1);
    *plus = j0 < nyy;
    return j0 < nyy ? j0 : (j1 < nyy ? j1 : -1);
  };
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    const double2* hc = col + (int64_t)half * NH * kColBlock;
    // the lane index re-issued per half: the compiler kept the transform's
    // t-derived LDS addresses live from the first half to the second, and they
    // spilled
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    double2 v[16];
    if (rowbits) {
      // H row n of a half is grid row 2 n + half, tile row n / 16: the word of
      // element r ((t + r T) / 512 = r) is uniform over the block
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = t + r * S::T;
        const uint32_t word = rowbits[(r * S::T) >> 9];
        v[r] = make_double2(0.0, 0.0);
        if ((word >> ((n >> 4) & 31)) & 1u) v[r] = hc[(int64_t)n * kColBlock];
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = hc[(int64_t)(t + r * S::T) * kColBlock];
    }
    fft_core<NH, double2, 2, true>(v, t, lds, tw);
    asm volatile("" : "+v"(tt), "+s"(nyy)::"memory");
    if (half == 0) {
#pragma unroll
      for (int x = 0; x < 16; ++x) {
        bool plus;
        const int j = cell(x, &plus);
        if (j >= 0) orow[j] = v[x].x;
      }
    } else {
      // z = Re(w^k' O[k']), w^k' = w^t (w^T)^m i^r: one table load per lane
      // and the 8 constants w^(m T) = exp(2 pi i m / 32) (immediates: loaded
      // from the table, the compiler hoisted them into the transform, where
      // they spilled); formed for all 16 elements first, so the transform's
      // registers are free for the loads below
      static_assert(N / S::T == 32, "w^T = exp(2 pi i / 32)");
      constexpr double kc[8] = {1.0, 0.9807852804032304, 0.9238795325112867, 0.8314696123025452,
                                0.7071067811865476, 0.5555702330196023, 0.38268343236508984, 0.19509032201612833};
      constexpr double ks[8] = {0.0, 0.19509032201612825, 0.3826834323650898, 0.5555702330196022,
                                0.7071067811865475, 0.8314696123025452, 0.9238795325112867, 0.9807852804032304};
      const double2 wt = tw[t];
      double z[16];
#pragma unroll
      for (int x = 0; x < 16; ++x) {
        const double2 wm = cmul(wt, make_double2(kc[x / 2], ks[x / 2]));
        const double2 w = (x % 2) ? make_double2(-wm.y, wm.x) : wm;  // times i^r, r = x % 2
        z[x] = fma(w.x, v[x].x, -w.y * v[x].y);
      }
#pragma unroll
      for (int c = 0; c < 16; c += 4) {
        double e[4], cyv[4];
#pragma unroll
        for (int x = c; x < c + 4; ++x) {
          bool plus;
          const int j = cell(x, &plus);
          e[x - c] = orow[j >= 0 ? j : 0];
          cyv[x - c] = ep.cy[j >= 0 ? j : 0];
        }
#pragma unroll
        for (int x = c; x < c + 4; ++x) {
          bool plus;
          const int j = cell(x, &plus);
          const int q = j - nyi / 2;
          const double sgn = ((p + q) & 1) ? -1.0 : 1.0;
          e[x - c] = sgn * (plus ? e[x - c] + z[x] : e[x - c] - z[x]) * cxi * cyv[x - c];
        }
#pragma unroll
        for (int x = c; x < c + 4; ++x) {
          bool plus;
          const int j = cell(x, &plus);
          if (j >= 0) orow[j] = e[x - c];
        }
      }
    }
  }
}

// CIP_FFT_F32=0: the packed class's complex64 planes transformed in fp64
// (the round-4 form); default: in fp32, the class's own precision
bool fft_f32_enabled() {
  static const bool on = [] {
    const char* e = getenv("CIP_FFT_F32");
    return !(e && e[0] == '0');
  }();
  return on;
}

static bool fft_len_ok(int64_t n) { return n == 1024 || n == 2048 || n == 4096 || n == 8192 || n == 16384; }

bool fast_fft_supported(int64_t nu, int64_t nv, int64_t nx, int64_t ny) {
  return fft_len_ok(nu) && fft_len_ok(nv) && nx > 0 && ny > 0 && nx <= nu && ny <= nv && nx % kColBlock == 0 &&
         ny % 2 == 0;
}

bool fft_cols_eo(int64_t nv, int64_t ny, bool grid_f32, int mode) {
  return CIP_FFT_EO && nv == 16384 && ny <= nv / 2 && !grid_f32 && mode == 0;
}

hipError_t launch_fft_rows(double* gT, int64_t nu, int64_t nv, int64_t nx, const double* tw_u, double* H,
                           const uint32_t* dmask, int64_t ntx, bool skip_clean, hipStream_t s, bool grid_f32,
                           bool eo) {
  if (!fft_len_ok(nu) || !fft_len_ok(nv) || nx > nu) return hipErrorInvalidValue;
  if (eo && (grid_f32 || nv % 2 != 0)) return hipErrorInvalidValue;
  if (dmask && (nu % kTile != 0 || nv % kTile != 0 || ntx * kTile != nu || ntx % 32 != 0))
    return hipErrorInvalidValue;
  const dim3 gd((unsigned)nv);
  double2* g = (double2*)gT;
  float2* gf = (float2*)gT;
  const double2* tw = (const double2*)tw_u;
  double2* h = (double2*)H;
  float2* hf = (float2*)H;  // complex64 planes: complex64 pass-A output
  const bool fft_f32 = fft_f32_enabled();
#define ROWS(NN)                                                                                              \
  case NN:                                                                                                    \
    if (grid_f32 && dmask && fft_f32)                                                                         \
      fft_rows_kernel<NN, true, false, float2, float2, float2><<<gd, dim3(NN / 16), 0, s>>>(                  \
          gf, nv, nx, tw, hf, dmask, ntx, 0, 0, skip_clean);                                                  \
    else if (grid_f32 && fft_f32)                                                                             \
      fft_rows_kernel<NN, false, false, float2, float2, float2><<<gd, dim3(NN / 16), 0, s>>>(gf, nv, nx, tw,  \
                                                                                             hf, nullptr, 0); \
    else if (grid_f32 && dmask)                                                                               \
      fft_rows_kernel<NN, true, false, float2, float2><<<gd, dim3(NN / 16), 0, s>>>(gf, nv, nx, tw, hf, dmask, \
                                                                                    ntx, 0, 0, skip_clean);   \
    else if (grid_f32)                                                                                        \
      fft_rows_kernel<NN, false, false, float2, float2><<<gd, dim3(NN / 16), 0, s>>>(gf, nv, nx, tw, hf,      \
                                                                                     nullptr, 0);             \
    else if (dmask && eo)                                                                                     \
      fft_rows_kernel<NN, true, false, double2, double2, double2, true><<<gd, dim3(NN / 16), 0, s>>>(         \
          g, nv, nx, tw, h, dmask, ntx, 0, 0, skip_clean);                                                    \
    else if (eo)                                                                                              \
      fft_rows_kernel<NN, false, false, double2, double2, double2, true><<<gd, dim3(NN / 16), 0, s>>>(        \
          g, nv, nx, tw, h, nullptr, 0);                                                                      \
    else if (dmask)                                                                                           \
      fft_rows_kernel<NN, true><<<gd, dim3(NN / 16), 0, s>>>(g, nv, nx, tw, h, dmask, ntx, 0, 0, skip_clean); \
    else                                                                                                      \
      fft_rows_kernel<NN, false><<<gd, dim3(NN / 16), 0, s>>>(g, nv, nx, tw, h, nullptr, 0);                  \
    break;
  switch (nu) {
    ROWS(1024)
    ROWS(2048)
    ROWS(4096)
    ROWS(8192)
    ROWS(16384)
    default: return hipErrorInvalidValue;
  }
#undef ROWS
  return hipGetLastError();
}

hipError_t launch_fft_rows_strip(double* gT, int64_t nu, int64_t nv, int64_t nx, const double* tw_u, int64_t y0,
                                 int64_t y1, double* H, hipStream_t s, const uint32_t* dmask, int64_t row0,
                                 const int64_t* row_slot, int64_t nlive) {
  if (!fft_len_ok(nu) || !fft_len_ok(nv) || nx > nu || y0 < 0 || y1 > nv || y1 <= y0) return hipErrorInvalidValue;
  if (dmask && (nu % kTile != 0 || nv % kTile != 0 || (nu / kTile) % 32 != 0)) return hipErrorInvalidValue;
  const dim3 gd((unsigned)(y1 - y0));
  double2* g = (double2*)gT;
  const double2* tw = (const double2*)tw_u;
  double2* h = (double2*)H;
  const int64_t ntx = nu / kTile;
#define ROWS(NN)                                                                                               \
  case NN:                                                                                                     \
    if (dmask)                                                                                                 \
      fft_rows_kernel<NN, true, false><<<gd, dim3(NN / 16), 0, s>>>(g, row_slot ? nlive : y1 - y0, nx, tw, h,   \
                                                                     dmask, ntx, y0, y0, false, row0, nv,      \
                                                                     row_slot);                                \
    else                                                                                                       \
      fft_rows_kernel<NN, false, true><<<gd, dim3(NN / 16), 0, s>>>(g, y1 - y0, nx, tw, h, nullptr, 0, y0, y0); \
    break;
  switch (nu) {
    ROWS(1024)
    ROWS(2048)
    ROWS(4096)
    ROWS(8192)
    ROWS(16384)
    default: return hipErrorInvalidValue;
  }
#undef ROWS
  return hipGetLastError();
}

hipError_t launch_fft_cols_strip(const double* H, int64_t nv, int64_t nx, int64_t ny, const double* tw_v, int64_t i0,
                                 int64_t i1, double* out, const double* cx, const double* cy, const double* norm,
                                 hipStream_t s) {
  if (i0 < 0 || i1 > nx || i1 <= i0 || i0 % kColBlock != 0 || (i1 - i0) % kColBlock != 0)
    return hipErrorInvalidValue;
  const dim3 gd((unsigned)(i1 - i0));
  const double2* h = (const double2*)H;
  const double2* tw = (const double2*)tw_v;
  const ColEpilogue ep{out, cx, cy, 0.0, 0.0, 0.0, 1, norm};
#define COLS(NN)                                                                          \
  case NN:                                                                                \
    fft_cols_kernel<NN, 0><<<gd, dim3(NN / 16), 0, s>>>(h, nx, ny, tw, ep, i0);           \
    break;
  switch (nv) {
    COLS(1024)
    COLS(2048)
    COLS(4096)
    COLS(8192)
    COLS(16384)
    default:
      return hipErrorInvalidValue;
  }
#undef COLS
  return hipGetLastError();
}

hipError_t launch_fft_cols_strip_wplane(const double* H, int64_t nv, int64_t nx, int64_t ny, const double* tw_v,
                                        int64_t i0, int64_t i1, double* acc, double px, double py, double w_plane,
                                        bool first, hipStream_t s) {
  if (i0 < 0 || i1 > nx || i1 <= i0 || i0 % kColBlock != 0 || (i1 - i0) % kColBlock != 0)
    return hipErrorInvalidValue;
  const dim3 gd((unsigned)(i1 - i0));
  const double2* h = (const double2*)H;
  const double2* tw = (const double2*)tw_v;
  const ColEpilogue ep{acc, nullptr, nullptr, px, py, w_plane, first ? 1 : 0, nullptr};
#define COLS(NN)                                                                \
  case NN:                                                                      \
    fft_cols_kernel<NN, 1><<<gd, dim3(NN / 16), 0, s>>>(h, nx, ny, tw, ep, i0); \
    break;
  switch (nv) {
    COLS(1024)
    COLS(2048)
    COLS(4096)
    COLS(8192)
    COLS(16384)
    default:
      return hipErrorInvalidValue;
  }
#undef COLS
  return hipGetLastError();
}

hipError_t launch_fft_cols(const double* H, int64_t nv, int64_t nx, int64_t ny, const double* tw_v, int mode,
                           double* out, const double* cx, const double* cy, double px, double py, double w_plane,
                           int first, const double* norm, const uint32_t* rowbits, hipStream_t s, bool h_f32,
                           bool acc_f32, bool eo) {
  const dim3 gd((unsigned)nx);
  const double2* h = (const double2*)H;
  const float2* hf = (const float2*)H;
  const double2* tw = (const double2*)tw_v;
  const ColEpilogue ep{out, cx, cy, px, py, w_plane, first, norm};
  if (eo) {
    // pass A wrote the even / odd H halves (launch_fft_rows eo)
    if (!fft_cols_eo(nv, ny, h_f32, mode)) return hipErrorInvalidValue;
    fft_cols_eo_kernel<8192><<<gd, dim3(8192 / 16), 0, s>>>(h, nx, ny, tw, ep, rowbits);
    return hipGetLastError();
  }
  const bool fft_f32 = fft_f32_enabled();
  // the float plane accumulator exists only beside fp32 transforms of
  // complex64 planes (with CIP_FFT_F32=0 the fp64-output kernel
  // would write doubles across twice the float buffer's bytes)
  if (acc_f32 && !(h_f32 && fft_f32 && mode == 1)) return hipErrorInvalidValue;
#define COLS(NN)                                                                                           \
  case NN:                                                                                                 \
    if (h_f32 && fft_f32 && mode == 1 && acc_f32)                                                          \
      fft_cols_kernel<NN, 1, float2, float2, float><<<gd, dim3(NN / 16), 0, s>>>(hf, nx, ny, tw, ep, 0,     \
                                                                                 rowbits);                \
    else if (h_f32 && fft_f32 && mode == 0)                                                                \
      fft_cols_kernel<NN, 0, float2, float2><<<gd, dim3(NN / 16), 0, s>>>(hf, nx, ny, tw, ep, 0, rowbits);  \
    else if (h_f32 && fft_f32)                                                                             \
      fft_cols_kernel<NN, 1, float2, float2><<<gd, dim3(NN / 16), 0, s>>>(hf, nx, ny, tw, ep, 0, rowbits);  \
    else if (h_f32 && mode == 0) fft_cols_kernel<NN, 0, float2><<<gd, dim3(NN / 16), 0, s>>>(hf, nx, ny, tw, ep, 0, rowbits); \
    else if (h_f32) fft_cols_kernel<NN, 1, float2><<<gd, dim3(NN / 16), 0, s>>>(hf, nx, ny, tw, ep, 0, rowbits);         \
    else if (mode == 0) fft_cols_kernel<NN, 0><<<gd, dim3(NN / 16), 0, s>>>(h, nx, ny, tw, ep, 0, rowbits); \
    else fft_cols_kernel<NN, 1><<<gd, dim3(NN / 16), 0, s>>>(h, nx, ny, tw, ep, 0, rowbits);              \
    break;
  switch (nv) {
    COLS(1024)
    COLS(2048)
    COLS(4096)
    COLS(8192)
    COLS(16384)
    default:
      return hipErrorInvalidValue;
  }
#undef COLS
  return hipGetLastError();
}

// out[k] /= *sumw (CIP_NORMALISE on the paths without the fused epilogue)
__global__ void scale_inverse_kernel(double* __restrict__ out, int64_t n, const double* __restrict__ sumw) {
  const double d = *sumw;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
    out[k] /= d;
}

hipError_t launch_scale_inverse(double* out, int64_t n, const double* sumw, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t nb = std::min<int64_t>((n + 255) / 256, 4096);
  scale_inverse_kernel<<<dim3((unsigned)nb), dim3(256), 0, s>>>(out, n, sumw);
  return hipGetLastError();
}

}  // namespace cip
