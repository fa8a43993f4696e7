// cip_fft.hip - the dirty image's first FFT axis as a hand-written row FFT
// with a pruned output.
//
// The image only needs the npix_y frequencies q in [-npix_y/2, npix_y/2) of
// each grid row, i.e. half of them for sigma = 2. row_fft_kernel transforms
// one grid row (length N = nv, a power of two from 1024 to 8192) per
// workgroup of N/16 threads, each holding 16 complex values in registers:
// radix-16 (and a last radix-2/4/8) Stockham passes, exchanged through a
// "half" LDS array (real parts, then imaginary parts: 17/16 N doubles = 68 KiB
// at N = 8192, two workgroups per CU), and writes only the kept columns,
// H[x, j] = sum_y G[x, y] exp(+2 pi i y (j - npix_y/2) / nv), as a
// (nu, npix_y) row-major array. The column FFT (along x) then runs on half
// the data (hipFFT, strided batch) and the crop kernels read H directly.
// HBM traffic of this pass: 16 nu nv bytes read + 16 nu npix_y written,
// against 32 nu nv for a full c2c pass of hipFFT's row transform.
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

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}

// v * exp(+2 pi i k / M) for compile-time k, M (exact special cases)
template <int K, int M>
__device__ __forceinline__ double2 twc(double2 v) {
  constexpr int k = ((K % M) + M) % M;
  if constexpr (k == 0) return v;
  else if constexpr (4 * k == M) return make_double2(-v.y, v.x);          // * i
  else if constexpr (2 * k == M) return make_double2(-v.x, -v.y);         // * -1
  else if constexpr (4 * k == 3 * M) return make_double2(v.y, -v.x);      // * -i
  else {
    static_assert(16 % M == 0, "twiddle table covers M | 16");
    constexpr int idx = k * (16 / M);
    const double c = kW16c[idx], s = kW16c[(idx + 12) & 15];  // sin(t) = cos(t - pi/2)
    return make_double2(fma(v.x, c, -v.y * s), fma(v.x, s, v.y * c));
  }
}

// In-register DFT of size R (R | 16), natural order in and out, sign +.
// Radix-2 decimation in frequency, then the bit-reversed result re-indexed
// at compile time.
template <int R>
__device__ __forceinline__ void dft(double2* v) {
#pragma unroll
  for (int span = R / 2; span >= 1; span >>= 1) {
#pragma unroll
    for (int b = 0; b < R; b += 2 * span) {
#pragma unroll
      for (int i = 0; i < span; ++i) {
        const double2 a = v[b + i], c = v[b + i + span];
        v[b + i] = make_double2(a.x + c.x, a.y + c.y);
        const double2 d = make_double2(a.x - c.x, a.y - c.y);
        // twiddle exp(+2 pi i i / (2 span)) = W16^(i * 16 / (2 span))
        switch (2 * span) {
          case 2: v[b + i + span] = d; break;
          case 4: v[b + i + span] = (i == 0) ? d : make_double2(-d.y, d.x); break;
          default: {
            const int idx = (i * 16 / (2 * span)) & 15;
            const double cc = kW16c[idx], ss = kW16c[(idx + 12) & 15];
            v[b + i + span] = (i == 0) ? d : make_double2(fma(d.x, cc, -d.y * ss), fma(d.x, ss, d.y * cc));
          }
        }
      }
    }
  }
  double2 t[R];
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
template <int N, int R>
__device__ __forceinline__ void stockham_pass(double2* v, int t, int ns, const double2* __restrict__ tw) {
  constexpr int T = N / 16;
#pragma unroll
  for (int m = 0; m < 16 / R; ++m) {
    const int j = t + m * T;
    const int k = j & (ns - 1);
    if (ns > 1) {
#pragma unroll
      for (int r = 1; r < R; ++r) {
        // exp(+2 pi i r k / (ns R)) = tw[r k N / (ns R)]
        const int e = (r * k * (N / (ns * R))) & (N - 1);
        v[m * R + r] = cmul(v[m * R + r], tw[e]);
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

// one padding double per 16: a thread's 16 consecutive outputs (first
// exchange) then start 17 doubles apart, so 32 lanes cover all 64 banks
__device__ __forceinline__ int pad(int p) { return p + (p >> 4); }

template <int N, int R, int R2>
__device__ __forceinline__ void exchange(double2* v, int t, int ns, double* lds) {
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
        const double x = lds[pad(in_pos<N, R2>(t, m, r))];
        if (half) v[m * R2 + r].y = x;
        else v[m * R2 + r].x = x;
      }
    __syncthreads();
  }
}

// log2 N = 4 P + B: P radix-16 passes then one radix-2^B pass (B = 0: none)
template <int N>
__global__ __launch_bounds__(N / 16) void row_fft_kernel(const double2* __restrict__ grid, int64_t ny,
                                                         const double2* __restrict__ tw, double2* __restrict__ out) {
  constexpr int T = N / 16;
  constexpr int L = __builtin_ctz(N);
  constexpr int P = L / 4, B = L % 4, RL = 1 << B;
  __shared__ double lds[N + N / 16];
  const int t = threadIdx.x;
  const int64_t x = blockIdx.x;
  const double2* row = grid + x * N;
  double2 v[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = row[t + r * T];
  int ns = 1;
  stockham_pass<N, 16>(v, t, ns, tw);
#pragma unroll
  for (int p = 1; p < P; ++p) {
    exchange<N, 16, 16>(v, t, ns, lds);
    ns *= 16;
    stockham_pass<N, 16>(v, t, ns, tw);
  }
  constexpr int RF = B ? RL : 16;  // radix of the final pass
  if constexpr (B != 0) {
    exchange<N, 16, RL>(v, t, ns, lds);
    ns *= 16;
    stockham_pass<N, RL>(v, t, ns, tw);
  }
  // final outputs: frequency k = out_pos (< N); keep j = (k + ny/2) mod N < ny
  double2* orow = out + x * ny;
#pragma unroll
  for (int m = 0; m < 16 / RF; ++m)
#pragma unroll
    for (int r = 0; r < RF; ++r) {
      const int k = out_pos<N, RF>(t, m, r, ns);
      const int64_t j = (int64_t)((k + (int)(ny / 2)) & (N - 1));
      if (j < ny) orow[j] = v[m * RF + r];
    }
}

bool row_fft_supported(int64_t nv, int64_t ny) {
  return (nv == 1024 || nv == 2048 || nv == 4096 || nv == 8192) && ny <= nv && ny > 0 && (ny % 2) == 0;
}

hipError_t launch_row_fft(const double* grid, int64_t nu, int64_t nv, int64_t ny, const double* twiddles,
                          double* out, hipStream_t s) {
  const dim3 gd((unsigned)nu);
  const double2* g = (const double2*)grid;
  const double2* tw = (const double2*)twiddles;
  double2* o = (double2*)out;
  switch (nv) {
    case 1024: row_fft_kernel<1024><<<gd, dim3(64), 0, s>>>(g, ny, tw, o); break;
    case 2048: row_fft_kernel<2048><<<gd, dim3(128), 0, s>>>(g, ny, tw, o); break;
    case 4096: row_fft_kernel<4096><<<gd, dim3(256), 0, s>>>(g, ny, tw, o); break;
    case 8192: row_fft_kernel<8192><<<gd, dim3(512), 0, s>>>(g, ny, tw, o); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace cip
