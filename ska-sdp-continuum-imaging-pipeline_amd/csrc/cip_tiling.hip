// cip_tiling.hip - reference-exact UVW tile keys / runs (uvw_tiling API) and
// the Stokes-I gridder-input conversion.
//
// Tile key (reference uvw_tiling/tiling_plan.py:41-51):
//   wavelength_inv = channel_freqs / 299792458.0          (correctly rounded)
//   key = floor(wavelength_inv * (row_uvw / tile_size) + 0.5)
// evaluated in that order in fp64 with no contraction, so every sample lands in
// exactly the reference's tile, including samples on a tile boundary. Runs of
// constant key along the channel axis replace the reference's recursive
// bisection (tiling_plan.py:150-181): keys are monotone in frequency, so the
// maximal constant runs are the same set, found here by one linear pass per
// row on the device.
#include "cip_internal.h"

namespace cip {

__global__ void wavelength_inv_kernel(const double* freq, int64_t nchan, double* winv) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c < nchan) winv[c] = freq[c] / CIP_SPEED_OF_LIGHT;
}

hipError_t launch_wavelength_inv(const double* freq, int64_t nchan, double* winv, hipStream_t s) {
  wavelength_inv_kernel<<<dim3((unsigned)((nchan + 255) / 256)), dim3(256), 0, s>>>(freq, nchan, winv);
  return hipGetLastError();
}

__device__ __forceinline__ void ref_key(double a0, double a1, double a2, double wi, int64_t* k) {
#pragma clang fp contract(off)
  k[0] = (int64_t)floor(wi * a0 + 0.5);
  k[1] = (int64_t)floor(wi * a1 + 0.5);
  k[2] = (int64_t)floor(wi * a2 + 0.5);
}

template <bool EMIT>
__global__ __launch_bounds__(256) void tile_runs_kernel(const double* __restrict__ uvw, int64_t nrow,
                                                        const double* __restrict__ winv, int64_t nchan, double t0,
                                                        double t1, double t2, int64_t row_offset,
                                                        int64_t* row_runs, const int64_t* __restrict__ row_off,
                                                        int64_t* run_key, int64_t* run_row, int32_t* run_c0,
                                                        int32_t* run_c1) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrow) return;
  // row_uvw / tile_size, correctly rounded as numpy does
  const double a0 = uvw[3 * r] / t0, a1 = uvw[3 * r + 1] / t1, a2 = uvw[3 * r + 2] / t2;
  int64_t prev[3];
  ref_key(a0, a1, a2, winv[0], prev);
  int64_t start = 0, n = 0, out = EMIT ? row_off[r] : 0;
  for (int64_t c = 1; c <= nchan; ++c) {
    int64_t k[3] = {0, 0, 0};
    bool change = true;
    if (c < nchan) {
      ref_key(a0, a1, a2, winv[c], k);
      change = (k[0] != prev[0]) || (k[1] != prev[1]) || (k[2] != prev[2]);
    }
    if (change) {
      if (EMIT) {
        run_key[3 * out] = prev[0];
        run_key[3 * out + 1] = prev[1];
        run_key[3 * out + 2] = prev[2];
        run_row[out] = r + row_offset;
        run_c0[out] = (int32_t)start;
        run_c1[out] = (int32_t)c;
        ++out;
      } else {
        ++n;
      }
      start = c;
      prev[0] = k[0];
      prev[1] = k[1];
      prev[2] = k[2];
    }
  }
  if (!EMIT) row_runs[r] = n;
}

hipError_t launch_tile_run_count(const double* uvw, int64_t nrow, const double* winv, int64_t nchan, double t0,
                                 double t1, double t2, int64_t* row_runs, hipStream_t s) {
  tile_runs_kernel<false><<<dim3((unsigned)((nrow + 255) / 256)), dim3(256), 0, s>>>(
      uvw, nrow, winv, nchan, t0, t1, t2, 0, row_runs, nullptr, nullptr, nullptr, nullptr, nullptr);
  return hipGetLastError();
}

hipError_t launch_tile_run_emit(const double* uvw, int64_t nrow, const double* winv, int64_t nchan, double t0,
                                double t1, double t2, int64_t row_offset, const int64_t* row_off, int64_t* run_key,
                                int64_t* run_row, int32_t* run_c0, int32_t* run_c1, hipStream_t s) {
  tile_runs_kernel<true><<<dim3((unsigned)((nrow + 255) / 256)), dim3(256), 0, s>>>(
      uvw, nrow, winv, nchan, t0, t1, t2, row_offset, nullptr, row_off, run_key, run_row, run_c0, run_c1);
  return hipGetLastError();
}

// Stokes parameters from linear feeds (XX, XY, YX, YY) = pols (0, 1, 2, 3),
// one thread per (row, chan). I (reference invert.py:86-116, :72-76, its
// numpy float32 arithmetic): 0.5 (XX + YY), flags F0 | F3, weight
// 4 / (1/w0 + 1/w3). Q = 0.5 (XX - YY) with I's flags and weights; U =
// 0.5 (XY + YX) and V = -0.5 i (XY - YX) with pols 1 and 2's.
template <int STOKES>
__global__ void stokes_kernel(const float2* __restrict__ vis4, const uint8_t* __restrict__ flags4,
                              const float* __restrict__ wgt4, int64_t n, float2* vis_i, uint8_t* flag_i,
                              float* wgt_i, float* eff_w) {
  constexpr int A = STOKES <= 1 ? 0 : 1, B = STOKES <= 1 ? 3 : 2;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (vis_i) {
    const float2 a = vis4[4 * i + A], d = vis4[4 * i + B];
    // numpy: 0.5 * (vis[..., 0] + vis[..., 3]) in complex64
    if constexpr (STOKES == 0 || STOKES == 2) vis_i[i] = make_float2(0.5f * (a.x + d.x), 0.5f * (a.y + d.y));
    if constexpr (STOKES == 1) vis_i[i] = make_float2(0.5f * (a.x - d.x), 0.5f * (a.y - d.y));
    if constexpr (STOKES == 3) vis_i[i] = make_float2(0.5f * (a.y - d.y), -0.5f * (a.x - d.x));
  }
  bool fl = false;
  if (flags4) fl = (flags4[4 * i + A] != 0) || (flags4[4 * i + B] != 0);
  if (flag_i) flag_i[i] = fl ? 1 : 0;
  if (wgt4) {
    const float wa = wgt4[4 * i + A], wb = wgt4[4 * i + B];
    // numpy float32: 4.0 / (1.0 / wxx + 1.0 / wyy); a zero weight gives
    // 1/0 = inf and 4/inf = 0 exactly as in the reference.
    const float w = 4.0f / (1.0f / wa + 1.0f / wb);
    if (wgt_i) wgt_i[i] = w;
    // numpy: logical_not(flags) * weights (so 0 * inf / nan propagate)
    if (eff_w) eff_w[i] = (fl ? 0.0f : 1.0f) * w;
  }
}

hipError_t launch_stokes(int stokes, const void* vis4, const uint8_t* flags4, const float* wgt4, int64_t n,
                         void* vis_i, uint8_t* flag_i, float* wgt_i, float* eff_w, hipStream_t s) {
  const dim3 gd((unsigned)((n + 255) / 256)), bd(256);
#define STK(K)                                                                                              \
  stokes_kernel<K><<<gd, bd, 0, s>>>((const float2*)vis4, flags4, wgt4, n, (float2*)vis_i, flag_i, wgt_i, eff_w)
  switch (stokes) {
    case 0: STK(0); break;
    case 1: STK(1); break;
    case 2: STK(2); break;
    case 3: STK(3); break;
    default: return hipErrorInvalidValue;
  }
#undef STK
  return hipGetLastError();
}

// ------------------------------------------------------------ facets ----
// Rephase to a facet centre s0 = (l0, m0, n0) of the original tangent plane
// and rotate the baselines into the facet's frame. In the convention of
// ms2dirty (dirty = sum Re{V exp(2 pi i f/c (u l + v m - w (n - 1)))}) a source
// at s has delay d(s) = b.s - b.z with b = (u, v, -w); the facet data are
// V' = V exp(+2 pi i f/c d(s0)) and b' = Q^T b (Q: the rotation taking z to
// s0, rows q_k), stored back as (u', v', w') = (b'_0, b'_1, -b'_2).
// One thread per row rotates uvw; one per visibility rotates the phase.
struct Rot3 {
  double q[9];  // row-major Q^T
};

__global__ void facet_uvw_kernel(const double* __restrict__ uvw, int64_t nrow, Rot3 qt, double l0, double m0,
                                 double n0m1, double* __restrict__ uvw_out, double* __restrict__ delay) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrow) return;
  const double b0 = uvw[3 * r], b1 = uvw[3 * r + 1], b2 = -uvw[3 * r + 2];
  delay[r] = b0 * l0 + b1 * m0 + b2 * n0m1;  // b.s0 - b.z (metres)
  uvw_out[3 * r] = qt.q[0] * b0 + qt.q[1] * b1 + qt.q[2] * b2;
  uvw_out[3 * r + 1] = qt.q[3] * b0 + qt.q[4] * b1 + qt.q[5] * b2;
  uvw_out[3 * r + 2] = -(qt.q[6] * b0 + qt.q[7] * b1 + qt.q[8] * b2);
}

template <typename VisT>
__global__ void facet_phase_kernel(const VisT* __restrict__ vis, const double* __restrict__ delay,
                                   const double* __restrict__ freq, int64_t nrow, int64_t nchan,
                                   VisT* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nrow * nchan) return;
  const int64_t r = i / nchan, c = i - r * nchan;
  // phase in turns, reduced before sincospi keeps the argument small
  double turns = delay[r] * (freq[c] / CIP_SPEED_OF_LIGHT);
  turns -= rint(turns);
  double sn, cs;
  sincospi(2.0 * turns, &sn, &cs);
  const double vr = (double)vis[i].x, vi = (double)vis[i].y;
  VisT o;
  o.x = vr * cs - vi * sn;
  o.y = vr * sn + vi * cs;
  out[i] = o;
}

hipError_t launch_facet_rephase(const double* uvw, int64_t nrow, const double* freq, int64_t nchan, const void* vis,
                                int vis_c128, const double qt[9], double l0, double m0, double* uvw_out,
                                double* delay, void* vis_out, hipStream_t s) {
  Rot3 q;
  for (int k = 0; k < 9; ++k) q.q[k] = qt[k];
  const double n0m1 = -(l0 * l0 + m0 * m0) / (sqrt(1.0 - l0 * l0 - m0 * m0) + 1.0);  // n0 - 1, no cancellation
  facet_uvw_kernel<<<dim3((unsigned)((nrow + 255) / 256)), dim3(256), 0, s>>>(uvw, nrow, q, l0, m0, n0m1, uvw_out,
                                                                               delay);
  const int64_t n = nrow * nchan;
  if (n > 0 && vis != nullptr && vis_out != nullptr) {  // uvw only (PSF): no phase pass
    const dim3 gd((unsigned)((n + 255) / 256));
    if (vis_c128)
      facet_phase_kernel<double2><<<gd, dim3(256), 0, s>>>((const double2*)vis, delay, freq, nrow, nchan,
                                                           (double2*)vis_out);
    else
      facet_phase_kernel<float2><<<gd, dim3(256), 0, s>>>((const float2*)vis, delay, freq, nrow, nchan,
                                                          (float2*)vis_out);
  }
  return hipGetLastError();
}

}  // namespace cip
