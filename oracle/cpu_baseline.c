/*
 * cpu_baseline.c - TEST / BENCHMARK INFRASTRUCTURE ONLY: the CPU baseline that
 * bench.py times beside the GPU (BASELINE.md "CPU baseline plan"). ducc0 0.34.0
 * (the reference's gridder, /root/reference/src/ska_sdp_cip/invert.py:170-183,
 * pinned at /root/reference/poetry.lock:421-422) is not importable on the GPU
 * box, so the baseline is this restatement of ducc0's published CPU design
 * (SURVEY.md 3.4 step 3): visibilities bucketed by 32 x 32 grid tile of their
 * footprint origin, each thread grids a tile into a small private
 * (T + W - 1)^2 buffer and adds it to the shared grid; tiles run in four
 * colour phases (tile x, y parity) so the buffers of one phase never overlap
 * and no locks or atomics are needed. Same kernel (es_kernels.h pieces, even /
 * odd Horner), same placement and periodic wrap as oracle/cip_oracle.c, fp64
 * accumulation; complex64 visibilities and float32 weights are read as given
 * (no widening copy). Not the parity oracle (contraction allowed, -O3): the
 * tests hold it to the oracle at 1e-12 of sum |w V| (tests/test_oracle_golden.py).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "es_kernels.h"

#define SPEED_OF_LIGHT 299792458.0
#define TILE 32

static const double b4[2][CIP_ES_DEGREE_4 + 1] = CIP_ES_COEFFS_4;
static const double b6[3][CIP_ES_DEGREE_6 + 1] = CIP_ES_COEFFS_6;
static const double b8[4][CIP_ES_DEGREE_8 + 1] = CIP_ES_COEFFS_8;
static const double b10[5][CIP_ES_DEGREE_10 + 1] = CIP_ES_COEFFS_10;
static const double b12[6][CIP_ES_DEGREE_12 + 1] = CIP_ES_COEFFS_12;
static const double b14[7][CIP_ES_DEGREE_14 + 1] = CIP_ES_COEFFS_14;
static const double b16[8][CIP_ES_DEGREE_16 + 1] = CIP_ES_COEFFS_16;

static int kernel_table(int W, int* D, const double** coef) {
  switch (W) {
    case 4: *D = CIP_ES_DEGREE_4; *coef = &b4[0][0]; return 0;
    case 6: *D = CIP_ES_DEGREE_6; *coef = &b6[0][0]; return 0;
    case 8: *D = CIP_ES_DEGREE_8; *coef = &b8[0][0]; return 0;
    case 10: *D = CIP_ES_DEGREE_10; *coef = &b10[0][0]; return 0;
    case 12: *D = CIP_ES_DEGREE_12; *coef = &b12[0][0]; return 0;
    case 14: *D = CIP_ES_DEGREE_14; *coef = &b14[0][0]; return 0;
    case 16: *D = CIP_ES_DEGREE_16; *coef = &b16[0][0]; return 0;
    default: return -1;
  }
}

/* all W kernel values at y: pieces k and W-1-k from the even / odd halves */
static inline void eval_pieces(int W, int D, const double* coef, double y, double* out) {
  const double z = y * y;
  for (int k = 0; k < W / 2; ++k) {
    const double* c = coef + k * (D + 1);
    const int de = (D & 1) ? D - 1 : D, dd = (D & 1) ? D : D - 1;
    double e = c[de], o = c[dd];
    for (int d = de - 2; d >= 0; d -= 2) e = e * z + c[d];
    for (int d = dd - 2; d >= 1; d -= 2) o = o * z + c[d];
    out[k] = e + y * o;
    out[W - 1 - k] = e - y * o;
  }
}

typedef struct {
  int64_t ix0, iy0;
  double yu, yv;
} place_t;

static inline int place(double u, double v, double fx, double su, double sv, int64_t nu, int64_t nv, int hw,
                        place_t* p) {
  const double x = (u * fx) * su + (double)(nu / 2);
  const double y = (v * fx) * sv + (double)(nv / 2);
  if (!isfinite(x) || !isfinite(y)) return 0;
  const double sx = x - (double)hw, sy = y - (double)hw;
  const double fxl = floor(sx), fyl = floor(sy);
  p->yu = 2.0 * (sx - fxl) - 1.0;
  p->yv = 2.0 * (sy - fyl) - 1.0;
  int64_t a = (int64_t)fxl + 1, b = (int64_t)fyl + 1;
  /* one compare-and-add in the common case (no 64-bit division) */
  if (a >= nu) a = (a - nu < nu) ? a - nu : a % nu;
  if (a < 0) a = (a + nu >= 0) ? a + nu : ((a % nu) + nu) % nu;
  if (b >= nv) b = (b - nv < nv) ? b - nv : b % nv;
  if (b < 0) b = (b + nv >= 0) ? b + nv : ((b % nv) + nv) % nv;
  p->ix0 = a;
  p->iy0 = b;
  return 1;
}

/*
 * 2-D gridding of (nrow, nchan) complex64 visibilities with float32 weights
 * (NULL = 1) onto grid (nu * nv complex128, row-major g[x][y], caller-zeroed).
 * Returns the number of non-finite placements skipped, or -1.
 */
int64_t cpu_grid_tiled(const double* uvw, int64_t nrow, const double* freq, int64_t nchan, const float* vis,
                       const float* wgt, int64_t nu, int64_t nv, double px, double py, int W, int nthreads,
                       double* grid) {
  int D;
  const double* coef;
  if (kernel_table(W, &D, &coef) || W > TILE + 1 || nchan > 65535) return -1;
  if (nthreads > 0) omp_set_num_threads(nthreads);
  const int nt = omp_get_max_threads();
  const double su = (double)nu * px, sv = (double)nv * py;
  const int hw = W / 2;
  const int64_t ntx = (nu + TILE - 1) / TILE, nty = (nv + TILE - 1) / TILE, ntiles = ntx * nty;
  double* fx = (double*)malloc(sizeof(double) * nchan);
  for (int64_t c = 0; c < nchan; ++c) fx[c] = freq[c] / SPEED_OF_LIGHT;
  int64_t* cnt = (int64_t*)calloc((size_t)nt * ntiles, sizeof(int64_t));
  int64_t bad = 0;
  /* pass 1: per-thread tile histograms over contiguous row blocks */
#pragma omp parallel reduction(+ : bad)
  {
    const int t = omp_get_thread_num();
    const int64_t r0 = nrow * t / nt, r1 = nrow * (t + 1) / nt;
    int64_t* h = cnt + (size_t)t * ntiles;
    for (int64_t r = r0; r < r1; ++r)
      for (int64_t c = 0; c < nchan; ++c) {
        const int64_t i = r * nchan + c;
        if (wgt && wgt[i] == 0.0f) continue;
        place_t p;
        if (!place(uvw[3 * r], uvw[3 * r + 1], fx[c], su, sv, nu, nv, hw, &p)) {
          ++bad;
          continue;
        }
        ++h[(p.ix0 / TILE) * nty + p.iy0 / TILE];
      }
  }
  /* offsets in (tile, thread) order: each thread's visibilities of a tile stay
   * in row order */
  int64_t* toff = (int64_t*)malloc(sizeof(int64_t) * (ntiles + 1));
  int64_t run = 0;
  for (int64_t k = 0; k < ntiles; ++k) {
    toff[k] = run;
    for (int t = 0; t < nt; ++t) {
      const int64_t n = cnt[(size_t)t * ntiles + k];
      cnt[(size_t)t * ntiles + k] = run;
      run += n;
    }
  }
  toff[ntiles] = run;
  int64_t* bucket = (int64_t*)malloc(sizeof(int64_t) * (run > 0 ? run : 1));
  /* pass 2: bucket the visibility indices */
#pragma omp parallel
  {
    const int t = omp_get_thread_num();
    const int64_t r0 = nrow * t / nt, r1 = nrow * (t + 1) / nt;
    int64_t* o = cnt + (size_t)t * ntiles;
    for (int64_t r = r0; r < r1; ++r)
      for (int64_t c = 0; c < nchan; ++c) {
        const int64_t i = r * nchan + c;
        if (wgt && wgt[i] == 0.0f) continue;
        place_t p;
        if (!place(uvw[3 * r], uvw[3 * r + 1], fx[c], su, sv, nu, nv, hw, &p)) continue;
        bucket[o[(p.ix0 / TILE) * nty + p.iy0 / TILE]++] = (r << 16) | c;  /* nchan <= 65535 */
      }
  }
  /* pass 3: four colour phases of tiles, private sub-grid per tile; with an
   * odd tile count on an axis the last tile's halo wraps onto tile 0 of the
   * same parity, so those edge tiles run in a fifth, serial phase */
  const int P = TILE + W - 1;
  for (int color = 0; color < 5; ++color) {
    const int cx = color & 1, cy = (color >> 1) & 1;
#pragma omp parallel if (color < 4)
    {
      double* sub = (double*)malloc(sizeof(double) * 2 * P * P);
      double ku[16], kv[16];
#pragma omp for schedule(dynamic, 4)
      for (int64_t k = 0; k < ntiles; ++k) {
        const int64_t tx = k / nty, ty = k % nty;
        const int edge = ((ntx & 1) && tx == ntx - 1) || ((nty & 1) && ty == nty - 1);
        if (toff[k + 1] == toff[k]) continue;
        if (color == 4 ? !edge : (edge || (tx & 1) != cx || (ty & 1) != cy)) continue;
        memset(sub, 0, sizeof(double) * 2 * P * P);
        const int64_t X0 = tx * TILE, Y0 = ty * TILE;
        for (int64_t q = toff[k]; q < toff[k + 1]; ++q) {
          const int64_t r = bucket[q] >> 16, c = bucket[q] & 0xffff, i = r * nchan + c;
          place_t p;
          place(uvw[3 * r], uvw[3 * r + 1], fx[c], su, sv, nu, nv, hw, &p);
          const double w = wgt ? (double)wgt[i] : 1.0;
          const double vr = w * (double)vis[2 * i], vi = w * (double)vis[2 * i + 1];
          eval_pieces(W, D, coef, p.yu, ku);
          eval_pieces(W, D, coef, p.yv, kv);
          double* s = sub + 2 * ((p.ix0 - X0) * P + (p.iy0 - Y0));
          for (int a = 0; a < W; ++a) {
            const double ar = ku[a] * vr, ai = ku[a] * vi;
            double* row = s + 2 * a * P;
            for (int b = 0; b < W; ++b) {
              row[2 * b] += ar * kv[b];
              row[2 * b + 1] += ai * kv[b];
            }
          }
        }
        for (int a = 0; a < P; ++a) {
          int64_t gx = X0 + a;
          if (gx >= nu) gx -= nu;
          double* dst = grid + 2 * gx * nv;
          const double* src = sub + 2 * a * P;
          for (int b = 0; b < P; ++b) {
            int64_t gy = Y0 + b;
            if (gy >= nv) gy -= nv;
            dst[2 * gy] += src[2 * b];
            dst[2 * gy + 1] += src[2 * b + 1];
          }
        }
      }
      free(sub);
    }
  }
  free(bucket);
  free(toff);
  free(cnt);
  free(fx);
  return bad;
}
