/*
 * cip.h - C ABI of libcip_hip.so, the MI355X-native invert hot path of
 * ska_sdp_cip (SKA SDP continuum imaging pipeline).
 *
 * Every entry point is `extern "C"`, takes plain pointers and sizes, returns
 * 0 (CIP_OK) on success or a negative CIP_E* code; the message of the last
 * failure on the calling thread is returned by cip_last_error(). The library
 * never frees or retains caller memory. Device pointers are HIP device memory
 * on the current device (torch tensors' data_ptr() in the Python host code).
 *
 * Reference interfaces replaced (see INTEGRATION.md for the bindings):
 *   cip_ms2dirty       <- ducc0.wgridder.ms2dirty as called at
 *                         /root/reference/src/ska_sdp_cip/invert.py:170-183
 *                         (plus the sum of weights of invert.py:184)
 *   cip_choose_params  <- ducc0's internal parameter choice (grid size,
 *                         kernel support, w-planes), SURVEY.md 8(a) a4.1/a4.2
 *   cip_tile_runs      <- create_uvw_tile_mapping_sequential's per-row key and
 *                         run search, uvw_tiling/tiling_plan.py:29-61,150-181
 *   cip_stokes_i       <- StokesIGridderInput.from_measurement_set_reader +
 *                         effective_weights, invert.py:72-116
 *   cip_release_workspace - frees the calling thread's workspace cache on the
 *                         current device (no reference
 *                         counterpart; ducc allocates per call).
 *   cip_profile_*      <- observability of the hot path (the reference's
 *                         dask task stream, task_metrics.py:88-135).
 */
#ifndef CIP_H
#define CIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CIP_OK 0
#define CIP_EINVAL (-1)  /* bad argument (ValueError in Python) */
#define CIP_ERANGE (-2)  /* uv(w) outside the grid (ValueError) */
#define CIP_EHIP (-3)    /* HIP / hipFFT runtime failure (RuntimeError) */
#define CIP_ENOMEM (-4)  /* device allocation failure (MemoryError) */

/* dtype codes for cip_ms2dirty */
#define CIP_C64 1
#define CIP_C128 2
#define CIP_F32 3
#define CIP_F64 4
#define CIP_NONE 0 /* wgt == NULL: all weights 1 */

/* flags of cip_ms2dirty / cip_grid_plane */
#define CIP_WSTACKING 1  /* w-stacking planes (cip_ms2dirty only; else 2-D) */
#define CIP_NORMALISE 8  /* cip_ms2dirty only: dirty_out is divided by the
                          * call's weight sum (the reference's
                          * (1 / total_weight) * image, invert.py:119-149),
                          * fused into the pruned FFT's epilogue in 2-D mode.
                          * sum_wgt_out still receives the raw sum. Not for
                          * partial images that are reduced across ranks. */
#define CIP_PSF 4        /* grid unit visibilities (vis ignored, may be NULL):
                          * the point-spread function with the same weights
                          * (cip_ms2dirty, cip_grid_ms, cip_grid_tiles) */
#define CIP_ASYNC 16     /* cip_ms2dirty only: return once the work is queued on
                          * hip_stream instead of synchronising it (the
                          * planner's two readbacks still synchronise mid-call).
                          * dirty_out / sum_wgt_out are valid when the stream
                          * reaches this point. Ignored while profiling is on. */
#define CIP_PIPELINE 32  /* with CIP_ASYNC (cip_ms2dirty): the caller promises
                          * that uvw, freq, vis and wgt were complete before the
                          * previous CIP_ASYNC call of this thread returned and
                          * stay unchanged (resident inputs, e.g. re-imaging the
                          * same chunk): the planner then runs on the
                          * workspace's own stream beside the previous calls'
                          * scatter and FFT instead of after everything queued
                          * on hip_stream. Without it, CIP_ASYNC work starts in
                          * hip_stream order. Outputs are in stream order
                          * either way. */
#define CIP_REUSE_PLAN 64 /* cip_ms2dirty only, not with CIP_PIPELINE: the caller
                          * promises that uvw, freq and the row layout are those
                          * of this thread's previous planned call (e.g. the
                          * Stokes parameters and PSF of one facet): when the
                          * previous call's geometry (nrow, nchan, npix, pixel
                          * sizes, epsilon / support, w-stacking, accumulation
                          * class) matches, its tile plan (bucket, chunks,
                          * bank-class order, dirty-tile masks) is used again
                          * and only the weight sum and max |w V| are reduced;
                          * otherwise the call plans as usual. Images are
                          * identical to a planned call's. */
#define CIP_GRID_ZEROED 128 /* cip_grid_ms, cip_grid_ms_stokes_i, cip_grid_tiles:
                          * the caller promises the planes are all zero (the
                          * first chunk onto cleared planes, or planes kept
                          * clean by cip_strip_rows): on planes of >= 16384^2
                          * cells the scatter then stores the cells only one
                          * of its work units writes instead of adding them
                          * with atomics (same values). The stores are 16-byte
                          * cells: planes that are not 16-byte aligned ignore
                          * the flag (atomic adds, same result). */
#define CIP_ACC_SINGLE 2 /* complex64 only: single-precision accumulation
                          * class, the reference's ducc0 float gridding (re/im
                          * packed in one 64-bit fixed-point LDS cell, W^2
                          * instead of 2 W^2 atomics per visibility). Without
                          * it every input accumulates in 64-bit fixed point
                          * (2^-46 of max|w V|, fp64 class). */

typedef struct cip_gridder_params {
  int64_t nu, nv;      /* oversampled grid size (cells), even, 2/3/5/7-smooth */
  int32_t support;     /* kernel support W: even 4..16, or 24/32/48/64 (2-D;
                          w-stacking up to 48) */
  int32_t degree;      /* polynomial degree of each kernel piece (W + 3;
                          15 for the large supports) */
  double beta;         /* ES shape parameter (2.3 W) */
  double sigma;        /* oversampling factor (2.0) */
  int32_t do_wstacking;/* 1: w-stacking planes; 0: 2-D (w ignored) */
  int32_t tile;        /* grid tile edge T (cells) used by the scatter */
  int64_t nplanes;     /* number of w planes (1 in 2-D mode) */
  double w0, dw;       /* plane p sits at w = w0 + p dw (wavelengths) */
  double nmin;         /* min over the field of n - 1 (<= 0) */
} cip_gridder_params;

/* Grid/kernel/w-plane parameters for an image of npix_x x npix_y pixels of
 * pixsize (radians, sin-projected). support <= 0 selects W from epsilon
 * (4..16); an explicit support may also be 24, 32, 48 or 64 (the
 * wave-per-visibility scatter; fp64 class only; w-stacking up to 48).
 * wmin/wmax: range of w in wavelengths (only used when do_wstacking). */
int cip_choose_params(int64_t npix_x, int64_t npix_y, double pixsize_x,
                      double pixsize_y, double epsilon, int support,
                      int do_wstacking, double wmin, double wmax,
                      cip_gridder_params* out);

/* Dirty image (drop-in for ms2dirty): uvw (nrow,3) f64 metres, freq (nchan)
 * f64 Hz, vis (nrow,nchan) complex64/complex128, wgt (nrow,nchan) f32/f64 or
 * NULL. All pointers are DEVICE pointers. dirty_out: device (npix_x,npix_y)
 * f64, row-major, axis 0 <-> l <-> u. sum_wgt_out: device f64 scalar, the sum
 * of wgt (the reference's total_weight, invert.py:184), may be NULL.
 * Runs on hip_stream (NULL = default stream) and returns when the result is
 * complete on that stream (synchronous). params_out may be NULL. */
int cip_ms2dirty(const double* uvw, int64_t nrow, const double* freq,
                 int64_t nchan, const void* vis, int vis_dtype,
                 const void* wgt, int wgt_dtype, int64_t npix_x,
                 int64_t npix_y, double pixsize_x, double pixsize_y,
                 double epsilon, int support, int flags,
                 void* hip_stream, double* dirty_out, double* sum_wgt_out,
                 cip_gridder_params* params_out);

/* cip_ms2dirty restricted to w planes [plane_begin, plane_end) of the
 * w-stacking stack (CIP_WSTACKING required): the multi-GPU split of ONE
 * w-stacking image by plane groups (SURVEY.md 8(e) option 2; ska_sdp_cip_amd
 * wplanes.py). The planner still reads every visibility (the weight sum and
 * the stack's parameters are those of the whole call) but keeps only those
 * feeding a plane of the range; the scatter and the FFT run for those planes
 * only. dirty_out = that range's share of the image, with the final w and grid
 * correction (and CIP_NORMALISE) applied - all linear, so the shares of a
 * partition of [0, nplanes) sum to cip_ms2dirty's image. An empty range gives
 * zeros; plane_end > nplanes is CIP_EINVAL. No reference counterpart (the
 * reference's dask tasks split rows, invert.py:248-270). */
int cip_ms2dirty_wplanes(const double* uvw, int64_t nrow, const double* freq,
                         int64_t nchan, const void* vis, int vis_dtype,
                         const void* wgt, int wgt_dtype, int64_t npix_x,
                         int64_t npix_y, double pixsize_x, double pixsize_y,
                         double epsilon, int support, int flags,
                         int64_t plane_begin, int64_t plane_end,
                         void* hip_stream, double* dirty_out,
                         double* sum_wgt_out, cip_gridder_params* params_out);

/* cip_ms2dirty on the raw linear-feed columns (the reference's
 * StokesIGridderInput + effective weights, invert.py:78-116, fused into the
 * gridder): vis4 (nrow, nchan, 4) complex64 correlations XX, XY, YX, YY,
 * flags4 (nrow, nchan, 4) uint8 (NULL: none flagged; 4-byte aligned), wgt4
 * (nrow, nchan, 4) float32, all device pointers. The planner and the scatter
 * form Stokes I = 0.5 (XX + YY) and the weight !(F_XX | F_YY) * 4 /
 * (1 / w_XX + 1 / w_YY) in float32 as they load each visibility: the image,
 * weight sum and parameters equal cip_stokes_i followed by cip_ms2dirty on its
 * (vis_i, eff_w) bit for bit, without the 12 B/visibility intermediate
 * columns. Other arguments and flags as cip_ms2dirty (CIP_PSF: unit
 * visibilities with these weights; CIP_ACC_SINGLE allowed). Replaces
 * invert.py:170-183's ms2dirty call on StokesIGridderInput's outputs. */
int cip_ms2dirty_stokes_i(const double* uvw, int64_t nrow, const double* freq,
                          int64_t nchan, const void* vis4, const uint8_t* flags4,
                          const float* wgt4, int64_t npix_x, int64_t npix_y,
                          double pixsize_x, double pixsize_y, double epsilon,
                          int support, int flags, void* hip_stream,
                          double* dirty_out, double* sum_wgt_out,
                          cip_gridder_params* params_out);

/* Uniform-grid ("grid only") variant used by the benchmark and the parity
 * tests: fills grid_out (device, nu x nv complex128, row-major) for w-plane
 * `plane` (0 in 2-D mode) with the gridded visibilities, using params from
 * cip_choose_params. Zeroes grid_out first. */
int cip_grid_plane(const double* uvw, int64_t nrow, const double* freq,
                   int64_t nchan, const void* vis, int vis_dtype,
                   const void* wgt, int wgt_dtype,
                   const cip_gridder_params* params, double pixsize_x,
                   double pixsize_y, int64_t plane, int flags,
                   void* hip_stream, double* grid_out);

/* Accumulating gridder (chunked / streamed inputs): grids
 * holds params->nplanes planes of nu x nv complex128 (DEVICE, zeroed by the
 * caller before the first chunk) in the layout cip_grid_layout reports for
 * the target image (1: each plane stored transposed, gT[y][x]; 0: g[x][y]).
 * Every call adds its visibilities onto the planes and its weight sum onto
 * *sum_wgt (device f64, may be NULL); params must be the same for every chunk
 * (cip_choose_params over the whole data set's w range). */
int cip_grid_layout(const cip_gridder_params* params, int64_t npix_x,
                    int64_t npix_y);

/* w planes one w-stacking scatter pass grids together (the plane group: a
 * visibility is placed once per group; 1 in 2-D mode and for supports > 16).
 * packed != 0: the packed single class (CIP_ACC_SINGLE). Host-only. A w-plane
 * split (cip_ms2dirty_wplanes ranges) cut on multiples of it runs no group
 * pass twice. Replaces no reference call (ducc0 internal). */
int cip_plane_group(const cip_gridder_params* params, int packed);

/* Dense chunk: MS rows, as cip_ms2dirty (uvw (nrow,3), vis/wgt (nrow,nchan)). */
int cip_grid_ms(const double* uvw, int64_t nrow, const double* freq,
                int64_t nchan, const void* vis, int vis_dtype,
                const void* wgt, int wgt_dtype,
                const cip_gridder_params* params, double pixsize_x,
                double pixsize_y, int64_t npix_x, int64_t npix_y, int flags,
                void* hip_stream, double* grids, double* sum_wgt);

/* cip_grid_ms on the raw linear-feed columns (Stokes I formed on load, as
 * cip_ms2dirty_stokes_i): vis4 / flags4 / wgt4 (nrow, nchan, 4) complex64 /
 * uint8 (NULL: none flagged; 4-byte aligned) / float32 device pointers. */
int cip_grid_ms_stokes_i(const double* uvw, int64_t nrow, const double* freq,
                         int64_t nchan, const void* vis4, const uint8_t* flags4,
                         const float* wgt4, const cip_gridder_params* params,
                         double pixsize_x, double pixsize_y, int64_t npix_x,
                         int64_t npix_y, int flags, void* hip_stream,
                         double* grids, double* sum_wgt);

/* Tile-sorted chunk (the uvw_tiling Tile layout, reference
 * uvw_tiling/tile.py:14-124, the reorder output): nslices row slices with
 * uvw (nslices,3) f64 metres and channel ranges [chan_start, chan_stop)
 * (int32); vis (nvis) and wgt (nvis, or NULL) hold the slices' visibilities
 * concatenated in slice order (nvis = sum of the range lengths). */
int cip_grid_tiles(const double* slice_uvw, const int32_t* chan_start,
                   const int32_t* chan_stop, int64_t nslices,
                   const double* freq, int64_t nchan, const void* vis,
                   int64_t nvis, int vis_dtype, const void* wgt, int wgt_dtype,
                   const cip_gridder_params* params, double pixsize_x,
                   double pixsize_y, int64_t npix_x, int64_t npix_y, int flags,
                   void* hip_stream, double* grids, double* sum_wgt);

/* cip_grid_tiles onto ONE uv strip's buffer instead of the whole grid (the
 * strong-scaling ranks of DESIGN.md 7 hold only their strip + halo rows): the
 * grid must be in the pruned-FFT layout (cip_grid_layout == 1, stored
 * gT[y][x]); `strip` holds, per w plane (nplanes of them, 1 in 2-D), nrows
 * rows of nu complex128 cells, buffer row k = grid row (row0 + k) mod nv
 * (plane p at strip + 2 nu nrows p). Every visibility's footprint must fall inside
 * those rows (a strip's slices from its footprint-origin rows [y0, y1) need
 * nrows = y1 - y0 + W - 1): a cell outside is dropped and the call returns
 * CIP_ERANGE. Flags as cip_grid_tiles (CIP_GRID_ZEROED: buffer all zero).
 * No reference counterpart (the reference grids whole images per task). */
int cip_grid_tiles_strip(const double* slice_uvw, const int32_t* chan_start,
                         const int32_t* chan_stop, int64_t nslices,
                         const double* freq, int64_t nchan, const void* vis,
                         int64_t nvis, int vis_dtype, const void* wgt,
                         int wgt_dtype, const cip_gridder_params* params,
                         double pixsize_x, double pixsize_y, int64_t npix_x,
                         int64_t npix_y, int64_t row0, int64_t nrows, int flags,
                         void* hip_stream, double* strip, double* sum_wgt);

/* cip_grid_tiles_strip that also writes the strip's dirty-tile bits for its
 * masked pass A (cip_strip_rows_masked / _packed): tile_bits (device, per w
 * plane (nv / 32) x (nu / 1024) uint32 words, the layout those calls read) =
 * the tiles this call's scatter flush writes a cell of (exact: reported by
 * each work unit's flush) plus every tile of the tile rows holding grid rows
 * row0 .. row0 + W - 2 (the previous rank's halo is added there). Replaces
 * strips.py's torch restatement of the mask (round 5) - every call computes
 * its own. */
int cip_grid_tiles_strip_mask(const double* slice_uvw, const int32_t* chan_start,
                              const int32_t* chan_stop, int64_t nslices,
                              const double* freq, int64_t nchan, const void* vis,
                              int64_t nvis, int vis_dtype, const void* wgt,
                              int wgt_dtype, const cip_gridder_params* params,
                              double pixsize_x, double pixsize_y, int64_t npix_x,
                              int64_t npix_y, int64_t row0, int64_t nrows, int flags,
                              void* hip_stream, double* strip, double* sum_wgt,
                              uint32_t* tile_bits);

/* The uv-strip split of the strong-scaling path on the device (round 6;
 * the reference's offline bucket step, uvw_tiling/tiling_plan.py:29-61 and
 * reorder.py:19-111, cut by footprint-origin grid row). Power-of-two grids
 * of 32 .. 16384 rows; uvw (nrow, 3), freq (nchan) DEVICE pointers; every
 * visibility is placed with the gridder's own fp64 arithmetic.
 * cip_strip_histogram: hist (device int64, 2 nv) = per grid row the
 *   visibilities whose footprint origin lies in it, then the row slices
 *   starting there (a slice starts at channel 0 and wherever the origin's
 *   32-cell tile changes) - the strip cost model's inputs. Stream-ordered.
 * cip_strip_split: the strip of origin rows [y0, y1) in the Tile layout
 *   (uvw_tiling/tile.py:14-124): maximal channel runs per MS row, slices in
 *   (row, channel) order. Two-phase: slice_uvw == NULL -> counts[0] = slices,
 *   counts[1] = visibilities (host, one stream wait); then with device
 *   buffers of those sizes: slice_uvw (n, 3) f64, chan_start / chan_stop (n)
 *   int32, slice_row (n) int64 (the MS row), and, when vis != NULL (dense
 *   (nrow, nchan) complex64 / complex128), vis_out (nvis) and - wgt != NULL
 *   (float32 / float64) - wgt_out gathered into slice order. */
int cip_strip_histogram(const double* uvw, int64_t nrow, const double* freq,
                        int64_t nchan, const cip_gridder_params* params,
                        double pixsize_x, double pixsize_y, void* hip_stream,
                        int64_t* hist);
int cip_strip_split(const double* uvw, int64_t nrow, const double* freq,
                    int64_t nchan, const void* vis, int vis_dtype, const void* wgt,
                    int wgt_dtype, const cip_gridder_params* params,
                    double pixsize_y, int64_t y0, int64_t y1, void* hip_stream,
                    int64_t* counts, double* slice_uvw, int32_t* chan_start,
                    int32_t* chan_stop, int64_t* slice_row, void* vis_out,
                    void* wgt_out);

/* The accumulated planes -> dirty image (device (npix_x,npix_y) f64, not
 * normalised): FFT, w-screens and grid correction as in cip_ms2dirty. The
 * planes are consumed (used as FFT scratch). */
int cip_grid_to_dirty(double* grids, const cip_gridder_params* params,
                      int64_t npix_x, int64_t npix_y, double pixsize_x,
                      double pixsize_y, void* hip_stream, double* dirty_out);

/* Strips of the dirty-image FFT: the multi-GPU strong-scaling split of one
 * grid (SURVEY.md 8(e) option 1, the north star's UVW-tile
 * shards with a partial-grid halo exchange before the FFT). Rank r owns grid
 * rows [y0, y1) of the transposed 2-D grid (cip_grid_layout == 1, power-of-
 * two grids) and image rows [i0, i1) (multiples of 4).
 * cip_strip_rows: pass A over rows [y0, y1) of `grid` (nu x nv complex128 as
 * gT[y][x]) -> H (device, (npix_x / 4) blocks x (y1 - y0) rows x 4
 * complex128: row y of block b at ((b (y1 - y0)) + y - y0) 4); the rows read
 * are zeroed (the grid is left clean for the next call).
 * cip_strip_cols: pass B for image rows [i0, i1) from H holding blocks
 * [i0 / 4, i1 / 4), nv rows each (the strips' pass-A outputs exchanged block
 * by block), written to dirty_rows ((i1 - i0) x npix_y f64) with the crop and
 * grid correction, divided by *norm (device f64) when norm != NULL. Both
 * synchronous on hip_stream. */
int cip_strip_rows(double* grid, const cip_gridder_params* params,
                   int64_t npix_x, int64_t npix_y, int64_t y0, int64_t y1,
                   void* hip_stream, double* H);
int cip_strip_cols(const double* H, const cip_gridder_params* params,
                   int64_t npix_x, int64_t npix_y, int64_t i0, int64_t i1,
                   const double* norm, void* hip_stream, double* dirty_rows);
/* cip_strip_rows that reads and zeroes only the dirty tiles' cells: tile_bits
 * (device) holds the dirty-tile bits of the whole grid's plane, (nv / 32)
 * rows of (nu / 1024) uint32 words, bit tx % 32 of word [ty][tx / 32] for
 * tile (tx, ty) of 32 x 32 cells; buffer row y is grid row (row0 + y) mod nv.
 * Every non-zero cell of rows [y0, y1) must lie in a marked tile (the rest is
 * neither read nor zeroed). */
int cip_strip_rows_masked(double* grid, const cip_gridder_params* params,
                          int64_t npix_x, int64_t npix_y, int64_t y0,
                          int64_t y1, int64_t row0, const uint32_t* tile_bits,
                          void* hip_stream, double* H);
/* cip_strip_rows_masked's packed form (round 5, the sparse all-to-all's send
 * buffer written by pass A itself): buffer row y goes to H row
 * row_slot[y - y0] of an H with nlive rows per 4-column block ((npix_x / 4,
 * nlive, 4) complex128); rows with row_slot < 0 must hold no dirty tile and
 * are skipped (device int64, y1 - y0 entries). */
int cip_strip_rows_packed(double* grid, const cip_gridder_params* params,
                          int64_t npix_x, int64_t npix_y, int64_t y0,
                          int64_t y1, int64_t row0, const uint32_t* tile_bits,
                          const int64_t* row_slot, int64_t nlive,
                          void* hip_stream, double* H);
/* The strips' sparse all-to-all of pass-A rows (round 5). A record is row y
 * of one 4-column block of H ((nb, rows, 4) complex elements of elem_bytes =
 * 16 (complex128) or 8 (complex64)). cip_strip_pack_rows: out (nb, nlive, 4)
 * <- the rows y of H (nb, h, 4) with slot[y] >= 0, at position slot[y]
 * (device int64, h entries). cip_strip_unpack_rows: H (nb, nv, 4) <- row y
 * from recv record rec[y] + b * stride[y] for block b, zeros where
 * rec[y] < 0 (device int64, nv entries each). Stream-ordered on hip_stream
 * (no host wait). Replace: strips.py's index_select / advanced-index copies. */
int cip_strip_pack_rows(const void* H, int64_t nb, int64_t h, int elem_bytes,
                        const int64_t* slot, int64_t nlive, void* hip_stream,
                        void* out);
int cip_strip_unpack_rows(const void* recv, int64_t nb, int64_t nv, int elem_bytes,
                          const int64_t* rec, const int64_t* stride,
                          void* hip_stream, void* H);
/* w-stacking strips (the reference's own gridding mode split by uv strips):
 * cip_strip_rows runs per w plane (grid = the plane's rows of the strip
 * buffer); cip_strip_cols_wplane is pass B for plane `plane` of image rows
 * [i0, i1) with the w screen, adding into acc_rows ((i1 - i0) x npix_y f64;
 * first != 0 overwrites: the rank's first plane); after the last plane
 * cip_strip_wfinal applies the final w correction and grid correction to
 * those rows, divided by *norm (device f64) when norm != NULL. Synchronous
 * on hip_stream. */
int cip_strip_cols_wplane(const double* H, const cip_gridder_params* params,
                          int64_t npix_x, int64_t npix_y, double pixsize_x,
                          double pixsize_y, int64_t i0, int64_t i1,
                          int64_t plane, int first, void* hip_stream,
                          double* acc_rows);
int cip_strip_wfinal(double* acc_rows, const cip_gridder_params* params,
                     int64_t npix_x, int64_t npix_y, double pixsize_x,
                     double pixsize_y, int64_t i0, int64_t i1,
                     const double* norm, void* hip_stream);

/* Reference-exact UVW tile keys and constant-key channel runs (one run per
 * maximal range of channels with equal (iu, iv, iw) in a row), rows in
 * order, runs in channel order: key = floor(f/c * (uvw / tile) + 0.5) in
 * fp64 without contraction. uvw/freq are DEVICE pointers. Two-phase: call
 * with runs_* == NULL to get *n_runs, then with buffers of that size (device
 * pointers): run_key (n_runs,3) int64, run_row (n_runs) int64 (row_offset
 * added), run_c0/run_c1 (n_runs) int32. */
int cip_tile_runs(const double* uvw, int64_t nrow, const double* freq,
                  int64_t nchan, const double* tile_size3, int64_t row_offset,
                  void* hip_stream, int64_t* n_runs, int64_t* run_key,
                  int64_t* run_row, int32_t* run_c0, int32_t* run_c1);

/* Stokes-I gridder input from raw (nrow,nchan,4) columns (device pointers):
 * vis_i = 0.5 (V0 + V3) complex64, flag_i = F0 | F3, wgt_i = 4/(1/w0 + 1/w3)
 * (0 when either is 0), eff_w = !flag_i * wgt_i (float32). Any output may be
 * NULL. */
int cip_stokes_i(const void* vis4, const uint8_t* flags4, const float* wgt4,
                 int64_t n, void* hip_stream, void* vis_i, uint8_t* flag_i,
                 float* wgt_i, float* eff_w);

/* Any Stokes parameter from linear feeds (pols XX, XY, YX, YY): I as
 * cip_stokes_i; Q = 0.5 (XX - YY) with I's flags and weights; U =
 * 0.5 (XY + YX), V = -0.5 i (XY - YX) with flags XY | YX and weights
 * 4/(1/w_XY + 1/w_YX). Beyond the reference (Stokes I only), SURVEY.md 8(f)4. */
#define CIP_STOKES_I 0
#define CIP_STOKES_Q 1
#define CIP_STOKES_U 2
#define CIP_STOKES_V 3
int cip_stokes(const void* vis4, const uint8_t* flags4, const float* wgt4,
               int64_t n, int stokes, void* hip_stream, void* vis_out,
               uint8_t* flag_out, float* wgt_out, float* eff_w);

/* Facet: rephase the data to the facet centre
 * (l0, m0) of the original tangent plane and rotate the baselines into the
 * facet's frame (minimal rotation taking the phase centre to the facet
 * centre), so that cip_ms2dirty of (uvw_out, vis_out) is the dirty image on
 * the facet's own tangent plane, centred on (l0, m0). uvw_out (nrow,3) f64;
 * vis_out (nrow,nchan) of vis_dtype, may equal vis (in place) or be NULL
 * (uvw only, e.g. for a PSF). DEVICE pointers. */
int cip_facet_rephase(const double* uvw, int64_t nrow, const double* freq,
                      int64_t nchan, const void* vis, int vis_dtype, double l0,
                      double m0, void* hip_stream, double* uvw_out,
                      void* vis_out);

/* RCCL reduction (sum, fp64) of nelem values held by each of ndev devices
 * in ONE process: grids[k] is a device pointer on
 * devices[k]; root >= 0 sums onto grids[root] (ncclReduce), root < 0 sums
 * into every grid (ncclAllReduce). hip_streams: one per device, or NULL.
 * Returns when done. The communicator clique is cached per device list
 * (cip_release_collectives frees them). */
int cip_allreduce_grid(void* const* grids, const int* devices, int ndev,
                       int64_t nelem, int root, void* const* hip_streams);
int cip_release_collectives(void);

/* Last error message of the calling thread ("" if none). */
const char* cip_last_error(void);

/* Free the calling thread's workspace cached for the current device: its
 * buffers, FFT plans, pinned staging, side stream and events (workspaces are
 * per device and host thread: two threads may each run calls on their own
 * stream, on one GPU, without sharing buffers). The workspaces of a worker
 * thread are also freed automatically when that thread exits; those of the
 * thread that loaded the library live until the process ends. */
int cip_release_workspace(void);

/* Per-phase timing of cip_ms2dirty / cip_grid_plane on the calling thread
 * (no reference counterpart; the reference records dask task streams,
 * task_metrics.py:88-135). When enabled, hipEvents are recorded on the call's
 * stream around each phase; cip_profile_last fills
 *   ms[0..5]     = prep, plan, scatter, fft, correct, total  (milliseconds)
 *   counts[0..5] = visibilities, runs (row slices), chunks, planes, scatter launches,
 *                  reserved (0)
 * of the most recent call. */
#define CIP_PROFILE_PHASES 6
#define CIP_PROFILE_COUNTS 6
int cip_profile_enable(int on);
int cip_profile_last(double* ms, int64_t* counts);

/* Library build identification (architecture, version). */
const char* cip_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* CIP_H */
