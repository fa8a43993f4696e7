// cip_internal.h - host-side launch wrappers shared between the translation
// units of libcip_hip.so. Not part of the C ABI (include/cip.h is).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "cip.h"
#include "cip_common.h"

namespace cip {

// error helper: sets the thread-local message, returns code
int set_error(int code, const std::string& msg);
#define CIP_HIP_CHECK(expr)                                                     \
  do {                                                                          \
    hipError_t e_ = (expr);                                                     \
    if (e_ != hipSuccess)                                                       \
      return ::cip::set_error(CIP_EHIP, std::string(#expr) + ": " +            \
                                            hipGetErrorString(e_));            \
  } while (0)

// ---- scan (cip_plan.hip) -------------------------------------------------
// In-place exclusive scan of n int64 values; tmp must hold scan_tmp_elems(n).
int64_t scan_tmp_elems(int64_t n);
// run_goff[k] = sum of the lengths of runs [0, k), k in [0, nruns] (fused
// run-length + exclusive scan)
// run lengths from the run records, or (run_keys, RowMap::pk_runs) from the
// sorted keys' bits 26-31
hipError_t scan_run_offsets(const uint64_t* runs, int64_t nruns, int64_t* run_goff, int64_t* tmp, hipStream_t s,
                            const uint32_t* run_keys = nullptr);
hipError_t exclusive_scan_i64(int64_t* data, int64_t n, int64_t* tmp, hipStream_t s);

// ---- gridder planner (cip_plan.hip) ----------------------------------------
// err (may be NULL): bit 2 set when a frequency is not finite and positive
hipError_t launch_freq_scale(const double* freq, int64_t nchan, double* fx, unsigned* err, hipStream_t s);
// per-row w range over channels (only f min/max matter): out[0]=min, out[1]=max
hipError_t launch_w_range(const double* uvw, int64_t nrow, double fxmin, double fxmax, double* partial,
                          int nblocks, hipStream_t s);
// place pass: the runs of place block b (4096 visibilities) parked with their
// tile keys at slots [4096 b, 4096 b + blk_cnt[b]), per-block {sum w, max |w V|}
// partials (2 * plan_place_blocks) and the radix pass-0 histogram of the parked
// keys (hist0[d * nblocks + b], 256 * nblocks + 1 entries, last one zeroed);
// vis_class (optional, nvis bytes): each visibility's LDS bank class.
// err_flag: bit 0 non-finite uvw / w off the stack, bit 1 non-finite vis or weight.
int plan_place_blocks(int64_t nvis);
// the place pass's reduction alone (sum of weights, max |w V|, non-finite
// check -> partial, err_flag bit 2), in its order: for calls reusing a plan
hipError_t launch_prep_reduce(const RowMap& m, const void* vis, int vis_dtype, const void* wgt, int wgt_dtype,
                              const GridGeometry& g, unsigned* err_flag, double* partial, hipStream_t s);
hipError_t launch_plan_place(const double* uvw, const double* fx, const RowMap& m,
                             const void* vis, int vis_dtype, const void* wgt, int wgt_dtype, const GridGeometry& g,
                             unsigned* err_flag, uint8_t* vis_class, int64_t* blk_cnt, uint32_t* park_key,
                             uint64_t* park_run, double* partial, int64_t* hist0, hipStream_t s);
// ragged rows: out[r] = chan_stop[r] - chan_start[r] (out[nrow] = 0; err bit
// set for a range outside [0, nchan)); after the exclusive scan (off[r] = row
// r's first visibility), launch_ragged_expand writes delta[r] = off[r] -
// chan_start[r] and seg_row[k] = the row of visibility 64 k.
hipError_t launch_ragged_lengths(const int32_t* c0, const int32_t* c1, int64_t nrow, int64_t nchan, int64_t* out,
                                 unsigned* err, hipStream_t s);
hipError_t launch_ragged_expand(const int64_t* off, const int32_t* c0, int64_t nrow, int64_t* delta,
                                uint32_t* seg_row, hipStream_t s);
// one stable LSD radix sort pass on digit (key >> shift) & 255 over nblocks
// blocks of 4096 slots: dense (blk_cnt NULL, n items) or the place pass's
// parked runs (blk_cnt). hist: 256 * nblocks + 1 entries, exclusive-scanned
// between the two calls (its last entry then holds the item count).
int64_t radix_blocks(int64_t n);
// G: sub-blocks (of <= 4096 items) per workgroup; hist is digit-major per
// group of G sub-blocks (see cip_plan.hip)
hipError_t launch_radix_hist(const uint32_t* keys, int64_t n, const int64_t* blk_cnt, int64_t nsub, int G, int shift,
                             int64_t* hist, hipStream_t s);
hipError_t launch_radix_group_hist(const int64_t* hist0, int64_t nsub, int G, int64_t* hg, hipStream_t s);
hipError_t launch_radix_scatter(const uint32_t* keys, const uint64_t* vals, int64_t n, const int64_t* blk_cnt,
                                int64_t nsub, int G, int shift, const int64_t* hist, uint32_t* keys_out,
                                uint64_t* vals_out, hipStream_t s);
hipError_t launch_tile_offsets(const uint32_t* keys, int64_t nruns, int64_t ntiles, int64_t* tile_run_off,
                               hipStream_t s, uint32_t kmask = 0xffffffffu);
// per grid plane (nplanes x ntx x nty bytes); bits (optional, ntx % 32 ==
// 0): the masks bit-packed, ntx / 32 words per tile row, ntx nty / 32 per plane
hipError_t launch_dirty_mask(const int64_t* tile_vis, int64_t ntx, int64_t nty, int64_t ntw, int support,
                             int64_t nplanes, uint8_t* mask, uint32_t* bits, hipStream_t s);
hipError_t launch_tile_vis(const int64_t* run_goff, const int64_t* tile_run_off, int64_t ntiles,
                           int64_t* tile_vis_off, int64_t* tile_vis, hipStream_t s);
hipError_t launch_run_lengths(const uint64_t* runs, int64_t nruns, int64_t* out, hipStream_t s);
// full_first: full chunks of every tile before the partial ones (chunk_off
// then has 2 ntiles + 1 entries), else per tile in tile order (ntiles + 1)
hipError_t launch_chunk_counts(const int64_t* tile_vis, int64_t ntiles, int64_t chunk_vis, int full_first,
                               int64_t* out, hipStream_t s);
hipError_t launch_chunk_emit(const int64_t* tile_vis_off, const int64_t* tile_vis, const int64_t* chunk_off,
                             const int64_t* run_goff, const int64_t* tile_run_off, int64_t ntiles,
                             int64_t chunk_vis, int full_first, int64_t nchunks, Chunk* chunks, hipStream_t s);
// w-stacking: per (plane, uv tile) work units over the tile's merged layer range
// per plane group (planes [q G, q G + G), ngroups groups): its work units per uv tile
hipError_t launch_plane_chunk_counts(const int64_t* tile_vis_off, int64_t ntxy, int64_t ntw, int64_t ngroups,
                                     int group, int support, int64_t cv, int64_t* out, hipStream_t s);
hipError_t launch_plane_chunk_emit(const int64_t* tile_vis_off, const int64_t* chunk_off, const int64_t* run_goff,
                                   const int64_t* tile_run_off, int64_t ntxy, int64_t ntw, int64_t ngroups,
                                   int group, int support, int64_t cv, int64_t nchunks, Chunk* chunks, hipStream_t s);
hipError_t launch_gather_i64(const int64_t* src, int64_t stride, int64_t count, int64_t* dst,
                             hipStream_t s);

// ---- gridding (cip_grid.hip) -----------------------------------------------
// out2 = {sum, max} of the place pass's 2 * nblocks partials
hipError_t launch_add_scalar(const double* src, double* dst, hipStream_t s);
hipError_t launch_prep_final(const double* partial, int nblocks, double* out2, hipStream_t s);
// packed: single-precision class (re/im packed in one 64-bit integer), complex64
// only. perm: bank-class ordered stream from launch_order, or NULL (visibilities
// located through the tile's row slices in tile order).
// one kernel support W (instantiated in cip_scatter_w.hip for W = 4, 6, ..., 16)
template <int W>
hipError_t launch_scatter_w(int vis_dtype, int wgt_dtype, bool pack, int group, unsigned lds_extra,
                            int store_private, dim3 gd, hipStream_t s,
                            const double* uvw,
                            const double* fx, const void* vis, const void* wgt, const RowMap& m,
                            const uint64_t* runs, const int64_t* run_goff, const int64_t* tile_run_off,
                            const void* perm, const Chunk* chunks, int64_t cb, const GridGeometry& g,
                            int64_t plane, double fs, double* grid);
// the large supports W = 24, 32, 48, 64 (cip_scatter_large.hip, wave per
// visibility; one translation unit per W)
template <int W>
hipError_t launch_scatter_large_w(int vis_dtype, int wgt_dtype, dim3 gd, hipStream_t s, const double* uvw,
                                  const double* fx, const void* vis, const void* wgt, const RowMap& m,
                                  const uint64_t* runs, const int64_t* run_goff, const void* perm,
                                  const Chunk* chunks, int64_t cb, const GridGeometry& g, int64_t plane, double fs,
                                  double* grid);
// group: w planes per work unit (w-stacking plane groups, 1 or 2; grid = the
// group's planes, 2 nu nv doubles apart)
// share_cus: cap the scatter at three 256-thread blocks per CU (extra dynamic
// LDS) so kernels of another stream - the next pipelined call's planner - run
// beside it
// store_private: the grid planes are zero (a cip_ms2dirty plane, not an
// accumulating one), so a tile's only work unit stores its private cells
hipError_t launch_scatter(int support, int vis_dtype, int wgt_dtype, bool packed, int group, bool share_cus,
                          bool store_private,
                          const double* uvw,
                          const double* fx, const void* vis, const void* wgt, const RowMap& m, const uint64_t* runs,
                          const int64_t* run_goff, const int64_t* tile_run_off, const void* perm,
                          const Chunk* chunks, int64_t chunk_begin, int64_t nchunks, const GridGeometry& g,
                          int64_t plane, double fixed_scale, double* grid, hipStream_t s);
// perm (nvis 32-bit records, nvis < 2^32): the tile-order visibilities as
// row * nchan + channel, bank-class sorted within each window (the tiles split
// into <= kOrderWindow pieces by chunk_emit with cv = kOrderWindow)
// vis_class: the place pass's class byte per visibility (required)
// phase_support: the support W of the lane scatter that reads perm, which then
// carries row phases (bit 31 of dense entries, cip_grid.hip order_kernel);
// 0: no phases
// (phases only where order_phases_ok; the scatter then needs RowMap::row_phase)
hipError_t launch_order(const uint8_t* vis_class, const RowMap& m, const uint64_t* runs, const int64_t* run_goff,
                        const Chunk* windows, int64_t nwindows, void* perm, hipStream_t s, int phase_support = 0);
bool order_phases_ok(const RowMap& m, int support);
hipError_t launch_crop_correct_2d(const double* grid, const GridGeometry& g, int64_t npix_x, int64_t npix_y,
                                  const double* cx, const double* cy, double* dirty, hipStream_t s);
hipError_t launch_wplane_accumulate(const double* grid, const GridGeometry& g, int64_t npix_x, int64_t npix_y,
                                    double pixsize_x, double pixsize_y, double w_plane, int first,
                                    double* acc, hipStream_t s);
// image rows [i0, i0 + nrows) held as acc rows 0.. (nrows < 0: to npix_x);
// norm (may be NULL): also / *norm; acc_f32 (may be NULL): the planes were
// accumulated in this float buffer (the packed class) - corrected into acc
hipError_t launch_wfinal_correct(double* acc, int64_t npix_x, int64_t npix_y, double pixsize_x, double pixsize_y,
                                 const double* cx, const double* cy, const double* fw_table, int64_t fw_n,
                                 double fw_dnu, double dw, hipStream_t s, int64_t i0 = 0, int64_t nrows = -1,
                                 const double* norm = nullptr, const float* acc_f32 = nullptr);

// ---- pruned 2-D FFT (cip_fft.hip) -----------------------------------------
// gT: the grid transposed (nv rows of nu cells); H: (nx / 8) x nv x 8 complex;
// tw_u / tw_v: exp(+2 pi i m / n), m < n (interleaved re, im).
// mode 0: out = dirty (crop + cx cy); mode 1: out = w-plane accumulator.
bool fast_fft_supported(int64_t nu, int64_t nv, int64_t nx, int64_t ny);
// dmask (bit-packed dirty tiles, ntx / 32 words per 32-cell tile row of gT,
// NULL = dense): cells of tiles whose bit is 0 are known zero and not read;
// cells of marked tiles are read and then ZEROED (the grid is left all-zero
// for the next scatter)
// grid_f32: the planes hold complex64 cells (the packed class, GridGeometry::grid_f32)
// and H complex64 values (pass A's output; launch_fft_cols with h_f32)
hipError_t launch_fft_rows(double* gT, int64_t nu, int64_t nv, int64_t nx, const double* tw_u, double* H,
                           const uint32_t* dmask, int64_t ntx, bool skip_clean, hipStream_t s,
                           bool grid_f32 = false, bool eo = false);
hipError_t launch_fft_cols(const double* H, int64_t nv, int64_t nx, int64_t ny, const double* tw_v, int mode,
                           double* out, const double* cx, const double* cy, double px, double py, double w_plane,
                           int first, const double* norm, const uint32_t* rowbits, hipStream_t s,
                           bool h_f32 = false, bool acc_f32 = false, bool eo = false);
// pass B of a 2-D crop by even / odd column halves (fp64, nv = 16384, ny <=
// nv / 2): pass A and pass B of one plane both take eo = fft_cols_eo(...)
bool fft_cols_eo(int64_t nv, int64_t ny, bool grid_f32, int mode);
// acc_f32: out is the packed class's float plane accumulator (mode 1, h_f32,
// fp32 transforms only: hipErrorInvalidValue otherwise - the fp64-output
// kernels would write doubles into a float buffer)
bool fft_f32_enabled();
// strips (multi-GPU strong scaling): pass A over rows [y0, y1)
// of gT (zeroed after reading) into H with y1 - y0 rows per block; pass B for
// image rows [i0, i1) (multiples of the column block) from an H holding those
// blocks (nv rows each), out = the strip's rows (2-D epilogue, / *norm if set)
// dmask (may be NULL): dirty-tile bits of the whole grid (as launch_fft_rows),
// buffer row y = grid row (row0 + y) mod nv; only the dirty tiles' cells are
// read and zeroed (the rest of the buffer is zero)
// row_slot (with dmask; may be NULL): the packed form - buffer row y goes to
// H row row_slot[y - y0] of an H with nlive rows per block, rows with
// row_slot < 0 (no dirty tile in their tile row) are skipped
hipError_t launch_fft_rows_strip(double* gT, int64_t nu, int64_t nv, int64_t nx, const double* tw_u, int64_t y0,
                                 int64_t y1, double* H, hipStream_t s, const uint32_t* dmask = nullptr,
                                 int64_t row0 = 0, const int64_t* row_slot = nullptr, int64_t nlive = 0);
hipError_t launch_fft_cols_strip(const double* H, int64_t nv, int64_t nx, int64_t ny, const double* tw_v, int64_t i0,
                                 int64_t i1, double* out, const double* cx, const double* cy, const double* norm,
                                 hipStream_t s);
// the same for one w plane of a w-stacking strip: acc rows (+)= the plane's
// screened contribution (mode 1 epilogue; first: overwrite)
hipError_t launch_fft_cols_strip_wplane(const double* H, int64_t nv, int64_t nx, int64_t ny, const double* tw_v,
                                        int64_t i0, int64_t i1, double* acc, double px, double py, double w_plane,
                                        bool first, hipStream_t s);
// out[0..n) /= *sumw (device scalar)
hipError_t launch_scale_inverse(double* out, int64_t n, const double* sumw, hipStream_t s);

// ---- reference tiling + Stokes I (cip_tiling.hip) --------------------------
hipError_t launch_tile_run_count(const double* uvw, int64_t nrow, const double* winv, int64_t nchan,
                                 double t0, double t1, double t2, int64_t* row_runs, hipStream_t s);
hipError_t launch_tile_run_emit(const double* uvw, int64_t nrow, const double* winv, int64_t nchan,
                                double t0, double t1, double t2, int64_t row_offset, const int64_t* row_off,
                                int64_t* run_key, int64_t* run_row, int32_t* run_c0, int32_t* run_c1,
                                hipStream_t s);
hipError_t launch_wavelength_inv(const double* freq, int64_t nchan, double* winv, hipStream_t s);
hipError_t launch_facet_rephase(const double* uvw, int64_t nrow, const double* freq, int64_t nchan, const void* vis,
                                int vis_c128, const double qt[9], double l0, double m0, double* uvw_out,
                                double* delay, void* vis_out, hipStream_t s);
hipError_t launch_stokes(int stokes, const void* vis4, const uint8_t* flags4, const float* wgt4, int64_t n,
                         void* vis_i, uint8_t* flag_i, float* wgt_i, float* eff_w, hipStream_t s);

// the uv-strip split (cip_strips.hip): per grid row, the visibilities whose
// footprint origin lies in it and the row slices starting there (hist: 2 nv
// int64, stream-ordered; partial: strip_hist_blocks(nrow) * 2 nv uint32); per
// MS row the strip [y0, y1)'s runs and visibilities (row_runs / row_vis,
// nrow + 1 entries, exclusive-scanned by the caller); the runs as row slices
// with the visibilities (vis_bytes 8 / 16, 0: none) and weights (wgt_bytes
// 4 / 8, 0: none) gathered into slice order
int strip_hist_blocks(int64_t nrow);
hipError_t launch_strip_hist(const double* uvw, int64_t nrow, const double* fx, int64_t nchan,
                             const GridGeometry& g, uint32_t* partial, int nblocks, int64_t* hist, hipStream_t s);
hipError_t launch_strip_count(const double* uvw, int64_t nrow, const double* fx, int64_t nchan,
                              const GridGeometry& g, int64_t y0, int64_t y1, int64_t* row_runs, int64_t* row_vis,
                              hipStream_t s);
hipError_t launch_strip_emit(const double* uvw, int64_t nrow, const double* fx, int64_t nchan, const GridGeometry& g,
                             int64_t y0, int64_t y1, const int64_t* run_off, const int64_t* vis_off, const void* vis,
                             int vis_bytes, const void* wgt, int wgt_bytes, double* slice_uvw, int32_t* chan_start,
                             int32_t* chan_stop, int64_t* slice_row, void* vis_out, void* wgt_out, hipStream_t s);
// a strip's dirty-tile bits: the plan's mask (may be NULL) | the tile rows of
// grid rows row0 .. row0 + halo - 1 (nplanes * nty * ntx / 32 words)
hipError_t launch_strip_mask(const uint32_t* dmask, const GridGeometry& g, int64_t row0, int64_t halo, uint32_t* out,
                             hipStream_t s);

// the strips' sparse all-to-all: pack this rank's live pass-A rows / unpack
// a receiver's pass-B input (cip_grid.hip; units = 16-B units per record)
hipError_t launch_strip_pack(const void* H, int64_t nb, int64_t h, int units, const int64_t* slot, int64_t nlive,
                             void* out, hipStream_t s);
hipError_t launch_strip_unpack(const void* recv, int64_t nb, int64_t nv, int units, const int64_t* rec,
                               const int64_t* stride, void* H, hipStream_t s);

}  // namespace cip
