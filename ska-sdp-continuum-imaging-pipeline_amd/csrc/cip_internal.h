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
hipError_t exclusive_scan_i64(int64_t* data, int64_t n, int64_t* tmp, hipStream_t s);

// ---- gridder planner (cip_plan.hip) ----------------------------------------
hipError_t launch_freq_scale(const double* freq, int64_t nchan, double* fx, hipStream_t s);
// per-row w range over channels (only f min/max matter): out[0]=min, out[1]=max
hipError_t launch_w_range(const double* uvw, int64_t nrow, double fxmin, double fxmax, double* partial,
                          int nblocks, hipStream_t s);
// place pass: runs per tile (atomics), per-visibility bank class, parked runs
// (park_* hold 64 slots per 64-visibility segment, seg_nruns the used ones)
hipError_t launch_plan_place(const double* uvw, int64_t nrow, const double* fx, int64_t nchan,
                             const GridGeometry& g, int64_t* tile_runs, unsigned* err_flag, uint8_t* vis_class,
                             uint8_t* seg_nruns, int64_t* park_key, uint64_t* park_run, hipStream_t s);
hipError_t launch_plan_distribute(int64_t nvis, const uint8_t* seg_nruns, const int64_t* park_key,
                                  const uint64_t* park_run, const int64_t* tile_run_off, int64_t* tile_cursor,
                                  uint64_t* runs, hipStream_t s);
hipError_t launch_tile_vis(const int64_t* run_goff, const int64_t* tile_run_off, int64_t ntiles,
                           int64_t* tile_vis_off, int64_t* tile_vis, hipStream_t s);
hipError_t launch_run_lengths(const uint64_t* runs, int64_t nruns, int64_t* out, hipStream_t s);
hipError_t launch_chunk_counts(const int64_t* tile_vis, int64_t ntiles, int64_t chunk_vis,
                               int64_t* out, hipStream_t s);
hipError_t launch_chunk_emit(const int64_t* tile_vis_off, const int64_t* tile_vis, const int64_t* chunk_off,
                             const int64_t* run_goff, const int64_t* tile_run_off, int64_t ntiles,
                             int64_t chunk_vis, Chunk* chunks, hipStream_t s);
hipError_t launch_gather_i64(const int64_t* src, int64_t stride, int64_t count, int64_t* dst,
                             hipStream_t s);

// ---- gridding (cip_grid.hip) -----------------------------------------------
// vis_dtype/wgt_dtype: CIP_* codes. partial needs 2 * nblocks doubles.
hipError_t launch_prep_reduce(const void* vis, int vis_dtype, const void* wgt, int wgt_dtype, int64_t n,
                              double* partial, int nblocks, double* out2, hipStream_t s);
int prep_blocks();
// packed: single-precision class (re/im packed in one 64-bit integer), complex64
// only. perm: bank-class ordered stream from launch_order, or NULL (visibilities
// located through the tile's row slices in tile order).
hipError_t launch_scatter(int support, int vis_dtype, int wgt_dtype, bool packed, const double* uvw,
                          const double* fx, const void* vis, const void* wgt, int64_t nchan, const uint64_t* runs,
                          const int64_t* run_goff, const int64_t* tile_run_off, const uint64_t* perm,
                          const Chunk* chunks, int64_t chunk_begin, int64_t nchunks, const GridGeometry& g,
                          int64_t plane, double fixed_scale, double* grid, hipStream_t s);
// perm[g] for every tile-order position g of every chunk (cip_grid.hip)
hipError_t launch_order(const uint8_t* vis_class, int64_t nchan, const uint64_t* runs, const int64_t* run_goff,
                        const int64_t* tile_run_off, const Chunk* chunks, int64_t nchunks, uint64_t* perm,
                        hipStream_t s);
hipError_t launch_crop_correct_2d(const double* grid, const GridGeometry& g, int64_t npix_x, int64_t npix_y,
                                  const double* cx, const double* cy, double* dirty, hipStream_t s);
hipError_t launch_wplane_accumulate(const double* grid, const GridGeometry& g, int64_t npix_x, int64_t npix_y,
                                    double pixsize_x, double pixsize_y, double w_plane, int first,
                                    double* acc, hipStream_t s);
hipError_t launch_wfinal_correct(double* acc, int64_t npix_x, int64_t npix_y, double pixsize_x, double pixsize_y,
                                 const double* cx, const double* cy, const double* fw_table, int64_t fw_n,
                                 double fw_dnu, double dw, hipStream_t s);

// ---- reference tiling + Stokes I (cip_tiling.hip) --------------------------
hipError_t launch_tile_run_count(const double* uvw, int64_t nrow, const double* winv, int64_t nchan,
                                 double t0, double t1, double t2, int64_t* row_runs, hipStream_t s);
hipError_t launch_tile_run_emit(const double* uvw, int64_t nrow, const double* winv, int64_t nchan,
                                double t0, double t1, double t2, int64_t row_offset, const int64_t* row_off,
                                int64_t* run_key, int64_t* run_row, int32_t* run_c0, int32_t* run_c1,
                                hipStream_t s);
hipError_t launch_wavelength_inv(const double* freq, int64_t nchan, double* winv, hipStream_t s);
hipError_t launch_stokes_i(const void* vis4, const uint8_t* flags4, const float* wgt4, int64_t n,
                           void* vis_i, uint8_t* flag_i, float* wgt_i, float* eff_w, hipStream_t s);

}  // namespace cip
