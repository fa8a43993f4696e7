// cip_scatter_w.hip - one kernel support per translation unit: compiled once
// per W in {4, 6, ..., 16} with -DCIP_SCATTER_W=W (Makefile), so the scatter
// instantiations build in parallel.
#include "cip_scatter.h"

#ifndef CIP_SCATTER_W
#error "compile with -DCIP_SCATTER_W=<support>"
#endif

namespace cip {
template hipError_t launch_scatter_w<CIP_SCATTER_W>(int, int, bool, int, unsigned, int, dim3, hipStream_t, const double*, const double*,
                                                    const void*, const void*, const RowMap&, const uint64_t*,
                                                    const int64_t*, const int64_t*, const void*,
                                                    const Chunk*, int64_t, const GridGeometry&, int64_t, double,
                                                    double*);
}  // namespace cip

#ifdef CIP_COUNT_KBLOCKS
// experiment builds only (tools): the packed plane-group scatter's block counters
namespace cip {
__device__ unsigned long long cip_kblock_count[192];
}
extern "C" int cip_debug_kblocks(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(cip::cip_kblock_count), sizeof(unsigned long long) * 192) != hipSuccess)
    return 1;
  if (reset) {
    unsigned long long z[192] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(cip::cip_kblock_count), z, sizeof(z)) != hipSuccess) return 2;
  }
  return 0;
}
#endif
