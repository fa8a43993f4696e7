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
