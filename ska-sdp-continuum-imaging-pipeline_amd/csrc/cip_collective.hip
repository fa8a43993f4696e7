// cip_collective.hip - RCCL (over xGMI) reduction of per-device partial grids
// or images for a single process driving several GPUs (SURVEY.md 8(b)
// cip_allreduce_grid, 8(e)). The product's multi-GPU path is one process per
// GPU with torch.distributed (RCCL) in the host layer; this entry point is the
// native equivalent for a C/C++ host that owns all the devices itself.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "cip_internal.h"

namespace {

std::mutex g_comm_mutex;
std::map<std::vector<int>, std::vector<ncclComm_t>> g_comms;  // one clique per device list

int nccl_fail(ncclResult_t r, const char* what) {
  return cip::set_error(CIP_EHIP, std::string(what) + ": " + ncclGetErrorString(r));
}

// Restores the caller's current device on every exit path.
struct DeviceGuard {
  int prev = 0;
  bool ok = false;
  DeviceGuard() { ok = hipGetDevice(&prev) == hipSuccess; }
  ~DeviceGuard() {
    if (ok) (void)hipSetDevice(prev);
  }
};

}  // namespace

extern "C" int cip_allreduce_grid(void* const* grids, const int* devices, int ndev, int64_t nelem, int root,
                                  void* const* hip_streams) {
  if (!grids || !devices || ndev < 1 || nelem < 0)
    return cip::set_error(CIP_EINVAL, "need grids, devices, ndev >= 1, nelem >= 0");
  if (root >= ndev) return cip::set_error(CIP_EINVAL, "root must be < ndev (or < 0 for all-reduce)");
  for (int k = 0; k < ndev; ++k)
    if (!grids[k]) return cip::set_error(CIP_EINVAL, "NULL grid");
  std::vector<int> devs(devices, devices + ndev);
  {
    std::vector<int> sorted = devs;
    std::sort(sorted.begin(), sorted.end());
    if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end())
      return cip::set_error(CIP_EINVAL, "devices must be distinct (one communicator rank per device)");
    if (sorted.front() < 0) return cip::set_error(CIP_EINVAL, "negative device index");
  }
  if (nelem == 0) return CIP_OK;
  const DeviceGuard guard;  // ncclCommInitAll and the synchronisation loop switch devices
  std::vector<ncclComm_t>* comms = nullptr;
  {
    std::lock_guard<std::mutex> lock(g_comm_mutex);
    auto it = g_comms.find(devs);
    if (it == g_comms.end()) {
      std::vector<ncclComm_t> c(ndev);
      const ncclResult_t r = ncclCommInitAll(c.data(), ndev, devs.data());
      if (r != ncclSuccess) return nccl_fail(r, "ncclCommInitAll");
      it = g_comms.emplace(devs, std::move(c)).first;
    }
    comms = &it->second;
  }
  // fp64 sums (the grids / images are fp64); one group call over all devices
  ncclResult_t r = ncclGroupStart();
  if (r != ncclSuccess) return nccl_fail(r, "ncclGroupStart");
  for (int k = 0; k < ndev; ++k) {
    hipStream_t s = hip_streams ? (hipStream_t)hip_streams[k] : nullptr;
    if (root < 0)
      r = ncclAllReduce(grids[k], grids[k], (size_t)nelem, ncclFloat64, ncclSum, (*comms)[k], s);
    else
      r = ncclReduce(grids[k], grids[k], (size_t)nelem, ncclFloat64, ncclSum, root, (*comms)[k], s);
    if (r != ncclSuccess) {
      (void)ncclGroupEnd();
      return nccl_fail(r, "ncclAllReduce/ncclReduce");
    }
  }
  r = ncclGroupEnd();
  if (r != ncclSuccess) return nccl_fail(r, "ncclGroupEnd");
  for (int k = 0; k < ndev; ++k) {
    if (hipSetDevice(devs[k]) != hipSuccess) return cip::set_error(CIP_EHIP, "hipSetDevice failed");
    hipStream_t s = hip_streams ? (hipStream_t)hip_streams[k] : nullptr;
    if (hipStreamSynchronize(s) != hipSuccess) return cip::set_error(CIP_EHIP, "hipStreamSynchronize failed");
  }
  return CIP_OK;
}

extern "C" int cip_release_collectives(void) {
  std::lock_guard<std::mutex> lock(g_comm_mutex);
  for (auto& kv : g_comms)
    for (auto c : kv.second) (void)ncclCommDestroy(c);
  g_comms.clear();
  return CIP_OK;
}
