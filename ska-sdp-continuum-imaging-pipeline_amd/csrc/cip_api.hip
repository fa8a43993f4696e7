// cip_api.hip - the C ABI of libcip_hip.so (include/cip.h): parameter choice,
// per-device workspace, the plan -> scatter -> FFT -> correct pipeline of
// ms2dirty, the reference tiling runs and the Stokes-I conversion.
#include <hipfft/hipfft.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "cip_internal.h"

namespace cip {

static thread_local std::string g_last_error;

int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

// ----------------------------------------------------------- profiler ----
// hipEvents recorded on the call's stream around each phase (cip_profile_*).
struct Profiler {
  bool on = false;
  int device = -1;
  std::vector<hipEvent_t> pool;
  size_t used = 0;
  struct Span {
    int phase;
    hipEvent_t a, b;
  };
  std::vector<Span> spans;
  double ms[CIP_PROFILE_PHASES] = {0};
  int64_t counts[CIP_PROFILE_COUNTS] = {0};

  void reset() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev != device) {  // events belong to a device
      for (auto e : pool) (void)hipEventDestroy(e);
      pool.clear();
      device = dev;
    }
    used = 0;
    spans.clear();
    for (auto& m : ms) m = 0.0;
    for (auto& c : counts) c = 0;
  }
  hipEvent_t mark(hipStream_t s) {
    if (!on) return nullptr;
    if (used == pool.size()) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return nullptr;
      pool.push_back(e);
    }
    hipEvent_t e = pool[used++];
    if (hipEventRecord(e, s) != hipSuccess) return nullptr;
    return e;
  }
  void span(int phase, hipEvent_t a, hipEvent_t b) {
    if (on && a && b) spans.push_back({phase, a, b});
  }
  void finish() {  // stream already synchronised
    if (!on) return;
    for (auto& sp : spans) {
      float t = 0.f;
      if (hipEventElapsedTime(&t, sp.a, sp.b) == hipSuccess) ms[sp.phase] += t;
    }
  }
};
static thread_local Profiler g_prof;

// ------------------------------------------------------------ kernels ----
// Host copies of the kernel coefficient tables (same data as the device side).
struct HostKernel {
  int W, D;
  double beta;
  const double* coef;  // [W/2][D+1]
};

#define CIP_HOST_TABLE(WW)                                                          \
  static const double host_coef_##WW[WW / 2][CIP_ES_DEGREE_##WW + 1] = CIP_ES_COEFFS_##WW;
CIP_HOST_TABLE(4)
CIP_HOST_TABLE(6)
CIP_HOST_TABLE(8)
CIP_HOST_TABLE(10)
CIP_HOST_TABLE(12)
CIP_HOST_TABLE(14)
CIP_HOST_TABLE(16)
CIP_HOST_TABLE(24)
CIP_HOST_TABLE(32)
CIP_HOST_TABLE(48)
CIP_HOST_TABLE(64)
#undef CIP_HOST_TABLE

static bool host_kernel(int W, HostKernel* k) {
  switch (W) {
#define CASE(WW)                                                              \
  case WW:                                                                    \
    *k = {WW, CIP_ES_DEGREE_##WW, CIP_ES_BETA_##WW, &host_coef_##WW[0][0]};  \
    return true;
    CASE(4) CASE(6) CASE(8) CASE(10) CASE(12) CASE(14) CASE(16) CASE(24) CASE(32) CASE(48) CASE(64)
#undef CASE
    default:
      return false;
  }
}

static double piece_value(const HostKernel& k, int piece, double y) {
  const int half = k.W / 2;
  const double* c = (piece < half) ? k.coef + piece * (k.D + 1) : k.coef + (k.W - 1 - piece) * (k.D + 1);
  const double yy = (piece < half) ? y : -y;
  double r = c[k.D];
  for (int d = k.D - 1; d >= 0; --d) r = r * yy + c[d];
  return r;
}

// Gauss-Legendre nodes/weights on [-1, 1]
static void gauss_legendre(int n, std::vector<double>& x, std::vector<double>& w) {
  x.resize(n);
  w.resize(n);
  for (int i = 0; i < n; ++i) {
    double z = std::cos(M_PI * (i + 0.75) / (n + 0.5));
    for (int it = 0; it < 100; ++it) {
      double p0 = 1.0, p1 = z;
      for (int j = 2; j <= n; ++j) {
        const double p2 = ((2.0 * j - 1.0) * z * p1 - (j - 1.0) * p0) / j;
        p0 = p1;
        p1 = p2;
      }
      const double dp = n * (z * p1 - p0) / (z * z - 1.0);
      const double dz = p1 / dp;
      z -= dz;
      if (std::fabs(dz) < 1e-16) break;
    }
    double p0 = 1.0, p1 = z;
    for (int j = 2; j <= n; ++j) {
      const double p2 = ((2.0 * j - 1.0) * z * p1 - (j - 1.0) * p0) / j;
      p0 = p1;
      p1 = p2;
    }
    const double dp = n * (z * p1 - p0) / (z * z - 1.0);
    x[i] = z;
    w[i] = 2.0 / ((1.0 - z * z) * dp * dp);
  }
}

// F(nu) = integral of the piecewise kernel phi(d) cos(2 pi d nu) over its support
// (d in cells); the grid correction of axis u is 1 / F(p / n_u).
struct KernelFT {
  HostKernel k;
  std::vector<double> gx, gw;
  explicit KernelFT(const HostKernel& kk) : k(kk) { gauss_legendre(24, gx, gw); }
  double operator()(double nu) const {
    double acc = 0.0;
    for (int piece = 0; piece < k.W; ++piece) {
      const double a = piece - 0.5 * k.W;  // piece spans d in [a, a + 1]
      for (size_t i = 0; i < gx.size(); ++i) {
        const double d = a + 0.5 * (gx[i] + 1.0);
        const double y = 2.0 * piece + 1.0 - k.W - 2.0 * d;
        acc += 0.5 * gw[i] * piece_value(k, piece, y) * std::cos(2.0 * M_PI * d * nu);
      }
    }
    return acc;
  }
};

// ------------------------------------------------------------- params ----
static int64_t good_size(int64_t n) {
  if (n < 16) n = 16;
  for (int64_t m = n + (n & 1);; m += 2) {
    int64_t r = m;
    for (int64_t p : {2, 3, 5, 7})
      while (r % p == 0) r /= p;
    if (r == 1) return m;
  }
}

static int support_for_epsilon(double eps) {
  // calibrated against the fp64 direct DFT (DESIGN.md "Accuracy")
  // max |err| / sum(w) vs the direct DFT measured 2e-3, 2e-5, 3e-7, 4e-9,
  // 5e-11, 6e-13, 2e-14 for W = 4 .. 16 (tests/test_oracle_accuracy.py)
  if (eps >= 2e-3) return 4;
  if (eps >= 2e-5) return 6;
  if (eps >= 3e-7) return 8;
  if (eps >= 4e-9) return 10;
  if (eps >= 5e-11) return 12;
  if (eps >= 6e-13) return 14;
  return 16;
}

static int choose(int64_t npix_x, int64_t npix_y, double px, double py, double epsilon, int support,
                  int do_wstacking, double wmin, double wmax, cip_gridder_params* out) {
  if (npix_x < 2 || npix_y < 2 || (npix_x & 1) || (npix_y & 1))
    return set_error(CIP_EINVAL, "npix_x and npix_y must be even and >= 2");
  if (!(px > 0.0) || !(py > 0.0)) return set_error(CIP_EINVAL, "pixel sizes must be positive");
  if (support > 0) {
    // W <= 16: lane-per-visibility scatter; 24..64 (BASELINE configs[2]'s
    // LDS-tile stress case): wave-per-visibility scatter (cip_scatter_large.hip)
    const bool small = !(support & 1) && support >= 4 && support <= 16;
    const bool large = support == 24 || support == 32 || support == 48 || support == 64;
    if (!small && !large)
      return set_error(CIP_EINVAL, "support must be an even number in [4, 16] or one of 24, 32, 48, 64");
    // (the large supports' shape beta keeps W = 16's edge ratio F(1/4)/F(0),
    // tools/gen_es_kernels.py, so their grid and w corrections amplify the
    // fixed-point quantum no more than W = 16's: w-stacking at every support)
  } else {
    if (!(epsilon > 0.0)) return set_error(CIP_EINVAL, "epsilon must be positive");
    support = support_for_epsilon(epsilon);
  }
  HostKernel hk;
  host_kernel(support, &hk);
  cip_gridder_params p;
  std::memset(&p, 0, sizeof(p));
  p.sigma = 2.0;
  p.nu = good_size((int64_t)std::ceil(p.sigma * npix_x));
  p.nv = good_size((int64_t)std::ceil(p.sigma * npix_y));
  // a footprint wraps around the periodic grid at most once
  if (p.nu < support || p.nv < support) return set_error(CIP_EINVAL, "grid smaller than the kernel support");
  p.support = support;
  p.degree = hk.D;
  p.beta = hk.beta;
  p.tile = kTile;
  const double x0 = -0.5 * npix_x * px, y0 = -0.5 * npix_y * py;
  const double e = x0 * x0 + y0 * y0;
  if (e >= 1.0) return set_error(CIP_EINVAL, "field of view extends beyond the horizon");
  p.nmin = -e / (std::sqrt(1.0 - e) + 1.0);
  p.do_wstacking = do_wstacking ? 1 : 0;
  if (do_wstacking) {
    if (!(wmax >= wmin)) return set_error(CIP_EINVAL, "invalid w range");
    p.dw = 0.5 / p.sigma / std::fabs(p.nmin);
    p.nplanes = (int64_t)std::ceil((wmax - wmin) / p.dw) + support;
    p.w0 = 0.5 * (wmin + wmax) - 0.5 * (double)(p.nplanes - 1) * p.dw;
  } else {
    p.nplanes = 1;
    p.w0 = 0.0;
    p.dw = 1.0;
  }
  *out = p;
  return CIP_OK;
}

static GridGeometry geometry(const cip_gridder_params& p, double px, double py) {
  GridGeometry g;
  g.nu = p.nu;
  g.nv = p.nv;
  g.support = p.support;
  g.scale_u = (double)p.nu * px;
  g.scale_v = (double)p.nv * py;
  g.do_wstacking = p.do_wstacking;
  g.w0 = p.w0;
  g.dw = p.dw;
  g.inv_dw = 1.0 / p.dw;
  g.nplanes = p.nplanes;
  g.tile = p.tile;
  g.ntx = (p.nu + p.tile - 1) / p.tile;
  g.nty = (p.nv + p.tile - 1) / p.tile;
  g.ntw = p.do_wstacking ? (p.nplanes - p.support + 1) : 1;
  g.transposed = 0;
  g.row0 = 0;
  g.rows = p.nv;
  g.oob = nullptr;
  g.plane_lo = 0;
  g.plane_hi = p.nplanes;
  g.grid_f32 = 0;
  g.wmask = nullptr;
  return g;
}

// ---------------------------------------------------------- workspace ----
struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
};

struct FftPlan {
  hipfftHandle h;
  int64_t nu, nv;
};

struct PlanResult {
  int64_t nruns = 0, ntiles = 0, nchunks = 0;
  std::vector<int64_t> plane_chunk_off;  // chunk offset of each range: w plane group q (ngroups + 1), or the 2-D layer
  int group = 1;                         // w planes per work unit (w-stacking plane groups)
  uint64_t* runs = nullptr;
  int64_t* run_goff = nullptr;
  int64_t* tile_run_off = nullptr;
  Chunk* chunks = nullptr;
  void* perm = nullptr;  // bank-class ordered visibility stream (perm_encode entries), or NULL
  bool phases = false;   // perm's entries carry row phases (RowMap::row_phase for the scatter)
  uint32_t* dmask = nullptr;  // grid tiles the scatter writes, per plane (bit-packed, ntx / 32 words per tile row)
};

struct Workspace {
  int device = 0;  // the device every buffer, stream and event belongs to
  std::map<std::string, DevBuf> bufs;
  std::vector<FftPlan> plans;
  void* pinned = nullptr;  // small host staging
  size_t pinned_bytes = 0;
  std::vector<int64_t> corr_key;  // (npix_x, npix_y, nu, nv, W) of the cached cx / cy
  std::vector<double> fw_key;     // (W, dw |nmin|) of the cached w-correction table
  std::vector<int64_t> tw_ready;  // lengths whose FFT twiddle tables are on the device
  // second stream: zeroes the first grid plane while the planner runs
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  bool side_pending = false;
  // the "grid" buffer when it is known all-zero (the masked FFT pass A zeroes
  // what the scatter wrote), else NULL
  double* grid_clean = nullptr;
  // how many of its leading BYTES are known zero: a call on a smaller grid
  // zeroes (and keeps clean) only its own planes' bytes, so the state is a byte
  // count, not a plane count (a later larger-geometry call must not trust it)
  size_t grid_clean_bytes = 0;
  // CIP_ASYNC pipelining (cip_ms2dirty): consecutive calls alternate between
  // two sets of planner buffers (parity; buf() appends the parity to buffer
  // names while parity_scope is set), so the planner of call k + 1 runs on
  // plan_stream beside call k's scatter and FFT; it only waits for
  // call k - 1's work on the caller's stream (ev_done[parity]: its scatter
  // read the plan, its FFT the masks and weight sum); the caller's stream
  // waits for the plan (ev_planned). One plan stream per parity.
  hipStream_t plan_stream = nullptr, plan_stream1 = nullptr;
  hipEvent_t ev_done[2] = {nullptr, nullptr}, ev_planned = nullptr, ev_entry = nullptr;
  uint64_t call_seq = 0;
  int parity = 0;
  bool parity_scope = false;
  // a planner ran on a caller's stream (parity-0 buffer names) since the last
  // pipelined call: the next pipelined planner waits for that stream
  bool plan_unscoped = false;
  // the stream of the last CIP_ASYNC call, whose work may still be queued: a
  // call on another stream first waits for it (the workspace is shared)
  hipStream_t async_stream = nullptr;
  // the last complete plan (its buffers stay untouched until the next planner
  // runs) and the geometry it was made for: CIP_REUSE_PLAN calls with the
  // same key grid through it. Cleared when a planner starts; never set for
  // ragged rows (their row map lives in per-call buffers).
  bool saved_valid = false;
  std::vector<double> saved_key;
  cip_gridder_params saved_p;
  PlanResult saved_plan;
};

static int settle_async(Workspace* ws, hipStream_t s) {
  hipStream_t prev = ws->async_stream;
  ws->async_stream = nullptr;
  if (prev && prev != s) CIP_HIP_CHECK(hipStreamSynchronize(prev));
  return CIP_OK;
}

// Zero `bytes` at `p` on the workspace's side stream, ordered after the work
// already queued on s; join_side() makes s wait for it.
static int zero_on_side(Workspace* ws, void* p, size_t bytes, hipStream_t s) {
  if (!ws->side) {
    CIP_HIP_CHECK(hipStreamCreateWithFlags(&ws->side, hipStreamNonBlocking));
    CIP_HIP_CHECK(hipEventCreateWithFlags(&ws->ev_fork, hipEventDisableTiming));
    CIP_HIP_CHECK(hipEventCreateWithFlags(&ws->ev_join, hipEventDisableTiming));
  }
  CIP_HIP_CHECK(hipEventRecord(ws->ev_fork, s));
  CIP_HIP_CHECK(hipStreamWaitEvent(ws->side, ws->ev_fork, 0));
  CIP_HIP_CHECK(hipMemsetAsync(p, 0, bytes, ws->side));
  CIP_HIP_CHECK(hipEventRecord(ws->ev_join, ws->side));
  ws->side_pending = true;
  return CIP_OK;
}

static int join_side(Workspace* ws, hipStream_t s) {
  if (!ws->side_pending) return CIP_OK;
  ws->side_pending = false;
  CIP_HIP_CHECK(hipStreamWaitEvent(s, ws->ev_join, 0));
  return CIP_OK;
}

static std::mutex g_ws_mutex;
// One workspace per (device, host thread): calls from different threads (e.g.
// two inverts in flight on one GPU, each thread on its own stream) never
// share buffers, the side stream or the clean-grid state. A workspace holds
// the uv grid (16 nu nv bytes) and planner buffers that grow with the
// visibility count, so it lives only as long as its thread: a thread-exit hook
// frees the workspaces of every worker thread that made one (dask worker
// pools keep HBM use at one workspace per live thread), and
// cip_release_workspace frees the calling thread's on demand.
static std::map<std::pair<int, std::thread::id>, Workspace*> g_ws;
// the thread that loaded the library: its workspaces are left to process
// teardown (its thread-exit hook runs inside exit(), where the HIP runtime
// may already be shutting down)
static const std::thread::id g_load_thread = std::this_thread::get_id();

static void destroy_workspace(Workspace* ws) {
  // the workspace's device current while its buffers go (the reaper may run on
  // a thread whose current device differs), and a CIP_ASYNC call's work drained
  // first: its scatter / FFT may still be queued on the caller's stream
  int prev_dev = -1;
  (void)hipGetDevice(&prev_dev);
  if (prev_dev != ws->device) (void)hipSetDevice(ws->device);
  if (ws->async_stream) (void)hipStreamSynchronize(ws->async_stream);
  if (ws->plan_stream) (void)hipStreamSynchronize(ws->plan_stream);
  if (ws->plan_stream1) (void)hipStreamSynchronize(ws->plan_stream1);
  for (auto& kv : ws->bufs)
    if (kv.second.ptr) (void)hipFree(kv.second.ptr);
  for (auto& p : ws->plans) (void)hipfftDestroy(p.h);
  if (ws->pinned) (void)hipHostFree(ws->pinned);
  if (ws->side) {
    (void)hipStreamSynchronize(ws->side);
    (void)hipStreamDestroy(ws->side);
  }
  if (ws->ev_fork) (void)hipEventDestroy(ws->ev_fork);
  if (ws->ev_join) (void)hipEventDestroy(ws->ev_join);
  for (hipStream_t ps : {ws->plan_stream, ws->plan_stream1})
    if (ps) {
      (void)hipStreamSynchronize(ps);
      (void)hipStreamDestroy(ps);
    }
  for (hipEvent_t e : ws->ev_done)
    if (e) (void)hipEventDestroy(e);
  if (ws->ev_planned) (void)hipEventDestroy(ws->ev_planned);
  if (ws->ev_entry) (void)hipEventDestroy(ws->ev_entry);
  const int dev = ws->device;
  delete ws;
  if (prev_dev >= 0 && prev_dev != dev) (void)hipSetDevice(prev_dev);
}

// Frees the calling thread's workspaces (every device) when the thread ends.
struct WorkspaceReaper {
  bool armed = false;
  ~WorkspaceReaper() {
    if (!armed || std::this_thread::get_id() == g_load_thread) return;
    std::vector<Workspace*> mine;
    {
      std::lock_guard<std::mutex> lock(g_ws_mutex);
      for (auto it = g_ws.begin(); it != g_ws.end();) {
        if (it->first.second == std::this_thread::get_id()) {
          mine.push_back(it->second);
          it = g_ws.erase(it);
        } else {
          ++it;
        }
      }
    }
    for (Workspace* ws : mine) destroy_workspace(ws);
  }
};
static thread_local WorkspaceReaper g_reaper;

static Workspace* workspace() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  const auto key = std::make_pair(dev, std::this_thread::get_id());
  g_reaper.armed = true;
  std::lock_guard<std::mutex> lock(g_ws_mutex);
  auto it = g_ws.find(key);
  if (it != g_ws.end()) {
    ++it->second->call_seq;  // every entry point takes its workspace once per call
    return it->second;
  }
  Workspace* ws = new Workspace();
  ws->device = dev;
  g_ws[key] = ws;
  return ws;
}

// grow-only device buffer; returns nullptr (and sets the error) on failure
template <typename T>
static T* buf(Workspace* ws, const char* name, int64_t count) {
  const size_t bytes = (size_t)(count > 0 ? count : 1) * sizeof(T);
  DevBuf& b = ws->bufs[(ws->parity_scope && ws->parity) ? std::string(name) + "~1" : std::string(name)];
  if (b.bytes < bytes) {
    if (b.ptr && b.ptr == (void*)ws->grid_clean) ws->grid_clean = nullptr;  // a new buffer is not known zero
    if (b.ptr) ws->saved_valid = false;  // the saved plan may point into it
    if (b.ptr) (void)hipFree(b.ptr);
    b.ptr = nullptr;
    b.bytes = 0;
    // 12.5 % headroom so slowly growing inputs do not reallocate every call
    const size_t want = bytes + bytes / 8;
    if (hipMalloc(&b.ptr, want) != hipSuccess) {
      (void)hipGetLastError();
      set_error(CIP_ENOMEM, std::string("hipMalloc failed for workspace buffer ") + name);
      return nullptr;
    }
    b.bytes = want;
  }
  return (T*)b.ptr;
}

static void* pinned(Workspace* ws, size_t bytes) {
  if (ws->pinned_bytes < bytes) {
    if (ws->pinned) (void)hipHostFree(ws->pinned);
    ws->pinned = nullptr;
    ws->pinned_bytes = 0;
    if (hipHostMalloc(&ws->pinned, bytes) != hipSuccess) return nullptr;
    ws->pinned_bytes = bytes;
  }
  return ws->pinned;
}

static int fft_plan(Workspace* ws, int64_t nu, int64_t nv, hipStream_t s, hipfftHandle* out) {
  for (auto& p : ws->plans)
    if (p.nu == nu && p.nv == nv) {
      if (hipfftSetStream(p.h, s) != HIPFFT_SUCCESS) return set_error(CIP_EHIP, "hipfftSetStream failed");
      *out = p.h;
      return CIP_OK;
    }
  hipfftHandle h;
  if (hipfftPlan2d(&h, (int)nu, (int)nv, HIPFFT_Z2Z) != HIPFFT_SUCCESS)
    return set_error(CIP_EHIP, "hipfftPlan2d failed");
  if (hipfftSetStream(h, s) != HIPFFT_SUCCESS) return set_error(CIP_EHIP, "hipfftSetStream failed");
  ws->plans.push_back({h, nu, nv});
  *out = h;
  return CIP_OK;
}

// exp(+2 pi i m / n), m < n, for the pruned FFT passes (cached per length)
static int fft_twiddles(Workspace* ws, int64_t n, hipStream_t s, double** out) {
  const std::string name = "fft_twiddle_" + std::to_string(n);
  double* tw = buf<double>(ws, name.c_str(), 2 * n);
  if (!tw) return CIP_ENOMEM;
  if (std::find(ws->tw_ready.begin(), ws->tw_ready.end(), n) == ws->tw_ready.end()) {
    std::vector<double> h(2 * n);
    for (int64_t m = 0; m < n; ++m) {
      // long double arguments: each entry correctly rounded (to within an ulp)
      const long double a = 2.0L * 3.14159265358979323846264338327950288L * (long double)m / (long double)n;
      h[2 * m] = (double)cosl(a);
      h[2 * m + 1] = (double)sinl(a);
    }
    CIP_HIP_CHECK(hipMemcpyAsync(tw, h.data(), sizeof(double) * 2 * n, hipMemcpyHostToDevice, s));
    CIP_HIP_CHECK(hipStreamSynchronize(s));
    ws->tw_ready.push_back(n);
  }
  *out = tw;
  return CIP_OK;
}

#define CIP_ALLOC(var, T, name, n)  \
  T* var = buf<T>(ws, name, (n));   \
  if (!var) return CIP_ENOMEM;

// ------------------------------------------------------------- planner ----
// Visibilities per scatter work unit: <= kChunkVis (64-bit fixed point) or
// kChunkVisPacked (packed class, complex64 input); multiples of kOrderWindow,
// so 2-D ordering windows never straddle chunks (w-stacking units: see
// kOrderWindow in cip_common.h).
static int64_t chunk_vis(bool packed, int64_t nu) {
  // grids of 16384+ cells per axis (C4): half-size work units - shorter slices
  // on finer cells, the scatter's tail matters more (interleaved A/B at C4:
  // scatter 4.76 vs 4.89 ms, profiles/r02_ab_c4.txt)
  return packed ? kChunkVisPacked : (nu >= 16384 ? kChunkVis / 2 : kChunkVis);
}


// CIP_FFT_PRUNED=0 selects the full 2-D hipFFT transform (A/B experiments)
static bool fft_pruned() {
  static const bool on = [] {
    const char* e = getenv("CIP_FFT_PRUNED");
    return !(e && e[0] == '0');
  }();
  return on;
}

// CIP_GRID_MASK=0: no dirty-tile mask - the grid is zeroed in full before
// every scatter and pass A reads all of it (A/B experiments)
static bool grid_mask() {
  static const bool on = [] {
    const char* e = getenv("CIP_GRID_MASK");
    return !(e && e[0] == '0');
  }();
  return on;
}

// CIP_SCATTER_ORDER=0 skips the bank-class order (A/B experiments)
static bool scatter_order() {
  static const bool on = [] {
    const char* e = getenv("CIP_SCATTER_ORDER");
    return !(e && e[0] == '0');
  }();
  return on;
}

// CIP_PACKED_RUNS=0: ragged runs keep the (row, channel start, channel stop)
// record and the order pass gathers delta[row] per run (A/B experiments)
static bool packed_runs() {
  const char* e = getenv("CIP_PACKED_RUNS");  // read per call (tests switch it)
  return !(e && e[0] == '0');
}

// CIP_RAGGED_PACK=0: ragged ordered-stream entries in the (row << 16) |
// channel form with the delta[row] gather, as for inputs too large to pack
// (tests: the fallback form on small inputs)
static bool ragged_pack() {
  const char* e = getenv("CIP_RAGGED_PACK");  // read per call
  return !(e && e[0] == '0');
}

// CIP_ROW_PHASES=0: the order pass assigns no row phases (cip_grid.hip
// order_kernel; A/B experiments and the phase test)
static bool row_phases() {
  static const bool on = [] {
    const char* e = getenv("CIP_ROW_PHASES");
    return !(e && e[0] == '0');
  }();
  return on;
}

// sub-blocks per radix workgroup: pass 0 (place blocks of ~500 runs) and the
// dense passes (4096 runs)
static int radix_group(int pass) { return pass ? 1 : 8; }

// Also reduces {sum w, max |w V|} into red (device) and returns max |w V| in
// *maxabs (the place pass reads the visibilities anyway).
static int make_plan(Workspace* ws, const double* uvw, const double* fx, const RowMap& m,
                     const void* vis, int vis_dtype, const void* wgt, int wgt_dtype, double* red,
                     const GridGeometry& g, int64_t cv, hipStream_t s, PlanResult* pr, double* maxabs,
                     int group = 1) {
  const int64_t ntiles = g.ntx * g.nty * g.ntw;
  pr->ntiles = ntiles;
  pr->phases = false;
  CIP_ALLOC(tile_runs, int64_t, "tile_runs", ntiles + 1)
  CIP_ALLOC(tile_vis, int64_t, "tile_vis", ntiles + 1)
  CIP_ALLOC(tile_vis_off, int64_t, "tile_vis_off", ntiles + 1)
  CIP_ALLOC(chunk_off, int64_t, "chunk_off", 2 * ntiles + 1)
  CIP_ALLOC(err, unsigned, "err_flag", 1)  // cleared by prepare() before the frequency check
  CIP_ALLOC(scan_tmp, int64_t, "scan_tmp", scan_tmp_elems(ntiles + 1))
  const int64_t nvis = m.nvis;
  const int nblk = plan_place_blocks(nvis);
  // the bank-class order of dense rows stores 32-bit flattened indices (larger
  // inputs grid in plain tile order); ragged row slices store 64-bit
  // (row, channel) entries
  const bool ragged = m.delta != nullptr;
  const bool order = scatter_order() && (ragged || nvis < ((int64_t)1 << 32));
  uint8_t* vis_class = nullptr;
  if (order) {
    vis_class = buf<uint8_t>(ws, "vis_class", nvis);
    if (!vis_class) return CIP_ENOMEM;
  }
  CIP_ALLOC(blk_cnt, int64_t, "blk_cnt", nblk)
  CIP_ALLOC(park_key, uint32_t, "park_key", (int64_t)nblk * 4096)
  CIP_ALLOC(park_run, uint64_t, "park_run", (int64_t)nblk * 4096)
  CIP_ALLOC(partial, double, "prep_partial", 2 * nblk)
  // the place pass also writes radix pass 0's histogram per place block; summed
  // per radix group of g0 blocks, its scan's last entry = runs
  const int g0 = radix_group(0), g1 = radix_group(1);
  const int64_t ng0 = (nblk + g0 - 1) / g0;
  CIP_ALLOC(hist0, int64_t, "radix_hist0", 256 * (int64_t)nblk + 1)
  CIP_ALLOC(hist0g, int64_t, "radix_hist0g", 256 * ng0 + 1)
  CIP_ALLOC(scan_h0, int64_t, "scan_hist0", scan_tmp_elems(256 * ng0 + 1))
  int key_bits = 1;
  while (key_bits < 32 && ((int64_t)1 << key_bits) < ntiles) ++key_bits;
  const int npass = (key_bits + 7) / 8;
  // packed ragged runs (RowMap::pk_runs): the lane scatter's ordered plans
  // whose radix digits stay below the length bits
  RowMap mp = m;
  mp.pk_runs = (ragged && m.pk_cbits && order && g.support <= 16 && 8 * npass <= kRunLenShift && packed_runs()) ? 1 : 0;
  CIP_HIP_CHECK(launch_plan_place(uvw, fx, mp, vis, vis_dtype, wgt, wgt_dtype, g, err, vis_class, blk_cnt, park_key,
                                  park_run, partial, hist0, s));
  CIP_HIP_CHECK(launch_prep_final(partial, nblk, red, s));
  CIP_HIP_CHECK(launch_radix_group_hist(hist0, nblk, g0, hist0g, s));
  CIP_HIP_CHECK(exclusive_scan_i64(hist0g, 256 * ng0 + 1, scan_h0, s));
  int64_t* h = (int64_t*)pinned(ws, 4 * sizeof(int64_t));
  if (!h) return set_error(CIP_ENOMEM, "hipHostMalloc failed");
  CIP_HIP_CHECK(hipMemcpyAsync(&h[0], hist0g + 256 * ng0, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  CIP_HIP_CHECK(hipMemcpyAsync(&h[1], err, sizeof(unsigned), hipMemcpyDeviceToHost, s));
  CIP_HIP_CHECK(hipMemcpyAsync(&h[2], red + 1, sizeof(double), hipMemcpyDeviceToHost, s));
  CIP_HIP_CHECK(hipStreamSynchronize(s));
  const int64_t nruns = h[0];
  const unsigned errbits = (unsigned)h[1];
  std::memcpy(maxabs, &h[2], sizeof(double));
  if (errbits & 4u) return set_error(CIP_EINVAL, "channel frequencies must be positive");
  if (errbits & 2u) return set_error(CIP_EINVAL, "non-finite visibility or weight");
  if (errbits & 1u)
    return set_error(CIP_ERANGE, "non-finite (u, v, w) coordinates, or w outside the w-plane stack");
  pr->nruns = nruns;
  // bucket the runs by tile: stable LSD radix sort, pass 0 from the parked runs
  CIP_ALLOC(key_a, uint32_t, "sort_key_a", nruns)
  CIP_ALLOC(key_b, uint32_t, "sort_key_b", nruns)
  CIP_ALLOC(run_a, uint64_t, "sort_run_a", nruns)
  CIP_ALLOC(run_b, uint64_t, "sort_run_b", nruns)
  const int64_t nbd = radix_blocks(nruns);
  const int64_t ng1 = (nbd + g1 - 1) / g1;
  CIP_ALLOC(hist, int64_t, "radix_hist", 256 * ng1 + 1)
  CIP_ALLOC(scan_h, int64_t, "scan_hist", scan_tmp_elems(256 * ng1 + 1))
  CIP_HIP_CHECK(launch_radix_scatter(park_key, park_run, 0, blk_cnt, nblk, g0, 0, hist0g, key_a, run_a, s));
  uint32_t *kin = key_a, *kout = key_b;
  uint64_t *rin = run_a, *rout = run_b;
  for (int p = 1; p < npass; ++p) {
    CIP_HIP_CHECK(launch_radix_hist(kin, nruns, nullptr, nbd, g1, 8 * p, hist, s));
    CIP_HIP_CHECK(exclusive_scan_i64(hist, 256 * ng1 + 1, scan_h, s));
    CIP_HIP_CHECK(launch_radix_scatter(kin, rin, nruns, nullptr, nbd, g1, 8 * p, hist, kout, rout, s));
    std::swap(kin, kout);
    std::swap(rin, rout);
  }
  uint64_t* runs = rin;
  CIP_HIP_CHECK(launch_tile_offsets(kin, nruns, ntiles, tile_runs, s, mp.pk_runs ? kRunKeyMask : 0xffffffffu));
  const int64_t* tile_run_off = tile_runs;
  CIP_ALLOC(run_goff, int64_t, "run_goff", nruns + 1)
  CIP_ALLOC(scan_tmp2, int64_t, "scan_tmp2", scan_tmp_elems(nruns + 1))
  CIP_HIP_CHECK(scan_run_offsets(runs, nruns, run_goff, scan_tmp2, s, mp.pk_runs ? kin : nullptr));
  CIP_HIP_CHECK(launch_tile_vis(run_goff, tile_run_off, ntiles, tile_vis_off, tile_vis, s));
  if (g.ntx % 32 == 0 && grid_mask()) {
    CIP_ALLOC(dmask, uint8_t, "dirty_mask", g.ntx * g.nty * g.nplanes)
    // tile bits, then tile-row bits (row_bits_kernel), per plane
    CIP_ALLOC(dbits, uint32_t, "dirty_bits", g.ntx * g.nty / 32 * g.nplanes + (g.nty + 31) / 32 * g.nplanes)
    CIP_HIP_CHECK(hipMemsetAsync(dmask, 0, (size_t)(g.ntx * g.nty * g.nplanes), s));
    CIP_HIP_CHECK(launch_dirty_mask(tile_vis, g.ntx, g.nty, g.ntw, g.support, g.nplanes, dmask, dbits, s));
    pr->dmask = dbits;
  }
  // 2-D: the scatter's work units largest first (one tile layer, so the
  // plane's chunk range stays contiguous); w-stacking: per plane, one unit
  // sequence per uv tile over its layers feeding the plane (tile-major keys
  // make that a contiguous range), plane after plane
  const int64_t ntxy = g.ntx * g.nty;
  const bool per_plane = g.do_wstacking != 0;
  pr->group = per_plane ? group : 1;
  const int64_t ngroups = per_plane ? (g.nplanes + group - 1) / group : 1;
  const int64_t nrange = ngroups;  // chunk ranges: per plane group, or the one 2-D layer
  const int full_first = per_plane ? 0 : 1;
  CIP_ALLOC(layer_off, int64_t, "layer_off", nrange + 1)
  int64_t* pc_off = nullptr;
  if (per_plane) {
    const int64_t nentp = ngroups * ntxy;
    pc_off = buf<int64_t>(ws, "plane_chunk_cnt", nentp + 1);
    int64_t* scan_tmpp = buf<int64_t>(ws, "scan_tmp_pchunks", scan_tmp_elems(nentp + 1));
    if (!pc_off || !scan_tmpp) return CIP_ENOMEM;
    CIP_HIP_CHECK(launch_plane_chunk_counts(tile_vis_off, ntxy, g.ntw, ngroups, group, g.support, cv, pc_off, s));
    CIP_HIP_CHECK(exclusive_scan_i64(pc_off, nentp + 1, scan_tmpp, s));
    CIP_HIP_CHECK(launch_gather_i64(pc_off, ntxy, nrange + 1, layer_off, s));
  } else {
    const int64_t nent = full_first ? 2 * ntiles : ntiles;
    CIP_ALLOC(scan_tmpc, int64_t, "scan_tmp_chunks", scan_tmp_elems(2 * ntiles + 1))
    CIP_HIP_CHECK(launch_chunk_counts(tile_vis, ntiles, cv, full_first, chunk_off, s));
    CIP_HIP_CHECK(exclusive_scan_i64(chunk_off, nent + 1, scan_tmpc, s));
    CIP_HIP_CHECK(launch_gather_i64(chunk_off, full_first ? nent : ntiles, nrange + 1, layer_off, s));
  }
  // bank-class ordering windows: the same split with kOrderWindow, per tile key
  CIP_ALLOC(win_off, int64_t, "win_off", ntiles + 1)
  if (order) {
    CIP_HIP_CHECK(launch_chunk_counts(tile_vis, ntiles, kOrderWindow, 0, win_off, s));
    CIP_HIP_CHECK(exclusive_scan_i64(win_off, ntiles + 1, scan_tmp, s));
  }
  int64_t* hl = (int64_t*)pinned(ws, sizeof(int64_t) * (nrange + 2));
  if (!hl) return set_error(CIP_ENOMEM, "hipHostMalloc failed");
  CIP_HIP_CHECK(hipMemcpyAsync(hl, layer_off, sizeof(int64_t) * (nrange + 1), hipMemcpyDeviceToHost, s));
  if (order) CIP_HIP_CHECK(hipMemcpyAsync(hl + nrange + 1, win_off + ntiles, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  CIP_HIP_CHECK(hipStreamSynchronize(s));
  pr->plane_chunk_off.assign(hl, hl + nrange + 1);
  const int64_t nwin = order ? hl[nrange + 1] : 0;
  pr->nchunks = pr->plane_chunk_off.back();
  CIP_ALLOC(chunks, Chunk, "chunks", pr->nchunks)
  if (per_plane)
    CIP_HIP_CHECK(launch_plane_chunk_emit(tile_vis_off, pc_off, run_goff, tile_runs, ntxy, g.ntw, ngroups, group,
                                          g.support, cv, pr->nchunks, chunks, s));
  else
    CIP_HIP_CHECK(launch_chunk_emit(tile_vis_off, tile_vis, chunk_off, run_goff, tile_runs, ntiles, cv, full_first,
                                    pr->nchunks, chunks, s));
  pr->runs = runs;
  pr->run_goff = run_goff;
  pr->tile_run_off = tile_runs;
  pr->chunks = chunks;
  if (order && nwin > 0) {
    CIP_ALLOC(windows, Chunk, "windows", nwin)
    CIP_HIP_CHECK(launch_chunk_emit(tile_vis_off, tile_vis, win_off, run_goff, tile_runs, ntiles, kOrderWindow, 0, nwin,
                                    windows, s));
    CIP_ALLOC(perm, uint32_t, "perm", ragged ? 2 * nvis : nvis)
    const bool ph = row_phases() && order_phases_ok(mp, g.support);
    CIP_HIP_CHECK(launch_order(vis_class, mp, runs, run_goff, windows, nwin, perm, s, ph ? g.support : 0));
    pr->phases = ph;
    pr->perm = perm;
  }
  return CIP_OK;
}

// the internal raw linear-feed code is reached through cip_ms2dirty_stokes_i only
static bool public_dtypes(int vis_dtype, int wgt_dtype) {
  return vis_dtype != CIP_POL4I && wgt_dtype != CIP_POL4I;
}
static bool vis_dtype_ok(int d) { return d == CIP_C64 || d == CIP_C128 || d == CIP_POL4I; }
static bool wgt_dtype_ok(int d) { return d == CIP_NONE || d == CIP_F32 || d == CIP_F64 || d == CIP_POL4I; }

// w planes per scatter work unit in w-stacking mode: G = 3 (a visibility
// placed and its u, v, w kernels evaluated once for three planes; the unit
// holds G sub-grids in 512-thread blocks), fewer where two such blocks would
// not fit a CU's LDS (W >= 10: 2); the packed class's 8-byte cells allow up to
// 7 (round 5); CIP_WSTACK_GROUP=1..7 caps it (tests compare the groups with
// G = 1); the large supports always 1. Refcall C3 (round 3, fp64 taps): G = 1
// / 2 / 3 -> 13.4 / 12.2 / 11.8 ms of scatter (profiles/r03_ab_wstack_group*.txt).
// One 14-plane group per CU (W = 6) measured slower: 6.94 -> 8.34 ms
// (profiles/r05at_ab_wstack_g14.txt).
static int wstack_group(const GridGeometry& g, bool packed) {
  static const int env = [] {
    const char* e = getenv("CIP_WSTACK_GROUP");
    const int v = e ? atoi(e) : 0;
    return v < 0 ? 0 : (v > 7 ? 7 : v);
  }();
  if (!g.do_wstacking || g.support > 16 || g.nplanes < 2) return 1;
  const int64_t P = kTile + g.support - 1;
  if (packed) {
    // 8-byte cells: up to 7 sub-grids in one 512-thread block, two blocks per
    // CU (<= 80 KB of static LDS each; cip_scatter.h kFitG7 .. kFitG4). Round
    // 5: G = 7 at W = 6 (the reference call: 14 planes in two groups, a
    // visibility visits 1.6 groups instead of 2) scatter 7.15 -> 6.93 ms,
    // call 7.35 -> 7.51-7.54 Gvis/s (profiles/r05ah_ab_wstack_group.txt)
    int G = env ? env : 7;
    while (G > 5 && G <= 7 && G * P * P * 8 + 4200 > 81920) --G;
    while (G > 3 && G <= 5 && G * P * P * 8 + 4200 > 65536) --G;
    return G;
  }
  // two 512-thread blocks per CU must fit their G sub-grids in 160 KB of LDS
  const int64_t per_plane = P * P * 16;
  int G = env ? (env > 3 ? 3 : env) : 3;
  while (G > 1 && 2 * G * per_plane > 160 * 1024) --G;
  return G;
}

static bool grid_is_transposed(const GridGeometry& g, int64_t npix_x, int64_t npix_y);
static bool grid_f32_enabled();

struct Prepared {
  cip_gridder_params p;
  GridGeometry g;
  double fixed_scale;
  bool packed;  // single-precision class (CIP_ACC_SINGLE)
  double* fx;
  double* red;  // device [sum_w, max|wV|]
  RowMap m;     // (row, channel) -> visibility index
  PlanResult plan;
};

// Row slices of the ragged (tile) input layout: row r holds channels
// [chan_start[r], chan_stop[r]) and the visibilities are concatenated in row
// order (reference uvw_tiling/tile.py:83-115), nvis in total.
struct RaggedRows {
  const int32_t* chan_start;
  const int32_t* chan_stop;
  int64_t nvis;
};

static int prepare(Workspace* ws, const double* uvw, int64_t nrow, const double* freq, int64_t nchan,
                   const void* vis, int vis_dtype, const void* wgt, int wgt_dtype, int64_t npix_x, int64_t npix_y,
                   double px, double py, double epsilon, int support, int do_wstacking, bool packed,
                   const cip_gridder_params* given, hipStream_t s, Prepared* out, double** grid_out = nullptr,
                   const RaggedRows* ragged = nullptr, bool reuse = false, const uint8_t* flags4 = nullptr,
                   bool want_group = true, int64_t plane_begin = 0, int64_t plane_end = -1) {
  if (!ws->parity_scope) ws->plan_unscoped = true;
  if (!vis_dtype_ok(vis_dtype)) return set_error(CIP_EINVAL, "vis dtype must be complex64 or complex128");
  if (!wgt_dtype_ok(wgt_dtype)) return set_error(CIP_EINVAL, "wgt dtype must be float32, float64 or none");
  if (wgt == nullptr) wgt_dtype = CIP_NONE;
  // raw linear-feed columns: visibilities and weights come as one (internal) pair
  if ((vis_dtype == CIP_POL4I) != (wgt_dtype == CIP_POL4I))
    return set_error(CIP_EINVAL, "raw linear-feed visibilities need their raw weights");
  if (nrow < 0 || nchan < 1 || nchan > 65535) return set_error(CIP_EINVAL, "need 1 <= nchan <= 65535, nrow >= 0");
  if (nrow >= ((int64_t)1 << 32)) return set_error(CIP_EINVAL, "nrow must be < 2^32");
  CIP_ALLOC(fx, double, "fx", nchan)
  CIP_ALLOC(red, double, "red", 4)
  // the planner's error bits: cleared here, read back with the run count
  CIP_ALLOC(err, unsigned, "err_flag", 1)
  CIP_HIP_CHECK(hipMemsetAsync(err, 0, sizeof(unsigned), s));
  CIP_HIP_CHECK(launch_freq_scale(freq, nchan, fx, err, s));
  // the frequency range on the host only where the w range needs it (the
  // positivity check otherwise travels as error bit 2 to the planner's
  // readback: one host synchronisation less per 2-D call)
  const bool host_fx = nrow == 0 || (do_wstacking && given == nullptr);
  double fxmin = 0.0, fxmax = 0.0;
  if (host_fx) {
    double* h = (double*)pinned(ws, sizeof(double) * (4 + (size_t)nchan));
    if (!h) return set_error(CIP_ENOMEM, "hipHostMalloc failed");
    CIP_HIP_CHECK(hipMemcpyAsync(h + 4, fx, sizeof(double) * nchan, hipMemcpyDeviceToHost, s));
    CIP_HIP_CHECK(hipStreamSynchronize(s));
    fxmin = h[4];
    fxmax = h[4];
    for (int64_t c = 1; c < nchan; ++c) {
      fxmin = std::fmin(fxmin, h[4 + c]);
      fxmax = std::fmax(fxmax, h[4 + c]);
    }
    if (!(fxmin > 0.0) || !std::isfinite(fxmax)) return set_error(CIP_EINVAL, "channel frequencies must be positive");
  }
  RowMap& m = out->m;
  m.nchan = nchan;
  m.inv_nchan = 1.0 / (double)nchan;
  m.delta = nullptr;
  m.off = nullptr;
  m.seg_row = nullptr;
  m.nrow = 0;
  m.pk_cbits = m.pk_rbits = 0;
  m.flags4 = vis_dtype == CIP_POL4I ? flags4 : nullptr;
  m.nvis = nrow * nchan;
  if (ragged) {
    if (ragged->nvis < 0 || ragged->nvis >= ((int64_t)1 << 40)) return set_error(CIP_EINVAL, "bad visibility count");
    m.nvis = ragged->nvis;
    if (nrow > 0) {
      int64_t* off = buf<int64_t>(ws, "ragged_off", nrow + 1);
      int64_t* delta = buf<int64_t>(ws, "ragged_delta", nrow);
      uint32_t* seg_row = buf<uint32_t>(ws, "ragged_seg_row", (ragged->nvis + 63) / 64 + 1);
      int64_t* scan_tmp = buf<int64_t>(ws, "ragged_scan", scan_tmp_elems(nrow + 1));
      unsigned* rerr = buf<unsigned>(ws, "ragged_err", 1);
      if (!off || !delta || !seg_row || !scan_tmp || !rerr) return CIP_ENOMEM;
      CIP_HIP_CHECK(hipMemsetAsync(rerr, 0, sizeof(unsigned), s));
      CIP_HIP_CHECK(launch_ragged_lengths(ragged->chan_start, ragged->chan_stop, nrow, nchan, off, rerr, s));
      CIP_HIP_CHECK(exclusive_scan_i64(off, nrow + 1, scan_tmp, s));
      int64_t* hr = (int64_t*)pinned(ws, 2 * sizeof(int64_t));
      if (!hr) return set_error(CIP_ENOMEM, "hipHostMalloc failed");
      CIP_HIP_CHECK(hipMemcpyAsync(&hr[0], off + nrow, sizeof(int64_t), hipMemcpyDeviceToHost, s));
      CIP_HIP_CHECK(hipMemcpyAsync(&hr[1], rerr, sizeof(unsigned), hipMemcpyDeviceToHost, s));
      CIP_HIP_CHECK(hipStreamSynchronize(s));
      if ((unsigned)hr[1] != 0u) return set_error(CIP_EINVAL, "row slice channel range outside [0, nchan)");
      if (hr[0] != ragged->nvis) return set_error(CIP_EINVAL, "visibility count differs from the row slices' total");
      CIP_HIP_CHECK(launch_ragged_expand(off, ragged->chan_start, nrow, delta, seg_row, s));
      m.delta = delta;
      m.off = off;
      m.seg_row = seg_row;
      m.nrow = nrow;
      // ordered-stream entries (index, row, channel) when they fit 64 bits
      auto bits = [](int64_t n) {
        int b = 1;
        while (b < 62 && ((int64_t)1 << b) < n) ++b;
        return b;
      };
      const int cb = bits(nchan), rb = bits(nrow), ib = bits(ragged->nvis);
      if (cb + rb + ib <= 64 && ragged_pack()) {
        m.pk_cbits = cb;
        m.pk_rbits = rb;
      }
    }
  }
  // CIP_REUSE_PLAN: the previous plan, if it was made for this geometry (its
  // parameters then also stand in for the w range: same uvw by the caller's
  // promise)
  const std::vector<double> key = {(double)nrow, (double)nchan, (double)npix_x, (double)npix_y, px, py, epsilon,
                                   (double)support, (double)do_wstacking, (double)packed,
                                   given ? 1.0 : 0.0, want_group ? 1.0 : 0.0, (double)plane_begin,
                                   (double)plane_end};
  const bool reusing = reuse && !ragged && given == nullptr && ws->saved_valid && ws->saved_key == key;
  if (reusing) given = &ws->saved_p;
  double wmin = 0.0, wmax = 0.0;
  if (do_wstacking && nrow > 0 && given == nullptr) {
    const int nb = 256;
    CIP_ALLOC(wpart, double, "w_partial", 2 * nb)
    CIP_HIP_CHECK(launch_w_range(uvw, nrow, fxmin, fxmax, wpart, nb, s));
    double* hw = (double*)pinned(ws, sizeof(double) * 2 * nb);
    if (!hw) return set_error(CIP_ENOMEM, "hipHostMalloc failed");
    CIP_HIP_CHECK(hipMemcpyAsync(hw, wpart, sizeof(double) * 2 * nb, hipMemcpyDeviceToHost, s));
    CIP_HIP_CHECK(hipStreamSynchronize(s));
    wmin = INFINITY;
    wmax = -INFINITY;
    for (int i = 0; i < nb; ++i) {
      wmin = std::fmin(wmin, hw[2 * i]);
      wmax = std::fmax(wmax, hw[2 * i + 1]);
    }
  }
  if (given) {
    out->p = *given;
  } else {
    const int rc = choose(npix_x, npix_y, px, py, epsilon, support, do_wstacking, wmin, wmax, &out->p);
    if (rc != CIP_OK) return rc;
  }
  out->g = geometry(out->p, px, py);
  if (plane_end >= 0) {
    // a range of the w-plane stack (cip_ms2dirty_wplanes)
    if (plane_begin < 0 || plane_begin > plane_end || plane_end > out->p.nplanes)
      return set_error(CIP_EINVAL, "w-plane range outside [0, nplanes]");
    out->g.plane_lo = plane_begin;
    out->g.plane_hi = plane_end;
  }
  // tile keys are 32-bit ((iy0 / T) ntx + ix0 / T) ntw + iw0 (cip_plan.hip):
  // a larger key space would wrap and mis-sort the runs
  if ((double)out->g.ntx * (double)out->g.nty * (double)out->g.ntw >= 4294967295.0)
    return set_error(CIP_EINVAL, "grid tiles x w layers exceed the 32-bit tile key space");
  if (packed && vis_dtype != CIP_C64 && vis_dtype != CIP_POL4I)
    return set_error(CIP_EINVAL, "single-precision accumulation needs complex64 visibilities");
  if (packed && out->g.support > 16)
    return set_error(CIP_EINVAL, "single-precision accumulation supports kernel supports <= 16");
  out->packed = packed;
  out->fixed_scale = 1.0;
  out->fx = fx;
  out->red = red;
  if (grid_out) {
    // the grid is known now: zero its first plane group beside the planner
    // (complex64 cells for the packed class on the pruned-FFT path, as
    // ms2dirty_impl lays them out)
    const int64_t gplanes = want_group ? wstack_group(out->g, packed) : 1;
    const bool f32 = packed && grid_is_transposed(out->g, npix_x, npix_y) && grid_f32_enabled();
    const size_t gbytes = (f32 ? sizeof(float) : sizeof(double)) * 2 * out->g.nu * out->g.nv * gplanes;
    double* grid = buf<double>(ws, "grid", 2 * out->g.nu * out->g.nv * gplanes);
    if (!grid) return CIP_ENOMEM;
    if (ws->grid_clean != grid || ws->grid_clean_bytes < gbytes) {
      const int zr = zero_on_side(ws, grid, gbytes, s);
      if (zr != CIP_OK) return zr;
    }
    *grid_out = grid;
  }
  hipEvent_t e_prep = g_prof.mark(s);
  g_prof.span(0, g_prof.pool.empty() ? nullptr : g_prof.pool[0], e_prep);
  if (nrow == 0) {
    CIP_HIP_CHECK(hipMemsetAsync(red, 0, 2 * sizeof(double), s));
    out->plan = PlanResult();
    out->plan.plane_chunk_off.assign((out->g.do_wstacking ? out->g.nplanes : 1) + 1, 0);  // group 1
    return CIP_OK;
  }
  double maxabs = 0.0;
  if (m.nvis == 0) {
    CIP_HIP_CHECK(hipMemsetAsync(red, 0, 2 * sizeof(double), s));
    out->plan = PlanResult();
    out->plan.plane_chunk_off.assign((out->g.do_wstacking ? out->g.nplanes : 1) + 1, 0);  // group 1
    return CIP_OK;
  }
  int rc;
  if (reusing) {
    // the plan's buffers are read-only here; only the weight reduction runs
    const int nblk = plan_place_blocks(m.nvis);
    CIP_ALLOC(partial, double, "prep_partial_reuse", 2 * nblk)
    CIP_HIP_CHECK(launch_prep_reduce(m, vis, vis_dtype, wgt, wgt_dtype, out->g, err, partial, s));
    CIP_HIP_CHECK(launch_prep_final(partial, nblk, red, s));
    unsigned* h = (unsigned*)pinned(ws, 4 * sizeof(double));
    if (!h) return set_error(CIP_ENOMEM, "hipHostMalloc failed");
    CIP_HIP_CHECK(hipMemcpyAsync(h, err, sizeof(unsigned), hipMemcpyDeviceToHost, s));
    CIP_HIP_CHECK(hipMemcpyAsync((double*)h + 1, red + 1, sizeof(double), hipMemcpyDeviceToHost, s));
    CIP_HIP_CHECK(hipStreamSynchronize(s));
    const unsigned errbits = h[0];
    std::memcpy(&maxabs, (double*)h + 1, sizeof(double));
    if (errbits & 4u) return set_error(CIP_EINVAL, "channel frequencies must be positive");
    if (errbits & 2u) return set_error(CIP_EINVAL, "non-finite visibility or weight");
    out->plan = ws->saved_plan;
    rc = CIP_OK;
  } else {
    ws->saved_valid = false;
    rc = make_plan(ws, uvw, fx, m, vis, vis_dtype, wgt, wgt_dtype, red, out->g, chunk_vis(packed, out->g.nu), s,
                   &out->plan, &maxabs, want_group ? wstack_group(out->g, packed) : 1);
    if (rc == CIP_OK && !ragged) {
      ws->saved_key = key;
      ws->saved_p = out->p;
      ws->saved_plan = out->plan;
      ws->saved_valid = true;
    }
  }
  g_prof.span(1, e_prep, g_prof.mark(s));
  if (rc != CIP_OK) return rc;
  if (!std::isfinite(maxabs)) return set_error(CIP_EINVAL, "non-finite visibility or weight");
  // fixed point: max contribution <= 2^kFixedBits, or 2^kPackedBits for a
  // full packed chunk (the scatter raises it for shorter chunks)
  int e2 = 0;
  if (maxabs > 0.0) std::frexp(maxabs, &e2);  // maxabs < 2^e2
  out->fixed_scale = std::ldexp(1.0, (packed ? kPackedBits : kFixedBits) - e2);
  g_prof.counts[0] = m.nvis;
  g_prof.counts[1] = out->plan.nruns;
  g_prof.counts[2] = out->plan.nchunks;
  g_prof.counts[3] = out->g.nplanes;
  return rc;
}

// Work-unit range q of the plan (w-stacking: plane group q = planes
// [q G, q G + G), written to grid + k planes for plane q G + k; 2-D: q = 0).
// transposed: store the grid as gT[y, x] (input layout of the pruned FFT)
// zeroed: the group's planes were zeroed already (side stream, joined by the caller)
// Sole-unit private-cell stores in the scatter's flush (cip_scatter.h) on grid
// planes of >= 16384^2 cells: C4's flush goes to a 4 GiB plane that no cache
// holds, and stores cut the C4-shard scatter 4.87 -> 4.59 ms; on C3's 8192^2
// plane they cost 1-3 % (profiles/r03_ab_flush_store.txt). CIP_FLUSH_STORE=0 /
// 1 forces them off / on for any grid (A/B).
static bool flush_store_enabled(const GridGeometry& g) {
  static const int mode = [] {
    const char* e = getenv("CIP_FLUSH_STORE");
    return e ? (std::strcmp(e, "0") == 0 ? 0 : 1) : -1;
  }();
  return mode < 0 ? g.nu * g.nv >= ((int64_t)1 << 28) : mode == 1;
}

// zeroed: the planes are already zero (no memset); accumulate: they hold
// earlier chunks' sums (cip_grid_ms: += onto them), so the flush never stores
static int scatter_plane(const Prepared& pp, int64_t q, const double* uvw, const void* vis, int vis_dtype,
                         const void* wgt, int wgt_dtype, bool transposed, double* grid,
                         hipStream_t s, bool zeroed = false, bool share_cus = false, bool accumulate = false) {
  GridGeometry g = pp.g;
  g.transposed = transposed ? 1 : 0;
  const int G = pp.plan.group;
  const int64_t p0 = g.do_wstacking ? q * G : 0;
  const int64_t np = g.do_wstacking ? std::min<int64_t>(G, g.nplanes - p0) : 1;
  if (!zeroed)
    CIP_HIP_CHECK(hipMemsetAsync(grid, 0, (g.grid_f32 ? sizeof(float) : sizeof(double)) * 2 * g.nu * g.nv * np, s));
  if (pp.plan.nchunks == 0) return CIP_OK;
  const int64_t k = g.do_wstacking ? q : 0;
  const int64_t cb = pp.plan.plane_chunk_off[k], ce = pp.plan.plane_chunk_off[k + 1];
  if (wgt == nullptr) wgt_dtype = CIP_NONE;
  hipEvent_t a = g_prof.mark(s);
  RowMap ms = pp.m;
  ms.row_phase = pp.plan.phases ? 1 : 0;
  CIP_HIP_CHECK(launch_scatter(g.support, vis_dtype, wgt_dtype, pp.packed, G, share_cus,
                               !accumulate && flush_store_enabled(g), uvw, pp.fx, vis, wgt, ms,
                               pp.plan.runs, pp.plan.run_goff, pp.plan.tile_run_off, pp.plan.perm, pp.plan.chunks, cb,
                               ce - cb, g, p0, pp.fixed_scale, grid, s));
  g_prof.span(2, a, g_prof.mark(s));
  if (ce > cb) g_prof.counts[4] += 1;
  return CIP_OK;
}

// ------------------------------------------- grid -> dirty image (shared) ----
// Correction vectors, FFT plan / twiddles and the pass-A buffer for one
// (grid, image) geometry; then per plane: FFT + crop/correct (2-D) or the
// w-screen accumulation, and the final w-stacking correction.
struct DirtyStage {
  int64_t npix_x = 0, npix_y = 0;
  double px = 0, py = 0;
  bool fast = false;
  hipfftHandle plan = nullptr;
  double *tw_u = nullptr, *tw_v = nullptr, *fft_h = nullptr, *cx = nullptr, *cy = nullptr;
};

// the HBM layout of the uv grid the FFT stage expects: gT[y, x] when the
// pruned FFT runs
static bool grid_is_transposed(const GridGeometry& g, int64_t npix_x, int64_t npix_y) {
  return fft_pruned() && fast_fft_supported(g.nu, g.nv, npix_x, npix_y);
}

// the grid-correction vectors cx = 1 / F(p / nu), cy = 1 / F(q / nv) (cached
// per workspace and geometry)
static int correction_vectors(Workspace* ws, const GridGeometry& g, int64_t npix_x, int64_t npix_y, hipStream_t s,
                              double** cx_out, double** cy_out) {
  CIP_ALLOC(cx, double, "cx", npix_x)
  CIP_ALLOC(cy, double, "cy", npix_y)
  *cx_out = cx;
  *cy_out = cy;
  HostKernel hk;
  host_kernel(g.support, &hk);
  KernelFT F(hk);
  // the correction vectors depend only on (npix, grid, W): cache them per device
  const std::vector<int64_t> corr_key = {npix_x, npix_y, g.nu, g.nv, g.support};
  if (ws->corr_key != corr_key) {
    ws->corr_key.clear();
    std::vector<double> hx(npix_x), hy(npix_y);
    for (int64_t i = 0; i < npix_x; ++i) hx[i] = 1.0 / F((double)(i - npix_x / 2) / (double)g.nu);
    for (int64_t j = 0; j < npix_y; ++j) hy[j] = 1.0 / F((double)(j - npix_y / 2) / (double)g.nv);
    CIP_HIP_CHECK(hipMemcpyAsync(cx, hx.data(), sizeof(double) * npix_x, hipMemcpyHostToDevice, s));
    CIP_HIP_CHECK(hipMemcpyAsync(cy, hy.data(), sizeof(double) * npix_y, hipMemcpyHostToDevice, s));
    CIP_HIP_CHECK(hipStreamSynchronize(s));  // host vectors go out of scope
    ws->corr_key = corr_key;
  }
  return CIP_OK;
}

// CIP_GRID_F32=0: the packed class keeps complex128 grid planes (A/B)
static bool grid_f32_enabled() {
  static const bool on = [] {
    const char* e = getenv("CIP_GRID_F32");
    return !(e && e[0] == '0');
  }();
  return on;
}

// CIP_WACC_F32=0: the packed class's w planes accumulate in the fp64 image
// (A/B); default: a float accumulator
static bool wacc_f32_enabled() {
  static const bool on = [] {
    const char* e = getenv("CIP_WACC_F32");
    return !(e && e[0] == '0');
  }();
  return on;
}

static int dirty_stage(Workspace* ws, const GridGeometry& g, int64_t npix_x, int64_t npix_y, double px, double py,
                       hipStream_t s, DirtyStage* st) {
  st->npix_x = npix_x;
  st->npix_y = npix_y;
  st->px = px;
  st->py = py;
  if (const int rc = correction_vectors(ws, g, npix_x, npix_y, s, &st->cx, &st->cy); rc != CIP_OK) return rc;
  // pruned FFT (cip_fft.hip) for power-of-two grids; hipFFT 2-D otherwise
  // (CIP_FFT_PRUNED=0 forces the latter)
  st->fast = grid_is_transposed(g, npix_x, npix_y);
  if (st->fast) {
    int rc = fft_twiddles(ws, g.nu, s, &st->tw_u);
    if (rc != CIP_OK) return rc;
    rc = fft_twiddles(ws, g.nv, s, &st->tw_v);
    if (rc != CIP_OK) return rc;
    st->fft_h = buf<double>(ws, "fft_pass_a", 2 * npix_x * g.nv);
    if (!st->fft_h) return CIP_ENOMEM;
  } else {
    const int rc = fft_plan(ws, g.nu, g.nv, s, &st->plan);
    if (rc != CIP_OK) return rc;
  }
  return CIP_OK;
}

// plane p's grid (consumed: the hipFFT path transforms it in place) into
// dirty_out (overwritten for p == 0, accumulated after it)
// dmask (pruned FFT only, may be NULL): the grid tiles the scatter wrote; the
// rest of the grid is zero, and pass A zeroes the masked tiles after reading
// norm (pruned 2-D path only, may be NULL): device weight sum the image is
// divided by in pass B's epilogue (CIP_NORMALISE)
// CIP_FFT_ROWSKIP=0: pass A transforms (and pass B reads) clean tile rows too (A/B)
static bool fft_rowskip() {
  static const bool on = [] {
    const char* e = getenv("CIP_FFT_ROWSKIP");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  return on;
}

// rowbits (with dmask): the plane's tile-row bits (row_bits_kernel)
// acc_f32: dirty_out is the packed class's float plane accumulator
static int plane_to_dirty(const DirtyStage& st, const GridGeometry& g, int64_t p, double* grid, double* dirty_out,
                          hipStream_t s, const uint32_t* dmask = nullptr, const double* norm = nullptr,
                          const uint32_t* rowbits = nullptr, int first = -1, bool acc_f32 = false) {
  if (first < 0) first = p == 0;  // the first plane overwrites the image, later ones add
  hipEvent_t f0 = g_prof.mark(s);
  // 16384-point fp64 columns of a 2-D image: pass B by even / odd halves
  // (cip_fft.hip fft_cols_eo_kernel), pass A writing H in that order
  const bool eo = st.fast && fft_cols_eo(g.nv, st.npix_y, g.grid_f32 != 0, g.do_wstacking ? 1 : 0);
  if (st.fast) {
    if (!fft_rowskip()) rowbits = nullptr;
    CIP_HIP_CHECK(launch_fft_rows(grid, g.nu, g.nv, st.npix_x, st.tw_u, st.fft_h, dmask, g.ntx, rowbits != nullptr, s,
                                  g.grid_f32 != 0, eo));
  } else if (hipfftExecZ2Z(st.plan, (hipfftDoubleComplex*)grid, (hipfftDoubleComplex*)grid, HIPFFT_BACKWARD) !=
             HIPFFT_SUCCESS) {
    return set_error(CIP_EHIP, "hipfftExecZ2Z failed");
  }
  const double w_plane = g.w0 + (double)p * g.dw;
  // pass B carries the crop epilogue: it is booked under "fft"
  if (st.fast)
    CIP_HIP_CHECK(launch_fft_cols(st.fft_h, g.nv, st.npix_x, st.npix_y, st.tw_v, g.do_wstacking ? 1 : 0, dirty_out,
                                  st.cx, st.cy, st.px, st.py, w_plane, first, g.do_wstacking ? nullptr : norm,
                                  dmask ? rowbits : nullptr, s, g.grid_f32 != 0, acc_f32, eo));
  hipEvent_t f1 = g_prof.mark(s);
  g_prof.span(3, f0, f1);
  if (st.fast) {
  } else if (g.do_wstacking) {
    CIP_HIP_CHECK(launch_wplane_accumulate(grid, g, st.npix_x, st.npix_y, st.px, st.py, w_plane, first, dirty_out,
                                           s));
  } else {
    CIP_HIP_CHECK(launch_crop_correct_2d(grid, g, st.npix_x, st.npix_y, st.cx, st.cy, dirty_out, s));
  }
  g_prof.span(4, f1, g_prof.mark(s));
  return CIP_OK;
}

// after the last plane: the w-stacking correction (2-D: nothing)
// the w-stacking final correction's table of F (cached per workspace)
static int w_correction_table(Workspace* ws, const cip_gridder_params& prm, const GridGeometry& g, hipStream_t s,
                              double** table, int64_t* n, double* dnu_out) {
  HostKernel hk;
  host_kernel(g.support, &hk);
  KernelFT F(hk);
  const int64_t fw_n = 4100;
  const double numax = g.dw * std::fabs(prm.nmin);
  const double dnu = (numax > 0 ? numax : 1e-3) * 1.0001 / 4096.0;
  CIP_ALLOC(fwd, double, "fw_table", fw_n)
  const std::vector<double> fw_key = {(double)g.support, numax};
  if (ws->fw_key != fw_key) {
    ws->fw_key.clear();
    std::vector<double> fw(fw_n);
    for (int64_t k = 0; k < fw_n; ++k) fw[k] = F((double)k * dnu);
    CIP_HIP_CHECK(hipMemcpyAsync(fwd, fw.data(), sizeof(double) * fw_n, hipMemcpyHostToDevice, s));
    CIP_HIP_CHECK(hipStreamSynchronize(s));
    ws->fw_key = fw_key;
  }
  *table = fwd;
  *n = fw_n;
  *dnu_out = dnu;
  return CIP_OK;
}

static int finish_dirty(Workspace* ws, const DirtyStage& st, const cip_gridder_params& prm, const GridGeometry& g,
                        double* dirty_out, hipStream_t s, const float* acc_f32 = nullptr) {
  if (!g.do_wstacking) return CIP_OK;
  double* fwd = nullptr;
  int64_t fw_n = 0;
  double dnu = 0.0;
  if (const int rc = w_correction_table(ws, prm, g, s, &fwd, &fw_n, &dnu); rc != CIP_OK) return rc;
  CIP_HIP_CHECK(launch_wfinal_correct(dirty_out, st.npix_x, st.npix_y, st.px, st.py, st.cx, st.cy, fwd, fw_n, dnu,
                                      g.dw, s, 0, -1, nullptr, acc_f32));
  return CIP_OK;
}

// Grid visibilities (dense MS rows, or ragged row slices) onto nplanes
// resident accumulator planes (no zeroing: += onto what they hold), and add
// their weight sum to *sum_wgt.
static int grid_accumulate(const double* uvw, int64_t nrow, const double* freq, int64_t nchan, const void* vis,
                           int vis_dtype, const void* wgt, int wgt_dtype, const cip_gridder_params* params,
                           double pixsize_x, double pixsize_y, int64_t npix_x, int64_t npix_y, int flags,
                           void* hip_stream, double* grids, double* sum_wgt, const RaggedRows* ragged,
                           const uint8_t* flags4 = nullptr, int64_t row0 = 0, int64_t nrows = 0,
                           uint32_t* strip_bits = nullptr) {
  g_last_error.clear();
  if (flags & ~(CIP_ACC_SINGLE | CIP_PSF | CIP_GRID_ZEROED)) return set_error(CIP_EINVAL, "unknown flags");
  if (!params || !grids) return set_error(CIP_EINVAL, "NULL params or grids");
  // the flush's private-cell stores (CIP_GRID_ZEROED) write 16-byte cells:
  // planes that are only 8-byte aligned take the atomic path instead
  if (((uintptr_t)grids & 15u) != 0u) flags &= ~CIP_GRID_ZEROED;
  if (flags & CIP_PSF) {
    vis = nullptr;
    if (vis_dtype != CIP_POL4I) vis_dtype = CIP_C64;
  }
  if (nrow > 0 && (!uvw || !freq || (!vis && !(flags & CIP_PSF)))) return set_error(CIP_EINVAL, "NULL input pointer");
  hipStream_t s = (hipStream_t)hip_stream;
  Workspace* ws = workspace();
  if (!ws) return set_error(CIP_EHIP, "no HIP device");
  if (const int sr = settle_async(ws, s); sr != CIP_OK) return sr;
  g_prof.reset();
  hipEvent_t t_start = g_prof.mark(s);
  Prepared pp;
  int rc = prepare(ws, uvw, nrow, freq, nchan, vis, vis_dtype, wgt, wgt_dtype, 2, 2, pixsize_x, pixsize_y, 0.0,
                   params->support, params->do_wstacking, (flags & CIP_ACC_SINGLE) != 0, params, s, &pp, nullptr,
                   ragged, false, flags4);
  if (rc != CIP_OK) return rc;
  const bool transposed = grid_is_transposed(pp.g, npix_x, npix_y);
  unsigned* oob = nullptr;
  if (nrows > 0) {
    // a strip's row window (cip_grid_tiles_strip): rows [row0, row0 + nrows) mod nv
    if (!transposed) return set_error(CIP_EINVAL, "strip buffers need the pruned-FFT grid layout");
    if (row0 < 0 || row0 >= pp.g.nv || nrows > pp.g.nv) return set_error(CIP_EINVAL, "strip rows outside the grid");
    oob = buf<unsigned>(ws, "strip_oob", 1);
    if (!oob) return CIP_ENOMEM;
    CIP_HIP_CHECK(hipMemsetAsync(oob, 0, sizeof(unsigned), s));
    pp.g.row0 = row0;
    pp.g.rows = nrows;
    pp.g.oob = oob;
  }
  uint32_t* wmask = nullptr;
  if (strip_bits) {
    // the strip's dirty-tile bits for its masked pass A: the tiles this
    // call's flush writes (GridGeometry::wmask, exact) + the tile rows
    // receiving the previous rank's halo (after the scatter, below)
    if (pp.g.ntx % 32 != 0) return set_error(CIP_EINVAL, "tile masks need nu / 32 to be a multiple of 32 tiles");
    const int64_t words = pp.g.nplanes * pp.g.nty * (pp.g.ntx / 32);
    wmask = buf<uint32_t>(ws, "strip_wmask", words);
    if (!wmask) return CIP_ENOMEM;
    CIP_HIP_CHECK(hipMemsetAsync(wmask, 0, sizeof(uint32_t) * words, s));
    pp.g.wmask = wmask;
  }
  const GridGeometry& g = pp.g;
  const int64_t plane_elems = 2 * g.nu * g.rows;
  const int G = pp.plan.group;
  for (int64_t q = 0; q * G < g.nplanes; ++q) {
    rc = scatter_plane(pp, q, uvw, vis, vis_dtype, wgt, wgt_dtype, transposed, grids + q * G * plane_elems, s, true,
                       false, (flags & CIP_GRID_ZEROED) == 0);
    if (rc != CIP_OK) return rc;
  }
  if (sum_wgt) CIP_HIP_CHECK(launch_add_scalar(pp.red, sum_wgt, s));
  if (strip_bits) CIP_HIP_CHECK(launch_strip_mask(wmask, g, row0, g.support - 1, strip_bits, s));
  g_prof.span(5, t_start, g_prof.mark(s));
  unsigned* h_oob = nullptr;
  if (oob) {
    h_oob = (unsigned*)pinned(ws, sizeof(unsigned));
    if (!h_oob) return set_error(CIP_ENOMEM, "hipHostMalloc failed");
    CIP_HIP_CHECK(hipMemcpyAsync(h_oob, oob, sizeof(unsigned), hipMemcpyDeviceToHost, s));
  }
  CIP_HIP_CHECK(hipStreamSynchronize(s));
  g_prof.finish();
  if (h_oob && *h_oob != 0u)
    return set_error(CIP_ERANGE, "a visibility's footprint leaves the strip's rows (cells dropped)");
  return CIP_OK;
}

}  // namespace cip

using namespace cip;

extern "C" {

const char* cip_last_error(void) { return g_last_error.c_str(); }

const char* cip_build_info(void) { return "libcip_hip gfx950 (CDNA4) v0.1.0"; }

int cip_choose_params(int64_t npix_x, int64_t npix_y, double pixsize_x, double pixsize_y, double epsilon,
                      int support, int do_wstacking, double wmin, double wmax, cip_gridder_params* out) {
  if (!out) return set_error(CIP_EINVAL, "out is NULL");
  return choose(npix_x, npix_y, pixsize_x, pixsize_y, epsilon, support, do_wstacking, wmin, wmax, out);
}

}  // extern "C"

namespace cip {
static int ms2dirty_impl(const double* uvw, int64_t nrow, const double* freq, int64_t nchan, const void* vis,
                         int vis_dtype, const void* wgt, int wgt_dtype, const uint8_t* flags4, int64_t npix_x,
                         int64_t npix_y, double pixsize_x, double pixsize_y, double epsilon, int support, int flags,
                         void* hip_stream, double* dirty_out, double* sum_wgt_out, cip_gridder_params* params_out,
                         int64_t plane_begin = 0, int64_t plane_end = -1) {
  if (flags & ~(CIP_WSTACKING | CIP_ACC_SINGLE | CIP_PSF | CIP_NORMALISE | CIP_ASYNC | CIP_PIPELINE | CIP_REUSE_PLAN))
    return set_error(CIP_EINVAL, "unknown flags");
  if ((flags & CIP_REUSE_PLAN) && (flags & CIP_PIPELINE))
    return set_error(CIP_EINVAL, "CIP_REUSE_PLAN cannot be combined with CIP_PIPELINE");
  const int do_wstacking = (flags & CIP_WSTACKING) ? 1 : 0;
  const bool normalise = (flags & CIP_NORMALISE) != 0;
  const bool packed = (flags & CIP_ACC_SINGLE) != 0;
  if (flags & CIP_PSF) {
    vis = nullptr;
    if (vis_dtype != CIP_POL4I) vis_dtype = CIP_C64;
  }
  if (!dirty_out) return set_error(CIP_EINVAL, "dirty_out is NULL");
  if (nrow > 0 && (!uvw || !freq || (!vis && !(flags & CIP_PSF)))) return set_error(CIP_EINVAL, "NULL input pointer");
  hipStream_t s = (hipStream_t)hip_stream;
  Workspace* ws = workspace();
  if (!ws) return set_error(CIP_EHIP, "no HIP device");
  if (const int sr = settle_async(ws, s); sr != CIP_OK) return sr;
  g_prof.reset();
  hipEvent_t t_start = g_prof.mark(s);
  // CIP_ASYNC | CIP_PIPELINE (resident inputs): the planner on the
  // workspace's plan stream with this call's parity of planner buffers, after
  // the last scatter of the call before the previous one (the last user of
  // those buffers) - it then runs beside the previous call's scatter and FFT
  // on s. It does not wait for s: the caller promised the inputs are complete.
  const bool pipelined = (flags & CIP_ASYNC) && (flags & CIP_PIPELINE) && !g_prof.on;
  hipStream_t ps = s;
  if (pipelined) {
    if (!ws->plan_stream) {
      // the plan streams at the lowest priority: the scatter on s keeps first
      // call on freed wave slots (C3 pipelined 21.58-21.62 vs 21.46-21.53
      // Gvis/s at the default priority, 21.15-21.24 at the highest,
      // profiles/r05v_ab_plan_priority.txt)
      int prio_lo = 0, prio_hi = 0;
      CIP_HIP_CHECK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
      CIP_HIP_CHECK(hipStreamCreateWithPriority(&ws->plan_stream, hipStreamNonBlocking, prio_lo));
      CIP_HIP_CHECK(hipStreamCreateWithPriority(&ws->plan_stream1, hipStreamNonBlocking, prio_lo));
      CIP_HIP_CHECK(hipEventCreateWithFlags(&ws->ev_planned, hipEventDisableTiming));
      CIP_HIP_CHECK(hipEventCreateWithFlags(&ws->ev_entry, hipEventDisableTiming));
      for (hipEvent_t& e : ws->ev_done) {
        CIP_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        // the first pipelined calls: the planner starts after the work already on s
        CIP_HIP_CHECK(hipEventRecord(e, s));
      }
    }
    if (ws->plan_unscoped) {
      // a planner ran on s since the last pipelined call: its buffers (parity
      // 0) may still be read there - both plan streams wait for it
      CIP_HIP_CHECK(hipEventRecord(ws->ev_entry, s));
      CIP_HIP_CHECK(hipStreamWaitEvent(ws->plan_stream, ws->ev_entry, 0));
      CIP_HIP_CHECK(hipStreamWaitEvent(ws->plan_stream1, ws->ev_entry, 0));
      ws->plan_unscoped = false;
    }
    ws->parity ^= 1;
    ps = ws->parity ? ws->plan_stream1 : ws->plan_stream;
    CIP_HIP_CHECK(hipStreamWaitEvent(ps, ws->ev_done[ws->parity], 0));
  } else if (ws->parity) {
    // back to the parity-0 buffers: their last pipelined user may still be queued on s
    ws->parity = 0;
  }
  // the next pipelined call with this parity plans only after everything this
  // call queued on s - the scatter reads the plan, the FFT the dirty-tile
  // masks and the weight sum (recorded on every return path)
  struct DoneMark {
    Workspace* ws;
    hipStream_t s;
    bool armed;
    ~DoneMark() {
      if (armed) (void)hipEventRecord(ws->ev_done[ws->parity], s);
    }
  } done_mark{ws, s, pipelined};
  Prepared pp;
  double* grid = nullptr;
  ws->parity_scope = pipelined;
  int rc = prepare(ws, uvw, nrow, freq, nchan, vis, vis_dtype, wgt, wgt_dtype, npix_x, npix_y, pixsize_x, pixsize_y,
                   epsilon, support, do_wstacking, packed, nullptr, ps, &pp,
                   pipelined ? nullptr : &grid, nullptr, (flags & CIP_REUSE_PLAN) != 0, flags4,
                   true, plane_begin, plane_end);
  ws->parity_scope = false;
  // s continues once the plan exists (also after a failed one, or any early
  // return: nothing then runs on it)
  struct PlanJoin {
    Workspace* ws;
    hipStream_t ps, s;
    bool joined;
    int join() {
      if (joined) return CIP_OK;
      joined = true;
      CIP_HIP_CHECK(hipEventRecord(ws->ev_planned, ps));
      CIP_HIP_CHECK(hipStreamWaitEvent(s, ws->ev_planned, 0));
      return CIP_OK;
    }
    ~PlanJoin() { (void)join(); }
  } plan_join{ws, ps, s, !pipelined};
  if (rc != CIP_OK) (void)plan_join.join();
  if (grid) {
    // join the side stream whatever happened (the workspace grid must not be
    // written by a later call while its memset is still queued)
    const int jr = join_side(ws, s);
    if (rc == CIP_OK) rc = jr;
  }
  if (rc != CIP_OK) return rc;
  if (params_out) *params_out = pp.p;
  DirtyStage st;
  rc = dirty_stage(ws, pp.g, npix_x, npix_y, pixsize_x, pixsize_y, s, &st);
  if (rc != CIP_OK) return rc;
  // the packed class grids into complex64 planes on the pruned-FFT path (half
  // the flush and pass-A bytes); CIP_GRID_F32=0 keeps complex128 (A/B)
  pp.g.grid_f32 = (packed && st.fast && grid_f32_enabled()) ? 1 : 0;
  const GridGeometry& g = pp.g;
  // zeroed beside the planner, or left all-zero by the previous call
  bool clean = grid != nullptr;
  const int G = pp.plan.group;
  const int64_t plane_elems = 2 * g.nu * g.nv;
  const size_t cell_bytes = g.grid_f32 ? sizeof(float) : sizeof(double);  // per real component
  if (!grid) grid = buf<double>(ws, "grid", plane_elems * G);
  if (!grid) return CIP_ENOMEM;
  const size_t group_bytes = cell_bytes * (size_t)plane_elems * (size_t)G;
  const size_t prev_clean = ws->grid_clean == grid ? ws->grid_clean_bytes : 0;
  clean = clean || prev_clean >= group_bytes;
  ws->grid_clean = nullptr;  // dirty until a masked pass A has consumed every written tile
  const uint32_t* dmask = st.fast ? pp.plan.dmask : nullptr;
  // the plane groups holding planes [plane_lo, plane_hi) (the whole stack
  // unless cip_ms2dirty_wplanes); an empty range leaves a zero image
  const int64_t p_lo = g.plane_lo, p_hi = g.plane_hi;
  if (p_lo >= p_hi) CIP_HIP_CHECK(hipMemsetAsync(dirty_out, 0, sizeof(double) * npix_x * npix_y, s));
  const int64_t rb_stride = (g.nty + 31) / 32;
  const uint32_t* rowbits0 = dmask ? dmask + g.nplanes * (g.ntx * g.nty / 32) : nullptr;
  if (const int jr = plan_join.join(); jr != CIP_OK) return jr;
  // the packed class's w planes accumulate in a float image (its own
  // precision, one rounding per plane; the final correction writes the fp64
  // image): half the per-plane read-modify-write of pass B. Only beside fp32
  // transforms of complex64 planes (launch_fft_cols refuses any other pairing).
  float* wacc = nullptr;
  if (st.fast && g.do_wstacking && g.grid_f32 && fft_f32_enabled() && p_lo < p_hi && wacc_f32_enabled()) {
    wacc = buf<float>(ws, "wacc_f32", npix_x * npix_y);
    if (!wacc) return CIP_ENOMEM;
  }
  for (int64_t q = p_lo / G; q * G < p_hi; ++q) {
    // pipelined calls: leave CU slots to the next call's planner (profiles/r03_ab_scatter_share.txt)
    rc = scatter_plane(pp, q, uvw, vis, vis_dtype, wgt, wgt_dtype, st.fast, grid, s, clean, pipelined);
    if (rc != CIP_OK) return rc;
    for (int64_t p = std::max(q * G, p_lo); p < std::min<int64_t>(q * G + G, p_hi); ++p) {
      double* plane_p = (double*)((char*)grid + (size_t)(p - q * G) * (size_t)plane_elems * cell_bytes);
      const uint32_t* dm = dmask ? dmask + p * (g.ntx * g.nty / 32) : nullptr;
      const uint32_t* rbp = rowbits0 ? rowbits0 + p * rb_stride : nullptr;
      rc = plane_to_dirty(st, g, p, plane_p, wacc ? (double*)wacc : dirty_out, s, dm, normalise ? pp.red : nullptr,
                          rbp, p == p_lo, wacc != nullptr);
      if (rc != CIP_OK) return rc;
    }
    // a group's planes outside the range were neither written (the scatter
    // skips them) nor read, so a masked pass A still leaves the group clean
    clean = dmask != nullptr;
  }
  rc = finish_dirty(ws, st, pp.p, g, dirty_out, s, wacc);
  if (rc != CIP_OK) return rc;
  // fused into pass B on the pruned 2-D path; a separate pass otherwise
  if (normalise && (!st.fast || g.do_wstacking))
    CIP_HIP_CHECK(launch_scale_inverse(dirty_out, npix_x * npix_y, pp.red, s));
  if (sum_wgt_out) CIP_HIP_CHECK(hipMemcpyAsync(sum_wgt_out, pp.red, sizeof(double), hipMemcpyDeviceToDevice, s));
  g_prof.span(5, t_start, g_prof.mark(s));
  // CIP_ASYNC: the workspace (grid, planner buffers) is reused by later calls
  // of this thread in stream order, so nothing on the host waits for it; the
  // grid-clean mark holds in stream order too
  if (!(flags & CIP_ASYNC) || g_prof.on) CIP_HIP_CHECK(hipStreamSynchronize(s));
  else ws->async_stream = s;
  if (clean) {
    ws->grid_clean = grid;
    ws->grid_clean_bytes = std::max(prev_clean, group_bytes);
  }
  g_prof.finish();
  return CIP_OK;
}
}  // namespace cip

extern "C" {

int cip_ms2dirty(const double* uvw, int64_t nrow, const double* freq, int64_t nchan, const void* vis, int vis_dtype,
                 const void* wgt, int wgt_dtype, int64_t npix_x, int64_t npix_y, double pixsize_x,
                 double pixsize_y, double epsilon, int support, int flags, void* hip_stream,
                 double* dirty_out, double* sum_wgt_out, cip_gridder_params* params_out) {
  g_last_error.clear();
  if (vis_dtype != CIP_C64 && vis_dtype != CIP_C128 && !(flags & CIP_PSF))
    return set_error(CIP_EINVAL, "vis dtype must be complex64 or complex128");
  if (wgt_dtype != CIP_NONE && wgt_dtype != CIP_F32 && wgt_dtype != CIP_F64)
    return set_error(CIP_EINVAL, "wgt dtype must be float32, float64 or none");
  return ms2dirty_impl(uvw, nrow, freq, nchan, vis, vis_dtype, wgt, wgt_dtype, nullptr, npix_x, npix_y, pixsize_x,
                       pixsize_y, epsilon, support, flags, hip_stream, dirty_out, sum_wgt_out, params_out);
}

int cip_ms2dirty_wplanes(const double* uvw, int64_t nrow, const double* freq, int64_t nchan, const void* vis,
                         int vis_dtype, const void* wgt, int wgt_dtype, int64_t npix_x, int64_t npix_y,
                         double pixsize_x, double pixsize_y, double epsilon, int support, int flags,
                         int64_t plane_begin, int64_t plane_end, void* hip_stream, double* dirty_out,
                         double* sum_wgt_out, cip_gridder_params* params_out) {
  g_last_error.clear();
  if (!(flags & CIP_WSTACKING)) return set_error(CIP_EINVAL, "a w-plane range needs CIP_WSTACKING");
  if (plane_begin < 0 || plane_end < plane_begin) return set_error(CIP_EINVAL, "invalid w-plane range");
  if (vis_dtype != CIP_C64 && vis_dtype != CIP_C128 && !(flags & CIP_PSF))
    return set_error(CIP_EINVAL, "vis dtype must be complex64 or complex128");
  if (wgt_dtype != CIP_NONE && wgt_dtype != CIP_F32 && wgt_dtype != CIP_F64)
    return set_error(CIP_EINVAL, "wgt dtype must be float32, float64 or none");
  return ms2dirty_impl(uvw, nrow, freq, nchan, vis, vis_dtype, wgt, wgt_dtype, nullptr, npix_x, npix_y, pixsize_x,
                       pixsize_y, epsilon, support, flags, hip_stream, dirty_out, sum_wgt_out, params_out,
                       plane_begin, plane_end);
}

int cip_ms2dirty_stokes_i(const double* uvw, int64_t nrow, const double* freq, int64_t nchan, const void* vis4,
                          const uint8_t* flags4, const float* wgt4, int64_t npix_x, int64_t npix_y,
                          double pixsize_x, double pixsize_y, double epsilon, int support, int flags,
                          void* hip_stream, double* dirty_out, double* sum_wgt_out, cip_gridder_params* params_out) {
  g_last_error.clear();
  if (nrow > 0 && (!wgt4 || (!vis4 && !(flags & CIP_PSF)))) return set_error(CIP_EINVAL, "NULL vis4 or wgt4");
  if (((uintptr_t)flags4 & 3u) != 0u) return set_error(CIP_EINVAL, "flags4 must be 4-byte aligned");
  return ms2dirty_impl(uvw, nrow, freq, nchan, vis4, CIP_POL4I, wgt4, CIP_POL4I, flags4, npix_x, npix_y, pixsize_x,
                       pixsize_y, epsilon, support, flags, hip_stream, dirty_out, sum_wgt_out, params_out);
}

int cip_grid_layout(const cip_gridder_params* params, int64_t npix_x, int64_t npix_y) {
  g_last_error.clear();
  if (!params) return set_error(CIP_EINVAL, "params is NULL");
  return fft_pruned() && fast_fft_supported(params->nu, params->nv, npix_x, npix_y) ? 1 : 0;
}

int cip_plane_group(const cip_gridder_params* params, int packed) {
  g_last_error.clear();
  if (!params) return set_error(CIP_EINVAL, "params is NULL");
  return wstack_group(geometry(*params, 1.0, 1.0), packed != 0);
}

int cip_grid_ms(const double* uvw, int64_t nrow, const double* freq, int64_t nchan, const void* vis, int vis_dtype,
                const void* wgt, int wgt_dtype, const cip_gridder_params* params, double pixsize_x, double pixsize_y,
                int64_t npix_x, int64_t npix_y, int flags, void* hip_stream, double* grids, double* sum_wgt) {
  if (nrow < 0) return set_error(CIP_EINVAL, "nrow must be >= 0");
  if (!public_dtypes(vis_dtype, wgt_dtype)) return set_error(CIP_EINVAL, "vis dtype must be complex64 or complex128");
  return grid_accumulate(uvw, nrow, freq, nchan, vis, vis_dtype, wgt, wgt_dtype, params, pixsize_x, pixsize_y,
                         npix_x, npix_y, flags, hip_stream, grids, sum_wgt, nullptr);
}

int cip_grid_ms_stokes_i(const double* uvw, int64_t nrow, const double* freq, int64_t nchan, const void* vis4,
                         const uint8_t* flags4, const float* wgt4, const cip_gridder_params* params,
                         double pixsize_x, double pixsize_y, int64_t npix_x, int64_t npix_y, int flags,
                         void* hip_stream, double* grids, double* sum_wgt) {
  if (nrow < 0) return set_error(CIP_EINVAL, "nrow must be >= 0");
  if (nrow > 0 && (!wgt4 || (!vis4 && !(flags & CIP_PSF)))) return set_error(CIP_EINVAL, "NULL vis4 or wgt4");
  if (((uintptr_t)flags4 & 3u) != 0u) return set_error(CIP_EINVAL, "flags4 must be 4-byte aligned");
  return grid_accumulate(uvw, nrow, freq, nchan, vis4, CIP_POL4I, wgt4, CIP_POL4I, params, pixsize_x, pixsize_y,
                         npix_x, npix_y, flags, hip_stream, grids, sum_wgt, nullptr, flags4);
}

int cip_grid_tiles(const double* slice_uvw, const int32_t* chan_start, const int32_t* chan_stop, int64_t nslices,
                   const double* freq, int64_t nchan, const void* vis, int64_t nvis, int vis_dtype, const void* wgt,
                   int wgt_dtype, const cip_gridder_params* params, double pixsize_x, double pixsize_y,
                   int64_t npix_x, int64_t npix_y, int flags, void* hip_stream, double* grids, double* sum_wgt) {
  if (nslices < 0 || nvis < 0) return set_error(CIP_EINVAL, "nslices and nvis must be >= 0");
  if (nslices > 0 && (!chan_start || !chan_stop)) return set_error(CIP_EINVAL, "NULL channel ranges");
  if (nslices >= ((int64_t)1 << 32) - 1) return set_error(CIP_EINVAL, "nslices must be < 2^32 - 1");
  if (!public_dtypes(vis_dtype, wgt_dtype)) return set_error(CIP_EINVAL, "vis dtype must be complex64 or complex128");
  const RaggedRows rr{chan_start, chan_stop, nvis};
  return grid_accumulate(slice_uvw, nslices, freq, nchan, vis, vis_dtype, wgt, wgt_dtype, params, pixsize_x,
                         pixsize_y, npix_x, npix_y, flags, hip_stream, grids, sum_wgt, &rr);
}

int cip_grid_tiles_strip(const double* slice_uvw, const int32_t* chan_start, const int32_t* chan_stop,
                         int64_t nslices, const double* freq, int64_t nchan, const void* vis, int64_t nvis,
                         int vis_dtype, const void* wgt, int wgt_dtype, const cip_gridder_params* params,
                         double pixsize_x, double pixsize_y, int64_t npix_x, int64_t npix_y, int64_t row0,
                         int64_t nrows, int flags, void* hip_stream, double* strip, double* sum_wgt) {
  if (nslices < 0 || nvis < 0) return set_error(CIP_EINVAL, "nslices and nvis must be >= 0");
  if (nslices > 0 && (!chan_start || !chan_stop)) return set_error(CIP_EINVAL, "NULL channel ranges");
  if (nslices >= ((int64_t)1 << 32) - 1) return set_error(CIP_EINVAL, "nslices must be < 2^32 - 1");
  if (nrows < 1) return set_error(CIP_EINVAL, "nrows must be >= 1");
  if (!public_dtypes(vis_dtype, wgt_dtype)) return set_error(CIP_EINVAL, "vis dtype must be complex64 or complex128");
  const RaggedRows rr{chan_start, chan_stop, nvis};
  return grid_accumulate(slice_uvw, nslices, freq, nchan, vis, vis_dtype, wgt, wgt_dtype, params, pixsize_x,
                         pixsize_y, npix_x, npix_y, flags, hip_stream, strip, sum_wgt, &rr, nullptr, row0, nrows);
}

int cip_grid_tiles_strip_mask(const double* slice_uvw, const int32_t* chan_start, const int32_t* chan_stop,
                              int64_t nslices, const double* freq, int64_t nchan, const void* vis, int64_t nvis,
                              int vis_dtype, const void* wgt, int wgt_dtype, const cip_gridder_params* params,
                              double pixsize_x, double pixsize_y, int64_t npix_x, int64_t npix_y, int64_t row0,
                              int64_t nrows, int flags, void* hip_stream, double* strip, double* sum_wgt,
                              uint32_t* tile_bits) {
  if (nslices < 0 || nvis < 0) return set_error(CIP_EINVAL, "nslices and nvis must be >= 0");
  if (nslices > 0 && (!chan_start || !chan_stop)) return set_error(CIP_EINVAL, "NULL channel ranges");
  if (nslices >= ((int64_t)1 << 32) - 1) return set_error(CIP_EINVAL, "nslices must be < 2^32 - 1");
  if (nrows < 1) return set_error(CIP_EINVAL, "nrows must be >= 1");
  if (!tile_bits) return set_error(CIP_EINVAL, "NULL tile_bits");
  if (!public_dtypes(vis_dtype, wgt_dtype)) return set_error(CIP_EINVAL, "vis dtype must be complex64 or complex128");
  const RaggedRows rr{chan_start, chan_stop, nvis};
  return grid_accumulate(slice_uvw, nslices, freq, nchan, vis, vis_dtype, wgt, wgt_dtype, params, pixsize_x,
                         pixsize_y, npix_x, npix_y, flags, hip_stream, strip, sum_wgt, &rr, nullptr, row0, nrows,
                         tile_bits);
}

// ---- the uv-strip split on the device (cip_strips.hip) ----
static int strip_split_check(const cip_gridder_params* params, const double* uvw, int64_t nrow, const double* freq,
                             int64_t nchan, GridGeometry* g) {
  if (!params) return set_error(CIP_EINVAL, "params is NULL");
  if (nrow < 0 || nchan < 1 || nchan > 65535) return set_error(CIP_EINVAL, "need nrow >= 0 and 1 <= nchan <= 65535");
  if (nrow > 0 && (!uvw || !freq)) return set_error(CIP_EINVAL, "NULL uvw or freq");
  const bool pow2 = params->nu > 0 && params->nv > 0 && (params->nu & (params->nu - 1)) == 0 &&
                    (params->nv & (params->nv - 1)) == 0;
  if (!pow2 || params->nv < 32 || params->nv > 16384)
    return set_error(CIP_EINVAL, "strips need a power-of-two grid of 32 .. 16384 rows");
  *g = geometry(*params, 1.0, 1.0);
  return CIP_OK;
}

int cip_strip_histogram(const double* uvw, int64_t nrow, const double* freq, int64_t nchan,
                        const cip_gridder_params* params, double pixsize_x, double pixsize_y, void* hip_stream,
                        int64_t* hist) {
  g_last_error.clear();
  GridGeometry g;
  if (const int rc = strip_split_check(params, uvw, nrow, freq, nchan, &g); rc != CIP_OK) return rc;
  if (!hist) return set_error(CIP_EINVAL, "NULL hist");
  g = geometry(*params, pixsize_x, pixsize_y);
  hipStream_t s = (hipStream_t)hip_stream;
  Workspace* ws = workspace();
  if (!ws) return set_error(CIP_EHIP, "no HIP device");
  if (const int sr = settle_async(ws, s); sr != CIP_OK) return sr;
  if (nrow == 0) {
    CIP_HIP_CHECK(hipMemsetAsync(hist, 0, sizeof(int64_t) * 2 * g.nv, s));
    return CIP_OK;
  }
  CIP_ALLOC(fx, double, "strip_fx", nchan)
  CIP_HIP_CHECK(launch_freq_scale(freq, nchan, fx, nullptr, s));
  const int nb = strip_hist_blocks(nrow);
  CIP_ALLOC(partial, uint32_t, "strip_hist_partial", (int64_t)nb * 2 * g.nv)
  CIP_HIP_CHECK(launch_strip_hist(uvw, nrow, fx, nchan, g, partial, nb, hist, s));
  return CIP_OK;
}

int cip_strip_split(const double* uvw, int64_t nrow, const double* freq, int64_t nchan, const void* vis,
                    int vis_dtype, const void* wgt, int wgt_dtype, const cip_gridder_params* params, double pixsize_y,
                    int64_t y0, int64_t y1, void* hip_stream, int64_t* counts, double* slice_uvw,
                    int32_t* chan_start, int32_t* chan_stop, int64_t* slice_row, void* vis_out, void* wgt_out) {
  g_last_error.clear();
  GridGeometry g;
  if (const int rc = strip_split_check(params, uvw, nrow, freq, nchan, &g); rc != CIP_OK) return rc;
  g = geometry(*params, 1.0, pixsize_y);
  if (!counts) return set_error(CIP_EINVAL, "NULL counts");
  if (y0 < 0 || y1 > g.nv || y1 <= y0) return set_error(CIP_EINVAL, "strip rows outside the grid");
  const int vb = vis ? (vis_dtype == CIP_C64 ? 8 : (vis_dtype == CIP_C128 ? 16 : -1)) : 0;
  const int wb = (vis && wgt) ? (wgt_dtype == CIP_F32 ? 4 : (wgt_dtype == CIP_F64 ? 8 : -1)) : 0;
  if (vb < 0) return set_error(CIP_EINVAL, "vis dtype must be complex64 or complex128");
  if (wb < 0) return set_error(CIP_EINVAL, "wgt dtype must be float32 or float64");
  hipStream_t s = (hipStream_t)hip_stream;
  Workspace* ws = workspace();
  if (!ws) return set_error(CIP_EHIP, "no HIP device");
  if (const int sr = settle_async(ws, s); sr != CIP_OK) return sr;
  CIP_ALLOC(fx, double, "strip_fx", nchan)
  CIP_ALLOC(row_runs, int64_t, "strip_row_runs", nrow + 1)
  CIP_ALLOC(row_vis, int64_t, "strip_row_vis", nrow + 1)
  CIP_ALLOC(scan_tmp, int64_t, "strip_scan_tmp", scan_tmp_elems(nrow + 1))
  CIP_HIP_CHECK(launch_freq_scale(freq, nchan, fx, nullptr, s));
  // the counts and their scans: phase 1 (slice_uvw == NULL) reports the totals;
  // phase 2 recounts (the same arithmetic, the same numbers) and emits
  CIP_HIP_CHECK(launch_strip_count(uvw, nrow, fx, nchan, g, y0, y1, row_runs, row_vis, s));
  CIP_HIP_CHECK(exclusive_scan_i64(row_runs, nrow + 1, scan_tmp, s));
  CIP_HIP_CHECK(exclusive_scan_i64(row_vis, nrow + 1, scan_tmp, s));
  if (!slice_uvw) {
    int64_t* h = (int64_t*)pinned(ws, 2 * sizeof(int64_t));
    if (!h) return set_error(CIP_ENOMEM, "hipHostMalloc failed");
    CIP_HIP_CHECK(hipMemcpyAsync(&h[0], row_runs + nrow, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    CIP_HIP_CHECK(hipMemcpyAsync(&h[1], row_vis + nrow, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    CIP_HIP_CHECK(hipStreamSynchronize(s));
    counts[0] = h[0];
    counts[1] = h[1];
    return CIP_OK;
  }
  if (!chan_start || !chan_stop || !slice_row) return set_error(CIP_EINVAL, "NULL slice outputs");
  if (vb > 0 && !vis_out) return set_error(CIP_EINVAL, "NULL vis_out");
  if (wb > 0 && !wgt_out) return set_error(CIP_EINVAL, "NULL wgt_out");
  if (nrow > 0)
    CIP_HIP_CHECK(launch_strip_emit(uvw, nrow, fx, nchan, g, y0, y1, row_runs, row_vis, vis, vb, wgt, wb, slice_uvw,
                                    chan_start, chan_stop, slice_row, vb ? vis_out : nullptr, wb ? wgt_out : nullptr,
                                    s));
  return CIP_OK;
}

int cip_grid_to_dirty(double* grids, const cip_gridder_params* params, int64_t npix_x, int64_t npix_y,
                      double pixsize_x, double pixsize_y, void* hip_stream, double* dirty_out) {
  g_last_error.clear();
  if (!params || !grids || !dirty_out) return set_error(CIP_EINVAL, "NULL params, grids or dirty_out");
  if (npix_x < 1 || npix_y < 1 || npix_x > params->nu || npix_y > params->nv)
    return set_error(CIP_EINVAL, "image larger than the grid");
  hipStream_t s = (hipStream_t)hip_stream;
  Workspace* ws = workspace();
  if (!ws) return set_error(CIP_EHIP, "no HIP device");
  if (const int sr = settle_async(ws, s); sr != CIP_OK) return sr;
  g_prof.reset();
  hipEvent_t t_start = g_prof.mark(s);
  const GridGeometry g = geometry(*params, pixsize_x, pixsize_y);
  DirtyStage st;
  int rc = dirty_stage(ws, g, npix_x, npix_y, pixsize_x, pixsize_y, s, &st);
  if (rc != CIP_OK) return rc;
  for (int64_t p = 0; p < g.nplanes; ++p) {
    rc = plane_to_dirty(st, g, p, grids + p * 2 * g.nu * g.nv, dirty_out, s);
    if (rc != CIP_OK) return rc;
  }
  rc = finish_dirty(ws, st, *params, g, dirty_out, s);
  if (rc != CIP_OK) return rc;
  g_prof.span(5, t_start, g_prof.mark(s));
  CIP_HIP_CHECK(hipStreamSynchronize(s));
  g_prof.finish();
  return CIP_OK;
}

int cip_grid_plane(const double* uvw, int64_t nrow, const double* freq, int64_t nchan, const void* vis,
                   int vis_dtype, const void* wgt, int wgt_dtype, const cip_gridder_params* params,
                   double pixsize_x, double pixsize_y, int64_t plane, int flags, void* hip_stream,
                   double* grid_out) {
  g_last_error.clear();
  if (flags & ~CIP_ACC_SINGLE) return set_error(CIP_EINVAL, "unknown flags");
  if (!params || !grid_out) return set_error(CIP_EINVAL, "NULL params or grid_out");
  if (plane < 0 || plane >= params->nplanes) return set_error(CIP_EINVAL, "plane out of range");
  if (!public_dtypes(vis_dtype, wgt_dtype)) return set_error(CIP_EINVAL, "vis dtype must be complex64 or complex128");
  hipStream_t s = (hipStream_t)hip_stream;
  Workspace* ws = workspace();
  if (!ws) return set_error(CIP_EHIP, "no HIP device");
  if (const int sr = settle_async(ws, s); sr != CIP_OK) return sr;
  g_prof.reset();
  hipEvent_t t_start = g_prof.mark(s);
  Prepared pp;
  int rc = prepare(ws, uvw, nrow, freq, nchan, vis, vis_dtype, wgt, wgt_dtype, 2, 2, pixsize_x, pixsize_y, 0.0,
                   params->support, params->do_wstacking, (flags & CIP_ACC_SINGLE) != 0, params, s, &pp, nullptr,
                   nullptr, false, nullptr, false);
  if (rc != CIP_OK) return rc;
  rc = scatter_plane(pp, plane, uvw, vis, vis_dtype, wgt, wgt_dtype, false, grid_out, s);
  if (rc != CIP_OK) return rc;
  g_prof.span(5, t_start, g_prof.mark(s));
  CIP_HIP_CHECK(hipStreamSynchronize(s));
  g_prof.finish();
  return CIP_OK;
}

// strips of the pruned FFT (multi-GPU strong scaling)
static int strip_check(const cip_gridder_params* params, int64_t npix_x, int64_t npix_y, GridGeometry* g) {
  if (!params) return set_error(CIP_EINVAL, "params is NULL");
  *g = geometry(*params, 1.0, 1.0);
  if (!grid_is_transposed(*g, npix_x, npix_y))
    return set_error(CIP_EINVAL, "strips need the pruned-FFT grid layout (power-of-two grids, cip_grid_layout == 1)");
  return CIP_OK;
}

int cip_strip_rows(double* grid, const cip_gridder_params* params, int64_t npix_x, int64_t npix_y, int64_t y0,
                   int64_t y1, void* hip_stream, double* H) {
  g_last_error.clear();
  GridGeometry g;
  if (const int rc = strip_check(params, npix_x, npix_y, &g); rc != CIP_OK) return rc;
  if (!grid || !H) return set_error(CIP_EINVAL, "NULL grid or H");
  if (y0 < 0 || y1 > g.nv || y1 <= y0) return set_error(CIP_EINVAL, "row range outside the grid");
  hipStream_t s = (hipStream_t)hip_stream;
  Workspace* ws = workspace();
  if (!ws) return set_error(CIP_EHIP, "no HIP device");
  if (const int sr = settle_async(ws, s); sr != CIP_OK) return sr;
  double* tw_u = nullptr;
  if (const int rc = fft_twiddles(ws, g.nu, s, &tw_u); rc != CIP_OK) return rc;
  CIP_HIP_CHECK(launch_fft_rows_strip(grid, g.nu, g.nv, npix_x, tw_u, y0, y1, H, s));
  CIP_HIP_CHECK(hipStreamSynchronize(s));
  return CIP_OK;
}

int cip_strip_rows_masked(double* grid, const cip_gridder_params* params, int64_t npix_x, int64_t npix_y,
                          int64_t y0, int64_t y1, int64_t row0, const uint32_t* tile_bits, void* hip_stream,
                          double* H) {
  g_last_error.clear();
  GridGeometry g;
  if (const int rc = strip_check(params, npix_x, npix_y, &g); rc != CIP_OK) return rc;
  if (!grid || !H || !tile_bits) return set_error(CIP_EINVAL, "NULL grid, H or tile_bits");
  if (y0 < 0 || y1 > g.nv || y1 <= y0) return set_error(CIP_EINVAL, "row range outside the grid");
  if (row0 < 0 || row0 >= g.nv) return set_error(CIP_EINVAL, "row0 outside the grid");
  if (g.ntx % 32 != 0) return set_error(CIP_EINVAL, "tile masks need nu / 32 to be a multiple of 32 tiles");
  hipStream_t s = (hipStream_t)hip_stream;
  Workspace* ws = workspace();
  if (!ws) return set_error(CIP_EHIP, "no HIP device");
  if (const int sr = settle_async(ws, s); sr != CIP_OK) return sr;
  double* tw_u = nullptr;
  if (const int rc = fft_twiddles(ws, g.nu, s, &tw_u); rc != CIP_OK) return rc;
  CIP_HIP_CHECK(launch_fft_rows_strip(grid, g.nu, g.nv, npix_x, tw_u, y0, y1, H, s, tile_bits, row0));
  CIP_HIP_CHECK(hipStreamSynchronize(s));
  return CIP_OK;
}

int cip_strip_rows_packed(double* grid, const cip_gridder_params* params, int64_t npix_x, int64_t npix_y,
                          int64_t y0, int64_t y1, int64_t row0, const uint32_t* tile_bits, const int64_t* row_slot,
                          int64_t nlive, void* hip_stream, double* H) {
  g_last_error.clear();
  GridGeometry g;
  if (const int rc = strip_check(params, npix_x, npix_y, &g); rc != CIP_OK) return rc;
  if (!grid || !tile_bits || !row_slot) return set_error(CIP_EINVAL, "NULL grid, tile_bits or row_slot");
  if (y0 < 0 || y1 > g.nv || y1 <= y0) return set_error(CIP_EINVAL, "row range outside the grid");
  if (row0 < 0 || row0 >= g.nv) return set_error(CIP_EINVAL, "row0 outside the grid");
  if (nlive < 0 || nlive > y1 - y0) return set_error(CIP_EINVAL, "nlive outside [0, y1 - y0]");
  if (nlive > 0 && !H) return set_error(CIP_EINVAL, "NULL H");
  if (g.ntx % 32 != 0) return set_error(CIP_EINVAL, "tile masks need nu / 32 to be a multiple of 32 tiles");
  hipStream_t s = (hipStream_t)hip_stream;
  Workspace* ws = workspace();
  if (!ws) return set_error(CIP_EHIP, "no HIP device");
  if (const int sr = settle_async(ws, s); sr != CIP_OK) return sr;
  double* tw_u = nullptr;
  if (const int rc = fft_twiddles(ws, g.nu, s, &tw_u); rc != CIP_OK) return rc;
  CIP_HIP_CHECK(launch_fft_rows_strip(grid, g.nu, g.nv, npix_x, tw_u, y0, y1, H, s, tile_bits, row0, row_slot,
                                      nlive));
  CIP_HIP_CHECK(hipStreamSynchronize(s));
  return CIP_OK;
}

int cip_strip_cols(const double* H, const cip_gridder_params* params, int64_t npix_x, int64_t npix_y, int64_t i0,
                   int64_t i1, const double* norm, void* hip_stream, double* dirty_rows) {
  g_last_error.clear();
  GridGeometry g;
  if (const int rc = strip_check(params, npix_x, npix_y, &g); rc != CIP_OK) return rc;
  if (params->do_wstacking)
    return set_error(CIP_EINVAL, "cip_strip_cols: 2-D grids only (w-stacking strips use cip_strip_cols_wplane + "
                                 "cip_strip_wfinal)");
  if (!H || !dirty_rows) return set_error(CIP_EINVAL, "NULL H or dirty_rows");
  if (i0 < 0 || i1 > npix_x || i1 <= i0 || i0 % 4 || i1 % 4)
    return set_error(CIP_EINVAL, "image row range must be multiples of 4 inside [0, npix_x]");
  hipStream_t s = (hipStream_t)hip_stream;
  Workspace* ws = workspace();
  if (!ws) return set_error(CIP_EHIP, "no HIP device");
  if (const int sr = settle_async(ws, s); sr != CIP_OK) return sr;
  double *tw_v = nullptr, *cx = nullptr, *cy = nullptr;
  if (const int rc = fft_twiddles(ws, g.nv, s, &tw_v); rc != CIP_OK) return rc;
  if (const int rc = correction_vectors(ws, g, npix_x, npix_y, s, &cx, &cy); rc != CIP_OK) return rc;
  CIP_HIP_CHECK(launch_fft_cols_strip(H, g.nv, npix_x, npix_y, tw_v, i0, i1, dirty_rows, cx, cy, norm, s));
  CIP_HIP_CHECK(hipStreamSynchronize(s));
  return CIP_OK;
}

int cip_strip_pack_rows(const void* H, int64_t nb, int64_t h, int elem_bytes, const int64_t* slot, int64_t nlive,
                        void* hip_stream, void* out) {
  g_last_error.clear();
  if (elem_bytes != 8 && elem_bytes != 16) return set_error(CIP_EINVAL, "elem_bytes must be 8 or 16");
  if (nb < 0 || h < 0 || nlive < 0 || nlive > h) return set_error(CIP_EINVAL, "bad pack sizes");
  if (nb > 65535) return set_error(CIP_EINVAL, "more than 65535 column blocks");
  if (nb * h * nlive > 0 && (!H || !slot || !out)) return set_error(CIP_EINVAL, "NULL pointer");
  CIP_HIP_CHECK(launch_strip_pack(H, nb, h, elem_bytes / 4, slot, nlive, out, (hipStream_t)hip_stream));
  return CIP_OK;
}

int cip_strip_unpack_rows(const void* recv, int64_t nb, int64_t nv, int elem_bytes, const int64_t* rec,
                          const int64_t* stride, void* hip_stream, void* H) {
  g_last_error.clear();
  if (elem_bytes != 8 && elem_bytes != 16) return set_error(CIP_EINVAL, "elem_bytes must be 8 or 16");
  if (nb < 0 || nv < 0) return set_error(CIP_EINVAL, "bad unpack sizes");
  if (nb > 65535) return set_error(CIP_EINVAL, "more than 65535 column blocks");
  if (nb * nv > 0 && (!rec || !stride || !H)) return set_error(CIP_EINVAL, "NULL pointer");
  CIP_HIP_CHECK(launch_strip_unpack(recv, nb, nv, elem_bytes / 4, rec, stride, H, (hipStream_t)hip_stream));
  return CIP_OK;
}

int cip_strip_cols_wplane(const double* H, const cip_gridder_params* params, int64_t npix_x, int64_t npix_y,
                          double pixsize_x, double pixsize_y, int64_t i0, int64_t i1, int64_t plane, int first,
                          void* hip_stream, double* acc_rows) {
  g_last_error.clear();
  GridGeometry g;
  if (const int rc = strip_check(params, npix_x, npix_y, &g); rc != CIP_OK) return rc;
  if (!params->do_wstacking) return set_error(CIP_EINVAL, "cip_strip_cols_wplane: w-stacking parameters only");
  if (!H || !acc_rows) return set_error(CIP_EINVAL, "NULL H or acc_rows");
  if (plane < 0 || plane >= params->nplanes) return set_error(CIP_EINVAL, "plane out of range");
  if (i0 < 0 || i1 > npix_x || i1 <= i0 || i0 % 4 || i1 % 4)
    return set_error(CIP_EINVAL, "image row range must be multiples of 4 inside [0, npix_x]");
  hipStream_t s = (hipStream_t)hip_stream;
  Workspace* ws = workspace();
  if (!ws) return set_error(CIP_EHIP, "no HIP device");
  if (const int sr = settle_async(ws, s); sr != CIP_OK) return sr;
  double* tw_v = nullptr;
  if (const int rc = fft_twiddles(ws, g.nv, s, &tw_v); rc != CIP_OK) return rc;
  CIP_HIP_CHECK(launch_fft_cols_strip_wplane(H, g.nv, npix_x, npix_y, tw_v, i0, i1, acc_rows, pixsize_x, pixsize_y,
                                             params->w0 + (double)plane * params->dw, first != 0, s));
  CIP_HIP_CHECK(hipStreamSynchronize(s));
  return CIP_OK;
}

int cip_strip_wfinal(double* acc_rows, const cip_gridder_params* params, int64_t npix_x, int64_t npix_y,
                     double pixsize_x, double pixsize_y, int64_t i0, int64_t i1, const double* norm,
                     void* hip_stream) {
  g_last_error.clear();
  GridGeometry g;
  if (const int rc = strip_check(params, npix_x, npix_y, &g); rc != CIP_OK) return rc;
  if (!params->do_wstacking) return set_error(CIP_EINVAL, "cip_strip_wfinal: w-stacking parameters only");
  if (!acc_rows) return set_error(CIP_EINVAL, "NULL acc_rows");
  if (i0 < 0 || i1 > npix_x || i1 <= i0) return set_error(CIP_EINVAL, "image rows outside [0, npix_x)");
  hipStream_t s = (hipStream_t)hip_stream;
  Workspace* ws = workspace();
  if (!ws) return set_error(CIP_EHIP, "no HIP device");
  if (const int sr = settle_async(ws, s); sr != CIP_OK) return sr;
  double *cx = nullptr, *cy = nullptr, *fwd = nullptr;
  int64_t fw_n = 0;
  double dnu = 0.0;
  if (const int rc = correction_vectors(ws, g, npix_x, npix_y, s, &cx, &cy); rc != CIP_OK) return rc;
  if (const int rc = w_correction_table(ws, *params, g, s, &fwd, &fw_n, &dnu); rc != CIP_OK) return rc;
  CIP_HIP_CHECK(launch_wfinal_correct(acc_rows, npix_x, npix_y, pixsize_x, pixsize_y, cx, cy, fwd, fw_n, dnu, g.dw, s,
                                      i0, i1 - i0, norm));
  CIP_HIP_CHECK(hipStreamSynchronize(s));
  return CIP_OK;
}

int cip_tile_runs(const double* uvw, int64_t nrow, const double* freq, int64_t nchan, const double* tile_size3,
                  int64_t row_offset, void* hip_stream, int64_t* n_runs, int64_t* run_key, int64_t* run_row,
                  int32_t* run_c0, int32_t* run_c1) {
  g_last_error.clear();
  if (!tile_size3 || !n_runs) return set_error(CIP_EINVAL, "NULL tile_size or n_runs");
  if (nrow < 0 || nchan < 1) return set_error(CIP_EINVAL, "need nrow >= 0 and nchan >= 1");
  hipStream_t s = (hipStream_t)hip_stream;
  Workspace* ws = workspace();
  if (!ws) return set_error(CIP_EHIP, "no HIP device");
  if (const int sr = settle_async(ws, s); sr != CIP_OK) return sr;
  if (nrow == 0) {
    *n_runs = 0;
    return CIP_OK;
  }
  CIP_ALLOC(winv, double, "winv", nchan)
  CIP_ALLOC(row_runs, int64_t, "row_runs", nrow + 1)
  CIP_ALLOC(tmp, int64_t, "scan_tmp_rows", scan_tmp_elems(nrow + 1))
  CIP_HIP_CHECK(launch_wavelength_inv(freq, nchan, winv, s));
  CIP_HIP_CHECK(hipMemsetAsync(row_runs + nrow, 0, sizeof(int64_t), s));
  CIP_HIP_CHECK(launch_tile_run_count(uvw, nrow, winv, nchan, tile_size3[0], tile_size3[1], tile_size3[2], row_runs,
                                      s));
  CIP_HIP_CHECK(exclusive_scan_i64(row_runs, nrow + 1, tmp, s));
  int64_t* h = (int64_t*)pinned(ws, sizeof(int64_t));
  if (!h) return set_error(CIP_ENOMEM, "hipHostMalloc failed");
  CIP_HIP_CHECK(hipMemcpyAsync(h, row_runs + nrow, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  CIP_HIP_CHECK(hipStreamSynchronize(s));
  const int64_t total = h[0];
  if (run_key == nullptr) {
    *n_runs = total;
    return CIP_OK;
  }
  if (*n_runs < total) return set_error(CIP_EINVAL, "output buffers too small (pass *n_runs = capacity)");
  if (!run_row || !run_c0 || !run_c1) return set_error(CIP_EINVAL, "NULL output buffer");
  CIP_HIP_CHECK(launch_tile_run_emit(uvw, nrow, winv, nchan, tile_size3[0], tile_size3[1], tile_size3[2],
                                     row_offset, row_runs, run_key, run_row, run_c0, run_c1, s));
  CIP_HIP_CHECK(hipStreamSynchronize(s));
  *n_runs = total;
  return CIP_OK;
}

int cip_stokes(const void* vis4, const uint8_t* flags4, const float* wgt4, int64_t n, int stokes, void* hip_stream,
               void* vis_out, uint8_t* flag_out, float* wgt_out, float* eff_w) {
  g_last_error.clear();
  if (n < 0) return set_error(CIP_EINVAL, "n must be >= 0");
  if (stokes < CIP_STOKES_I || stokes > CIP_STOKES_V) return set_error(CIP_EINVAL, "stokes must be I, Q, U or V");
  if (n == 0) return CIP_OK;
  if (vis_out && !vis4) return set_error(CIP_EINVAL, "visibilities requested without vis4");
  if ((wgt_out || eff_w) && !wgt4) return set_error(CIP_EINVAL, "weights requested without wgt4");
  if ((flag_out || eff_w) && !flags4) return set_error(CIP_EINVAL, "flags requested without flags4");
  hipStream_t s = (hipStream_t)hip_stream;
  CIP_HIP_CHECK(launch_stokes(stokes, vis4, flags4, wgt4, n, vis_out, flag_out, wgt_out, eff_w, s));
  CIP_HIP_CHECK(hipStreamSynchronize(s));
  return CIP_OK;
}

int cip_stokes_i(const void* vis4, const uint8_t* flags4, const float* wgt4, int64_t n, void* hip_stream,
                 void* vis_i, uint8_t* flag_i, float* wgt_i, float* eff_w) {
  return cip_stokes(vis4, flags4, wgt4, n, CIP_STOKES_I, hip_stream, vis_i, flag_i, wgt_i, eff_w);
}

int cip_facet_rephase(const double* uvw, int64_t nrow, const double* freq, int64_t nchan, const void* vis,
                      int vis_dtype, double l0, double m0, void* hip_stream, double* uvw_out, void* vis_out) {
  g_last_error.clear();
  if (nrow < 0 || nchan < 1) return set_error(CIP_EINVAL, "need nrow >= 0 and nchan >= 1");
  if (!vis_dtype_ok(vis_dtype)) return set_error(CIP_EINVAL, "vis dtype must be complex64 or complex128");
  if (!(l0 * l0 + m0 * m0 < 1.0)) return set_error(CIP_EINVAL, "facet centre outside the unit circle");
  if (nrow == 0) return CIP_OK;
  if (!uvw || !freq || !uvw_out || (vis_out && !vis)) return set_error(CIP_EINVAL, "NULL pointer");
  hipStream_t s = (hipStream_t)hip_stream;
  Workspace* ws = workspace();
  if (!ws) return set_error(CIP_EHIP, "no HIP device");
  if (const int sr = settle_async(ws, s); sr != CIP_OK) return sr;
  CIP_ALLOC(delay, double, "facet_delay", nrow)
  // Q: the minimal rotation taking z = (0, 0, 1) to s0 (Rodrigues about z x s0)
  const double n0 = std::sqrt(1.0 - l0 * l0 - m0 * m0);
  const double kx = -m0, ky = l0;  // z x s0 (unnormalised; |k| = sin theta)
  const double sn2 = kx * kx + ky * ky, c = n0;
  double Q[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  if (sn2 > 0.0) {
    const double f = (1.0 - c) / sn2;  // (1 - cos) / sin^2 on the unnormalised axis
    // Q = I + [k]x + f [k]x^2, [k]x = ((0, 0, ky), (0, 0, -kx), (-ky, kx, 0))
    Q[0] = 1.0 - f * ky * ky;
    Q[1] = f * kx * ky;
    Q[2] = ky;
    Q[3] = f * kx * ky;
    Q[4] = 1.0 - f * kx * kx;
    Q[5] = -kx;
    Q[6] = -ky;
    Q[7] = kx;
    Q[8] = 1.0 - f * sn2;
  }
  double qt[9];
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b) qt[3 * a + b] = Q[3 * b + a];
  CIP_HIP_CHECK(launch_facet_rephase(uvw, nrow, freq, nchan, vis_out ? vis : nullptr, vis_dtype == CIP_C128, qt, l0, m0,
                                     uvw_out, delay, vis_out, s));
  CIP_HIP_CHECK(hipStreamSynchronize(s));
  return CIP_OK;
}

int cip_profile_enable(int on) {
  g_prof.on = (on != 0);
  return CIP_OK;
}

int cip_profile_last(double* ms, int64_t* counts) {
  if (ms)
    for (int i = 0; i < CIP_PROFILE_PHASES; ++i) ms[i] = g_prof.ms[i];
  if (counts)
    for (int i = 0; i < CIP_PROFILE_COUNTS; ++i) counts[i] = g_prof.counts[i];
  return CIP_OK;
}

int cip_release_workspace(void) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return set_error(CIP_EHIP, "no HIP device");
  std::lock_guard<std::mutex> lock(g_ws_mutex);
  auto it = g_ws.find(std::make_pair(dev, std::this_thread::get_id()));
  if (it == g_ws.end()) return CIP_OK;
  Workspace* ws = it->second;
  g_ws.erase(it);
  destroy_workspace(ws);
  return CIP_OK;
}

}  // extern "C"
