// kd_capi.cpp -- workspace sizing, error reporting and version of the C ABI.
#include "kd_capi.hpp"

#include "kd_binning.hpp"

#include <atomic>
#include <mutex>
#include <vector>

namespace kd {
char *error_buffer() {
  static thread_local char buf[512] = {0};
  return buf;
}

std::atomic<int> g_debug{0};
#if KD_DIAG
int debug_flags() { return g_debug.load(); }
#endif
std::atomic<int> g_forms{0};
int test_forms() { return g_forms.load(); }
std::atomic<int> g_split{0};
int tile_split() { return g_split.load(); }
std::atomic<int> g_ct{0};
int coarse_tile_hook() { return g_ct.load(); }
// The device a stream belongs to (the null stream: the calling thread's current device).  The C
// ABI launches on the caller's stream whatever device is current, so per-device state (the tile
// history, the CU count) is keyed by the stream's device, never by hipGetDevice alone.
int stream_device(hipStream_t stream) {
  hipDevice_t d = -1;
  if (stream && hipStreamGetDevice(stream, &d) == hipSuccess && d >= 0) return (int)d;
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) cur = 0;
  return cur;
}
namespace {
constexpr int kMaxDevices = 64;
std::atomic<int> g_cus[kMaxDevices];  // 0: not queried yet
}  // namespace
int device_cus(hipStream_t stream) {
  const int dev = stream_device(stream);
  if (dev < 0 || dev >= kMaxDevices) return 256;
  int n = g_cus[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
    n = 256;
  g_cus[dev].store(n, std::memory_order_relaxed);
  return n;
}
std::atomic<int> g_hist{1};
namespace {
struct HistSlot {
  unsigned short *buf = nullptr;  // the caller's buffer (kd_tile_history_attach), not owned
  long long tag = -1;
};
HistSlot g_hist_slots[kMaxDevices];
std::mutex g_hist_mu;
}  // namespace
// One caller-owned buffer per device (kd_tile_history_attach): streams, threads and captured
// graphs of that device share it.  Sharing can only degrade the dispatch order
// (tile_order reads each entry once, so any history gives a permutation of the tiles), never a
// result.  The library allocates nothing here: without an attached buffer there is no history.
unsigned short *tile_history(int64_t n, long long tag, hipStream_t stream) {
  if (!g_hist.load() || n <= 0 || n > kTileHistCap) return nullptr;
  const int dev = stream_device(stream);  // the device the launches will run on
  if (dev < 0 || dev >= kMaxDevices) return nullptr;
  std::lock_guard<std::mutex> lk(g_hist_mu);
  HistSlot &h = g_hist_slots[dev];
  if (!h.buf) return nullptr;
  if (h.tag == tag) return h.buf;  // the common case: no fill, no capture query
  // a new shape: only outside a stream capture (a captured zero fill would clear the history on
  // every replay)
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(stream, &st) != hipSuccess || st != hipStreamCaptureStatusNone)
    return nullptr;
  if (zero_words(h.buf, sizeof(unsigned short) * (size_t)n, stream) != hipSuccess) return nullptr;
  h.tag = tag;
  return h.buf;
}
int tile_history_attach(hipStream_t stream, void *buf, size_t bytes) {
  const int dev = stream_device(stream);
  if (dev < 0 || dev >= kMaxDevices)
    return set_error(KD_ERR_INVALID_ARGUMENT, "tile history: device %d out of range", dev);
  if (buf && bytes < sizeof(unsigned short) * (size_t)kTileHistCap)
    return set_error(KD_ERR_INVALID_ARGUMENT, "tile history: %zu bytes < %zu", bytes,
                     sizeof(unsigned short) * (size_t)kTileHistCap);
  std::lock_guard<std::mutex> lk(g_hist_mu);
  HistSlot &h = g_hist_slots[dev];
  h.buf = (unsigned short *)buf;
  h.tag = -1;  // zeroed by the next forward of any shape
  return KD_OK;
}
std::atomic<long long *> g_tbuf{nullptr};
std::atomic<float> g_lim_bins{1.f}, g_lim_pairs{1.f};
float pool_limit_bins() { return g_lim_bins.load(); }
float pool_limit_pairs() { return g_lim_pairs.load(); }
std::atomic<bool> g_lim_ever{false};
bool pool_limits_ever_set() { return g_lim_ever.load(); }
long long *debug_tile_buffer() {
  return (KD_DIAG && (g_debug.load() & 64)) ? g_tbuf.load() : nullptr;
}

namespace {
std::atomic<bool> g_prof{false};
std::mutex g_prof_mu;
struct Rec {
  int id;
  hipEvent_t start, stop;
};
std::vector<Rec> g_recs;
const char *kNames[K_NUM_KERNELS] = {
    "kd_bin_count", "kd_bin_scan", "kd_bin_scatter", "kd_raster_fwd", "kd_soft_fwd",
    "kd_raster_bwd_tile", "kd_soft_bwd_tile", "kd_raster_bwd_atomic", "kd_soft_bwd_atomic",
    "kd_zero", "kd_soft_pairs", "kd_soft_pair_math", "kd_soft_reduce", "kd_soft_bwd_pairs",
    "kd_prepare_fwd", "kd_prepare_bwd", "kd_tile_order", "kd_iou_partial", "kd_iou_bwd",
    "kd_tex_fwd", "kd_tex_bwd", "kd_rast_interp", "kd_dt_bin",
    "kd_dt_fwd", "kd_dibr_bwd", "kd_dibr_fwd", "kd_soft_ovf_fwd", "kd_soft_ovf_bwd",
    "kd_dt_bwd"};
}  // namespace

ProfScope::ProfScope(int id_, hipStream_t s) : id(id_), stream(s), on(g_prof.load()) {
  if (on) {
    on = hipEventCreate(&start) == hipSuccess && hipEventCreate(&stop) == hipSuccess &&
         hipEventRecord(start, stream) == hipSuccess;
  }
}
ProfScope::~ProfScope() {
  if (!on) return;
  if (hipEventRecord(stop, stream) != hipSuccess) return;
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_recs.push_back({id, start, stop});
}
}  // namespace kd

extern "C" {

size_t kd_workspace_size(int kind, int B, int H, int W, int64_t num_faces_total,
                         int64_t max_faces_per_view) {
  if (B < 0 || H < 0 || W < 0 || num_faces_total < 0 || max_faces_per_view < 0) return 0;
  switch (kind) {
    case KD_WS_RASTER_PACKED:
    case KD_WS_RASTER:
    case KD_WS_SOFT_MASK:
      return kd::bin_workspace_bytes(B, H, W, num_faces_total, max_faces_per_view);
    default:
      return 0;
  }
}

const char *kd_last_error(void) { return kd::error_buffer(); }

int kd_version(void) { return 1; }

void kd_profile_enable(int on) { kd::g_prof.store(on != 0); }

int kd_debug_set(int flags) {
  if (!KD_DIAG && flags != 0)
    return kd::set_error(KD_ERR_INVALID_ARGUMENT, "debug flags: diagnostic build only");
  kd::g_debug.store(flags);
  return KD_OK;
}

int kd_set_test_forms(int forms) {
  if (forms & ~(KD_FORM_SPLIT_FWD | KD_FORM_SPLIT_BWD | KD_FORM_SOFT_SPLIT))
    return kd::set_error(KD_ERR_INVALID_ARGUMENT, "unknown launch form bits 0x%x", forms);
  kd::g_forms.store(forms);
  return KD_OK;
}

int kd_set_tile_split(int split) {
  if (split != 0 && split != 1 && split != 2 && split != 4)
    return kd::set_error(KD_ERR_INVALID_ARGUMENT, "tile split must be 0, 1, 2 or 4 (got %d)", split);
  kd::g_split.store(split);
  return KD_OK;
}

int kd_set_coarse_tile(int px) {
  if (px != 0 && px != 16 && px != 32)
    return kd::set_error(KD_ERR_INVALID_ARGUMENT, "coarse tile must be 0, 16 or 32 (got %d)", px);
  kd::g_ct.store(px);
  return KD_OK;
}

int kd_set_tile_history(int on) {
  if (on != 0 && on != 1)
    return kd::set_error(KD_ERR_INVALID_ARGUMENT, "tile history must be 0 or 1 (got %d)", on);
  kd::g_hist.store(on);
  return KD_OK;
}

int kd_stream_device(void *stream, int *compute_units) {
  if (compute_units) *compute_units = kd::device_cus((hipStream_t)stream);
  return kd::stream_device((hipStream_t)stream);
}

size_t kd_tile_history_bytes(void) { return sizeof(unsigned short) * (size_t)kd::kTileHistCap; }

int kd_tile_history_attach(void *stream, void *device_buffer, size_t bytes) {
  return kd::tile_history_attach((hipStream_t)stream, device_buffer, bytes);
}

int kd_set_pool_limits(double bins, double pairs) {
  if (!(bins >= 0.0 && bins <= 1.0 && pairs >= 0.0 && pairs <= 1.0))
    return kd::set_error(KD_ERR_INVALID_ARGUMENT, "pool limits must be in [0, 1]");
  kd::g_lim_bins.store((float)bins);
  kd::g_lim_pairs.store((float)pairs);
  if (bins < 1.0 || pairs < 1.0) kd::g_lim_ever.store(true);
  return KD_OK;
}

int kd_debug_buffer(void *device_ptr) {
  kd::g_tbuf.store((long long *)device_ptr);
  return KD_OK;
}

int kd_profile_collect(double *total_ms, int64_t *launches, int n) {
  std::vector<kd::Rec> recs;
  {
    std::lock_guard<std::mutex> lk(kd::g_prof_mu);
    recs.swap(kd::g_recs);
  }
  for (auto &r : recs) {
    float ms = 0.f;
    if (hipEventSynchronize(r.stop) == hipSuccess &&
        hipEventElapsedTime(&ms, r.start, r.stop) == hipSuccess && r.id < n) {
      if (total_ms) total_ms[r.id] += ms;
      if (launches) launches[r.id] += 1;
    }
    (void)hipEventDestroy(r.start);
    (void)hipEventDestroy(r.stop);
  }
  return n < kd::K_NUM_KERNELS ? n : kd::K_NUM_KERNELS;  // the entries written
}

const char *kd_profile_kernel_name(int id) {
  return (id >= 0 && id < kd::K_NUM_KERNELS) ? kd::kNames[id] : "";
}

}  // extern "C"
