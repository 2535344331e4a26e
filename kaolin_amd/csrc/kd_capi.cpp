// kd_capi.cpp -- workspace sizing, error reporting and version of the C ABI.
#include "kd_capi.hpp"

#include "kd_binning.hpp"

namespace kd {
char *error_buffer() {
  static thread_local char buf[512] = {0};
  return buf;
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
    case KD_WS_GATHER_BWD:
      return 0;
    default:
      return 0;
  }
}

const char *kd_last_error(void) { return kd::error_buffer(); }

int kd_version(void) { return 1; }

}  // extern "C"
