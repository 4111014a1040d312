// nmg_host_stubs.cpp -- the device half of the C-ABI, absent, for the
// sanitizer build of the host-only sources (tools/sanitize.sh).
//
// build_san/libnmg_host_san.so = nmg_report.cpp + nmg_replay.cpp + this file,
// compiled by g++ with -fsanitize=address,undefined.  The CPU tests that load
// the library (the report writer through nmg_report_host, the replay writer,
// error strings) run against it; every call that needs a GPU returns
// NMG_ERR_HIP, as the real library does on a host without one.
#include <cstring>

#include "nmg_internal.h"

namespace nmg {
uint32_t engine_nb_threads(nmg_engine*) { return 0; }
int engine_download(nmg_engine*, HostResults&, bool, bool) { return NMG_ERR_HIP; }
}  // namespace nmg

extern "C" {
const char* nmg_strerror(int status) {
  switch (status) {
    case NMG_OK: return "ok";
    case NMG_ERR_HIP: return "no HIP device (sanitizer build: host code only)";
    default: return "error (sanitizer build: host code only)";
  }
}
int nmg_get_last_error_detail(nmg_engine*, char* buf, size_t len) {
  if (buf && len) buf[0] = 0;
  return NMG_OK;
}
int nmg_create(nmg_engine** out, const nmg_options*) {
  if (out) *out = nullptr;
  return NMG_ERR_HIP;
}
void nmg_destroy(nmg_engine*) {}
int nmg_set_objects(nmg_engine*, const uint64_t*, const uint32_t*, uint32_t, const nmg_object*, uint32_t) {
  return NMG_ERR_HIP;
}
int nmg_submit_ring(nmg_engine*, const void*, uint64_t, uint64_t, uint64_t, uint32_t, uint32_t) {
  return NMG_ERR_HIP;
}
int nmg_submit_buffers(nmg_engine*, uint32_t, const void* const*, const uint64_t*, const uint32_t*,
                       const uint32_t*) {
  return NMG_ERR_HIP;
}
int nmg_register_host(nmg_engine*, void*, uint64_t) { return NMG_ERR_HIP; }
int nmg_stream_begin(nmg_engine*, uint64_t, uint32_t) { return NMG_ERR_HIP; }
int nmg_analyze(nmg_engine*) { return NMG_ERR_HIP; }
int nmg_synchronize(nmg_engine*) { return NMG_ERR_HIP; }
int64_t nmg_count_page_cells(nmg_engine*) { return NMG_ERR_HIP; }
int nmg_get_page_cells(nmg_engine*, uint32_t*, int64_t) { return NMG_ERR_HIP; }
int nmg_report(nmg_engine*, const nmg_object_meta*, const nmg_report_options*, const char*) {
  return NMG_ERR_HIP;
}
}
