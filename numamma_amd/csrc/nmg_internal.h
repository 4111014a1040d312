// nmg_internal.h -- engine internals shared by the HIP engine, the host report
// writer and the replay driver.  Not part of the C-ABI.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "numamma_gpu.h"

namespace nmg {

// Layout of the flat merge arrays (see nmg_export_array):
//   sum64: [2 access][39] global sums   (total_count, total_weight, na_miss_count,
//                                         18 x (count, sum_weight))
//          [2 access][2][E]              per-entry count, weight (SoA: a flush in
//                                         entry order coalesces its atomics)
//          [E][2 access][37]             per-entry levels (na, 18 x (count, sum)), optional
//   min64: [2][18] global bucket min_weight, [E] first-match ordinal, [1] error word
//   max64: [2][18] global bucket max_weight
constexpr uint32_t kGlobalSums = 39;
constexpr uint32_t kLevelWords = 37;
constexpr uint64_t kHistSparse = ~0ull;
constexpr uint32_t kPageSize = 4096;  // src/mem_analyzer.c:471

constexpr uint64_t gsum_index(uint32_t access, uint32_t i) { return access * kGlobalSums + i; }
constexpr uint64_t objcw_index(uint64_t e, uint32_t access, uint32_t w, uint64_t nb_entries) {
  return 2 * kGlobalSums + (uint64_t(access) * 2 + w) * nb_entries + e;
}

// Error word: min over ((seq << 40) | (byte offset << 8) | code) so the first
// failing record in analysis order wins, as the reference's abort() would.
enum ErrCode : uint32_t {
  kErrNone = 0,
  kErrZeroSize = 1,
  kErrTruncated = 2,
  kErrUnaligned = 3,
  kErrCapacity = 4,
  kErrRange = 5,
  kErrRouteOverflow = 6,  // partition-first path: more short SAMPLE records than its overflow list holds
};

struct HostResults {
  nmg_mem_counters global[2];
  uint64_t nb_samples_total = 0, nb_found_total = 0;
  std::vector<uint32_t> buf_samples, buf_found;
  std::vector<uint64_t> buf_bytes;
  std::vector<uint64_t> first;        // [E]
  std::vector<uint64_t> count_weight; // [E][2][2]
  std::vector<uint64_t> levels;       // [E][2][37] (empty unless NMG_F_OBJECT_LEVELS)
};

// ---- engine accessors used by the report writer (implemented in nmg_engine.hip)
uint32_t engine_nb_threads(nmg_engine* h);
uint32_t engine_nb_entries(nmg_engine* h);
uint32_t engine_flags(nmg_engine* h);
const std::vector<uint64_t>& engine_hist_base(nmg_engine* h);  // per entry, kHistSparse if sparse/none
const std::vector<uint64_t>& engine_npages(nmg_engine* h);     // per entry: buffer_size/4096 + 1
const std::vector<uint32_t>& engine_sparse_entries(nmg_engine* h);  // sparse idx -> entry
// entries: the per-entry arrays too; buffer_found: the per-buffer matched
// counts too (the report needs only their total, nb_found_total)
int engine_download(nmg_engine* h, HostResults& out, bool entries = true, bool buffer_found = true);
int engine_download_hist(nmg_engine* h, std::vector<uint32_t>& cells);
void engine_set_error(nmg_engine* h, const std::string& msg);

// sparse key packing: (sparse idx:22 | thread:10 | page:32)
constexpr uint64_t sparse_key(uint32_t sidx, uint32_t th, uint32_t page) {
  return (uint64_t(sidx) << 42) | (uint64_t(th) << 32) | page;
}
constexpr uint32_t sparse_key_idx(uint64_t k) { return uint32_t(k >> 42); }
constexpr uint32_t sparse_key_thread(uint64_t k) { return uint32_t((k >> 32) & 0x3ff); }
constexpr uint32_t sparse_key_page(uint64_t k) { return uint32_t(k); }

// ---- dump modes: what the report writer needs besides the counters
struct DumpBuffer {
  const uint8_t* data;    // the linearised buffer
  uint64_t len;
  uint32_t thread_rank, access;
  const uint32_t* match;  // [byte offset / 8] = entry + 1 for SAMPLE records, 0 = unmatched
};
struct DumpInput {
  std::vector<DumpBuffer> buffers;  // analysis order
  const uint64_t* entry_addr;       // [E] buffer_addr (sample offsets)
  const uint64_t* levels;           // [E][2][kLevelWords] (callsite_summary_<id>.dat)
};

// ---- report writer (nmg_report.cpp)
// found_total: the matched-sample total when r->buf_found is not filled in
// (the engine's report: the analysis counts it, Params::found)
int write_report(const nmg_host_results* r, const nmg_object_meta* meta, const nmg_report_options* opts,
                 const char* stdout_path, std::string& err, const DumpInput* dump = nullptr,
                 const uint64_t* found_total = nullptr);

}  // namespace nmg
