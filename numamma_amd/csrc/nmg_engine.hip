// nmg_engine.hip -- host side of the MI355X sample-attribution engine: the
// C-ABI (include/numamma_gpu.h), table upload and lookup-structure build, the
// stream-sorted schedule, the streaming pipeline (copy stream + double-buffered
// pinned staging), launches and result downloads.  The kernels are in
// nmg_kernels.hip (DESIGN.md "Kernels").
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <chrono>
#include <cinttypes>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstddef>
#include <cstring>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "nmg_kernels.h"
#include "nmg_route.h"

// ===========================================================================
// host side

using namespace nmg;

// roctx range over one host-side stage (rocprofv3 --marker-trace): stage,
// attribution enqueue, merge, table swap, report
struct Range {
  explicit Range(const char* what) { roctxRangePushA(what); }
  ~Range() { roctxRangePop(); }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;
};

// Persistent host threads for the staging copies of nmg_submit_buffers (a
// batch per alarm in streaming mode would otherwise pay a thread start per
// copy thread per batch).
struct CopyPool {
  std::vector<std::thread> workers;
  std::mutex m;
  std::condition_variable wake, idle;
  std::function<void(uint32_t)> job;
  uint64_t gen = 0;
  uint32_t pending = 0;
  bool stop = false;

  explicit CopyPool(uint32_t n) {
    for (uint32_t w = 1; w < n; w++)
      workers.emplace_back([this, w] {
        uint64_t seen = 0;
        for (;;) {
          std::function<void(uint32_t)> f;
          {
            std::unique_lock<std::mutex> lk(m);
            wake.wait(lk, [&] { return stop || gen != seen; });
            if (stop) return;
            seen = gen;
            f = job;
          }
          f(w);
          std::lock_guard<std::mutex> lk(m);
          if (--pending == 0) idle.notify_one();
        }
      });
  }
  // run f(0..n-1) with worker w taking part w (the caller runs part 0)
  void run(const std::function<void(uint32_t)>& f) {
    {
      std::lock_guard<std::mutex> lk(m);
      job = f;
      pending = (uint32_t)workers.size();
      gen++;
    }
    wake.notify_all();
    f(0);
    std::unique_lock<std::mutex> lk(m);
    idle.wait(lk, [&] { return pending == 0; });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(m);
      stop = true;
    }
    wake.notify_all();
    for (auto& t : workers) t.join();
  }
};

struct nmg_engine {
  int device = 0;
  uint32_t flags = NMG_F_DEFAULT;
  uint32_t T = 1;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  static constexpr int kRing = 64;  // per-launch timing events (nmg_get_launch_times)
  hipEvent_t ring0[kRing] = {}, ring1[kRing] = {};
  hipEvent_t ringm[kRing] = {};  // after the attribution kernel (before the log reduce)
  hipEvent_t ringr[kRing] = {};  // after the first kernel (route_kernel / attribute_kernel)
  uint64_t nlaunch = 0;
  int num_cus = 256;
  int blocks_per_cu = 0;
  bool launched = false;

  // object table
  bool have_table = false;
  // results epoch: bumped by every call that can change a counter; the page
  // cells counted by nmg_count_page_cells stay on the device (cells_*) until
  // nmg_get_page_cells of the same epoch copies them out
  uint64_t epoch = 1, cells_epoch = 0;
  // host memory registered with nmg_register_host (device-visible, pinned):
  // a submitted buffer inside it is read by the kernels in place over PCIe
  // (zc_dev[i] = its device address, 0 = staged)
  struct HostReg {
    uintptr_t lo, hi;  // the caller's range
    uint64_t dev;      // device address of lo
    void* pages;       // the registered whole pages around it
  };
  std::vector<HostReg> hostregs;
  std::vector<uint64_t> zc_dev;
  int64_t cells_n = 0;
  void* d_cells_rows = nullptr;  // uint4 [cells_n] dense rows (sparse rows: cells_sparse)
  size_t cells_rows_cap = 0;
  struct SparseRows {
    uint64_t off;  // first row
    uint32_t e;
    std::vector<std::pair<uint64_t, uint32_t>> cells;  // ((thread << 32 | page), count)
  };
  std::vector<SparseRows> cells_sparse;
  uint32_t K = 0, E = 0;
  uint64_t* d_keys = nullptr;
  DevEntry* d_nodes = nullptr;
  uint64_t* d_efences = nullptr;  // small tables: Eytzinger-ordered keys / node records
  DevEntry* d_enodes = nullptr;
  uint32_t elevels = 0;
  DevEntry* d_entries = nullptr;  // by entry id (the nmg_set_objects table)
  DevEntry* d_chain = nullptr;    // table order of the current lookup table; == d_entries until
                                  // the first nmg_update_objects
  uint64_t* d_ffences = nullptr;  // large tables: Eytzinger fences, directory shifts, directory
  uint8_t* d_fshift = nullptr;
  uint2* d_dir = nullptr;
  uint32_t nb_fences = 0, fence_log2 = 0, dir_log2 = 0;
  std::vector<uint64_t> hist_base, npages, buffer_size, entry_addr;
  std::vector<DevEntry> dev_entries;  // host copy of d_entries (nmg_update_objects builds from it)
  std::vector<nmg_object> objects;  // each entry as the latest table lists it (the report's objects)
  std::vector<uint32_t> order;      // report walk order (position -> id) when it is not the id order:
                                    // the latest table that listed every entry (nmg_update_objects)
  std::vector<uint32_t> sparse_entries;
  uint64_t hist_cells = 0;
  uint64_t hist_budget = 4ull << 30;
  uint64_t sparse_cap = 1u << 20;

  // counters
  uint64_t *d_sum64 = nullptr, *d_min64 = nullptr, *d_max64 = nullptr;
  uint64_t n_sum64 = 0, n_min64 = 0, n_max64 = 0;
  uint32_t* d_hist = nullptr;
  unsigned long long* d_found = nullptr;  // matched SAMPLEs since the last reset (Params::found)
  uint64_t* d_scratch = nullptr;          // [2] small device results (nmg_hist_pack / unpack)
  uint64_t* d_sparse_keys = nullptr;
  uint32_t* d_sparse_vals = nullptr;
  uint64_t* d_objcw = nullptr;       // [objcw_cap][4] per-object counters laid out for the D2H
  uint64_t objcw_cap = 0;
  uint64_t* d_sparse_ck = nullptr;  // [sparse_cap + 1] compacted (key, count) words + the count (sparse_download)
  uint32_t* d_sparse_dirty = nullptr;  // [2] parity flags (see reset_kernel)
  uint32_t* d_smatch = nullptr;        // NMG_F_SAMPLE_MATCHES: per 8 B of the arena span
  unsigned long long* d_pk64 = nullptr;  // hashed object mode: packed long-tail counters (0 between launches)
  uint4* d_tlog = nullptr;  // hashed object mode: long-tail log (see Params::tlog)
  size_t tlog_bytes = 0;
  uint32_t* d_tlog_cnt = nullptr;
  size_t tlog_cnt_cap = 0;
  size_t smatch_cap = 0;
  uint64_t nreset = 0;

  // buffers
  std::vector<BufDesc> descs;
  std::vector<uint64_t> buf_bytes;
  uint8_t* h_stage = nullptr;
  size_t stage_cap = 0, stage_len = 0;
  uint8_t* d_arena = nullptr;
  size_t arena_cap = 0;
  const uint8_t* d_data = nullptr;
  bool external = false;
  bool staged_dirty = false;
  BufDesc* d_descs = nullptr;
  size_t descs_cap = 0;
  BufDesc* d_sdescs = nullptr;   // descriptors in stream-sorted schedule order
  uint32_t* d_ranges = nullptr;  // per-workgroup [begin, end) in d_order
  uint32_t sched_grid = 0;       // grid the current schedule was built for
  bool descs_dirty = false;
  bool multi_staged = false;  // the workers' arenas hold the current buffers (multi_analyze)
  uint32_t* d_bufcnt = nullptr;
  size_t bufcnt_cap = 0;     // buffers the per-buffer count array holds ([2][bufcnt_stride] u32)
  size_t bufcnt_stride = 0;

  // streaming (nmg_stream_begin): two staging halves, each a chunk in flight
  struct StreamSlot {
    uint8_t* h_stage = nullptr;  // pinned
    size_t cap = 0, len = 0;
    uint8_t* d_arena = nullptr;
    size_t dcap = 0;
    BufDesc* h_sdescs = nullptr;  // pinned schedule (sorted descriptors, then ranges)
    size_t hs_cap = 0;            // bytes
    BufDesc* d_sdescs = nullptr;
    size_t ds_cap = 0;            // bytes
    std::vector<BufDesc> descs;   // this chunk: offset in the slot, global seq, .pad = global index
    hipEvent_t copied = nullptr;  // H2D of the chunk done: the host may refill h_stage
    hipEvent_t done = nullptr;    // kernel of the chunk done: the device may refill d_arena
    bool used = false;
  };
  bool streaming = false, streamed = false;
  uint64_t chunk_cap = 0;
  uint32_t copy_threads = 1;
  std::unique_ptr<CopyPool> pool;  // copy_threads - 1 workers, started on first use
  StreamSlot slots[2];
  int cur_slot = 0;
  hipStream_t copy_stream = nullptr;

  // multi-GPU override of per-buffer counts (rank 0 reporting)
  bool counts_override = false;
  std::vector<uint32_t> ov_samples, ov_found;
  std::vector<uint64_t> ov_bytes;

  std::string last_error;
  float last_ms = 0.f;

  // multi-GPU (nmg_options.nb_gpus > 1): this handle holds the submitted
  // buffers, the table and the merged counters; `workers` (one engine per
  // device, worker 0 on this handle's device) analyse contiguous ranges
  std::vector<nmg_engine*> workers;
  std::vector<int> devices;
  bool multi = false, multi_distinct = false, multi_pending = false;
  uint64_t multi_found = 0;  // matched SAMPLEs of the workers (multi_finish)
  std::vector<void*> comms;  // ncclComm_t per worker (distinct devices)
  std::vector<uint8_t*> warena;
  std::vector<size_t> warena_cap;

  // partition-first path for large tables (nmg_route.h): the partitions of
  // the current table, and the per-analysis chunk pool
  bool route_ok = false;          // partitions built for the current table
  uint64_t route_launches = 0;    // analyses (or streamed chunks) that took the partition-first path
  uint32_t nparts = 0;
  PartInfo* d_parts = nullptr;
  uint64_t* d_pbounds = nullptr;  // [kMaxParts + 1] partition starts, ascending
  uint16_t* d_pdir = nullptr;     // [kRouteDir] the route pass's directory over them
  RSeg rsegs[kRouteSegs];         // its segments
  uint64_t route_tbase = 0;       // compact records: timestamps relative to this (XLayout)
  uint32_t nrsegs = 0;
  uint64_t* d_pe_keys = nullptr;  // [nparts][kPartSlots]
  uint4* d_pe_nodes = nullptr;    // [nparts][kPartSlots][2]
  uint2* d_pe_info = nullptr;     // [nparts][kPartSlots]
  uint32_t* d_pe_dir = nullptr;   // [nparts][kPartDir]
  uint32_t* d_pe_ids = nullptr;   // [table entries] entry id per table position (online tables; else null)
  uint32_t* d_pe_lrel = nullptr;  // [table entries] first packed LDS cell (online tables)
  uint32_t* d_pe_cmap = nullptr;  // packed cell -> histogram cell (online tables)
  uint4* d_rec16 = nullptr;       // chunk pool: [chunks][kChunk] (addr, ts) and X words
  uint32_t* d_cmeta = nullptr;
  unsigned long long* d_cmatch = nullptr;
  uint32_t* d_clist = nullptr;
  size_t route_chunk_cap = 0;
  uint4* d_items = nullptr;
  size_t items_cap = 0;
  uint32_t* d_chunk0 = nullptr;   // [grid + 1]
  uint32_t* d_used = nullptr;     // [grid]
  uint32_t* d_pcnt = nullptr;     // [grid][nparts]
  uint32_t* d_pbase = nullptr;    // [nparts]
  uint32_t* d_ctl = nullptr;      // [3] items, dequeue head, overflow records
  uint4* d_ovf16 = nullptr;       // overflow list (route pass, pool exhausted)
  unsigned long long* d_ovfx = nullptr;
  size_t ovf_cap = 0;
  size_t route_grid_cap = 0;
  bool sched_route = false;       // d_sdescs / d_ranges hold the analysis-order schedule
  uint32_t route_sched_key = 0;   // nparts (| tiny-pool switch) the pools were sized for
  bool route_pending = false;     // per-buffer match counts of the last route analysis not yet summed
  uint32_t route_grid = 0;
  XLayout route_xl{};

  // kDbgTiming (internal): per-wave phase cycles of the last launch
  uint64_t* d_dbg = nullptr;
  size_t dbg_cap = 0, dbg_len = 0;
};

#define HIP_TRY(h, expr)                                                        \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess) {                                                     \
      (h)->last_error = std::string(#expr) + ": " + hipGetErrorString(_e);      \
      return NMG_ERR_HIP;                                                       \
    }                                                                           \
  } while (0)

static int fail(nmg_engine* h, int code, const std::string& msg) {
  if (h) h->last_error = msg;
  return code;
}

namespace nmg {
uint32_t engine_nb_threads(nmg_engine* h) { return h->T; }
uint32_t engine_nb_entries(nmg_engine* h) { return h->E; }
uint32_t engine_flags(nmg_engine* h) { return h->flags; }
const std::vector<uint64_t>& engine_hist_base(nmg_engine* h) { return h->hist_base; }
const std::vector<uint64_t>& engine_npages(nmg_engine* h) { return h->npages; }
const std::vector<uint32_t>& engine_sparse_entries(nmg_engine* h) { return h->sparse_entries; }
void engine_set_error(nmg_engine* h, const std::string& msg) { h->last_error = msg; }
}  // namespace nmg

extern "C" const char* nmg_strerror(int status) {
  switch (status) {
    case NMG_OK: return "ok";
    case NMG_ERR_INVALID: return "invalid argument";
    case NMG_ERR_HIP: return "HIP runtime error";
    case NMG_ERR_NOMEM: return "out of host memory";
    case NMG_ERR_ZERO_SIZE: return "record with size 0 (the reference aborts, mem_sampling.c:857-860)";
    case NMG_ERR_TRUNCATED: return "SAMPLE record truncated at the end of its buffer";
    case NMG_ERR_STATE: return "call out of order";
    case NMG_ERR_RANGE: return "value out of range (thread rank, buffer size)";
    case NMG_ERR_CAPACITY: return "sparse page-histogram table full";
    case NMG_ERR_UNALIGNED: return "record size not a multiple of 8";
    case NMG_ERR_IO: return "report file could not be written";
    default: return "unknown error";
  }
}

// detail of the last failed nmg_create (no handle exists to hold it)
static thread_local std::string g_create_error;

extern "C" int nmg_get_last_error_detail(nmg_engine* h, char* buf, size_t len) {
  if (!buf || !len) return NMG_ERR_INVALID;
  snprintf(buf, len, "%s", h ? h->last_error.c_str() : g_create_error.c_str());
  return NMG_OK;
}

static void free_counters(nmg_engine* h) {
  (void)hipFree(h->d_sum64);
  (void)hipFree(h->d_min64);
  (void)hipFree(h->d_max64);
  (void)hipFree(h->d_hist);
  (void)hipFree(h->d_sparse_keys);
  (void)hipFree(h->d_sparse_vals);
  h->d_sum64 = h->d_min64 = h->d_max64 = nullptr;
  h->d_hist = nullptr;
  h->d_sparse_keys = nullptr;
  h->d_sparse_vals = nullptr;
  (void)hipFree(h->d_sparse_ck);
  h->d_sparse_ck = nullptr;
  (void)hipFree(h->d_objcw);
  h->d_objcw = nullptr;
  h->objcw_cap = 0;
  (void)hipFree(h->d_sparse_dirty);
  h->d_sparse_dirty = nullptr;
  (void)hipFree(h->d_pk64);
  h->d_pk64 = nullptr;
  (void)hipFree(h->d_tlog);
  h->d_tlog = nullptr;
  h->tlog_bytes = 0;
  (void)hipFree(h->d_tlog_cnt);
  h->d_tlog_cnt = nullptr;
  h->tlog_cnt_cap = 0;
}

// the lookup structures of one table (keys, node records, LDS tree or fences
// + directory, table-order entries)
static void free_lookup(nmg_engine* h) {
  (void)hipFree(h->d_keys);
  (void)hipFree(h->d_nodes);
  (void)hipFree(h->d_efences);
  (void)hipFree(h->d_enodes);
  (void)hipFree(h->d_ffences);
  (void)hipFree(h->d_fshift);
  (void)hipFree(h->d_dir);
  if (h->d_chain != h->d_entries) (void)hipFree(h->d_chain);
  h->d_keys = nullptr;
  h->d_nodes = nullptr;
  h->d_efences = nullptr;
  h->d_enodes = nullptr;
  h->d_ffences = nullptr;
  h->d_fshift = nullptr;
  h->d_dir = nullptr;
  h->d_chain = nullptr;
}

// the partitions of the partition-first path (built with the table)
static void free_route_table(nmg_engine* h) {
  (void)hipFree(h->d_parts);
  (void)hipFree(h->d_pbounds);
  (void)hipFree(h->d_pdir);
  (void)hipFree(h->d_pe_keys);
  (void)hipFree(h->d_pe_nodes);
  (void)hipFree(h->d_pe_info);
  (void)hipFree(h->d_pe_dir);
  (void)hipFree(h->d_pe_ids);
  (void)hipFree(h->d_pe_lrel);
  (void)hipFree(h->d_pe_cmap);
  h->d_pe_dir = nullptr;
  h->d_pe_ids = nullptr;
  h->d_pe_lrel = nullptr;
  h->d_pe_cmap = nullptr;
  h->d_parts = nullptr;
  h->d_pbounds = nullptr;
  h->d_pdir = nullptr;
  h->d_pe_keys = nullptr;
  h->d_pe_nodes = nullptr;
  h->d_pe_info = nullptr;
  h->route_ok = false;
  h->nparts = 0;
}

// the per-analysis buffers of the partition-first path
static void free_route_pool(nmg_engine* h) {
  for (void* q : {(void*)h->d_rec16, (void*)h->d_cmeta, (void*)h->d_cmatch, (void*)h->d_clist,
                  (void*)h->d_items, (void*)h->d_chunk0, (void*)h->d_used, (void*)h->d_pcnt, (void*)h->d_pbase,
                  (void*)h->d_ctl, (void*)h->d_ovf16, (void*)h->d_ovfx})
    (void)hipFree(q);
  h->d_rec16 = nullptr;
  h->d_cmeta = nullptr;
  h->d_cmatch = nullptr;
  h->d_clist = nullptr;
  h->d_items = nullptr;
  h->d_chunk0 = nullptr;
  h->d_used = nullptr;
  h->d_pcnt = nullptr;
  h->d_pbase = nullptr;
  h->d_ctl = nullptr;
  h->d_ovf16 = nullptr;
  h->d_ovfx = nullptr;
  h->ovf_cap = 0;
  h->route_chunk_cap = h->items_cap = h->route_grid_cap = 0;
  h->route_pending = false;
}

// The lookup structures' pointers and shape, moved out of the engine so that
// a new table can be built beside them (nmg_update_objects swaps only on
// success).
struct LookupSet {
  uint64_t* keys;
  DevEntry* nodes;
  uint64_t* efences;
  DevEntry* enodes;
  uint64_t* ffences;
  uint8_t* fshift;
  uint2* dir;
  DevEntry* chain;
  uint32_t K, elevels, nb_fences, fence_log2, dir_log2;
};

static LookupSet take_lookup(nmg_engine* h) {
  LookupSet l{h->d_keys, h->d_nodes, h->d_efences, h->d_enodes, h->d_ffences, h->d_fshift, h->d_dir, h->d_chain,
              h->K, h->elevels, h->nb_fences, h->fence_log2, h->dir_log2};
  h->d_keys = nullptr;
  h->d_nodes = nullptr;
  h->d_efences = nullptr;
  h->d_enodes = nullptr;
  h->d_ffences = nullptr;
  h->d_fshift = nullptr;
  h->d_dir = nullptr;
  h->d_chain = nullptr;
  return l;
}

static void put_lookup(nmg_engine* h, const LookupSet& l) {
  h->d_keys = l.keys;
  h->d_nodes = l.nodes;
  h->d_efences = l.efences;
  h->d_enodes = l.enodes;
  h->d_ffences = l.ffences;
  h->d_fshift = l.fshift;
  h->d_dir = l.dir;
  h->d_chain = l.chain;
  h->K = l.K;
  h->elevels = l.elevels;
  h->nb_fences = l.nb_fences;
  h->fence_log2 = l.fence_log2;
  h->dir_log2 = l.dir_log2;
}

static void free_table(nmg_engine* h) {
  free_route_table(h);
  free_lookup(h);
  (void)hipFree(h->d_entries);
  h->d_entries = nullptr;
}

static hipError_t alloc_copy(nmg_engine* h, void** dptr, const void* src, size_t bytes) {
  hipError_t e = hipMalloc(dptr, bytes ? bytes : 16);
  if (e != hipSuccess) return e;
  if (bytes) return hipMemcpyAsync(*dptr, src, bytes, hipMemcpyHostToDevice, h->stream);
  return hipSuccess;
}

// keys strictly ascending, every key with >= 1 entry, entry_off a prefix array over n entries
static int check_table(nmg_engine* h, const uint64_t* keys, const uint32_t* entry_off, uint32_t nb_keys,
                       uint32_t n) {
  if (entry_off && (entry_off[0] != 0 || entry_off[nb_keys] != n))
    return fail(h, NMG_ERR_INVALID, "entry_off[0] must be 0 and entry_off[nb_keys] == the number of entries");
  for (uint32_t i = 0; i < nb_keys; i++) {
    if (entry_off[i + 1] <= entry_off[i]) return fail(h, NMG_ERR_INVALID, "every key needs >= 1 entry");
    if (i && keys[i] <= keys[i - 1]) return fail(h, NMG_ERR_INVALID, "keys must be strictly ascending");
  }
  return NMG_OK;
}

static int multi_create(nmg_engine* h, const nmg_options* opt);
static void multi_destroy(nmg_engine* h);

static_assert(offsetof(nmg_options, nb_gpus) == NMG_OPTIONS_V1_SIZE, "first nmg_options version");

// internal (ablation / test) flag bits are accepted only with NMG_INTERNAL_FLAGS
// set in the environment: they change what the kernels compute
static bool internal_flags_allowed() {
  const char* e = getenv("NMG_INTERNAL_FLAGS");
  return e && *e && strcmp(e, "0") != 0;
}

static int create_impl(nmg_engine** out, const nmg_options* opt_in, size_t opt_size, bool v2_declared);

// nmg_create reads the whole current struct, but a binary built against the
// first version (32 bytes) may call it too: bytes 32..47 are then whatever
// follows its struct.  So, as before the v2 fields existed, nb_gpus / devices
// count only with abi_version == NMG_OPTIONS_ABI and are otherwise ignored;
// the rejection of a v2 caller's nb_gpus > 1 without the ABI word is
// nmg_create_ex's, whose opt_size says the caller declared those fields.
extern "C" int nmg_create(nmg_engine** out, const nmg_options* opt) {
  return create_impl(out, opt, sizeof(nmg_options), false);
}

extern "C" int nmg_create_ex(nmg_engine** out, const nmg_options* opt_in, size_t opt_size) {
  return create_impl(out, opt_in, opt_size, opt_size >= sizeof(nmg_options));
}

static int create_impl(nmg_engine** out, const nmg_options* opt_in, size_t opt_size, bool v2_declared) {
  if (!out) return NMG_ERR_INVALID;
  *out = nullptr;
  // only the caller's bytes of the struct are read (a first-version caller's
  // struct ends at NMG_OPTIONS_V1_SIZE); the rest is zero
  nmg_options o2{};
  const nmg_options* opt = nullptr;
  if (opt_in) {
    if (opt_size < NMG_OPTIONS_V1_SIZE) {
      g_create_error = "nmg_create_ex: opt_size smaller than the first nmg_options version";
      return NMG_ERR_INVALID;
    }
    memcpy(&o2, opt_in, std::min(opt_size, sizeof(nmg_options)));
    opt = &o2;
    if ((o2.flags & ~(uint32_t)NMG_F_ALL) && !internal_flags_allowed()) {
      char msg[128];
      snprintf(msg, sizeof(msg), "nmg_create: flags 0x%x outside NMG_F_ALL (0x%x)", o2.flags & ~(uint32_t)NMG_F_ALL,
               (uint32_t)NMG_F_ALL);
      g_create_error = msg;
      return NMG_ERR_INVALID;
    }
    if (o2.abi_version != NMG_OPTIONS_ABI) {
      if (v2_declared && o2.nb_gpus > 1) {  // (a multi-GPU caller without the ABI word: not silently one GPU)
        g_create_error = "nmg_create: nb_gpus > 1 needs abi_version = NMG_OPTIONS_ABI";
        return NMG_ERR_INVALID;
      }
      o2.nb_gpus = 0;
      o2.devices = nullptr;
    }
  }
  nmg_engine* h = new (std::nothrow) nmg_engine();
  if (!h) return NMG_ERR_NOMEM;
  if (opt) {
    h->device = opt->nb_gpus >= 1 && opt->devices ? opt->devices[0] : opt->device;
    h->flags = opt->flags;
    h->T = opt->nb_threads ? opt->nb_threads : 1;
    h->copy_threads = opt->copy_threads ? opt->copy_threads : 1;
    if (opt->hist_budget_bytes) h->hist_budget = opt->hist_budget_bytes;
    if (opt->sparse_capacity) {
      uint64_t c = 1;
      while (c < opt->sparse_capacity) c <<= 1;
      h->sparse_cap = c;
    }
  }
  if (h->T > NMG_MAX_THREADS || h->sparse_cap > (1ull << 31)) {
    delete h;
    return NMG_ERR_RANGE;
  }
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev <= 0 || h->device < 0 || h->device >= ndev) {
    g_create_error = std::string("hipGetDeviceCount: ") + hipGetErrorString(e) + " (" + std::to_string(ndev) +
                     " devices, device " + std::to_string(h->device) + ")";
    delete h;
    return NMG_ERR_HIP;
  }
  const char* what = "hipSetDevice";
  e = hipSetDevice(h->device);
  if (e == hipSuccess) {
    what = "hipStreamCreateWithFlags";
    e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
  }
  if (e == hipSuccess) {
    what = "hipEventCreate";
    e = hipEventCreate(&h->ev0);
    if (e == hipSuccess) e = hipEventCreate(&h->ev1);
  }
  if (e != hipSuccess) {
    g_create_error = std::string(what) + ": " + hipGetErrorString(e);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return NMG_ERR_HIP;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, h->device) == hipSuccess) h->num_cus = prop.multiProcessorCount;
  if (opt && (opt->nb_gpus > 1 || (opt->flags & kDbgMultiRccl))) {
    const int rc = multi_create(h, opt);
    if (rc) {
      g_create_error = h->last_error;
      nmg_destroy(h);
      return rc;
    }
  }
  *out = h;
  return NMG_OK;
}

extern "C" void nmg_destroy(nmg_engine* h) {
  if (!h) return;
  multi_destroy(h);
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  free_table(h);
  free_counters(h);
  free_route_pool(h);
  for (const auto& r : h->hostregs) (void)hipHostUnregister(r.pages);
  (void)hipFree(h->d_cells_rows);
  (void)hipFree(h->d_arena);
  (void)hipFree(h->d_descs);
  (void)hipFree(h->d_bufcnt);
  (void)hipFree(h->d_found);
  (void)hipFree(h->d_scratch);
  (void)hipFree(h->d_sdescs);
  (void)hipFree(h->d_ranges);
  (void)hipFree(h->d_dbg);
  (void)hipFree(h->d_smatch);
  if (h->h_stage) (void)hipHostFree(h->h_stage);
  if (h->copy_stream) (void)hipStreamSynchronize(h->copy_stream);
  for (auto& sl : h->slots) {
    if (sl.h_stage) (void)hipHostFree(sl.h_stage);
    if (sl.h_sdescs) (void)hipHostFree(sl.h_sdescs);
    (void)hipFree(sl.d_arena);
    (void)hipFree(sl.d_sdescs);
    if (sl.copied) (void)hipEventDestroy(sl.copied);
    if (sl.done) (void)hipEventDestroy(sl.done);
  }
  if (h->copy_stream) (void)hipStreamDestroy(h->copy_stream);
  if (h->ev0) (void)hipEventDestroy(h->ev0);
  if (h->ev1) (void)hipEventDestroy(h->ev1);
  for (int i = 0; i < nmg_engine::kRing; i++) {
    if (h->ring0[i]) (void)hipEventDestroy(h->ring0[i]);
    if (h->ring1[i]) (void)hipEventDestroy(h->ring1[i]);
    if (h->ringm[i]) (void)hipEventDestroy(h->ringm[i]);
    if (h->ringr[i]) (void)hipEventDestroy(h->ringr[i]);
  }
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

static int multi_finish(nmg_engine* h);

extern "C" int nmg_reset_counters(nmg_engine* h) {
  if (h) h->epoch++;
  if (!h) return NMG_ERR_INVALID;
  if (!h->have_table) return fail(h, NMG_ERR_STATE, "nmg_reset_counters before nmg_set_objects");
  if (h->multi_pending) {  // the merges in flight write the arrays being reset: let them finish (their
                           // per-buffer gathers are not needed)
    h->multi_pending = false;
    for (nmg_engine* w : h->workers) {
      HIP_TRY(h, hipSetDevice(w->device));
      HIP_TRY(h, hipStreamSynchronize(w->stream));
    }
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
  }
  for (nmg_engine* w : h->workers) {
    const int rc = nmg_reset_counters(w);
    if (rc) return fail(h, rc, w->last_error);
  }
  if (h->multi && h->counts_override) {  // merged per-buffer counts (multi_finish)
    std::fill(h->ov_samples.begin(), h->ov_samples.end(), 0u);
    std::fill(h->ov_found.begin(), h->ov_found.end(), 0u);
  }
  h->multi_found = 0;
  HIP_TRY(h, hipSetDevice(h->device));
  h->route_pending = false;  // the counts found_kernel would add are zeroed here
  ResetParams r;
  memset(&r, 0, sizeof(r));
  r.sum64 = h->d_sum64;
  r.n_sum64 = h->n_sum64;
  r.min64 = h->d_min64;
  r.n_min64 = h->n_min64;
  r.max64 = h->d_max64;
  r.n_max64 = h->n_max64;
  r.found = h->d_found;
  const uint64_t hist_bytes = h->hist_cells * h->T * 4;
  if (hist_bytes & 15) HIP_TRY(h, hipMemsetAsync(h->d_hist, 0, hist_bytes, h->stream));  // (16 B multiple always)
  r.hist = reinterpret_cast<uint4*>(h->d_hist);
  r.n_hist16 = hist_bytes / 16;
  if (h->d_sparse_keys) {
    r.sparse_keys = h->d_sparse_keys;
    r.sparse_vals = h->d_sparse_vals;
    r.sparse_cap = h->sparse_cap;
    // reset #n reads the flag the analyses since reset #n-1 set, and clears
    // the one the analyses after it will set
    r.sparse_read = h->d_sparse_dirty + (h->nreset & 1);
    r.sparse_clear = h->d_sparse_dirty + ((h->nreset + 1) & 1);
  }
  // (a pending descriptor upload zeroes the per-buffer counts itself)
  if (h->d_bufcnt && (h->streaming || h->streamed || (!h->descs_dirty && !h->descs.empty()))) {
    r.bufcnt = h->d_bufcnt;
    r.n_bufcnt = h->bufcnt_stride * 2;
  }
  // grid sized to the work (~16 stores per thread of the longest array), at
  // most 4 workgroups per CU: small tables reset in one short launch
  const uint64_t longest = std::max<uint64_t>({r.n_hist16, r.n_sum64, r.n_min64, r.sparse_cap, r.n_bufcnt, 1});
  const uint32_t rgrid = (uint32_t)std::min<uint64_t>((longest + 256 * 16 - 1) / (256 * 16), (uint64_t)h->num_cus * 4);
  HIP_TRY(h, launch_reset(rgrid, h->stream, r));
  h->nreset++;
  return NMG_OK;
}

// Lookup structure of a table larger than kLdsNodes keys (see lower_key):
// fence b = keys[b << fence_log2] (<= kMaxFences fences, Eytzinger order),
// and per bucket a directory of 2^dir_log2 equal-width slots over the bucket's
// key span [first key, last key].
struct BigLookup {
  uint32_t nb_fences = 0, fence_log2 = 0, dir_log2 = 0;
  std::vector<uint64_t> efences;  // [kMaxFences + 1]
  std::vector<uint8_t> shift;     // [nb_fences]
  std::vector<uint2> dir;         // [nb_fences << dir_log2]
};

static void build_big_lookup(const uint64_t* keys, uint32_t K, bool no_dir, BigLookup& bl) {
  while (((uint64_t)K + (1u << bl.fence_log2) - 1) >> bl.fence_log2 > kMaxFences) bl.fence_log2++;
  const uint32_t S = 1u << bl.fence_log2;
  bl.nb_fences = (uint32_t)(((uint64_t)K + S - 1) >> bl.fence_log2);
  // Eytzinger order: an in-order walk of the complete 12-level tree hands out
  // the fences in sorted order; the slots after the last fence hold ~0
  bl.efences.assign(kMaxFences + 1, ~0ull);
  {
    uint32_t r = 0, i = 1;
    std::vector<uint32_t> stack;
    while (i <= kMaxFences || !stack.empty()) {
      while (i <= kMaxFences) {
        stack.push_back(i);
        i = 2 * i;
      }
      i = stack.back();
      stack.pop_back();
      if (r < bl.nb_fences) bl.efences[i] = keys[(uint64_t)r << bl.fence_log2];
      r++;
      i = 2 * i + 1;
    }
  }
  bl.shift.assign(bl.nb_fences, kShiftSearch);
  // bucket-relative indices and counts are 16-bit: S <= 2^16 (larger
  // buckets -- more than 4095 << 16 keys -- are binary-searched)
  if (S == 1 || S > (1u << 16) || no_dir) return;
  bl.dir_log2 = bl.fence_log2 + 1;  // two slots per key
  const uint32_t D = 1u << bl.dir_log2;
  bl.dir.assign((size_t)bl.nb_fences << bl.dir_log2, make_uint2(0, 0));
  for (uint32_t b = 0; b < bl.nb_fences; b++) {
    const uint32_t k0 = b * S, k1 = std::min<uint64_t>((uint64_t)k0 + S, K);
    const uint64_t f = keys[k0], span = keys[k1 - 1] - f;
    uint32_t sh = 0;
    while (sh < 64 && (span >> sh) >= D) sh++;
    if (sh > 32) continue;  // slot offsets must fit 32 bits: binary search instead
    bl.shift[b] = (uint8_t)sh;
    uint2* dd = &bl.dir[(size_t)b << bl.dir_log2];
    uint32_t k = k0;  // largest key <= slot start
    for (uint32_t j = 0; j < D; j++) {
      const uint64_t s0 = (uint64_t)j << sh;  // slot [s0, s0 + 2^sh) relative to f; the last slot is open
      while (k + 1 < k1 && keys[k + 1] - f <= s0) k++;
      uint32_t c = 0;
      while (k + 1 + c < k1 && (j == D - 1 || keys[k + 1 + c] - f < s0 + (1ull << sh))) c++;
      dd[j].x = (k - k0) | (std::min<uint32_t>(c, 0xffffu) << 16);
      dd[j].y = c ? (uint32_t)(keys[k + 1] - f - s0) : 0u;
    }
  }
}

// Lookup structures of a flattened table whose entries, in table order, are
// chain[] (ids in DevEntry::id): node records, then the LDS Eytzinger tree
// (<= kLdsNodes keys) or the fences + directory of the large-table path.
// chain_dev: chain already on the device (the by-id array), else uploaded.
static int build_lookup(nmg_engine* h, const uint64_t* keys, const uint32_t* entry_off, uint32_t nb_keys,
                        const std::vector<DevEntry>& chain, DevEntry* chain_dev) {
  h->K = nb_keys;
  std::vector<DevEntry> nodes(nb_keys);
  for (uint32_t k = 0; k < nb_keys; k++) {
    nodes[k] = chain[entry_off[k]];
    nodes[k].first = entry_off[k];
    nodes[k].count = entry_off[k + 1] - entry_off[k];
  }
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_keys, keys, (size_t)nb_keys * 8));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_nodes, nodes.data(), (size_t)nb_keys * sizeof(DevEntry)));
  if (chain_dev) h->d_chain = chain_dev;
  else HIP_TRY(h, alloc_copy(h, (void**)&h->d_chain, chain.data(), chain.size() * sizeof(DevEntry)));
  if (nb_keys <= kLdsNodes) {
    // Eytzinger (BFS) order for the LDS search: an in-order walk of the
    // complete tree of 2^L - 1 nodes hands out the keys in sorted order; the
    // slots after the last key are ~0 keys carrying a copy of the last node
    // (reached only for addr == UINT64_MAX, where the last key is the answer)
    h->elevels = 0;
    while (((1u << h->elevels) - 1) < nb_keys) h->elevels++;
    const uint32_t n = 1u << h->elevels;
    std::vector<uint64_t> ef(n, ~0ull);
    std::vector<DevEntry> en(n);
    memset(en.data(), 0, n * sizeof(DevEntry));
    uint32_t r = 0;
    std::vector<uint32_t> stack;
    uint32_t i = 1;
    while (i < n || !stack.empty()) {  // iterative in-order walk
      while (i < n) {
        stack.push_back(i);
        i = 2 * i;
      }
      i = stack.back();
      stack.pop_back();
      if (r < nb_keys) {
        ef[i] = keys[r];
        en[i] = nodes[r];
      } else if (nb_keys) {
        en[i] = nodes[nb_keys - 1];
      }
      r++;
      i = 2 * i + 1;
    }
    HIP_TRY(h, alloc_copy(h, (void**)&h->d_efences, ef.data(), n * 8));
    HIP_TRY(h, alloc_copy(h, (void**)&h->d_enodes, en.data(), n * sizeof(DevEntry)));
  }
  h->nb_fences = h->fence_log2 = h->dir_log2 = 0;
  if (nb_keys > kLdsNodes) {
    BigLookup bl;
    build_big_lookup(keys, nb_keys, (h->flags & kDbgNoDir) != 0, bl);
    h->nb_fences = bl.nb_fences;
    h->fence_log2 = bl.fence_log2;
    h->dir_log2 = bl.dir_log2;
    HIP_TRY(h, alloc_copy(h, (void**)&h->d_ffences, bl.efences.data(), bl.efences.size() * 8));
    HIP_TRY(h, alloc_copy(h, (void**)&h->d_fshift, bl.shift.data(), bl.shift.size()));
    HIP_TRY(h, alloc_copy(h, (void**)&h->d_dir, bl.dir.data(), bl.dir.size() * sizeof(uint2)));
  }
  return NMG_OK;
}

// The route pass's partition search (route_partition, nmg_route.hip) over
// the P ascending partition starts b: up to kRouteSegs segments, split at the
// gaps between consecutive starts that dwarf the median gap (address spaces
// are clustered: globals, heap, mmap'd regions, the stack), each with
// directory slots in proportion to its partitions.  Slot j of a segment holds
// the last partition starting at or before the slot start, and how many
// starts lie inside the slot (saturated at kDirCntSat: search to the
// segment's last partition).
static void route_segments(const uint64_t* b, uint32_t P, RSeg* seg, uint32_t* nseg, std::vector<uint16_t>& dir) {
  std::vector<uint32_t> cuts{0};  // segment k starts at partition cuts[k]
  if (P > 1) {
    std::vector<uint64_t> gaps(P - 1);
    for (uint32_t q = 0; q + 1 < P; q++) gaps[q] = b[q + 1] - b[q];
    std::vector<uint64_t> med(gaps);
    std::nth_element(med.begin(), med.begin() + med.size() / 2, med.end());
    const uint64_t m = std::max<uint64_t>(med[med.size() / 2], 1);
    std::vector<uint32_t> idx(P - 1);
    for (uint32_t q = 0; q + 1 < P; q++) idx[q] = q;
    std::sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) { return gaps[x] > gaps[y]; });
    for (uint32_t i = 0; i < idx.size() && cuts.size() < kRouteSegs; i++) {
      if (gaps[idx[i]] / 64 <= m) break;
      cuts.push_back(idx[i] + 1);
    }
    std::sort(cuts.begin(), cuts.end());
  }
  const uint32_t S = (uint32_t)cuts.size();
  dir.assign(kRouteDir, 0);
  uint32_t used = 0;
  for (uint32_t k = 0; k < kRouteSegs; k++) {
    if (k >= S) {
      seg[k] = RSeg{~0ull, 0, 1, 0, 0};
      continue;
    }
    const uint32_t qa = cuts[k], qb = k + 1 < S ? cuts[k + 1] : P;
    const uint32_t ns = (uint32_t)((uint64_t)(kRouteDir - S) * (qb - qa) / P) + 1;
    const uint64_t span = b[qb - 1] - b[qa];
    uint32_t sh = 0;
    while (sh < 63 && (span >> sh) >= ns) sh++;
    seg[k] = RSeg{b[qa], used, ns, sh, qb - 1};
    uint32_t q = qa;
    for (uint32_t j = 0; j < ns; j++) {
      // slot [s0, s1) relative to the segment start
      const unsigned __int128 s0 = (unsigned __int128)j << sh, s1 = (unsigned __int128)(j + 1) << sh;
      while (q + 1 < qb && (unsigned __int128)(b[q + 1] - b[qa]) <= s0) q++;
      uint32_t c = 0;
      if (j == ns - 1) c = qb - 1 - q;
      else
        while (q + 1 + c < qb && (unsigned __int128)(b[q + 1 + c] - b[qa]) < s1) c++;
      dir[used + j] = (uint16_t)(q | (std::min(c, kDirCntSat) << 11));
    }
    used += ns;
  }
  *nseg = S;
}

// Partitions of the partition-first path (nmg_route.h): runs of consecutive
// keys, each at most kPartKeys keys and kPartEntries entries, and -- where
// the keys allow it -- at most kPartCells dense page cells over all threads,
// so that a partition's lookup tree, node records, object counters and page
// cells fit one workgroup's LDS.  A key range owns a range of table
// positions; `ids` (an online table, nmg_update_objects) maps a position to
// its entry id (null: the id is the position).  An online table's entries
// have their page cells in id order, scattered over the address order, so
// its partitions are not cut by cells (the cells of a partition whose span is
// too wide for LDS take global atomics).  Only for engines that count per
// object (NMG_F_MATCH_SAMPLES) without the dump modes' per-sample output or
// per-object levels; otherwise the table keeps attribute_kernel.
static int build_partitions(nmg_engine* h, const uint64_t* keys, const uint32_t* entry_off, uint32_t K,
                            const std::vector<DevEntry>& dev, const uint32_t* ids) {
  free_route_table(h);
  if (K <= kLdsNodes || !(h->flags & NMG_F_MATCH_SAMPLES) || (h->flags & (NMG_F_SAMPLE_MATCHES | NMG_F_OBJECT_LEVELS)))
    return NMG_OK;
  if (ids) {  // the identity map is the offline case
    uint32_t e = 0;
    while (e < entry_off[K] && ids[e] == e) e++;
    if (e == entry_off[K]) ids = nullptr;
  }
  if (ids && h->hist_cells >= (1ull << 31)) return NMG_OK;  // (cell indices of an online table: 32-bit)
  const uint64_t T = h->T;
  std::vector<PartInfo> parts;
  // an online table: the partition's dense cells packed in LDS in table
  // order (lrel: an entry's first LDS cell per table position; cmap: the
  // histogram cell of every packed cell, per partition from PartInfo::cmap)
  std::vector<uint32_t> lrel, cmap;
  if (ids) lrel.assign(entry_off[K], kEmpty32);
  uint32_t k = 0;
  while (k < K) {
    PartInfo pi;
    memset(&pi, 0, sizeof(pi));
    pi.k0 = k;
    pi.e0 = entry_off[k];
    pi.cmap = ~0u;
    uint64_t cb = ~0ull, ce = 0, cc = 0;  // dense cells in [cb, ce), cc of them
    while (k < K && k - pi.k0 < kPartKeys) {
      // a partition's keys span less than 2^(kAddrBits - 1) bytes, so that the
      // compact records' address field (relative to the partition's first key)
      // holds every address its objects cover: a run of keys across a wide gap
      // in the address space (the heap, then the stack) starts a new partition
      if (k > pi.k0 && keys[k] - keys[pi.k0] >= (1ull << (kAddrBits - 1))) break;
      const uint32_t ea = entry_off[k], eb = entry_off[k + 1];
      if (eb - pi.e0 > kPartEntries) {
        if (k == pi.k0) return NMG_OK;  // one address reused more than kPartEntries times: keep attribute_kernel
        break;
      }
      uint64_t ncb = cb, nce = ce, ncc = cc;
      for (uint32_t e = ea; e < eb; e++)
        if (dev[e].hist != kHistSparse) {
          const uint64_t np = h->npages[dev[e].id];
          ncb = std::min<uint64_t>(ncb, dev[e].hist);
          nce = std::max<uint64_t>(nce, dev[e].hist + np);
          ncc += np;
        }
      if (k > pi.k0 && ncb != ~0ull && (ids ? ncc : nce - ncb) * T > kPartCells)
        break;  // (one key alone may exceed: global cells)
      cb = ncb;
      ce = nce;
      cc = ncc;
      k++;
    }
    pi.nk = k - pi.k0;
    pi.ne = entry_off[k] - pi.e0;
    pi.cb = cb == ~0ull ? 0 : cb;
    pi.span = cb == ~0ull ? 0 : (uint32_t)(ce - cb);
    pi.pages_lds = pi.span && (uint64_t)pi.span * T <= kPartCells;
    if (ids && cc && cc * T <= kPartCells) {  // online: the cells packed (cmap), always in LDS
      pi.cmap = (uint32_t)cmap.size();
      pi.span = (uint32_t)cc;
      pi.pages_lds = 1;
      uint32_t off = 0;
      for (uint32_t e = pi.e0; e < pi.e0 + pi.ne; e++)
        if (dev[e].hist != kHistSparse) {
          const uint32_t np = (uint32_t)h->npages[dev[e].id];
          lrel[e] = off;
          for (uint32_t g = 0; g < np; g++) cmap.push_back((uint32_t)(dev[e].hist + g));
          off += np;
        }
    }
    const uint64_t kspan = keys[k - 1] - keys[pi.k0];
    while (pi.dshift < 63 && (kspan >> pi.dshift) >= kPartDir) pi.dshift++;
    parts.push_back(pi);
    if (parts.size() > kMaxParts) return NMG_OK;  // too many partitions for the route pass's LDS tree
  }
  const uint32_t P = (uint32_t)parts.size();
  // the compact records' timestamp base: the earliest allocation (a sample
  // before it can only match objects allocated at time 0, and escapes)
  h->route_tbase = ~0ull;
  for (const DevEntry& d : dev)
    if (d.alloc) h->route_tbase = std::min<uint64_t>(h->route_tbase, d.alloc);
  if (h->route_tbase == ~0ull) h->route_tbase = 0;
  // per partition: keys ascending with their newest entry's node record and
  // info, and a directory over the key span: slot j starts at first key + (j
  // << dshift) and holds the index of the largest key <= that start and the
  // number of keys inside the slot (the last slot: every key after its start)
  std::vector<uint64_t> pk((size_t)P * kPartSlots, ~0ull);
  std::vector<uint4> pn((size_t)P * kPartSlots * 2, make_uint4(0, 0, 0, 0));
  std::vector<uint2> pinf((size_t)P * kPartSlots, make_uint2(kEmpty32, 0));
  std::vector<uint32_t> pdir((size_t)P * kPartDir, 0);
  for (uint32_t q = 0; q < P; q++) {
    const PartInfo& pi = parts[q];
    for (uint32_t r = 0; r < pi.nk; r++) {
      const uint32_t kk = pi.k0 + r;
      const DevEntry& d = dev[entry_off[kk]];
      const size_t o = (size_t)q * kPartSlots + r;
      pk[o] = keys[kk];
      pn[2 * o] = make_uint4((uint32_t)d.addr, (uint32_t)(d.addr >> 32), (uint32_t)d.end, (uint32_t)(d.end >> 32));
      pn[2 * o + 1] = make_uint4((uint32_t)d.alloc, (uint32_t)(d.alloc >> 32), (uint32_t)d.free, (uint32_t)(d.free >> 32));
      const uint32_t older = entry_off[kk + 1] - entry_off[kk] > 1 ? 0x80000000u : 0u;
      const uint32_t hrel = d.hist == kHistSparse ? kEmpty32
                            : pi.cmap != ~0u         ? lrel[entry_off[kk]]
                                                     : (uint32_t)(d.hist - pi.cb);
      pinf[o] = make_uint2(hrel, (entry_off[kk] - pi.e0) | older);
    }
    const uint64_t f = keys[pi.k0];
    uint32_t lo = 0;
    for (uint32_t j = 0; j < kPartDir; j++) {
      const uint64_t s0 = (uint64_t)j << pi.dshift;  // slot start relative to the first key
      while (lo + 1 < pi.nk && keys[pi.k0 + lo + 1] - f <= s0) lo++;
      uint32_t c = 0;
      while (lo + 1 + c < pi.nk &&
             (j == kPartDir - 1 || keys[pi.k0 + lo + 1 + c] - f < s0 + (1ull << pi.dshift)))
        c++;
      pdir[(size_t)q * kPartDir + j] = lo | (c << 16);
    }
  }
  // the route pass's partition search: the partitions' first keys ascending,
  // and a directory over them (route_segments)
  std::vector<uint64_t> pb(kMaxParts + 1, ~0ull);
  for (uint32_t q = 0; q < P; q++) pb[q] = keys[parts[q].k0];
  std::vector<uint16_t> rdir;
  route_segments(pb.data(), P, h->rsegs, &h->nrsegs, rdir);
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_parts, parts.data(), parts.size() * sizeof(PartInfo)));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_pbounds, pb.data(), pb.size() * 8));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_pdir, rdir.data(), rdir.size() * 2));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_pe_keys, pk.data(), pk.size() * 8));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_pe_nodes, pn.data(), pn.size() * sizeof(uint4)));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_pe_info, pinf.data(), pinf.size() * sizeof(uint2)));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_pe_dir, pdir.data(), pdir.size() * 4));
  if (ids) {
    HIP_TRY(h, alloc_copy(h, (void**)&h->d_pe_ids, ids, (size_t)entry_off[K] * 4));
    HIP_TRY(h, alloc_copy(h, (void**)&h->d_pe_lrel, lrel.data(), lrel.size() * 4));
    if (!cmap.empty()) HIP_TRY(h, alloc_copy(h, (void**)&h->d_pe_cmap, cmap.data(), cmap.size() * 4));
  }
  HIP_TRY(h, hipStreamSynchronize(h->stream));  // (pageable sources)
  h->nparts = P;
  h->route_ok = true;
  return NMG_OK;
}

extern "C" int nmg_set_objects(nmg_engine* h, const uint64_t* keys, const uint32_t* entry_off,
                               uint32_t nb_keys, const nmg_object* entries, uint32_t nb_entries) {
  if (h) h->epoch++;
  Range range("nmg_set_objects");
  if (!h || (nb_keys && (!keys || !entry_off)) || (nb_entries && !entries))
    return NMG_ERR_INVALID;
  int rc = check_table(h, keys, entry_off, nb_keys, nb_entries);
  if (rc) return rc;
  if (nb_entries >= (1u << 31)) return fail(h, NMG_ERR_RANGE, "too many entries");
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  free_table(h);
  free_counters(h);
  h->K = nb_keys;
  h->E = nb_entries;

  // page-histogram layout: dense [page][thread] block per entry within the
  // budget, otherwise sparse hashed cells (e.g. the 412 GB [stack] range)
  const uint64_t T = h->T;
  const uint64_t max_cells_per_entry = 1ull << 24;
  h->hist_base.assign(nb_entries, kHistSparse);
  h->npages.resize(nb_entries);
  h->buffer_size.resize(nb_entries);
  h->entry_addr.resize(nb_entries);
  h->objects.assign(entries, entries + nb_entries);
  h->order.clear();
  h->sparse_entries.clear();
  h->hist_cells = 0;
  std::vector<DevEntry> dev(nb_entries);
  const bool want_hist = (h->flags & NMG_F_PAGE_HIST) && (h->flags & NMG_F_MATCH_SAMPLES);
  const uint64_t budget_cells = h->hist_budget / 4;
  for (uint32_t e = 0; e < nb_entries; e++) {
    const nmg_object& o = entries[e];
    DevEntry& d = dev[e];
    memset(&d, 0, sizeof(d));
    d.addr = o.buffer_addr;
    d.end = o.buffer_addr + o.buffer_size;
    d.alloc = o.alloc_date;
    d.free = o.free_date;
    uint64_t np = o.buffer_size / kPageSize + 1;
    h->npages[e] = np;
    h->buffer_size[e] = o.buffer_size;
    h->entry_addr[e] = o.buffer_addr;
    d.hist = kHistSparse;
    d.sidx = ~0u;
    d.id = e;
    if (!want_hist) continue;
    // dense cells: histogram index = thread * hist_cells + hist_base(entry) + page
    if (np * T <= max_cells_per_entry && (h->hist_cells + np) * T <= budget_cells &&
        h->hist_cells + np < 0xffffffffull) {
      d.hist = h->hist_cells;
      h->hist_base[e] = h->hist_cells;
      h->hist_cells += np;
    } else {
      if (h->sparse_entries.size() >= (1u << 22)) return fail(h, NMG_ERR_CAPACITY, "too many sparse entries");
      d.sidx = (uint32_t)h->sparse_entries.size();
      h->sparse_entries.push_back(e);
    }
  }
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_entries, dev.data(), (size_t)nb_entries * sizeof(DevEntry)));
  rc = build_lookup(h, keys, entry_off, nb_keys, dev, h->d_entries);
  if (rc) return rc;
  rc = build_partitions(h, keys, entry_off, nb_keys, dev, nullptr);
  if (rc) return rc;
  h->dev_entries = std::move(dev);


  h->n_sum64 = 2 * kGlobalSums + (uint64_t)nb_entries * 4;
  if (h->flags & NMG_F_OBJECT_LEVELS) h->n_sum64 += (uint64_t)nb_entries * 2 * kLevelWords;
  h->n_min64 = 36 + (uint64_t)nb_entries + 1;
  h->n_max64 = 36;
  HIP_TRY(h, hipMalloc(&h->d_sum64, h->n_sum64 * 8));
  HIP_TRY(h, hipMalloc(&h->d_min64, h->n_min64 * 8));
  HIP_TRY(h, hipMalloc(&h->d_max64, h->n_max64 * 8));
  if (!h->d_found) HIP_TRY(h, hipMalloc(&h->d_found, 8));
  if (nb_entries > kObjSlots) {  // hashed object mode (see launch_attribution)
    HIP_TRY(h, hipMalloc(&h->d_pk64, (size_t)nb_entries * 2 * 8));
    HIP_TRY(h, hipMemset(h->d_pk64, 0, (size_t)nb_entries * 2 * 8));
  }
  // pad the dense arena to a multiple of 4 cells per thread so it is zeroed in 16 B units
  h->hist_cells = (h->hist_cells + 3) & ~uint64_t(3);
  if (h->hist_cells) HIP_TRY(h, hipMalloc(&h->d_hist, h->hist_cells * h->T * 4));
  if (!h->sparse_entries.empty()) {
    HIP_TRY(h, hipMalloc(&h->d_sparse_keys, h->sparse_cap * 8));
    HIP_TRY(h, hipMalloc(&h->d_sparse_vals, h->sparse_cap * 4));
    HIP_TRY(h, hipMalloc(&h->d_sparse_dirty, 2 * 4));
    const uint32_t ones[2] = {1u, 1u};  // the first reset clears the fresh table
    HIP_TRY(h, hipMemcpy(h->d_sparse_dirty, ones, 8, hipMemcpyHostToDevice));
  }
  h->have_table = true;
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  for (nmg_engine* w : h->workers) {  // multi-GPU: the table on every device
    const int rc = nmg_set_objects(w, keys, entry_off, nb_keys, entries, nb_entries);
    if (rc) return fail(h, rc, w->last_error);
  }
  return nmg_reset_counters(h);
}

static int stream_flush(nmg_engine* h);
static int route_settle(nmg_engine* h);

// A live --online-analysis table (nmg_update_objects) may hold entries the
// engine has not seen: objects created since the previous alarm (ids E ..
// newE - 1, _init_mem_info's next id, mem_analyzer.c:567-568, with their
// counters from creation, :569-572), and objects whose size at free
// (ma_record_free, :1287) outgrew their page cells.  New entries get page
// cells like nmg_set_objects gives them (dense within the budget, sparse
// otherwise); a dense entry that outgrew its cells moves to a new range with
// its counts.  Every id-indexed counter array is re-laid out on the device
// for the new entry count, counters kept.  (The stream is idle here.)
static int grow_entries(nmg_engine* h, uint32_t newE, const uint32_t* ids, const nmg_object* objs, uint32_t n) {
  const uint32_t oldE = h->E;
  const uint64_t T = h->T;
  const bool want_hist = (h->flags & NMG_F_PAGE_HIST) && (h->flags & NMG_F_MATCH_SAMPLES);
  const uint64_t max_cells_per_entry = 1ull << 24, budget_cells = h->hist_budget / 4;
  const uint64_t oldCells = h->hist_cells;
  uint64_t cells = oldCells;
  struct Move {
    uint64_t from, to, np;
  };
  std::vector<Move> moves;
  const size_t nsparse0 = h->sparse_entries.size();
  // Host state is changed in place below; every error return first undoes
  // it (the sizes before the call, and the old fields of the entries that
  // moved), so that a failed update keeps the engine as it was.
  struct Old {
    uint32_t id;
    uint64_t hist, np;
    DevEntry d;
  };
  std::vector<Old> changed;
  auto rollback = [&]() {
    for (auto it = changed.rbegin(); it != changed.rend(); ++it) {
      h->hist_base[it->id] = it->hist;
      h->npages[it->id] = it->np;
      h->dev_entries[it->id] = it->d;
    }
    h->hist_base.resize(oldE);
    h->npages.resize(oldE);
    h->buffer_size.resize(oldE);
    h->entry_addr.resize(oldE);
    h->objects.resize(oldE);
    h->dev_entries.resize(oldE);
    h->sparse_entries.resize(nsparse0);
  };
  auto fail_rb = [&](int code, const std::string& msg) {
    rollback();
    return fail(h, code, msg);
  };
  h->hist_base.resize(newE, kHistSparse);
  h->npages.resize(newE, 1);
  h->buffer_size.resize(newE, 0);
  h->entry_addr.resize(newE, 0);
  h->objects.resize(newE, nmg_object{0, 0, 0, 0});
  h->dev_entries.resize(newE);
  for (uint32_t e = oldE; e < newE; e++) {
    DevEntry& d = h->dev_entries[e];
    memset(&d, 0, sizeof(d));
    d.hist = kHistSparse;
    d.sidx = ~0u;
    d.id = e;
  }
  for (uint32_t j = 0; j < n; j++) {
    const uint32_t id = ids[j];
    const uint64_t np = objs[j].buffer_size / kPageSize + 1;
    DevEntry& d = h->dev_entries[id];
    if (id >= oldE) {
      h->npages[id] = np;
      if (!want_hist) continue;
      if (np * T <= max_cells_per_entry && (cells + np) * T <= budget_cells && cells + np < 0xffffffffull) {
        d.hist = h->hist_base[id] = cells;
        cells += np;
      } else {
        if (h->sparse_entries.size() >= (1u << 22)) return fail_rb(NMG_ERR_CAPACITY, "too many sparse entries");
        d.sidx = (uint32_t)h->sparse_entries.size();
        h->sparse_entries.push_back(id);
      }
    } else if (np > h->npages[id]) {
      changed.push_back({id, h->hist_base[id], h->npages[id], d});
      if (want_hist && h->hist_base[id] != kHistSparse) {
        if (np * T > max_cells_per_entry || (cells + np) * T > budget_cells || cells + np >= 0xffffffffull)
          return fail_rb(NMG_ERR_CAPACITY, "an object outgrew its page cells past the histogram budget");
        moves.push_back({h->hist_base[id], cells, h->npages[id]});
        d.hist = h->hist_base[id] = cells;
        cells += np;
      }
      h->npages[id] = np;
    }
  }
  cells = (cells + 3) & ~uint64_t(3);
  // id-indexed counters, re-laid out for newE entries
  const uint64_t n_sum = 2 * kGlobalSums + (uint64_t)newE * 4 +
                         ((h->flags & NMG_F_OBJECT_LEVELS) ? (uint64_t)newE * 2 * kLevelWords : 0);
  const uint64_t n_min = 36 + (uint64_t)newE + 1;
  uint64_t *sum = nullptr, *mn = nullptr;
  uint32_t* hist = nullptr;
  unsigned long long* pk = nullptr;
  DevEntry* ent = nullptr;
  uint64_t* skeys = nullptr;
  uint32_t *svals = nullptr, *sdirty = nullptr;
  const bool new_sparse = nsparse0 == 0 && !h->sparse_entries.empty() && !h->d_sparse_keys;
  auto undo = [&](hipError_t e, const char* what) {
    (void)hipStreamSynchronize(h->stream);
    (void)hipFree(sum);
    (void)hipFree(mn);
    (void)hipFree(hist);
    (void)hipFree(pk);
    (void)hipFree(ent);
    (void)hipFree(skeys);
    (void)hipFree(svals);
    (void)hipFree(sdirty);
    return fail_rb(NMG_ERR_HIP, std::string("nmg_update_objects: ") + what + ": " + hipGetErrorString(e));
  };
  hipError_t e;
  if ((e = hipMalloc(&sum, n_sum * 8)) != hipSuccess) return undo(e, "counters");
  if ((e = hipMalloc(&mn, n_min * 8)) != hipSuccess) return undo(e, "ordinals");
  if (cells && cells * T != oldCells * T && (e = hipMalloc(&hist, cells * T * 4)) != hipSuccess)
    return undo(e, "page histogram");
  if (newE > kObjSlots && (e = hipMalloc(&pk, (size_t)newE * 2 * 8)) != hipSuccess) return undo(e, "packed counters");
  if ((e = hipMalloc(&ent, (size_t)newE * sizeof(DevEntry))) != hipSuccess) return undo(e, "entries");
  hipStream_t st = h->stream;
  if (new_sparse) {  // the first sparse entry: its table
    if ((e = hipMalloc(&skeys, h->sparse_cap * 8)) != hipSuccess || (e = hipMalloc(&svals, h->sparse_cap * 4)) != hipSuccess ||
        (e = hipMalloc(&sdirty, 2 * 4)) != hipSuccess || (e = hipMemsetAsync(skeys, 0xff, h->sparse_cap * 8, st)) != hipSuccess ||
        (e = hipMemsetAsync(svals, 0, h->sparse_cap * 4, st)) != hipSuccess ||
        (e = hipMemsetAsync(sdirty, 0, 2 * 4, st)) != hipSuccess)
      return undo(e, "sparse page table");
  }
  if ((e = hipMemsetAsync(sum, 0, n_sum * 8, st)) != hipSuccess ||
      (e = hipMemcpyAsync(sum, h->d_sum64, 2 * kGlobalSums * 8, hipMemcpyDeviceToDevice, st)) != hipSuccess ||
      (oldE && (e = hipMemcpy2DAsync(sum + 2 * kGlobalSums, (size_t)newE * 8, h->d_sum64 + 2 * kGlobalSums,
                                     (size_t)oldE * 8, (size_t)oldE * 8, 4, hipMemcpyDeviceToDevice, st)) != hipSuccess) ||
      ((h->flags & NMG_F_OBJECT_LEVELS) && oldE &&
       (e = hipMemcpyAsync(sum + 2 * kGlobalSums + (uint64_t)newE * 4, h->d_sum64 + 2 * kGlobalSums + (uint64_t)oldE * 4,
                           (size_t)oldE * 2 * kLevelWords * 8, hipMemcpyDeviceToDevice, st)) != hipSuccess) ||
      (e = hipMemsetAsync(mn, 0xff, n_min * 8, st)) != hipSuccess ||
      (e = hipMemcpyAsync(mn, h->d_min64, (36 + (size_t)oldE) * 8, hipMemcpyDeviceToDevice, st)) != hipSuccess ||
      (e = hipMemcpyAsync(mn + 36 + newE, h->d_min64 + 36 + oldE, 8, hipMemcpyDeviceToDevice, st)) != hipSuccess ||
      (pk && (e = hipMemsetAsync(pk, 0, (size_t)newE * 2 * 8, st)) != hipSuccess) ||
      (e = hipMemcpyAsync(ent, h->dev_entries.data(), (size_t)newE * sizeof(DevEntry), hipMemcpyHostToDevice, st)) !=
          hipSuccess)
    return undo(e, "re-layout");
  if (hist) {  // [thread][cell] rows with the new stride; moved entries' counts to their new range
    if ((e = hipMemsetAsync(hist, 0, cells * T * 4, st)) != hipSuccess ||
        (oldCells && (e = hipMemcpy2DAsync(hist, cells * 4, h->d_hist, oldCells * 4, oldCells * 4, T,
                                           hipMemcpyDeviceToDevice, st)) != hipSuccess))
      return undo(e, "page histogram re-layout");
    for (const Move& m : moves)
      if ((e = hipMemcpy2DAsync(hist + m.to, cells * 4, hist + m.from, cells * 4, m.np * 4, T, hipMemcpyDeviceToDevice,
                                st)) != hipSuccess ||
          (e = hipMemset2DAsync(hist + m.from, cells * 4, 0, m.np * 4, T, st)) != hipSuccess)
        return undo(e, "page cells of a grown object");
  }
  if ((e = hipStreamSynchronize(st)) != hipSuccess) return undo(e, "re-layout");
  (void)hipFree(h->d_sum64);
  (void)hipFree(h->d_min64);
  (void)hipFree(h->d_pk64);
  if (h->d_chain == h->d_entries) h->d_chain = ent;
  (void)hipFree(h->d_entries);
  h->d_sum64 = sum;
  h->d_min64 = mn;
  h->d_pk64 = pk;
  h->d_entries = ent;
  if (hist) {
    (void)hipFree(h->d_hist);
    h->d_hist = hist;
  }
  h->n_sum64 = n_sum;
  h->n_min64 = n_min;
  h->hist_cells = cells;
  h->E = newE;
  if (new_sparse) {
    h->d_sparse_keys = skeys;
    h->d_sparse_vals = svals;
    h->d_sparse_dirty = sdirty;
  }
  return NMG_OK;
}

// --online-analysis: the table at an alarm, counters kept (mem_sampling.c:953-954
// against the live mem_list).  Entry ids index the counters: ids of the
// nmg_set_objects table, and (live hosts) ids past it for objects created
// since (grow_entries).  The report describes each entry as the latest table
// lists it, in the order of the latest table that lists every entry.
extern "C" int nmg_update_objects(nmg_engine* h, const uint64_t* keys, const uint32_t* entry_off,
                                  uint32_t nb_keys, const uint32_t* entry_ids, const nmg_object* objects) {
  if (h) h->epoch++;
  Range range("nmg_update_objects");
  if (!h || (nb_keys && (!keys || !entry_off || !entry_ids || !objects))) return NMG_ERR_INVALID;
  if (!h->have_table) return fail(h, NMG_ERR_STATE, "nmg_update_objects before nmg_set_objects");
  const uint32_t n = nb_keys ? entry_off[nb_keys] : 0;
  int rc = check_table(h, keys, nb_keys ? entry_off : nullptr, nb_keys, n);
  if (rc) return rc;
  // ids: each at most once; new ones (>= E) consecutive from E
  uint32_t newE = h->E;
  for (uint32_t j = 0; j < n; j++) newE = std::max(newE, entry_ids[j] + 1);
  if (entry_ids && n && (uint64_t)newE > (1ull << 31)) return fail(h, NMG_ERR_RANGE, "too many entries");
  uint64_t nb_grown = 0;
  {
    std::vector<uint8_t> seen(newE, 0);
    for (uint32_t j = 0; j < n; j++) {
      const uint32_t id = entry_ids[j];
      if (seen[id]) return fail(h, NMG_ERR_INVALID, "an entry id listed twice in one table");
      seen[id] = 1;
      if (id < h->E && objects[j].buffer_size / kPageSize + 1 > h->npages[id]) nb_grown++;
    }
    for (uint32_t id = h->E; id < newE; id++)
      if (!seen[id]) return fail(h, NMG_ERR_RANGE, "new entry ids must be consecutive from the current entry count");
  }
  HIP_TRY(h, hipSetDevice(h->device));
  if (h->streaming) {  // the open chunk belongs to the previous alarms' table
    rc = stream_flush(h);
    if (rc) return rc;
  }
  rc = route_settle(h);  // (reads the pool only, not the table)
  if (rc) return rc;
  HIP_TRY(h, hipStreamSynchronize(h->stream));  // launches in flight read the old table and counters
  if (h->multi_pending) {  // merges in flight write the counters being re-laid out
    rc = multi_finish(h);
    if (rc) return rc;
  }
  if (newE > h->E || nb_grown) {
    rc = grow_entries(h, newE, entry_ids, objects, n);
    if (rc) return rc;
  }
  std::vector<DevEntry> chain(n);
  for (uint32_t j = 0; j < n; j++) {
    const uint32_t id = entry_ids[j];
    const nmg_object& o = objects[j];
    DevEntry& d = chain[j];
    d = h->dev_entries[id];  // hist, sidx, id
    d.addr = o.buffer_addr;
    d.end = o.buffer_addr + o.buffer_size;
    d.alloc = o.alloc_date;
    d.free = o.free_date;
    d.count = d.first = 0;
  }
  free_route_table(h);  // (the partitions describe the previous table)
  // build the alarm's lookup beside the current one; keep the current one if that fails
  const LookupSet prev = take_lookup(h);
  rc = build_lookup(h, keys, entry_off, nb_keys, chain, nullptr);
  if (rc == NMG_OK && hipStreamSynchronize(h->stream) != hipSuccess)
    rc = fail(h, NMG_ERR_HIP, "nmg_update_objects: table upload failed");
  if (rc) {
    (void)hipStreamSynchronize(h->stream);
    free_lookup(h);
    put_lookup(h, prev);
    return rc;
  }
  {
    const LookupSet cur = take_lookup(h);
    put_lookup(h, prev);
    free_lookup(h);  // (keeps d_chain when it is the by-id entry array)
    put_lookup(h, cur);
  }
  // the report's view: every listed entry as this table lists it, and this
  // table's order when it lists every entry (ma_finalize walks the table it
  // has at exit, FOREACH_HASH, mem_analyzer.c:1381-1383)
  for (uint32_t j = 0; j < n; j++) {
    const uint32_t id = entry_ids[j];
    h->objects[id] = objects[j];
    h->buffer_size[id] = objects[j].buffer_size;
    h->entry_addr[id] = objects[j].buffer_addr;
  }
  if (n == h->E) {
    bool identity = true;
    for (uint32_t j = 0; j < n && identity; j++) identity = entry_ids[j] == j;
    if (identity) h->order.clear();
    else h->order.assign(entry_ids, entry_ids + n);
  } else if (!h->order.empty()) {
    // a partial table that brought new entries: they follow the known ones,
    // in id order, until a table lists every entry
    for (uint32_t id = (uint32_t)h->order.size(); id < h->E; id++) h->order.push_back(id);
  }
  // the alarm table's partitions.  The new table is committed above, so a
  // failure here is not the update's: the table stays on attribute_kernel
  // (no partitions) and the update goes on to the workers, which must get
  // the same table (a half-applied update would leave them on the old one).
  if (build_partitions(h, keys, entry_off, nb_keys, chain, entry_ids) != NMG_OK) {
    (void)hipGetLastError();
    free_route_table(h);
  }
  for (nmg_engine* w : h->workers) {  // multi-GPU: the table on every device
    rc = nmg_update_objects(w, keys, entry_off, nb_keys, entry_ids, objects);
    if (rc) return fail(h, rc, w->last_error);
  }
  return NMG_OK;
}

static int stage_reserve(nmg_engine* h, size_t need) {
  if (need <= h->stage_cap) return NMG_OK;
  size_t cap = std::max(need, h->stage_cap * 2 + (1u << 20));
  uint8_t* p = nullptr;
  // (portable: a multi-GPU engine's workers copy from it on every device)
  HIP_TRY(h, hipHostMalloc((void**)&p, cap, h->multi ? hipHostMallocPortable : hipHostMallocDefault));
  if (h->stage_len) memcpy(p, h->h_stage, h->stage_len);
  if (h->h_stage) {
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    (void)hipHostFree(h->h_stage);
  }
  h->h_stage = p;
  h->stage_cap = cap;
  return NMG_OK;
}

static int append_desc(nmg_engine* h, uint64_t len, uint32_t thread_rank, uint32_t access) {
  if (!h->zc_dev.empty()) h->zc_dev.push_back(0);
  BufDesc d;
  d.offset = h->stage_len;
  d.len = (uint32_t)len;
  d.thread_rank = thread_rank;
  d.access = access;
  d.pad = 0;
  d.seq = h->descs.size();
  h->descs.push_back(d);
  h->buf_bytes.push_back(len);
  h->stage_len = (h->stage_len + len + 15) & ~size_t(15);
  h->staged_dirty = true;
  h->descs_dirty = true;
  h->multi_staged = false;
  return NMG_OK;
}

// The device address of [p, p + len) when it lies in memory registered with
// nmg_register_host and starts 16-byte aligned (the kernels' record loads);
// 0 otherwise.  Only for the batch path of a single-GPU engine without the
// dump modes (their per-record arrays are indexed by staging offsets).
static uint64_t zero_copy_dev(nmg_engine* h, const void* p, uint64_t len) {
  if (h->hostregs.empty() || h->streaming || h->multi || (h->flags & NMG_F_SAMPLE_MATCHES)) return 0;
  const uintptr_t a = (uintptr_t)p;
  for (const auto& r : h->hostregs)
    if (a >= r.lo && a + len <= r.hi) {
      const uint64_t dev = r.dev + (a - r.lo);
      return (dev & 15) ? 0 : dev;
    }
  return 0;
}

// a buffer read in place (zero_copy_dev): its offset is fixed up against the
// arena base at upload (upload_buffers)
static int append_desc_zc(nmg_engine* h, uint64_t dev, uint64_t len, uint32_t thread_rank, uint32_t access) {
  if (h->zc_dev.size() < h->descs.size()) h->zc_dev.resize(h->descs.size(), 0);
  h->zc_dev.push_back(dev);
  BufDesc d;
  d.offset = 0;
  d.len = (uint32_t)len;
  d.thread_rank = thread_rank;
  d.access = access;
  d.pad = 0;
  d.seq = h->descs.size();
  h->descs.push_back(d);
  h->buf_bytes.push_back(len);
  h->descs_dirty = true;
  h->multi_staged = false;
  return NMG_OK;
}

static int check_buffer_args(nmg_engine* h, uint64_t len, uint32_t thread_rank, uint32_t access) {
  if (access > 1) return fail(h, NMG_ERR_INVALID, "access_type must be 0 (read) or 1 (write)");
  if (thread_rank >= h->T)
    return fail(h, NMG_ERR_RANGE, "thread_rank >= nb_threads (set nmg_options.nb_threads)");
  if (len >= (1ull << 32)) return fail(h, NMG_ERR_RANGE, "buffer >= 4 GiB (unsigned cursors, mem_sampling.c:831-834)");
  if (h->external) return fail(h, NMG_ERR_STATE, "device buffers are set; call nmg_clear_buffers first");
  if (h->streamed && !h->streaming) return fail(h, NMG_ERR_STATE, "stream ended; call nmg_clear_buffers first");
  return NMG_OK;
}

// a host copy into pinned staging, run by one of the copy threads
struct CopyTask {
  uint8_t* dst;
  const uint8_t* src;
  uint64_t len;
};
static int stream_dst(nmg_engine* h, uint64_t len, uint8_t** dst, std::vector<CopyTask>* pending);
static void ensure_occupancy(nmg_engine* h);
static uint32_t attribution_grid(nmg_engine* h, uint32_t nb);
static void make_schedule(const std::vector<BufDesc>& descs, uint32_t grid, uint32_t index_base, BufDesc* sorted,
                          uint32_t* ranges, bool by_stream = true);
static int launch_attribution(nmg_engine* h, const uint8_t* data, const BufDesc* sdescs, const uint32_t* ranges,
                              uint32_t nb, uint32_t grid, uint64_t nbytes);
static int stream_append(nmg_engine* h, uint64_t len, uint32_t thread_rank, uint32_t access);
static bool route_eligible(nmg_engine* h);
// One partition-first analysis: a buffer set in HBM with its analysis-order
// schedule (the submitted buffers, or a streamed chunk whose per-buffer count
// slots start at index_base; a chunk settles its per-buffer matched counts at
// once, before the next chunk reuses the pool).
struct RouteJob {
  const std::vector<BufDesc>* descs;
  const uint8_t* data;
  const BufDesc* sdescs;
  const uint32_t* ranges;
  const uint32_t* chunk0;
  uint32_t grid, index_base;
  bool settle_now;
};

static int route_analyze_job(nmg_engine* h, const RouteJob& job);
static bool route_eligible(nmg_engine* h, const std::vector<BufDesc>& descs);
static int route_pool(nmg_engine* h, const std::vector<BufDesc>& descs, uint32_t grid, const uint32_t* ranges,
                      std::vector<uint32_t>& c0);
static int route_prepare(nmg_engine* h, uint32_t grid, const std::vector<uint32_t>& ranges);
static int route_analyze(nmg_engine* h, uint32_t nb, uint32_t grid);
static int route_settle(nmg_engine* h);

extern "C" int nmg_register_host(nmg_engine* h, void* ptr, uint64_t bytes) {
  if (!h || !ptr || !bytes) return NMG_ERR_INVALID;
  if (h->multi) return fail(h, NMG_ERR_STATE, "nmg_register_host: single-GPU engines only");
  // whole pages are pinned and mapped, and HIP then treats every address in
  // them as this registration's: they must be the caller's alone (another
  // allocation sharing the last page would be misread by later copies)
  if ((uintptr_t)ptr & 4095) return fail(h, NMG_ERR_INVALID, "nmg_register_host: ptr must be page-aligned (4 KiB)");
  const uintptr_t a = (uintptr_t)ptr;
  for (const auto& r : h->hostregs)  // (pages: two ranges must not share one)
    if ((a & ~uintptr_t(4095)) < ((r.hi + 4095) & ~uintptr_t(4095)) && ((uintptr_t)r.pages) < a + bytes)
      return fail(h, NMG_ERR_INVALID, "nmg_register_host: overlaps (shares a page with) a registered range");
  const uintptr_t pg = 4096, p0 = a, p1 = (a + bytes + pg - 1) & ~(pg - 1);
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipHostRegister((void*)p0, p1 - p0, hipHostRegisterMapped));
  void* dev = nullptr;
  if (hipHostGetDevicePointer(&dev, (void*)p0, 0) != hipSuccess || !dev) {
    (void)hipHostUnregister((void*)p0);
    return fail(h, NMG_ERR_HIP, "nmg_register_host: no device address for the range");
  }
  h->hostregs.push_back({a, a + bytes, (uint64_t)(uintptr_t)dev + (a - p0), (void*)p0});
  return NMG_OK;
}

extern "C" int nmg_unregister_host(nmg_engine* h, void* ptr) {
  if (!h || !ptr) return NMG_ERR_INVALID;
  for (size_t i = 0; i < h->hostregs.size(); i++) {
    if (h->hostregs[i].lo != (uintptr_t)ptr) continue;
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, hipStreamSynchronize(h->stream));  // (a launch in flight may still read it)
    for (uint64_t z : h->zc_dev)
      if (z && z - h->hostregs[i].dev < h->hostregs[i].hi - h->hostregs[i].lo)
        return fail(h, NMG_ERR_STATE, "nmg_unregister_host: submitted buffers lie in the range; nmg_clear_buffers first");
    HIP_TRY(h, hipHostUnregister(h->hostregs[i].pages));
    h->hostregs.erase(h->hostregs.begin() + i);
    return NMG_OK;
  }
  return fail(h, NMG_ERR_INVALID, "nmg_unregister_host: not a registered range");
}

extern "C" int nmg_submit_buffer(nmg_engine* h, const void* bytes, uint64_t len, uint32_t thread_rank,
                                 uint32_t access_type) {
  if (!h || (len && !bytes)) return NMG_ERR_INVALID;
  int rc = check_buffer_args(h, len, thread_rank, access_type);
  if (rc) return rc;
  if (len == 0) return NMG_OK;  // __copy_buffer drops empty segments (mem_sampling.c:680-682)
  if (const uint64_t dev = zero_copy_dev(h, bytes, len)) return append_desc_zc(h, dev, len, thread_rank, access_type);
  if (h->streaming) {
    uint8_t* dst = nullptr;
    rc = stream_dst(h, len, &dst, nullptr);
    if (rc) return rc;
    memcpy(dst, bytes, len);
    return stream_append(h, len, thread_rank, access_type);
  }
  rc = stage_reserve(h, h->stage_len + len + 16);
  if (rc) return rc;
  memcpy(h->h_stage + h->stage_len, bytes, len);
  return append_desc(h, len, thread_rank, access_type);
}

extern "C" int nmg_submit_ring(nmg_engine* h, const void* ring, uint64_t ring_size, uint64_t data_tail,
                               uint64_t data_head, uint32_t thread_rank, uint32_t access_type) {
  if (!h || !ring || data_tail > ring_size || data_head > ring_size) return NMG_ERR_INVALID;
  if (data_head == data_tail) return NMG_OK;  // nothing to do (mem_sampling.c:680-682)
  uint64_t len = data_head - data_tail;
  if (data_head < data_tail) len = ring_size - data_tail + data_head;  // :687-694
  int rc = check_buffer_args(h, len, thread_rank, access_type);
  if (rc) return rc;
  if (data_head > data_tail)  // one segment: in place if the ring is registered
    if (const uint64_t dev = zero_copy_dev(h, (const uint8_t*)ring + data_tail, len))
      return append_desc_zc(h, dev, len, thread_rank, access_type);
  uint8_t* dst = nullptr;
  if (h->streaming) {
    rc = stream_dst(h, len, &dst, nullptr);
  } else {
    rc = stage_reserve(h, h->stage_len + len + 16);
    dst = h->h_stage + h->stage_len;
  }
  if (rc) return rc;
  const uint8_t* r = (const uint8_t*)ring;
  if (data_head < data_tail) {  // :704-713: two segments
    uint64_t first = ring_size - data_tail;
    memcpy(dst, r + data_tail, first);
    memcpy(dst + first, r, data_head);
  } else {
    memcpy(dst, r + data_tail, len);
  }
  return h->streaming ? stream_append(h, len, thread_rank, access_type) : append_desc(h, len, thread_rank, access_type);
}

// ---------------------------------------------------------------------------
// host copies split over threads (nmg_submit_buffers)

static void run_copies(nmg_engine* h, const std::vector<CopyTask>& tasks) {
  if (tasks.empty()) return;
  uint64_t total = 0;
  for (const auto& t : tasks) total += t.len;
  const uint32_t nthreads = h->copy_threads;
  if (nthreads <= 1 || total < (2u << 20)) {
    for (const auto& t : tasks) memcpy(t.dst, t.src, t.len);
    return;
  }
  if (!h->pool) h->pool.reset(new CopyPool(nthreads));
  const uint32_t T = nthreads;
  // contiguous task ranges of about equal bytes
  std::vector<size_t> cut(T + 1, tasks.size());
  cut[0] = 0;
  uint64_t acc = 0;
  uint32_t k = 1;
  for (size_t i = 0; i < tasks.size() && k < T; i++) {
    acc += tasks[i].len;
    if (acc * T >= total * k) cut[k++] = i + 1;
  }
  h->pool->run([&](uint32_t w) {
    for (size_t i = cut[w]; i < cut[w + 1]; i++) memcpy(tasks[i].dst, tasks[i].src, tasks[i].len);
  });
}

// ---------------------------------------------------------------------------
// streaming: chunks of submitted buffers staged in one of two pinned halves,
// uploaded on the copy stream and analysed on the engine stream

// wait until the host may refill slot s (its previous chunk's H2D is done)
static int slot_acquire(nmg_engine* h, int s) {
  auto& sl = h->slots[s];
  if (sl.used) HIP_TRY(h, hipEventSynchronize(sl.copied));
  sl.len = 0;
  sl.descs.clear();
  return NMG_OK;
}

// per-buffer count array for `need` buffers; its stride stays fixed while
// chunks are in flight (grown by doubling after draining the engine stream)
static int ensure_bufcnt(nmg_engine* h, size_t need) {
  if (need <= h->bufcnt_stride) return NMG_OK;
  if (h->bufcnt_stride == 0 && need <= h->bufcnt_cap) {  // a kept array, first chunk
    h->bufcnt_stride = h->bufcnt_cap;
    HIP_TRY(h, hipMemsetAsync(h->d_bufcnt, 0, h->bufcnt_cap * 2 * 4, h->stream));
    return NMG_OK;
  }
  const size_t cap = std::max<size_t>({need, h->bufcnt_cap * 2, (size_t)4096});
  uint32_t* nb = nullptr;
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  HIP_TRY(h, hipMalloc(&nb, cap * 2 * 4));
  HIP_TRY(h, hipMemsetAsync(nb, 0, cap * 2 * 4, h->stream));
  if (h->d_bufcnt && h->bufcnt_stride) {
    HIP_TRY(h, hipMemcpyAsync(nb, h->d_bufcnt, h->bufcnt_stride * 4, hipMemcpyDeviceToDevice, h->stream));
    HIP_TRY(h, hipMemcpyAsync(nb + cap, h->d_bufcnt + h->bufcnt_stride, h->bufcnt_stride * 4,
                              hipMemcpyDeviceToDevice, h->stream));
  }
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  (void)hipFree(h->d_bufcnt);
  h->d_bufcnt = nb;
  h->bufcnt_cap = cap;
  h->bufcnt_stride = cap;
  return NMG_OK;
}

// Enqueue the open chunk: schedule on the host, H2D on the copy stream (after
// the slot's previous kernel released its device arena), then the kernel on
// the engine stream once the copy has landed.
static int stream_flush(nmg_engine* h) {
  if (h) h->epoch++;
  Range range("nmg_stream_chunk");
  auto& sl = h->slots[h->cur_slot];
  if (sl.descs.empty()) return NMG_OK;
  const uint32_t nb = (uint32_t)sl.descs.size();
  const uint32_t grid = attribution_grid(h, nb);
  int rc = ensure_bufcnt(h, h->descs.size());
  if (rc) return rc;
  // large tables: the partition-first passes over the chunk (analysis-order
  // schedule, then the ranges and the workgroups' chunk pools)
  const bool route = route_eligible(h, sl.descs);
  const size_t sched_bytes = nb * sizeof(BufDesc) + (grid + 1) * 4 * (route ? 2 : 1);
  if (sched_bytes > sl.hs_cap) {  // (slot acquired: its previous H2D is done)
    if (sl.h_sdescs) (void)hipHostFree(sl.h_sdescs);
    sl.h_sdescs = nullptr;
    sl.hs_cap = std::max<size_t>(sched_bytes * 2, 64 << 10);
    HIP_TRY(h, hipHostMalloc((void**)&sl.h_sdescs, sl.hs_cap, hipHostMallocDefault));
  }
  const uint32_t index_base = (uint32_t)(h->descs.size() - nb);
  uint32_t* h_ranges = reinterpret_cast<uint32_t*>(sl.h_sdescs + nb);
  make_schedule(sl.descs, grid, index_base, sl.h_sdescs, h_ranges, !route);
  if (route) {
    std::vector<uint32_t> c0;
    rc = route_pool(h, sl.descs, grid, h_ranges, c0);  // (may wait for the stream to grow the pool)
    if (rc) return rc;
    memcpy(h_ranges + grid + 1, c0.data(), (grid + 1) * 4);
  }
  if (sl.len + 64 > sl.dcap || sched_bytes > sl.ds_cap) {  // grow the device side: wait for its last kernel
    if (sl.used) HIP_TRY(h, hipEventSynchronize(sl.done));
    if (sl.len + 64 > sl.dcap) {
      (void)hipFree(sl.d_arena);
      sl.d_arena = nullptr;
      sl.dcap = std::max<size_t>(sl.len + 64, sl.cap + 64);
      HIP_TRY(h, hipMalloc(&sl.d_arena, sl.dcap));
    }
    if (sched_bytes > sl.ds_cap) {
      (void)hipFree(sl.d_sdescs);
      sl.d_sdescs = nullptr;
      sl.ds_cap = sl.hs_cap;
      HIP_TRY(h, hipMalloc(&sl.d_sdescs, sl.ds_cap));
    }
  }
  if (sl.used) HIP_TRY(h, hipStreamWaitEvent(h->copy_stream, sl.done, 0));
  HIP_TRY(h, hipMemcpyAsync(sl.d_arena, sl.h_stage, sl.len, hipMemcpyHostToDevice, h->copy_stream));
  HIP_TRY(h, hipMemcpyAsync(sl.d_sdescs, sl.h_sdescs, sched_bytes, hipMemcpyHostToDevice, h->copy_stream));
  HIP_TRY(h, hipEventRecord(sl.copied, h->copy_stream));
  HIP_TRY(h, hipStreamWaitEvent(h->stream, sl.copied, 0));
  const uint32_t* d_ranges = reinterpret_cast<const uint32_t*>(sl.d_sdescs + nb);
  if (route) {
    const RouteJob job{&sl.descs, sl.d_arena, sl.d_sdescs, d_ranges, d_ranges + grid + 1, grid, index_base, true};
    rc = route_analyze_job(h, job);
  } else {
    rc = launch_attribution(h, sl.d_arena, sl.d_sdescs, d_ranges, nb, grid, sl.len);
  }
  if (rc) return rc;
  HIP_TRY(h, hipEventRecord(sl.done, h->stream));
  sl.used = true;
  // switch halves; the next submit refills the other one once its H2D is done
  h->cur_slot ^= 1;
  return slot_acquire(h, h->cur_slot);
}

// Destination in the open chunk for `len` bytes; flushes the chunk first when
// it is full (running the batch's pending copies into it before the upload).
static int stream_dst(nmg_engine* h, uint64_t len, uint8_t** dst, std::vector<CopyTask>* pending) {
  auto* sl = &h->slots[h->cur_slot];
  if (!sl->descs.empty() && sl->len + len + 16 > h->chunk_cap) {
    if (pending) {
      run_copies(h, *pending);
      pending->clear();
    }
    int rc = stream_flush(h);
    if (rc) return rc;
    sl = &h->slots[h->cur_slot];
  }
  if (sl->len + len + 16 > sl->cap) {  // first use, or one buffer larger than a chunk
    const size_t cap = std::max<size_t>(h->chunk_cap, sl->len + len + 16);
    uint8_t* p = nullptr;
    HIP_TRY(h, hipHostMalloc((void**)&p, cap, hipHostMallocDefault));
    if (sl->len) {
      if (pending) {  // pending copies target the old block
        run_copies(h, *pending);
        pending->clear();
      }
      memcpy(p, sl->h_stage, sl->len);
    }
    if (sl->h_stage) (void)hipHostFree(sl->h_stage);
    sl->h_stage = p;
    sl->cap = cap;
  }
  *dst = sl->h_stage + sl->len;
  return NMG_OK;
}

static int stream_append(nmg_engine* h, uint64_t len, uint32_t thread_rank, uint32_t access) {
  auto& sl = h->slots[h->cur_slot];
  BufDesc d;
  d.offset = sl.len;
  d.len = (uint32_t)len;
  d.thread_rank = thread_rank;
  d.access = access;
  d.pad = 0;
  d.seq = h->descs.size();  // analysis order across chunks
  sl.descs.push_back(d);
  h->descs.push_back(d);
  h->buf_bytes.push_back(len);
  sl.len = (sl.len + len + 15) & ~size_t(15);
  return NMG_OK;
}

extern "C" int nmg_stream_begin(nmg_engine* h, uint64_t chunk_bytes, uint32_t copy_threads) {
  if (!h || copy_threads == 0) return NMG_ERR_INVALID;
  if (h->multi) return fail(h, NMG_ERR_STATE, "streaming is single-GPU (nmg_options.nb_gpus <= 1)");
  if (h->external) return fail(h, NMG_ERR_STATE, "device buffers are set; call nmg_clear_buffers first");
  if (h->flags & NMG_F_SAMPLE_MATCHES)
    return fail(h, NMG_ERR_STATE, "dump modes (NMG_F_SAMPLE_MATCHES) need nmg_analyze over submitted buffers");
  if (h->staged_dirty || (!h->streaming && !h->streamed && !h->descs.empty()))
    return fail(h, NMG_ERR_STATE, "buffers already submitted; call nmg_clear_buffers first");
  HIP_TRY(h, hipSetDevice(h->device));
  if (!h->copy_stream) {
    HIP_TRY(h, hipStreamCreateWithFlags(&h->copy_stream, hipStreamNonBlocking));
    for (auto& sl : h->slots) {
      HIP_TRY(h, hipEventCreateWithFlags(&sl.copied, hipEventDisableTiming));
      HIP_TRY(h, hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
    }
  }
  h->chunk_cap = std::max<uint64_t>(chunk_bytes, 64 << 10);
  if (copy_threads != h->copy_threads) h->pool.reset();
  h->copy_threads = copy_threads;
  h->streaming = true;
  h->streamed = true;
  return NMG_OK;
}

extern "C" int nmg_stream_end(nmg_engine* h) {
  if (!h) return NMG_ERR_INVALID;
  if (!h->streaming) return NMG_OK;
  HIP_TRY(h, hipSetDevice(h->device));
  int rc = h->have_table ? stream_flush(h) : NMG_OK;
  h->streaming = false;
  return rc;
}

extern "C" int nmg_submit_buffers(nmg_engine* h, uint32_t n, const void* const* bytes, const uint64_t* lens,
                                  const uint32_t* thread_ranks, const uint32_t* access_types) {
  if (!h || (n && (!bytes || !lens || !thread_ranks || !access_types))) return NMG_ERR_INVALID;
  for (uint32_t i = 0; i < n; i++) {
    if (lens[i] && !bytes[i]) return NMG_ERR_INVALID;
    int rc = check_buffer_args(h, lens[i], thread_ranks[i], access_types[i]);
    if (rc) return rc;
  }
  std::vector<CopyTask> tasks;
  tasks.reserve(n);
  if (!h->streaming) {
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) total += (lens[i] + 15) & ~uint64_t(15);
    int rc = stage_reserve(h, h->stage_len + total + 16);
    if (rc) return rc;
    for (uint32_t i = 0; i < n; i++) {
      if (!lens[i]) continue;
      if (const uint64_t dev = zero_copy_dev(h, bytes[i], lens[i])) {
        append_desc_zc(h, dev, lens[i], thread_ranks[i], access_types[i]);
        continue;
      }
      tasks.push_back({h->h_stage + h->stage_len, (const uint8_t*)bytes[i], lens[i]});
      append_desc(h, lens[i], thread_ranks[i], access_types[i]);
    }
    run_copies(h, tasks);
    return NMG_OK;
  }
  for (uint32_t i = 0; i < n; i++) {
    if (!lens[i]) continue;
    uint8_t* dst = nullptr;
    int rc = stream_dst(h, lens[i], &dst, &tasks);
    if (rc) return rc;
    tasks.push_back({dst, (const uint8_t*)bytes[i], lens[i]});
    stream_append(h, lens[i], thread_ranks[i], access_types[i]);
  }
  run_copies(h, tasks);
  return NMG_OK;
}

extern "C" int nmg_set_device_buffers(nmg_engine* h, const void* d_data, const uint64_t* offsets,
                                      const uint64_t* lengths, const uint32_t* thread_ranks,
                                      const uint32_t* access_types, uint32_t nb_buffers, uint64_t seq_base) {
  if (!h || (nb_buffers && (!d_data || !offsets || !lengths || !thread_ranks || !access_types)))
    return NMG_ERR_INVALID;
  if (h->multi) return fail(h, NMG_ERR_STATE, "a multi-GPU engine takes host buffers (nmg_submit_*)");
  if (h->streaming || h->streamed) return fail(h, NMG_ERR_STATE, "streaming buffers are set; call nmg_clear_buffers first");
  std::vector<BufDesc> descs;
  std::vector<uint64_t> bytes;
  descs.reserve(nb_buffers);
  for (uint32_t b = 0; b < nb_buffers; b++) {
    if (offsets[b] & 15) return fail(h, NMG_ERR_INVALID, "device buffer offsets must be 16-byte aligned");
    if (access_types[b] > 1) return fail(h, NMG_ERR_INVALID, "access_type must be 0 or 1");
    if (thread_ranks[b] >= h->T) return fail(h, NMG_ERR_RANGE, "thread_rank >= nb_threads");
    if (lengths[b] >= (1ull << 32)) return fail(h, NMG_ERR_RANGE, "buffer >= 4 GiB");
    if (lengths[b] == 0) continue;
    BufDesc d;
    d.offset = offsets[b];
    d.len = (uint32_t)lengths[b];
    d.thread_rank = thread_ranks[b];
    d.access = access_types[b];
    d.pad = 0;
    d.seq = seq_base + descs.size();
    descs.push_back(d);
    bytes.push_back(lengths[b]);
  }
  h->descs.swap(descs);
  h->zc_dev.clear();
  h->buf_bytes.swap(bytes);
  h->d_data = (const uint8_t*)d_data;
  h->external = true;
  h->staged_dirty = false;
  h->descs_dirty = true;
  h->multi_staged = false;
  h->stage_len = 0;
  return NMG_OK;
}

extern "C" int nmg_clear_buffers(nmg_engine* h) {
  if (!h) return NMG_ERR_INVALID;
  if (h->route_pending) {
    const int rc = route_settle(h);
    if (rc) return rc;
  }
  if (h->streaming || h->streamed) {
    HIP_TRY(h, hipSetDevice(h->device));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    HIP_TRY(h, hipStreamSynchronize(h->copy_stream));
    for (auto& sl : h->slots) {
      sl.descs.clear();
      sl.len = 0;
      sl.used = false;
    }
    h->streamed = false;
    h->bufcnt_stride = 0;  // per-buffer counts restart (the array is kept)
  }
  for (nmg_engine* w : h->workers) nmg_clear_buffers(w);
  h->descs.clear();
  h->buf_bytes.clear();
  h->zc_dev.clear();
  h->stage_len = 0;
  h->external = false;
  h->d_data = nullptr;
  h->descs_dirty = true;
  h->multi_staged = false;
  h->counts_override = false;
  return NMG_OK;
}

static int upload_buffers(nmg_engine* h) {
  Range range("nmg_stage_h2d");
  if (!h->external && h->staged_dirty) {
    if (h->stage_len + 64 > h->arena_cap) {
      HIP_TRY(h, hipStreamSynchronize(h->stream));
      (void)hipFree(h->d_arena);
      h->d_arena = nullptr;
      h->arena_cap = h->stage_len + 64;
      HIP_TRY(h, hipMalloc(&h->d_arena, h->arena_cap));
    }
    if (h->stage_len) HIP_TRY(h, hipMemcpyAsync(h->d_arena, h->h_stage, h->stage_len, hipMemcpyHostToDevice, h->stream));
    h->d_data = h->d_arena;
    h->staged_dirty = false;
  }
  if (h->descs_dirty) {
    size_t n = h->descs.size();
    // in-place buffers: offsets against the arena base (u64 arithmetic, as the kernels' data + offset)
    for (size_t i = 0; i < h->zc_dev.size() && i < n; i++)
      if (h->zc_dev[i]) h->descs[i].offset = h->zc_dev[i] - (uint64_t)(uintptr_t)h->d_data;
    if (n > h->descs_cap) {
      HIP_TRY(h, hipStreamSynchronize(h->stream));
      (void)hipFree(h->d_descs);
      (void)hipFree(h->d_bufcnt);
      h->d_descs = nullptr;
      h->d_bufcnt = nullptr;
      h->descs_cap = n;
      h->bufcnt_cap = n;
      HIP_TRY(h, hipMalloc(&h->d_descs, n * sizeof(BufDesc)));
      HIP_TRY(h, hipMalloc(&h->d_bufcnt, n * 2 * 4));
    }
    h->bufcnt_stride = n;
    if (n) {
      HIP_TRY(h, hipMemcpyAsync(h->d_descs, h->descs.data(), n * sizeof(BufDesc), hipMemcpyHostToDevice, h->stream));
      HIP_TRY(h, hipMemsetAsync(h->d_bufcnt, 0, n * 2 * 4, h->stream));
      HIP_TRY(h, hipStreamSynchronize(h->stream));  // descs come from pageable memory
    }
    h->descs_dirty = false;
  }
  return NMG_OK;
}

// Work schedule: buffers sorted by stream (access type, thread rank) -- the
// order in which they are analysed changes no result (all merges are sums,
// mins and maxes; first-match ordinals carry the analysis position) -- and
// cut into `grid` contiguous ranges of about equal bytes.
// Host half: `sorted` = descs in schedule order with .pad = index_base + the
// buffer's position in `descs` (its per-buffer count slot), `ranges` = grid + 1
// cut points of about equal bytes.
static void make_schedule(const std::vector<BufDesc>& descs, uint32_t grid, uint32_t index_base, BufDesc* sorted,
                          uint32_t* ranges, bool by_stream) {
  const uint32_t nb = (uint32_t)descs.size();
  std::vector<uint32_t> order(nb);
  for (uint32_t i = 0; i < nb; i++) order[i] = i;
  if (by_stream) std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
    const BufDesc &x = descs[a], &y = descs[b];
    if (x.access != y.access) return x.access < y.access;
    return x.thread_rank < y.thread_rank;
  });
  std::vector<uint64_t> csum(nb + 1, 0);
  for (uint32_t i = 0; i < nb; i++) csum[i + 1] = csum[i] + descs[order[i]].len + 64;
  ranges[0] = 0;
  for (uint32_t w = 1; w < grid; w++) {
    const uint64_t target = csum[nb] * w / grid;
    uint32_t c = (uint32_t)(std::lower_bound(csum.begin(), csum.end(), target) - csum.begin());
    ranges[w] = std::max(ranges[w - 1], std::min(c, nb));
  }
  ranges[grid] = nb;
  for (uint32_t i = 0; i < nb; i++) {
    sorted[i] = descs[order[i]];
    sorted[i].pad = index_base + order[i];
  }
}

// by_stream: sorted by (access, thread) for attribute_kernel's per-stream
// tables; otherwise analysis order (the partition-first route pass)
static int build_schedule(nmg_engine* h, uint32_t grid, bool by_stream = true) {
  const uint32_t nb = (uint32_t)h->descs.size();
  std::vector<uint32_t> ranges(grid + 1, 0);
  std::vector<BufDesc> sorted(nb);
  make_schedule(h->descs, grid, 0, sorted.data(), ranges.data(), by_stream);
  (void)hipFree(h->d_sdescs);
  (void)hipFree(h->d_ranges);
  h->d_sdescs = nullptr;
  h->d_ranges = nullptr;
  HIP_TRY(h, hipMalloc(&h->d_sdescs, std::max<size_t>(nb, 1) * sizeof(BufDesc)));
  HIP_TRY(h, hipMalloc(&h->d_ranges, (grid + 1) * 4));
  if (nb) HIP_TRY(h, hipMemcpy(h->d_sdescs, sorted.data(), nb * sizeof(BufDesc), hipMemcpyHostToDevice));
  HIP_TRY(h, hipMemcpy(h->d_ranges, ranges.data(), (grid + 1) * 4, hipMemcpyHostToDevice));
  h->sched_grid = grid;
  h->sched_route = !by_stream;
  if (!by_stream) return route_prepare(h, grid, ranges);
  return NMG_OK;
}

static void ensure_occupancy(nmg_engine* h) {
  if (h->blocks_per_cu <= 0) {
    h->blocks_per_cu = attribute_blocks_per_cu();
  }
}

// persistent grid: one resident workgroup per slot, each with a byte-balanced range
static uint32_t attribution_grid(nmg_engine* h, uint32_t nb) {
  ensure_occupancy(h);
  return nb ? std::min<uint32_t>(nb, (uint32_t)(h->num_cus * h->blocks_per_cu)) : 0;
}

// One attribution launch over `nb` buffers whose stream-sorted descriptors and
// per-workgroup ranges are already on the device, on the engine stream,
// bracketed by the launch-timing events.
// The kernels' view of the engine: buffers, table, counters.
static Params base_params(nmg_engine* h, const uint8_t* data, const BufDesc* sdescs, const uint32_t* ranges) {
  Params p;
  memset(&p, 0, sizeof(p));
  p.data = data;
  p.sbufs = sdescs;
  p.ranges = ranges;
  p.nb_bufs = (uint32_t)h->bufcnt_stride;
  p.nb_keys = h->K;
  p.keys = h->d_keys;
  p.nodes = h->d_nodes;
  p.entries = h->d_entries;
  p.chain = h->d_chain;
  p.ffences = h->d_ffences;
  p.fshift = h->d_fshift;
  p.dir = h->d_dir;
  p.nb_fences = h->nb_fences;
  p.fence_log2 = h->fence_log2;
  p.dir_log2 = h->dir_log2;
  p.nb_threads = h->T;
  p.flags = h->flags;
  p.nb_entries = h->E;
  p.lds_nodes = h->K <= kLdsNodes;
  p.elevels = h->elevels;
  p.efences = h->d_efences;
  p.enodes = h->d_enodes;
  p.sparse_mask = (uint32_t)(h->sparse_cap - 1);
  p.hist_cells = h->hist_cells;
  p.sum64 = h->d_sum64;
  p.min64 = h->d_min64;
  p.max64 = h->d_max64;
  p.hist = h->d_hist;
  p.bufcnt = h->d_bufcnt;
  p.found = h->d_found;
  p.sparse_keys = h->d_sparse_keys;
  p.sparse_vals = h->d_sparse_vals;
  p.sparse_dirty = h->d_sparse_dirty ? h->d_sparse_dirty + (h->nreset & 1) : nullptr;
  p.smatch = (h->flags & NMG_F_SAMPLE_MATCHES) ? h->d_smatch : nullptr;
  return p;
}

// timing events of launch slot nlaunch % kRing (created on first use)
static int launch_events(nmg_engine* h, int* slot_out) {
  const int slot = (int)(h->nlaunch % nmg_engine::kRing);
  if (!h->ring0[slot]) {
    HIP_TRY(h, hipEventCreate(&h->ring0[slot]));
    HIP_TRY(h, hipEventCreate(&h->ringr[slot]));
    HIP_TRY(h, hipEventCreate(&h->ringm[slot]));
    HIP_TRY(h, hipEventCreate(&h->ring1[slot]));
  }
  *slot_out = slot;
  return NMG_OK;
}

static int launch_attribution(nmg_engine* h, const uint8_t* data, const BufDesc* sdescs, const uint32_t* ranges,
                              uint32_t nb, uint32_t grid, uint64_t nbytes) {
  Range range("nmg_attribute");
  Params p = base_params(h, data, sdescs, ranges);
  // dense LDS tables when the table is small enough (DESIGN.md "Kernels");
  // large tables: their own kernel instances (fences + directory + node records)
  const int mode = (h->E <= kObjSlots ? kModeDenseObj : 0) | (h->hist_cells <= kDensePageCells ? kModeDensePage : 0) |
                   (p.lds_nodes ? 0 : kModeLarge);
  if (!(mode & kModeDenseObj) && h->d_pk64 && !(h->flags & kDbgNoPack)) {
    // < 2^cbits packed samples in this launch (only SAMPLE records of at
    // least 40 B are packed: the kernel keeps shorter ones, which the
    // reference's byte cursor accepts, on the plain path); packed weights
    // < 2^(64 - 2 cbits), so any entry's packed sum < 2^(64 - cbits)
    const uint32_t cbits = 64 - (uint32_t)__builtin_clzll(nbytes / kRecBytes + 1);
    if (2 * cbits < 64) {
      p.pk64 = h->d_pk64;
      p.pk_shift = 64 - cbits;
      p.pk_wlim = 1ull << (64 - 2 * cbits);
    }
  }
  if (!(mode & kModeDenseObj) && nb && grid <= kLogMaxGrid && (h->flags & NMG_F_MATCH_SAMPLES) &&
      nbytes / 8 < (1ull << 32)) {  // (u32 per-entry sums in tlog_reduce; records are >= 8 B)
    uint32_t rshift = 0;
    while ((((uint64_t)h->E + (1ull << rshift) - 1) >> rshift) > kLogParts) rshift++;
    const uint32_t parts = (uint32_t)(((uint64_t)h->E + (1ull << rshift) - 1) >> rshift);
    // sized for about every sample of the launch spread evenly; a full
    // sub-log only sends its overflow to the atomics
    const uint64_t cap = (h->flags & kDbgTinyLog)
                             ? 2
                             : std::min<uint64_t>(1u << 20, (nbytes / kRecBytes) / ((uint64_t)grid * parts) * 5 / 4 + 32);
    const size_t need = (size_t)grid * parts * cap * sizeof(uint4);  // (16 B slots; flushed slots take two)
    if (need > h->tlog_bytes || (size_t)grid * parts > h->tlog_cnt_cap) {
      HIP_TRY(h, hipStreamSynchronize(h->stream));  // an earlier launch may still read the old log
      if (need > h->tlog_bytes) {
        (void)hipFree(h->d_tlog);
        h->d_tlog = nullptr;
        h->tlog_bytes = 0;
        HIP_TRY(h, hipMalloc(&h->d_tlog, need));
        h->tlog_bytes = need;
      }
      if ((size_t)grid * parts > h->tlog_cnt_cap) {
        (void)hipFree(h->d_tlog_cnt);
        h->d_tlog_cnt = nullptr;
        h->tlog_cnt_cap = 0;
        HIP_TRY(h, hipMalloc(&h->d_tlog_cnt, (size_t)grid * parts * 4));
        h->tlog_cnt_cap = (size_t)grid * parts;
      }
    }
    p.tlog = h->d_tlog;
    p.tlog_cnt = h->d_tlog_cnt;
    p.tlog_cap = (uint32_t)cap;
    p.tlog_rshift = rshift;
    p.tlog_parts = parts;
  }
  int slot = 0;
  int rc = launch_events(h, &slot);
  if (rc) return rc;
  HIP_TRY(h, hipEventRecord(h->ring0[slot], h->stream));
  if (nb) {
    if (h->flags & kDbgTiming) {
      const size_t n = (size_t)grid * (kWG / 64) * kTimingWords;
      if (n > h->dbg_cap) {
        (void)hipFree(h->d_dbg);
        h->d_dbg = nullptr;
        HIP_TRY(h, hipMalloc(&h->d_dbg, n * 8));
        h->dbg_cap = n;
      }
      HIP_TRY(h, hipMemsetAsync(h->d_dbg, 0, n * 8, h->stream));
      h->dbg_len = n;
      p.dbg = reinterpret_cast<unsigned long long*>(h->d_dbg);
      HIP_TRY(h, launch_attribute(true, mode, grid, h->stream, p));
    } else {
      HIP_TRY(h, launch_attribute(false, mode, grid, h->stream, p));
    }
    HIP_TRY(h, hipEventRecord(h->ringr[slot], h->stream));
    HIP_TRY(h, hipEventRecord(h->ringm[slot], h->stream));
    if (p.tlog) {  // sums the log per entry range, folds the packed counters
      TlogParams r;
      r.tlog = p.tlog;
      r.tlog_cnt = p.tlog_cnt;
      r.sum64 = h->d_sum64;
      r.min64 = h->d_min64;
      r.pk64 = p.pk64;
      r.grid = grid;
      r.parts = p.tlog_parts;
      r.cap = p.tlog_cap;
      r.rshift = p.tlog_rshift;
      r.nb_entries = h->E;
      r.pk_shift = p.pk_shift;
      HIP_TRY(h, launch_tlog_reduce(p.tlog_parts, h->stream, r));
    } else if (p.pk64) {
      const uint32_t blocks = (uint32_t)std::min<uint64_t>(2048, (2ull * h->E + 255) / 256);
      HIP_TRY(h, launch_unpack(blocks, h->stream, h->d_sum64, p.pk64, h->E, p.pk_shift));
    }
  }
  if (!nb) {
    HIP_TRY(h, hipEventRecord(h->ringr[slot], h->stream));
    HIP_TRY(h, hipEventRecord(h->ringm[slot], h->stream));
  }
  HIP_TRY(h, hipEventRecord(h->ring1[slot], h->stream));
  h->nlaunch++;
  h->launched = true;
  return NMG_OK;
}

// ---------------------------------------------------------------------------
// partition-first path (nmg_route.h): eligibility, pool sizing, launches

static uint32_t bits_for(uint64_t v) {  // smallest b with v < 2^b
  uint32_t b = 0;
  while (b < 64 && (v >> b) != 0) b++;
  return b;
}

// X word layout of the current buffers; false when the weight field would
// be narrower than kMinWeightBits (escapes would be common)
static bool route_layout(nmg_engine* h, const std::vector<BufDesc>& descs, XLayout& xl) {
  uint64_t maxlen = 1;
  for (const BufDesc& d : descs) maxlen = std::max<uint64_t>(maxlen, d.len);
  xl.gbits = bits_for(descs.size() - 1);
  xl.obits = bits_for((maxlen - 1) / 8);
  xl.tbits = bits_for(h->T - 1);
  const uint32_t loc = xl.gbits + xl.obits + xl.tbits + 1;  // (+ access bit)
  if (loc > 48 - kMinWeightBits || xl.gbits > 31 || xl.obits > 31 || xl.tbits > 31) return false;
  xl.wbits = std::min<uint32_t>(48 - loc, 16);  // (the decode reads at most 16 bits of weight)
  xl.wesc = (1ull << xl.wbits) - 1;
  xl.tbase = h->route_tbase;
  return true;
}

// the partition-first path for this buffer set (the submitted buffers, or a
// streamed chunk of them)
static bool route_eligible(nmg_engine* h, const std::vector<BufDesc>& descs) {
  constexpr uint32_t kLegacyOnly = kDbgLoadOnly | kDbgNoGlobal | kDbgNoFlush | kDbgNoTables | kDbgTiming |
                                   kDbgTinyLog | kDbgNoPack | kDbgNoDir | kDbgNoRoute | NMG_F_SINGLE_PASS;
  if (!h->route_ok || (h->flags & kLegacyOnly) || descs.empty()) return false;
  // the first-match ordinal is rebuilt from the buffer index: seq = seq0 + index
  uint64_t bytes = 0;
  for (size_t i = 0; i < descs.size(); i++) {
    if (descs[i].seq != descs[0].seq + i) return false;
    bytes += descs[i].len;
  }
  // chunk ids (route pass LDS: id << 7 | fill) -- an upper bound of the pool
  const uint64_t chunks = (bytes / kRecBytes + descs.size()) / kChunk + (uint64_t)h->num_cus * (2 * h->nparts + 2);
  if (chunks >= (1ull << kChunkIdBits)) return false;
  XLayout xl;
  return route_layout(h, descs, xl);
}
static bool route_eligible(nmg_engine* h) { return route_eligible(h, h->descs); }

// per-workgroup private chunk pools for a new schedule: every SAMPLE record
// of at least 40 B fits (a partition's chunks are full but for its open and
// next chunks); shorter records past that are attributed directly
static int route_pool(nmg_engine* h, const std::vector<BufDesc>& descs, uint32_t grid, const uint32_t* ranges,
                      std::vector<uint32_t>& c0) {
  const uint32_t P = h->nparts;
  c0.assign(grid + 1, 0);
  uint64_t tot = 0;
  for (uint32_t w = 0; w < grid; w++) {
    uint64_t rec = 0;
    for (uint32_t b = ranges[w]; b < ranges[w + 1]; b++) rec += (descs[b].len + kRecBytes - 1) / kRecBytes;
    // (route2_kernel keeps two chunks open per partition: the open one and
    // the next, opened ahead)
    const uint64_t cap = (h->flags & kDbgTinyPool) ? 2 : (rec + kChunk - 1) / kChunk + 2 * P;
    c0[w] = (uint32_t)tot;
    tot += cap;
  }
  c0[grid] = (uint32_t)tot;
  if (tot >= (1ull << kChunkIdBits)) return fail(h, NMG_ERR_RANGE, "partition-first chunk pool too large");
  const size_t items = tot / kItemChunks + P + 1;
  // overflow list: records past a full pool (only SAMPLE records shorter than
  // 40 B can get there; kDbgTinyPool sends nearly all of them)
  uint64_t recs = 0;
  for (const BufDesc& d : descs) recs += (d.len + kRecBytes - 1) / kRecBytes;
  // (a quarter of the records, plus up to three times them for batches under 4M records)
  const size_t ovf = (size_t)((h->flags & kDbgTinyPool) ? recs : recs / 4 + std::min<uint64_t>(3 * recs, 4u << 20)) + 65536;
  if (tot > h->route_chunk_cap || items > h->items_cap || grid > h->route_grid_cap || ovf > h->ovf_cap) {
    HIP_TRY(h, hipStreamSynchronize(h->stream));  // a launch in flight may still read the old pool
    const bool pending = h->route_pending;
    free_route_pool(h);
    h->route_pending = pending;
    const size_t cap = std::max<size_t>(tot, 1);
    HIP_TRY(h, hipMalloc(&h->d_rec16, cap * kChunk * sizeof(uint4)));
    HIP_TRY(h, hipMalloc(&h->d_cmeta, cap * 4));
    HIP_TRY(h, hipMalloc(&h->d_cmatch, cap * 8));
    HIP_TRY(h, hipMalloc(&h->d_clist, cap * 4));
    HIP_TRY(h, hipMalloc(&h->d_items, items * sizeof(uint4)));
    HIP_TRY(h, hipMalloc(&h->d_chunk0, (grid + 1) * 4));
    HIP_TRY(h, hipMalloc(&h->d_used, grid * 4));
    HIP_TRY(h, hipMalloc(&h->d_pcnt, (size_t)grid * (kMaxParts + 1) * 4));
    HIP_TRY(h, hipMalloc(&h->d_pbase, (kMaxParts + 1) * 4));
    HIP_TRY(h, hipMalloc(&h->d_ctl, 3 * 4));
    HIP_TRY(h, hipMemset(h->d_ctl, 0, 3 * 4));
    HIP_TRY(h, hipMalloc(&h->d_ovf16, ovf * sizeof(uint4)));
    HIP_TRY(h, hipMalloc(&h->d_ovfx, ovf * 8));
    h->ovf_cap = ovf;
    h->route_chunk_cap = cap;
    h->items_cap = items;
    h->route_grid_cap = grid;
  }
  return NMG_OK;
}

static int route_prepare(nmg_engine* h, uint32_t grid, const std::vector<uint32_t>& ranges) {
  std::vector<uint32_t> c0;
  const int rc = route_pool(h, h->descs, grid, ranges.data(), c0);
  if (rc) return rc;
  HIP_TRY(h, hipMemcpy(h->d_chunk0, c0.data(), (grid + 1) * 4, hipMemcpyHostToDevice));
  h->route_sched_key = h->nparts | ((h->flags & kDbgTinyPool) ? 0x80000000u : 0u);
  return NMG_OK;
}



// Route -> plan -> scatter -> local over the buffers of the current schedule
// (analysis order), bracketed by the launch-timing events.
static int route_analyze(nmg_engine* h, uint32_t nb, uint32_t grid) {
  (void)nb;
  RouteJob job{&h->descs, h->d_data, h->d_sdescs, h->d_ranges, h->d_chunk0, grid, 0, false};
  return route_analyze_job(h, job);
}

static int route_analyze_job(nmg_engine* h, const RouteJob& job) {
  Range range("nmg_route");
  XLayout xl;
  if (!route_layout(h, *job.descs, xl)) return fail(h, NMG_ERR_STATE, "route layout");
  const uint32_t grid = job.grid;
  Params base = base_params(h, job.data, job.sdescs, job.ranges);
  base.bufcnt = h->d_bufcnt + job.index_base;  // (count slots of the set's first buffer)
  const uint64_t seq0 = (*job.descs)[0].seq;
  h->route_launches++;
  int slot = 0;
  int rc = launch_events(h, &slot);
  if (rc) return rc;
  HIP_TRY(h, hipEventRecord(h->ring0[slot], h->stream));
  RouteParams rp;
  memset(&rp, 0, sizeof(rp));
  rp.p = base;
  rp.pbounds = h->d_pbounds;
  rp.pdir = h->d_pdir;
  for (uint32_t k = 0; k < kRouteSegs; k++) rp.seg[k] = h->rsegs[k];
  rp.nseg = h->nrsegs;
  rp.nparts = h->nparts;
  rp.xl = xl;
  rp.seq0 = seq0;
  rp.rec16 = h->d_rec16;
  rp.cmeta = h->d_cmeta;
  rp.chunk0 = job.chunk0;
  rp.used = h->d_used;
  rp.ovf16 = h->d_ovf16;
  rp.ovfx = h->d_ovfx;
  rp.ovf_cnt = h->d_ctl + 2;
  rp.ovf_cap = (uint32_t)std::min<size_t>(h->ovf_cap, 0xffffffffu);
  if (h->flags & kDbgTinyOvf) rp.ovf_cap = std::min<uint32_t>(rp.ovf_cap, 64);  // (tests: the direct attribution past a full list)
  if (h->flags & kDbgRouteTiming) {  // (internal) per-wave phase cycles, read by nmg_debug_timing
    const size_t n = (size_t)grid * (kWG / 64) * kRouteTimingWords;
    if (n > h->dbg_cap) {
      (void)hipFree(h->d_dbg);
      h->d_dbg = nullptr;
      HIP_TRY(h, hipMalloc(&h->d_dbg, n * 8));
      h->dbg_cap = n;
    }
    HIP_TRY(h, hipMemsetAsync(h->d_dbg, 0, n * 8, h->stream));
    h->dbg_len = n;
    rp.p.dbg = reinterpret_cast<unsigned long long*>(h->d_dbg);
  }
  HIP_TRY(h, launch_route(grid, h->stream, rp));
  HIP_TRY(h, hipEventRecord(h->ringr[slot], h->stream));
  HIP_TRY(h, launch_overflow(h->stream, rp));
  ScatterParams sc;
  sc.cmeta = h->d_cmeta;
  sc.chunk0 = job.chunk0;
  sc.used = h->d_used;
  sc.pcnt = h->d_pcnt;
  sc.pbase = h->d_pbase;
  sc.clist = h->d_clist;
  sc.nparts = h->nparts;
  CountParams cp;
  memset(&cp, 0, sizeof(cp));
  cp.sc = sc;
  HIP_TRY(h, launch_count(grid, h->stream, cp));
  PlanParams pl;
  pl.pcnt = h->d_pcnt;
  pl.pbase = h->d_pbase;
  pl.items = h->d_items;
  pl.ctl = h->d_ctl;
  pl.grid = grid;
  pl.nparts = h->nparts;
  HIP_TRY(h, launch_plan(h->stream, pl));
  HIP_TRY(h, launch_scatter(grid, h->stream, sc));
  LocalParams lp;
  memset(&lp, 0, sizeof(lp));
  lp.p = base;
  lp.parts = h->d_parts;
  lp.pe_keys = h->d_pe_keys;
  lp.pe_nodes = h->d_pe_nodes;
  lp.pe_info = h->d_pe_info;
  lp.pe_dir = h->d_pe_dir;
  lp.pe_ids = h->d_pe_ids;
  lp.pe_lrel = h->d_pe_lrel;
  lp.pe_cmap = h->d_pe_cmap;
  lp.rec16 = h->d_rec16;
  lp.cmeta = h->d_cmeta;
  lp.clist = h->d_clist;
  lp.items = h->d_items;
  lp.ctl = h->d_ctl;
  lp.cmatch = h->d_cmatch;
  lp.descs = job.sdescs;
  lp.xl = xl;
  lp.seq0 = seq0;
  if ((h->flags & kDbgLocalTiming) && !(h->flags & kDbgRouteTiming)) {  // (internal) per-wave phase cycles
    const size_t n = (size_t)h->num_cus * (kWG / 64) * kRouteTimingWords;
    if (n > h->dbg_cap) {
      (void)hipFree(h->d_dbg);
      h->d_dbg = nullptr;
      HIP_TRY(h, hipMalloc(&h->d_dbg, n * 8));
      h->dbg_cap = n;
    }
    HIP_TRY(h, hipMemsetAsync(h->d_dbg, 0, n * 8, h->stream));
    h->dbg_len = n;
    lp.p.dbg = reinterpret_cast<unsigned long long*>(h->d_dbg);
  }
  HIP_TRY(h, launch_local((uint32_t)h->num_cus, h->stream, lp));
  HIP_TRY(h, hipEventRecord(h->ringm[slot], h->stream));
  HIP_TRY(h, hipEventRecord(h->ring1[slot], h->stream));
  h->nlaunch++;
  h->launched = true;
  if (job.settle_now) {  // (a streamed chunk: the next one reuses the pool)
    FoundParams f;
    f.ranges = job.ranges;
    f.chunk0 = job.chunk0;
    f.used = h->d_used;
    f.cmeta = h->d_cmeta;
    f.cmatch = h->d_cmatch;
    f.rec16 = h->d_rec16;
    f.bufcnt = h->d_bufcnt + job.index_base;
    f.nb_bufs = (uint32_t)h->bufcnt_stride;
    f.gbits = xl.gbits;
    f.gshift = 16 + xl.wbits;
    HIP_TRY(h, launch_found(grid, h->stream, f));
    return NMG_OK;
  }
  h->route_pending = true;
  h->route_grid = grid;
  h->route_xl = xl;
  return NMG_OK;
}

// Per-buffer matched-sample counts of the last route analysis (found_kernel),
// enqueued before anything reads or replaces them.  A reset drops them
// instead: it zeroes those counts anyway.
static int route_settle(nmg_engine* h) {
  if (!h->route_pending) return NMG_OK;
  h->route_pending = false;
  FoundParams f;
  f.ranges = h->d_ranges;
  f.chunk0 = h->d_chunk0;
  f.used = h->d_used;
  f.cmeta = h->d_cmeta;
  f.cmatch = h->d_cmatch;
  f.rec16 = h->d_rec16;
  f.bufcnt = h->d_bufcnt;
  f.nb_bufs = (uint32_t)h->bufcnt_stride;
  f.gbits = h->route_xl.gbits;
  f.gshift = 16 + h->route_xl.wbits;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, launch_found(h->route_grid, h->stream, f));
  return NMG_OK;
}

static int stream_flush(nmg_engine* h);

static int multi_analyze(nmg_engine* h);
static int multi_finish(nmg_engine* h);
static int multi_buffer_found(nmg_engine* h, std::vector<uint32_t>& nf);

extern "C" int nmg_analyze(nmg_engine* h) {
  if (h) h->epoch++;
  Range range("nmg_analyze");
  if (!h) return NMG_ERR_INVALID;
  if (!h->have_table) return fail(h, NMG_ERR_STATE, "nmg_analyze before nmg_set_objects");
  if (h->multi) return multi_analyze(h);
  HIP_TRY(h, hipSetDevice(h->device));
  int rc = route_settle(h);  // the previous analysis' per-buffer counts, before the pool is reused
  if (rc) return rc;
  if (h->streaming) return stream_flush(h);  // earlier chunks are already enqueued
  if (h->streamed) return NMG_OK;             // nmg_stream_end flushed everything
  const bool resched = h->descs_dirty;
  rc = upload_buffers(h);
  if (rc) return rc;
  const uint32_t nb = (uint32_t)h->descs.size();
  if (h->flags & NMG_F_SAMPLE_MATCHES) {  // one u32 per 8 B of the buffers' arena span
    uint64_t span = 0;
    for (const BufDesc& d : h->descs) span = std::max<uint64_t>(span, d.offset + d.len);
    const size_t need = (size_t)(span / 8 + 1);
    if (need > h->smatch_cap) {
      HIP_TRY(h, hipStreamSynchronize(h->stream));
      (void)hipFree(h->d_smatch);
      h->d_smatch = nullptr;
      HIP_TRY(h, hipMalloc(&h->d_smatch, need * 4));
      h->smatch_cap = need;
    }
  }
  const uint32_t grid = attribution_grid(h, nb);
  if (route_eligible(h)) {
    if (nb && (resched || grid != h->sched_grid || !h->sched_route ||
               h->route_sched_key != (h->nparts | ((h->flags & kDbgTinyPool) ? 0x80000000u : 0u)))) {
      rc = build_schedule(h, grid, false);
      if (rc) return rc;
    }
    return route_analyze(h, nb, grid);
  }
  if (nb && (resched || grid != h->sched_grid || h->sched_route)) {
    rc = build_schedule(h, grid);
    if (rc) return rc;
  }
  uint64_t nbytes = 0;
  for (const BufDesc& d : h->descs) nbytes += d.len;
  return launch_attribution(h, h->d_data, h->d_sdescs, h->d_ranges, nb, grid, nbytes);
}

static int decode_error_word(nmg_engine* h, uint64_t w) {
  if (w == ~0ull) return NMG_OK;
  uint32_t code = w & 0xff;
  uint64_t seq = w >> 40;
  uint32_t off = (uint32_t)((w >> 8) & 0xffffffffu);
  char msg[256];
  snprintf(msg, sizeof(msg), "buffer %llu (analysis order), byte offset %u: ", (unsigned long long)seq, off);
  switch (code) {
    case kErrZeroSize: return fail(h, NMG_ERR_ZERO_SIZE, std::string(msg) + "invalid header size = 0");
    case kErrTruncated: return fail(h, NMG_ERR_TRUNCATED, std::string(msg) + "truncated record");
    case kErrUnaligned: return fail(h, NMG_ERR_UNALIGNED, std::string(msg) + "unaligned record");
    case kErrCapacity: return fail(h, NMG_ERR_CAPACITY, std::string(msg) + "sparse table full");
    case kErrRouteOverflow:
      return fail(h, NMG_ERR_CAPACITY, std::string(msg) + "too many SAMPLE records shorter than 40 B for the "
                  "partition-first overflow list (use NMG_F_SINGLE_PASS)");
    default: return fail(h, NMG_ERR_RANGE, std::string(msg) + "range error");
  }
}

extern "C" int nmg_synchronize(nmg_engine* h) {
  if (!h) return NMG_ERR_INVALID;
  if (h->multi_pending) {
    const int rc = multi_finish(h);
    if (rc) return rc;
  }
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  if (h->launched) {  // the most recent launch's start / end events
    const int slot = (int)((h->nlaunch - 1) % nmg_engine::kRing);
    HIP_TRY(h, hipEventElapsedTime(&h->last_ms, h->ring0[slot], h->ring1[slot]));
  }
  if (!h->have_table) return NMG_OK;
  uint64_t w = ~0ull;
  HIP_TRY(h, hipMemcpy(&w, h->d_min64 + 36 + h->E, 8, hipMemcpyDeviceToHost));
  return decode_error_word(h, w);
}

extern "C" int nmg_get_launch_times(nmg_engine* h, float* ms, int n) {
  if (!h || (n > 0 && !ms)) return NMG_ERR_INVALID;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  const int avail = (int)std::min<uint64_t>(h->nlaunch, nmg_engine::kRing);
  const int cnt = std::min(n, avail);
  for (int i = 0; i < cnt; i++) {  // the cnt most recent launches, oldest first
    const int slot = (int)((h->nlaunch - cnt + i) % nmg_engine::kRing);
    HIP_TRY(h, hipEventElapsedTime(&ms[i], h->ring0[slot], h->ring1[slot]));
  }
  return cnt;
}

extern "C" int nmg_get_kernel_times(nmg_engine* h, float* attribute_ms, float* total_ms, int n) {
  if (!h || (n > 0 && (!attribute_ms || !total_ms))) return NMG_ERR_INVALID;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  const int avail = (int)std::min<uint64_t>(h->nlaunch, nmg_engine::kRing);
  const int cnt = std::min(n, avail);
  for (int i = 0; i < cnt; i++) {
    const int slot = (int)((h->nlaunch - cnt + i) % nmg_engine::kRing);
    HIP_TRY(h, hipEventElapsedTime(&attribute_ms[i], h->ring0[slot], h->ringm[slot]));
    HIP_TRY(h, hipEventElapsedTime(&total_ms[i], h->ring0[slot], h->ring1[slot]));
  }
  return cnt;
}

extern "C" int nmg_last_analyze_ms(nmg_engine* h, float* ms) {
  if (!h || !ms) return NMG_ERR_INVALID;
  *ms = h->last_ms;
  return NMG_OK;
}

extern "C" uint32_t nmg_get_nb_buffers(nmg_engine* h) {
  if (!h) return 0;
  return h->counts_override ? (uint32_t)h->ov_samples.size() : (uint32_t)h->descs.size();
}

namespace nmg {
int engine_download(nmg_engine* h, HostResults& r, bool entries, bool buffer_found) {
  if (buffer_found && !h->counts_override && !h->multi) {
    // per-buffer matched counts of the partition-first path: found_kernel
    // over the match bits (only for callers of the per-buffer counts; the
    // total below is counted by the analysis itself)
    HIP_TRY(h, hipSetDevice(h->device));
    const int rc = route_settle(h);
    if (rc) return rc;
  }
  int rc = nmg_synchronize(h);
  if (rc) return rc;
  // (entries == false: the global counters and per-buffer counts only, not
  // the per-entry arrays -- 40 MB at 1M entries)
  const uint64_t ns = entries ? h->n_sum64 : 2 * kGlobalSums, nm = entries ? h->n_min64 : 36;
  std::vector<uint64_t> sum(ns), mn(nm), mx(h->n_max64);
  HIP_TRY(h, hipMemcpy(sum.data(), h->d_sum64, ns * 8, hipMemcpyDeviceToHost));
  HIP_TRY(h, hipMemcpy(mn.data(), h->d_min64, nm * 8, hipMemcpyDeviceToHost));
  HIP_TRY(h, hipMemcpy(mx.data(), h->d_max64, h->n_max64 * 8, hipMemcpyDeviceToHost));
  for (int a = 0; a < 2; a++) {
    nmg_mem_counters& c = r.global[a];
    const uint64_t* s = sum.data() + gsum_index(a, 0);
    c.total_count = s[0];
    c.total_weight = s[1];
    c.na_miss_count = s[2];
    for (int k = 0; k < 18; k++) {
      c.b[k].count = s[3 + 2 * k];
      c.b[k].sum_weight = s[4 + 2 * k];
      c.b[k].min_weight = mn[a * 18 + k];
      c.b[k].max_weight = mx[a * 18 + k];
    }
  }
  const uint64_t E = entries ? h->E : 0;
  r.first.assign(mn.begin() + 36, mn.begin() + 36 + E);
  r.count_weight.resize(4 * E);  // SoA [2][2][E] -> [E][2][2]
  for (uint64_t e = 0; e < E; e++)
    for (uint32_t a = 0; a < 2; a++)
      for (uint32_t w = 0; w < 2; w++) r.count_weight[e * 4 + a * 2 + w] = sum[objcw_index(e, a, w, E)];
  if ((h->flags & NMG_F_OBJECT_LEVELS) && entries)
    r.levels.assign(sum.begin() + 2 * kGlobalSums + 4 * E, sum.end());
  else
    r.levels.clear();
  // mem_sampling_finalize accumulates the per-buffer int counters (:334-335);
  // a buffer holds < 2^29 records (< 4 GiB, Q14), so their sum is the
  // matched-sample total the kernels count (Params::found)
  r.nb_samples_total = 0;
  r.nb_found_total = 0;
  if (h->multi) {
    r.buf_samples = h->ov_samples;
    r.buf_bytes = h->ov_bytes;
    r.buf_found.assign(r.buf_samples.size(), 0);
    if (buffer_found && !r.buf_samples.empty()) {
      const int frc = multi_buffer_found(h, r.buf_found);
      if (frc) return frc;
    }
    r.nb_found_total = h->multi_found;
  } else if (h->counts_override) {
    r.buf_samples = h->ov_samples;
    r.buf_found = h->ov_found;
    r.buf_bytes = h->ov_bytes;
    for (size_t b = 0; b < r.buf_found.size(); b++) r.nb_found_total += (uint64_t)(int64_t)(int32_t)r.buf_found[b];
  } else {
    const size_t n = h->descs.size();
    r.buf_samples.assign(n, 0);
    r.buf_found.assign(n, 0);
    if (n) {
      HIP_TRY(h, hipMemcpy(r.buf_samples.data(), h->d_bufcnt, n * 4, hipMemcpyDeviceToHost));
      if (buffer_found)
        HIP_TRY(h, hipMemcpy(r.buf_found.data(), h->d_bufcnt + h->bufcnt_stride, n * 4, hipMemcpyDeviceToHost));
    }
    r.buf_bytes = h->buf_bytes;
    uint64_t found = 0;
    if (h->d_found) HIP_TRY(h, hipMemcpy(&found, h->d_found, 8, hipMemcpyDeviceToHost));
    r.nb_found_total = found;
  }
  for (size_t b = 0; b < r.buf_samples.size(); b++) r.nb_samples_total += (uint64_t)(int64_t)(int32_t)r.buf_samples[b];
  return NMG_OK;
}

int engine_download_hist(nmg_engine* h, std::vector<uint32_t>& cells) {
  int rc = nmg_synchronize(h);
  if (rc) return rc;
  cells.resize(h->hist_cells * h->T);
  if (h->hist_cells) HIP_TRY(h, hipMemcpy(cells.data(), h->d_hist, cells.size() * 4, hipMemcpyDeviceToHost));
  return NMG_OK;
}
}  // namespace nmg

extern "C" int nmg_get_global_counters(nmg_engine* h, nmg_mem_counters out[2], uint64_t* nb_samples,
                                       uint64_t* nb_found) {
  if (!h || !out) return NMG_ERR_INVALID;
  if (!h->have_table) return fail(h, NMG_ERR_STATE, "no object table");
  HostResults r;
  int rc = engine_download(h, r, false, false);
  if (rc) return rc;
  out[0] = r.global[0];
  out[1] = r.global[1];
  if (nb_samples) *nb_samples = r.nb_samples_total;
  if (nb_found) *nb_found = r.nb_found_total;
  return NMG_OK;
}

extern "C" int nmg_get_buffer_counts(nmg_engine* h, uint32_t* nb_samples, uint32_t* nb_found) {
  if (!h) return NMG_ERR_INVALID;
  if (!h->have_table) return fail(h, NMG_ERR_STATE, "no object table");
  HostResults r;
  int rc = engine_download(h, r, false, true);
  if (rc) return rc;
  if (nb_samples) memcpy(nb_samples, r.buf_samples.data(), r.buf_samples.size() * 4);
  if (nb_found) memcpy(nb_found, r.buf_found.data(), r.buf_found.size() * 4);
  return NMG_OK;
}

extern "C" int nmg_get_object_counters(nmg_engine* h, uint64_t* first_ordinal, uint64_t* count_weight) {
  if (!h) return NMG_ERR_INVALID;
  if (!h->have_table) return fail(h, NMG_ERR_STATE, "no object table");
  int rc = nmg_synchronize(h);
  if (rc) return rc;
  if (first_ordinal && h->E)
    HIP_TRY(h, hipMemcpy(first_ordinal, h->d_min64 + 36, (size_t)h->E * 8, hipMemcpyDeviceToHost));
  if (count_weight && h->E) {  // the SoA rows laid out per entry on the device, then one copy
    static_assert(objcw_index(1, 0, 0, 8) - objcw_index(0, 0, 0, 8) == 1 && objcw_index(0, 0, 1, 8) - objcw_index(0, 0, 0, 8) == 8 &&
                      objcw_index(0, 1, 0, 8) - objcw_index(0, 0, 0, 8) == 16,
                  "objcw_aos_kernel reads rows access * 2 + w");
    if (h->E > h->objcw_cap) {
      (void)hipFree(h->d_objcw);
      h->d_objcw = nullptr;
      h->objcw_cap = 0;
      HIP_TRY(h, hipMalloc(&h->d_objcw, (size_t)h->E * 32));
      h->objcw_cap = h->E;
    }
    HIP_TRY(h, launch_objcw_aos(h->stream, h->d_sum64 + 2 * kGlobalSums, h->E, h->d_objcw));
    HIP_TRY(h, hipMemcpyAsync(count_weight, h->d_objcw, (size_t)h->E * 32, hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(h, hipStreamSynchronize(h->stream));
  }
  return NMG_OK;
}

extern "C" int nmg_get_object_levels(nmg_engine* h, uint64_t* levels) {
  if (!h || !levels) return NMG_ERR_INVALID;
  if (!(h->flags & NMG_F_OBJECT_LEVELS)) return fail(h, NMG_ERR_STATE, "engine created without NMG_F_OBJECT_LEVELS");
  int rc = nmg_synchronize(h);
  if (rc) return rc;
  if (h->E)
    HIP_TRY(h, hipMemcpy(levels, h->d_sum64 + 2 * kGlobalSums + (uint64_t)h->E * 4,
                         (size_t)h->E * 2 * kLevelWords * 8, hipMemcpyDeviceToHost));
  return NMG_OK;
}

static int sparse_nonempty(nmg_engine* h, bool* out);
static int sparse_download(nmg_engine* h, std::vector<uint64_t>& k, std::vector<uint32_t>& v);

// Every non-zero (entry, thread, page) cell, entries in id order, each
// entry's cells in (thread, page) order.  Dense cells are counted and
// compacted into rows on the device (cells_count / cells_emit); the rows stay
// there (d_cells_rows) until copied out, so only they cross PCIe, once.  The
// sparse table's cells (entries past the dense budget, e.g. [stack]) are
// grouped on the host and placed at their entries' offsets.  Cached per
// results epoch: nmg_count_page_cells then nmg_get_page_cells does the work
// once.
static int cells_prepare(nmg_engine* h) {
  if (h->cells_epoch == h->epoch) return NMG_OK;
  int rc = nmg_synchronize(h);
  if (rc) return rc;
  const uint32_t E = h->E;
  // sparse cells grouped per entry
  std::vector<std::vector<std::pair<uint64_t, uint32_t>>> sparse(h->sparse_entries.size());
  bool any_sparse = false;
  rc = sparse_nonempty(h, &any_sparse);
  if (rc) return rc;
  if (any_sparse) {
    std::vector<uint64_t> k;
    std::vector<uint32_t> v;
    rc = sparse_download(h, k, v);
    if (rc) return rc;
    for (size_t i = 0; i < k.size(); i++)
      if (k[i] != ~0ull && v[i]) {
        uint32_t s = sparse_key_idx(k[i]);
        // order within an entry: (thread, page)
        sparse[s].push_back({(uint64_t(sparse_key_thread(k[i])) << 32) | sparse_key_page(k[i]), v[i]});
      }
    for (auto& l : sparse) std::sort(l.begin(), l.end());
  }
  std::vector<int64_t> sidx_of(E, -1);
  for (size_t s = 0; s < h->sparse_entries.size(); s++) sidx_of[h->sparse_entries[s]] = (int64_t)s;
  std::vector<uint32_t> cnt(E, 0);
  uint64_t *d_base = nullptr, *d_off = nullptr;
  uint32_t *d_np = nullptr, *d_cnt = nullptr;
  auto cleanup = [&]() {
    (void)hipFree(d_base);
    (void)hipFree(d_off);
    (void)hipFree(d_np);
    (void)hipFree(d_cnt);
  };
  auto hip = [&](hipError_t e, const char* what) {
    if (e == hipSuccess) return NMG_OK;
    cleanup();
    return fail(h, NMG_ERR_HIP, std::string("page cells: ") + what + ": " + hipGetErrorString(e));
  };
  const bool dense = h->hist_cells && E;
  if (dense) {
    std::vector<uint32_t> np(E);
    for (uint32_t e = 0; e < E; e++) np[e] = h->hist_base[e] == kHistSparse ? 0u : (uint32_t)h->npages[e];
    if ((rc = hip(hipMalloc(&d_base, (size_t)E * 8), "alloc")) || (rc = hip(hipMalloc(&d_np, (size_t)E * 4), "alloc")) ||
        (rc = hip(hipMalloc(&d_cnt, (size_t)E * 4), "alloc")) ||
        (rc = hip(hipMemcpyAsync(d_base, h->hist_base.data(), (size_t)E * 8, hipMemcpyHostToDevice, h->stream), "upload")) ||
        (rc = hip(hipMemcpyAsync(d_np, np.data(), (size_t)E * 4, hipMemcpyHostToDevice, h->stream), "upload")) ||
        (rc = hip(launch_cells_count(h->stream, h->d_hist, h->hist_cells, h->T, d_base, d_np, E, d_cnt), "count")) ||
        (rc = hip(hipMemcpyAsync(cnt.data(), d_cnt, (size_t)E * 4, hipMemcpyDeviceToHost, h->stream), "counts")) ||
        (rc = hip(hipStreamSynchronize(h->stream), "count")))
      return rc;
  }
  std::vector<uint64_t> off(E);
  uint64_t n = 0;
  h->cells_sparse.clear();
  for (uint32_t e = 0; e < E; e++) {
    off[e] = n;
    if (sidx_of[e] >= 0 && h->hist_base[e] == kHistSparse) {
      auto& l = sparse[sidx_of[e]];
      const uint64_t k = l.size();
      if (k) h->cells_sparse.push_back({n, e, std::move(l)});
      n += k;
    } else {
      n += cnt[e];
    }
  }
  if (dense && n) {
    if (n > h->cells_rows_cap) {
      (void)hipFree(h->d_cells_rows);
      h->d_cells_rows = nullptr;
      h->cells_rows_cap = 0;
      if ((rc = hip(hipMalloc(&h->d_cells_rows, n * 16), "alloc"))) return rc;
      h->cells_rows_cap = n;
    }
    if ((rc = hip(hipMalloc(&d_off, (size_t)E * 8), "alloc")) ||
        (rc = hip(hipMemcpyAsync(d_off, off.data(), (size_t)E * 8, hipMemcpyHostToDevice, h->stream), "upload")) ||
        (rc = hip(launch_cells_emit(h->stream, h->d_hist, h->hist_cells, h->T, d_base, d_np, E, d_off,
                                    (uint4*)h->d_cells_rows), "emit")) ||
        (rc = hip(hipStreamSynchronize(h->stream), "emit")))
      return rc;
  }
  cleanup();
  h->cells_n = (int64_t)n;
  h->cells_epoch = h->epoch;
  return NMG_OK;
}

// the prepared rows into rows[cells_n * 4]: dense rows D2H, sparse rows placed
static int cells_fill(nmg_engine* h, uint32_t* rows) {
  const bool dense = h->hist_cells && h->E;
  if (dense && h->cells_n)
    HIP_TRY(h, hipMemcpy(rows, h->d_cells_rows, (size_t)h->cells_n * 16, hipMemcpyDeviceToHost));
  for (const auto& g : h->cells_sparse) {
    uint32_t* r = rows + g.off * 4;
    for (const auto& kv : g.cells) {
      r[0] = g.e;
      r[1] = (uint32_t)(kv.first >> 32);
      r[2] = (uint32_t)kv.first;
      r[3] = kv.second;
      r += 4;
    }
  }
  return NMG_OK;
}
static int collect_page_cells(nmg_engine* h, std::vector<uint32_t>* rows, int64_t* count) {
  int rc = cells_prepare(h);
  if (rc) return rc;
  *count = h->cells_n;
  rows->resize((size_t)h->cells_n * 4);
  return cells_fill(h, rows->data());
}

extern "C" int64_t nmg_count_page_cells(nmg_engine* h) {
  if (!h || !h->have_table) return NMG_ERR_INVALID;
  int rc = cells_prepare(h);
  return rc ? rc : h->cells_n;
}

extern "C" int nmg_get_page_cells(nmg_engine* h, uint32_t* rows, int64_t n) {
  if (!h || !h->have_table || (n && !rows)) return NMG_ERR_INVALID;
  int rc = cells_prepare(h);
  if (rc) return rc;
  if (h->cells_n != n) return fail(h, NMG_ERR_INVALID, "row count mismatch");
  return n ? cells_fill(h, rows) : NMG_OK;
}

// ---- multi-GPU merge support

extern "C" uint64_t nmg_array_size(nmg_engine* h, int which) {
  if (!h || !h->have_table) return 0;
  switch (which) {
    case NMG_ARR_SUM64: return h->n_sum64;
    case NMG_ARR_MIN64: return h->n_min64;
    case NMG_ARR_MAX64: return h->n_max64;
    case NMG_ARR_HIST32: return h->hist_cells * h->T;
    default: return 0;
  }
}

static void* array_ptr(nmg_engine* h, int which, size_t* bytes) {
  switch (which) {
    case NMG_ARR_SUM64: *bytes = h->n_sum64 * 8; return h->d_sum64;
    case NMG_ARR_MIN64: *bytes = h->n_min64 * 8; return h->d_min64;
    case NMG_ARR_MAX64: *bytes = h->n_max64 * 8; return h->d_max64;
    case NMG_ARR_HIST32: *bytes = h->hist_cells * h->T * 4; return h->d_hist;
    default: *bytes = 0; return nullptr;
  }
}

extern "C" int nmg_export_array(nmg_engine* h, int which, void* d_dst) {
  Range range("nmg_export_array");
  if (!h || !h->have_table) return NMG_ERR_INVALID;
  size_t bytes = 0;
  void* src = array_ptr(h, which, &bytes);
  if (!bytes) return NMG_OK;
  if (!src || !d_dst) return NMG_ERR_INVALID;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipMemcpyAsync(d_dst, src, bytes, hipMemcpyDeviceToDevice, h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  return NMG_OK;
}

extern "C" int nmg_import_array(nmg_engine* h, int which, const void* d_src) {
  if (h) h->epoch++;
  Range range("nmg_import_array");
  if (!h || !h->have_table) return NMG_ERR_INVALID;
  size_t bytes = 0;
  void* dst = array_ptr(h, which, &bytes);
  if (!bytes) return NMG_OK;
  if (!dst || !d_src) return NMG_ERR_INVALID;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipMemcpyAsync(dst, d_src, bytes, hipMemcpyDeviceToDevice, h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  return NMG_OK;
}

static int scratch_u64(nmg_engine* h) {
  if (!h->d_scratch) HIP_TRY(h, hipMalloc(&h->d_scratch, 2 * 8 + 1024 * 4));  // + nmg_hist_pack's range counts
  return NMG_OK;
}

extern "C" int nmg_hist_pack(nmg_engine* h, uint32_t threshold, void* d_u8, void* d_ovf, uint64_t ovf_cap,
                             uint64_t* n_ovf) {
  Range range("nmg_hist_pack");
  if (!h || !h->have_table || !n_ovf || threshold > 255) return NMG_ERR_INVALID;
  const uint64_t cells = h->hist_cells * h->T;
  *n_ovf = 0;
  if (!cells) return NMG_OK;
  if (!d_u8 || (ovf_cap && !d_ovf)) return NMG_ERR_INVALID;
  if (cells > (1ull << 32)) return fail(h, NMG_ERR_RANGE, "nmg_hist_pack: more than 2^32 cells");
  int rc = scratch_u64(h);
  if (rc) return rc;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipMemsetAsync(h->d_scratch, 0, 8, h->stream));
  HIP_TRY(h, launch_hist_pack(h->stream, h->d_hist, cells, threshold, d_u8, d_ovf, ovf_cap,
                              reinterpret_cast<unsigned long long*>(h->d_scratch),
                              reinterpret_cast<uint32_t*>(h->d_scratch + 2)));
  HIP_TRY(h, hipMemcpyAsync(n_ovf, h->d_scratch, 8, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  return NMG_OK;
}

extern "C" int nmg_hist_unpack(nmg_engine* h, const void* d_u8, const void* d_ovf, uint64_t n_ovf) {
  if (h) h->epoch++;
  Range range("nmg_hist_unpack");
  if (!h || !h->have_table || (n_ovf && !d_ovf)) return NMG_ERR_INVALID;
  const uint64_t cells = h->hist_cells * h->T;
  if (!cells) return NMG_OK;
  if (!d_u8) return NMG_ERR_INVALID;
  int rc = scratch_u64(h);
  if (rc) return rc;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipMemsetAsync(h->d_scratch + 1, 0, 8, h->stream));
  HIP_TRY(h, launch_hist_unpack(h->stream, h->d_hist, cells, d_u8, d_ovf, n_ovf,
                                reinterpret_cast<unsigned long long*>(h->d_scratch + 1)));
  uint64_t bad = 0;
  HIP_TRY(h, hipMemcpyAsync(&bad, h->d_scratch + 1, 8, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  if (bad) return fail(h, NMG_ERR_RANGE, "nmg_hist_unpack: overflow entries outside the histogram");
  return NMG_OK;
}

// The sparse cells can be non-empty only when something was inserted (or
// imported) since the last reset: that reset cleared the table if it had been
// written, and the flag of the analyses after it is d_sparse_dirty[nreset & 1]
// (reset_kernel).  A 4-byte read instead of the whole table.
static int sparse_nonempty(nmg_engine* h, bool* out) {
  *out = false;
  if (!h->d_sparse_keys) return NMG_OK;
  uint32_t dirty = 1;
  HIP_TRY(h, hipMemcpy(&dirty, h->d_sparse_dirty + (h->nreset & 1), 4, hipMemcpyDeviceToHost));
  *out = dirty != 0;
  return NMG_OK;
}

static int sparse_download(nmg_engine* h, std::vector<uint64_t>& k, std::vector<uint32_t>& v) {
  int rc = nmg_synchronize(h);
  if (rc) return rc;
  bool any = false;
  rc = sparse_nonempty(h, &any);
  if (rc) return rc;
  if (!any) {
    k.clear();
    v.clear();
    return NMG_OK;
  }
  // the used slots compacted on the device (key, count pairs), so only they
  // cross PCIe (the whole table is 12 MB at the default capacity)
  HIP_TRY(h, hipSetDevice(h->device));
  if (!h->d_sparse_ck) HIP_TRY(h, hipMalloc(&h->d_sparse_ck, (h->sparse_cap * 2 + 1) * 8));
  unsigned long long* cnt = reinterpret_cast<unsigned long long*>(h->d_sparse_ck + 2 * h->sparse_cap);
  HIP_TRY(h, hipMemsetAsync(cnt, 0, 8, h->stream));
  HIP_TRY(h, launch_sparse_compact(h->stream, h->d_sparse_keys, h->d_sparse_vals, h->sparse_cap, h->d_sparse_ck, cnt));
  uint64_t n = 0;
  HIP_TRY(h, hipMemcpyAsync(&n, cnt, 8, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  std::vector<uint64_t> kv(2 * n);
  if (n) HIP_TRY(h, hipMemcpy(kv.data(), h->d_sparse_ck, 2 * n * 8, hipMemcpyDeviceToHost));
  k.resize(n);
  v.resize(n);
  for (uint64_t i = 0; i < n; i++) {
    k[i] = kv[2 * i];
    v[i] = (uint32_t)kv[2 * i + 1];
  }
  return NMG_OK;
}

extern "C" int64_t nmg_sparse_count(nmg_engine* h) {
  if (!h || !h->have_table) return NMG_ERR_INVALID;
  std::vector<uint64_t> k;
  std::vector<uint32_t> v;
  int rc = sparse_download(h, k, v);
  return rc ? rc : (int64_t)k.size();
}

extern "C" int nmg_sparse_export(nmg_engine* h, uint64_t* keys, uint32_t* counts, int64_t n) {
  if (!h || !h->have_table || (n && (!keys || !counts))) return NMG_ERR_INVALID;
  std::vector<uint64_t> k;
  std::vector<uint32_t> v;
  int rc = sparse_download(h, k, v);
  if (rc) return rc;
  if ((int64_t)k.size() != n) return fail(h, NMG_ERR_INVALID, "sparse count mismatch");
  // in key order (the device compaction reserves its output slots per wave
  // with an atomic, so its order varies from run to run; keys are unique)
  std::vector<uint32_t> ord(k.size());
  for (uint32_t i = 0; i < (uint32_t)ord.size(); i++) ord[i] = i;
  std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return k[a] < k[b]; });
  for (int64_t i = 0; i < n; i++) {
    keys[i] = k[ord[i]];
    counts[i] = v[ord[i]];
  }
  return NMG_OK;
}

extern "C" int nmg_sparse_import(nmg_engine* h, const uint64_t* keys, const uint32_t* counts, int64_t n) {
  if (h) h->epoch++;
  // Re-inserts merged (key, count) pairs into an empty table on this rank.
  if (!h || !h->have_table || (n && (!keys || !counts))) return NMG_ERR_INVALID;
  if (!h->d_sparse_keys) return n ? fail(h, NMG_ERR_STATE, "no sparse table") : NMG_OK;
  if ((uint64_t)n > h->sparse_cap) return fail(h, NMG_ERR_CAPACITY, "sparse table too small");
  // the table cleared and the pairs inserted on the device (sparse_add's hash
  // and probing): only the pairs cross PCIe
  HIP_TRY(h, hipSetDevice(h->device));
  int rc = nmg_synchronize(h);
  if (rc) return rc;
  if (!h->d_sparse_ck) HIP_TRY(h, hipMalloc(&h->d_sparse_ck, (h->sparse_cap * 2 + 1) * 8));
  HIP_TRY(h, hipMemsetAsync(h->d_sparse_keys, 0xff, h->sparse_cap * 8, h->stream));
  HIP_TRY(h, hipMemsetAsync(h->d_sparse_vals, 0, h->sparse_cap * 4, h->stream));
  if (n) {
    std::vector<uint64_t> kv(2 * (size_t)n);
    for (int64_t i = 0; i < n; i++) {
      kv[2 * i] = keys[i];
      kv[2 * i + 1] = counts[i];
    }
    HIP_TRY(h, hipMemcpyAsync(h->d_sparse_ck, kv.data(), kv.size() * 8, hipMemcpyHostToDevice, h->stream));
    HIP_TRY(h, launch_sparse_insert(h->stream, h->d_sparse_keys, h->d_sparse_vals, h->sparse_cap, h->d_sparse_ck,
                                    (uint64_t)n));
    HIP_TRY(h, hipStreamSynchronize(h->stream));  // (kv is pageable)
  }
  const uint32_t one = 1;  // imported cells: the next reset must clear the table
  HIP_TRY(h, hipMemcpy(h->d_sparse_dirty + (h->nreset & 1), &one, 4, hipMemcpyHostToDevice));
  return NMG_OK;
}

extern "C" int nmg_set_buffer_counts(nmg_engine* h, uint32_t nb_buffers, const uint32_t* nb_samples,
                                     const uint32_t* nb_found, const uint64_t* buffer_bytes) {
  if (h) h->epoch++;
  if (!h || (nb_buffers && (!nb_samples || !nb_found || !buffer_bytes))) return NMG_ERR_INVALID;
  h->counts_override = true;
  h->ov_samples.assign(nb_samples, nb_samples + nb_buffers);
  h->ov_found.assign(nb_found, nb_found + nb_buffers);
  h->ov_bytes.assign(buffer_bytes, buffer_bytes + nb_buffers);
  return NMG_OK;
}

// ---------------------------------------------------------------------------
// multi-GPU from one host process (nmg_options.nb_gpus > 1)

// RCCL, loaded at run time (only distinct-device engines use it)
struct Rccl {
  void* so = nullptr;
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclReduce) reduce = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};
static Rccl* rccl() {
  static Rccl r;
  static bool tried = false;
  if (!tried) {
    tried = true;
    r.so = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!r.so) r.so = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (r.so) {
      r.init_all = (decltype(r.init_all))dlsym(r.so, "ncclCommInitAll");
      r.destroy = (decltype(r.destroy))dlsym(r.so, "ncclCommDestroy");
      r.reduce = (decltype(r.reduce))dlsym(r.so, "ncclReduce");
      r.group_start = (decltype(r.group_start))dlsym(r.so, "ncclGroupStart");
      r.group_end = (decltype(r.group_end))dlsym(r.so, "ncclGroupEnd");
      r.error_string = (decltype(r.error_string))dlsym(r.so, "ncclGetErrorString");
    }
  }
  return r.so && r.init_all && r.destroy && r.reduce && r.group_start && r.group_end && r.error_string ? &r : nullptr;
}

static int multi_create(nmg_engine* h, const nmg_options* opt) {
  const uint32_t n = std::max<uint32_t>(opt->nb_gpus, 1);  // (1: kDbgMultiRccl, a one-rank communicator)
  for (uint32_t i = 0; i < n; i++) h->devices.push_back(opt->devices ? opt->devices[i] : opt->device + (int)i);
  bool all_same = true, all_distinct = true;
  for (uint32_t i = 0; i < n; i++)
    for (uint32_t j = 0; j < i; j++) {
      if (h->devices[i] != h->devices[j]) all_same = false;
      else all_distinct = false;
    }
  if (!all_same && !all_distinct)
    return fail(h, NMG_ERR_INVALID, "nb_gpus: devices must be all distinct (RCCL) or all one device (testing)");
  for (uint32_t i = 0; i < n; i++) {
    nmg_options o = *opt;
    o.nb_gpus = 0;
    o.devices = nullptr;
    o.flags &= ~kDbgMultiRccl;
    o.device = h->devices[i];
    nmg_engine* w = nullptr;
    const int rc = nmg_create(&w, &o);
    if (rc) return fail(h, rc, "worker engine on device " + std::to_string(h->devices[i]) + ": " + g_create_error);
    h->workers.push_back(w);
  }
  h->warena.assign(n, nullptr);
  h->warena_cap.assign(n, 0);
  h->multi = true;
  h->multi_distinct = all_distinct;
  if (all_distinct) {
    Rccl* r = rccl();
    if (!r) return fail(h, NMG_ERR_HIP, "librccl.so.1 not loadable (multi-GPU merge)");
    std::vector<ncclComm_t> c(n);
    const ncclResult_t e = r->init_all(c.data(), (int)n, h->devices.data());
    if (e != ncclSuccess) return fail(h, NMG_ERR_HIP, std::string("ncclCommInitAll: ") + r->error_string(e));
    for (auto x : c) h->comms.push_back(x);
  }
  return NMG_OK;
}

static void multi_destroy(nmg_engine* h) {
  if (!h->multi) return;
  for (size_t i = 0; i < h->workers.size(); i++) {
    if (h->warena[i]) {
      (void)hipSetDevice(h->workers[i]->device);
      (void)hipFree(h->warena[i]);
    }
  }
  if (Rccl* r = rccl())
    for (void* c : h->comms) r->destroy((ncclComm_t)c);
  for (nmg_engine* w : h->workers) nmg_destroy(w);
  h->workers.clear();
  h->comms.clear();
  h->multi = false;
}

// Shard the submitted buffers (analysis order) into contiguous byte-balanced
// ranges, one per worker: H2D from this handle's pinned staging into the
// worker's arena, analysed there with its global analysis index (seq_base);
// then merge every worker's counters into this handle (sum / min / max):
// RCCL reduces to worker 0 then a device add into this handle (distinct
// devices), or device-side merges (one device).  Per-buffer counts and sparse
// cells are gathered at nmg_synchronize (multi_finish).
static int multi_analyze(nmg_engine* h) {
  Range range("nmg_multi_analyze");
  if (h->multi_pending) {
    const int rc = multi_finish(h);
    if (rc) return rc;
  }
  const uint32_t n = (uint32_t)h->workers.size(), nb = (uint32_t)h->descs.size();
  // the buffers go to the workers once; later steps re-analyse them in place
  const bool stage = !h->multi_staged;
  std::vector<uint64_t> csum(nb + 1, 0);
  for (uint32_t b = 0; b < nb; b++) csum[b + 1] = csum[b] + h->descs[b].len + 64;
  std::vector<uint32_t> cut(n + 1, nb);
  cut[0] = 0;
  for (uint32_t i = 1; i < n; i++)
    cut[i] = std::max(cut[i - 1], (uint32_t)(std::lower_bound(csum.begin(), csum.end(), csum[nb] * i / n) - csum.begin()));
  for (uint32_t i = 0; i < n; i++) {
    nmg_engine* w = h->workers[i];
    const uint32_t a = cut[i], b = cut[i + 1];
    std::vector<uint64_t> offs, lens;
    std::vector<uint32_t> ranks, acc;
    const uint64_t base = a < b ? h->descs[a].offset : 0;
    const uint64_t span = a < b ? h->descs[b - 1].offset + h->descs[b - 1].len - base : 0;
    for (uint32_t k = a; k < b; k++) {
      offs.push_back(h->descs[k].offset - base);
      lens.push_back(h->descs[k].len);
      ranks.push_back(h->descs[k].thread_rank);
      acc.push_back(h->descs[k].access);
    }
    HIP_TRY(h, hipSetDevice(w->device));
    int rc = NMG_OK;
    if (stage) {
      if (span + 64 > h->warena_cap[i]) {
        HIP_TRY(h, hipStreamSynchronize(w->stream));
        (void)hipFree(h->warena[i]);
        h->warena[i] = nullptr;
        h->warena_cap[i] = span + 64;
        HIP_TRY(h, hipMalloc(&h->warena[i], h->warena_cap[i]));
      }
      if (span) HIP_TRY(h, hipMemcpyAsync(h->warena[i], h->h_stage + base, span, hipMemcpyHostToDevice, w->stream));
      rc = nmg_set_device_buffers(w, h->warena[i], offs.data(), lens.data(), ranks.data(), acc.data(), b - a, a);
    }
    if (!rc) rc = nmg_analyze(w);
    if (rc) return fail(h, rc, w->last_error);
  }
  struct Arr {
    int which, op;
  };
  const Arr arrs[4] = {{NMG_ARR_SUM64, 0}, {NMG_ARR_MIN64, 1}, {NMG_ARR_MAX64, 2}, {NMG_ARR_HIST32, 3}};
  // The workers' counters accumulate like this handle's would (they are
  // reset only with it), so the handle's arrays are rebuilt as the merge of
  // the workers' -- no pass of its own over the old values.
  if (h->multi_distinct) {  // one RCCL reduce per array, straight into this handle's array (rank 0), over xGMI
    Rccl* r = rccl();
    HIP_TRY(h, hipSetDevice(h->device));
    r->group_start();
    for (const Arr& x : arrs) {
      size_t hb = 0;
      void* root = array_ptr(h, x.which, &hb);
      for (uint32_t i = 0; i < n; i++) {
        nmg_engine* w = h->workers[i];
        size_t bytes = 0;
        void* p = array_ptr(w, x.which, &bytes);
        if (!bytes) continue;
        const ncclRedOp_t op = x.op == 1 ? ncclMin : (x.op == 2 ? ncclMax : ncclSum);
        const ncclDataType_t dt = x.op == 3 ? ncclUint32 : ncclUint64;
        const size_t count = bytes / (x.op == 3 ? 4 : 8);
        // (recvbuff is read on the root only)
        const ncclResult_t e = r->reduce(p, i == 0 ? root : p, count, dt, op, 0, (ncclComm_t)h->comms[i], w->stream);
        if (e != ncclSuccess) {
          r->group_end();
          return fail(h, NMG_ERR_HIP, std::string("ncclReduce: ") + r->error_string(e));
        }
      }
    }
    const ncclResult_t e = r->group_end();
    if (e != ncclSuccess) return fail(h, NMG_ERR_HIP, std::string("ncclGroupEnd: ") + r->error_string(e));
    // the handle's stream (report downloads) after worker 0's, which carries the root's reduces
    HIP_TRY(h, hipSetDevice(h->device));
    hipEvent_t ev;
    HIP_TRY(h, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HIP_TRY(h, hipEventRecord(ev, h->workers[0]->stream));
    HIP_TRY(h, hipStreamWaitEvent(h->stream, ev, 0));
    (void)hipEventDestroy(ev);
  } else {  // workers on one device (tests): this handle = worker 0, then op= every other worker
    HIP_TRY(h, hipSetDevice(h->device));
    for (uint32_t i = 0; i < n; i++) {
      nmg_engine* w = h->workers[i];
      hipEvent_t ev;
      HIP_TRY(h, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      HIP_TRY(h, hipEventRecord(ev, w->stream));
      HIP_TRY(h, hipStreamWaitEvent(h->stream, ev, 0));
      (void)hipEventDestroy(ev);
      for (const Arr& x : arrs) {
        size_t bytes = 0, wb = 0;
        void* dst = array_ptr(h, x.which, &bytes);
        const void* src = array_ptr(w, x.which, &wb);
        if (!bytes) continue;
        if (i == 0) HIP_TRY(h, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, h->stream));
        else HIP_TRY(h, launch_merge(h->stream, dst, src, bytes / (x.op == 3 ? 4 : 8), x.op));
      }
    }
  }
  h->multi_staged = true;
  h->multi_pending = true;
  h->launched = false;
  return NMG_OK;
}

// after the merges: per-buffer counts (concatenated in analysis order) and
// sparse cells (summed by key) into this handle; the workers are reset so
// that a later nmg_analyze adds only its own samples
static int multi_finish(nmg_engine* h) {
  Range range("nmg_multi_merge");
  h->multi_pending = false;
  for (nmg_engine* w : h->workers) {
    const int rc = nmg_synchronize(w);
    if (rc) return fail(h, rc, w->last_error);
  }
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  // per-buffer SAMPLE counts (concatenated in analysis order), matched-sample
  // totals and sparse cells (summed by key) of the workers, whose counters are
  // cumulative: the per-buffer matched counts are gathered only when asked
  // (engine_download), the report needs their total
  std::vector<uint32_t> ns;
  std::vector<uint64_t> keys;
  std::vector<uint32_t> vals;
  std::vector<uint64_t> k0;
  std::vector<uint32_t> v0;
  uint64_t found = 0;
  int rc = NMG_OK;
  for (nmg_engine* w : h->workers) {
    const uint32_t nb = nmg_get_nb_buffers(w);
    std::vector<uint32_t> a(nb);
    if (nb) {
      HIP_TRY(h, hipSetDevice(w->device));
      HIP_TRY(h, hipMemcpy(a.data(), w->d_bufcnt, nb * 4, hipMemcpyDeviceToHost));
    }
    ns.insert(ns.end(), a.begin(), a.end());
    uint64_t f = 0;
    if (w->d_found) HIP_TRY(h, hipMemcpy(&f, w->d_found, 8, hipMemcpyDeviceToHost));
    found += f;
    rc = sparse_download(w, k0, v0);
    if (rc) return fail(h, rc, w->last_error);
    keys.insert(keys.end(), k0.begin(), k0.end());
    vals.insert(vals.end(), v0.begin(), v0.end());
  }
  HIP_TRY(h, hipSetDevice(h->device));
  if (h->d_sparse_keys) {
    std::vector<size_t> ord(keys.size());
    for (size_t i = 0; i < ord.size(); i++) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return keys[a] < keys[b]; });
    std::vector<uint64_t> mk;
    std::vector<uint32_t> mv;
    for (size_t i : ord) {
      if (!mk.empty() && mk.back() == keys[i]) mv.back() += vals[i];
      else {
        mk.push_back(keys[i]);
        mv.push_back(vals[i]);
      }
    }
    rc = nmg_sparse_import(h, mk.data(), mv.data(), (int64_t)mk.size());
    if (rc) return rc;
  }
  std::vector<uint32_t> nf(ns.size(), 0);
  rc = nmg_set_buffer_counts(h, (uint32_t)ns.size(), ns.data(), nf.data(), h->buf_bytes.data());
  if (rc) return rc;
  h->multi_found = found;
  return NMG_OK;
}

// per-buffer matched counts of a multi-GPU handle: the workers' (cumulative)
static int multi_buffer_found(nmg_engine* h, std::vector<uint32_t>& nf) {
  nf.clear();
  for (nmg_engine* w : h->workers) {
    const uint32_t nb = nmg_get_nb_buffers(w);
    std::vector<uint32_t> a(nb), b(nb);
    const int rc = nmg_get_buffer_counts(w, a.data(), b.data());
    if (rc) return fail(h, rc, w->last_error);
    nf.insert(nf.end(), b.begin(), b.end());
  }
  return NMG_OK;
}

extern "C" int nmg_report(nmg_engine* h, const nmg_object_meta* meta, const nmg_report_options* opts,
                          const char* stdout_path) {
  Range range("nmg_report");
  if (!h || (h->E && !meta)) return NMG_ERR_INVALID;
  if (!h->have_table) return fail(h, NMG_ERR_STATE, "nmg_report before nmg_set_objects");
  const bool timing = getenv("NMG_REPORT_TIMING") != nullptr;  // phase times on stderr
  auto t0 = std::chrono::steady_clock::now();
  HostResults r;
  int rc = engine_download(h, r, true, false);  // (the total only: no found_kernel)
  if (rc) return rc;
  auto t1 = std::chrono::steady_clock::now();
  std::vector<uint32_t> rows;
  int64_t ncells = 0;
  if ((h->flags & NMG_F_PAGE_HIST) && (!opts || opts->dump_single_items)) {
    rc = collect_page_cells(h, &rows, &ncells);
    if (rc) return rc;
  }
  if (timing)
    fprintf(stderr, "nmg_report: counters D2H %.3f s, page cells D2H + rows %.3f s (%" PRId64 " cells)\n",
            std::chrono::duration<double>(t1 - t0).count(),
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count(), ncells);
  nmg_host_results res;
  memset(&res, 0, sizeof(res));
  res.global[0] = r.global[0];
  res.global[1] = r.global[1];
  res.nb_buffers = (uint32_t)r.buf_samples.size();
  res.nb_entries = h->E;
  res.buf_samples = r.buf_samples.data();
  res.buf_found = r.buf_found.data();
  res.buf_bytes = r.buf_bytes.data();
  res.buffer_size = h->buffer_size.data();
  res.first_ordinal = r.first.data();
  res.count_weight = r.count_weight.data();
  res.cells = rows.data();
  res.nb_cells = ncells;
  res.nb_threads = h->T;
  res.match_samples = (h->flags & NMG_F_MATCH_SAMPLES) ? 1 : 0;
  res.objects = h->objects.data();
  // live online tables: entries walked in the order of the latest table that
  // listed them all (ids are creation order there); meta follows that order
  std::vector<uint64_t> w_size, w_first, w_cw;
  std::vector<nmg_object> w_obj;
  std::vector<uint32_t> w_rows;
  if (!h->order.empty()) {
    if (opts && opts->dump_flags) return fail(h, NMG_ERR_STATE, "dump modes need the entries in id order");
    const uint32_t E = h->E;
    if (h->order.size() != E) return fail(h, NMG_ERR_STATE, "report walk order does not cover every entry");
    std::vector<uint32_t> pos(E);
    w_size.resize(E);
    w_first.resize(E);
    w_cw.resize((size_t)E * 4);
    w_obj.resize(E);
    for (uint32_t k = 0; k < E; k++) {
      const uint32_t id = h->order[k];
      pos[id] = k;
      w_size[k] = h->buffer_size[id];
      w_first[k] = r.first[id];
      for (int q = 0; q < 4; q++) w_cw[(size_t)k * 4 + q] = r.count_weight[(size_t)id * 4 + q];
      w_obj[k] = h->objects[id];
    }
    // page rows (entry, thread, page, count), grouped by walk position
    std::vector<uint32_t> idx((size_t)ncells);
    for (uint32_t i = 0; i < (uint32_t)ncells; i++) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return pos[rows[4 * a]] < pos[rows[4 * b]]; });
    w_rows.resize(rows.size());
    for (size_t i = 0; i < idx.size(); i++) {
      const uint32_t* q = &rows[4 * (size_t)idx[i]];
      w_rows[4 * i] = pos[q[0]];
      w_rows[4 * i + 1] = q[1];
      w_rows[4 * i + 2] = q[2];
      w_rows[4 * i + 3] = q[3];
    }
    res.buffer_size = w_size.data();
    res.first_ordinal = w_first.data();
    res.count_weight = w_cw.data();
    res.cells = w_rows.data();
    res.objects = w_obj.data();
  }
  // dump modes: the buffers' bytes (staging, or D2H of device-resident ones)
  // and every SAMPLE record's match
  DumpInput dump;
  std::vector<uint8_t> dev_bytes;
  std::vector<uint32_t> smatch;
  const bool dumps = opts && opts->dump_flags && (h->flags & NMG_F_MATCH_SAMPLES);
  if (dumps) {
    if (!(h->flags & NMG_F_SAMPLE_MATCHES) || !(h->flags & NMG_F_OBJECT_LEVELS))
      return fail(h, NMG_ERR_STATE, "dump modes need an engine created with NMG_F_SAMPLE_MATCHES | NMG_F_OBJECT_LEVELS");
    if (h->streamed || h->counts_override)
      return fail(h, NMG_ERR_STATE, "dump modes need the buffers of one nmg_analyze on this engine");
    uint64_t span = 0;
    for (const BufDesc& d : h->descs) span = std::max<uint64_t>(span, d.offset + d.len);
    smatch.resize(span / 8 + 1);
    if (!h->descs.empty()) {
      HIP_TRY(h, hipMemcpy(smatch.data(), h->d_smatch, smatch.size() * 4, hipMemcpyDeviceToHost));
    }
    const uint8_t* base = h->h_stage;
    if (h->external) {
      dev_bytes.resize(span);
      if (span) HIP_TRY(h, hipMemcpy(dev_bytes.data(), h->d_data, span, hipMemcpyDeviceToHost));
      base = dev_bytes.data();
    }
    for (const BufDesc& d : h->descs)
      dump.buffers.push_back({base + d.offset, d.len, d.thread_rank, d.access, smatch.data() + d.offset / 8});
    dump.entry_addr = h->entry_addr.data();
    dump.levels = r.levels.data();
  }
  std::string err;
  rc = write_report(&res, meta, opts, stdout_path, err, dumps ? &dump : nullptr, &r.nb_found_total);
  if (rc && !err.empty()) h->last_error = err;
  return rc;
}

// Internal (not in include/numamma_gpu.h; bench.py): the first kernel's
// time (route_kernel, or attribute_kernel) and the rest of the attribution
// (the partition-first path's overflow, count, plan, scatter and local
// kernels; the single-pass path's nothing) of up to n recent launches.
extern "C" int nmg_debug_phase_times(nmg_engine* h, float* first_ms, float* rest_ms, int n) {
  if (!h || (n > 0 && (!first_ms || !rest_ms))) return NMG_ERR_INVALID;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  const int avail = (int)std::min<uint64_t>(h->nlaunch, nmg_engine::kRing);
  const int cnt = std::min(n, avail);
  for (int i = 0; i < cnt; i++) {
    const int slot = (int)((h->nlaunch - cnt + i) % nmg_engine::kRing);
    HIP_TRY(h, hipEventElapsedTime(&first_ms[i], h->ring0[slot], h->ringr[slot]));
    HIP_TRY(h, hipEventElapsedTime(&rest_ms[i], h->ringr[slot], h->ringm[slot]));
  }
  return cnt;
}

// Internal (not in include/numamma_gpu.h): analyses (streamed chunks) that
// took the partition-first path so far (tests)
extern "C" int nmg_debug_route_count(nmg_engine* h, uint64_t* n) {
  if (!h || !n) return NMG_ERR_INVALID;
  *n = h->route_launches;
  return NMG_OK;
}

// Internal (not in include/numamma_gpu.h): per-wave phase cycle counts of the
// last launch made with flag 0x1000, [grid][16 waves][8] u64:
// load+check, barrier, process, rest, total, windows.  tools/phase_timing.py.
extern "C" int nmg_debug_timing(nmg_engine* h, uint64_t* out, size_t n, size_t* len) {
  if (!h || !len) return NMG_ERR_INVALID;
  *len = h->dbg_len;
  if (!out || !h->dbg_len) return NMG_OK;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  HIP_TRY(h, hipMemcpy(out, h->d_dbg, std::min(n, h->dbg_len) * 8, hipMemcpyDeviceToHost));
  return NMG_OK;
}
