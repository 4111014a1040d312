// nmg_engine_impl.h -- the host engine's internals, shared by its translation
// units (not part of the C-ABI):
//   nmg_engine.hip      C-ABI core: create / destroy / reset, analyze / synchronize,
//                       timers, nmg_report, debug getters
//   nmg_table.hip       object tables: upload, lookup structures, partitions,
//                       nmg_set_objects / nmg_update_objects (online growth)
//   nmg_submit.hip      buffer submission, zero-copy registration, the streaming
//                       pipeline, schedules and the single-pass launch
//   nmg_route_host.hip  the partition-first path's host side (pools, launches)
//   nmg_results.hip     result getters, page cells, merge arrays, sparse cells
//   nmg_multi.hip       multi-GPU handles (RCCL group reduce / device merge)
#pragma once

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
  // the counter arrays hold what the last reset wrote (no analysis, import or
  // table update since): the local pass may store instead of adding
  bool counters_fresh = false;
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
  // results snapshot (nmg_results_begin / nmg_results_end, nmg_results.hip)
  struct ResSnap {
    hipStream_t stream = nullptr;
    hipEvent_t ready = nullptr, copied = nullptr;
    bool pending = false;
    bool meta_dirty = true;            // hist_base / npages / sparse entries changed: re-upload
    uint64_t E = 0, nb = 0, nsent = 0, rows_dev = 0, rows_host = 0, sparse_cap = 0;
    uint64_t *d_base = nullptr, *d_off = nullptr, *d_part = nullptr, *d_soff = nullptr;
    uint32_t *d_np = nullptr, *d_cnt = nullptr, *d_sent = nullptr;
    uint64_t *d_sum = nullptr, *d_min = nullptr, *d_max = nullptr, *d_objcw = nullptr, *d_found = nullptr;
    uint32_t* d_bufcnt = nullptr;
    uint64_t* d_ck = nullptr;          // the sparse table's used slots, compacted (+ their count)
    void* d_rows = nullptr;            // uint4 rows
    // pinned host copies
    uint64_t *h_sum = nullptr, *h_min = nullptr, *h_max = nullptr, *h_objcw = nullptr, *h_small = nullptr,
             *h_soff = nullptr;        // h_small: [0] matched total, [1] rows, [2] sparse cells
    uint32_t* h_bufcnt = nullptr;
    uint32_t* h_rows = nullptr;        // mapped: copy_rows_kernel writes it
    uint64_t h_cap_E = 0, h_cap_nb = 0, h_cap_sent = 0;
    std::vector<uint32_t> sent_entry;  // begin-time table: sparse idx -> entry (~0: no longer sparse)
  } snap;
  uint64_t snap_nb = 0;  // buffers of the snapshot in flight
  // the synchronous page-cell getters' device buffers (cells_prepare), kept across calls
  struct CellsPrep {
    uint64_t E = 0, nsent = 0;
    bool meta_dirty = true;
    uint64_t *d_base = nullptr, *d_off = nullptr, *d_part = nullptr, *d_soff = nullptr;
    uint32_t *d_np = nullptr, *d_cnt = nullptr, *d_sent = nullptr;
  } cprep;
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
  size_t sdescs_cap = 0, ranges_cap = 0;
  // pinned staging of an analysis' small uploads (descriptors, schedule,
  // chunk pools): copied on the engine stream without a host wait
  uint8_t* up_pin = nullptr;
  size_t up_cap = 0, up_off = 0;
  hipEvent_t up_ev = nullptr;
  bool up_recorded = false;
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
  // the merge of the last multi_analyze, timed on the root device's stream that
  // carries it (worker 0's for RCCL, this handle's for device merges): from
  // the end of worker 0's analysis to the end of the merges (nmg_get_merge_stats)
  hipEvent_t merge_ev0 = nullptr, merge_ev1 = nullptr;
  bool merge_timed = false;
  uint64_t merge_bytes = 0;  // counter bytes each worker contributes per merge
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
  uint32_t* d_pdead = nullptr;    // [(kMaxParts + 1) / 32] partitions no sample with ts != 0 can match
  RSeg rsegs[kRouteSegs];         // its segments
  uint64_t route_tbase = 0;       // compact records: timestamps relative to this (XLayout)
  uint32_t nrsegs = 0;
  uint64_t* d_pe_keys = nullptr;  // [nparts][kPartSlots]
  uint4* d_pe_nodes = nullptr;    // [nparts][kPartSlots][2]
  uint4* d_pe_pnode = nullptr;    // [nparts][kPartSlots] packed node records (PackedNode)
  uint4* d_pe_old = nullptr;      // [nparts][kOldLds] older entries, packed
  uint32_t* d_pe_oinf = nullptr;  // [nparts][kOldLds]
  uint2* d_pe_info = nullptr;     // [nparts][kPartSlots]
  uint4* d_pe_dir = nullptr;      // [nparts][kPartDir] (PartDir)
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

// a host copy into pinned staging, run by one of the copy threads
struct CopyTask {
  uint8_t* dst;
  const uint8_t* src;
  uint64_t len;
};

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

// engine-internal functions (hidden: not exported from the library)
#pragma GCC visibility push(hidden)
extern thread_local std::string g_create_error;  // detail of the last failed nmg_create (no handle holds it)
int fail(nmg_engine* h, int code, const std::string& msg);
void free_counters(nmg_engine* h);
void free_lookup(nmg_engine* h);
void free_route_table(nmg_engine* h);
void snap_free(nmg_engine* h);  // the results snapshot's buffers and stream
// an H2D copy of n bytes from host memory the caller may reuse at once:
// through the pinned staging, on the engine stream, no host wait
int stage_h2d(nmg_engine* h, void* d_dst, const void* src, size_t n);
void stage_reset(nmg_engine* h);  // (an analysis' first upload: the staging from its start again)
void free_route_pool(nmg_engine* h);
LookupSet take_lookup(nmg_engine* h);
void put_lookup(nmg_engine* h, const LookupSet& l);
void free_table(nmg_engine* h);
hipError_t alloc_copy(nmg_engine* h, void** dptr, const void* src, size_t bytes);
int check_table(nmg_engine* h, const uint64_t* keys, const uint32_t* entry_off, uint32_t nb_keys,
                       uint32_t n);
int build_lookup(nmg_engine* h, const uint64_t* keys, const uint32_t* entry_off, uint32_t nb_keys,
                        const std::vector<DevEntry>& chain, DevEntry* chain_dev);
void route_segments(const uint64_t* b, uint32_t P, RSeg* seg, uint32_t* nseg, std::vector<uint16_t>& dir);
int build_partitions(nmg_engine* h, const uint64_t* keys, const uint32_t* entry_off, uint32_t K,
                            const std::vector<DevEntry>& dev, const uint32_t* ids);
int grow_entries(nmg_engine* h, uint32_t newE, const uint32_t* ids, const nmg_object* objs, uint32_t n);
int stage_reserve(nmg_engine* h, size_t need);
int append_desc(nmg_engine* h, uint64_t len, uint32_t thread_rank, uint32_t access);
uint64_t zero_copy_dev(nmg_engine* h, const void* p, uint64_t len);
int append_desc_zc(nmg_engine* h, uint64_t dev, uint64_t len, uint32_t thread_rank, uint32_t access);
int check_buffer_args(nmg_engine* h, uint64_t len, uint32_t thread_rank, uint32_t access);
void run_copies(nmg_engine* h, const std::vector<CopyTask>& tasks);
int slot_acquire(nmg_engine* h, int s);
int ensure_bufcnt(nmg_engine* h, size_t need);
int stream_flush(nmg_engine* h);
int stream_dst(nmg_engine* h, uint64_t len, uint8_t** dst, std::vector<CopyTask>* pending);
int stream_append(nmg_engine* h, uint64_t len, uint32_t thread_rank, uint32_t access);
int upload_buffers(nmg_engine* h);
void make_schedule(const std::vector<BufDesc>& descs, uint32_t grid, uint32_t index_base, BufDesc* sorted,
                          uint32_t* ranges, bool by_stream);
int build_schedule(nmg_engine* h, uint32_t grid, bool by_stream = true);
void ensure_occupancy(nmg_engine* h);
uint32_t attribution_grid(nmg_engine* h, uint32_t nb);
Params base_params(nmg_engine* h, const uint8_t* data, const BufDesc* sdescs, const uint32_t* ranges);
int launch_events(nmg_engine* h, int* slot_out);
int launch_attribution(nmg_engine* h, const uint8_t* data, const BufDesc* sdescs, const uint32_t* ranges,
                              uint32_t nb, uint32_t grid, uint64_t nbytes);
uint32_t bits_for(uint64_t v);
bool route_layout(nmg_engine* h, const std::vector<BufDesc>& descs, XLayout& xl);
bool route_eligible(nmg_engine* h, const std::vector<BufDesc>& descs);
bool route_eligible(nmg_engine* h);
int route_pool(nmg_engine* h, const std::vector<BufDesc>& descs, uint32_t grid, const uint32_t* ranges,
                      std::vector<uint32_t>& c0);
int route_prepare(nmg_engine* h, uint32_t grid, const std::vector<uint32_t>& ranges);
int route_analyze(nmg_engine* h, uint32_t nb, uint32_t grid);
int route_analyze_job(nmg_engine* h, const RouteJob& job);
int route_settle(nmg_engine* h);
int decode_error_word(nmg_engine* h, uint64_t w);
int cells_prepare(nmg_engine* h);
int cells_fill(nmg_engine* h, uint32_t* rows);
int collect_page_cells(nmg_engine* h, std::vector<uint32_t>* rows, int64_t* count);
void* array_ptr(nmg_engine* h, int which, size_t* bytes);
int scratch_u64(nmg_engine* h);
int sparse_nonempty(nmg_engine* h, bool* out);
int sparse_download(nmg_engine* h, std::vector<uint64_t>& k, std::vector<uint32_t>& v);
int multi_create(nmg_engine* h, const nmg_options* opt);
void multi_destroy(nmg_engine* h);
int multi_analyze(nmg_engine* h);
int multi_finish(nmg_engine* h);
int multi_buffer_found(nmg_engine* h, std::vector<uint32_t>& nf);
#pragma GCC visibility pop
