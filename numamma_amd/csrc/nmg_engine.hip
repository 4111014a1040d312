// nmg_engine.hip -- host side of the MI355X sample-attribution engine, C-ABI
// core (include/numamma_gpu.h): engine lifetime, counter resets, nmg_analyze /
// nmg_synchronize, timers, nmg_report.  The other host translation units are
// listed in nmg_engine_impl.h; the kernels are in nmg_kernels.hip and
// nmg_route.hip (DESIGN.md "Kernels").
#include "nmg_engine_impl.h"

int fail(nmg_engine* h, int code, const std::string& msg) {
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
thread_local std::string g_create_error;

extern "C" int nmg_get_last_error_detail(nmg_engine* h, char* buf, size_t len) {
  if (!buf || !len) return NMG_ERR_INVALID;
  snprintf(buf, len, "%s", h ? h->last_error.c_str() : g_create_error.c_str());
  return NMG_OK;
}

void free_counters(nmg_engine* h) {
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
void free_lookup(nmg_engine* h) {
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
void free_route_table(nmg_engine* h) {
  (void)hipFree(h->d_parts);
  (void)hipFree(h->d_pbounds);
  (void)hipFree(h->d_pdir);
  (void)hipFree(h->d_pdead);
  (void)hipFree(h->d_pe_keys);
  (void)hipFree(h->d_pe_nodes);
  (void)hipFree(h->d_pe_info);
  (void)hipFree(h->d_pe_pnode);
  (void)hipFree(h->d_pe_old);
  (void)hipFree(h->d_pe_oinf);
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
  h->d_pdead = nullptr;
  h->d_pe_keys = nullptr;
  h->d_pe_nodes = nullptr;
  h->d_pe_info = nullptr;
  h->d_pe_pnode = nullptr;
  h->d_pe_old = nullptr;
  h->d_pe_oinf = nullptr;
  h->route_ok = false;
  h->nparts = 0;
}

// the per-analysis buffers of the partition-first path
void free_route_pool(nmg_engine* h) {
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


LookupSet take_lookup(nmg_engine* h) {
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

void put_lookup(nmg_engine* h, const LookupSet& l) {
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

void free_table(nmg_engine* h) {
  free_route_table(h);
  free_lookup(h);
  (void)hipFree(h->d_entries);
  h->d_entries = nullptr;
}

hipError_t alloc_copy(nmg_engine* h, void** dptr, const void* src, size_t bytes) {
  hipError_t e = hipMalloc(dptr, bytes ? bytes : 16);
  if (e != hipSuccess) return e;
  if (bytes) return hipMemcpyAsync(*dptr, src, bytes, hipMemcpyHostToDevice, h->stream);
  return hipSuccess;
}

// keys strictly ascending, every key with >= 1 entry, entry_off a prefix array over n entries
int check_table(nmg_engine* h, const uint64_t* keys, const uint32_t* entry_off, uint32_t nb_keys,
                       uint32_t n) {
  if (entry_off && (entry_off[0] != 0 || entry_off[nb_keys] != n))
    return fail(h, NMG_ERR_INVALID, "entry_off[0] must be 0 and entry_off[nb_keys] == the number of entries");
  for (uint32_t i = 0; i < nb_keys; i++) {
    if (entry_off[i + 1] <= entry_off[i]) return fail(h, NMG_ERR_INVALID, "every key needs >= 1 entry");
    if (i && keys[i] <= keys[i - 1]) return fail(h, NMG_ERR_INVALID, "keys must be strictly ascending");
  }
  return NMG_OK;
}


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
  if (h->up_recorded) (void)hipEventSynchronize(h->up_ev);
  if (h->up_ev) (void)hipEventDestroy(h->up_ev);
  (void)hipHostFree(h->up_pin);
  for (void* q : {(void*)h->cprep.d_base, (void*)h->cprep.d_off, (void*)h->cprep.d_part, (void*)h->cprep.d_np,
                  (void*)h->cprep.d_cnt, (void*)h->cprep.d_sent, (void*)h->cprep.d_soff})
    (void)hipFree(q);
  snap_free(h);
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
  } else if (h->counts_override) {  // a job's counts (nmg_set_buffer_counts): back to this engine's buffers
    h->counts_override = false;
    h->ov_samples.clear();
    h->ov_found.clear();
    h->ov_bytes.clear();
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
  h->counters_fresh = true;
  return NMG_OK;
}


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

int decode_error_word(nmg_engine* h, uint64_t w) {
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

extern "C" int nmg_get_merge_stats(nmg_engine* h, float* merge_ms, uint64_t* payload_bytes) {
  if (!h || !merge_ms || !payload_bytes) return NMG_ERR_INVALID;
  *merge_ms = 0.f;
  *payload_bytes = 0;
  if (!h->multi || !h->merge_timed) return NMG_OK;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipEventSynchronize(h->merge_ev1));
  HIP_TRY(h, hipEventElapsedTime(merge_ms, h->merge_ev0, h->merge_ev1));
  *payload_bytes = h->merge_bytes;
  return NMG_OK;
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
