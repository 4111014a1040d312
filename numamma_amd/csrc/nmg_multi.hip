// nmg_multi.hip -- one host process over several GPUs (nmg_options.nb_gpus;
// SURVEY.md 8(e)): worker engines, byte-balanced shards, RCCL group reduce
// over xGMI or the device merge kernel for workers sharing a device.
#include "nmg_engine_impl.h"

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

int multi_create(nmg_engine* h, const nmg_options* opt) {
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

void multi_destroy(nmg_engine* h) {
  if (!h->multi) return;
  for (size_t i = 0; i < h->workers.size(); i++) {
    if (h->warena[i]) {
      (void)hipSetDevice(h->workers[i]->device);
      (void)hipFree(h->warena[i]);
    }
  }
  if (Rccl* r = rccl())
    for (void* c : h->comms) r->destroy((ncclComm_t)c);
  (void)hipSetDevice(h->device);
  if (h->merge_ev0) (void)hipEventDestroy(h->merge_ev0);
  if (h->merge_ev1) (void)hipEventDestroy(h->merge_ev1);
  h->merge_ev0 = h->merge_ev1 = nullptr;
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
int multi_analyze(nmg_engine* h) {
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
  // merge timing (nmg_get_merge_stats): worker 0 shares this handle's device
  HIP_TRY(h, hipSetDevice(h->device));
  if (!h->merge_ev0) {
    HIP_TRY(h, hipEventCreate(&h->merge_ev0));
    HIP_TRY(h, hipEventCreate(&h->merge_ev1));
  }
  hipStream_t mst = h->multi_distinct ? h->workers[0]->stream : h->stream;
  if (!h->multi_distinct) {  // (the device merges run on this handle's stream after worker 0's analysis)
    hipEvent_t ev;
    HIP_TRY(h, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HIP_TRY(h, hipEventRecord(ev, h->workers[0]->stream));
    HIP_TRY(h, hipStreamWaitEvent(h->stream, ev, 0));
    (void)hipEventDestroy(ev);
  }
  HIP_TRY(h, hipEventRecord(h->merge_ev0, mst));
  h->merge_bytes = 0;
  for (const Arr& x : arrs) {
    size_t bytes = 0;
    (void)array_ptr(h->workers[0], x.which, &bytes);
    h->merge_bytes += bytes;
  }
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
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipEventRecord(h->merge_ev1, mst));
  h->merge_timed = true;
  h->multi_staged = true;
  h->multi_pending = true;
  h->launched = false;
  return NMG_OK;
}

// after the merges: per-buffer counts (concatenated in analysis order) and
// sparse cells (summed by key) into this handle; the workers are reset so
// that a later nmg_analyze adds only its own samples
int multi_finish(nmg_engine* h) {
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
int multi_buffer_found(nmg_engine* h, std::vector<uint32_t>& nf) {
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
