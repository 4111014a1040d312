// nmg_results.hip -- result getters (global and per-object counters, page
// cells), the merge arrays of the multi-GPU chain (export / import, packed page
// histogram, sparse cells, per-buffer counts).
#include "nmg_engine_impl.h"

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


// Every non-zero (entry, thread, page) cell, entries in id order, each
// entry's cells in (thread, page) order.  Dense cells are counted and
// compacted into rows on the device (cells_count / cells_emit); the rows stay
// there (d_cells_rows) until copied out, so only they cross PCIe, once.  The
// sparse table's cells (entries past the dense budget, e.g. [stack]) are
// grouped on the host and placed at their entries' offsets.  Cached per
// results epoch: nmg_count_page_cells then nmg_get_page_cells does the work
// once.
int cells_prepare(nmg_engine* h) {
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
int cells_fill(nmg_engine* h, uint32_t* rows) {
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
int collect_page_cells(nmg_engine* h, std::vector<uint32_t>* rows, int64_t* count) {
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

void* array_ptr(nmg_engine* h, int which, size_t* bytes) {
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
  if (h) h->counters_fresh = false;
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

int scratch_u64(nmg_engine* h) {
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
  if (h) h->counters_fresh = false;
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

extern "C" int nmg_objcw_pack(nmg_engine* h, const void* d_sum64, uint64_t threshold, void* d_u32, void* d_ovf,
                              uint64_t ovf_cap, uint64_t* n_ovf) {
  Range range("nmg_objcw_pack");
  if (!h || !h->have_table || !n_ovf || !threshold) return NMG_ERR_INVALID;
  const uint64_t n = 4ull * h->E;
  *n_ovf = 0;
  if (!n) return NMG_OK;
  if (!d_sum64 || !d_u32 || (ovf_cap && !d_ovf)) return NMG_ERR_INVALID;
  int rc = scratch_u64(h);
  if (rc) return rc;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipMemsetAsync(h->d_scratch, 0, 8, h->stream));
  const uint64_t* rows = reinterpret_cast<const uint64_t*>(d_sum64) + objcw_index(0, 0, 0, h->E);
  HIP_TRY(h, launch_objcw_pack(h->stream, rows, n, threshold, d_u32, d_ovf, ovf_cap,
                               reinterpret_cast<unsigned long long*>(h->d_scratch)));
  HIP_TRY(h, hipMemcpyAsync(n_ovf, h->d_scratch, 8, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  return NMG_OK;
}

extern "C" int nmg_objcw_unpack(nmg_engine* h, void* d_sum64, const void* d_u32, const void* d_ovf, uint64_t n_ovf) {
  Range range("nmg_objcw_unpack");
  if (!h || !h->have_table || (n_ovf && !d_ovf)) return NMG_ERR_INVALID;
  const uint64_t n = 4ull * h->E;
  if (!n) return NMG_OK;
  if (!d_sum64 || !d_u32) return NMG_ERR_INVALID;
  int rc = scratch_u64(h);
  if (rc) return rc;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipMemsetAsync(h->d_scratch + 1, 0, 8, h->stream));
  uint64_t* rows = reinterpret_cast<uint64_t*>(d_sum64) + objcw_index(0, 0, 0, h->E);
  HIP_TRY(h, launch_objcw_unpack(h->stream, rows, n, d_u32, d_ovf, n_ovf,
                                 reinterpret_cast<unsigned long long*>(h->d_scratch + 1)));
  uint64_t bad = 0;
  HIP_TRY(h, hipMemcpyAsync(&bad, h->d_scratch + 1, 8, hipMemcpyDeviceToHost, h->stream));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  if (bad) return fail(h, NMG_ERR_RANGE, "nmg_objcw_unpack: overflow entries outside the rows");
  return NMG_OK;
}

// The sparse cells can be non-empty only when something was inserted (or
// imported) since the last reset: that reset cleared the table if it had been
// written, and the flag of the analyses after it is d_sparse_dirty[nreset & 1]
// (reset_kernel).  A 4-byte read instead of the whole table.
int sparse_nonempty(nmg_engine* h, bool* out) {
  *out = false;
  if (!h->d_sparse_keys) return NMG_OK;
  uint32_t dirty = 1;
  HIP_TRY(h, hipMemcpy(&dirty, h->d_sparse_dirty + (h->nreset & 1), 4, hipMemcpyDeviceToHost));
  *out = dirty != 0;
  return NMG_OK;
}

int sparse_download(nmg_engine* h, std::vector<uint64_t>& k, std::vector<uint32_t>& v) {
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
