// nmg_results.hip -- result getters (global and per-object counters, page
// cells), the merge arrays of the multi-GPU chain (export / import, packed page
// histogram, sparse cells, per-buffer counts).
#include <chrono>
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
// entry's cells in (thread, page) order.  On the device, in buffers kept
// across calls (the table's cell layout uploaded once per table): dense cells
// counted per entry (cells_count), the sparse table's cells (entries past the
// dense budget, e.g. [stack]) counted per entry from its compacted slots, an
// exclusive scan into row offsets, the dense rows emitted (cells_emit).  The
// rows stay on the device (d_cells_rows) until copied out, so only they cross
// PCIe, once; the sparse rows are sorted on the host and placed at their
// entries' offsets.  Cached per results epoch: nmg_count_page_cells then
// nmg_get_page_cells does the work once.
int cells_prepare(nmg_engine* h) {
  if (h->cells_epoch == h->epoch) return NMG_OK;
  const bool timing = getenv("NMG_CELLS_TIMING") != nullptr;  // (phase times on stderr)
  auto tp = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!timing) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "cells_prepare: %-10s %.3f ms\n", what, std::chrono::duration<double, std::milli>(now - tp).count());
    tp = now;
  };
  int rc = nmg_synchronize(h);
  if (rc) return rc;
  lap("sync");
  const uint64_t E = h->E, nsent = h->sparse_entries.size();
  auto& C = h->cprep;
  if (E != C.E || !C.d_off || nsent > C.nsent) {  // (grown only with the table)
    for (void* q : {(void*)C.d_base, (void*)C.d_off, (void*)C.d_part, (void*)C.d_np, (void*)C.d_cnt,
                    (void*)C.d_sent, (void*)C.d_soff})
      (void)hipFree(q);
    C = nmg_engine::CellsPrep();
    HIP_TRY(h, hipMalloc(&C.d_base, (E + 1) * 8));
    HIP_TRY(h, hipMalloc(&C.d_off, (E + 1) * 8));
    HIP_TRY(h, hipMalloc(&C.d_part, (scan_parts(E) + 1) * 8));
    HIP_TRY(h, hipMalloc(&C.d_np, (E + 1) * 4));
    HIP_TRY(h, hipMalloc(&C.d_cnt, (E + 1) * 4));
    HIP_TRY(h, hipMalloc(&C.d_sent, (nsent + 1) * 4));
    HIP_TRY(h, hipMalloc(&C.d_soff, (nsent + 1) * 8));
    C.E = E;
    C.nsent = nsent;
    C.meta_dirty = true;
  }
  if (C.meta_dirty) {  // (the table's cell layout)
    std::vector<uint32_t> np(E);
    for (uint64_t e = 0; e < E; e++) np[e] = h->hist_base[e] == kHistSparse ? 0u : (uint32_t)h->npages[e];
    if (E) {
      HIP_TRY(h, hipMemcpy(C.d_base, h->hist_base.data(), E * 8, hipMemcpyHostToDevice));
      HIP_TRY(h, hipMemcpy(C.d_np, np.data(), E * 4, hipMemcpyHostToDevice));
    }
    if (nsent) HIP_TRY(h, hipMemcpy(C.d_sent, h->sparse_entries.data(), nsent * 4, hipMemcpyHostToDevice));
    C.meta_dirty = false;
  }
  lap("meta");
  // sparse cells: compacted on the device (sparse_download, which leaves
  // them in d_sparse_ck) and grouped per entry here
  std::vector<uint64_t> k;
  std::vector<uint32_t> v;
  rc = sparse_download(h, k, v);
  if (rc) return rc;
  std::vector<std::vector<std::pair<uint64_t, uint32_t>>> sparse(nsent);
  for (size_t i = 0; i < k.size(); i++) {
    const uint32_t s = sparse_key_idx(k[i]);
    if (k[i] == ~0ull || !v[i] || s >= nsent || h->hist_base[h->sparse_entries[s]] != kHistSparse) continue;
    // order within an entry: (thread, page)
    sparse[s].push_back({(uint64_t(sparse_key_thread(k[i])) << 32) | sparse_key_page(k[i]), v[i]});
  }
  for (auto& l : sparse) std::sort(l.begin(), l.end());
  lap("sparse");
  const bool dense = h->hist_cells && E;
  uint64_t n = 0;
  std::vector<uint64_t> soff(nsent, 0);
  if (E) {
    hipStream_t st = h->stream;
    if (dense)
      HIP_TRY(h, launch_cells_count(st, h->d_hist, h->hist_cells, h->T, C.d_base, C.d_np, (uint32_t)E, C.d_cnt));
    else
      HIP_TRY(h, hipMemsetAsync(C.d_cnt, 0, E * 4, st));
    if (!k.empty())
      HIP_TRY(h, launch_cells_sparse_count(st, h->d_sparse_ck,
                                           reinterpret_cast<const unsigned long long*>(h->d_sparse_ck + 2 * h->sparse_cap),
                                           h->sparse_cap, C.d_sent, (uint32_t)nsent, C.d_base, C.d_cnt));
    HIP_TRY(h, launch_scan_u32(st, C.d_cnt, E, C.d_off, C.d_part));
    HIP_TRY(h, hipMemcpyAsync(&n, C.d_off + E, 8, hipMemcpyDeviceToHost, st));
    if (!k.empty()) {
      HIP_TRY(h, launch_gather_off(st, C.d_off, C.d_sent, (uint32_t)nsent, C.d_soff));
      HIP_TRY(h, hipMemcpyAsync(soff.data(), C.d_soff, nsent * 8, hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(h, hipStreamSynchronize(st));
    lap("count");
    if (dense && n) {
      if (n > h->cells_rows_cap) {
        (void)hipFree(h->d_cells_rows);
        h->d_cells_rows = nullptr;
        h->cells_rows_cap = 0;
        HIP_TRY(h, hipMalloc(&h->d_cells_rows, n * 16));
        h->cells_rows_cap = n;
      }
      HIP_TRY(h, launch_cells_emit(st, h->d_hist, h->hist_cells, h->T, C.d_base, C.d_np, (uint32_t)E, C.d_off,
                                   (uint4*)h->d_cells_rows));
      HIP_TRY(h, hipStreamSynchronize(st));
    }
    lap("emit");
  }
  h->cells_sparse.clear();
  for (uint64_t s = 0; s < nsent; s++)
    if (!sparse[s].empty()) h->cells_sparse.push_back({soff[s], h->sparse_entries[s], std::move(sparse[s])});
  if (timing) fprintf(stderr, "cells_prepare: %llu rows\n", (unsigned long long)n);
  h->cells_n = (int64_t)n;
  h->cells_epoch = h->epoch;
  return NMG_OK;
}

// the prepared rows into rows[cells_n * 4]: dense rows D2H, sparse rows placed
int cells_fill(nmg_engine* h, uint32_t* rows) {
  const bool dense = h->hist_cells && h->E;
  const auto t0 = std::chrono::steady_clock::now();
  if (dense && h->cells_n)
    HIP_TRY(h, hipMemcpy(rows, h->d_cells_rows, (size_t)h->cells_n * 16, hipMemcpyDeviceToHost));
  if (getenv("NMG_CELLS_TIMING"))
    fprintf(stderr, "cells_fill: rows D2H %.3f ms\n",
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
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

// ---- results snapshot (include/numamma_gpu.h: nmg_results_begin / end)

namespace nmg {
// device and pinned buffers of the snapshot, (re)allocated when the table or
// the buffer list outgrows them
static int snap_alloc(nmg_engine* h) {
  auto& S = h->snap;
  const uint64_t E = h->E, nb = h->descs.size(), nsent = h->sparse_entries.size();
  const uint64_t rows = h->hist_cells * h->T + (h->d_sparse_keys ? h->sparse_cap : 0);
  if (!S.stream) {
    HIP_TRY(h, hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking));
    HIP_TRY(h, hipEventCreateWithFlags(&S.ready, hipEventDisableTiming));
    HIP_TRY(h, hipEventCreateWithFlags(&S.copied, hipEventDisableTiming));
  }
  if (E != S.E || !S.d_min) {
    for (void* q : {(void*)S.d_base, (void*)S.d_off, (void*)S.d_np, (void*)S.d_cnt, (void*)S.d_min, (void*)S.d_objcw,
                    (void*)S.d_part})
      (void)hipFree(q);
    S.d_base = S.d_off = S.d_part = S.d_min = S.d_objcw = nullptr;
    S.d_np = S.d_cnt = nullptr;
    HIP_TRY(h, hipMalloc(&S.d_base, (E + 1) * 8));
    HIP_TRY(h, hipMalloc(&S.d_off, (E + 1) * 8));
    HIP_TRY(h, hipMalloc(&S.d_part, (scan_parts(E) + 1) * 8));
    HIP_TRY(h, hipMalloc(&S.d_np, (E + 1) * 4));
    HIP_TRY(h, hipMalloc(&S.d_cnt, (E + 1) * 4));
    HIP_TRY(h, hipMalloc(&S.d_min, (36 + E + 1) * 8));
    HIP_TRY(h, hipMalloc(&S.d_objcw, (E + 1) * 32));
    S.E = E;
    S.meta_dirty = true;
  }
  if (!S.d_sum) {
    HIP_TRY(h, hipMalloc(&S.d_sum, 2 * kGlobalSums * 8));
    HIP_TRY(h, hipMalloc(&S.d_max, 36 * 8));
    HIP_TRY(h, hipMalloc(&S.d_found, 8));
    HIP_TRY(h, hipHostMalloc((void**)&S.h_sum, 2 * kGlobalSums * 8, 0));
    HIP_TRY(h, hipHostMalloc((void**)&S.h_max, 36 * 8, 0));
    HIP_TRY(h, hipHostMalloc((void**)&S.h_small, 4 * 8, 0));
  }
  if (nb > S.nb || !S.d_bufcnt) {
    (void)hipFree(S.d_bufcnt);
    S.d_bufcnt = nullptr;
    HIP_TRY(h, hipMalloc(&S.d_bufcnt, (2 * nb + 1) * 4));
    S.nb = nb;
  }
  if (nsent > S.nsent || !S.d_sent) {
    (void)hipFree(S.d_sent);
    (void)hipFree(S.d_soff);
    S.d_sent = nullptr;
    S.d_soff = nullptr;
    HIP_TRY(h, hipMalloc(&S.d_sent, (nsent + 1) * 4));
    HIP_TRY(h, hipMalloc(&S.d_soff, (nsent + 1) * 8));
    S.nsent = nsent;
    S.meta_dirty = true;
  }
  if (rows > S.rows_dev || !S.d_rows) {
    (void)hipFree(S.d_rows);
    S.d_rows = nullptr;
    HIP_TRY(h, hipMalloc(&S.d_rows, (rows + 1) * 16));
    S.rows_dev = rows;
  }
  if (h->d_sparse_keys && (S.sparse_cap != h->sparse_cap || !S.d_ck)) {
    (void)hipFree(S.d_ck);
    S.d_ck = nullptr;
    HIP_TRY(h, hipMalloc(&S.d_ck, (2 * h->sparse_cap + 1) * 8));
    S.sparse_cap = h->sparse_cap;
  }
  // pinned host copies (the rows grow on demand in nmg_results_end)
  if (E > S.h_cap_E || !S.h_min) {
    (void)hipHostFree(S.h_min);
    (void)hipHostFree(S.h_objcw);
    S.h_min = S.h_objcw = nullptr;
    HIP_TRY(h, hipHostMalloc((void**)&S.h_min, (36 + E + 1) * 8, 0));
    HIP_TRY(h, hipHostMalloc((void**)&S.h_objcw, (E + 1) * 32, 0));
    S.h_cap_E = E;
  }
  if (nb > S.h_cap_nb || !S.h_bufcnt) {
    (void)hipHostFree(S.h_bufcnt);
    S.h_bufcnt = nullptr;
    HIP_TRY(h, hipHostMalloc((void**)&S.h_bufcnt, (2 * nb + 1) * 4, 0));
    S.h_cap_nb = nb;
  }
  if (nsent > S.h_cap_sent || !S.h_soff) {
    (void)hipHostFree(S.h_soff);
    S.h_soff = nullptr;
    HIP_TRY(h, hipHostMalloc((void**)&S.h_soff, (nsent + 1) * 8, 0));
    S.h_cap_sent = nsent;
  }
  return NMG_OK;
}

}  // namespace nmg

void snap_free(nmg_engine* h) {
  auto& S = h->snap;
  if (S.stream) (void)hipStreamSynchronize(S.stream);
  for (void* q : {(void*)S.d_base, (void*)S.d_off, (void*)S.d_part, (void*)S.d_soff, (void*)S.d_np, (void*)S.d_cnt,
                  (void*)S.d_sent, (void*)S.d_sum, (void*)S.d_min, (void*)S.d_max, (void*)S.d_objcw, (void*)S.d_found,
                  (void*)S.d_bufcnt, (void*)S.d_ck, S.d_rows})
    (void)hipFree(q);
  for (void* q : {(void*)S.h_sum, (void*)S.h_min, (void*)S.h_max, (void*)S.h_objcw, (void*)S.h_small, (void*)S.h_soff,
                  (void*)S.h_bufcnt, (void*)S.h_rows})
    (void)hipHostFree(q);
  if (S.ready) (void)hipEventDestroy(S.ready);
  if (S.copied) (void)hipEventDestroy(S.copied);
  if (S.stream) (void)hipStreamDestroy(S.stream);
  S = nmg_engine::ResSnap();
}

extern "C" int nmg_results_begin(nmg_engine* h) {
  Range range("nmg_results_begin");
  if (!h) return NMG_ERR_INVALID;
  if (!h->have_table) return fail(h, NMG_ERR_STATE, "nmg_results_begin before nmg_set_objects");
  if (h->multi || h->counts_override)
    return fail(h, NMG_ERR_STATE, "nmg_results_begin: a multi-GPU handle or merged per-buffer counts");
  if (h->streaming) return fail(h, NMG_ERR_STATE, "nmg_results_begin while streaming");
  auto& S = h->snap;
  HIP_TRY(h, hipSetDevice(h->device));
  if (S.pending) {  // (a snapshot nobody ended: its copy must finish before the buffers are reused)
    HIP_TRY(h, hipStreamSynchronize(S.stream));
    S.pending = false;
  }
  int rc = route_settle(h);  // (the per-buffer matched counts of the last route analysis, enqueued)
  if (rc) return rc;
  rc = snap_alloc(h);
  if (rc) return rc;
  const uint64_t E = h->E, nb = h->descs.size(), nsent = h->sparse_entries.size();
  hipStream_t st = h->stream;
  if (S.meta_dirty) {  // (the table's cell layout: uploaded once per table, through the
                       // pinned staging on the engine stream -- begin never waits for it)
    std::vector<uint32_t> np(E);
    for (uint64_t e = 0; e < E; e++) np[e] = h->hist_base[e] == kHistSparse ? 0u : (uint32_t)h->npages[e];
    rc = stage_h2d(h, S.d_base, h->hist_base.data(), E * 8);
    if (!rc) rc = stage_h2d(h, S.d_np, np.data(), E * 4);
    if (!rc) rc = stage_h2d(h, S.d_sent, h->sparse_entries.data(), nsent * 4);
    if (rc) return rc;
    S.meta_dirty = false;
  }
  // the sparse entries as this table has them: nmg_results_end places the
  // sparse rows with these, whatever table the engine holds by then
  S.sent_entry.resize(nsent);
  for (uint64_t s = 0; s < nsent; s++) {
    const uint32_t e = h->sparse_entries[s];
    S.sent_entry[s] = h->hist_base[e] == kHistSparse ? e : ~0u;
  }
  // the device snapshot, behind the enqueued analyses
  HIP_TRY(h, hipMemcpyAsync(S.d_sum, h->d_sum64, 2 * kGlobalSums * 8, hipMemcpyDeviceToDevice, st));
  HIP_TRY(h, hipMemcpyAsync(S.d_min, h->d_min64, (36 + E) * 8, hipMemcpyDeviceToDevice, st));
  HIP_TRY(h, hipMemcpyAsync(S.d_max, h->d_max64, 36 * 8, hipMemcpyDeviceToDevice, st));
  if (nb) {
    HIP_TRY(h, hipMemcpyAsync(S.d_bufcnt, h->d_bufcnt, nb * 4, hipMemcpyDeviceToDevice, st));
    HIP_TRY(h, hipMemcpyAsync(S.d_bufcnt + nb, h->d_bufcnt + h->bufcnt_stride, nb * 4, hipMemcpyDeviceToDevice, st));
  }
  if (h->d_found) HIP_TRY(h, hipMemcpyAsync(S.d_found, h->d_found, 8, hipMemcpyDeviceToDevice, st));
  else HIP_TRY(h, hipMemsetAsync(S.d_found, 0, 8, st));
  if (E) HIP_TRY(h, launch_objcw_aos(st, h->d_sum64 + 2 * kGlobalSums, E, S.d_objcw));
  // page-cell rows: per-entry counts (dense, then the sparse table's), their
  // exclusive scan, the dense rows; the sparse ones are placed by the host
  unsigned long long* nsp = S.d_ck ? reinterpret_cast<unsigned long long*>(S.d_ck + 2 * S.sparse_cap) : nullptr;
  if (E) {
    if (h->hist_cells)
      HIP_TRY(h, launch_cells_count(st, h->d_hist, h->hist_cells, h->T, S.d_base, S.d_np, (uint32_t)E, S.d_cnt));
    else
      HIP_TRY(h, hipMemsetAsync(S.d_cnt, 0, E * 4, st));
    if (nsp) {
      HIP_TRY(h, hipMemsetAsync(nsp, 0, 8, st));
      HIP_TRY(h, launch_sparse_compact(st, h->d_sparse_keys, h->d_sparse_vals, h->sparse_cap, S.d_ck, nsp));
      HIP_TRY(h, launch_cells_sparse_count(st, S.d_ck, nsp, h->sparse_cap, S.d_sent, (uint32_t)nsent, S.d_base,
                                           S.d_cnt));
    }
    HIP_TRY(h, launch_scan_u32(st, S.d_cnt, E, S.d_off, S.d_part));
    if (h->hist_cells)
      HIP_TRY(h, launch_cells_emit(st, h->d_hist, h->hist_cells, h->T, S.d_base, S.d_np, (uint32_t)E, S.d_off,
                                   (uint4*)S.d_rows));
    HIP_TRY(h, launch_gather_off(st, S.d_off, S.d_sent, (uint32_t)nsent, S.d_soff));
  } else {
    HIP_TRY(h, hipMemsetAsync(S.d_off, 0, 8, st));
  }
  HIP_TRY(h, hipEventRecord(S.ready, st));
  // the copy to pinned host memory, on the snapshot's own stream
  hipStream_t cs = S.stream;
  HIP_TRY(h, hipStreamWaitEvent(cs, S.ready, 0));
  HIP_TRY(h, hipMemcpyAsync(S.h_sum, S.d_sum, 2 * kGlobalSums * 8, hipMemcpyDeviceToHost, cs));
  HIP_TRY(h, hipMemcpyAsync(S.h_min, S.d_min, (36 + E) * 8, hipMemcpyDeviceToHost, cs));
  HIP_TRY(h, hipMemcpyAsync(S.h_max, S.d_max, 36 * 8, hipMemcpyDeviceToHost, cs));
  if (nb) HIP_TRY(h, hipMemcpyAsync(S.h_bufcnt, S.d_bufcnt, 2 * nb * 4, hipMemcpyDeviceToHost, cs));
  HIP_TRY(h, hipMemcpyAsync(S.h_small, S.d_found, 8, hipMemcpyDeviceToHost, cs));
  HIP_TRY(h, hipMemcpyAsync(S.h_small + 1, S.d_off + E, 8, hipMemcpyDeviceToHost, cs));
  if (nsp) HIP_TRY(h, hipMemcpyAsync(S.h_small + 2, nsp, 8, hipMemcpyDeviceToHost, cs));
  else S.h_small[2] = 0;
  if (E) HIP_TRY(h, hipMemcpyAsync(S.h_objcw, S.d_objcw, E * 32, hipMemcpyDeviceToHost, cs));
  if (nsent) HIP_TRY(h, hipMemcpyAsync(S.h_soff, S.d_soff, nsent * 8, hipMemcpyDeviceToHost, cs));
  if (S.h_rows && S.rows_host) {  // (the rows' number is on the device: a kernel copies them)
    void* dst = nullptr;
    HIP_TRY(h, hipHostGetDevicePointer(&dst, S.h_rows, 0));
    HIP_TRY(h, launch_copy_rows(cs, S.d_rows, S.d_off + E, S.rows_host, dst));
  }
  HIP_TRY(h, hipEventRecord(S.copied, cs));
  S.pending = true;
  h->snap_nb = nb;
  return NMG_OK;
}

extern "C" int nmg_results_end(nmg_engine* h, nmg_results_view* out) {
  Range range("nmg_results_end");
  if (!h || !out) return NMG_ERR_INVALID;
  auto& S = h->snap;
  if (!S.pending) return fail(h, NMG_ERR_STATE, "nmg_results_end without nmg_results_begin");
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipEventSynchronize(S.copied));
  S.pending = false;
  const uint64_t E = S.E, nb = h->snap_nb, nsent = S.sent_entry.size();  // (the begin-time table's)
  const uint64_t nrows = S.h_small[1], nspc = S.h_small[2];
  if (nrows > S.rows_host) {  // (the pinned rows outgrown: grown, and this time copied here)
    (void)hipHostFree(S.h_rows);
    S.h_rows = nullptr;
    S.rows_host = 0;
    const uint64_t cap = nrows + nrows / 4 + 1024;
    HIP_TRY(h, hipHostMalloc((void**)&S.h_rows, cap * 16, 0));
    S.rows_host = cap;
    HIP_TRY(h, hipMemcpy(S.h_rows, S.d_rows, nrows * 16, hipMemcpyDeviceToHost));
  }
  if (nspc) {  // the sparse cells, each entry's in (thread, page) order at its rows
    std::vector<uint64_t> kv(2 * nspc);
    HIP_TRY(h, hipMemcpy(kv.data(), S.d_ck, 2 * nspc * 8, hipMemcpyDeviceToHost));
    std::vector<std::vector<std::pair<uint64_t, uint32_t>>> per(nsent);
    for (uint64_t i = 0; i < nspc; i++) {
      const uint64_t k = kv[2 * i];
      const uint32_t v = (uint32_t)kv[2 * i + 1];
      const uint32_t s = sparse_key_idx(k);
      if (k == ~0ull || !v || s >= nsent || S.sent_entry[s] == ~0u) continue;
      per[s].push_back({(uint64_t(sparse_key_thread(k)) << 32) | sparse_key_page(k), v});
    }
    for (uint64_t s = 0; s < nsent; s++) {
      auto& l = per[s];
      if (l.empty()) continue;
      std::sort(l.begin(), l.end());
      uint32_t* r = S.h_rows + S.h_soff[s] * 4;
      for (const auto& c : l) {
        r[0] = S.sent_entry[s];
        r[1] = (uint32_t)(c.first >> 32);
        r[2] = (uint32_t)c.first;
        r[3] = c.second;
        r += 4;
      }
    }
  }
  memset(out, 0, sizeof(*out));
  for (int a = 0; a < 2; a++) {  // (as engine_download)
    nmg_mem_counters& c = out->global[a];
    const uint64_t* s = S.h_sum + gsum_index(a, 0);
    c.total_count = s[0];
    c.total_weight = s[1];
    c.na_miss_count = s[2];
    for (int k = 0; k < 18; k++) {
      c.b[k].count = s[3 + 2 * k];
      c.b[k].sum_weight = s[4 + 2 * k];
      c.b[k].min_weight = S.h_min[a * 18 + k];
      c.b[k].max_weight = S.h_max[a * 18 + k];
    }
  }
  uint64_t ns = 0;
  for (uint64_t b = 0; b < nb; b++) ns += (uint64_t)(int64_t)(int32_t)S.h_bufcnt[b];
  out->nb_samples = ns;
  out->nb_found = S.h_small[0];
  out->nb_buffers = (uint32_t)nb;
  out->nb_entries = (uint32_t)E;
  out->buffer_samples = S.h_bufcnt;
  out->buffer_found = S.h_bufcnt + nb;
  out->first_ordinal = S.h_min + 36;
  out->count_weight = S.h_objcw;
  out->nb_cells = (int64_t)nrows;
  out->cells = S.h_rows;
  return NMG_OK;
}
