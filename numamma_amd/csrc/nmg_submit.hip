// nmg_submit.hip -- buffer submission (the staging point of __copy_buffer,
// src/mem_sampling.c:675-738), zero-copy host registration, the streaming
// pipeline of --online-analysis (__process_samples, :929-966), schedules and
// the single-pass attribution launch.
#include "nmg_engine_impl.h"

int stage_reserve(nmg_engine* h, size_t need) {
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

int append_desc(nmg_engine* h, uint64_t len, uint32_t thread_rank, uint32_t access) {
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
uint64_t zero_copy_dev(nmg_engine* h, const void* p, uint64_t len) {
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
int append_desc_zc(nmg_engine* h, uint64_t dev, uint64_t len, uint32_t thread_rank, uint32_t access) {
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

int check_buffer_args(nmg_engine* h, uint64_t len, uint32_t thread_rank, uint32_t access) {
  if (access > 1) return fail(h, NMG_ERR_INVALID, "access_type must be 0 (read) or 1 (write)");
  if (thread_rank >= h->T)
    return fail(h, NMG_ERR_RANGE, "thread_rank >= nb_threads (set nmg_options.nb_threads)");
  if (len >= (1ull << 32)) return fail(h, NMG_ERR_RANGE, "buffer >= 4 GiB (unsigned cursors, mem_sampling.c:831-834)");
  if (h->external) return fail(h, NMG_ERR_STATE, "device buffers are set; call nmg_clear_buffers first");
  if (h->streamed && !h->streaming) return fail(h, NMG_ERR_STATE, "stream ended; call nmg_clear_buffers first");
  return NMG_OK;
}


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

void run_copies(nmg_engine* h, const std::vector<CopyTask>& tasks) {
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
int slot_acquire(nmg_engine* h, int s) {
  auto& sl = h->slots[s];
  if (sl.used) HIP_TRY(h, hipEventSynchronize(sl.copied));
  sl.len = 0;
  sl.descs.clear();
  return NMG_OK;
}

// per-buffer count array for `need` buffers; its stride stays fixed while
// chunks are in flight (grown by doubling after draining the engine stream)
int ensure_bufcnt(nmg_engine* h, size_t need) {
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
int stream_flush(nmg_engine* h) {
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
int stream_dst(nmg_engine* h, uint64_t len, uint8_t** dst, std::vector<CopyTask>* pending) {
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

int stream_append(nmg_engine* h, uint64_t len, uint32_t thread_rank, uint32_t access) {
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

int stage_h2d(nmg_engine* h, void* d_dst, const void* src, size_t n) {
  if (!n) return NMG_OK;
  const size_t need = (n + 255) & ~size_t(255);
  if (h->up_off + need > h->up_cap) {  // full: every copy from it done first, then from its start
    if (h->up_recorded) HIP_TRY(h, hipEventSynchronize(h->up_ev));
    h->up_off = 0;
    if (need > h->up_cap) {
      (void)hipHostFree(h->up_pin);
      h->up_pin = nullptr;
      h->up_cap = 0;
      const size_t cap = std::max<size_t>(need * 2, 4u << 20);
      HIP_TRY(h, hipHostMalloc((void**)&h->up_pin, cap, 0));
      h->up_cap = cap;
    }
  }
  if (!h->up_ev) HIP_TRY(h, hipEventCreateWithFlags(&h->up_ev, hipEventDisableTiming));
  uint8_t* p = h->up_pin + h->up_off;
  memcpy(p, src, n);
  HIP_TRY(h, hipMemcpyAsync(d_dst, p, n, hipMemcpyHostToDevice, h->stream));
  HIP_TRY(h, hipEventRecord(h->up_ev, h->stream));
  h->up_recorded = true;
  h->up_off += need;
  return NMG_OK;
}

void stage_reset(nmg_engine* h) {
  // the previous analysis' copies ran before its kernels, so this wait is
  // normally already satisfied
  if (h->up_recorded) (void)hipEventSynchronize(h->up_ev);
  h->up_off = 0;
}

int upload_buffers(nmg_engine* h) {
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
      stage_reset(h);
      const int rc = stage_h2d(h, h->d_descs, h->descs.data(), n * sizeof(BufDesc));
      if (rc) return rc;
      HIP_TRY(h, hipMemsetAsync(h->d_bufcnt, 0, n * 2 * 4, h->stream));
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
void make_schedule(const std::vector<BufDesc>& descs, uint32_t grid, uint32_t index_base, BufDesc* sorted,
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
int build_schedule(nmg_engine* h, uint32_t grid, bool by_stream) {
  const uint32_t nb = (uint32_t)h->descs.size();
  std::vector<uint32_t> ranges(grid + 1, 0);
  std::vector<BufDesc> sorted(nb);
  make_schedule(h->descs, grid, 0, sorted.data(), ranges.data(), by_stream);
  if (nb > h->sdescs_cap || grid + 1 > h->ranges_cap || !h->d_sdescs) {  // (grown only: a free waits for the device)
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    (void)hipFree(h->d_sdescs);
    (void)hipFree(h->d_ranges);
    h->d_sdescs = nullptr;
    h->d_ranges = nullptr;
    h->sdescs_cap = std::max<size_t>(nb, 1);
    h->ranges_cap = grid + 1;
    HIP_TRY(h, hipMalloc(&h->d_sdescs, h->sdescs_cap * sizeof(BufDesc)));
    HIP_TRY(h, hipMalloc(&h->d_ranges, h->ranges_cap * 4));
  }
  int rc = stage_h2d(h, h->d_sdescs, sorted.data(), nb * sizeof(BufDesc));
  if (!rc) rc = stage_h2d(h, h->d_ranges, ranges.data(), (grid + 1) * 4);
  if (rc) return rc;
  h->sched_grid = grid;
  h->sched_route = !by_stream;
  if (!by_stream) return route_prepare(h, grid, ranges);
  return NMG_OK;
}

void ensure_occupancy(nmg_engine* h) {
  if (h->blocks_per_cu <= 0) {
    h->blocks_per_cu = attribute_blocks_per_cu();
  }
}

// persistent grid: one resident workgroup per slot, each with a byte-balanced range
uint32_t attribution_grid(nmg_engine* h, uint32_t nb) {
  ensure_occupancy(h);
  return nb ? std::min<uint32_t>(nb, (uint32_t)(h->num_cus * h->blocks_per_cu)) : 0;
}

// One attribution launch over `nb` buffers whose stream-sorted descriptors and
// per-workgroup ranges are already on the device, on the engine stream,
// bracketed by the launch-timing events.
// The kernels' view of the engine: buffers, table, counters.
Params base_params(nmg_engine* h, const uint8_t* data, const BufDesc* sdescs, const uint32_t* ranges) {
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
int launch_events(nmg_engine* h, int* slot_out) {
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

int launch_attribution(nmg_engine* h, const uint8_t* data, const BufDesc* sdescs, const uint32_t* ranges,
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
      h->counters_fresh = false;
      HIP_TRY(h, launch_attribute(true, mode, grid, h->stream, p));
    } else {
      h->counters_fresh = false;
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
