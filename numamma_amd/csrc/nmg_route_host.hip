// nmg_route_host.hip -- host side of the partition-first path (nmg_route.h):
// eligibility, compact-record layout, chunk pools, the route / count / plan /
// scatter / local launches.
#include "nmg_engine_impl.h"

// ---------------------------------------------------------------------------
// partition-first path (nmg_route.h): eligibility, pool sizing, launches

uint32_t bits_for(uint64_t v) {  // smallest b with v < 2^b
  uint32_t b = 0;
  while (b < 64 && (v >> b) != 0) b++;
  return b;
}

// X word layout of the current buffers; false when the weight field would
// be narrower than kMinWeightBits (escapes would be common)
bool route_layout(nmg_engine* h, const std::vector<BufDesc>& descs, XLayout& xl) {
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
bool route_eligible(nmg_engine* h, const std::vector<BufDesc>& descs) {
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
bool route_eligible(nmg_engine* h) { return route_eligible(h, h->descs); }

// per-workgroup private chunk pools for a new schedule: every SAMPLE record
// of at least 40 B fits (a partition's chunks are full but for its open and
// next chunks); shorter records past that are attributed directly
int route_pool(nmg_engine* h, const std::vector<BufDesc>& descs, uint32_t grid, const uint32_t* ranges,
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
    HIP_TRY(h, hipMalloc(&h->d_ctl, 4 * 4));
    HIP_TRY(h, hipMemset(h->d_ctl, 0, 4 * 4));
    HIP_TRY(h, hipMalloc(&h->d_ovf16, ovf * sizeof(uint4)));
    HIP_TRY(h, hipMalloc(&h->d_ovfx, ovf * 8));
    h->ovf_cap = ovf;
    h->route_chunk_cap = cap;
    h->items_cap = items;
    h->route_grid_cap = grid;
  }
  return NMG_OK;
}

int route_prepare(nmg_engine* h, uint32_t grid, const std::vector<uint32_t>& ranges) {
  std::vector<uint32_t> c0;
  const int rc = route_pool(h, h->descs, grid, ranges.data(), c0);
  if (rc) return rc;
  const int rc2 = stage_h2d(h, h->d_chunk0, c0.data(), (grid + 1) * 4);
  if (rc2) return rc2;
  h->route_sched_key = h->nparts | ((h->flags & kDbgTinyPool) ? 0x80000000u : 0u);
  return NMG_OK;
}


// Route -> plan -> scatter -> local over the buffers of the current schedule
// (analysis order), bracketed by the launch-timing events.
int route_analyze(nmg_engine* h, uint32_t nb, uint32_t grid) {
  (void)nb;
  RouteJob job{&h->descs, h->d_data, h->d_sdescs, h->d_ranges, h->d_chunk0, grid, 0, false};
  return route_analyze_job(h, job);
}

int route_analyze_job(nmg_engine* h, const RouteJob& job) {
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
  rp.pdead = h->d_pdead;
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
  lp.pe_pnode = h->d_pe_pnode;
  lp.pe_old = h->d_pe_old;
  lp.pe_oinf = h->d_pe_oinf;
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
  lp.fresh = h->counters_fresh ? 1u : 0u;
  h->counters_fresh = false;
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
    f.gshift = 16 + xl.wbits + xl.obits;
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
int route_settle(nmg_engine* h) {
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
  f.gshift = 16 + h->route_xl.wbits + h->route_xl.obits;
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, launch_found(h->route_grid, h->stream, f));
  return NMG_OK;
}
