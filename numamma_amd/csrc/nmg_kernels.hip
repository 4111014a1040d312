// nmg_kernels.hip -- MI355X (gfx950) device code of the sample-attribution engine.
//
// Replaces NumaMMa's offline analysis loop (src/mem_sampling.c:311-346 ->
// __analyze_buffer :815-927 -> update_counters :517-592 / __match_sample
// :594-673 -> ma_find_mem_info_from_sample src/mem_analyzer.c:249-306 ->
// ma_get_block :494-534).
//
// Kernel shape (DESIGN.md "Kernels"):
//   * persistent grid, one 1024-thread workgroup per CU, each owning a
//     byte-balanced range of the buffer list sorted by stream (access type,
//     thread rank); a buffer is walked in windows of 1024 stride slots of
//     40 B, one per lane, loaded straight into registers, the next window
//     issued before the current one is processed;
//   * fast path when every slot of a window holds a whole 40 B record (the
//     record chain is then known without reading it sequentially); otherwise
//     wave 0 follows the header chain exactly as the reference's byte cursor
//     does (variable-size non-SAMPLE records, size==0 abort, truncation);
//   * global counters (mem_counters[2]) in per-lane registers / LDS, flushed
//     once per stream run;
//   * object lookup: <= 1023 keys, an Eytzinger search of keys + node records
//     held in LDS; larger tables, an Eytzinger search of up to 4095 LDS fences,
//     one 8 B load of the fence bucket's directory slot, then the node record
//     (L2 / MALL) -> older entries of the node (quirks Q1-Q4);
//   * per-object and per-page counters aggregated in LDS tables (dense by
//     entry id / cell for small tables, first-come 8-way buckets otherwise),
//     flushed with global atomics at stream ends and on a window cadence;
//     integer adds, mins and maxes are order independent, so results are
//     bit-exact;
//   * the long-tail log's range reduce, the packed-counter fold and the
//     counter reset; the host side is nmg_engine.hip.
#include <algorithm>

#include "nmg_device.h"

namespace nmg {

// Largest key <= addr (ht_lower_key, tools/hash.c:63-77) for tables larger
// than kLdsNodes.  Returns nb_keys when no key <= addr.
//  1. LDS: branch-free search of the 12-level Eytzinger fence tree -> bucket b
//     (keys [b*S, (b+1)*S), S = fence_step);
//  2. global: one 8 B directory slot of bucket b.  The bucket's key span is
//     cut into 2^dir_log2 equal slots of 2^shift bytes; a slot holds the
//     bucket-relative index of the largest key <= the slot start, the number
//     of keys strictly inside the slot and the offset of the first of them.
//     Zero or one key inside the slot is resolved by that one load;
//  3. more keys inside the slot (or a bucket too wide for a directory): a
//     binary search of those keys in global memory (L2 / MALL resident).
// A lane's lookup of the next window started early (large tables): the fence
// node of `addr` and, when the lookup needs it, its directory slot, loaded
// while the current window is processed.  Valid for a record whose address
// on the record the lane processes in that window when it is a fast-path
// window (`on`; idx 0: none).
struct SpecDir {
  uint32_t idx;
  uint2 de;
  bool on;
};


// The directory slot that lower_key reads for (addr, fence node idx), or
// null when it reads none.
__device__ __forceinline__ const uint2* dir_slot(const Params& p, const uint64_t* s_fences, const uint8_t* s_shift,
                                                 uint64_t addr, uint32_t idx) {
  if (idx == 0 || p.dir_log2 == 0) return nullptr;
  const uint32_t d = 31 - __builtin_clz(idx);
  const uint32_t b = (((idx - (1u << d)) * 2 + 1) << (kFenceLevels - 1 - d)) - 1;
  if (b >= p.nb_fences) return nullptr;
  const uint32_t sh = s_shift[b];
  if (sh == kShiftSearch) return nullptr;
  const uint64_t rel = addr - s_fences[idx];
  const uint32_t j = (uint32_t)min(rel >> sh, (uint64_t)((1u << p.dir_log2) - 1));
  return p.dir + ((uint64_t(b) << p.dir_log2) + j);
}

__device__ __forceinline__ uint32_t lower_key(const Params& p, const uint64_t* s_fences, const uint8_t* s_shift,
                                              uint64_t addr, const SpecDir& sp) {
  const bool spec = sp.idx != 0 && sp.on;
  const uint32_t idx = spec ? sp.idx : fence_node(s_fences, addr);
  if (idx == 0) return p.nb_keys;                    // addr < first key
  // in-order rank of Eytzinger node idx at depth d of a complete tree
  const uint32_t d = 31 - __builtin_clz(idx);
  const uint32_t b = (((idx - (1u << d)) * 2 + 1) << (kFenceLevels - 1 - d)) - 1;
  if (b >= p.nb_fences) return p.nb_keys - 1;  // ~0 padding: addr == UINT64_MAX
  const uint32_t k0 = b << p.fence_log2;
  if (p.fence_log2 == 0) return k0;  // one key per fence
  // (buckets without a directory -- more than 2^16 keys per bucket, or the
  // kDbgNoDir switch -- have shift kShiftSearch: binary search below)
  const uint32_t kend = min(k0 + (1u << p.fence_log2), p.nb_keys);
  const uint32_t sh = s_shift[b];
  uint32_t lo, n;  // answer in [lo, lo + n): keys[lo] <= addr known
  if (sh != kShiftSearch) {
    const uint64_t f = s_fences[idx];
    const uint32_t slots = 1u << p.dir_log2;
    const uint64_t rel = addr - f;
    const uint32_t j = (uint32_t)min(rel >> sh, (uint64_t)(slots - 1));
    const uint2 de = spec ? sp.de : p.dir[(uint64_t(b) << p.dir_log2) + j];
    lo = k0 + (de.x & 0xffffu);
    const uint32_t cnt = de.x >> 16;
    // first key inside the slot is <= addr: the answer is among the cnt keys
    if (cnt == 0 || rel - (uint64_t(j) << sh) < de.y) return lo;
    lo += 1;
    n = cnt;
  } else {
    lo = k0;
    n = kend - k0;
  }
  while (n > 1) {  // keys[lo] <= addr < keys[lo + n] (or lo + n == bucket end)
    const uint32_t half = n >> 1;
    const bool le = p.keys[lo + half] <= addr;
    lo = le ? lo + half : lo;
    n = le ? n - half : half;
  }
  return lo;
}

// Per-workgroup privatised counters of the stream (access type, thread rank)
// being analysed.  One stream at a time per workgroup, so (entry) and
// (entry, page) are the keys of the aggregation tables.
struct WgCounters {
  unsigned long long sums[kGlobalSums];  // total_count, total_weight, na, 18 x (count, sum)
  unsigned long long mins[18];
  unsigned long long maxs[18];
  alignas(16) unsigned int okey[kObjSlots];  // entry id, 8 per bucket (hashed modes)
  unsigned long long ofirst[kObjSlots];  // smallest (seq << 32 | offset): first match
  unsigned long long owt[kObjSlots];     // count << kPackShift | weight sum (weights < kLaneMaxWeight)
  union {
    struct {
      uint4 pkey4[kPageSlots / 4];  // dense cell index (hist_base(entry) + page), 8 per bucket
      unsigned int pcnt[kPageSlots];
    };
    unsigned int pdense[kDensePageCells / 2];  // kModeDensePage: u16 count per cell, two per word
  };
  unsigned int tcur[kLogParts];  // long-tail sub-log cursors
};

// Entries (tables with more than kObjSlots entries): a Fibonacci hash picks
// one 8-slot bucket, found with two 16 B LDS reads; a missing entry takes the
// first empty slot by CAS (same protocol as page_slot below).  Slots are
// first come, first served until the next flush (stream end or the
// kTableWindows cadence): the hot entries of a Zipf-like stream claim them
// in its first windows, and a full bucket sends the sample straight to the
// global counters -- no probe chains and no fill-level flushes.
__device__ __forceinline__ uint32_t obj_bucket(uint32_t e) {
  return (uint32_t)(((uint64_t)(e * 0x9E3779B1u) * kObjBuckets) >> 32);
}

__device__ __forceinline__ int obj_slot(WgCounters& wc, uint32_t e) {
  const uint32_t hb = obj_bucket(e);
  const int j = bucket_slot(&wc.okey[hb * 8], e);
  return j < 0 ? -1 : (int)(hb * 8 + (uint32_t)j);
}

// Page cells: a Fibonacci hash picks one 8-slot bucket (two 16 B LDS reads,
// no probe chain).  A missing cell takes the first empty slot by CAS; every
// inserter scans the bucket in the same order and a slot leaves "empty" only
// once, so a cell never lands in two slots.  A full bucket returns -1 (the
// caller then updates global memory directly).
__device__ __forceinline__ uint32_t page_bucket(uint32_t cell) {
  return (uint32_t)(((uint64_t)(cell * 0x9E3779B1u) * kPageBuckets) >> 32);
}

__device__ __forceinline__ int page_slot_at(uint4* pkey4, uint32_t cell) {
  const uint32_t hb = page_bucket(cell);
  const int j = bucket_slot(reinterpret_cast<unsigned int*>(&pkey4[2 * hb]), cell);
  return j < 0 ? -1 : (int)(hb * 8 + (uint32_t)j);
}

__device__ __forceinline__ int page_slot(WgCounters& wc, uint32_t cell) {
  return page_slot_at(wc.pkey4, cell);
}

// The object table as the kernel sees it: node records in LDS (small tables)
// or in global memory (L2/MALL resident) behind the LDS fence table.
struct Lookup {
  const uint64_t* fences;  // LDS: Eytzinger keys (small tables) or fences (large tables)
  const uint4* nodes;      // LDS (small tables): 2 x uint4 per node: (addr, end), (alloc, free)
  const uint2* ninfo;      // LDS (small tables): (dense histogram base or ~0, entry id | older-entries << 31)
  const uint8_t* shift;    // LDS (large tables): per-bucket directory shift
};

// __ma_find_mem_info_from_sample_generic (mem_analyzer.c:249-286): the
// lower-bound node only (ht_lower_key, tools/hash.c:63-77), newest entry
// first, inclusive timestamp window (is_sample_in_buffer, :141-155).
template <int MODE>
__device__ __forceinline__ Match find_entry(const Params& p, const Lookup& L, uint64_t addr, uint64_t ts,
                                            const SpecDir& sp) {
  Match m;
  m.e = -1;
  m.baddr = 0;
  m.hist = kHistSparse;
  if (!(MODE & kModeLarge)) {
    // Eytzinger tree: node i has children 2i, 2i+1; a fixed number of levels,
    // one LDS read each, branch-free.  The levels above the 7th fit in one
    // 256 B bank row, so the search is conflict-free where every lane reads.
    const uint32_t i = eytz_descend(L.fences, p.elevels, addr);
    // largest key <= addr = the node of the last right turn (0: none)
    const uint32_t idx = i >> (__builtin_ctz(i) + 1);
    if (idx == 0) return m;
    const uint4 a = L.nodes[2 * idx], b = L.nodes[2 * idx + 1];
    const uint2 inf = L.ninfo[idx];
    if (entry_match(a, b, addr, ts)) {
      m.e = inf.y & 0x7fffffffu;
      m.baddr = (uint64_t(a.y) << 32) | a.x;
      m.hist = inf.x == kEmpty32 ? kHistSparse : (uint64_t)inf.x;
    } else if (inf.y >> 31) {
      match_older(p, p.enodes[idx].first, p.enodes[idx].count, addr, ts, m);
    }
    return m;
  }
  return m;
}

// Large tables, in two halves so that independent work can run while the node
// record is in flight: node_issue (lower bound + the node record's loads),
// node_match (the newest entry, then the older ones).
struct NodePre {
  uint32_t k;  // lower-bound key index (nb_keys: none)
  uint4 a, b, c;
};

__device__ __forceinline__ NodePre node_issue(const Params& p, const Lookup& L, bool valid, uint64_t addr,
                                              const SpecDir& sp) {
  NodePre n;
  n.k = valid ? lower_key(p, L.fences, L.shift, addr, sp) : p.nb_keys;
  n.a = n.b = n.c = make_uint4(0, 0, 0, 0);
  if (n.k < p.nb_keys) {
    const uint4* q = reinterpret_cast<const uint4*>(p.nodes + n.k);
    n.a = q[0];
    n.b = q[1];
    n.c = q[2];
  }
  return n;
}

__device__ __forceinline__ Match node_match(const Params& p, const NodePre& n, uint64_t addr, uint64_t ts) {
  Match m;
  m.e = -1;
  m.baddr = 0;
  m.hist = kHistSparse;
  if (n.k >= p.nb_keys) return m;
  const uint4 a = n.a, b = n.b, c = n.c;
  if (entry_match(a, b, addr, ts)) {
    m.e = c.w;
    m.baddr = (uint64_t(a.y) << 32) | a.x;
    m.hist = (uint64_t(c.y) << 32) | c.x;
    return m;
  }
  const uint4 d = reinterpret_cast<const uint4*>(p.nodes + n.k)[3];
  if (d.x > 1) match_older(p, d.y, d.x, addr, ts, m);  // (count, first)
  return m;
}

// One long-tail contribution to this workgroup's sub-log of entry e; false
// when the sub-log is full (the caller then issues the global atomics).
__device__ __forceinline__ bool tlog_append(const Params& p, WgCounters& wc, uint32_t e, uint32_t a, uint32_t cnt,
                                            uint64_t wt, uint64_t ord) {
  return tlog_put(p, wc.tcur, e, a, cnt, wt, ord);
}

// kDbgTiming sub-phases of the window's processing (per wave, cycles)
struct SubTimer {
  uint64_t acc[7];
  uint64_t last;
};
template <bool TIMING>
__device__ __forceinline__ void sub_stamp(SubTimer& st, int i) {
  if (TIMING) {
    const uint64_t t = stamp();
    st.acc[i] += t - st.last;
    st.last = t;
  }
}

// Process one decoded record (`valid` = it is a SAMPLE).  Every lane of the
// wave calls this together (wave-level reductions inside); vmask / fmask are
// the wave's SAMPLE and matched lanes.
template <int MODE, bool TIMING>
__device__ __forceinline__ void process_sample(Params& p, WgCounters& wc, LaneAcc& acc, const Lookup& L, SubTimer& st,
                                               bool valid, bool shortrec, uint64_t ts, uint64_t addr,
                                               uint64_t w, uint64_t dsrc, uint32_t access,
                                               uint32_t th, const BufDesc& b0, const BufDesc& b1, bool in1, uint32_t off,
                                               uint64_t& vmask, uint64_t& fmask, const SpecDir& sp) {
  // (the lane's buffer: b1 when in1; selected where used, so no 64-bit
  // per-lane copy stays live across the window)
  const uint32_t lvl = uint32_t(dsrc >> 5) & 0x3fff;  // data_src.mem_lvl
  // ---- global counters: update_counters(global_counters, ...) (mem_sampling.c:882)
  vmask = __ballot(valid);
  fmask = 0;
  if (vmask == 0) return;
  // large tables: the node record's loads go out first; the global counters
  // below do not depend on them and run while they are in flight
  NodePre np;
  if ((MODE & kModeLarge) && (p.flags & NMG_F_MATCH_SAMPLES)) np = node_issue(p, L, valid, addr, sp);
  if (valid && !(p.flags & kDbgNoGlobal)) global_count(acc, wc.sums, wc.mins, wc.maxs, lvl, w);
  sub_stamp<TIMING>(st, 0);
  if (!(p.flags & NMG_F_MATCH_SAMPLES)) return;

  // ---- __match_sample (mem_sampling.c:594-673)
  Match m;
  m.e = -1;
  if (MODE & kModeLarge) {
    if (valid) m = node_match(p, np, addr, ts);
  } else if (valid) {
    m = find_entry<MODE>(p, L, addr, ts, sp);
  }
  const int64_t e = m.e;
  fmask = __ballot(e >= 0);
  sub_stamp<TIMING>(st, 1);
  // dump modes: every SAMPLE record's match at its arena position (host
  // formats the per-sample lines in analysis order)
  if (p.smatch && valid) p.smatch[((in1 ? b1.offset : b0.offset) + off) >> 3] = e >= 0 ? (uint32_t)e + 1u : 0u;
  if (e < 0 || (p.flags & kDbgNoTables)) return;
  // per-object counters, aggregated per stream in LDS.  (Admitting an entry
  // only on its second sample -- a doorkeeper bitset -- was measured slower at
  // 1M intervals: the per-sample bit test costs more than the flushes it saves.)
  // A slot sums (count << kPackShift | weight) in one u64 LDS add, for weights
  // < kLaneMaxWeight (dense: bounded by the kDensePageWindows cadence, < 2^16
  // samples; hashed: by kTableWindows, < 2^17 samples).  With the packed
  // long-tail counters on, a hashed slot only takes weights they can pack too
  // (its flush is packed as well); any other sample takes the table-full path.
  const bool pk = !(MODE & kModeDenseObj) && p.pk64 && w < p.pk_wlim && !shortrec;
  const bool lds_ok = w < kLaneMaxWeight && (!(MODE & kModeDenseObj) ? (!p.pk64 || pk) : kPackObj);
  const int os = !lds_ok ? -1 : ((MODE & kModeDenseObj) ? (int)e : obj_slot(wc, (uint32_t)e));
  const unsigned long long ord = ((in1 ? b1.seq : b0.seq) << 32) | off;  // first match in analysis order (quirk Q7)
  if (os >= 0) {
    atomicAdd(&wc.owt[os], (1ull << kPackShift) | w);
    if (ord < wc.ofirst[os]) atomicMin(&wc.ofirst[os], ord);
  } else if (!(MODE & kModeDenseObj) && p.tlog && tlog_append(p, wc, (uint32_t)e, access, 1u, w, ord)) {
    // table full: logged for tlog_reduce_kernel
  } else if (pk) {  // table full: one packed global add
    atomicAdd(p.pk64 + uint64_t(access) * p.nb_entries + e, (1ull << p.pk_shift) | w);
    unsigned long long* fp = reinterpret_cast<unsigned long long*>(p.min64 + 36 + e);
    atomicMin(fp, ord);
  } else {  // table full (or a weight >= 2^23 in dense mode): straight to global
    atomicAdd(reinterpret_cast<unsigned long long*>(p.sum64 + objcw_index(e, access, 0, p.nb_entries)), 1ull);
    if (w)
      atomicAdd(reinterpret_cast<unsigned long long*>(p.sum64 + objcw_index(e, access, 1, p.nb_entries)),
                (unsigned long long)w);
    unsigned long long* fp = reinterpret_cast<unsigned long long*>(p.min64 + 36 + e);
    atomicMin(fp, ord);
  }
  sub_stamp<TIMING>(st, 2);
  if (p.flags & NMG_F_PAGE_HIST) {
    // ma_get_block: page_no = (int)((addr - buffer_addr) / 4096) (mem_analyzer.c:530-531)
    const uint32_t page = uint32_t(int(uint64_t(addr - m.baddr) / kPageSize));
    if (m.hist != kHistSparse) {
      const uint32_t cell = uint32_t(m.hist + page);
      if (MODE & kModeDensePage) {
        atomicAdd(&wc.pdense[cell >> 1], 1u << (16 * (cell & 1)));
      } else {
        const int ps = page_slot(wc, cell);
        if (ps >= 0) atomicAdd(&wc.pcnt[ps], 1u);
        else
          atomicAdd(p.hist + uint64_t(th) * p.hist_cells + cell, 1u);
      }
    } else {
      const uint32_t sidx = p.entries[e].sidx;
      if (sidx != ~0u)  // huge objects ([stack]): hashed cells in global memory
        sparse_add(p, sparse_key(sidx, th, page), in1 ? b1.seq : b0.seq, off, 1u);
    }
  }
  sub_stamp<TIMING>(st, 3);
  if (p.flags & NMG_F_OBJECT_LEVELS) {
    unsigned long long* lv = reinterpret_cast<unsigned long long*>(
        p.sum64 + 2 * kGlobalSums + uint64_t(p.nb_entries) * 4 + (uint64_t(e) * 2 + access) * kLevelWords);
    if (lvl & LVL_NA) atomicAdd(lv, 1ull);
    for (int g = 0; g < 9; g++) {
      if (!(lvl & level_mask(g))) continue;
      int bucket = (lvl & LVL_HIT) ? g : ((lvl & LVL_MISS) ? 9 + g : -1);
      if (bucket < 0) continue;
      atomicAdd(lv + 1 + 2 * bucket, 1ull);
      if (w) atomicAdd(lv + 2 + 2 * bucket, (unsigned long long)w);
    }
  }
}

// ---------------------------------------------------------------------------
// per-workgroup aggregation state: flush to global memory and clear, slot by
// slot (each thread owns the slots it flushes; callers fence with barriers)

template <int MODE>
__device__ __forceinline__ void flush_objects(Params& p, WgCounters& wc, int tid, uint32_t a) {
  const bool write = !(p.flags & kDbgNoFlush);
  const int n = (MODE & kModeDenseObj) ? (int)p.nb_entries : (int)kObjSlots;
  for (int i = tid; i < n; i += kWG) {
    const uint32_t e = (MODE & kModeDenseObj) ? (uint32_t)i : wc.okey[i];
    if ((MODE & kModeDenseObj) ? wc.owt[i] == 0 : e == kEmpty32) continue;
    const uint64_t cnt = wc.owt[i] >> kPackShift;
    const uint64_t wt = wc.owt[i] & ((1ull << kPackShift) - 1);
    if (write && !(MODE & kModeDenseObj) && p.tlog && tlog_append(p, wc, e, a, (uint32_t)cnt, wt, wc.ofirst[i])) {
      // logged
    } else if (write && !(MODE & kModeDenseObj) && p.pk64) {
      atomicAdd(p.pk64 + uint64_t(a) * p.nb_entries + e, (cnt << p.pk_shift) | wt);
      atomicMin(reinterpret_cast<unsigned long long*>(p.min64 + 36 + e), wc.ofirst[i]);
    } else if (write) {
      atomicAdd(reinterpret_cast<unsigned long long*>(p.sum64 + objcw_index(e, a, 0, p.nb_entries)),
                (unsigned long long)cnt);
      if (wt)
        atomicAdd(reinterpret_cast<unsigned long long*>(p.sum64 + objcw_index(e, a, 1, p.nb_entries)),
                  (unsigned long long)wt);
      unsigned long long* fp = reinterpret_cast<unsigned long long*>(p.min64 + 36 + e);
      atomicMin(fp, wc.ofirst[i]);  // no read first: a returning load would stall the flush
    }
    wc.okey[i] = kEmpty32;
    wc.ofirst[i] = kEmpty64;
    wc.owt[i] = 0;
  }
}

template <int MODE>
__device__ __forceinline__ void flush_pages(Params& p, WgCounters& wc, int tid, uint32_t th) {
  const bool write = !(p.flags & kDbgNoFlush);
  unsigned int* hrow = p.hist + uint64_t(th) * p.hist_cells;
  if (MODE & kModeDensePage) {  // cells in order: consecutive lanes add to consecutive words
    const uint32_t nw = (uint32_t)(p.hist_cells + 1) / 2;
    for (uint32_t i = tid; i < nw; i += kWG) {
      const uint32_t v = wc.pdense[i];
      if (!v) continue;
      if (write) {
        if (v & 0xffffu) atomicAdd(hrow + 2 * i, v & 0xffffu);
        if (v >> 16) atomicAdd(hrow + 2 * i + 1, v >> 16);
      }
      wc.pdense[i] = 0;
    }
    return;
  }
  unsigned int* pkey = reinterpret_cast<unsigned int*>(wc.pkey4);
  for (int i = tid; i < (int)kPageSlots; i += kWG) {
    const uint32_t cell = pkey[i];
    if (cell == kEmpty32) continue;
    if (write) atomicAdd(hrow + cell, wc.pcnt[i]);
    pkey[i] = kEmpty32;
    wc.pcnt[i] = 0;
  }
}

// global mem_counters[a] of the stream (after the lanes were drained)
__device__ __forceinline__ void flush_sums(Params& p, WgCounters& wc, int tid, uint32_t a) {
  const bool write = !(p.flags & kDbgNoFlush);
  if (tid < (int)kGlobalSums) {
    if (write && wc.sums[tid])
      atomicAdd(reinterpret_cast<unsigned long long*>(p.sum64 + gsum_index(a, tid)), wc.sums[tid]);
  }
  if (tid < 18) {
    if (write && wc.sums[3 + 2 * tid]) {
      atomicMin(reinterpret_cast<unsigned long long*>(p.min64 + a * 18 + tid), wc.mins[tid]);
      atomicMax(reinterpret_cast<unsigned long long*>(p.max64 + a * 18 + tid), wc.maxs[tid]);
    }
  }
  // (cleared after a barrier: sums[3 + 2 * tid] is read by other threads above)
}

__device__ __forceinline__ void clear_sums(WgCounters& wc, int tid) {
  if (tid < (int)kGlobalSums) wc.sums[tid] = 0;
  if (tid < 18) {
    wc.mins[tid] = ~0ull;  // INIT_COUNTER: min = UINT64_MAX (mem_analyzer.c:415-420)
    wc.maxs[tid] = 0;
  }
}

template <int MODE>
__device__ __forceinline__ void clear_state(WgCounters& wc, int tid) {
  clear_sums(wc, tid);
  for (int i = tid; i < (int)kObjSlots; i += kWG) {
    wc.okey[i] = kEmpty32;
    wc.ofirst[i] = kEmpty64;
    wc.owt[i] = 0;
  }
  if (MODE & kModeDensePage) {
    for (int i = tid; i < (int)(kDensePageCells / 2); i += kWG) wc.pdense[i] = 0;
  } else {
    for (int i = tid; i < (int)kPageSlots; i += kWG) {
      reinterpret_cast<unsigned int*>(wc.pkey4)[i] = kEmpty32;
      wc.pcnt[i] = 0;
    }
  }
}

// ---------------------------------------------------------------------------
// the attribution kernel
//
// One 1024-thread workgroup per CU (LDS: fences 8 KiB, node records 40 KiB,
// object table 48 KiB, page table 56 KiB, slow-path list 4 KiB), persistent
// over a byte-balanced range of the stream-sorted buffer list.  A window is
// 1024 stride slots of 40 B, one per lane, loaded straight into registers;
// the next window (of this buffer or the next one) is issued before the
// current one is processed.  One barrier per window: it publishes the window's
// "irregular" bit through rotating flag words.
// One lane's stride slot in window (cur of d0) [+ head of d1 when d1 is the
// next buffer of the same stream].
struct WinLane {
  uint32_t pos;     // slot offset within its buffer (buffers are < 4 GiB)
  uint32_t n0, n1;  // slots in d0 / in d1 (uniform)
  bool in1;         // the slot is in d1
  bool cand;        // this lane has a slot
};

__device__ __forceinline__ WinLane win_lane(int tid, uint32_t cur, const BufDesc& d0, const BufDesc& d1, bool has1) {
  WinLane w;
  const uint32_t left = d0.len - cur;
  w.n0 = min(left / kRecBytes + (left % kRecBytes != 0), (uint32_t)kWG);
  w.n1 = 0;
  if (has1 && w.n0 < (uint32_t)kWG && d1.access == d0.access && d1.thread_rank == d0.thread_rank)
    w.n1 = min(d1.len / kRecBytes + (d1.len % kRecBytes != 0), (uint32_t)kWG - w.n0);
  w.in1 = (uint32_t)tid >= w.n0;
  w.cand = (uint32_t)tid < w.n0 + w.n1;
  w.pos = w.in1 ? (uint32_t(tid) - w.n0) * kRecBytes : cur + uint32_t(tid) * kRecBytes;
  return w;
}

__device__ __forceinline__ void load_slot(const Params& p, const WinLane& w, const BufDesc& d0, const BufDesc& d1,
                                          RawRec& r) {
  const uint64_t off = w.in1 ? d1.offset : d0.offset;
  const uint32_t len = w.cand ? (w.in1 ? d1.len : d0.len) : 0;
  load_rec(p.data + off, w.pos, len, r);
}

template <bool TIMING, int MODE>
__global__ __launch_bounds__(kWG, 1) void attribute_kernel(Params p) {
  __shared__ uint4 s_tab[kTabBytes / 16];  // lookup structure (layouts at kTabBytes)
  __shared__ uint32_t s_list[kMaxList];
  __shared__ WgCounters wc;
  __shared__ uint32_t s_flags[3], s_nlist, s_next, s_err, s_nfound;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  uint64_t* const s_fences = reinterpret_cast<uint64_t*>(s_tab);
  uint4* const s_nodes = s_tab + (kLdsNodes + 1) / 2;                    // after 8 KiB of keys
  uint2* const s_ninfo = reinterpret_cast<uint2*>(s_tab + (kLdsNodes + 1) * 5 / 2);  // after 40 KiB
  uint8_t* const s_shift = reinterpret_cast<uint8_t*>(s_tab + (kMaxFences + 1) / 2);  // after 32 KiB
  if (!(MODE & kModeLarge)) {
    const uint32_t n = 1u << p.elevels;
    for (uint32_t i = tid; i < n; i += kWG) s_fences[i] = p.efences[i];
    for (uint32_t i = 1 + tid; i < n; i += kWG) {
      const uint4* q = reinterpret_cast<const uint4*>(p.enodes + i);
      const uint4 a = q[0], b = q[1], c = q[2], d = q[3];
      s_nodes[2 * i] = a;
      s_nodes[2 * i + 1] = b;
      s_ninfo[i] = make_uint2(c.y == 0 ? c.x : kEmpty32, c.w | (d.x > 1 ? 0x80000000u : 0u));
    }
  } else if (p.nb_keys) {
    for (uint32_t i = tid; i <= kMaxFences; i += kWG) s_fences[i] = p.ffences[i];
    for (uint32_t i = tid; i < p.nb_fences; i += kWG) s_shift[i] = p.fshift[i];
  }
  clear_state<MODE>(wc, tid);
  constexpr bool kLog = !(MODE & kModeDenseObj);  // the long-tail log serves the hashed object mode
  if (kLog && p.tlog)
    for (uint32_t i = tid; i < kLogParts; i += kWG) wc.tcur[i] = 0;
  if (tid < 3) s_flags[tid] = 0;
  lds_sync();
  const Lookup L{s_fences, s_nodes, s_ninfo, s_shift};

  // A window is (idx, cur): up to kWG stride slots from byte `cur` of buffer
  // idx; when that buffer ends inside the window and the next buffer belongs
  // to the same stream, the remaining lanes take the head of the next buffer
  // (no partly idle window at every buffer end).
  const uint32_t r0 = p.ranges[blockIdx.x], r1 = p.ranges[blockIdx.x + 1];
  if (r0 >= r1) {
    if (kLog && p.tlog)
      for (uint32_t i = tid; i < p.tlog_parts; i += kWG) p.tlog_cnt[uint64_t(blockIdx.x) * p.tlog_parts + i] = 0;
    return;
  }
  uint32_t idx = r0;
  uint32_t cur = 0;  // byte cursor, as `cur_cpt` in __analyze_buffer (mem_sampling.c:836)
  BufDesc d0 = p.sbufs[idx];
  BufDesc d1 = idx + 1 < r1 ? p.sbufs[idx + 1] : d0;
  bool has1 = idx + 1 < r1;
  uint32_t cur_access = d0.access, cur_thread = d0.thread_rank;
  RawRec nx;
  {
    const WinLane wl = win_lane(tid, 0, d0, d1, has1);
    load_slot(p, wl, d0, d1, nx);
  }
  LaneAcc acc;
  lane_acc_clear(acc);
  uint32_t win = 0, acc_windows = 0, last_flush = 0;
  uint32_t ns0 = 0, nf0 = 0, ns1 = 0, nf1 = 0;  // per-buffer tallies: buffer idx, idx + 1
  // this wave's matched samples; Params::found gets one add per workgroup at
  // the end (an add per buffer from every wave, all on that one word, made
  // the kernel 3.4x slower at configs[1])
  uint32_t nfound = 0;
  if (tid == 0) s_nfound = 0;  // (read after the loop's barriers)
  uint64_t tacc[4] = {0, 0, 0, 0}, t_start = 0, t0 = 0, t1 = 0;
  if (TIMING) t_start = t0 = stamp();
  constexpr bool kSpec = (MODE & kModeLarge) && !(MODE & kModeDenseObj);
  SubTimer st;
  for (int k = 0; k < 7; k++) st.acc[k] = 0;
  st.last = 0;
  SpecDir sp;
  sp.on = false;
  sp.idx = 0;
  sp.de = make_uint2(0, 0);

  while (true) {
    const WinLane wl = win_lane(tid, cur, d0, d1, has1);
    const Rec r = decode_rec(nx, wl.pos);
    // ---- fast-path check: every 40 B stride slot holds a whole 40 B record
    const uint32_t wlen = wl.in1 ? d1.len : d0.len;
    const bool bad = (cur & 7) != 0 || (wl.cand && (uint64_t(wl.pos) + kRecBytes > wlen || (r.hdr >> 48) != kRecBytes));
    const uint64_t badm = __ballot(bad);
    if (TIMING) {
      t1 = stamp();
      tacc[0] += t1 - t0;
      t0 = t1;
    }
    // (Dropping this barrier -- each wave deciding from its own slots, exact
    // only on pure 40 B SAMPLE streams -- was timed as an upper bound for a
    // barrier-free protocol: c2 -7.6 %, 1M intervals +6 %: not worth one.)
    if (badm && lane == 0) atomicOr(&s_flags[win % 3], 1u);
    lds_sync();
    // (LDS broadcasts are made wave-uniform explicitly: the branches below
    // hold barriers and steer the scalar loop state)
    const uint32_t f = __builtin_amdgcn_readfirstlane(s_flags[win % 3]);
    sp.on = !(f & 1);  // a fast-path window: each lane's record is the one its spec was computed for
    if (tid == 0) s_flags[(win + 2) % 3] = 0;  // last read before the previous barrier
    win++;
    if (TIMING) {
      t1 = stamp();
      tacc[1] += t1 - t0;
      t0 = t1;
    }
    uint32_t nidx = idx;
    uint64_t ncur;
    // the record this lane processes in this window
    Rec rec = r;
    bool valid;
    bool rin1;  // the lane's record is in d1
    uint32_t roff;
    bool shortrec = false;  // a SAMPLE record shorter than 40 B (slow path only)
    if (!(f & 1)) {
      valid = wl.cand && uint32_t(r.hdr) == kSampleType;
      rin1 = wl.in1;
      roff = wl.pos;
      // ---- fast path: one record per lane
      if (wl.n1) {
        nidx = idx + 1;
        ncur = uint64_t(wl.n1) * kRecBytes;
        if (ncur >= d1.len) {
          nidx = idx + 2;
          ncur = 0;
        }
      } else {
        ncur = cur + uint64_t(wl.n0) * kRecBytes;
        if (ncur >= d0.len) {
          nidx = idx + 1;
          ncur = 0;
        }
      }
    } else {
      // ---- slow path (buffer idx only): wave 0 follows the header chain from
      // global memory, 64 stride slots per step (a run of regular 40 B records
      // is taken in one step, an irregular record is handled alone), listing
      // SAMPLE offsets; then every lane processes one listed record
      const uint8_t* base = p.data + d0.offset;
      const uint64_t len = d0.len;
      if (tid < 64) {
        uint64_t q0 = cur;
        uint32_t n = 0, err = 0;
        const uint64_t lim = min(uint64_t(cur) + kWinBytes, len);
        while (q0 < lim && n + 65 <= kMaxList) {
          const uint64_t q = q0 + uint64_t(lane) * kRecBytes;
          const uint64_t hdr = (q + 8 <= len) ? *reinterpret_cast<const uint64_t*>(base + q) : 0;
          const bool reg = q < lim && q + kRecBytes <= len && (hdr >> 48) == kRecBytes;
          const uint64_t rm = __ballot(reg);
          const uint32_t run = ~rm ? (uint32_t)__builtin_ctzll(~rm) : 64u;
          const bool smp = (uint32_t)lane < run && uint32_t(hdr) == kSampleType;
          const uint64_t sm = __ballot(smp);
          if (smp) s_list[n + (uint32_t)__popcll(sm & ((1ull << lane) - 1))] = (uint32_t)q;
          n += (uint32_t)__popcll(sm);
          q0 += uint64_t(run) * kRecBytes;
          if (run == 64 || q0 >= lim) continue;
          // record at q0 (lane `run`'s slot) is not a whole 40 B record
          if (q0 + 8 > len) { err = kErrTruncated; break; }
          const uint64_t h = (uint64_t)__shfl(hdr, (int)run, 64);
          const uint32_t size = uint32_t(h >> 48);
          if (size == 0) { err = kErrZeroSize; break; }  // mem_sampling.c:857-860
          if (size & 7) { err = kErrUnaligned; break; }  // perf records are 8-byte multiples
          if (uint32_t(h) == kSampleType) {
            if (q0 + kRecBytes > len || q0 + size > len) { err = kErrTruncated; break; }
            // (offsets are 8-aligned: bit 0 marks a SAMPLE shorter than 40 B,
            // which the reference's byte cursor accepts; it stays out of the
            // packed long-tail counters, whose bound counts 40 B records)
            if (lane == 0) s_list[n] = (uint32_t)q0 | (size < kRecBytes ? 1u : 0u);
            n++;
          }
          q0 += size;  // non-SAMPLE records are skipped by their size (:918)
        }
        if (lane == 0) {
          if (err) set_error(p, d0.seq, (uint32_t)q0, err);
          s_err = err;
          s_nlist = n;
          s_next = (uint32_t)min(q0, len);
        }
      }
      lds_sync();
      const uint32_t n = __builtin_amdgcn_readfirstlane(s_nlist);
      const uint32_t serr = __builtin_amdgcn_readfirstlane(s_err);
      ncur = serr ? len : __builtin_amdgcn_readfirstlane(s_next);  // the reference aborts on an error: stop this buffer
      if (ncur >= len) {
        nidx = idx + 1;
        ncur = 0;
      }
      valid = (uint32_t)tid < n;
      roff = valid ? s_list[tid] : 0;
      shortrec = (roff & 1u) != 0;
      roff &= ~1u;
      rin1 = false;
      RawRec rr;
      load_rec(base, roff, valid ? len : 0, rr);
      rec = decode_rec(rr, roff);
    }

    // ---- descriptors of the next window, and its loads (issued before this
    // window's records are processed)
    BufDesc nd0 = d0, nd1 = d1;
    if (nidx == idx + 1) {
      nd0 = d1;
      if (nidx + 1 < r1) nd1 = p.sbufs[nidx + 1];
    } else if (nidx == idx + 2) {
      if (nidx < r1) nd0 = p.sbufs[nidx];
      if (nidx + 1 < r1) nd1 = p.sbufs[nidx + 1];
    }
    const bool nhas1 = nidx + 1 < r1;
    uint32_t npos = 0;
    bool ncand = false;
    if (nidx < r1) {
      const WinLane nl = win_lane(tid, (uint32_t)ncur, nd0, nd1, nhas1);
      load_slot(p, nl, nd0, nd1, nx);
      npos = nl.pos;
      ncand = nl.cand;
    }

    if (TIMING) st.last = stamp();
    if (TIMING && tid == 0 && win <= 4) {
      unsigned long long* o = p.dbg + uint64_t(blockIdx.x) * (kWG / 64) * kTimingWords + 8 + 2 * (win - 1);
      o[0] = (uint64_t(idx) << 40) | cur;
      o[1] = uint64_t(wl.n0) | (uint64_t(wl.n1) << 11) | (uint64_t(f) << 22) | (uint64_t(nidx) << 24) |
             (uint64_t((uint32_t)ncur) << 32);
    }
    uint64_t vm = 0, fm = 0;
    if (!(p.flags & kDbgLoadOnly))
      process_sample<MODE, TIMING>(p, wc, acc, L, st, valid, shortrec, rec.ts, rec.addr, rec.w, rec.dsrc, d0.access, d0.thread_rank, d0, d1, rin1,
                           roff, vm, fm, sp);
    sub_stamp<TIMING>(st, 4);
    if (kSpec && (p.flags & NMG_F_MATCH_SAMPLES)) {
      // start the next window's lookup: its record (loaded above, arrived
      // during this window's lookups) -> fence node -> directory slot load,
      // in flight across the flush and the barrier.  Used when the record
      // this lane processes next has the same address (fast-path windows).
      sp.idx = 0;
      if (nidx < r1 && ncand) {
        const uint64_t saddr = decode_rec(nx, npos).addr;
        sp.idx = fence_node(L.fences, saddr);
        const uint2* ds = dir_slot(p, L.fences, L.shift, saddr, sp.idx);
        if (ds) sp.de = *ds;
      }
      sub_stamp<TIMING>(st, 5);
    }
    {
      // lanes of this wave in buffer idx + 1 (tid >= n0)
      const uint32_t w0 = uint32_t(tid) & ~63u;
      const uint64_t m1 = ((f & 1) || wl.n0 >= w0 + 64) ? 0ull : (wl.n0 <= w0 ? ~0ull : (~0ull << (wl.n0 - w0)));
      ns0 += (uint32_t)__popcll(vm & ~m1);
      nf0 += (uint32_t)__popcll(fm & ~m1);
      ns1 += (uint32_t)__popcll(vm & m1);
      nf1 += (uint32_t)__popcll(fm & m1);
    }
    if (TIMING) {
      t1 = stamp();
      tacc[2] += t1 - t0;
      t0 = t1;
      st.acc[6] += t1 - st.last;
    }
    // end of the stream run (or of this workgroup's range): publish the
    // stream's counters; tables over their fill threshold (as of this
    // window's barrier) are flushed here too -- the single flush site
    const bool stream_end = nidx != idx && (nidx >= r1 || nd0.access != cur_access || nd0.thread_rank != cur_thread);
    if (++acc_windows == kDrainWindows || stream_end) {  // keep the per-lane u32 sums bounded
      lane_acc_drain(acc, wc.sums, lane);
      acc_windows = 0;
    }
    if (nidx != idx) {
      // buffer idx (and idx + 1 when skipped over) done: sample / match
      // tallies (mem_sampling.c:921-926)
      if (lane == 0) {
        if (ns0) atomicAdd(p.bufcnt + d0.pad, ns0);
        if (nf0) atomicAdd(p.bufcnt + p.nb_bufs + d0.pad, nf0);
        nfound += nf0;
        if (nidx == idx + 2) {
          if (ns1) atomicAdd(p.bufcnt + d1.pad, ns1);
          if (nf1) atomicAdd(p.bufcnt + p.nb_bufs + d1.pad, nf1);
          nfound += nf1;
        }
      }
      if (nidx == idx + 1) {
        ns0 = ns1;
        nf0 = nf1;
      } else {
        ns0 = nf0 = 0;
      }
      ns1 = nf1 = 0;
    }
    const uint32_t cadence = (MODE & (kModeDensePage | kModeDenseObj)) ? kDensePageWindows : kTableWindows;
    if (stream_end || win - last_flush >= cadence) {
      lds_sync();  // every insert and drain of this window is done
      if (stream_end) flush_sums(p, wc, tid, cur_access);
      flush_objects<MODE>(p, wc, tid, cur_access);
      flush_pages<MODE>(p, wc, tid, cur_thread);
      last_flush = win;
      lds_sync();
      if (stream_end) {
        clear_sums(wc, tid);  // (sums are next written after the next window's barrier)
        cur_access = nd0.access;
        cur_thread = nd0.thread_rank;
      }
    }
    idx = nidx;
    cur = (uint32_t)ncur;
    d0 = nd0;
    d1 = nd1;
    has1 = nhas1;
    if (TIMING) {
      t1 = stamp();
      tacc[3] += t1 - t0;
      t0 = t1;
    }
    if (idx >= r1) break;  // the loop's only exit, after the state update
  }
  if (lane == 0 && nfound) atomicAdd(&s_nfound, nfound);
  lds_sync();
  if (tid == 0 && s_nfound) atomicAdd(p.found, (unsigned long long)s_nfound);
  if (kLog && p.tlog) {  // the sub-logs' fill (every append of this workgroup is done)
    lds_sync();
    if (kLog && p.tlog)
      for (uint32_t i = tid; i < p.tlog_parts; i += kWG)
        p.tlog_cnt[uint64_t(blockIdx.x) * p.tlog_parts + i] = min(wc.tcur[i], p.tlog_cap);
  }
  if (TIMING && lane == 0) {
    unsigned long long* o = p.dbg + (uint64_t(blockIdx.x) * (kWG / 64) + tid / 64) * kTimingWords;
    for (int k = 0; k < 4; k++) o[k] = tacc[k];
    for (int k = 0; k < 7; k++) o[16 + k] = st.acc[k];
    o[4] = stamp() - t_start;
    o[5] = win;
  }
}

// Sums the long-tail log of one attribution launch: workgroup `part` owns the
// entries [part << rshift, (part + 1) << rshift), reads that range's sub-log
// of every attribution workgroup, adds counts / weights and takes the first
// ordinal in LDS, then updates sum64 / min64 with plain read-modify-writes
// (no other writer of those words is running).  Folds the packed counters of
// the range too.
__global__ __launch_bounds__(1024, 1) void tlog_reduce_kernel(TlogParams r) {
  __shared__ uint32_t s_cnt[2][kLogChunk];
  __shared__ unsigned long long s_wt[2][kLogChunk];
  __shared__ unsigned long long s_ord[kLogChunk];
  __shared__ uint32_t s_pre[kLogMaxGrid];  // slots of each source workgroup's sub-log
  const uint32_t part = blockIdx.x, tid = threadIdx.x;
  for (uint32_t w = tid; w < r.grid; w += 1024) s_pre[w] = r.tlog_cnt[uint64_t(w) * r.parts + part];
  __syncthreads();
  const uint64_t e0 = uint64_t(part) << r.rshift;
  const uint64_t e1 = min(e0 + (1ull << r.rshift), (uint64_t)r.nb_entries);
  for (uint64_t base = e0; base < e1; base += kLogChunk) {
    const uint32_t n = (uint32_t)min((uint64_t)kLogChunk, e1 - base);
    for (uint32_t j = tid; j < n; j += 1024) {
      s_cnt[0][j] = s_cnt[1][j] = 0;
      s_wt[0][j] = s_wt[1][j] = 0;
      s_ord[j] = ~0ull;
    }
    __syncthreads();
    // each wave walks whole source sub-logs (contiguous slots), kU slots per
    // lane in flight; sub-logs are about equally long (byte-balanced schedule)
    constexpr int kU = 4;
    const uint32_t wave = tid >> 6, lane = tid & 63;
    for (uint32_t w = wave; w < r.grid; w += 1024 / 64) {
      const uint32_t cnt = s_pre[w];
      const uint4* src = r.tlog + (uint64_t(w) * r.parts + part) * r.cap;
      for (uint32_t i0 = lane; i0 < cnt; i0 += kU * 64) {
        uint4 sv[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
          const uint32_t i = i0 + u * 64;
          sv[u] = i < cnt ? src[i] : make_uint4(~0u, 0, kTlogCont, 0);  // (no slot: skipped like a continuation)
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
          const uint4 v = sv[u];
          if (v.z == kTlogCont) continue;  // second slot of a two-slot record (read with its head)
          const uint32_t e = v.x & 0x7fffffffu, a = v.x >> 31;
          const uint64_t j = e - base;
          if (e < base || j >= n) continue;
          uint32_t c = 1;
          uint64_t wt = v.y, ord = (uint64_t(v.w) << 32) | v.z;
          if (v.z == kTlogHead) {
            const uint4 q = src[i0 + u * 64 + 1];
            c = v.y;
            wt = (uint64_t(q.y) << 32) | q.x;
            ord = (uint64_t(v.w) << 32) | q.w;
          }
          atomicAdd(&s_cnt[a][j], c);
          if (wt) atomicAdd(&s_wt[a][j], (unsigned long long)wt);
          atomicMin(&s_ord[j], (unsigned long long)ord);
        }
      }
    }
    __syncthreads();
    // every global word of kU entries loaded before any is updated (the
    // read-modify-writes would otherwise wait on one load at a time)
    for (uint32_t j0 = tid; j0 < n; j0 += kU * 1024) {
      uint64_t gc[kU][2], gw[kU][2], pv[kU][2], gm[kU];
#pragma unroll
      for (int u = 0; u < kU; u++) {
        const uint32_t j = j0 + u * 1024;
        if (j >= n) continue;
        const uint64_t e = base + j;
#pragma unroll
        for (uint32_t a = 0; a < 2; a++) {
          gc[u][a] = r.sum64[objcw_index(e, a, 0, r.nb_entries)];
          gw[u][a] = r.sum64[objcw_index(e, a, 1, r.nb_entries)];
          pv[u][a] = r.pk64 ? r.pk64[uint64_t(a) * r.nb_entries + e] : 0;
        }
        gm[u] = r.min64[36 + e];
      }
#pragma unroll
      for (int u = 0; u < kU; u++) {
        const uint32_t j = j0 + u * 1024;
        if (j >= n) continue;
        const uint64_t e = base + j;
#pragma unroll
        for (uint32_t a = 0; a < 2; a++) {
          uint64_t c = s_cnt[a][j], w = s_wt[a][j];
          const uint64_t v = pv[u][a];
          if (v) {
            c += v >> r.pk_shift;
            w += v & ((1ull << r.pk_shift) - 1);
            r.pk64[uint64_t(a) * r.nb_entries + e] = 0;
          }
          if (c) r.sum64[objcw_index(e, a, 0, r.nb_entries)] = gc[u][a] + c;
          if (w) r.sum64[objcw_index(e, a, 1, r.nb_entries)] = gw[u][a] + w;
        }
        if (s_ord[j] < gm[u]) r.min64[36 + e] = s_ord[j];
      }
    }
    __syncthreads();
  }
}

// Adds the launch's packed long-tail object counters into sum64 and clears
// them (same stream, after attribute_kernel).
__global__ __launch_bounds__(256) void unpack_kernel(uint64_t* sum64, unsigned long long* pk64, uint32_t nb_entries,
                                                     uint32_t shift) {
  const uint64_t n = 2ull * nb_entries;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint64_t v = pk64[i];
    if (!v) continue;
    const uint32_t a = i >= nb_entries;
    const uint64_t e = i - uint64_t(a) * nb_entries;
    sum64[objcw_index(e, a, 0, nb_entries)] += v >> shift;
    sum64[objcw_index(e, a, 1, nb_entries)] += v & ((1ull << shift) - 1);
    pk64[i] = 0;
  }
}

// One launch re-initialises every counter array (INIT_COUNTER semantics:
// sums and maxes 0, mins and first-match ordinals UINT64_MAX; sparse keys empty).
__global__ __launch_bounds__(256) void reset_kernel(ResetParams r) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  const uint64_t i0 = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  for (uint64_t i = i0; i < r.n_hist16; i += stride) r.hist[i] = make_uint4(0, 0, 0, 0);
  for (uint64_t i = i0; i < r.n_sum64; i += stride) r.sum64[i] = 0;
  for (uint64_t i = i0; i < r.n_min64; i += stride) r.min64[i] = ~0ull;
  for (uint64_t i = i0; i < r.n_max64; i += stride) r.max64[i] = 0;
  // the sparse table is cleared only when something was inserted since the
  // last reset (it is large, and the [stack] range it serves never matches, Q4)
  if (i0 == 0 && r.sparse_clear) *r.sparse_clear = 0u;
  const uint64_t scap = (r.sparse_read && *r.sparse_read) ? r.sparse_cap : 0;
  for (uint64_t i = i0; i < scap; i += stride) {
    r.sparse_keys[i] = ~0ull;
    r.sparse_vals[i] = 0;
  }
  for (uint64_t i = i0; i < r.n_bufcnt; i += stride) r.bufcnt[i] = 0;
  if (i0 == 0 && r.found) *r.found = 0;
}

// Multi-GPU merge when the shards share one device: dst op= src over n words
// (op 0: u64 sum, 1: u64 min, 2: u64 max, 3: u32 sum).
__global__ __launch_bounds__(256) void merge_kernel(void* dst, const void* src, uint64_t n, int op) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (op == 3) {
      reinterpret_cast<uint32_t*>(dst)[i] += reinterpret_cast<const uint32_t*>(src)[i];
    } else {
      uint64_t& d = reinterpret_cast<uint64_t*>(dst)[i];
      const uint64_t v = reinterpret_cast<const uint64_t*>(src)[i];
      d = op == 0 ? d + v : (op == 1 ? min(d, v) : max(d, v));
    }
  }
}

// Packed page histogram for the multi-GPU merge (nmg_hist_pack): cells of at
// most `thr` as bytes (4 per thread, one 16 B load), larger ones to the
// overflow list as (cell << 32 | count), in cell order.  Two passes over
// contiguous per-workgroup ranges, no shared counter: hist_count_kernel
// counts each range's large cells, hist_pack_kernel takes its range's offset
// as the sum of the earlier ranges' counts (one reservation per wave on a
// shared word had serialised ~10^5 atomics: 0.8 ms at the c4 shard).
constexpr uint32_t kPackGrid = 1024, kPackWG = 256;

__device__ __forceinline__ uint32_t big_cells(uint4 v, uint32_t thr) {
  return (v.x > thr) + (v.y > thr) + (v.z > thr) + (v.w > thr);
}
// cells 4i .. 4i + 3 (those past ncells read as 0; the last, partial quad by
// single loads)
__device__ __forceinline__ uint4 load_quad(const uint32_t* hist, uint64_t i, uint64_t ncells) {
  if (4 * i + 3 < ncells) return reinterpret_cast<const uint4*>(hist)[i];
  uint32_t c[4];
#pragma unroll
  for (int k = 0; k < 4; k++) c[k] = 4 * i + k < ncells ? hist[4 * i + k] : 0u;
  return make_uint4(c[0], c[1], c[2], c[3]);
}

__global__ __launch_bounds__(kPackWG) void hist_count_kernel(const uint32_t* hist, uint64_t ncells, uint32_t thr,
                                                             uint32_t* wgcnt) {
  const uint64_t n4 = (ncells + 3) / 4;
  __shared__ uint32_t s_sum[kPackWG / 64];
  const uint64_t per = (n4 + kPackGrid - 1) / kPackGrid, i0 = uint64_t(blockIdx.x) * per;
  const uint64_t i1 = min(i0 + per, n4);
  uint32_t nbig = 0;
  for (uint64_t i = i0 + threadIdx.x; i < i1; i += kPackWG) nbig += big_cells(load_quad(hist, i, ncells), thr);
  nbig = wave_sum_u32(nbig);
  if ((threadIdx.x & 63) == 0) s_sum[threadIdx.x >> 6] = nbig;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t w = 0; w < kPackWG / 64; w++) t += s_sum[w];
    wgcnt[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kPackWG) void hist_pack_kernel(const uint32_t* hist, uint64_t ncells, uint32_t thr,
                                                            uint8_t* u8, unsigned long long* ovf, uint64_t cap,
                                                            const uint32_t* wgcnt, unsigned long long* cnt) {
  const uint64_t n4 = (ncells + 3) / 4;
  __shared__ uint32_t s_w[kPackWG / 64];
  __shared__ unsigned long long s_base;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t per = (n4 + kPackGrid - 1) / kPackGrid, i0 = uint64_t(blockIdx.x) * per;
  const uint64_t i1 = min(i0 + per, n4);
  // this range's first overflow slot: the earlier ranges' counts
  uint32_t pre = 0;
  for (uint32_t w = tid; w < blockIdx.x; w += kPackWG) pre += wgcnt[w];
  pre = wave_sum_u32(pre);
  if (lane == 0) s_w[wave] = pre;
  __syncthreads();
  if (tid == 0) {
    unsigned long long t = 0;
    for (uint32_t w = 0; w < kPackWG / 64; w++) t += s_w[w];
    s_base = t;
    if (blockIdx.x == gridDim.x - 1) *cnt = t + wgcnt[blockIdx.x];  // (the list's length)
  }
  __syncthreads();
  unsigned long long base = s_base;
  for (uint64_t j = i0; j < i1; j += kPackWG) {  // (uniform trip count: the scans below are workgroup-wide)
    const uint64_t i = j + tid;
    const uint4 v = i < i1 ? load_quad(hist, i, ncells) : make_uint4(0, 0, 0, 0);
    const uint32_t c[4] = {v.x, v.y, v.z, v.w};
    uint32_t packed = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) packed |= (c[k] <= thr ? c[k] : 0u) << (8 * k);
    if (i < i1) {
      if (4 * i + 3 < ncells) {
        reinterpret_cast<uint32_t*>(u8)[i] = packed;
      } else {  // (the partial last quad: the byte buffer holds ncells bytes)
        for (uint32_t k = 0; 4 * i + k < ncells; k++) u8[4 * i + k] = uint8_t(packed >> (8 * k));
      }
    }
    const uint32_t nbig = i < i1 ? big_cells(v, thr) : 0u;
    // workgroup-wide exclusive scan of nbig (cell order)
    const uint32_t inc = wave_incl_scan_u32(nbig);
    __syncthreads();  // (s_w of the previous iteration read by every wave)
    if (lane == 63) s_w[wave] = inc;
    __syncthreads();
    uint32_t wpre = 0, tot = 0;
    for (int w = 0; w < kPackWG / 64; w++) {
      wpre += w < wave ? s_w[w] : 0u;
      tot += s_w[w];
    }
    uint64_t slot = base + wpre + inc - nbig;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (c[k] <= thr) continue;
      if (slot < cap) ovf[slot] = ((unsigned long long)(4 * i + k) << 32) | c[k];
      slot++;
    }
    base += tot;
  }
}

// Packed per-object counters for the multi-GPU merge (nmg_objcw_pack): the
// four SoA rows [access][count, weight][E] of a sum64 image as u32 words where
// a value is below thr (a rank's share of 2^32, so that the sum over the ranks
// still fits), 0 there and a (row word, value) pair in the overflow list
// where it is not.  The list's order does not matter: unpack adds.
__global__ __launch_bounds__(256) void objcw_pack_kernel(const uint64_t* rows, uint64_t n, uint64_t thr,
                                                         uint32_t* u32, unsigned long long* ovf, uint64_t cap,
                                                         unsigned long long* cnt) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t v = rows[i];
    const bool big = v >= thr;
    u32[i] = big ? 0u : (uint32_t)v;
    if (big) {
      const unsigned long long k = atomicAdd(cnt, 1ull);
      if (k < cap) {
        ovf[2 * k] = i;
        ovf[2 * k + 1] = v;
      }
    }
  }
}

// nmg_objcw_unpack: the rows = the summed u32 words, then += every listed value
__global__ __launch_bounds__(256) void objcw_unpack_kernel(uint64_t* rows, uint64_t n, const uint32_t* u32) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) rows[i] = u32[i];
}

__global__ __launch_bounds__(256) void objcw_ovf_add_kernel(uint64_t* rows, uint64_t n, const unsigned long long* ovf,
                                                            uint64_t m, unsigned long long* bad) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t k = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; k < m; k += stride) {
    const uint64_t i = ovf[2 * k];
    if (i < n) atomicAdd(reinterpret_cast<unsigned long long*>(rows + i), ovf[2 * k + 1]);
    else atomicAdd(bad, 1ull);
  }
}

hipError_t launch_objcw_pack(hipStream_t s, const uint64_t* rows, uint64_t n, uint64_t thr, void* u32, void* ovf,
                             uint64_t cap, unsigned long long* cnt) {
  if (n) {
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(objcw_pack_kernel, dim3(grid), dim3(256), 0, s, rows, n, thr, reinterpret_cast<uint32_t*>(u32),
                       reinterpret_cast<unsigned long long*>(ovf), cap, cnt);
  }
  return hipGetLastError();
}

hipError_t launch_objcw_unpack(hipStream_t s, uint64_t* rows, uint64_t n, const void* u32, const void* ovf,
                               uint64_t m, unsigned long long* bad) {
  if (n) {
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(objcw_unpack_kernel, dim3(grid), dim3(256), 0, s, rows, n, reinterpret_cast<const uint32_t*>(u32));
  }
  if (m) {
    const uint32_t grid = (uint32_t)std::min<uint64_t>((m + 255) / 256, 1024);
    hipLaunchKernelGGL(objcw_ovf_add_kernel, dim3(grid), dim3(256), 0, s, rows, n,
                       reinterpret_cast<const unsigned long long*>(ovf), m, bad);
  }
  return hipGetLastError();
}

// nmg_get_object_counters: the per-object counts and weights from their four
// SoA rows (objcw_index: row access * 2 + w of E words) to [E][access][w],
// one 32 B record per entry (a single contiguous D2H)
__global__ __launch_bounds__(256) void objcw_aos_kernel(const uint64_t* soa, uint64_t E, uint4* aos) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t e = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < E; e += stride) {
    const uint64_t r0 = soa[e], r1 = soa[E + e], r2 = soa[2 * E + e], r3 = soa[3 * E + e];
    aos[2 * e] = make_uint4((uint32_t)r0, (uint32_t)(r0 >> 32), (uint32_t)r1, (uint32_t)(r1 >> 32));
    aos[2 * e + 1] = make_uint4((uint32_t)r2, (uint32_t)(r2 >> 32), (uint32_t)r3, (uint32_t)(r3 >> 32));
  }
}

hipError_t launch_objcw_aos(hipStream_t s, const uint64_t* soa, uint64_t E, void* aos) {
  if (E) {
    const uint32_t grid = (uint32_t)std::min<uint64_t>((E + 255) / 256, 4096);
    hipLaunchKernelGGL(objcw_aos_kernel, dim3(grid), dim3(256), 0, s, soa, E, reinterpret_cast<uint4*>(aos));
  }
  return hipGetLastError();
}

// nmg_hist_unpack: hist = summed bytes, then += every overflow entry
__global__ __launch_bounds__(256) void hist_unpack_kernel(uint32_t* hist, uint64_t ncells, const uint8_t* u8) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x, n4 = (ncells + 3) / 4;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n4; i += stride) {
    if (4 * i + 3 < ncells) {
      const uint32_t p = reinterpret_cast<const uint32_t*>(u8)[i];
      reinterpret_cast<uint4*>(hist)[i] = make_uint4(p & 0xffu, (p >> 8) & 0xffu, (p >> 16) & 0xffu, p >> 24);
    } else {
      for (uint64_t c = 4 * i; c < ncells; c++) hist[c] = u8[c];
    }
  }
}

__global__ __launch_bounds__(256) void hist_ovf_add_kernel(uint32_t* hist, uint64_t ncells,
                                                           const unsigned long long* ovf, uint64_t n,
                                                           unsigned long long* bad) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const unsigned long long e = ovf[i];
    const uint64_t cell = e >> 32;
    const uint32_t c = (uint32_t)e;
    if (!c) continue;  // (padding)
    if (cell < ncells) atomicAdd(hist + cell, c);
    else atomicAdd(bad, 1ull);
  }
}

// The sparse table's used slots as (key, count) pairs (order: any; the host
// sorts), one counter add per wave that holds one.
__global__ __launch_bounds__(256) void sparse_compact_kernel(const uint64_t* keys, const uint32_t* vals, uint64_t cap,
                                                             uint64_t* out, unsigned long long* cnt) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  const int lane = threadIdx.x & 63;
  for (uint64_t base = uint64_t(blockIdx.x) * blockDim.x; base < cap; base += stride) {
    const uint64_t i = base + threadIdx.x;
    const uint64_t key = i < cap ? keys[i] : ~0ull;
    const uint32_t v = i < cap ? vals[i] : 0u;
    const bool used = key != ~0ull && v != 0;
    const uint64_t m = __ballot(used);
    if (!m) continue;
    unsigned long long at = 0;
    if (lane == 0) at = atomicAdd(cnt, (unsigned long long)__popcll(m));
    at = __shfl(at, 0, 64);
    if (used) {
      const uint64_t slot = at + __popcll(m & ((1ull << lane) - 1));
      out[2 * slot] = key;
      out[2 * slot + 1] = v;
    }
  }
}

// nmg_sparse_import: (key, count) pairs into a cleared table, with
// sparse_add's hash and linear probing (n <= cap: every probe sequence ends)
__global__ __launch_bounds__(256) void sparse_insert_kernel(uint64_t* keys, uint32_t* vals, uint64_t mask,
                                                            const uint64_t* pairs, uint64_t n) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t key = pairs[2 * i];
    const uint32_t cnt = (uint32_t)pairs[2 * i + 1];
    uint64_t slot = ((key * 0x9E3779B97F4A7C15ull) >> 20) & mask;
    for (uint64_t probe = 0; probe <= mask; probe++) {
      const unsigned long long prev =
          atomicCAS(reinterpret_cast<unsigned long long*>(keys + slot), ~0ull, (unsigned long long)key);
      if (prev == ~0ull || prev == key) {
        atomicAdd(vals + slot, cnt);
        break;
      }
      slot = (slot + 1) & mask;
    }
  }
}

// ---------------------------------------------------------------------------
// launchers

typedef void (*AttributeKernel)(Params);

hipError_t launch_attribute(bool timing, int mode, uint32_t grid, hipStream_t s, const Params& p) {
  static const AttributeKernel k[2][8] = {
      {attribute_kernel<false, 0>, attribute_kernel<false, 1>, attribute_kernel<false, 2>, attribute_kernel<false, 3>,
       attribute_kernel<false, 4>, attribute_kernel<false, 5>, attribute_kernel<false, 6>, attribute_kernel<false, 7>},
      {attribute_kernel<true, 0>, attribute_kernel<true, 1>, attribute_kernel<true, 2>, attribute_kernel<true, 3>,
       attribute_kernel<true, 4>, attribute_kernel<true, 5>, attribute_kernel<true, 6>, attribute_kernel<true, 7>}};
  hipLaunchKernelGGL(k[timing ? 1 : 0][mode & 7], dim3(grid), dim3(kWG), 0, s, p);
  return hipGetLastError();
}

int attribute_blocks_per_cu() {
  int bpc = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, attribute_kernel<false, 0>, kWG, 0) != hipSuccess || bpc <= 0)
    bpc = 1;
  return bpc;
}

hipError_t launch_tlog_reduce(uint32_t grid, hipStream_t s, const TlogParams& r) {
  hipLaunchKernelGGL(tlog_reduce_kernel, dim3(grid), dim3(1024), 0, s, r);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Page-cell rows (the report's per-(entry, thread, page) counts): one wave per
// entry, its T x np cells walked thread-major in 64-cell steps; a ballot
// gives each non-zero cell its row.  Sparse entries (base == kHistSparse)
// count 0 here: the host adds their rows from the sparse table.

__global__ __launch_bounds__(256) void cells_count_kernel(const uint32_t* hist, uint64_t hist_cells, uint32_t T,
                                                          const uint64_t* base, const uint32_t* np, uint32_t E,
                                                          uint32_t* cnt) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x / 64);
  for (uint32_t e = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; e < E; e += nw) {
    const uint64_t b = base[e];
    uint32_t n = 0;
    if (b != ~0ull) {
      const uint32_t pg = np[e], tot = pg * T;
      for (uint32_t i0 = 0; i0 < tot; i0 += 64) {
        const uint32_t i = i0 + lane;
        const uint32_t th = i / pg, p = i - th * pg;
        const bool nz = i < tot && hist[uint64_t(th) * hist_cells + b + p] != 0;
        n += (uint32_t)__popcll(__ballot(nz));
      }
    }
    if (lane == 0) cnt[e] = n;
  }
}

__global__ __launch_bounds__(256) void cells_emit_kernel(const uint32_t* hist, uint64_t hist_cells, uint32_t T,
                                                         const uint64_t* base, const uint32_t* np, uint32_t E,
                                                         const uint64_t* off, uint4* rows) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * (blockDim.x / 64);
  for (uint32_t e = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; e < E; e += nw) {
    const uint64_t b = base[e];
    if (b == ~0ull) continue;
    const uint32_t pg = np[e], tot = pg * T;
    uint64_t o = off[e];
    for (uint32_t i0 = 0; i0 < tot; i0 += 64) {
      const uint32_t i = i0 + lane;
      const uint32_t th = i / pg, p = i - th * pg;
      const uint32_t v = i < tot ? hist[uint64_t(th) * hist_cells + b + p] : 0u;
      const uint64_t m = __ballot(v != 0);
      if (v) rows[o + __popcll(m & ((1ull << lane) - 1))] = make_uint4(e, th, p, v);
      o += (uint64_t)__popcll(m);
    }
  }
}

// The results snapshot's cell rows (nmg_results_begin) without a host round
// trip: the sparse table's compacted cells counted per entry, an exclusive
// scan of the per-entry counts into row offsets on the device, the sparse
// entries' offsets gathered, and the rows copied into mapped host memory by
// a kernel that reads their number on the device.
__global__ __launch_bounds__(256) void cells_sparse_count_kernel(const uint64_t* ck, const unsigned long long* n_ptr,
                                                                 const uint32_t* sent, uint32_t nsent,
                                                                 const uint64_t* base, uint32_t* cnt) {
  const uint64_t n = *n_ptr;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint64_t key = ck[2 * i];
    const uint32_t s = uint32_t(key >> 42);  // (sparse_key_idx)
    // (an entry's sparse cells count only where it has no dense cells, as cells_prepare)
    if (key != ~0ull && ck[2 * i + 1] && s < nsent && base[sent[s]] == ~0ull) atomicAdd(&cnt[sent[s]], 1u);
  }
}

constexpr uint32_t kScanItems = 16, kScanBlock = 256 * kScanItems;
__device__ __forceinline__ uint32_t scan_thread_sum(const uint32_t* in, uint64_t n, uint64_t i0) {
  uint32_t t = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; k++) t += i0 + k < n ? in[i0 + k] : 0u;
  return t;
}
// the block's exclusive prefix of per-thread values (256 threads) and its total
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t* s_w, uint64_t& total) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(x, o, 64);
    if ((int)lane >= o) x += y;
  }
  if (lane == 63) s_w[wave] = x;
  __syncthreads();
  uint64_t base = 0;
  total = 0;
  for (uint32_t w = 0; w < 4; w++) {
    if (w < wave) base += s_w[w];
    total += s_w[w];
  }
  __syncthreads();
  return base + x - v;
}
__global__ __launch_bounds__(256) void scan_sums_kernel(const uint32_t* in, uint64_t n, uint64_t* part) {
  __shared__ uint64_t s_w[4];
  const uint64_t i0 = uint64_t(blockIdx.x) * kScanBlock + threadIdx.x * kScanItems;
  uint64_t total;
  (void)block_excl_scan(scan_thread_sum(in, n, i0), s_w, total);
  if (threadIdx.x == 0) part[blockIdx.x] = total;
}
__global__ __launch_bounds__(256) void scan_parts_kernel(uint64_t* part, uint32_t nb) {
  __shared__ uint64_t s_w[4];
  uint64_t carry = 0;
  for (uint32_t b0 = 0; b0 < nb; b0 += 256) {
    const uint32_t b = b0 + threadIdx.x;
    const uint64_t v = b < nb ? part[b] : 0ull;
    uint64_t total;
    const uint64_t pre = block_excl_scan(v, s_w, total);
    if (b < nb) part[b] = carry + pre;
    carry += total;
  }
  if (threadIdx.x == 0) part[nb] = carry;
}
__global__ __launch_bounds__(256) void scan_apply_kernel(const uint32_t* in, uint64_t n, const uint64_t* part,
                                                         uint64_t* out) {
  __shared__ uint64_t s_w[4];
  const uint64_t i0 = uint64_t(blockIdx.x) * kScanBlock + threadIdx.x * kScanItems;
  uint64_t total;
  uint64_t o = part[blockIdx.x] + block_excl_scan(scan_thread_sum(in, n, i0), s_w, total);
#pragma unroll
  for (uint32_t k = 0; k < kScanItems; k++)
    if (i0 + k < n) {
      out[i0 + k] = o;
      o += in[i0 + k];
    }
  if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = part[gridDim.x];  // (the grand total)
}
__global__ __launch_bounds__(256) void gather_off_kernel(const uint64_t* off, const uint32_t* sent, uint32_t nsent,
                                                         uint64_t* out) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < nsent; i += gridDim.x * 256) out[i] = off[sent[i]];
}
__global__ __launch_bounds__(256) void copy_rows_kernel(const uint4* src, const uint64_t* n_ptr, uint64_t cap,
                                                        uint4* dst) {
  const uint64_t n = min(*n_ptr, cap);
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) dst[i] = src[i];
}

hipError_t launch_cells_sparse_count(hipStream_t s, const uint64_t* ck, const unsigned long long* n_ptr, uint64_t cap,
                                     const uint32_t* sent, uint32_t nsent, const uint64_t* base, uint32_t* cnt) {
  const uint32_t grid = (uint32_t)std::min<uint64_t>((cap + 255) / 256, 1024);
  hipLaunchKernelGGL(cells_sparse_count_kernel, dim3(std::max<uint32_t>(grid, 1)), dim3(256), 0, s, ck, n_ptr, sent,
                     nsent, base, cnt);
  return hipGetLastError();
}
uint32_t scan_parts(uint64_t n) { return (uint32_t)((n + kScanBlock - 1) / kScanBlock); }
hipError_t launch_scan_u32(hipStream_t s, const uint32_t* in, uint64_t n, uint64_t* out, uint64_t* part) {
  const uint32_t nb = scan_parts(n);
  if (nb) hipLaunchKernelGGL(scan_sums_kernel, dim3(nb), dim3(256), 0, s, in, n, part);
  hipLaunchKernelGGL(scan_parts_kernel, dim3(1), dim3(256), 0, s, part, nb);
  if (nb) hipLaunchKernelGGL(scan_apply_kernel, dim3(nb), dim3(256), 0, s, in, n, part, out);
  return hipGetLastError();
}
hipError_t launch_gather_off(hipStream_t s, const uint64_t* off, const uint32_t* sent, uint32_t nsent, uint64_t* out) {
  if (nsent)
    hipLaunchKernelGGL(gather_off_kernel, dim3(std::min<uint32_t>((nsent + 255) / 256, 1024)), dim3(256), 0, s, off,
                       sent, nsent, out);
  return hipGetLastError();
}
hipError_t launch_copy_rows(hipStream_t s, const void* src, const uint64_t* n_ptr, uint64_t cap, void* dst) {
  const uint32_t grid = (uint32_t)std::min<uint64_t>((cap + 255) / 256, 4096);
  hipLaunchKernelGGL(copy_rows_kernel, dim3(std::max<uint32_t>(grid, 1)), dim3(256), 0, s,
                     reinterpret_cast<const uint4*>(src), n_ptr, cap, reinterpret_cast<uint4*>(dst));
  return hipGetLastError();
}

hipError_t launch_cells_count(hipStream_t s, const uint32_t* hist, uint64_t hist_cells, uint32_t T,
                              const uint64_t* base, const uint32_t* np, uint32_t E, uint32_t* cnt) {
  const uint32_t grid = (uint32_t)std::min<uint64_t>((E + 3) / 4, 8192);
  hipLaunchKernelGGL(cells_count_kernel, dim3(std::max<uint32_t>(grid, 1)), dim3(256), 0, s, hist, hist_cells, T,
                     base, np, E, cnt);
  return hipGetLastError();
}

hipError_t launch_cells_emit(hipStream_t s, const uint32_t* hist, uint64_t hist_cells, uint32_t T,
                             const uint64_t* base, const uint32_t* np, uint32_t E, const uint64_t* off, uint4* rows) {
  const uint32_t grid = (uint32_t)std::min<uint64_t>((E + 3) / 4, 8192);
  hipLaunchKernelGGL(cells_emit_kernel, dim3(std::max<uint32_t>(grid, 1)), dim3(256), 0, s, hist, hist_cells, T,
                     base, np, E, off, rows);
  return hipGetLastError();
}

hipError_t launch_unpack(uint32_t grid, hipStream_t s, uint64_t* sum64, unsigned long long* pk64, uint32_t nb_entries,
                         uint32_t shift) {
  hipLaunchKernelGGL(unpack_kernel, dim3(grid), dim3(256), 0, s, sum64, pk64, nb_entries, shift);
  return hipGetLastError();
}

hipError_t launch_hist_pack(hipStream_t s, const uint32_t* hist, uint64_t ncells, uint32_t thr, void* u8,
                            void* ovf, uint64_t cap, unsigned long long* cnt, uint32_t* wgcnt) {
  if (!ncells) return hipSuccess;
  hipLaunchKernelGGL(hist_count_kernel, dim3(kPackGrid), dim3(kPackWG), 0, s, hist, ncells, thr, wgcnt);
  hipLaunchKernelGGL(hist_pack_kernel, dim3(kPackGrid), dim3(kPackWG), 0, s, hist, ncells, thr,
                     reinterpret_cast<uint8_t*>(u8), reinterpret_cast<unsigned long long*>(ovf), cap, wgcnt, cnt);
  return hipGetLastError();
}

hipError_t launch_hist_unpack(hipStream_t s, uint32_t* hist, uint64_t ncells, const void* u8, const void* ovf,
                              uint64_t n, unsigned long long* bad) {
  const uint64_t n4 = (ncells + 3) / 4;
  if (n4) {
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n4 + 255) / 256, 4096);
    hipLaunchKernelGGL(hist_unpack_kernel, dim3(grid), dim3(256), 0, s, hist, ncells,
                       reinterpret_cast<const uint8_t*>(u8));
  }
  if (n) {
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(hist_ovf_add_kernel, dim3(grid), dim3(256), 0, s, hist, ncells,
                       reinterpret_cast<const unsigned long long*>(ovf), n, bad);
  }
  return hipGetLastError();
}

hipError_t launch_sparse_compact(hipStream_t s, const uint64_t* keys, const uint32_t* vals, uint64_t cap,
                                 uint64_t* out, unsigned long long* cnt) {
  if (!cap) return hipSuccess;
  const uint32_t grid = (uint32_t)std::min<uint64_t>((cap + 255) / 256, 2048);
  hipLaunchKernelGGL(sparse_compact_kernel, dim3(grid), dim3(256), 0, s, keys, vals, cap, out, cnt);
  return hipGetLastError();
}

hipError_t launch_sparse_insert(hipStream_t s, uint64_t* keys, uint32_t* vals, uint64_t cap, const uint64_t* pairs,
                                uint64_t n) {
  if (!n) return hipSuccess;
  const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(sparse_insert_kernel, dim3(grid), dim3(256), 0, s, keys, vals, cap - 1, pairs, n);
  return hipGetLastError();
}

hipError_t launch_merge(hipStream_t s, void* dst, const void* src, uint64_t n, int op) {
  if (!n) return hipSuccess;
  const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(merge_kernel, dim3(grid), dim3(256), 0, s, dst, src, n, op);
  return hipGetLastError();
}

hipError_t launch_reset(uint32_t grid, hipStream_t s, const ResetParams& r) {
  hipLaunchKernelGGL(reset_kernel, dim3(grid), dim3(256), 0, s, r);
  return hipGetLastError();
}

}  // namespace nmg
