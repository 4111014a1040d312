// nmg_route.hip -- MI355X (gfx950) device code of the partition-first path
// for large object tables (nmg_route.h; DESIGN.md "Partition-first").
//
// Same results as attribute_kernel, bit for bit: every merge is an integer
// sum, min or max, and the first-match ordinal carries the analysis position
// (seq << 32 | byte offset), so the order in which samples are attributed
// changes nothing.  What changes is where the table lookups go: instead of a
// directory slot and a node record in HBM per sample (two dependent random
// lines), the route pass finds a sample's partition in a 16 KiB LDS tree and
// writes a 24 B compact record; the local pass then resolves whole partitions
// with their keys and node records in LDS.
#include <algorithm>

#include "nmg_device.h"
#include "nmg_route.h"

// build-time A/B switches of route2_kernel (tools/ab_build.sh -D...; the
// defaults are the shipped kernel): workgroup size, the back stage of two
// windows at a time, the global minimum / maximum read from LDS per record
#ifndef NMG_R2WG
#define NMG_R2WG 768
#endif
#ifndef NMG_R2PAIR
#define NMG_R2PAIR 0
#endif
#ifndef NMG_R2LDSMM  // (1: the shipped way; 0: per-lane register minima / maxima, measured no faster)
#define NMG_R2LDSMM 1
#endif
#ifndef NMG_R2COAL  // route pass: whole-line record loads, dealt to the lanes through LDS (A/B)
#define NMG_R2COAL 0
#endif
#ifndef NMG_R2ONESTORE  // route pass: one store instruction for every record stored alone (shipped: 1)
#define NMG_R2ONESTORE 1
#endif
#ifndef NMG_LOCAL_ONEMATCH  // local pass: one store instruction for a chunk group's match bits (shipped: 1)
#define NMG_LOCAL_ONEMATCH 1
#endif
#ifndef NMG_ABL_NOSCATTER  // (ablation only, results wrong: no record stored outside the line stage)
#define NMG_ABL_NOSCATTER 0
#endif

namespace nmg {

static_assert((uint64_t)kItemChunks * kChunk * kLaneMaxWeight < (1ull << kPackShift), "packed weight per item");

// in-order rank of Eytzinger node idx >= 1 of a complete `levels`-level tree
__device__ __forceinline__ uint32_t eytz_rank(uint32_t idx, uint32_t levels) {
  const uint32_t d = 31 - __builtin_clz(idx);
  return (((idx - (1u << d)) * 2 + 1) << (levels - 1 - d)) - 1;
}

// The partition of addr >= the first key: the last partition whose first key
// <= addr.  Its
// segment by comparisons with the (uniform) segment starts, one directory
// slot, then a binary search over the partition starts inside that slot --
// usually none or one: one to two dependent LDS reads instead of a search over
// every start.
__device__ __forceinline__ uint32_t route_partition(const RouteParams& rp, const uint64_t* s_pb,
                                                    const uint16_t* s_pdir, uint64_t addr) {
  uint64_t s0 = rp.seg[0].start;
  uint32_t base = rp.seg[0].base, ns = rp.seg[0].nslots, sh = rp.seg[0].shift, ql = rp.seg[0].qlast;
  for (uint32_t k = 1; k < rp.nseg; k++) {  // (uniform bound: only the table's segments; 7 unrolled
    const bool in = addr >= rp.seg[k].start;   // selects cost the route pass 6 %)
    s0 = in ? rp.seg[k].start : s0;
    base = in ? rp.seg[k].base : base;
    ns = in ? rp.seg[k].nslots : ns;
    sh = in ? rp.seg[k].shift : sh;
    ql = in ? rp.seg[k].qlast : ql;
  }
  const uint64_t rel = (addr - s0) >> sh;
  const uint32_t e = s_pdir[base + (rel < ns ? (uint32_t)rel : ns - 1)];
  uint32_t q = e & 2047u;
  const uint32_t c = e >> 11;
  uint32_t n = (c == kDirCntSat ? ql - q : c) + 1;  // candidates q .. q + n - 1; s_pb[q] <= addr
  while (n > 1) {
    const uint32_t half = n >> 1;
    if (s_pb[q + half] <= addr) {
      q += half;
      n -= half;
    } else {
      n = half;
    }
  }
  return q;
}

// ---------------------------------------------------------------------------
// compact records (16 B, see XLayout)

struct XRec {
  uint64_t addr, ts, w;
  uint64_t loc;  // byte offset / 8 | buffer index << obits: ordered as the analysis position
  uint32_t th, acc;
  bool esc;  // addr, ts and w are still to be re-read from the raw record (x_resolve)
  __device__ __forceinline__ uint32_t g(const XLayout& xl) const { return uint32_t(loc >> xl.obits); }
  __device__ __forceinline__ uint32_t off(const XLayout& xl) const {
    return uint32_t(loc & ((1ull << xl.obits) - 1)) << 3;
  }
};

// the record of a SAMPLE routed to the partition starting at pb (addr >= pb)
__device__ __forceinline__ uint4 x_encode(const XLayout& xl, uint64_t pb, uint64_t addr, uint64_t ts, uint64_t w,
                                          uint32_t g, uint32_t off, uint32_t th, uint32_t acc) {
  const uint64_t ar = addr - pb, tr = ts - xl.tbase;
  const bool fit = (ar >> kAddrBits) == 0 && ts >= xl.tbase && (tr >> kTsBits) == 0 && w < xl.wesc;
  const uint64_t a = fit ? ar : 0ull, t = fit ? tr : 0ull, wq = fit ? w : xl.wesc;
  const uint64_t loc = uint64_t(off >> 3) | (uint64_t(g) << xl.obits);
  const uint64_t lo = a | (t << kAddrBits);
  const uint64_t hi = (t >> (64 - kAddrBits)) | (wq << 16) | (loc << (16 + xl.wbits)) |
                      (uint64_t(th) << (63 - xl.tbits)) | (uint64_t(acc) << 63);
  return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

// x_decode without the bases: addr = the offset from the partition's first
// key, ts = the offset from tbase (the local pass's common path)
__device__ __forceinline__ XRec x_decode_rel(const XLayout& xl, uint4 v) {
  XRec r;
  r.addr = u64of(v.x, v.y & 0xffu);
  r.ts = u64of(__builtin_amdgcn_alignbit(v.z, v.y, 8), (v.z >> 8) & 0xffu);
  const uint32_t wesc = (uint32_t)xl.wesc;
  r.w = __builtin_amdgcn_alignbit(v.w, v.z, 16) & wesc;
  r.esc = r.w == wesc;
  r.loc = (u64of(v.z, v.w) >> (16 + xl.wbits)) & ((1ull << (xl.obits + xl.gbits)) - 1);
  r.th = (v.w >> (31 - xl.tbits)) & ((1u << xl.tbits) - 1);
  r.acc = v.w >> 31;
  return r;
}

__device__ __forceinline__ XRec x_decode(const XLayout& xl, uint64_t pb, uint4 v) {
  XRec r = x_decode_rel(xl, v);
  r.addr += pb;
  r.ts += xl.tbase;
  return r;
}

// an escaped record's address, timestamp and weight from the raw record
// (struct mem_sample after the 8 B header: timestamp, addr, weight)
__device__ __forceinline__ void x_resolve(XRec& r, const XLayout& xl, const uint8_t* data, const BufDesc* descs) {
  const uint64_t* q = reinterpret_cast<const uint64_t*>(data + descs[r.g(xl)].offset + r.off(xl));
  r.ts = q[1];
  r.addr = q[2];
  r.w = q[3];
}

// ---------------------------------------------------------------------------
// direct attribution (overflow_kernel: a route workgroup's chunk pool was
// exhausted): the lookup of
// __ma_find_mem_info_from_sample_generic (mem_analyzer.c:249-286) in global
// memory -- binary search of the keys (ht_lower_key, tools/hash.c:63-77),
// node record, older entries -- and global atomics.  Correct for any input;
// only taken when a workgroup's samples outgrow its pool (SAMPLE records
// shorter than 40 B, or the kDbgTinyPool test switch).
__device__ __forceinline__ void direct_attribute(const Params& p, uint64_t addr, uint64_t ts, uint64_t w, uint32_t th,
                                                 uint32_t acc, uint32_t lvl, uint64_t seq, uint32_t off,
                                                 uint32_t slot) {
  // (update_counters of this record: the route pass counted it)
  if (p.nb_keys == 0 || p.keys[0] > addr) return;
  uint32_t lo = 0, n = p.nb_keys;
  while (n > 1) {
    const uint32_t half = n >> 1;
    if (p.keys[lo + half] <= addr) {
      lo += half;
      n -= half;
    } else {
      n = half;
    }
  }
  const uint4* q = reinterpret_cast<const uint4*>(p.nodes + lo);
  const uint4 a = q[0], b = q[1], c = q[2];
  Match m;
  m.e = -1;
  m.baddr = 0;
  m.hist = kHistSparse;
  if (entry_match(a, b, addr, ts)) {
    m.e = c.w;
    m.baddr = u64of(a.x, a.y);
    m.hist = u64of(c.x, c.y);
  } else {
    const uint4 d = q[3];
    if (d.x > 1) match_older(p, d.y, d.x, addr, ts, m);
  }
  if (m.e < 0) return;
  const uint64_t e = (uint64_t)m.e;
  atomicAdd(p.bufcnt + p.nb_bufs + slot, 1u);
  atomicAdd(p.found, 1ull);
  atomicAdd(reinterpret_cast<unsigned long long*>(p.sum64 + objcw_index(e, acc, 0, p.nb_entries)), 1ull);
  if (w) atomicAdd(reinterpret_cast<unsigned long long*>(p.sum64 + objcw_index(e, acc, 1, p.nb_entries)),
                   (unsigned long long)w);
  atomicMin(reinterpret_cast<unsigned long long*>(p.min64 + 36 + e), (unsigned long long)((seq << 32) | off));
  if (!(p.flags & NMG_F_PAGE_HIST)) return;
  const uint32_t page = uint32_t(int(uint64_t(addr - m.baddr) / kPageSize));
  if (m.hist != kHistSparse) {
    atomicAdd(p.hist + uint64_t(th) * p.hist_cells + m.hist + page, 1u);
  } else {
    const uint32_t sidx = p.entries[e].sidx;
    if (sidx != ~0u) sparse_add(p, sparse_key(sidx, th, page), seq, off, 1u);
  }
}

// ---------------------------------------------------------------------------
// pass 1: route

// A buffer descriptor of the route pass, in scalar registers (5 dwords):
// offset in the arena, length, thread rank | access type << 16, analysis index
struct RDesc {
  uint64_t offset;
  uint32_t len, ta, pad;
  __device__ __forceinline__ uint32_t thread_rank() const { return ta & 0xffffu; }
  __device__ __forceinline__ uint32_t access() const { return ta >> 16; }
};

// update_counters(global_counters, ...) (mem_sampling.c:517-592) in the
// route pass: per lane and access type, one u32 per counter pair, count << 24
// | weight sum, for the total and for kRtGroups buckets (the common PEBS
// levels: hits in L1, LFB, L2, L3, local RAM and remote RAM, L3 misses); the
// NA count; and per group the minimum and maximum weight of the records whose
// first group it is, as one u32 of two u16 fields, max << 16 | (0xffff -
// min) (0: no record; every record makes it non-zero), kept with one packed
// u16 max.  A record whose weight reaches 2^16, or that falls in another
// bucket, or in two, is counted -- those parts -- by LDS atomics.  Drained
// every kRouteDrain windows (255 records of < 2^16 fit 24 bits).
//
// A record's level class: the hit levels x = lvl >> 3 (11 bits) when HIT,
// else the miss levels at bit 11 when MISS (HIT beats MISS, quirk Q12).
// Group g covers class bits kRtMask[g] and is bucket nibble g of kRtBucketNib.
constexpr int kRtGroups = 7;
__device__ __forceinline__ uint32_t rt_class(uint32_t lvl) {
  const uint32_t x = lvl >> 3;
  return (lvl & LVL_HIT) ? x : (lvl & LVL_MISS) ? x << 11 : 0u;
}
// groups: x0 L1 (bucket 0), x1 LFB (3), x2 L2 (1), x3 L3 (2), x4 local RAM
// (4), x5|x6 remote RAM (5), miss x3 L3 (9 + 2)
constexpr uint32_t kRtMask[kRtGroups] = {1u, 2u, 4u, 8u, 16u, 0x60u, 8u << 11};
constexpr uint32_t kRtBucketNib = 0xB542130u;  // group g -> bucket (nibble g)
constexpr uint32_t kRtKnown = 0x7fu | (8u << 11);
constexpr uint32_t kRouteDrain = 128;
constexpr uint32_t kRtOne = 1u << 24;
struct RouteAcc {
  uint32_t tot, na, g[kRtGroups], mm[kRtGroups];
};
__device__ __forceinline__ void racc_clear(RouteAcc& a) {
  a.tot = a.na = 0;
#pragma unroll
  for (int g = 0; g < kRtGroups; g++) a.g[g] = a.mm[g] = 0;
}
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
// both u16 fields' maxima (v_pk_max_u16)
__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b) {
  const u16x2 r = __builtin_elementwise_max(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b));
  return __builtin_bit_cast(uint32_t, r);
}
// full-wave u32 maximum (DPP, as wave_sum_u32; lanes past a row's edge read 0)
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, dpp0<0x111, 0xf>(v));
  v = max(v, dpp0<0x112, 0xf>(v));
  v = max(v, dpp0<0x114, 0xf>(v));
  v = max(v, dpp0<0x118, 0xf>(v));
  v = max(v, dpp0<0x142, 0xa>(v));
  v = max(v, dpp0<0x143, 0xc>(v));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// the counting of one SAMPLE of access type ACC (a wave window lies in one
// buffer: the caller branches on the access once); every lane of the wave
// calls it, `valid` the ones with a SAMPLE.  The minimum / maximum of the
// record's first group is read from LDS and updated by an LDS atomic only when
// the record moves it (NMG_R2LDSMM=0: kept in the lane's registers until the
// drain instead -- measured no faster).
template <uint32_t ACC>
__device__ __forceinline__ void route_count(RouteAcc& a, unsigned long long (*sums)[kGlobalSums],
                                            unsigned long long (*mins)[18], unsigned long long (*maxs)[18],
                                            bool valid, uint32_t lvl, uint64_t w) {
  const uint32_t cls = rt_class(lvl);
  const bool big = w >= (1u << 16);
  const uint32_t term = (valid && !big) ? (uint32_t)w + kRtOne : 0u;
  a.tot += term;
  a.na += (valid && !big) ? (lvl & LVL_NA) : 0u;
  uint32_t gm = 0;  // the record's groups, one bit each
#pragma unroll
  for (int g = 0; g < kRtGroups; g++) {
    const bool in = (cls & kRtMask[g]) != 0;
    a.g[g] += in ? term : 0u;
    gm |= in ? 1u << g : 0u;
  }
  const uint32_t fb = gm ? (kRtBucketNib >> (4 * __builtin_ctz(gm))) & 15u : 0xffu;
#if NMG_R2LDSMM  // read the LDS minimum / maximum, an atomic when the record moves it
  if (valid && gm && !big) {
    const unsigned long long mn = mins[ACC][fb], mx = maxs[ACC][fb];
    if (w < mn) atomicMin(&mins[ACC][fb], (unsigned long long)w);
    if (w > mx) atomicMax(&maxs[ACC][fb], (unsigned long long)w);
  }
#else  // (A/B, round 6) the lane's registers, drained with the counts
  const uint32_t pw = (valid && !big) ? ((uint32_t)w << 16) | (0xffffu - (uint32_t)w) : 0u;
  const uint32_t first = gm & (0u - gm);  // the record's first group
#pragma unroll
  for (int g = 0; g < kRtGroups; g++) a.mm[g] = first == (1u << g) ? pk_max_u16(a.mm[g], pw) : a.mm[g];
#endif
  // (rare) every other bucket, and the whole record when its weight is big
  const bool rare = valid && (big || (cls & ~kRtKnown) || (gm & (gm - 1)));
  if (__ballot(rare)) {
    if (rare) {
      if (big) {
        atomicAdd(&sums[ACC][0], 1ull);
        atomicAdd(&sums[ACC][1], (unsigned long long)w);
        if (lvl & LVL_NA) atomicAdd(&sums[ACC][2], 1ull);
      }
      for (uint32_t m = bucket_mask(lvl); m; m &= m - 1) {
        const uint32_t bk = (uint32_t)__builtin_ctz(m);
        bool reg = false;  // (counted in registers unless big)
#pragma unroll
        for (int g = 0; g < kRtGroups; g++) reg |= ((gm >> g) & 1u) && ((kRtBucketNib >> (4 * g)) & 15u) == bk;
        if (big || !reg) {
          atomicAdd(&sums[ACC][3 + 2 * bk], 1ull);
          if (w) atomicAdd(&sums[ACC][4 + 2 * bk], (unsigned long long)w);
        }
        if (bk != fb || big) {  // (the first group's, in registers unless big)
          atomicMin(&mins[ACC][bk], (unsigned long long)w);
          atomicMax(&maxs[ACC][bk], (unsigned long long)w);
        }
      }
    }
  }
}

// lanes -> the workgroup's LDS counters (every lane of the wave calls this)
__device__ __forceinline__ void racc_drain(RouteAcc& a, unsigned long long* sums, unsigned long long* mins,
                                           unsigned long long* maxs, int lane) {
#pragma unroll
  for (int g = 0; g < kRtGroups; g++) {  // the groups' minimum / maximum weights
    if (__ballot(a.mm[g] != 0) == 0) continue;
    const uint32_t hi = wave_max_u32(a.mm[g] >> 16), lo = wave_max_u32(a.mm[g] & 0xffffu);
    const uint32_t bk = (kRtBucketNib >> (4 * g)) & 15u;
    if (lane == 0) {
      atomicMin(&mins[bk], (unsigned long long)(0xffffu - lo));
      atomicMax(&maxs[bk], (unsigned long long)hi);
    }
  }
  if (__ballot(a.tot != 0) == 0) {
    racc_clear(a);
    return;
  }  // (every register count comes with the total's)
  auto add = [&](uint32_t v, int word) {  // count << 24 | weight -> words word, word + 1
    if (__ballot(v != 0) == 0) return;
    const uint32_t c = wave_sum_u32(v >> 24), wt = wave_sum_u32(v & (kRtOne - 1));
    if (lane == 0) {
      atomicAdd(&sums[word], (unsigned long long)c);
      if (wt) atomicAdd(&sums[word + 1], (unsigned long long)wt);
    }
  };
  add(a.tot, 0);
  const uint32_t na = wave_sum_u32(a.na);
  if (lane == 0 && na) atomicAdd(&sums[2], (unsigned long long)na);
#pragma unroll
  for (int g = 0; g < kRtGroups; g++) add(a.g[g], 3 + 2 * int((kRtBucketNib >> (4 * g)) & 15u));
  racc_clear(a);
}

// kDbgRouteTiming: per-wave cycle accumulators of the route pass's phases
struct RTimer {
  uint64_t acc[12];
  uint64_t last;
};
template <bool TIMING>
__device__ __forceinline__ void rt_stamp(RTimer& t, int i) {
  if (TIMING) {
    const uint64_t now = stamp();
    t.acc[i] += now - t.last;
    t.last = now;
  }
}

// Descriptors of the workgroup's range staged in LDS (offset, len,
// thread | access << 16): a buffer transition reads LDS instead of waiting on
// a global load.  Ranges longer than kDescLds read the rest from global
// memory.  In the analysis-order schedule the count slot (.pad) is the
// index and seq = seq0 + index.
constexpr uint32_t kDescLds = NMG_R2COAL ? 160 : 512;

__device__ __forceinline__ RDesc route_desc(const RouteParams& rp, const uint4* s_desc, uint32_t r0, uint32_t i) {
  RDesc d;
  if (i - r0 < kDescLds) {
    // (uniform: scalar registers)
    const uint4 l = s_desc[i - r0];
    d.offset = u64of(__builtin_amdgcn_readfirstlane(l.x), __builtin_amdgcn_readfirstlane(l.y));
    d.len = __builtin_amdgcn_readfirstlane(l.z);
    d.ta = __builtin_amdgcn_readfirstlane(l.w);
    d.pad = i;
    return d;
  }
  const BufDesc g = rp.p.sbufs[i];
  vm_drain();  // (rare: ranges past kDescLds; keeps the waits on the common path exact)
  d.offset = u64of(__builtin_amdgcn_readfirstlane((uint32_t)g.offset),
                   __builtin_amdgcn_readfirstlane((uint32_t)(g.offset >> 32)));
  d.len = __builtin_amdgcn_readfirstlane(g.len);
  d.ta = __builtin_amdgcn_readfirstlane(g.thread_rank | (g.access << 16));
  d.pad = i;
  return d;
}

// ---------------------------------------------------------------------------
// pass 1: route2_kernel, per-wave record streams.
//
// Each wave owns whole buffers, dequeued from the workgroup's range through
// an LDS counter, and walks them with its own cursor in windows of 64 stride
// slots (__analyze_buffer's byte cursor, mem_sampling.c:836-926, per buffer
// as the reference does it): the fast-path check is a ballot, the slow path
// (LOST / short / irregular records) is the wave's own header walk, and the
// per-buffer SAMPLE tally is the wave's.  Nothing synchronises the workgroup
// between its first and last barrier: each record claims a slot of its
// partition's open chunk with one LDS atomic (the chunk protocol is at the
// claim) and goes to that slot through the partition's LDS line (below).
// The next window's loads stay in flight across the window.
//
// The line stage.  A record stored straight to its chunk slot is a 16 B
// store of its own: a wave-instruction of such stores touches 64 lines,
// which costs the CU ~10x the issue time of 64 B runs at a 2 GB footprint
// (tools/micro/vmem.hip), and a cold partition's line leaves L2 partly
// written.  So every partition has a 64 B line in LDS for its chunk lines
// (chunk slots 4l .. 4l + 3) in turn, and one 64-bit line word:
//   the staged line S (its chunk-line number, mod 4096) and the slots it
//   holds; for the lines S .. S + 7 the number of their records that are
//   in place (written to the LDS line, or stored to their slot); a
//   given-up bit.
// A record whose line is S is written to the LDS line; a record of a line
// ahead of S (a hot partition's records run ahead of its slowest writer) is
// stored straight to its slot.  Either way it then counts itself for its
// line with one LDS atomic; the record that brings S's count to 4 has the
// staged slots written out -- a full line by four lanes of its wave,
// sixteen lines per store instruction -- and moves S on, past any line
// already complete.  Nothing ever waits: a record 8 lines or more ahead of
// S gives the partition's line up (its later records are stored straight
// to their slots and not counted), and a staged line left incomplete -- a
// partition's last, or a given-up one -- is written out, the slots it
// holds, after the workgroup's last barrier.

// route2_kernel's workgroup: 12 waves (three per SIMD)
constexpr uint32_t kR2WG = NMG_R2WG;
// line stage: partitions q < kLineParts have an LDS line
constexpr uint32_t kLineParts = NMG_R2COAL ? 1152 : 1280;
// line word (u64): line l's count (3 bits) at 3 * (l mod 8), staged slots
// (4) at 24, given up at 28, S at 52
typedef unsigned long long LineWord;
constexpr uint32_t kLwMaskShift = 24, kLwSShift = 52, kLwLineMask = 4095, kLwAhead = 8;
constexpr LineWord kLwBroken = 1ull << 28;
constexpr LineWord kLwOne = 1;
__device__ __forceinline__ uint32_t lw_count(LineWord w, uint32_t l) { return uint32_t(w >> (3 * (l & (kLwAhead - 1)))) & 7u; }
__device__ __forceinline__ uint32_t lw_s(LineWord w) { return uint32_t(w >> kLwSShift); }
__device__ __forceinline__ uint32_t lw_mask(LineWord w) { return uint32_t(w >> kLwMaskShift) & 15u; }
constexpr uint32_t kWaves = kR2WG / 64;
constexpr uint32_t kWaveWinBytes = 64 * kRecBytes;  // one wave window: 64 stride slots
constexpr uint32_t kNoBuf = 0xffffffffu;            // RDesc::pad of "no buffer"

__device__ __forceinline__ RDesc no_buf() {
  RDesc d;
  d.offset = 0;
  d.len = 0;
  d.ta = 0;
  d.pad = kNoBuf;
  return d;
}

// The three record loads of a lane's stride slot of the wave window at
// (off, c): buffer loads through a resource covering exactly the buffer
// [off, off + len), so a slot past its end reads zeros without a branch or a
// select (a select of a loaded value, or a load the compiler sinks into a
// branch, would make the number of loads in flight path-dependent and every
// later wait a full drain).  A slot partly inside the buffer reads part of
// the record; the window's check sends it to the slow path.
__device__ __forceinline__ void wload(const uint8_t* data, uint64_t off, uint32_t len, uint32_t c, int lane,
                                      RawRec& r) {
  // (the stream's fields are wave-uniform but may live in vector registers:
  // read them into scalars, or every load becomes a waterfall loop over the
  // resource)
  off = u64of(__builtin_amdgcn_readfirstlane((uint32_t)off), __builtin_amdgcn_readfirstlane((uint32_t)(off >> 32)));
  len = __builtin_amdgcn_readfirstlane(len);
  c = __builtin_amdgcn_readfirstlane(c);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(data + off), (short)0, (int)len, 0x00020000);
  const uint32_t pos = c + uint32_t(lane) * kRecBytes;
  const uint32_t odd = (pos >> 3) & 1;  // 16 B aligned pieces, as load_rec
  const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, pos + (odd ? 8 : 0), 0, 0);
  const auto y = __builtin_amdgcn_raw_buffer_load_b128(rs, pos + (odd ? 24 : 16), 0, 0);
  const auto z = __builtin_amdgcn_raw_buffer_load_b64(rs, pos + (odd ? 0 : 32), 0, 0);
  r.x = make_uint4(x[0], x[1], x[2], x[3]);
  r.y = make_uint4(y[0], y[1], y[2], y[3]);
  r.z = make_uint2(z[0], z[1]);
}

// NMG_R2COAL: the wave window's bytes as three whole-line loads (lane l:
// bytes 16 l, 1024 + 16 l, 2048 + 16 l of the window; the third only for
// lanes < 32), dealt to the lanes' 40 B records through the wave's LDS stage
struct CRec {
  uint4 a, b, c;
};
__device__ __forceinline__ void cload(const uint8_t* data, uint64_t off, uint32_t len, uint32_t c, int lane,
                                      CRec& r) {
  off = u64of(__builtin_amdgcn_readfirstlane((uint32_t)off), __builtin_amdgcn_readfirstlane((uint32_t)(off >> 32)));
  len = __builtin_amdgcn_readfirstlane(len);
  c = __builtin_amdgcn_readfirstlane(c);
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(data + off), (short)0, (int)len, 0x00020000);
  const uint32_t pos = c + uint32_t(lane) * 16u;
  const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, pos, 0, 0);
  const auto y = __builtin_amdgcn_raw_buffer_load_b128(rs, pos + 1024u, 0, 0);
  const auto z = __builtin_amdgcn_raw_buffer_load_b128(rs, pos + 2048u, 0, 0);
  r.a = make_uint4(x[0], x[1], x[2], x[3]);
  r.b = make_uint4(y[0], y[1], y[2], y[3]);
  r.c = make_uint4(z[0], z[1], z[2], z[3]);
}
__device__ __forceinline__ Rec stage_rec(uint4* st, const CRec& r, int lane) {
  st[lane] = r.a;
  st[64 + lane] = r.b;
  if (lane < 32) st[128 + lane] = r.c;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
  const uint64_t* q = reinterpret_cast<const uint64_t*>(st) + 5 * lane;
  Rec d;
  d.hdr = q[0];
  d.ts = q[1];
  d.addr = q[2];
  d.w = q[3];
  d.dsrc = q[4];
  return d;
}
#if NMG_R2COAL
typedef CRec WRec;
#define NMG_WLOAD(d, o, l, c, ln, r) cload(d, o, l, c, ln, r)
#else
typedef RawRec WRec;
#define NMG_WLOAD(d, o, l, c, ln, r) wload(d, o, l, c, ln, r)
#endif

// route_partition with the segment table in LDS instead of kernel arguments
// (which the compiler would keep in scalar registers): the segment is the
// number of segment starts <= addr past the first (the starts in one group
// of broadcast reads, the unused ones ~0), then one read of its parameters
struct SegL {
  uint4 a;  // start lo, start hi, base, nslots
  uint4 b;  // shift, qlast
};
__device__ __forceinline__ uint32_t route_partition_l(const SegL* s_seg, const uint64_t* s_segst, uint32_t nseg,
                                                      const uint64_t* s_pb, const uint16_t* s_pdir, uint64_t addr) {
  uint32_t k = 0;
  uint64_t st[kRouteSegs];
#pragma unroll
  for (uint32_t j = 1; j < kRouteSegs; j++) st[j] = s_segst[j];
#pragma unroll
  for (uint32_t j = 1; j < kRouteSegs; j++) k += (uint32_t)(addr >= st[j]);
  k = min(k, nseg - 1);  // (addr = ~0 passes the unused starts too)
  const uint4 ak = s_seg[k].a, bk = s_seg[k].b;
  const uint64_t s0 = u64of(ak.x, ak.y);
  const uint32_t base = ak.z, ns = ak.w, sh = bk.x, ql = bk.y;
  const uint64_t rel = (addr - s0) >> sh;
  const uint32_t e = s_pdir[base + (rel < ns ? (uint32_t)rel : ns - 1)];
  uint32_t q = e & 2047u;
  const uint32_t c = e >> 11;
  uint32_t n = (c == kDirCntSat ? ql - q : c) + 1;  // candidates q .. q + n - 1; s_pb[q] <= addr
  while (n > 1) {
    const uint32_t half = n >> 1;
    if (s_pb[q + half] <= addr) {
      q += half;
      n -= half;
    } else {
      n = half;
    }
  }
  return q;
}

// route2's per-partition chunk state, one LDS word: open chunk (20 bits,
// index in the workgroup's pool) | next chunk (20) | generation (8) | claims
// (16).  Claim f < 64 takes slot f of the open chunk, 64 <= f < 128 slot
// f - 64 of the next one, which is opened in advance; claim 96 takes a new
// chunk from the pool and advances the generation (open <- next <- new,
// claims -= 64, by compare-and-swap, so claims past 128 made meanwhile are
// void: those lanes wait for the generation and claim again).  So every
// chunk's slots are taken by exactly the claims that map to them (no hole),
// and a claim needs one LDS round trip unless the partition is so hot that
// 32 claims arrive while one lane takes a chunk.  Chunk ids kStNone (before
// the partition's first claim) and kStOvf (pool exhausted: the overflow list).
constexpr uint32_t kStNone = 0xfffffu, kStOvf = 0xffffeu, kStMaxLocal = 0xffffdu;
__device__ __forceinline__ uint32_t st_cnt(uint64_t s) { return uint32_t(s) & 0xffffu; }
__device__ __forceinline__ uint32_t st_gen(uint64_t s) { return (uint32_t(s) >> 16) & 0xffu; }
__device__ __forceinline__ uint32_t st_next(uint64_t s) { return uint32_t(s >> 24) & 0xfffffu; }
__device__ __forceinline__ uint32_t st_cur(uint64_t s) { return uint32_t(s >> 44); }
__device__ __forceinline__ uint64_t st_pack(uint32_t cur, uint32_t next, uint32_t gen, uint32_t cnt) {
  return (uint64_t(cur) << 44) | (uint64_t(next) << 24) | (uint64_t(gen & 0xffu) << 16) | cnt;
}
// a chunk of the workgroup's pool (its pool index), or kStOvf
__device__ __forceinline__ uint32_t route2_take(uint32_t& taken, uint32_t cap) {
  const uint32_t t = atomicAdd(&taken, 1u);
  return t < cap ? t : kStOvf;
}
// generation g -> g + 1 of one partition: open <- next (or n1 on its first
// claim), next <- n2, claims -> min(claims, 128) - 64 (first claim: 1, the
// opener's own slot 0)
// (hint: the word after this lane's own claim, the value when no other claim
// came in between -- the first compare-and-swap usually succeeds)
__device__ __forceinline__ void route2_advance(unsigned long long* st, uint32_t g, uint32_t n1, uint32_t n2,
                                               bool first, unsigned long long hint) {
  unsigned long long cur = hint;
  while (true) {
    const uint32_t f = st_cnt(cur);
    const unsigned long long nw = first ? st_pack(n1, n2, g + 1, 1u)
                                        : st_pack(st_next(cur), n2, g + 1, min(f, 2 * kChunk) - kChunk);
    const unsigned long long prev = atomicCAS(st, cur, nw);
    if (prev == cur) break;
    cur = prev;
  }
}

// a claim's outcome: the rec16 slot (~0: none), its chunk line, the
// overflow list; !ok: a void claim, past the next chunk -- wait for
// generation waitg to end and claim again
struct Claim {
  uint64_t dst;
  uint32_t lid, waitg;
  bool ovf, ok;
};
__device__ __forceinline__ Claim route2_settle(uint64_t old, uint32_t q, unsigned long long* s_state, uint32_t& taken,
                                               uint32_t capl, uint32_t* cmeta, uint32_t c0) {
  Claim r;
  r.dst = ~0ull;
  r.lid = 0;
  r.waitg = 0;
  r.ovf = false;
  r.ok = true;
  const uint32_t f = st_cnt(old), g = st_gen(old), cu = st_cur(old), nx = st_next(old);
  if (cu != kStNone && f < 2 * kChunk) {  // a slot of the open chunk or of the next one
    const uint32_t c = f < kChunk ? cu : nx;
    if (c == kStOvf) r.ovf = true;
    else r.dst = uint64_t(c0 + c) * kChunk + (f & (kChunk - 1));
    r.lid = ((g << 6) + f) >> 2;  // (slot f - 64 of the next chunk = generation g + 1's slot)
    if (f == kChunk + kChunk / 2) {  // half of the next chunk claimed: open the one after it
      const uint32_t n2 = route2_take(taken, capl);
      if (n2 != kStOvf) cmeta[c0 + n2] = q | (kChunk << 24);
      route2_advance(&s_state[q], g, n2, n2, false, old + 1);
    }
  } else if (cu == kStNone && f == 2 * kChunk) {  // q's first claim: open two chunks
    const uint32_t n1 = route2_take(taken, capl);
    const uint32_t n2 = n1 == kStOvf ? kStOvf : route2_take(taken, capl);
    if (n1 != kStOvf) cmeta[c0 + n1] = q | (kChunk << 24);
    if (n2 != kStOvf) cmeta[c0 + n2] = q | (kChunk << 24);
    route2_advance(&s_state[q], g, n1, n2, true, old + 1);
    if (n1 == kStOvf) r.ovf = true;
    else r.dst = uint64_t(c0 + n1) * kChunk;
    r.lid = (g + 1) << 4;  // slot 0 of generation g + 1
  } else {
    r.waitg = g;
    r.ok = false;
  }
  return r;
}

template <int N>
__device__ __forceinline__ bool any_of(const bool (&b)[N]) {
  bool r = false;
#pragma unroll
  for (int i = 0; i < N; i++) r |= b[i];
  return r;
}

// a routed record between route2_kernel's front (stream, counters, partition,
// encode) and its back (claim, line stage, store)
struct XF {
  uint4 a;     // the compact record
  uint32_t q;  // its partition
  bool routed;
};

template <bool TIMING>
__global__ __launch_bounds__(kR2WG, 1) void route2_kernel(RouteParams rp) {
  __shared__ uint64_t s_pb[kMaxParts + 1];
  __shared__ uint16_t s_pdir[kRouteDir];
  __shared__ uint32_t s_dead[(kMaxParts + 1) / 32];
  __shared__ unsigned long long s_state[kMaxParts + 1];  // open chunk << 32 | slots claimed in it
  __shared__ uint4 s_desc[kDescLds];
#if NMG_R2COAL
  // per wave, used in turn: the window's bytes (front start), the slow path's
  // SAMPLE offsets, the line write-out table (back) -- one wave's LDS ops run in order
  __shared__ uint4 s_stage[kWaves][kWaveWinBytes / 16];
  uint32_t(*s_wlist)[kWaveWinBytes / 4] = reinterpret_cast<uint32_t(*)[kWaveWinBytes / 4]>(s_stage);
  uint2(*s_tab)[kWaveWinBytes / 8] = reinterpret_cast<uint2(*)[kWaveWinBytes / 8]>(s_stage);
#else
  __shared__ uint32_t s_wlist[kWaves][64];  // slow path: the wave window's SAMPLE offsets
#endif
  __shared__ uint32_t s_taken, s_bnext;
  __shared__ unsigned long long s_gsums[2][kGlobalSums], s_gmins[2][18], s_gmaxs[2][18];
  __shared__ SegL s_seg[kRouteSegs];
  __shared__ uint64_t s_segst[kRouteSegs];
  // the line stage: per partition a line of four compact records, its line
  // word and its chunk line (pool slot / 4); per wave the lines it writes out
  __shared__ uint4 s_line[kLineParts * 4];
  __shared__ LineWord s_lw[kLineParts];
  __shared__ uint32_t s_ldst[kLineParts];
#if !NMG_R2COAL
  __shared__ uint2 s_tab[kWaves][64];
#endif

  Params& p = rp.p;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  if (tid < (int)kRouteSegs) {
    const RSeg g = rp.seg[tid];
    s_seg[tid].a = make_uint4((uint32_t)g.start, (uint32_t)(g.start >> 32), g.base, g.nslots);
    s_seg[tid].b = make_uint4(g.shift, g.qlast, 0, 0);
    s_segst[tid] = tid < rp.nseg ? g.start : ~0ull;
  }
  const uint32_t nseg = rp.nseg;
  const uint64_t first_start = rp.seg[0].start;
  const uint32_t P = rp.nparts;
  const uint32_t c0 = rp.chunk0[blockIdx.x];
  const uint32_t cap = rp.chunk0[blockIdx.x + 1] - c0;
  const uint32_t capl = min(cap, kStMaxLocal + 1);  // (pool indices fit the state's 20-bit fields)
  for (uint32_t i = tid; i < kMaxParts + 1; i += kR2WG) s_pb[i] = rp.pbounds[i];
  for (uint32_t i = tid; i < kRouteDir; i += kR2WG) s_pdir[i] = rp.pdir[i];
  if (tid < (int)((kMaxParts + 1) / 32)) s_dead[tid] = rp.pdead[tid];
  for (uint32_t i = tid; i < P; i += kR2WG) s_state[i] = st_pack(kStNone, kStNone, 0, 2 * kChunk);
  // the first line of a partition: slot 0 of generation 1's open chunk
  const uint32_t nlp = !(p.flags & kDbgNoLines) ? min(P, kLineParts) : 0u;
  for (uint32_t i = tid; i < nlp; i += kR2WG) s_lw[i] = LineWord(kChunk / 4) << kLwSShift;
  // (kDbgLapNoWait: a record one line ahead of S already gives the line up -- tests)
  const uint32_t ahead_max = (p.flags & kDbgLapNoWait) ? 1u : kLwAhead;
  const uint32_t r0 = p.ranges[blockIdx.x], r1 = p.ranges[blockIdx.x + 1];
  for (uint32_t i = r0 + tid; i < r1 && i - r0 < kDescLds; i += kR2WG) {
    const BufDesc d = p.sbufs[i];
    s_desc[i - r0] = make_uint4((uint32_t)d.offset, (uint32_t)(d.offset >> 32), d.len, d.thread_rank | (d.access << 16));
  }
  if (tid == 0) {
    s_taken = 0;
    s_bnext = r0;
  }
  if (tid < (int)kGlobalSums) s_gsums[0][tid] = s_gsums[1][tid] = 0;
  if (tid < 18) {
    s_gmins[0][tid] = s_gmins[1][tid] = ~0ull;  // INIT_COUNTER (mem_analyzer.c:415-420)
    s_gmaxs[0][tid] = s_gmaxs[1][tid] = 0;
  }
  RouteAcc gacc[2];  // per-lane update_counters per access type, drained every kRouteDrain windows
  racc_clear(gacc[0]);
  racc_clear(gacc[1]);
  uint32_t gwin = 0;
  lds_sync();

  if (r0 < r1) {
    // (descriptors are assigned, never selected as whole structs: a select of
    // structs goes through scratch memory)
    auto dequeue = [&](RDesc& d) {
      uint32_t i = 0;
      if (lane == 0) i = atomicAdd(&s_bnext, 1u);
      i = __builtin_amdgcn_readfirstlane(i);
      if (i < r1) d = route_desc(rp, s_desc, r0, i);
      else d = no_buf();
    };
    // the wave's stream: buffer d0 at cursor cur; d1 = the buffer after it
    // once dequeued (have1): dequeued only when a window of d1 is prefetched,
    // so that a wave never holds a buffer it is not about to read
    RDesc d0, d1 = no_buf();
    dequeue(d0);
    bool have1 = false;
    uint32_t cur = 0;
    uint32_t ns = 0;  // SAMPLEs of d0 so far (mem_sampling.c:921-926)
    // the window after (b, c) if the window at (b, c) holds only whole 40 B
    // records (the fast path): its buffer and cursor
    uint32_t pidx, pcur;
    uint64_t eoff;  // the predicted window's buffer (offset, length)
    uint32_t elen;
    auto predict = [&]() {
      if (d0.pad == kNoBuf) {
        pidx = kNoBuf;
        pcur = 0;
        eoff = 0;
        elen = 0;
      } else if (cur + kWaveWinBytes < d0.len) {
        pidx = d0.pad;
        pcur = cur + kWaveWinBytes;
        eoff = d0.offset;
        elen = d0.len;
      } else {
        if (!have1) {
          dequeue(d1);
          have1 = true;
        }
        pidx = d1.pad;
        pcur = 0;
        eoff = d1.offset;
        elen = d1.len;
      }
    };
    WRec ra, rb;
    NMG_WLOAD(p.data, d0.offset, d0.len, 0, lane, ra);
    predict();
    NMG_WLOAD(p.data, eoff, elen, pcur, lane, rb);

    RTimer rt;  // (TIMING) per-wave phase cycles
#pragma unroll
    for (int k = 0; k < 12; k++) rt.acc[k] = 0;
    rt.last = TIMING ? stamp() : 0;
    uint32_t nwin = 0;

    // one window of this wave: A holds its slots, B the next window's (in
    // flight); k = the window's place in the batch (staging slots)
    // (the stream state is wave-uniform, but values merged across branches
    // may be kept in vector registers, and then every test of them is an
    // exec-mask branch: read them back into scalars once per window)
    auto uni = [&](RDesc& d) {
      d.offset = u64of(__builtin_amdgcn_readfirstlane((uint32_t)d.offset),
                       __builtin_amdgcn_readfirstlane((uint32_t)(d.offset >> 32)));
      d.len = __builtin_amdgcn_readfirstlane(d.len);
      d.ta = __builtin_amdgcn_readfirstlane(d.ta);
      d.pad = __builtin_amdgcn_readfirstlane(d.pad);
    };
    auto front = [&](WRec& A, WRec& B, XF& X) {
      uni(d0);
      uni(d1);
      cur = __builtin_amdgcn_readfirstlane(cur);
      ns = __builtin_amdgcn_readfirstlane(ns);
      const RDesc dw = d0;  // this window's buffer
      const uint32_t pos = cur + uint32_t(lane) * kRecBytes;
      const bool cand = pos < dw.len;
      if (TIMING) {
        asm volatile("s_waitcnt vmcnt(3)" ::: "memory");  // (this window's loads count as wait)
        nwin++;
      }
      rt_stamp<TIMING>(rt, 0);
#if NMG_R2COAL
      Rec rec = stage_rec(s_stage[wave], A, lane);
#else
      Rec rec = decode_rec(A, pos);
#endif
      const bool bad = cand && (uint64_t(pos) + kRecBytes > dw.len || (rec.hdr >> 48) != kRecBytes);
      bool valid;
      uint32_t roff = pos, ncur;
      if (!__ballot(bad) && !(cur & 7)) {
        valid = cand && uint32_t(rec.hdr) == kSampleType;
        ncur = cur + kWaveWinBytes;
      } else {
        // ---- slow path: the wave follows the header chain from cur
        // (non-SAMPLE records skipped by size, size 0 / truncation /
        // misalignment flagged), listing up to 64 SAMPLE offsets
        const uint8_t* base = p.data + dw.offset;
        const uint64_t len = dw.len;
        uint64_t q0 = cur;
        uint32_t n = 0, err = 0;
        if (cur & 7) err = kErrUnaligned;
        while (!err && q0 < len && n < 64) {
          const uint64_t q = q0 + uint64_t(lane) * kRecBytes;
          const uint64_t hdr = (q + 8 <= len) ? *reinterpret_cast<const uint64_t*>(base + q) : 0;
          const bool reg = q + kRecBytes <= len && (hdr >> 48) == kRecBytes;
          const uint64_t rm = __ballot(reg);
          const uint32_t run = ~rm ? (uint32_t)__builtin_ctzll(~rm) : 64u;
          const uint32_t take = min(run, 64u - n);
          const bool smp = (uint32_t)lane < take && uint32_t(hdr) == kSampleType;
          const uint64_t sm = __ballot(smp);
          if (smp) s_wlist[wave][n + (uint32_t)__popcll(sm & ((1ull << lane) - 1))] = (uint32_t)q;
          n += (uint32_t)__popcll(sm);
          q0 += uint64_t(take) * kRecBytes;
          if (take < run || run == 64 || q0 >= len || n >= 64) continue;
          if (q0 + 8 > len) {
            err = kErrTruncated;
            break;
          }
          const uint64_t h = (uint64_t)__shfl(hdr, (int)run, 64);
          const uint32_t size = uint32_t(h >> 48);
          if (size == 0) {  // mem_sampling.c:857-860
            err = kErrZeroSize;
            break;
          }
          if (size & 7) {
            err = kErrUnaligned;
            break;
          }
          if (uint32_t(h) == kSampleType) {
            if (q0 + kRecBytes > len || q0 + size > len) {
              err = kErrTruncated;
              break;
            }
            if (lane == 0) s_wlist[wave][n] = (uint32_t)q0;
            n++;
          }
          q0 += size;  // non-SAMPLE records are skipped by their size (:918)
        }
        if (err && lane == 0) set_error(p, rp.seq0 + dw.pad, (uint32_t)q0, err);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
        ncur = err ? (uint32_t)len : (uint32_t)min(q0, len);
        valid = (uint32_t)lane < n;
        roff = valid ? s_wlist[wave][lane] : 0u;
        RawRec rr;
        load_rec(base, roff, valid ? len : 0, rr);
        rec = decode_rec(rr, roff);
        vm_drain();
      }
      ns += (uint32_t)__popcll(__ballot(valid));
      // ---- advance the stream; dw's tally when it is done
      if (dw.pad != kNoBuf) {
        if (ncur >= dw.len) {
          if (lane == 0 && ns) atomicAdd(p.bufcnt + dw.pad, ns);
          ns = 0;
          cur = 0;
          if (have1) {
            d0 = d1;
          } else {
            dequeue(d0);
          }
          have1 = false;
          d1 = no_buf();
        } else {
          cur = ncur;
        }
      }
      // ---- the next window's loads again if it is not where B was loaded
      // (after a slow-path window), then the loads of the window after it
      if (d0.pad != pidx || (d0.pad != kNoBuf && cur != pcur)) {
        NMG_WLOAD(p.data, d0.offset, d0.len, cur, lane, B);
        vm_drain();  // (rare: keeps the waits on the common path exact)
      }
      predict();
      NMG_WLOAD(p.data, eoff, elen, pcur, lane, A);

      // ---- this window's records: update_counters(global_counters, sample)
      // (mem_sampling.c:882: every SAMPLE, matched or not), partition, chunk
      // slot, store
      rt_stamp<TIMING>(rt, 1);
      const uint32_t acc_l = dw.access();
      if (acc_l == 0) {  // (uniform)
        route_count<0>(gacc[0], s_gsums, s_gmins, s_gmaxs, valid, uint32_t(rec.dsrc >> 5) & 0x3fff, rec.w);
      } else {
        route_count<1>(gacc[1], s_gsums, s_gmins, s_gmaxs, valid, uint32_t(rec.dsrc >> 5) & 0x3fff, rec.w);
      }
      if (++gwin == kRouteDrain) {
        racc_drain(gacc[0], s_gsums[0], s_gmins[0], s_gmaxs[0], lane);
        racc_drain(gacc[1], s_gsums[1], s_gmins[1], s_gmaxs[1], lane);
        gwin = 0;
      }
      rt_stamp<TIMING>(rt, 2);
      // below the first key ht_lower_key finds no node: counted, not routed
      bool routed = valid && rec.addr >= first_start;
      const uint32_t q = routed ? route_partition_l(s_seg, s_segst, nseg, s_pb, s_pdir, rec.addr) : 0u;
      // a partition whose entries all have free_date 0 matches only timestamp-0
      // samples (RouteParams::pdead): the others are done (unmatched), not routed
      routed = routed && (rec.ts == 0 || !((s_dead[q >> 5] >> (q & 31)) & 1u));
      if (TIMING) (void)__builtin_amdgcn_readfirstlane(__ballot(q != 0));  // (the search ends here)
      rt_stamp<TIMING>(rt, 3);
      X.a = make_uint4(0, 0, 0, 0);
      X.q = q;
      X.routed = routed;
      if (routed) X.a = x_encode(rp.xl, s_pb[q], rec.addr, rec.ts, rec.w, dw.pad, roff, dw.thread_rank(), acc_l);
      rt_stamp<TIMING>(rt, 4);
    };

    // ---- the records of N windows (one; two in the NMG_R2PAIR A/B build,
    // their LDS round trips issued together): a slot in each record's
    // partition's open chunks (one LDS atomic on the partition's state,
    // route2_settle), the line stage, the stores.  (Two records of one lane
    // behave as the records of two lanes: every step below is correct for any
    // number of records of one partition.)  No barrier: the waves run on
    // their own streams.
    auto back = [&](const auto& X) {
      constexpr int N = (int)(sizeof(X) / sizeof(X[0]));
      uint64_t dst[N];   // rec16 slot, or ~0: no slot (not routed / overflow list)
      uint32_t lid[N];   // the slot's chunk line number (mod 4096): the lap that serves it
      bool ovf[N], lined[N];
      LineWord lw[N];
      uint32_t waitg[N];
      bool todo[N];
      unsigned long long old[N];
#pragma unroll
      for (int r = 0; r < N; r++) {
        dst[r] = ~0ull;
        lid[r] = 0;
        ovf[r] = false;
        waitg[r] = 0;
        todo[r] = false;
        lined[r] = X[r].routed && X[r].q < nlp;
        // (the line word read beside the claim: a lap can only move on once
        // this record's own line is written, so a lap that equals the
        // record's line here still does after the claim)
        lw[r] = lined[r] ? s_lw[X[r].q] : LineWord(0);
      }
#pragma unroll
      for (int r = 0; r < N; r++) old[r] = X[r].routed ? atomicAdd(&s_state[X[r].q], 1ull) : 0ull;
#pragma unroll
      for (int r = 0; r < N; r++) {
        if (X[r].routed) {
          const Claim c = route2_settle(old[r], X[r].q, s_state, s_taken, capl, rp.cmeta, c0);
          dst[r] = c.dst;
          lid[r] = c.lid;
          ovf[r] = c.ovf;
          waitg[r] = c.waitg;
          todo[r] = !c.ok;
        }
      }
      {
        bool spin[N];
#pragma unroll
        for (int r = 0; r < N; r++) spin[r] = todo[r];
        while (__ballot(any_of(todo))) {  // (rare) void claims
#pragma unroll
          for (int r = 0; r < N; r++) {
            if (!todo[r]) continue;
            if (!spin[r]) {
              const Claim c = route2_settle(atomicAdd(&s_state[X[r].q], 1ull), X[r].q, s_state, s_taken, capl, rp.cmeta, c0);
              dst[r] = c.dst;
              lid[r] = c.lid;
              ovf[r] = c.ovf;
              waitg[r] = c.waitg;
              todo[r] = !c.ok;
              spin[r] = todo[r];
            } else {
              const uint64_t st = __hip_atomic_load(&s_state[X[r].q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              spin[r] = st_gen(st) == waitg[r];
            }
          }
        }
      }
      rt_stamp<TIMING>(rt, 5);
      // ---- the line stage (see the comment above kR2WG)
      bool staged[N], counts[N];
#pragma unroll
      for (int r = 0; r < N; r++) staged[r] = counts[r] = false;
      if (__ballot(any_of(lined))) {
        bool done[N];
        uint32_t dmask[N];
#pragma unroll
        for (int r = 0; r < N; r++) {
          lid[r] &= kLwLineMask;
          const uint32_t j = (uint32_t)dst[r] & 3u, S = lw_s(lw[r]), ahead = (lid[r] - S) & kLwLineMask;
          // (a record of the overflow list has no slot but counts for its line)
          counts[r] = lined[r] && !(lw[r] & kLwBroken) && ahead < ahead_max;
          staged[r] = counts[r] && ahead == 0 && dst[r] != ~0ull;
          if (lined[r] && !(lw[r] & kLwBroken) && ahead >= ahead_max) atomicOr(&s_lw[X[r].q], kLwBroken);
          if (staged[r]) {
            s_line[X[r].q * 4 + j] = X[r].a;
            s_ldst[X[r].q] = (uint32_t)(dst[r] >> 2);
          } else if (counts[r] && dst[r] != ~0ull && !NMG_R2ONESTORE) {
            if (!NMG_ABL_NOSCATTER) rp.rec16[dst[r]] = X[r].a;
          }
        }
        // (the staged records before the counts that may complete their lines)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        LineWord o[N];
#pragma unroll
        for (int r = 0; r < N; r++) {
          o[r] = 0;
          if (counts[r]) {
            const uint32_t j = (uint32_t)dst[r] & 3u;
            o[r] = atomicAdd(&s_lw[X[r].q], (kLwOne << (3 * (lid[r] & (kLwAhead - 1)))) +
                                                (staged[r] ? kLwOne << (kLwMaskShift + j) : LineWord(0)));
          }
        }
#pragma unroll
        for (int r = 0; r < N; r++) {
          // the line's fourth record, the line being S (S may have reached it
          // since the read beside the claim)
          done[r] = counts[r] && lw_count(o[r], lid[r]) == 3 && lw_s(o[r]) == lid[r];
          dmask[r] = counts[r] ? lw_mask(o[r]) | (staged[r] ? 1u << ((uint32_t)dst[r] & 3u) : 0u) : 0u;
          if (TIMING) rt.acc[8] += (uint64_t)__popcll(__ballot(counts[r] && !staged[r]));
        }
#pragma unroll
        for (int r = 0; r < N; r++) {
          const uint64_t dm = __ballot(done[r]);
          if (!dm) continue;
          // the staged slots of the completed lines written out: four lanes per line
          if (done[r])
            s_tab[wave][__popcll(dm & ((1ull << lane) - 1))] =
                make_uint2(X[r].q | (dmask[r] << 11) | (lid[r] << 16), (uint32_t)(dst[r] >> 2));
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
          const uint32_t nd = (uint32_t)__popcll(dm);
          // a line's piece k: its staged slot (if any) stored, the line read by
          // all four pieces -- one instruction, waited for by the stores --
          // before S moves on and its slots are reused; piece 0 moves S on
          auto piece_done = [&](uint2 t, uint32_t k) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            if (k == 0) {  // S -> S + 1, past the lines already complete (all their records stored straight)
              const uint32_t tq = t.x & 2047u;
              uint32_t l = t.x >> 16, m = (t.x >> 11) & 15u;
              while (true) {
                const LineWord ow = atomicAdd(&s_lw[tq], (kLwOne << kLwSShift) - (LineWord(4) << (3 * (l & (kLwAhead - 1)))) -
                                                            (LineWord(m) << kLwMaskShift));
                l = (l + 1) & kLwLineMask;
                if (lw_count(ow, l) != 4) break;
                m = 0;
              }
            }
          };
          for (uint32_t j0 = 0; j0 < nd; j0 += 16) {
            const uint32_t jj = j0 + ((uint32_t)lane >> 2);
            if (jj < nd) {
              const uint2 t = s_tab[wave][jj];
              const uint32_t tq = t.x & 2047u, tm = (t.x >> 11) & 15u, k = lane & 3;
              if ((tm >> k) & 1) rp.rec16[uint64_t(t.y) * 4 + k] = s_line[tq * 4 + k];
              piece_done(t, k);
            }
          }
          // (s_tab reused by the second record's lines: every lane read its entry above)
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
        }
      }
      rt_stamp<TIMING>(rt, 9);
#pragma unroll
      for (int r = 0; r < N; r++) {
        // the records the line stage did not take: not lined, or given up
        const bool straight = dst[r] != ~0ull && !counts[r];
        // (NMG_R2ONESTORE: the records counted for a line ahead of the staged one
        // stored here too -- one store instruction for every record stored
        // alone; nothing reads the slots before the local pass)
        const bool alone = straight || (NMG_R2ONESTORE && counts[r] && !staged[r] && dst[r] != ~0ull);
        if (alone && !NMG_ABL_NOSCATTER) rp.rec16[dst[r]] = X[r].a;
        if (TIMING) {  // (records staged / stored straight to their slot)
          rt.acc[6] += (uint64_t)__popcll(__ballot(staged[r]));
          rt.acc[7] += (uint64_t)__popcll(__ballot(straight));
        }
      }
      if (__ballot(any_of(ovf))) {  // (rare) a workgroup's pool outgrown: SAMPLEs shorter than 40 B
#pragma unroll
        for (int r = 0; r < N; r++) {
          if (!ovf[r]) continue;
          const uint64_t pbq = s_pb[X[r].q];
          const uint32_t o = atomicAdd(rp.ovf_cnt, 1u);
          if (o < rp.ovf_cap) {
            rp.ovf16[o] = X[r].a;
            rp.ovfx[o] = pbq;
          } else {  // attributed at once
            XRec xr = x_decode(rp.xl, pbq, X[r].a);
            if (xr.esc) x_resolve(xr, rp.xl, p.data, p.sbufs);
            direct_attribute(p, xr.addr, xr.ts, xr.w, xr.th, xr.acc, 0, rp.seq0 + xr.g(rp.xl), xr.off(rp.xl),
                             xr.g(rp.xl));
          }
        }
        vm_drain();  // (rare: nothing of this path stays pending where it joins the window)
      }
      rt_stamp<TIMING>(rt, 10);
    };

#if NMG_R2PAIR
    XF X[2];  // (A/B: the back of two windows at a time -- measured slower, round 6)
    do {  // (d0: the wave's stream, uniform)
      front(ra, rb, X[0]);
      front(rb, ra, X[1]);
      back(X);
    } while (d0.pad != kNoBuf);
#else
    XF X[1];
    do {  // (d0: the wave's stream, uniform)
      front(ra, rb, X[0]);
      back(X);
      front(rb, ra, X[0]);
      back(X);
    } while (d0.pad != kNoBuf);
#endif

    if (TIMING && lane == 0) {
      unsigned long long* o = p.dbg + (uint64_t(blockIdx.x) * (kWG / 64) + tid / 64) * kRouteTimingWords;
      for (int k = 0; k < 9; k++) o[k] = rt.acc[k];
      o[9] = nwin;
      uint32_t nb = 0;  // (wave 0: the workgroup's partitions whose line was given up)
      if (wave == 0)
        for (uint32_t q = 0; q < nlp; q++) nb += (s_lw[q] & kLwBroken) ? 1u : 0u;
      o[10] = nb;
      o[11] = rt.acc[9];
      o[12] = rt.acc[10];
    }
  }
  racc_drain(gacc[0], s_gsums[0], s_gmins[0], s_gmaxs[0], lane);
  racc_drain(gacc[1], s_gsums[1], s_gmins[1], s_gmaxs[1], lane);
  lds_sync();
#pragma unroll
  for (uint32_t a = 0; a < 2; a++) {  // the global mem_counters of both access types
    if (tid < (int)kGlobalSums && s_gsums[a][tid])
      atomicAdd(reinterpret_cast<unsigned long long*>(p.sum64 + gsum_index(a, tid)), s_gsums[a][tid]);
    if (tid < 18 && s_gsums[a][3 + 2 * tid]) {
      atomicMin(reinterpret_cast<unsigned long long*>(p.min64 + a * 18 + tid), s_gmins[a][tid]);
      atomicMax(reinterpret_cast<unsigned long long*>(p.max64 + a * 18 + tid), s_gmaxs[a][tid]);
    }
  }
  // the open and next chunks' fill (claims end below 96: the 96th advanced
  // the generation); a next chunk nothing reached keeps fill 0, which the
  // count and scatter passes skip; pool use
  for (uint32_t q = tid; q < P; q += kR2WG) {
    const unsigned long long st = s_state[q];
    const uint32_t f = st_cnt(st), cu = st_cur(st), nx = st_next(st);
    if (cu == kStNone) continue;
    if (cu != kStOvf) rp.cmeta[c0 + cu] = q | (min(f, kChunk) << 24);
    if (nx != kStOvf) rp.cmeta[c0 + nx] = q | ((f > kChunk ? f - kChunk : 0u) << 24);
    // a line the stage still holds (the partition's last, or one a given-up
    // lap left incomplete): the slots it holds
    if (q < nlp) {
      const uint32_t m = lw_mask(s_lw[q]);
      for (uint32_t j = 0; j < 4; j++)
        if ((m >> j) & 1u) rp.rec16[uint64_t(s_ldst[q]) * 4 + j] = s_line[q * 4 + j];
    }
  }
  if (tid == 0) rp.used[blockIdx.x] = min(s_taken, capl);
}

// ---------------------------------------------------------------------------
// records that found no chunk (a workgroup's samples outgrew its pool:
// SAMPLE records shorter than 40 B, or the kDbgTinyPool switch): attributed
// one by one with global lookups and atomics

__global__ __launch_bounds__(256) void overflow_kernel(RouteParams rp) {
  const uint32_t n = min(*rp.ovf_cnt, rp.ovf_cap);
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    XRec xr = x_decode(rp.xl, rp.ovfx[i], rp.ovf16[i]);
    if (xr.esc) x_resolve(xr, rp.xl, rp.p.data, rp.p.sbufs);
    direct_attribute(rp.p, xr.addr, xr.ts, xr.w, xr.th, xr.acc, 0, rp.seq0 + xr.g(rp.xl), xr.off(rp.xl),
                     xr.g(rp.xl));
  }
}

// ---------------------------------------------------------------------------
// pass 2: count, plan (one workgroup) and scatter

// chunks per (route workgroup, partition) from the chunks' partition tags
__global__ __launch_bounds__(kWG) void count_kernel(CountParams cp) {
  __shared__ uint32_t s_cnt[kMaxParts + 1];
  const ScatterParams& r = cp.sc;
  const uint32_t tid = threadIdx.x, w = blockIdx.x, P = r.nparts;
  for (uint32_t q = tid; q < P; q += kWG) s_cnt[q] = 0;
  __syncthreads();
  const uint32_t c0 = r.chunk0[w], n = r.used[w];
  constexpr uint32_t kU = 8;  // chunk tags in flight per thread
  for (uint32_t b = 0; b < n; b += kU * kWG) {
    uint32_t m[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) {
      const uint32_t i = b + u * kWG + tid;
      m[u] = i < n ? r.cmeta[c0 + i] : 0u;
    }
#pragma unroll
    for (uint32_t u = 0; u < kU; u++)
      if (m[u] >> 24) atomicAdd(&s_cnt[m[u] & 0xffffffu], 1u);  // (fill 0: a chunk route2 opened and nothing reached)
  }
  __syncthreads();
  uint32_t* out = const_cast<uint32_t*>(r.pcnt) + uint64_t(w) * P;
  for (uint32_t q = tid; q < P; q += kWG) out[q] = s_cnt[q];
}

// pass 2a: per partition, the exclusive prefix of its chunk counts over the
// route workgroups (a column of pcnt), and the partition's total into pbase.
// 64 partitions per workgroup, the rows in 16 groups of consecutive
// workgroups: every count of a thread in flight at once, the groups' sums
// combined in LDS.
constexpr uint32_t kPlanRowGroups = kWG / 64;
__global__ __launch_bounds__(kWG) void plan_cols_kernel(PlanParams r) {
  __shared__ uint32_t s_sum[kPlanRowGroups][64];
  const uint32_t tid = threadIdx.x, c = tid & 63, rg = tid >> 6;
  const uint32_t P = r.nparts, q = blockIdx.x * 64 + c;
  const uint32_t per = (r.grid + kPlanRowGroups - 1) / kPlanRowGroups, w0 = rg * per;
  constexpr uint32_t kU = 16;  // counts in registers (groups of more rows: in steps of kU)
  uint32_t sum = 0;
  for (uint32_t b = 0; b < per; b += kU) {
    uint32_t v[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) {
      const uint32_t w = w0 + b + u;
      v[u] = (q < P && b + u < per && w < r.grid) ? r.pcnt[uint64_t(w) * P + q] : 0u;
    }
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) sum += v[u];
  }
  s_sum[rg][c] = sum;
  __syncthreads();
  uint32_t run = 0;
  for (uint32_t g = 0; g < rg; g++) run += s_sum[g][c];
  for (uint32_t b = 0; b < per; b += kU) {
    uint32_t v[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) {
      const uint32_t w = w0 + b + u;
      v[u] = (q < P && b + u < per && w < r.grid) ? r.pcnt[uint64_t(w) * P + q] : 0u;
    }
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) {
      const uint32_t w = w0 + b + u;
      if (q < P && b + u < per && w < r.grid) r.pcnt[uint64_t(w) * P + q] = run;
      run += v[u];
    }
  }
  if (q < P && rg == kPlanRowGroups - 1) r.pbase[q] = run;  // (the last group: the column's total)
}

// pass 2b (one workgroup): the partitions' first list slots and work items
// from their totals (plan_cols_kernel)
__global__ __launch_bounds__(kWG) void plan_kernel(PlanParams r) {
  __shared__ uint32_t s_tot[kMaxParts + 1], s_nit[kMaxParts + 1], s_wsum[2][kWG / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t P = r.nparts;
  for (uint32_t q = tid; q < P; q += kWG) {
    const uint32_t run = r.pbase[q];
    s_tot[q] = run;
    s_nit[q] = (run + kItemChunks - 1) / kItemChunks;
  }
  __syncthreads();
  // exclusive scans of the chunk totals and the item counts (two per thread)
  const uint32_t i0 = 2 * (uint32_t)tid;
  const uint32_t t0 = i0 < P ? s_tot[i0] : 0u, t1 = i0 + 1 < P ? s_tot[i0 + 1] : 0u;
  const uint32_t n0 = i0 < P ? s_nit[i0] : 0u, n1 = i0 + 1 < P ? s_nit[i0 + 1] : 0u;
  uint32_t it = t0 + t1, in = n0 + n1;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t a = __shfl_up(it, o, 64), b = __shfl_up(in, o, 64);
    if (lane >= o) {
      it += a;
      in += b;
    }
  }
  if (lane == 63) {
    s_wsum[0][wave] = it;
    s_wsum[1][wave] = in;
  }
  __syncthreads();
  uint32_t wt = 0, wn = 0;
  for (int w2 = 0; w2 < wave; w2++) {
    wt += s_wsum[0][w2];
    wn += s_wsum[1][w2];
  }
  const uint32_t tb = wt + it - (t0 + t1), nb = wn + in - (n0 + n1);
  for (uint32_t k = 0; k < 2; k++) {
    const uint32_t q = i0 + k;
    if (q >= P) break;
    const uint32_t base = tb + (k ? t0 : 0u), ibase = nb + (k ? n0 : 0u), tot = k ? t1 : t0;
    r.pbase[q] = base;
    for (uint32_t j = 0; j * kItemChunks < tot; j++)
      r.items[ibase + j] = make_uint4(q, base + j * kItemChunks, base + min(tot, (j + 1) * kItemChunks),
                                      tot <= kItemChunks ? 1u : 0u);  // .w: the partition's only item
  }
  if (tid == kWG - 1) {
    r.ctl[0] = wn + in;
    r.ctl[1] = 0;
    r.ctl[3] = r.ctl[2];  // this launch's overflow-path records (read by local_kernel)
    r.ctl[2] = 0;  // overflow list (read by overflow_kernel before this launch)
  }
}

__global__ __launch_bounds__(kWG) void scatter_kernel(ScatterParams r) {
  __shared__ uint32_t s_cnt[kMaxParts + 1];  // this workgroup's next list slot per partition
  const uint32_t tid = threadIdx.x, w = blockIdx.x, P = r.nparts;
  const uint32_t* off = r.pcnt + uint64_t(w) * P;
  for (uint32_t q = tid; q < P; q += kWG) s_cnt[q] = r.pbase[q] + off[q];
  __syncthreads();
  const uint32_t c0 = r.chunk0[w], n = r.used[w];
  constexpr uint32_t kU = 8;  // chunk tags in flight per thread
  for (uint32_t b = 0; b < n; b += kU * kWG) {
    uint32_t m[kU];
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) {
      const uint32_t i = b + u * kWG + tid;
      m[u] = i < n ? r.cmeta[c0 + i] : 0u;
    }
#pragma unroll
    for (uint32_t u = 0; u < kU; u++) {
      if (!(m[u] >> 24)) continue;
      const uint32_t k = atomicAdd(&s_cnt[m[u] & 0xffffffu], 1u);
      r.clist[k] = (c0 + b + u * kWG + tid) | ((m[u] >> 24) << kChunkIdBits);  // chunk id | fill
    }
  }
}

// ---------------------------------------------------------------------------
// pass 3: attribute one partition per workgroup at a time

// local pass: workgroup size and chunks per interleaved group (a wave holds
// two groups: one being attributed, the other's records in flight)
constexpr uint32_t kLWG = 1024;
// u16 page cells of items past 2^16 records (kPageCarry): at kCarryAt a
// cell moves kCarryMove of its count to global memory (at most kLWG * 2
// adds are in flight, far fewer than 2^16 - kCarryAt)
constexpr uint32_t kCarryAt = 0xf000u, kCarryMove = 0x8000u;
static_assert(2 * kLWG < 0x10000u - kCarryAt && kCarryMove < kCarryAt, "page cell carry margin");
constexpr int kLC = 2;  // (the timing wait below counts on it)

// a load served by L2, never by this CU's L1 (global_load ... sc1)
template <typename T>
__device__ __forceinline__ T l2_load(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A partition owns a range of table positions; the counters are indexed by
// entry id, which is the position for the nmg_set_objects table and
// pe_ids[position] for an online table (nmg_update_objects).
__device__ __forceinline__ uint64_t entry_id(const LocalParams& lp, uint32_t pos) {
  return lp.pe_ids ? lp.pe_ids[pos] : pos;
}

// match_older (nmg_device.h) giving the matching entry's table position
// (-1: none), its buffer_addr and its histogram base
__device__ __forceinline__ int32_t match_older_pos(const Params& p, uint32_t first, uint32_t count, uint64_t addr,
                                                   uint64_t ts, uint64_t& baddr, uint64_t& hist) {
  for (uint32_t j = first + 1; j < first + count; j++) {  // older entries of a reused address
    const uint4* r = reinterpret_cast<const uint4*>(p.chain + j);
    const uint4 ra = r[0], rb = r[1];
    if (entry_match(ra, rb, addr, ts)) {
      const uint4 rc = r[2];
      baddr = u64of(ra.x, ra.y);
      hist = u64of(rc.x, rc.y);
      return (int32_t)j;
    }
  }
  return -1;
}

// PACKED: an online table with packed page cells (LocalParams::pe_cmap; a
// variant of its own, so that the offline table's flush carries none of it)
template <bool TIMING, bool PACKED>
__global__ __launch_bounds__(kLWG, 1) void local_kernel(LocalParams lp) {
  __shared__ uint64_t s_keys[kPartSlots];
  __shared__ uint4 s_pn[kPartSlots];  // packed node records (PackedNode)
  __shared__ uint2 s_info[kPartSlots];
  __shared__ uint4 s_dir[kPartDir];   // directory slots (PartDir)
  __shared__ uint4 s_old[kOldLds];    // older entries of reused keys (kOldLds)
  __shared__ uint32_t s_oinf[kOldLds];
  __shared__ unsigned long long s_owt[2][kPartEntries];
  __shared__ unsigned long long s_first[kPartEntries];
  __shared__ uint32_t s_pg[kPartCells / 2];
  __shared__ uint32_t s_clist[kItemChunks];  // the item's chunk list entries
  __shared__ uint32_t s_item, s_cnext, s_nfound, s_big, s_took, s_carry;
  __shared__ uint4 s_nx[4];  // the next item's work item and PartInfo (take_next)

  Params& p = lp.p;
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t nitems = lp.ctl[0];
  const uint32_t T = p.nb_threads;
  const bool pages = (p.flags & NMG_F_PAGE_HIST) != 0;
  RTimer rt;  // (kDbgLocalTiming) per-wave phase cycles
#pragma unroll
  for (int k = 0; k < 12; k++) rt.acc[k] = 0;
  rt.last = TIMING ? stamp() : 0;
  uint32_t nchunks = 0, nit = 0;
  uint32_t nfound = 0;  // this wave's matched records (Params::found, added once per workgroup at the end)
  if (tid == 0) s_nfound = 0;  // (read after the item loop's barriers)
  // the item counters start zeroed; every flush re-zeroes what it reads
  for (uint32_t i = tid; i < kPartEntries; i += kLWG) {
    s_owt[0][i] = s_owt[1][i] = 0;
    s_first[i] = ~0ull;
  }
  for (uint32_t i = tid; i < kPartCells / 2; i += kLWG) s_pg[i] = 0;
  // the next item -- its index, work item and partition descriptor, into
  // LDS -- is taken by the first wave done with the current one's chunks:
  // those three dependent round trips hide behind the other waves' chunks and
  // the flush (one whole wave calls this)
  static_assert(sizeof(PartInfo) == 48, "PartInfo: three uint4");
  auto take_next = [&]() {
    uint32_t idx = 0;
    if (lane == 0) idx = atomicAdd(lp.ctl + 1, 1u);
    idx = __builtin_amdgcn_readfirstlane(idx);
    if (lane == 0) s_item = idx;
    if (idx < nitems) {
      const uint4 nx = lp.items[idx];
      const uint32_t nq = __builtin_amdgcn_readfirstlane(nx.x);
      if (lane == 0) s_nx[0] = nx;
      if (lane < 3) s_nx[1 + lane] = reinterpret_cast<const uint4*>(lp.parts + nq)[lane];
    }
  };
  if (tid < 64) take_next();
  if (tid == 0) s_took = 0;
  while (true) {
    lds_sync();
    const uint32_t it = __builtin_amdgcn_readfirstlane(s_item);
    rt_stamp<TIMING>(rt, 6);
    if (it >= nitems) break;
    nit++;
    const uint4 item = s_nx[0];
    const uint32_t q = __builtin_amdgcn_readfirstlane(item.x);
    PartInfo pi;
    {
      uint4* pw = reinterpret_cast<uint4*>(&pi);
      pw[0] = s_nx[1];
      pw[1] = s_nx[2];
      pw[2] = s_nx[3];
    }
    const uint32_t dshift = __builtin_amdgcn_readfirstlane(pi.dshift);
    {
      // the partition's tables and the item's chunk list: at most one element
      // of each table per thread (kClPer of the list), every load in flight
      // before the first LDS store
      static_assert(kPartKeys <= kLWG && kPartDir == kLWG && kOldLds <= kLWG, "one table element per thread");
      constexpr uint32_t kClPer = (kItemChunks + kLWG - 1) / kLWG;
      const uint32_t nk = pi.nk, nold = min(pi.ne - nk, kOldLds), ncl = item.z - item.y;
      uint64_t key = 0;
      uint4 pn = make_uint4(0, 0, 0, 0), od = pn;
      uint2 inf = make_uint2(0, 0);
      uint32_t oi = 0, cl[kClPer];
      if (tid < nk) {
        key = lp.pe_keys[uint64_t(q) * kPartSlots + tid];
        pn = lp.pe_pnode[uint64_t(q) * kPartSlots + tid];
        inf = lp.pe_info[uint64_t(q) * kPartSlots + tid];
      }
      const uint4 dd = lp.pe_dir[uint64_t(q) * kPartDir + tid];
      if (tid < nold) {
        od = lp.pe_old[uint64_t(q) * kOldLds + tid];
        oi = lp.pe_oinf[uint64_t(q) * kOldLds + tid];
      }
#pragma unroll
      for (uint32_t u = 0; u < kClPer; u++) cl[u] = tid + u * kLWG < ncl ? lp.clist[item.y + tid + u * kLWG] : 0u;
      if (tid < nk) {
        s_keys[tid] = key;
        s_pn[tid] = pn;
        s_info[tid] = inf;
      }
      s_dir[tid] = dd;
      if (tid < nold) {
        s_old[tid] = od;
        s_oinf[tid] = oi;
      }
#pragma unroll
      for (uint32_t u = 0; u < kClPer; u++)
        if (tid + u * kLWG < ncl) s_clist[tid + u * kLWG] = cl[u];
    }
    if (tid == 0) {
      s_cnext = 0;
      s_took = 0;
    }
    const uint32_t ncell = (pages && pi.pages_lds) ? T * pi.span : 0u;
    const bool excl = item.w != 0 && !(p.flags & kDbgLocalAtomics);  // no other workgroup writes this partition's
                                                                     // counters
    if (tid == 0) s_big = s_carry = 0;
    lds_sync();
    const uint64_t k0key = u64of(__builtin_amdgcn_readfirstlane((uint32_t)s_keys[0]),
                                 __builtin_amdgcn_readfirstlane((uint32_t)(s_keys[0] >> 32)));
    rt_stamp<TIMING>(rt, 7);

    // Each wave takes pairs of consecutive chunks of the item's list (in
    // LDS) from an LDS counter, so the waves end within a pair of each other
    // at the item's barrier, and works on two chunks at a time, their steps interleaved
    // (the LDS round trips of one cover the other's); the records of the next
    // two are in flight meanwhile (a wave's chunk is 1.5 KiB).  The compiler
    // waits for a chunk's loads with the smallest vmcnt any path allows, so
    // the loop is shaped for that: unrolled (the record registers are never
    // copied -- a copy of a load in flight waits for it), every chunk load
    // covers the whole wave (a fixed number of memory ops between a load and
    // its use), and the rare paths that issue global memory ops of their own
    // end with vmcnt(0).
    const uint32_t nl = item.z - item.y;
    auto chunk_load = [&](uint32_t l, uint4& a) {  // the chunk at list position l (l >= nl: none; no branch)
      const uint32_t e = l < nl ? s_clist[l] : 0u;
      a = lp.rec16[uint64_t(e & ((1u << kChunkIdBits) - 1)) * kChunk + lane];
    };
    // the kLC chunks at list positions l0, l0 + 1, ... (past the list: no valid lane)
    auto process = [&](uint32_t l0, const uint4 (&a16)[kLC]) {
      uint32_t li[kLC];
      bool valid[kLC];
      uint64_t addr[kLC], ts[kLC], w[kLC];
      XRec xr[kLC];
#pragma unroll
      for (int j = 0; j < kLC; j++) {
        li[j] = l0 + j;
        const uint32_t fill = li[j] < nl ? s_clist[li[j]] >> kChunkIdBits : 0u;
        valid[j] = (uint32_t)lane < fill;
      }
      if (TIMING) {  // (timing: these chunks' loads count as wait; the other group's kLC loads are younger)
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // (kLC)
        nchunks += kLC;
      }
      rt_stamp<TIMING>(rt, 0);
      if (p.flags & kDbgLocalNoWork) {  // (ablation) loads only
#pragma unroll
        for (int j = 0; j < kLC; j++)
          if (lane == 0 && li[j] < nl)
            lp.cmatch[s_clist[li[j]] & ((1u << kChunkIdBits) - 1)] = a16[j].x ^ a16[j].y ^ a16[j].z ^ a16[j].w;
        return;
      }
      // (update_counters of every routed SAMPLE: the route pass).  The common
      // path works on the compact record's offsets: the address from the
      // partition's first key (40 bits), the timestamp from tbase (40 bits).
      // An escaped record (its address, timestamp or weight did not fit) is
      // re-read from the raw record and decided on the exact node record.
      bool esc = false;
#pragma unroll
      for (int j = 0; j < kLC; j++) {
        xr[j] = x_decode_rel(lp.xl, a16[j]);
        esc |= valid[j] && xr[j].esc;
      }
      if (__ballot(esc)) {  // (rare) escaped records: address, timestamp and weight from the record
#pragma unroll
        for (int j = 0; j < kLC; j++)
          if (valid[j] && xr[j].esc) {
            x_resolve(xr[j], lp.xl, p.data, lp.descs);
            xr[j].addr -= k0key;  // (>= 0: routed to this partition); ts stays absolute
          }
        vm_drain();
      }
#pragma unroll
      for (int j = 0; j < kLC; j++) {
        addr[j] = xr[j].addr;  // offset from the partition's first key
        ts[j] = xr[j].ts;      // offset from tbase (escaped: absolute)
        w[j] = valid[j] ? xr[j].w : 0ull;
      }
      rt_stamp<TIMING>(rt, 1);
      // lower bound among the partition's keys (ht_lower_key, tools/hash.c:63-77):
      // the record's address is >= the partition's first key and < the next
      // partition's.  The directory slot gives the largest key <= the slot
      // start, the keys inside the slot and the first kDirInline of their
      // offsets: the answer is that key plus the offsets <= the record's; keys
      // are read only past them (or for a slot whose offsets do not fit).
      int32_t r[kLC];
      uint32_t sa[kLC], sn[kLC];
#pragma unroll
      for (int j = 0; j < kLC; j++) {
        r[j] = -1;
        sa[j] = sn[j] = 0;
        if (valid[j]) {
          const uint32_t slot = (uint32_t)min(addr[j] >> dshift, (uint64_t)(kPartDir - 1));
          const uint4 de = s_dir[slot];
          const uint32_t lo = de.x & 1023u, n = (de.x >> 10) & 2047u;
          uint32_t a = lo, m = n;
          if (n && ((de.x >> 21) & 1u)) {  // inline offsets
            const uint64_t rs64 = addr[j] - (uint64_t(slot) << dshift);
            const uint32_t rs = rs64 >> 16 ? 0x10000u : (uint32_t)rs64;
            const uint32_t c = (uint32_t)((de.y & 0xffffu) <= rs) + (uint32_t)((de.y >> 16) <= rs) +
                               (uint32_t)((de.z & 0xffffu) <= rs) + (uint32_t)((de.z >> 16) <= rs) +
                               (uint32_t)((de.w & 0xffffu) <= rs) + (uint32_t)((de.w >> 16) <= rs);
            a = lo + min(c, n);
            m = (c == kDirInline && n > kDirInline) ? n - kDirInline : 0u;  // past the listed keys: search
          }
          sa[j] = a;  // answer in [a, a + m]: keys[a] <= addr
          sn[j] = m;
          r[j] = 0;
        }
      }
      if (TIMING) {  // (records whose lookup reads keys)
#pragma unroll
        for (int j = 0; j < kLC; j++) rt.acc[11] += (uint64_t)__popcll(__ballot(sn[j] != 0));
      }
#pragma unroll
      for (int j = 0; j < kLC; j++) {
        uint32_t a = sa[j], n = sn[j];
        while (n) {
          const uint32_t half = (n + 1) >> 1;
          if (s_keys[a + half] - k0key <= addr[j]) {
            a += half;
            n -= half;
          } else {
            n = half - 1;
          }
        }
        if (r[j] >= 0) r[j] = (int32_t)a;
      }
      if (TIMING) {  // (the search ends here)
        bool any = false;
#pragma unroll
        for (int j = 0; j < kLC; j++) any |= r[j] >= 0;
        (void)__builtin_amdgcn_readfirstlane(__ballot(any));
      }
      rt_stamp<TIMING>(rt, 2);
      // is_sample_in_buffer (mem_analyzer.c:141-155) on the key's newest
      // entry, from its packed node record: the object starts at the key, so
      // key <= addr < end is addr - first key < end - first key; the dates
      // compare quantised, a timestamp in the quantum of either bound (or an
      // exact-marked key, or an escaped record) is decided on the exact node
      int32_t erel[kLC];
      uint64_t pofs[kLC];  // a match: addr - buffer_addr
      uint32_t hrel[kLC], pnw[kLC], tq[kLC];
      bool older[kLC], amb[kLC];
#pragma unroll
      for (int j = 0; j < kLC; j++) {
        erel[j] = -1;
        pofs[j] = 0;
        hrel[j] = kEmpty32;
        older[j] = false;
        amb[j] = false;
        pnw[j] = 0;
        // (the offsets are < 2^40: the timestamp's quantum fits 32 bits)
        tq[j] = __builtin_amdgcn_alignbit((uint32_t)(ts[j] >> 32), (uint32_t)ts[j], kPnQShift);
        if (r[j] >= 0 && !(p.flags & kDbgLocalNoSearch)) {
          const uint4 pn = s_pn[r[j]];
          const uint2 inf = s_info[r[j]];
          pnw[j] = pn.w;
          const bool in = addr[j] >= (uint64_t)inf.y && addr[j] < (uint64_t)pn.x;
          amb[j] = xr[j].esc || (pn.w & kPnExact) || (in && (tq[j] == pn.y || tq[j] == pn.z));
          if (!amb[j] && in && tq[j] > pn.y && tq[j] < pn.z) {
            erel[j] = (int32_t)(pn.w & 2047u);
            pofs[j] = addr[j] - inf.y;
            hrel[j] = inf.x;
          } else if (!amb[j]) {
            older[j] = (pn.w & kPnOlder) != 0;
          }
        }
      }
      bool anyamb = false;
#pragma unroll
      for (int j = 0; j < kLC; j++) {
        anyamb |= amb[j];
        if (TIMING) rt.acc[10] += (uint64_t)__popcll(__ballot(amb[j]));  // (records decided on the exact node)
      }
      if (__ballot(anyamb)) {  // (rare) the exact node record, from global memory
#pragma unroll
        for (int j = 0; j < kLC; j++) {
          if (!amb[j]) continue;
          const uint64_t fa = k0key + addr[j], ft = xr[j].esc ? ts[j] : lp.xl.tbase + ts[j];
          const uint4* gq = lp.pe_nodes + (uint64_t(q) * kPartSlots + (uint32_t)r[j]) * 2;
          const uint4 na = gq[0], nb = gq[1];
          if (entry_match(na, nb, fa, ft)) {
            erel[j] = (int32_t)(s_pn[r[j]].w & 2047u);
            pofs[j] = fa - u64of(na.x, na.y);
            hrel[j] = s_info[r[j]].x;
          } else {
            older[j] = (s_pn[r[j]].w & kPnOlder) != 0;
          }
        }
        vm_drain();
      }
      bool anyold = false;
#pragma unroll
      for (int j = 0; j < kLC; j++) anyold |= older[j];
      if (__ballot(anyold)) {  // older entries of a reused address (LIFO, tools/hash.c:108-114): the LDS list
#pragma unroll
        for (int j = 0; j < kLC; j++) {
          if (!older[j] || xr[j].esc || !(pnw[j] & kPnOldLds)) continue;
          const uint32_t e = pnw[j] & 2047u, base = e - (uint32_t)r[j], c = (pnw[j] >> kPnOldShift) & 2047u;
          bool glob = false;
          for (uint32_t i = 0; i < c; i++) {
            const uint4 o = s_old[base + i];
            const bool in = addr[j] >= (uint64_t)o.w && addr[j] < (uint64_t)o.x;
            if (in && (tq[j] == o.y || tq[j] == o.z)) {  // (a quantum of either date: the chain decides)
              glob = true;
              break;
            }
            if (in && tq[j] > o.y && tq[j] < o.z) {
              erel[j] = (int32_t)(e + 1 + i);
              pofs[j] = addr[j] - o.w;
              hrel[j] = s_oinf[base + i];
              break;
            }
          }
          older[j] = glob;
        }
        anyold = false;
#pragma unroll
        for (int j = 0; j < kLC; j++) anyold |= older[j];
      }
      if (__ballot(anyold)) {  // (rare) the chain in global memory: escaped records, keys past the list
#pragma unroll
        for (int j = 0; j < kLC; j++) {
          if (!older[j]) continue;
          const uint64_t fa = k0key + addr[j], ft = xr[j].esc ? ts[j] : lp.xl.tbase + ts[j];
          const uint4 d = reinterpret_cast<const uint4*>(p.nodes + pi.k0 + (uint32_t)r[j])[3];  // (count, first)
          uint64_t hist = kHistSparse, baddr = 0;
          const int32_t pos = match_older_pos(p, d.y, d.x, fa, ft, baddr, hist);
          if (pos >= 0) {
            erel[j] = pos - (int32_t)pi.e0;
            pofs[j] = fa - baddr;
            hrel[j] = hist == kHistSparse ? kEmpty32
                      : PACKED && pi.cmap != ~0u ? lp.pe_lrel[pos]
                                         : (uint32_t)(hist - pi.cb);
          }
        }
        vm_drain();
      }
      // the chunks' match bits (per-buffer counts, found_kernel) straight to
      // global memory, and this wave's matched total
#if NMG_LOCAL_ONEMATCH  // (lane j stores chunk j's bits: one store instruction for the group)
      {
        uint64_t mine = 0;
        uint32_t ml = 0;
#pragma unroll
        for (int j = 0; j < kLC; j++) {
          const uint64_t fm = __ballot(erel[j] >= 0);
          nfound += (uint32_t)__popcll(fm);
          mine = lane == j ? fm : mine;
          ml = lane == j ? li[j] : ml;
        }
        if (lane < kLC && ml < nl) lp.cmatch[s_clist[ml] & ((1u << kChunkIdBits) - 1)] = mine;
      }
#else
#pragma unroll
      for (int j = 0; j < kLC; j++) {
        const uint64_t fm = __ballot(erel[j] >= 0);
        nfound += (uint32_t)__popcll(fm);
        if (lane == 0 && li[j] < nl) lp.cmatch[s_clist[li[j]] & ((1u << kChunkIdBits) - 1)] = fm;
      }
#endif
      rt_stamp<TIMING>(rt, 3);
      const bool noobj = (p.flags & kDbgLocalNoObj) != 0;
#pragma unroll
      for (int j = 0; j < kLC; j++) {
        bool ok = erel[j] >= 0 && !noobj && w[j] < kLaneMaxWeight;
        if (ok) atomicAdd(&s_owt[xr[j].acc][erel[j]], (1ull << kPackShift) | w[j]);
      }
      bool anybig = false;
#pragma unroll
      for (int j = 0; j < kLC; j++) anybig |= erel[j] >= 0 && w[j] >= kLaneMaxWeight;
      if (__ballot(anybig) && !noobj) {  // (rare) large weights
        if (lane == 0) s_big = 1;  // (this item's counters are no longer fresh)
#pragma unroll
        for (int j = 0; j < kLC; j++) {
          if (erel[j] < 0 || w[j] < kLaneMaxWeight) continue;
          const uint64_t e = entry_id(lp, pi.e0 + (uint32_t)erel[j]);
          atomicAdd(reinterpret_cast<unsigned long long*>(p.sum64 + objcw_index(e, xr[j].acc, 0, p.nb_entries)), 1ull);
          atomicAdd(reinterpret_cast<unsigned long long*>(p.sum64 + objcw_index(e, xr[j].acc, 1, p.nb_entries)),
                    (unsigned long long)w[j]);
        }
        vm_drain();
      }
      // first match in analysis order (quirk Q7): the compact record's
      // location (buffer index, byte offset) orders as the ordinal does; the
      // flush turns the minimum into (seq << 32) | offset
      if (!noobj) {  // (read first: an unconditional LDS min per match was 9 % slower, hot entries)
        unsigned long long cur[kLC];
#pragma unroll
        for (int j = 0; j < kLC; j++) cur[j] = erel[j] >= 0 ? s_first[erel[j]] : 0ull;
#pragma unroll
        for (int j = 0; j < kLC; j++)
          if (erel[j] >= 0 && xr[j].loc < cur[j]) atomicMin(&s_first[erel[j]], (unsigned long long)xr[j].loc);
      }
      rt_stamp<TIMING>(rt, 4);
      if (pages && !(p.flags & kDbgLocalNoPage)) {
        // ma_get_block: page_no = (int)((addr - buffer_addr) / 4096) (mem_analyzer.c:530-531)
        uint32_t page[kLC];
        bool glob = false, carry[kLC];
#pragma unroll
        for (int j = 0; j < kLC; j++) {
          page[j] = uint32_t(int(pofs[j] / kPageSize));
          carry[j] = false;
          if (erel[j] >= 0 && hrel[j] != kEmpty32 && ncell) {
            const uint32_t c = xr[j].th * pi.span + hrel[j] + page[j], sh = 16 * (c & 1);
            if (kPageCarry) {  // (an item past 2^16 records: a cell could wrap its u16)
              const uint32_t o = atomicAdd(&s_pg[c >> 1], 1u << sh);
              carry[j] = ((o >> sh) & 0xffffu) == kCarryAt - 1;
            } else {
              atomicAdd(&s_pg[c >> 1], 1u << sh);
            }
          }
          glob |= erel[j] >= 0 && (hrel[j] == kEmpty32 || !ncell);
        }
        if (kPageCarry) {
          bool anyc = false;
#pragma unroll
          for (int j = 0; j < kLC; j++) anyc |= carry[j];
          // (rare) a cell reached kCarryAt: kCarryMove of its count go to the
          // histogram in global memory.  Exactly one add brings a cell from
          // kCarryAt - 1 to kCarryAt (only adds raise it, and the move takes it
          // far below), and fewer adds than 2^16 - kCarryAt can be in flight
          // in the workgroup before the move lands: no u16 wraps, no borrow
          // crosses into the neighbouring cell.
          if (__ballot(anyc)) {
            if (lane == 0) s_carry = 1;  // (the flush then adds to the cells instead of storing them)
#pragma unroll
            for (int j = 0; j < kLC; j++) {
              if (!carry[j]) continue;
              const uint32_t rel = hrel[j] + page[j], c = xr[j].th * pi.span + rel;
              atomicSub(&s_pg[c >> 1], kCarryMove << (16 * (c & 1)));
              const uint64_t cell = (PACKED && pi.cmap != ~0u) ? (uint64_t)lp.pe_cmap[pi.cmap + rel] : pi.cb + rel;
              atomicAdd(p.hist + uint64_t(xr[j].th) * p.hist_cells + cell, kCarryMove);
            }
            vm_drain();
          }
        }
        if (__ballot(glob)) {  // (rare) cells in global memory: dense or sparse
#pragma unroll
          for (int j = 0; j < kLC; j++) {
            if (erel[j] < 0) continue;
            if (hrel[j] != kEmpty32 && !ncell) {
              atomicAdd(p.hist + uint64_t(xr[j].th) * p.hist_cells + pi.cb + hrel[j] + page[j], 1u);
            } else if (hrel[j] == kEmpty32) {
              const uint32_t sidx = p.entries[entry_id(lp, pi.e0 + (uint32_t)erel[j])].sidx;
              if (sidx != ~0u)
                sparse_add(p, sparse_key(sidx, xr[j].th, page[j]), lp.seq0 + xr[j].g(lp.xl), xr[j].off(lp.xl), 1u);
            }
          }
          vm_drain();
        }
      }
      rt_stamp<TIMING>(rt, 5);
    };
    uint4 A[kLC], B[kLC];
    auto grab = [&]() -> uint32_t {
      uint32_t t = 0;
      if (lane == 0) t = atomicAdd(&s_cnext, (uint32_t)kLC);
      return __builtin_amdgcn_readfirstlane(t);
    };
    uint32_t la = grab(), lb = grab();
#pragma unroll
    for (int j = 0; j < kLC; j++) chunk_load(la + j, A[j]);
#pragma unroll
    for (int j = 0; j < kLC; j++) chunk_load(lb + j, B[j]);
    while (la < nl) {
      process(la, A);
      la = grab();
#pragma unroll
      for (int j = 0; j < kLC; j++) chunk_load(la + j, A[j]);
      if (lb < nl) process(lb, B);
      lb = grab();
#pragma unroll
      for (int j = 0; j < kLC; j++) chunk_load(lb + j, B[j]);
    }
    // (every wave read this item's index and descriptors before the setup's barrier)
    uint32_t won = 0;
    if (lane == 0) won = atomicExch(&s_took, 1u) == 0 ? 1u : 0u;
    if (__builtin_amdgcn_readfirstlane(won)) take_next();
    lds_sync();
    rt_stamp<TIMING>(rt, 9);  // (waiting for the item's slowest wave)
    // an item alone on its partition whose counters nothing else wrote since
    // the reset (no overflow-path record in this launch, no large weight in
    // this item) stores them without reading: counts and weights from zero,
    // first ordinals from ~0, page cells from zero
    const bool clean = excl && lp.fresh && __builtin_amdgcn_readfirstlane(lp.ctl[3]) == 0;
    const bool clean_obj = clean && __builtin_amdgcn_readfirstlane(s_big) == 0;
    const bool clean_pg = clean && __builtin_amdgcn_readfirstlane(s_carry) == 0;
    // the item's counters to global memory, consecutive lanes on consecutive
    // words, each LDS word zeroed for the next item as it is read; the only
    // item of its partition adds with plain loads and stores (no other
    // workgroup writes these words during the launch), the others with
    // atomics
    for (uint32_t i = tid; i < pi.ne; i += kLWG) {
      const uint64_t e = entry_id(lp, pi.e0 + i);
#pragma unroll
      for (uint32_t a = 0; a < 2; a++) {
        const uint64_t v = s_owt[a][i];
        if (!v) continue;
        s_owt[a][i] = 0;
        const uint64_t cnt = v >> kPackShift, wt = v & ((1ull << kPackShift) - 1);
        uint64_t* pc = p.sum64 + objcw_index(e, a, 0, p.nb_entries);
        uint64_t* pw = p.sum64 + objcw_index(e, a, 1, p.nb_entries);
        if (clean_obj) {
          *pc = cnt;
          if (wt) *pw = wt;
        } else if (excl) {  // (loads past L1: this workgroup's own large-weight atomics went to L2)
          *pc = l2_load(pc) + cnt;
          if (wt) *pw = l2_load(pw) + wt;
        } else {
          atomicAdd(reinterpret_cast<unsigned long long*>(pc), (unsigned long long)cnt);
          if (wt) atomicAdd(reinterpret_cast<unsigned long long*>(pw), (unsigned long long)wt);
        }
      }
      const uint64_t floc = s_first[i];
      if (floc != ~0ull) {
        s_first[i] = ~0ull;
        const uint64_t fo = ((lp.seq0 + (floc >> lp.xl.obits)) << 32) | ((floc & ((1ull << lp.xl.obits) - 1)) << 3);
        uint64_t* pf = p.min64 + 36 + e;
        if (clean) *pf = fo;
        else if (excl) *pf = min(l2_load(pf), fo);
        else atomicMin(reinterpret_cast<unsigned long long*>(pf), (unsigned long long)fo);
      }
    }
    // the cells kU words per thread at a time: every load of the group in
    // flight before the adds are stored (one L2 round trip per group, not per
    // word), the row of a cell by a multiply-high (li * span < 2^32: exact)
    {
      const uint32_t nw = (ncell + 1) / 2, span = pi.span;
      const uint32_t cmap = PACKED ? __builtin_amdgcn_readfirstlane(pi.cmap) : ~0u;
      const uint32_t smag = span ? 0xffffffffu / span + 1u : 0u;
      constexpr uint32_t kU = 4;
      for (uint32_t j0 = tid; j0 < nw; j0 += kU * kLWG) {
        uint32_t cnt[kU][2], old[kU][2];
        uint32_t* pc[kU][2];
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
          const uint32_t j = j0 + u * kLWG;
          const uint32_t v = j < nw ? s_pg[j] : 0u;
          if (v) s_pg[j] = 0;
#pragma unroll
          for (uint32_t h = 0; h < 2; h++) {
            cnt[u][h] = (v >> (16 * h)) & 0xffffu;
            const uint32_t li = 2 * j + h, th = __umulhi(li, smag), rel = li - th * span;
            uint64_t cell = pi.cb + rel;
            if (cmap != ~0u) cell = cnt[u][h] ? lp.pe_cmap[cmap + rel] : 0u;  // (online: packed cells)
            pc[u][h] = p.hist + uint64_t(th) * p.hist_cells + cell;
            old[u][h] = (excl && !clean_pg && cnt[u][h]) ? l2_load(pc[u][h]) : 0u;
          }
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; u++)
#pragma unroll
          for (uint32_t h = 0; h < 2; h++) {
            if (!cnt[u][h]) continue;
            if (excl) *pc[u][h] = old[u][h] + cnt[u][h];
            else atomicAdd(pc[u][h], cnt[u][h]);
          }
      }
    }
    lds_sync();
    rt_stamp<TIMING>(rt, 8);
  }
  if (lane == 0 && nfound) atomicAdd(&s_nfound, nfound);  // (one add to Params::found per workgroup)
  lds_sync();
  if (tid == 0 && s_nfound) atomicAdd(p.found, (unsigned long long)s_nfound);
  if (TIMING && lane == 0) {
    unsigned long long* o = p.dbg + (uint64_t(blockIdx.x) * (kWG / 64) + tid / 64) * kRouteTimingWords;
    for (int k = 0; k < 9; k++) o[k] = rt.acc[k];
    o[9] = nchunks;
    o[10] = nit;
    o[11] = rt.acc[9];
    o[12] = rt.acc[10];
    o[13] = rt.acc[11];
  }
}

// ---------------------------------------------------------------------------
// per-buffer matched-sample counts from the match bits (one workgroup per
// route workgroup: its chunks hold only its own buffers' records)

__global__ __launch_bounds__(kWG) void found_kernel(FoundParams r) {
  __shared__ uint32_t s_found[kFoundLds];
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t w = blockIdx.x;
  const uint32_t g0 = r.ranges[w], nbuf = r.ranges[w + 1] - g0, nl = min(nbuf, kFoundLds);
  for (uint32_t i = tid; i < nl; i += kWG) s_found[i] = 0;
  __syncthreads();
  const uint64_t k0 = uint64_t(r.chunk0[w]) * kChunk, k1 = k0 + uint64_t(r.used[w]) * kChunk;
  const uint64_t gmask = (1ull << r.gbits) - 1;
  // one record per lane, a chunk per wave-instruction: the bit word is a
  // wave-uniform load, the X words stream (bits past a chunk's fill are 0)
  constexpr int kU = 4;
  for (uint64_t k = k0 + tid; k < k1; k += kU * kWG) {
    uint64_t bits[kU], xw[kU];
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const uint64_t kk = k + u * kWG;
      // (a chunk of fill 0 -- route2 opened it and nothing reached it -- was
      // never given to the local pass: its match bits are stale)
      bits[u] = kk < k1 && (r.cmeta[kk / kChunk] >> 24) ? r.cmatch[kk / kChunk] : 0ull;
      xw[u] = ((bits[u] >> lane) & 1) ? reinterpret_cast<const uint64_t*>(r.rec16)[2 * kk + 1] >> r.gshift : 0ull;
    }
#pragma unroll
    for (int u = 0; u < kU; u++) {
      if (!((bits[u] >> lane) & 1)) continue;
      const uint32_t g = (uint32_t)(xw[u] & gmask);
      if (g - g0 < nl) atomicAdd(&s_found[g - g0], 1u);
      else atomicAdd(r.bufcnt + r.nb_bufs + g, 1u);
    }
  }
  __syncthreads();
  for (uint32_t i = tid; i < nl; i += kWG)
    if (s_found[i]) atomicAdd(r.bufcnt + r.nb_bufs + g0 + i, s_found[i]);
}

// ---------------------------------------------------------------------------
// launchers

hipError_t launch_route(uint32_t grid, hipStream_t s, const RouteParams& r) {
  if (r.p.flags & kDbgRouteTiming) hipLaunchKernelGGL(route2_kernel<true>, dim3(grid), dim3(kR2WG), 0, s, r);
  else hipLaunchKernelGGL(route2_kernel<false>, dim3(grid), dim3(kR2WG), 0, s, r);
  return hipGetLastError();
}

hipError_t launch_plan(hipStream_t s, const PlanParams& r) {
  if (r.nparts) hipLaunchKernelGGL(plan_cols_kernel, dim3((r.nparts + 63) / 64), dim3(kWG), 0, s, r);
  hipLaunchKernelGGL(plan_kernel, dim3(1), dim3(kWG), 0, s, r);
  return hipGetLastError();
}

hipError_t launch_overflow(hipStream_t s, const RouteParams& r) {
  hipLaunchKernelGGL(overflow_kernel, dim3(1024), dim3(256), 0, s, r);
  return hipGetLastError();
}

hipError_t launch_count(uint32_t grid, hipStream_t s, const CountParams& r) {
  hipLaunchKernelGGL(count_kernel, dim3(grid), dim3(kWG), 0, s, r);
  return hipGetLastError();
}

hipError_t launch_scatter(uint32_t grid, hipStream_t s, const ScatterParams& r) {
  hipLaunchKernelGGL(scatter_kernel, dim3(grid), dim3(kWG), 0, s, r);
  return hipGetLastError();
}

hipError_t launch_local(uint32_t grid, hipStream_t s, const LocalParams& r) {
  const bool timing = (r.p.flags & kDbgLocalTiming) != 0, packed = r.pe_cmap != nullptr;
  if (packed) {
    if (timing) hipLaunchKernelGGL((local_kernel<true, true>), dim3(grid), dim3(kLWG), 0, s, r);
    else hipLaunchKernelGGL((local_kernel<false, true>), dim3(grid), dim3(kLWG), 0, s, r);
  } else {
    if (timing) hipLaunchKernelGGL((local_kernel<true, false>), dim3(grid), dim3(kLWG), 0, s, r);
    else hipLaunchKernelGGL((local_kernel<false, false>), dim3(grid), dim3(kLWG), 0, s, r);
  }
  return hipGetLastError();
}

hipError_t launch_found(uint32_t grid, hipStream_t s, const FoundParams& r) {
  hipLaunchKernelGGL(found_kernel, dim3(grid), dim3(kWG), 0, s, r);
  return hipGetLastError();
}

}  // namespace nmg
