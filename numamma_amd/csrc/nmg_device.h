// nmg_device.h -- device helpers of the attribution kernels (nmg_kernels.hip):
// wave reductions, the level-bucket mask, record loads, the per-lane global
// counters, hash-bucket slots, the long-tail log, entry matching.
#pragma once

#include "nmg_kernels.h"

namespace nmg {

// ---------------------------------------------------------------------------
// device helpers

// PERF_MEM_LVL_* bits of level group g: L1, L2, L3, LFB, LOC_RAM,
// REM_RAM1|2, REM_CCE1|2, IO, UNC (the bucket order of struct mem_counters,
// mem_analyzer.h:23-40)
__device__ __forceinline__ uint32_t level_mask(int g) {
  return g == 0 ? 0x08u : g == 1 ? 0x20u : g == 2 ? 0x40u : g == 3 ? 0x10u : g == 4 ? 0x80u
       : g == 5 ? 0x300u : g == 6 ? 0xC00u : g == 7 ? 0x1000u : 0x2000u;
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Full-wave u32 sum with DPP (VALU only, no LDS traffic): Hillis-Steele
// within each 16-lane row, then row_bcast:15 / row_bcast:31; lane 63 holds
// the total.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp0(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xf, true);
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  v += dpp0<0x111, 0xf>(v);  // row_shr:1
  v += dpp0<0x112, 0xf>(v);  // row_shr:2
  v += dpp0<0x114, 0xf>(v);  // row_shr:4
  v += dpp0<0x118, 0xf>(v);  // row_shr:8
  v += dpp0<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
  v += dpp0<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
// Inclusive prefix sum over the wave (DPP, the steps of wave_sum_u32)
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
  v += dpp0<0x111, 0xf>(v);  // row_shr:1
  v += dpp0<0x112, 0xf>(v);  // row_shr:2
  v += dpp0<0x114, 0xf>(v);  // row_shr:4
  v += dpp0<0x118, 0xf>(v);  // row_shr:8
  v += dpp0<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
  v += dpp0<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3
  return v;
}
// Sum of per-lane weights; `big` (wave-uniform) = some weight >= 2^26, in
// which case 64 lanes could overflow 32 bits and the u64 path is taken.
__device__ __forceinline__ uint64_t wave_sum_w(uint64_t w, bool big) {
  return big ? wave_sum(w) : (uint64_t)wave_sum_u32((uint32_t)w);
}

// update_counters' level classification (mem_sampling.c:521-591) as an
// 18-bit mask: bit g (0..8) = hit bucket of level group g, bit 9+g = miss.
// Groups: L1, L2, L3, LFB, local RAM, remote RAM 1|2, remote cache 1|2, IO,
// uncached (the bucket order of struct mem_counters).  HIT beats MISS and
// every group is independent (quirk Q12).
__device__ __forceinline__ uint32_t bucket_mask(uint32_t lvl) {
  // group bits from x = lvl >> 3 (L1 L2 L3 LFB LOC_RAM REM_RAM1|2 REM_CCE1|2 IO UNC, from x0 x2 x3
  // x1 x4 x5|x6 x7|x8 x9 x10): six masked moves instead of one shift per bit
  // (lvl < 2^14; equal for every such value)
  const uint32_t x = lvl >> 3, y = x | (x >> 1);
  const uint32_t g = (x & 0x11u) | ((x >> 1) & 0x6u) | ((x & 2u) << 2) | (y & 0x20u) | ((y >> 1) & 0x40u) |
                     ((x >> 2) & 0x180u);
  if (lvl & LVL_HIT) return g;
  if (lvl & LVL_MISS) return g << 9;
  return 0;
}

__device__ __forceinline__ void set_error(const Params& p, uint64_t seq, uint32_t off, uint32_t code) {
  uint64_t w = (seq << 40) | (uint64_t(off) << 8) | code;
  atomicMin(reinterpret_cast<unsigned long long*>(p.min64 + 36 + p.nb_entries),
            (unsigned long long)w);
}

// Descend `levels` levels of an Eytzinger tree (node i has children 2i, 2i+1)
// from the root and return the index below the last level: one 8 B LDS read
// per level (reading three levels per round trip was measured slower: more
// LDS bytes and bank conflicts).  Reads stay below 2^levels.
__device__ __forceinline__ uint32_t eytz_descend(const uint64_t* F, uint32_t levels, uint64_t addr) {
  uint32_t i = 1;
  for (; levels > 0; levels--) i = 2 * i + (F[i] <= addr ? 1u : 0u);
  return i;
}


// __ma_find_mem_info_from_sample_generic (mem_analyzer.c:249-286) with
// is_sample_in_buffer (:141-155): only the lower-bound node, newest entry first.
// Eytzinger node of the largest fence <= addr (0: addr < every fence)
__device__ __forceinline__ uint32_t fence_node(const uint64_t* s_fences, uint64_t addr) {
  const uint32_t i = eytz_descend(s_fences, kFenceLevels, addr);
  return i >> (__builtin_ctz(i) + 1);  // node of the last right turn
}

// in-order rank (bucket) of Eytzinger node idx >= 1 of the complete
// kFenceLevels-level fence tree
__device__ __forceinline__ uint32_t fence_bucket(uint32_t idx) {
  const uint32_t d = 31 - __builtin_clz(idx);
  return (((idx - (1u << d)) * 2 + 1) << (kFenceLevels - 1 - d)) - 1;
}

__device__ __forceinline__ bool entry_match(uint4 a, uint4 b, uint64_t addr, uint64_t ts) {
  const uint64_t baddr = (uint64_t(a.y) << 32) | a.x, bend = (uint64_t(a.w) << 32) | a.z;
  const uint64_t alloc = (uint64_t(b.y) << 32) | b.x, fr = (uint64_t(b.w) << 32) | b.z;
  return baddr <= addr && addr < bend && alloc <= ts && ts <= fr;
}

__device__ __forceinline__ void sparse_add(const Params& p, uint64_t key, uint64_t seq, uint32_t off, uint32_t cnt) {
  *p.sparse_dirty = 1u;
  uint64_t h = (key * 0x9E3779B97F4A7C15ull) >> 20;
  uint32_t slot = uint32_t(h) & p.sparse_mask;
  for (uint32_t probe = 0; probe <= p.sparse_mask; probe++) {
    unsigned long long prev = atomicCAS(reinterpret_cast<unsigned long long*>(p.sparse_keys + slot),
                                        ~0ull, (unsigned long long)key);
    if (prev == ~0ull || prev == key) {
      atomicAdd(p.sparse_vals + slot, cnt);
      return;
    }
    slot = (slot + 1) & p.sparse_mask;
  }
  set_error(p, seq, off, kErrCapacity);
}


__device__ __forceinline__ int bucket_slot(unsigned int* slots8, uint32_t key) {
  const uint4 k0 = reinterpret_cast<const uint4*>(slots8)[0], k1 = reinterpret_cast<const uint4*>(slots8)[1];
  uint32_t k[8] = {k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w};
  int j = -1;
#pragma unroll
  for (int i = 7; i >= 0; i--) j = k[i] == key ? i : j;
  if (j >= 0) return j;
  for (int attempt = 0; attempt < 8; attempt++) {
    int f = -1;
#pragma unroll
    for (int i = 7; i >= 0; i--) f = k[i] == kEmpty32 ? i : f;
    if (f < 0) return -1;
    const unsigned prev = atomicCAS(&slots8[f], kEmpty32, key);
    if (prev == kEmpty32 || prev == key) return f;
#pragma unroll
    for (int i = 0; i < 8; i++) k[i] = i == f ? prev : k[i];
  }
  return -1;
}


// Per-lane privatised mem_counters of the current stream: packed u16 counts
// and u32 weight sums per bucket, plus total count / weight / N/A.  Bounded:
// drained at least every kDrainWindows windows (one record per lane per
// window) and only weights < 2^23 take this path, so nothing overflows
// (256 x 2^23 = 2^31).
constexpr uint32_t kDrainWindows = 256;
constexpr uint64_t kLaneMaxWeight = 1ull << 23;
static_assert((uint64_t)kDensePageWindows * kWG * kLaneMaxWeight < (1ull << kPackShift), "packed weight");
// hashed object slots: flushed at least every kTableWindows windows
static_assert((uint64_t)kTableWindows * kWG < (1ull << (64 - kPackShift)), "packed hashed count");
static_assert((uint64_t)kTableWindows * kWG * kLaneMaxWeight <= (1ull << kPackShift), "packed hashed weight");
// Only the hit buckets of the first kRegGroups level groups (L1, L2, L3: the
// common case in PEBS data) live in registers; the other hit buckets and every
// miss bucket are updated in LDS directly.  (Nine groups in registers left the
// large-table instance 28 B of scratch per lane; three groups: none spilled
// where five still spilled 12 B, and c2 -3 %, k1m -1.5 %.)
constexpr int kRegGroups = 3;
struct LaneAcc {
  uint32_t cnt2[(kRegGroups + 1) / 2];  // counts of hit buckets 2k (low 16 bits) and 2k+1 (high 16 bits)
  uint32_t sum[kRegGroups];
  uint32_t tc, tw, na;
};

__device__ __forceinline__ void lane_acc_clear(LaneAcc& a) {
#pragma unroll
  for (int k = 0; k < (kRegGroups + 1) / 2; k++) a.cnt2[k] = 0;
#pragma unroll
  for (int k = 0; k < kRegGroups; k++) a.sum[k] = 0;
  a.tc = a.tw = a.na = 0;
}

// exact sum over the wave of a u32 per lane (as two 16-bit halves, DPP)
__device__ __forceinline__ uint64_t wave_sum_u32x(uint32_t v) {
  const uint32_t lo = wave_sum_u32(v & 0xffffu), hi = wave_sum_u32(v >> 16);
  return (uint64_t)lo + ((uint64_t)hi << 16);
}

// lanes -> workgroup LDS counters (every lane of the wave calls this)
__device__ __forceinline__ void lane_acc_drain(LaneAcc& a, unsigned long long* sums, int lane) {
  if (__ballot(a.tc != 0) == 0) return;
  const uint64_t tc = wave_sum_u32x(a.tc), tw = wave_sum_u32x(a.tw), na = wave_sum_u32x(a.na);
  if (lane == 0) {
    atomicAdd(&sums[0], (unsigned long long)tc);
    if (tw) atomicAdd(&sums[1], (unsigned long long)tw);
    if (na) atomicAdd(&sums[2], (unsigned long long)na);
  }
#pragma unroll
  for (int k = 0; k < (kRegGroups + 1) / 2; k++) {
    if (__ballot(a.cnt2[k] != 0) == 0) continue;
    const uint32_t c0 = wave_sum_u32(a.cnt2[k] & 0xffffu), c1 = wave_sum_u32(a.cnt2[k] >> 16);
    if (lane == 0) {
      if (c0) atomicAdd(&sums[3 + 2 * (2 * k)], (unsigned long long)c0);
      if (c1 && 2 * k + 1 < kRegGroups) atomicAdd(&sums[3 + 2 * (2 * k + 1)], (unsigned long long)c1);
    }
  }
#pragma unroll
  for (int k = 0; k < kRegGroups; k++) {
    if (__ballot(a.sum[k] != 0) == 0) continue;
    const uint64_t sk = wave_sum_u32x(a.sum[k]);
    if (lane == 0) atomicAdd(&sums[4 + 2 * k], (unsigned long long)sk);
  }
  lane_acc_clear(a);
}


// update_counters(global_counters, sample) (mem_sampling.c:517-592) for one
// SAMPLE of level field `lvl` and weight w: per-lane registers for the common
// buckets, the workgroup's LDS words (sums [kGlobalSums], mins / maxs [18])
// for the rest.
__device__ __forceinline__ void global_count(LaneAcc& acc, unsigned long long* sums, unsigned long long* mins,
                                             unsigned long long* maxs, uint32_t lvl, uint64_t w) {
  const uint32_t bm = bucket_mask(lvl);
  if (w < kLaneMaxWeight) {  // register accumulation (no LDS traffic)
    const uint32_t w32 = (uint32_t)w;
    acc.tc += 1;
    acc.tw += w32;
    acc.na += lvl & LVL_NA;
#pragma unroll
    for (int k = 0; k < (kRegGroups + 1) / 2; k++)
      acc.cnt2[k] += ((bm >> (2 * k)) & 1) | ((2 * k + 1 < kRegGroups ? (bm >> (2 * k + 1)) & 1 : 0) << 16);
#pragma unroll
    for (int k = 0; k < kRegGroups; k++) acc.sum[k] += ((bm >> k) & 1) * w32;
    for (uint32_t m = bm >> kRegGroups; m; m &= m - 1) {  // rarer hit buckets, miss buckets
      const uint32_t b = kRegGroups + (uint32_t)__builtin_ctz(m);
      atomicAdd(&sums[3 + 2 * b], 1ull);
      if (w) atomicAdd(&sums[4 + 2 * b], (unsigned long long)w);
    }
  } else {  // weights >= 2^23 cycles: straight to the LDS counters
    atomicAdd(&sums[0], 1ull);
    atomicAdd(&sums[1], (unsigned long long)w);
    if (lvl & LVL_NA) atomicAdd(&sums[2], 1ull);
    for (uint32_t m = bm; m; m &= m - 1) {
      const uint32_t b = (uint32_t)__builtin_ctz(m);
      atomicAdd(&sums[3 + 2 * b], 1ull);
      atomicAdd(&sums[4 + 2 * b], (unsigned long long)w);
    }
  }
  // min / max only move monotonically: read first, atomic only on improvement
  if (bm) {
    const uint32_t b = (uint32_t)__builtin_ctz(bm);
    if (w < mins[b]) atomicMin(&mins[b], (unsigned long long)w);
    if (w > maxs[b]) atomicMax(&maxs[b], (unsigned long long)w);
    for (uint32_t m = bm & (bm - 1); m; m &= m - 1) {  // several level groups (rare)
      const uint32_t b2 = (uint32_t)__builtin_ctz(m);
      if (w < mins[b2]) atomicMin(&mins[b2], (unsigned long long)w);
      if (w > maxs[b2]) atomicMax(&maxs[b2], (unsigned long long)w);
    }
  }
}

// One long-tail object contribution of this workgroup (kTlogHead layouts,
// nmg_kernels.h) to the sub-log of entry e's range; false when it is full
// (the caller then takes the packed or plain atomics).
__device__ __forceinline__ bool tlog_put(const Params& p, unsigned int* tcur, uint32_t e, uint32_t a, uint32_t cnt,
                                         uint64_t wt, uint64_t ord) {
  const uint32_t part = e >> p.tlog_rshift;
  const bool one = cnt == 1 && wt < (1ull << 32);
  const uint32_t k = atomicAdd(&tcur[part], one ? 1u : 2u);
  if (k >= p.tlog_cap) return false;
  uint4* r = p.tlog + (uint64_t(blockIdx.x) * p.tlog_parts + part) * p.tlog_cap + k;
  const uint32_t ea = e | (a << 31);
  if (one) {
    r[0] = make_uint4(ea, (uint32_t)wt, (uint32_t)ord, (uint32_t)(ord >> 32));
    return true;
  }
  if (k + 1 >= p.tlog_cap) {  // only the last slot left: marked dead (skipped like a continuation)
    r[0] = make_uint4(0, 0, kTlogCont, 0);
    return false;
  }
  r[0] = make_uint4(ea, cnt, kTlogHead, (uint32_t)(ord >> 32));
  r[1] = make_uint4((uint32_t)wt, (uint32_t)(wt >> 32), kTlogCont, (uint32_t)ord);
  return true;
}

// ---------------------------------------------------------------------------
// record loads straight into registers

// One 40 B stride slot: 16 B + 16 B + 8 B loads whose offsets depend on the
// slot's 16 B parity (records are 8-aligned in a 16-aligned buffer), so every
// lane issues the same three instructions.  Decoded only when consumed, so a
// prefetched window stays in flight while the current one is processed.
struct RawRec {
  uint4 x, y;
  uint2 z;
};

__device__ __forceinline__ void load_rec(const uint8_t* base, uint64_t pos, uint64_t len, RawRec& r) {
  if (pos + kRecBytes <= len) {
    const uint32_t odd = uint32_t(pos >> 3) & 1;
    const uint8_t* q = base + pos;
    r.x = *reinterpret_cast<const uint4*>(q + (odd ? 8 : 0));
    r.y = *reinterpret_cast<const uint4*>(q + (odd ? 24 : 16));
    r.z = *reinterpret_cast<const uint2*>(q + (odd ? 0 : 32));
  } else {
    r.x = make_uint4(0, 0, 0, 0);
    r.y = make_uint4(0, 0, 0, 0);
    r.z = make_uint2(0, 0);
  }
}

struct Rec {
  uint64_t hdr, ts, addr, w, dsrc;
};

__device__ __forceinline__ uint64_t u64of(uint32_t lo, uint32_t hi) { return (uint64_t(hi) << 32) | lo; }

__device__ __forceinline__ Rec decode_rec(const RawRec& r, uint64_t pos) {
  Rec d;
  if ((pos >> 3) & 1) {  // hdr | ts addr | w dsrc
    d.hdr = u64of(r.z.x, r.z.y);
    d.ts = u64of(r.x.x, r.x.y);
    d.addr = u64of(r.x.z, r.x.w);
    d.w = u64of(r.y.x, r.y.y);
    d.dsrc = u64of(r.y.z, r.y.w);
  } else {  // hdr ts | addr w | dsrc
    d.hdr = u64of(r.x.x, r.x.y);
    d.ts = u64of(r.x.z, r.x.w);
    d.addr = u64of(r.y.x, r.y.y);
    d.w = u64of(r.y.z, r.y.w);
    d.dsrc = u64of(r.z.x, r.z.y);
  }
  return d;
}


// Workgroup barrier for LDS traffic only: the wave's LDS ops complete before
// it and the other waves' LDS writes are visible after it, while its global
// loads and stores stay in flight across it.  (__syncthreads()'s workgroup
// fence also covers global memory: s_waitcnt vmcnt(0) before every barrier,
// which drains a window's prefetched loads.)  For the kernels whose waves
// exchange data through LDS only.
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// s_waitcnt vmcnt(0) (expcnt / lgkmcnt left alone) as a real waitcnt
// instruction, which the compiler's own waitcnt pass accounts for: a rare
// path that issued global memory ops ends with it, so that the waits on the
// common path after it need not count them
__device__ __forceinline__ void vm_drain() { __builtin_amdgcn_s_waitcnt(0x0f70); }

// shader-clock stamp that the scheduler does not move work across
__device__ __forceinline__ uint64_t stamp() {
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  return t;
}


struct Match {
  int64_t e;       // entry id, -1 = no match
  uint64_t baddr;  // the entry's buffer_addr
  uint64_t hist;   // dense histogram base cell, or kHistSparse
};

__device__ __forceinline__ void match_older(const Params& p, uint32_t first, uint32_t count, uint64_t addr,
                                            uint64_t ts, Match& m) {
  for (uint32_t j = first + 1; j < first + count; j++) {  // older entries of a reused address
    const uint4* r = reinterpret_cast<const uint4*>(p.chain + j);
    const uint4 ra = r[0], rb = r[1];
    if (entry_match(ra, rb, addr, ts)) {
      const uint4 rc = r[2];
      m.e = rc.w;  // DevEntry::id
      m.baddr = (uint64_t(ra.y) << 32) | ra.x;
      m.hist = (uint64_t(rc.y) << 32) | rc.x;
      return;
    }
  }
}


}  // namespace nmg
