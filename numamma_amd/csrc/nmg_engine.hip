// nmg_engine.hip -- MI355X (gfx950) sample-attribution engine + C-ABI.
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
//   * host side: the C-ABI, the stream-sorted schedule, the streaming pipeline
//     (copy stream + double-buffered pinned staging), the reset kernel and the
//     result downloads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "nmg_internal.h"

namespace nmg {

constexpr int kWG = 1024;                      // one workgroup per CU
constexpr uint32_t kSampleType = 9;            // PERF_RECORD_SAMPLE
constexpr uint32_t kRecBytes = 40;             // perf_event_header (8) + struct mem_sample (32)
constexpr uint32_t kWinBytes = kWG * kRecBytes;  // one 40 B stride slot per lane per window
constexpr uint32_t kLdsNodes = 1023;           // keys held in LDS with their node records (<= 10 levels)
// Larger tables: up to 4095 fences (every S-th key) in a 12-level Eytzinger
// tree in LDS, then one load from a per-fence-bucket directory in global memory
constexpr uint32_t kFenceLevels = 12;
constexpr uint32_t kMaxFences = (1u << kFenceLevels) - 1;
constexpr uint32_t kShiftSearch = 0xff;        // bucket without a directory: binary search of its keys
// One LDS region holds the lookup structure of either mode:
//   <= kLdsNodes keys: Eytzinger keys (8 KiB) | node records (32 KiB) | node info (8 KiB)
//   larger tables:     Eytzinger fences (32 KiB) | per-bucket directory shift (4 KiB)
constexpr uint32_t kTabBytes = 48 * 1024;
static_assert((kLdsNodes + 1) * (8 + 32 + 8) <= kTabBytes, "small-table LDS layout");
static_assert((kMaxFences + 1) * (8 + 1) <= kTabBytes, "fence LDS layout");
constexpr uint32_t kMaxList = kWG;             // slow path: SAMPLE offsets listed per step
// per-stream LDS aggregation tables (flushed to global at a stream change and
// on a window cadence)
constexpr uint32_t kObjSlots = 2048;           // entry -> (count, weight, first ordinal)
// long-tail log (hashed object mode): per workgroup, kLogParts sub-logs by
// entry range of 24 B records {entry | access << 31, count, weight, ordinal}
constexpr uint32_t kLogParts = 256;
constexpr uint32_t kLogChunk = 4096;   // entries per LDS pass of tlog_reduce_kernel
constexpr uint32_t kLogMaxGrid = 1024;  // attribution workgroups a log can serve
constexpr uint32_t kPageBuckets = 896;         // dense page cell -> count: 8-slot buckets
constexpr uint32_t kPageSlots = kPageBuckets * 8;  // 7168 cells (56 KiB)
constexpr uint32_t kObjBuckets = kObjSlots / 8;
// hashed (non-dense) tables are flushed at least every kTableWindows windows:
// u32 counts stay far from overflow and the first-come slots are re-learnt
constexpr uint32_t kTableWindows = 256;
// Dense modes (template flags of attribute_kernel):
//   kModeDenseObj:  nb_entries <= kObjSlots: slot = entry id, no key check;
//   kModeDensePage: dense histogram cells per thread <= kDensePageCells: u16
//                   counts, two per LDS word, flushed at least every
//                   kDensePageWindows windows (<= 1024 samples per cell each,
//                   so a u16 cannot overflow into its neighbour)
constexpr int kModeDenseObj = 1, kModeDensePage = 2;
constexpr uint32_t kDensePageCells = kPageSlots * 4;  // the page table's 56 KiB as u16 cells
constexpr uint32_t kDensePageWindows = 62;
#ifdef NMG_NO_PACK_OBJ
constexpr bool kPackObj = false;
#else
constexpr bool kPackObj = true;
#endif
constexpr uint32_t kPackShift = 44;  // kModeDenseObj: per-entry count << 44 | weight sum
static_assert((uint64_t)kDensePageWindows * kWG < (1ull << (64 - kPackShift)), "packed count");
static_assert(kDensePageWindows * kWG < 65536u, "u16 page counts");
constexpr uint32_t kEmpty32 = 0xffffffffu;
constexpr uint64_t kEmpty64 = ~0ull;
// internal ablation switches (tools/ablate.py only; not part of the C-ABI)
constexpr uint32_t kDbgLoadOnly = 0x100;   // stage + validate windows, decode nothing
constexpr uint32_t kDbgNoGlobal = 0x200;   // skip the global mem_counters update
constexpr uint32_t kDbgNoFlush = 0x400;    // LDS tables filled but never written to global
constexpr uint32_t kDbgNoTables = 0x800;   // lookup only: no per-object / per-page accumulation
constexpr uint32_t kDbgTiming = 0x1000;    // per-wave phase cycle counts (tools/phase_timing.py)
constexpr int kTimingWords = 24;           // per wave: load+check, barrier, process, rest, total, windows, -, -,
                                           // then (wave 0) 8 x 2 words of window trace

// PERF_MEM_LVL_* (/usr/include/linux/perf_event.h:1250-1263)
constexpr uint32_t LVL_NA = 0x01, LVL_HIT = 0x02, LVL_MISS = 0x04;
__constant__ uint32_t c_level_mask[9] = {0x08,  0x20,  0x40,  0x10,  0x80,
                                         0x300, 0xC00, 0x1000, 0x2000};
// order: L1, L2, L3, LFB, LOC_RAM, REM_RAM1|2, REM_CCE1|2, IO, UNC
// (the bucket order of struct mem_counters, mem_analyzer.h:23-40)

struct BufDesc {
  uint64_t offset;  // byte offset in the data arena (16-aligned)
  uint32_t len;     // linearised length (< 4 GiB, mem_sampling.c:831-834)
  uint32_t thread_rank;
  uint32_t access;
  uint32_t pad;  // (schedule copy) index of the buffer in submission order
  uint64_t seq;  // analysis-order index (global across shards)
};
static_assert(sizeof(BufDesc) == 32, "BufDesc");

// One table entry (64 B).  The node array holds, for node k, a copy of its
// newest entry with `first` = its entry id and `count` = the node's number of
// entries, so the common one-entry node costs a single dependent load.
struct DevEntry {
  uint64_t addr;   // buffer_addr
  uint64_t end;    // buffer_addr + buffer_size (mod 2^64, as the reference's void* sum)
  uint64_t alloc;  // alloc_date
  uint64_t free;   // free_date
  uint64_t hist;   // dense histogram base cell, or kHistSparse
  uint32_t sidx;   // sparse index (valid when hist == kHistSparse && sidx != ~0u)
  uint32_t first;  // (node records) entry id of the node's newest entry
  uint32_t count;  // (node records) entries of the node
  uint32_t pad0;
  uint64_t pad1;
};
static_assert(sizeof(DevEntry) == 64, "DevEntry");

struct Params {
  const uint8_t* data;
  const BufDesc* sbufs;    // descriptors in schedule order (sorted by stream; .pad = buffer index)
  const uint32_t* ranges;  // [gridDim.x + 1]: workgroup w takes sbufs[ranges[w] .. ranges[w+1])
  uint32_t nb_bufs;
  uint32_t nb_keys;
  const uint64_t* keys;      // [nb_keys] sorted unique keys
  const DevEntry* nodes;     // [nb_keys] node records
  const DevEntry* entries;
  // large tables (nb_keys > kLdsNodes): fence b = keys[b * fence_step]
  const uint64_t* ffences;   // [2^kFenceLevels] fences in Eytzinger order, [0] unused, ~0 padding
  const uint8_t* fshift;     // [nb_fences] slot width log2 of bucket b's directory, or kShiftSearch
  const uint2* dir;          // [nb_fences << dir_log2] {lo | cnt << 16, offset of the slot's first key}
  uint32_t nb_fences;
  uint32_t fence_log2;       // fence_step = 2^fence_log2 keys per bucket
  uint32_t dir_log2;         // directory slots per bucket = 2^dir_log2 (0: fence_step == 1, no directory)
  uint32_t nb_threads;
  uint32_t flags;
  uint32_t nb_entries;
  uint32_t lds_nodes;    // nb_keys <= kLdsNodes: keys + node records in LDS, Eytzinger order
                         // (arrays of kLdsNodes + 1 = 2^10 slots, index 0 unused)
  uint32_t elevels;      // levels of the Eytzinger tree (2^elevels - 1 >= nb_keys)
  const uint64_t* efences;   // [2^elevels] keys in Eytzinger (BFS) order, [0] unused, ~0 padding
  const DevEntry* enodes;    // [2^elevels] node records in the same order
  uint32_t sparse_mask;  // capacity - 1 (power of two)
  uint64_t hist_cells;   // dense cells per thread: histogram index = thread * hist_cells + cell
  uint64_t* sum64;
  uint64_t* min64;
  uint64_t* max64;
  uint32_t* hist;
  uint32_t* bufcnt;  // [2][nb_bufs]: samples, found
  uint64_t* sparse_keys;
  uint32_t* sparse_vals;
  uint32_t* sparse_dirty;  // set on any sparse insert: the next reset must clear the table
  uint32_t* smatch;        // NMG_F_SAMPLE_MATCHES: [(buffer offset + record offset) / 8] = entry + 1, 0 = none
  unsigned long long* dbg;  // kDbgTiming: [grid][waves][kTimingWords]
  // hashed object mode: per-launch packed [2 access][E] (count << pk_shift |
  // weight) for the global path, one atomic instead of two; exact because
  // samples per launch < 2^(64 - pk_shift) and only weights < pk_wlim are
  // packed (their sum < 2^pk_shift); unpack_kernel adds it into sum64
  unsigned long long* pk64;  // null: packing off
  uint32_t pk_shift;
  uint64_t pk_wlim;
  // long-tail log: instead of scattered global atomics, table-full samples
  // and flushed slots append to sub-log (workgroup, entry >> tlog_rshift);
  // tlog_reduce_kernel sums each entry range from LDS.  A full sub-log falls
  // back to the atomics.
  unsigned long long* tlog;  // [grid][tlog_parts][tlog_cap][3] u64; null: off
  uint32_t* tlog_cnt;        // [grid][tlog_parts] records written
  uint32_t tlog_cap, tlog_rshift, tlog_parts;
};

// ---------------------------------------------------------------------------
// device helpers

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
  uint32_t g = ((lvl >> 3) & 1) | (((lvl >> 5) & 1) << 1) | (((lvl >> 6) & 1) << 2) |
               (((lvl >> 4) & 1) << 3) | (((lvl >> 7) & 1) << 4) | ((((lvl >> 8) | (lvl >> 9)) & 1) << 5) |
               ((((lvl >> 10) | (lvl >> 11)) & 1) << 6) | (((lvl >> 12) & 1) << 7) | (((lvl >> 13) & 1) << 8);
  if (lvl & LVL_HIT) return g;
  if (lvl & LVL_MISS) return g << 9;
  return 0;
}

__device__ __forceinline__ void set_error(Params& p, uint64_t seq, uint32_t off, uint32_t code) {
  uint64_t w = (seq << 40) | (uint64_t(off) << 8) | code;
  atomicMin(reinterpret_cast<unsigned long long*>(p.min64 + 36 + p.nb_entries),
            (unsigned long long)w);
}

// Descend `levels` levels of an Eytzinger tree (node i has children 2i, 2i+1)
// from the root and return the index below the last level: one 8 B LDS read
// per level.  (NMG_EYTZ_GROUPED reads node i, its children and grandchildren
// together -- one round trip per three levels -- but the extra LDS bytes and
// bank conflicts cost more than the shorter chain saves.)  Reads stay below
// 2^levels.
__device__ __forceinline__ uint32_t eytz_descend(const uint64_t* F, uint32_t levels, uint64_t addr) {
  uint32_t i = 1;
#ifdef NMG_EYTZ_GROUPED  // measured slower on c2 (0.196 vs 0.182 ms): more LDS bytes and conflicts
  for (; levels >= 3; levels -= 3) {
    const uint64_t k0 = F[i];
    const ulonglong2 k1 = *reinterpret_cast<const ulonglong2*>(F + 2 * i);
    const ulonglong2 k2a = *reinterpret_cast<const ulonglong2*>(F + 4 * i);
    const ulonglong2 k2b = *reinterpret_cast<const ulonglong2*>(F + 4 * i + 2);
    const bool b0 = k0 <= addr;
    const bool b1 = (b0 ? k1.y : k1.x) <= addr;
    const uint64_t kg = b0 ? (b1 ? k2b.y : k2b.x) : (b1 ? k2a.y : k2a.x);
    const bool b2 = kg <= addr;
    i = 8 * i + 4 * (uint32_t)b0 + 2 * (uint32_t)b1 + (uint32_t)b2;
  }
#endif
  for (; levels > 0; levels--) i = 2 * i + (F[i] <= addr ? 1u : 0u);
  return i;
}

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
// equals `addr` (idx 0: none).
struct SpecDir {
  uint64_t addr;
  uint32_t idx;
  uint2 de;
};

__device__ __forceinline__ uint32_t fence_node(const uint64_t* s_fences, uint64_t addr) {
  const uint32_t i = eytz_descend(s_fences, kFenceLevels, addr);
  return i >> (__builtin_ctz(i) + 1);  // node of the last right turn (0: addr < every fence)
}

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
  const bool spec = sp.idx != 0 && sp.addr == addr;
  const uint32_t idx = spec ? sp.idx : fence_node(s_fences, addr);
  if (idx == 0) return p.nb_keys;                    // addr < first key
  // in-order rank of Eytzinger node idx at depth d of a complete tree
  const uint32_t d = 31 - __builtin_clz(idx);
  const uint32_t b = (((idx - (1u << d)) * 2 + 1) << (kFenceLevels - 1 - d)) - 1;
  if (b >= p.nb_fences) return p.nb_keys - 1;  // ~0 padding: addr == UINT64_MAX
  const uint32_t k0 = b << p.fence_log2;
  if (p.dir_log2 == 0) return k0;  // one key per fence
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

// __ma_find_mem_info_from_sample_generic (mem_analyzer.c:249-286) with
// is_sample_in_buffer (:141-155): only the lower-bound node, newest entry first.
__device__ __forceinline__ bool entry_match(uint4 a, uint4 b, uint64_t addr, uint64_t ts) {
  const uint64_t baddr = (uint64_t(a.y) << 32) | a.x, bend = (uint64_t(a.w) << 32) | a.z;
  const uint64_t alloc = (uint64_t(b.y) << 32) | b.x, fr = (uint64_t(b.w) << 32) | b.z;
  return baddr <= addr && addr < bend && alloc <= ts && ts <= fr;
}

__device__ __forceinline__ void sparse_add(Params& p, uint64_t key, uint64_t seq, uint32_t off, uint32_t cnt) {
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

// Per-workgroup privatised counters of the stream (access type, thread rank)
// being analysed.  One stream at a time per workgroup, so (entry) and
// (entry, page) are the keys of the aggregation tables.
struct WgCounters {
  unsigned long long sums[kGlobalSums];  // total_count, total_weight, na, 18 x (count, sum)
  unsigned long long mins[18];
  unsigned long long maxs[18];
  alignas(16) unsigned int okey[kObjSlots];  // entry id, 8 per bucket (hashed modes)
  unsigned int ocnt[kObjSlots];
  unsigned long long ofirst[kObjSlots];  // smallest (seq << 32 | offset): first match
  unsigned long long owt[kObjSlots];
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

__device__ __forceinline__ int page_slot(WgCounters& wc, uint32_t cell) {
  const uint32_t hb = page_bucket(cell);
  const int j = bucket_slot(reinterpret_cast<unsigned int*>(&wc.pkey4[2 * hb]), cell);
  return j < 0 ? -1 : (int)(hb * 8 + (uint32_t)j);
}

// Per-lane privatised mem_counters of the current stream: packed u16 counts
// and u32 weight sums per bucket, plus total count / weight / N/A.  Bounded:
// drained at least every kDrainWindows windows (one record per lane per
// window) and only weights < 2^23 take this path, so nothing overflows
// (256 x 2^23 = 2^31).
constexpr uint32_t kDrainWindows = 256;
constexpr uint64_t kLaneMaxWeight = 1ull << 23;
static_assert((uint64_t)kDensePageWindows * kWG * kLaneMaxWeight < (1ull << kPackShift), "packed weight");
// Only the 9 hit buckets live in registers (the common case in PEBS data);
// miss buckets are updated in LDS directly.
struct LaneAcc {
  uint32_t cnt2[5];  // counts of hit buckets 2k (low 16 bits) and 2k+1 (high 16 bits)
  uint32_t sum[9];
  uint32_t tc, tw, na;
};

__device__ __forceinline__ void lane_acc_clear(LaneAcc& a) {
#pragma unroll
  for (int k = 0; k < 5; k++) a.cnt2[k] = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) a.sum[k] = 0;
  a.tc = a.tw = a.na = 0;
}

// exact sum over the wave of a u32 per lane (as two 16-bit halves, DPP)
__device__ __forceinline__ uint64_t wave_sum_u32x(uint32_t v) {
  const uint32_t lo = wave_sum_u32(v & 0xffffu), hi = wave_sum_u32(v >> 16);
  return (uint64_t)lo + ((uint64_t)hi << 16);
}

// lanes -> workgroup LDS counters (every lane of the wave calls this)
__device__ __forceinline__ void lane_acc_drain(LaneAcc& a, WgCounters& wc, int lane) {
  if (__ballot(a.tc != 0) == 0) return;
  const uint64_t tc = wave_sum_u32x(a.tc), tw = wave_sum_u32x(a.tw), na = wave_sum_u32x(a.na);
  if (lane == 0) {
    atomicAdd(&wc.sums[0], (unsigned long long)tc);
    if (tw) atomicAdd(&wc.sums[1], (unsigned long long)tw);
    if (na) atomicAdd(&wc.sums[2], (unsigned long long)na);
  }
#pragma unroll
  for (int k = 0; k < 5; k++) {
    if (__ballot(a.cnt2[k] != 0) == 0) continue;
    const uint32_t c0 = wave_sum_u32(a.cnt2[k] & 0xffffu), c1 = wave_sum_u32(a.cnt2[k] >> 16);
    if (lane == 0) {
      if (c0) atomicAdd(&wc.sums[3 + 2 * (2 * k)], (unsigned long long)c0);
      if (c1 && 2 * k + 1 < 9) atomicAdd(&wc.sums[3 + 2 * (2 * k + 1)], (unsigned long long)c1);
    }
  }
#pragma unroll
  for (int k = 0; k < 9; k++) {
    if (__ballot(a.sum[k] != 0) == 0) continue;
    const uint64_t sk = wave_sum_u32x(a.sum[k]);
    if (lane == 0) atomicAdd(&wc.sums[4 + 2 * k], (unsigned long long)sk);
  }
  lane_acc_clear(a);
}

// The object table as the kernel sees it: node records in LDS (small tables)
// or in global memory (L2/MALL resident) behind the LDS fence table.
struct Lookup {
  const uint64_t* fences;  // LDS: Eytzinger keys (small tables) or fences (large tables)
  const uint4* nodes;      // LDS (small tables): 2 x uint4 per node: (addr, end), (alloc, free)
  const uint2* ninfo;      // LDS (small tables): (dense histogram base or ~0, entry id | older-entries << 31)
  const uint8_t* shift;    // LDS (large tables): per-bucket directory shift
};

struct Match {
  int64_t e;       // entry id, -1 = no match
  uint64_t baddr;  // the entry's buffer_addr
  uint64_t hist;   // dense histogram base cell, or kHistSparse
};

__device__ __forceinline__ void match_older(const Params& p, uint32_t first, uint32_t count, uint64_t addr,
                                            uint64_t ts, Match& m) {
  for (uint32_t e = first + 1; e < first + count; e++) {  // older entries of a reused address
    const uint4* r = reinterpret_cast<const uint4*>(p.entries + e);
    const uint4 ra = r[0], rb = r[1];
    if (entry_match(ra, rb, addr, ts)) {
      const uint4 rc = r[2];
      m.e = e;
      m.baddr = (uint64_t(ra.y) << 32) | ra.x;
      m.hist = (uint64_t(rc.y) << 32) | rc.x;
      return;
    }
  }
}

// __ma_find_mem_info_from_sample_generic (mem_analyzer.c:249-286): the
// lower-bound node only (ht_lower_key, tools/hash.c:63-77), newest entry
// first, inclusive timestamp window (is_sample_in_buffer, :141-155).
__device__ __forceinline__ Match find_entry(const Params& p, const Lookup& L, uint64_t addr, uint64_t ts,
                                            const SpecDir& sp) {
  Match m;
  m.e = -1;
  m.baddr = 0;
  m.hist = kHistSparse;
  if (p.lds_nodes) {
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
      match_older(p, inf.y & 0x7fffffffu, p.enodes[idx].count, addr, ts, m);
    }
    return m;
  }
  const uint32_t k = lower_key(p, L.fences, L.shift, addr, sp);
  if (k >= p.nb_keys) return m;
  const uint4* q = reinterpret_cast<const uint4*>(p.nodes + k);
  const uint4 a = q[0], b = q[1], c = q[2];
  if (entry_match(a, b, addr, ts)) {
    m.e = c.w;
    m.baddr = (uint64_t(a.y) << 32) | a.x;
    m.hist = (uint64_t(c.y) << 32) | c.x;
    return m;
  }
  const uint4 d = q[3];
  if (d.x > 1) match_older(p, c.w, d.x, addr, ts, m);
  return m;
}

// One long-tail contribution to this workgroup's sub-log of entry e; false
// when the sub-log is full (the caller then issues the global atomics).
__device__ __forceinline__ bool tlog_append(const Params& p, WgCounters& wc, uint32_t e, uint32_t a, uint32_t cnt,
                                            uint64_t wt, uint64_t ord) {
  const uint32_t part = e >> p.tlog_rshift;
  const uint32_t k = atomicAdd(&wc.tcur[part], 1u);
  if (k >= p.tlog_cap) return false;
  unsigned long long* r = p.tlog + ((uint64_t(blockIdx.x) * p.tlog_parts + part) * p.tlog_cap + k) * 3;
  r[0] = (unsigned long long)(e | (a << 31)) | ((unsigned long long)cnt << 32);
  r[1] = wt;
  r[2] = ord;
  return true;
}

// Process one decoded record (`valid` = it is a SAMPLE).  Every lane of the
// wave calls this together (wave-level reductions inside); vmask / fmask are
// the wave's SAMPLE and matched lanes.
template <int MODE>
__device__ __forceinline__ void process_sample(Params& p, WgCounters& wc, LaneAcc& acc, const Lookup& L,
                                               bool valid, uint64_t ts, uint64_t addr,
                                               uint64_t w, uint64_t dsrc, uint32_t access,
                                               uint32_t th, uint64_t seq, uint32_t off, uint64_t rbase,
                                               uint64_t& vmask, uint64_t& fmask, const SpecDir& sp) {
  const uint32_t lvl = uint32_t(dsrc >> 5) & 0x3fff;  // data_src.mem_lvl
  // ---- global counters: update_counters(global_counters, ...) (mem_sampling.c:882)
  vmask = __ballot(valid);
  fmask = 0;
  if (vmask == 0) return;
  if (valid && !(p.flags & kDbgNoGlobal)) {
    const uint32_t bm = bucket_mask(lvl);
    if (w < kLaneMaxWeight) {  // register accumulation (no LDS traffic)
      const uint32_t w32 = (uint32_t)w;
      acc.tc += 1;
      acc.tw += w32;
      acc.na += lvl & LVL_NA;
#pragma unroll
      for (int k = 0; k < 5; k++) acc.cnt2[k] += ((bm >> (2 * k)) & 1) | ((k < 4 ? (bm >> (2 * k + 1)) & 1 : 0) << 16);
#pragma unroll
      for (int k = 0; k < 9; k++) acc.sum[k] += ((bm >> k) & 1) * w32;
      for (uint32_t m = bm >> 9; m; m &= m - 1) {  // miss buckets
        const uint32_t b = 9 + (uint32_t)__builtin_ctz(m);
        atomicAdd(&wc.sums[3 + 2 * b], 1ull);
        if (w) atomicAdd(&wc.sums[4 + 2 * b], (unsigned long long)w);
      }
    } else {  // weights >= 2^23 cycles: straight to the LDS counters
      atomicAdd(&wc.sums[0], 1ull);
      atomicAdd(&wc.sums[1], (unsigned long long)w);
      if (lvl & LVL_NA) atomicAdd(&wc.sums[2], 1ull);
      for (uint32_t m = bm; m; m &= m - 1) {
        const uint32_t b = (uint32_t)__builtin_ctz(m);
        atomicAdd(&wc.sums[3 + 2 * b], 1ull);
        atomicAdd(&wc.sums[4 + 2 * b], (unsigned long long)w);
      }
    }
    // min / max only move monotonically: read first, atomic only on improvement
    if (bm) {
      const uint32_t b = (uint32_t)__builtin_ctz(bm);
      if (w < wc.mins[b]) atomicMin(&wc.mins[b], (unsigned long long)w);
      if (w > wc.maxs[b]) atomicMax(&wc.maxs[b], (unsigned long long)w);
      for (uint32_t m = bm & (bm - 1); m; m &= m - 1) {  // several level groups (rare)
        const uint32_t b2 = (uint32_t)__builtin_ctz(m);
        if (w < wc.mins[b2]) atomicMin(&wc.mins[b2], (unsigned long long)w);
        if (w > wc.maxs[b2]) atomicMax(&wc.maxs[b2], (unsigned long long)w);
      }
    }
  }
  if (!(p.flags & NMG_F_MATCH_SAMPLES)) return;

  // ---- __match_sample (mem_sampling.c:594-673)
  Match m;
  m.e = -1;
  if (valid) m = find_entry(p, L, addr, ts, sp);
  const int64_t e = m.e;
  fmask = __ballot(e >= 0);
  // dump modes: every SAMPLE record's match at its arena position (host
  // formats the per-sample lines in analysis order)
  if (p.smatch && valid) p.smatch[(rbase + off) >> 3] = e >= 0 ? (uint32_t)e + 1u : 0u;
  if (e < 0 || (p.flags & kDbgNoTables)) return;
  // per-object counters, aggregated per stream in LDS.  (Admitting an entry
  // only on its second sample -- a doorkeeper bitset -- was measured slower at
  // 1M intervals: the per-sample bit test costs more than the flushes it saves.)
  // (with packing, a slot only sums packable weights: its flush is packed too)
  const bool pk = !(MODE & kModeDenseObj) && p.pk64 && w < p.pk_wlim;
  const int os = (MODE & kModeDenseObj) ? (int)e : ((p.pk64 && !pk) ? -1 : obj_slot(wc, (uint32_t)e));
  const unsigned long long ord = (seq << 32) | off;  // first match in analysis order (quirk Q7)
  if ((MODE & kModeDenseObj) && w < kLaneMaxWeight && kPackObj) {
    // one packed add: count in bits 44..63, weight below (bounded by the
    // kDensePageWindows flush cadence: < 2^16 samples of < 2^23 each)
    atomicAdd(&wc.owt[os], (1ull << kPackShift) | w);
    if (ord < wc.ofirst[os]) atomicMin(&wc.ofirst[os], ord);
  } else if (os >= 0 && !((MODE & kModeDenseObj) && kPackObj)) {
    atomicAdd(&wc.ocnt[os], 1u);
    if (w) atomicAdd(&wc.owt[os], (unsigned long long)w);
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
        else atomicAdd(p.hist + uint64_t(th) * p.hist_cells + cell, 1u);
      }
    } else {
      const uint32_t sidx = p.entries[e].sidx;
      if (sidx != ~0u)  // huge objects ([stack]): hashed cells in global memory
        sparse_add(p, sparse_key(sidx, th, page), seq, off, 1u);
    }
  }
  if (p.flags & NMG_F_OBJECT_LEVELS) {
    unsigned long long* lv = reinterpret_cast<unsigned long long*>(
        p.sum64 + 2 * kGlobalSums + uint64_t(p.nb_entries) * 4 + (uint64_t(e) * 2 + access) * kLevelWords);
    if (lvl & LVL_NA) atomicAdd(lv, 1ull);
    for (int g = 0; g < 9; g++) {
      if (!(lvl & c_level_mask[g])) continue;
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
    constexpr bool packed = (MODE & kModeDenseObj) && kPackObj;
    if ((MODE & kModeDenseObj) ? (packed ? wc.owt[i] == 0 : wc.ocnt[i] == 0) : e == kEmpty32) continue;
    const uint64_t cnt = packed ? wc.owt[i] >> kPackShift : wc.ocnt[i];
    const uint64_t wt = packed ? wc.owt[i] & ((1ull << kPackShift) - 1) : wc.owt[i];
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
    wc.ocnt[i] = 0;
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
    wc.ocnt[i] = 0;
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
#ifdef NMG_NT_LOADS
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(q + (odd ? 8 : 0)));
    const u32x4 b = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(q + (odd ? 24 : 16)));
    const u32x2 c = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(q + (odd ? 0 : 32)));
    r.x = make_uint4(a.x, a.y, a.z, a.w);
    r.y = make_uint4(b.x, b.y, b.z, b.w);
    r.z = make_uint2(c.x, c.y);
#else
    r.x = *reinterpret_cast<const uint4*>(q + (odd ? 8 : 0));
    r.y = *reinterpret_cast<const uint4*>(q + (odd ? 24 : 16));
    r.z = *reinterpret_cast<const uint2*>(q + (odd ? 0 : 32));
#endif
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

// shader-clock stamp that the scheduler does not move work across
__device__ __forceinline__ uint64_t stamp() {
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

template <bool TIMING, int MODE>
__global__ __launch_bounds__(kWG, 1) void attribute_kernel(Params p) {
  __shared__ uint4 s_tab[kTabBytes / 16];  // lookup structure (layouts at kTabBytes)
  __shared__ uint32_t s_list[kMaxList];
  __shared__ WgCounters wc;
  __shared__ uint32_t s_flags[3], s_nlist, s_next, s_err;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  uint64_t* const s_fences = reinterpret_cast<uint64_t*>(s_tab);
  uint4* const s_nodes = s_tab + (kLdsNodes + 1) / 2;                    // after 8 KiB of keys
  uint2* const s_ninfo = reinterpret_cast<uint2*>(s_tab + (kLdsNodes + 1) * 5 / 2);  // after 40 KiB
  uint8_t* const s_shift = reinterpret_cast<uint8_t*>(s_tab + (kMaxFences + 1) / 2);  // after 32 KiB
  if (p.lds_nodes) {
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
  __syncthreads();
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
  uint64_t tacc[4] = {0, 0, 0, 0}, t_start = 0, t0 = 0, t1 = 0;
  if (TIMING) t_start = t0 = stamp();
#ifndef NMG_NO_SPEC_DIR
  constexpr bool kSpec = !(MODE & kModeDenseObj);  // large tables come with the hashed object mode
#else
  constexpr bool kSpec = false;
#endif
  SpecDir sp;
  sp.addr = 0;
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
    __syncthreads();
    // (LDS broadcasts are made wave-uniform explicitly: the branches below
    // hold barriers and steer the scalar loop state)
    const uint32_t f = __builtin_amdgcn_readfirstlane(s_flags[win % 3]);
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
    uint64_t rseq, rbase;
    uint32_t roff;
    if (!(f & 1)) {
      valid = wl.cand && uint32_t(r.hdr) == kSampleType;
      rseq = wl.in1 ? d1.seq : d0.seq;
      rbase = wl.in1 ? d1.offset : d0.offset;
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
            if (lane == 0) s_list[n] = (uint32_t)q0;
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
      __syncthreads();
      const uint32_t n = __builtin_amdgcn_readfirstlane(s_nlist);
      const uint32_t serr = __builtin_amdgcn_readfirstlane(s_err);
      ncur = serr ? len : __builtin_amdgcn_readfirstlane(s_next);  // the reference aborts on an error: stop this buffer
      if (ncur >= len) {
        nidx = idx + 1;
        ncur = 0;
      }
      valid = (uint32_t)tid < n;
      roff = valid ? s_list[tid] : 0;
      rseq = d0.seq;
      rbase = d0.offset;
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

    if (TIMING && tid == 0 && win <= 8) {
      unsigned long long* o = p.dbg + uint64_t(blockIdx.x) * (kWG / 64) * kTimingWords + 8 + 2 * (win - 1);
      o[0] = (uint64_t(idx) << 40) | cur;
      o[1] = uint64_t(wl.n0) | (uint64_t(wl.n1) << 11) | (uint64_t(f) << 22) | (uint64_t(nidx) << 24) |
             (uint64_t((uint32_t)ncur) << 32);
    }
    uint64_t vm = 0, fm = 0;
    if (!(p.flags & kDbgLoadOnly))
      process_sample<MODE>(p, wc, acc, L, valid, rec.ts, rec.addr, rec.w, rec.dsrc, d0.access, d0.thread_rank, rseq, roff,
                           rbase, vm, fm, sp);
    if (kSpec && !p.lds_nodes && (p.flags & NMG_F_MATCH_SAMPLES)) {
      // start the next window's lookup: its record (loaded above, arrived
      // during this window's lookups) -> fence node -> directory slot load,
      // in flight across the flush and the barrier.  Used when the record
      // this lane processes next has the same address (fast-path windows).
      sp.idx = 0;
      if (nidx < r1 && ncand) {
        sp.addr = decode_rec(nx, npos).addr;
        sp.idx = fence_node(L.fences, sp.addr);
        const uint2* ds = dir_slot(p, L.fences, L.shift, sp.addr, sp.idx);
        if (ds) sp.de = *ds;
      }
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
    }
    // end of the stream run (or of this workgroup's range): publish the
    // stream's counters; tables over their fill threshold (as of this
    // window's barrier) are flushed here too -- the single flush site
    const bool stream_end = nidx != idx && (nidx >= r1 || nd0.access != cur_access || nd0.thread_rank != cur_thread);
    if (++acc_windows == kDrainWindows || stream_end) {  // keep the per-lane u32 sums bounded
      lane_acc_drain(acc, wc, lane);
      acc_windows = 0;
    }
    if (nidx != idx) {
      // buffer idx (and idx + 1 when skipped over) done: sample / match
      // tallies (mem_sampling.c:921-926)
      if (lane == 0) {
        if (ns0) atomicAdd(p.bufcnt + d0.pad, ns0);
        if (nf0) atomicAdd(p.bufcnt + p.nb_bufs + d0.pad, nf0);
        if (nidx == idx + 2) {
          if (ns1) atomicAdd(p.bufcnt + d1.pad, ns1);
          if (nf1) atomicAdd(p.bufcnt + p.nb_bufs + d1.pad, nf1);
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
      __syncthreads();  // every insert and drain of this window is done
      if (stream_end) flush_sums(p, wc, tid, cur_access);
      flush_objects<MODE>(p, wc, tid, cur_access);
      flush_pages<MODE>(p, wc, tid, cur_thread);
      last_flush = win;
      __syncthreads();
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
  if (kLog && p.tlog) {  // the sub-logs' fill (every append of this workgroup is done)
    __syncthreads();
    for (uint32_t i = tid; i < p.tlog_parts; i += kWG)
      p.tlog_cnt[uint64_t(blockIdx.x) * p.tlog_parts + i] = min(wc.tcur[i], p.tlog_cap);
  }
  if (TIMING && lane == 0) {
    unsigned long long* o = p.dbg + (uint64_t(blockIdx.x) * (kWG / 64) + tid / 64) * kTimingWords;
    for (int k = 0; k < 4; k++) o[k] = tacc[k];
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
struct TlogParams {
  const unsigned long long* tlog;
  const uint32_t* tlog_cnt;
  uint64_t* sum64;
  uint64_t* min64;
  unsigned long long* pk64;  // may be null
  uint32_t grid, parts, cap, rshift, nb_entries, pk_shift;
};

__global__ __launch_bounds__(1024, 1) void tlog_reduce_kernel(TlogParams r) {
  __shared__ uint32_t s_cnt[2][kLogChunk];
  __shared__ unsigned long long s_wt[2][kLogChunk];
  __shared__ unsigned long long s_ord[kLogChunk];
  __shared__ uint32_t s_pre[kLogMaxGrid + 1];
  const uint32_t part = blockIdx.x, tid = threadIdx.x;
  for (uint32_t w = tid; w < r.grid; w += 1024) s_pre[w + 1] = r.tlog_cnt[uint64_t(w) * r.parts + part];
  __syncthreads();
  if (tid < 64) {  // prefix over the source workgroups: a chunk per lane, then a wave scan
    const uint32_t per = (r.grid + 63) / 64, b = min(tid * per, r.grid), e = min(b + per, r.grid);
    uint32_t sum = 0;
    for (uint32_t w = b; w < e; w++) sum += s_pre[w + 1];
    uint32_t incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o, 64);
      if ((int)tid >= o) incl += t;
    }
    uint32_t run = incl - sum;
    for (uint32_t w = b; w < e; w++) {
      run += s_pre[w + 1];
      s_pre[w + 1] = run;
    }
    if (tid == 0) s_pre[0] = 0;
  }
  __syncthreads();
  const uint32_t total = s_pre[r.grid];
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
    constexpr int kU = 4;  // records per thread in flight
    for (uint32_t i0 = tid; i0 < total; i0 += kU * 1024) {
      unsigned long long kv[kU], wv[kU], ov[kU];
#pragma unroll
      for (int u = 0; u < kU; u++) {
        const uint32_t i = i0 + u * 1024;
        kv[u] = ~0ull;  // (no record: entry ids are < 2^31)
        if (i >= total) continue;
        uint32_t lo = 0, hi = r.grid;  // source workgroup: s_pre[lo] <= i < s_pre[lo + 1]
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (s_pre[mid] <= i) lo = mid;
          else hi = mid;
        }
        const unsigned long long* q = r.tlog + ((uint64_t(lo) * r.parts + part) * r.cap + (i - s_pre[lo])) * 3;
        kv[u] = q[0];
        wv[u] = q[1];
        ov[u] = q[2];
      }
#pragma unroll
      for (int u = 0; u < kU; u++) {
        if (kv[u] == ~0ull) continue;
        const uint32_t e = uint32_t(kv[u]) & 0x7fffffffu, a = uint32_t(kv[u]) >> 31;
        const uint64_t j = e - base;
        if (e < base || j >= n) continue;
        atomicAdd(&s_cnt[a][j], uint32_t(kv[u] >> 32));
        if (wv[u]) atomicAdd(&s_wt[a][j], wv[u]);
        atomicMin(&s_ord[j], ov[u]);
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
struct ResetParams {
  uint64_t* sum64;
  uint64_t n_sum64;
  uint64_t* min64;
  uint64_t n_min64;
  uint64_t* max64;
  uint64_t n_max64;
  uint4* hist;  // zeroed in 16 B units
  uint64_t n_hist16;
  uint64_t* sparse_keys;
  uint32_t* sparse_vals;
  uint64_t sparse_cap;
  const uint32_t* sparse_read;  // dirty flag of the analyses since the previous reset
  uint32_t* sparse_clear;       // the flag the analyses after this reset will set
  uint32_t* bufcnt;
  uint64_t n_bufcnt;
};

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
}

}  // namespace nmg

// ===========================================================================
// host side

using namespace nmg;

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
  uint64_t nlaunch = 0;
  int num_cus = 256;
  int blocks_per_cu = 0;
  bool launched = false;

  // object table
  bool have_table = false;
  uint32_t K = 0, E = 0;
  uint64_t* d_keys = nullptr;
  DevEntry* d_nodes = nullptr;
  uint64_t* d_efences = nullptr;  // small tables: Eytzinger-ordered keys / node records
  DevEntry* d_enodes = nullptr;
  uint32_t elevels = 0;
  DevEntry* d_entries = nullptr;
  uint64_t* d_ffences = nullptr;  // large tables: Eytzinger fences, directory shifts, directory
  uint8_t* d_fshift = nullptr;
  uint2* d_dir = nullptr;
  uint32_t nb_fences = 0, fence_log2 = 0, dir_log2 = 0;
  std::vector<uint64_t> hist_base, npages, buffer_size, entry_addr;
  std::vector<nmg_object> objects;  // the table as given (all_memory_objects.dat)
  std::vector<uint32_t> sparse_entries;
  uint64_t hist_cells = 0;
  uint64_t hist_budget = 4ull << 30;
  uint64_t sparse_cap = 1u << 20;

  // counters
  uint64_t *d_sum64 = nullptr, *d_min64 = nullptr, *d_max64 = nullptr;
  uint64_t n_sum64 = 0, n_min64 = 0, n_max64 = 0;
  uint32_t* d_hist = nullptr;
  uint64_t* d_sparse_keys = nullptr;
  uint32_t* d_sparse_vals = nullptr;
  uint32_t* d_sparse_dirty = nullptr;  // [2] parity flags (see reset_kernel)
  uint32_t* d_smatch = nullptr;        // NMG_F_SAMPLE_MATCHES: per 8 B of the arena span
  unsigned long long* d_pk64 = nullptr;  // hashed object mode: packed long-tail counters (0 between launches)
  unsigned long long* d_tlog = nullptr;  // hashed object mode: long-tail log (see Params::tlog)
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
  uint32_t sched_grid = 0;       // grid the current schedule was built for
  bool descs_dirty = false;
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

static int fail(nmg_engine* h, int code, const std::string& msg) {
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

extern "C" int nmg_get_last_error_detail(nmg_engine* h, char* buf, size_t len) {
  if (!h || !buf || !len) return NMG_ERR_INVALID;
  snprintf(buf, len, "%s", h->last_error.c_str());
  return NMG_OK;
}

static void free_counters(nmg_engine* h) {
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

static void free_table(nmg_engine* h) {
  (void)hipFree(h->d_keys);
  (void)hipFree(h->d_nodes);
  (void)hipFree(h->d_efences);
  (void)hipFree(h->d_enodes);
  h->d_efences = nullptr;
  h->d_enodes = nullptr;
  (void)hipFree(h->d_entries);
  (void)hipFree(h->d_ffences);
  (void)hipFree(h->d_fshift);
  (void)hipFree(h->d_dir);
  h->d_keys = nullptr;
  h->d_nodes = nullptr;
  h->d_entries = nullptr;
  h->d_ffences = nullptr;
  h->d_fshift = nullptr;
  h->d_dir = nullptr;
}

extern "C" int nmg_create(nmg_engine** out, const nmg_options* opt) {
  if (!out) return NMG_ERR_INVALID;
  *out = nullptr;
  nmg_engine* h = new (std::nothrow) nmg_engine();
  if (!h) return NMG_ERR_NOMEM;
  if (opt) {
    h->device = opt->device;
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
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || h->device < 0 || h->device >= ndev) {
    delete h;
    return NMG_ERR_HIP;
  }
  if (hipSetDevice(h->device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess) {
    delete h;
    return NMG_ERR_HIP;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, h->device) == hipSuccess) h->num_cus = prop.multiProcessorCount;
  *out = h;
  return NMG_OK;
}

extern "C" void nmg_destroy(nmg_engine* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  free_table(h);
  free_counters(h);
  (void)hipFree(h->d_arena);
  (void)hipFree(h->d_descs);
  (void)hipFree(h->d_bufcnt);
  (void)hipFree(h->d_sdescs);
  (void)hipFree(h->d_ranges);
  (void)hipFree(h->d_dbg);
  (void)hipFree(h->d_smatch);
  if (h->h_stage) (void)hipHostFree(h->h_stage);
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
  }
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

extern "C" int nmg_reset_counters(nmg_engine* h) {
  if (!h) return NMG_ERR_INVALID;
  if (!h->have_table) return fail(h, NMG_ERR_STATE, "nmg_reset_counters before nmg_set_objects");
  HIP_TRY(h, hipSetDevice(h->device));
  ResetParams r;
  memset(&r, 0, sizeof(r));
  r.sum64 = h->d_sum64;
  r.n_sum64 = h->n_sum64;
  r.min64 = h->d_min64;
  r.n_min64 = h->n_min64;
  r.max64 = h->d_max64;
  r.n_max64 = h->n_max64;
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
  hipLaunchKernelGGL(reset_kernel, dim3(rgrid), dim3(256), 0, h->stream, r);
  h->nreset++;
  HIP_TRY(h, hipGetLastError());
  return NMG_OK;
}

// Lookup structure of a table larger than kLdsNodes keys (see lower_key):
// fence b = keys[b << fence_log2] (<= kMaxFences fences, Eytzinger order),
// and per bucket a directory of 2^dir_log2 equal-width slots over the bucket's
// key span [first key, last key].
struct BigLookup {
  uint32_t nb_fences = 0, fence_log2 = 0, dir_log2 = 0;
  std::vector<uint64_t> efences;  // [kMaxFences + 1]
  std::vector<uint8_t> shift;     // [nb_fences]
  std::vector<uint2> dir;         // [nb_fences << dir_log2]
};

static void build_big_lookup(const uint64_t* keys, uint32_t K, BigLookup& bl) {
  while (((uint64_t)K + (1u << bl.fence_log2) - 1) >> bl.fence_log2 > kMaxFences) bl.fence_log2++;
  const uint32_t S = 1u << bl.fence_log2;
  bl.nb_fences = (uint32_t)(((uint64_t)K + S - 1) >> bl.fence_log2);
  // Eytzinger order: an in-order walk of the complete 12-level tree hands out
  // the fences in sorted order; the slots after the last fence hold ~0
  bl.efences.assign(kMaxFences + 1, ~0ull);
  {
    uint32_t r = 0, i = 1;
    std::vector<uint32_t> stack;
    while (i <= kMaxFences || !stack.empty()) {
      while (i <= kMaxFences) {
        stack.push_back(i);
        i = 2 * i;
      }
      i = stack.back();
      stack.pop_back();
      if (r < bl.nb_fences) bl.efences[i] = keys[(uint64_t)r << bl.fence_log2];
      r++;
      i = 2 * i + 1;
    }
  }
  bl.shift.assign(bl.nb_fences, kShiftSearch);
  // bucket-relative indices and counts are 16-bit: S <= 2^16
  if (S == 1 || S > (1u << 16)) return;
  bl.dir_log2 = bl.fence_log2 + 1;  // two slots per key
  const uint32_t D = 1u << bl.dir_log2;
  bl.dir.assign((size_t)bl.nb_fences << bl.dir_log2, make_uint2(0, 0));
  for (uint32_t b = 0; b < bl.nb_fences; b++) {
    const uint32_t k0 = b * S, k1 = std::min<uint64_t>((uint64_t)k0 + S, K);
    const uint64_t f = keys[k0], span = keys[k1 - 1] - f;
    uint32_t sh = 0;
    while (sh < 64 && (span >> sh) >= D) sh++;
    if (sh > 32) continue;  // slot offsets must fit 32 bits: binary search instead
    bl.shift[b] = (uint8_t)sh;
    uint2* dd = &bl.dir[(size_t)b << bl.dir_log2];
    uint32_t k = k0;  // largest key <= slot start
    for (uint32_t j = 0; j < D; j++) {
      const uint64_t s0 = (uint64_t)j << sh;  // slot [s0, s0 + 2^sh) relative to f; the last slot is open
      while (k + 1 < k1 && keys[k + 1] - f <= s0) k++;
      uint32_t c = 0;
      while (k + 1 + c < k1 && (j == D - 1 || keys[k + 1 + c] - f < s0 + (1ull << sh))) c++;
      dd[j].x = (k - k0) | (std::min<uint32_t>(c, 0xffffu) << 16);
      dd[j].y = c ? (uint32_t)(keys[k + 1] - f - s0) : 0u;
    }
  }
}

extern "C" int nmg_set_objects(nmg_engine* h, const uint64_t* keys, const uint32_t* entry_off,
                               uint32_t nb_keys, const nmg_object* entries, uint32_t nb_entries) {
  if (!h || (nb_keys && (!keys || !entry_off)) || (nb_entries && !entries))
    return NMG_ERR_INVALID;
  if (entry_off && (entry_off[0] != 0 || entry_off[nb_keys] != nb_entries))
    return fail(h, NMG_ERR_INVALID, "entry_off[0] must be 0 and entry_off[nb_keys] == nb_entries");
  for (uint32_t i = 0; i < nb_keys; i++) {
    if (entry_off[i + 1] <= entry_off[i]) return fail(h, NMG_ERR_INVALID, "every key needs >= 1 entry");
    if (i && keys[i] <= keys[i - 1]) return fail(h, NMG_ERR_INVALID, "keys must be strictly ascending");
  }
  if (nb_entries >= (1u << 31)) return fail(h, NMG_ERR_RANGE, "too many entries");
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  free_table(h);
  free_counters(h);
  h->K = nb_keys;
  h->E = nb_entries;

  // page-histogram layout: dense [page][thread] block per entry within the
  // budget, otherwise sparse hashed cells (e.g. the 412 GB [stack] range)
  const uint64_t T = h->T;
  const uint64_t max_cells_per_entry = 1ull << 24;
  h->hist_base.assign(nb_entries, kHistSparse);
  h->npages.resize(nb_entries);
  h->buffer_size.resize(nb_entries);
  h->entry_addr.resize(nb_entries);
  h->objects.assign(entries, entries + nb_entries);
  h->sparse_entries.clear();
  h->hist_cells = 0;
  std::vector<DevEntry> dev(nb_entries);
  const bool want_hist = (h->flags & NMG_F_PAGE_HIST) && (h->flags & NMG_F_MATCH_SAMPLES);
  const uint64_t budget_cells = h->hist_budget / 4;
  for (uint32_t e = 0; e < nb_entries; e++) {
    const nmg_object& o = entries[e];
    DevEntry& d = dev[e];
    memset(&d, 0, sizeof(d));
    d.addr = o.buffer_addr;
    d.end = o.buffer_addr + o.buffer_size;
    d.alloc = o.alloc_date;
    d.free = o.free_date;
    uint64_t np = o.buffer_size / kPageSize + 1;
    h->npages[e] = np;
    h->buffer_size[e] = o.buffer_size;
    h->entry_addr[e] = o.buffer_addr;
    d.hist = kHistSparse;
    d.sidx = ~0u;
    if (!want_hist) continue;
    // dense cells: histogram index = thread * hist_cells + hist_base(entry) + page
    if (np * T <= max_cells_per_entry && (h->hist_cells + np) * T <= budget_cells &&
        h->hist_cells + np < 0xffffffffull) {
      d.hist = h->hist_cells;
      h->hist_base[e] = h->hist_cells;
      h->hist_cells += np;
    } else {
      if (h->sparse_entries.size() >= (1u << 22)) return fail(h, NMG_ERR_CAPACITY, "too many sparse entries");
      d.sidx = (uint32_t)h->sparse_entries.size();
      h->sparse_entries.push_back(e);
    }
  }
  std::vector<DevEntry> nodes(nb_keys);
  for (uint32_t k = 0; k < nb_keys; k++) {
    nodes[k] = dev[entry_off[k]];
    nodes[k].first = entry_off[k];
    nodes[k].count = entry_off[k + 1] - entry_off[k];
  }

  auto alloc_copy = [&](void** dptr, const void* src, size_t bytes) -> hipError_t {
    hipError_t e = hipMalloc(dptr, bytes ? bytes : 16);
    if (e != hipSuccess) return e;
    if (bytes) return hipMemcpyAsync(*dptr, src, bytes, hipMemcpyHostToDevice, h->stream);
    return hipSuccess;
  };
  HIP_TRY(h, alloc_copy((void**)&h->d_keys, keys, (size_t)nb_keys * 8));
  HIP_TRY(h, alloc_copy((void**)&h->d_nodes, nodes.data(), (size_t)nb_keys * sizeof(DevEntry)));
  if (nb_keys <= kLdsNodes) {
    // Eytzinger (BFS) order for the LDS search: an in-order walk of the
    // complete tree of 2^L - 1 nodes hands out the keys in sorted order; the
    // slots after the last key are ~0 keys carrying a copy of the last node
    // (reached only for addr == UINT64_MAX, where the last key is the answer)
    h->elevels = 0;
    while (((1u << h->elevels) - 1) < nb_keys) h->elevels++;
    const uint32_t n = 1u << h->elevels;
    std::vector<uint64_t> ef(n, ~0ull);
    std::vector<DevEntry> en(n);
    memset(en.data(), 0, n * sizeof(DevEntry));
    uint32_t r = 0;
    std::vector<uint32_t> stack;
    uint32_t i = 1;
    while (i < n || !stack.empty()) {  // iterative in-order walk
      while (i < n) {
        stack.push_back(i);
        i = 2 * i;
      }
      i = stack.back();
      stack.pop_back();
      if (r < nb_keys) {
        ef[i] = keys[r];
        en[i] = nodes[r];
      } else if (nb_keys) {
        en[i] = nodes[nb_keys - 1];
      }
      r++;
      i = 2 * i + 1;
    }
    HIP_TRY(h, alloc_copy((void**)&h->d_efences, ef.data(), n * 8));
    HIP_TRY(h, alloc_copy((void**)&h->d_enodes, en.data(), n * sizeof(DevEntry)));
  }
  h->nb_fences = h->fence_log2 = h->dir_log2 = 0;
  if (nb_keys > kLdsNodes) {
    BigLookup bl;
    build_big_lookup(keys, nb_keys, bl);
    h->nb_fences = bl.nb_fences;
    h->fence_log2 = bl.fence_log2;
    h->dir_log2 = bl.dir_log2;
    HIP_TRY(h, alloc_copy((void**)&h->d_ffences, bl.efences.data(), bl.efences.size() * 8));
    HIP_TRY(h, alloc_copy((void**)&h->d_fshift, bl.shift.data(), bl.shift.size()));
    HIP_TRY(h, alloc_copy((void**)&h->d_dir, bl.dir.data(), bl.dir.size() * sizeof(uint2)));
  }
  HIP_TRY(h, alloc_copy((void**)&h->d_entries, dev.data(), (size_t)nb_entries * sizeof(DevEntry)));

  h->n_sum64 = 2 * kGlobalSums + (uint64_t)nb_entries * 4;
  if (h->flags & NMG_F_OBJECT_LEVELS) h->n_sum64 += (uint64_t)nb_entries * 2 * kLevelWords;
  h->n_min64 = 36 + (uint64_t)nb_entries + 1;
  h->n_max64 = 36;
  HIP_TRY(h, hipMalloc(&h->d_sum64, h->n_sum64 * 8));
  HIP_TRY(h, hipMalloc(&h->d_min64, h->n_min64 * 8));
  HIP_TRY(h, hipMalloc(&h->d_max64, h->n_max64 * 8));
  if (nb_entries > kObjSlots) {  // hashed object mode (see launch_attribution)
    HIP_TRY(h, hipMalloc(&h->d_pk64, (size_t)nb_entries * 2 * 8));
    HIP_TRY(h, hipMemset(h->d_pk64, 0, (size_t)nb_entries * 2 * 8));
  }
  // pad the dense arena to a multiple of 4 cells per thread so it is zeroed in 16 B units
  h->hist_cells = (h->hist_cells + 3) & ~uint64_t(3);
  if (h->hist_cells) HIP_TRY(h, hipMalloc(&h->d_hist, h->hist_cells * h->T * 4));
  if (!h->sparse_entries.empty()) {
    HIP_TRY(h, hipMalloc(&h->d_sparse_keys, h->sparse_cap * 8));
    HIP_TRY(h, hipMalloc(&h->d_sparse_vals, h->sparse_cap * 4));
    HIP_TRY(h, hipMalloc(&h->d_sparse_dirty, 2 * 4));
    const uint32_t ones[2] = {1u, 1u};  // the first reset clears the fresh table
    HIP_TRY(h, hipMemcpy(h->d_sparse_dirty, ones, 8, hipMemcpyHostToDevice));
  }
  h->have_table = true;
  HIP_TRY(h, hipStreamSynchronize(h->stream));
  return nmg_reset_counters(h);
}

static int stage_reserve(nmg_engine* h, size_t need) {
  if (need <= h->stage_cap) return NMG_OK;
  size_t cap = std::max(need, h->stage_cap * 2 + (1u << 20));
  uint8_t* p = nullptr;
  HIP_TRY(h, hipHostMalloc((void**)&p, cap, hipHostMallocDefault));
  if (h->stage_len) memcpy(p, h->h_stage, h->stage_len);
  if (h->h_stage) {
    HIP_TRY(h, hipStreamSynchronize(h->stream));
    (void)hipHostFree(h->h_stage);
  }
  h->h_stage = p;
  h->stage_cap = cap;
  return NMG_OK;
}

static int append_desc(nmg_engine* h, uint64_t len, uint32_t thread_rank, uint32_t access) {
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
  return NMG_OK;
}

static int check_buffer_args(nmg_engine* h, uint64_t len, uint32_t thread_rank, uint32_t access) {
  if (access > 1) return fail(h, NMG_ERR_INVALID, "access_type must be 0 (read) or 1 (write)");
  if (thread_rank >= h->T)
    return fail(h, NMG_ERR_RANGE, "thread_rank >= nb_threads (set nmg_options.nb_threads)");
  if (len >= (1ull << 32)) return fail(h, NMG_ERR_RANGE, "buffer >= 4 GiB (unsigned cursors, mem_sampling.c:831-834)");
  if (h->external) return fail(h, NMG_ERR_STATE, "device buffers are set; call nmg_clear_buffers first");
  if (h->streamed && !h->streaming) return fail(h, NMG_ERR_STATE, "stream ended; call nmg_clear_buffers first");
  return NMG_OK;
}

// a host copy into pinned staging, run by one of the copy threads
struct CopyTask {
  uint8_t* dst;
  const uint8_t* src;
  uint64_t len;
};
static int stream_dst(nmg_engine* h, uint64_t len, uint8_t** dst, std::vector<CopyTask>* pending);
static void ensure_occupancy(nmg_engine* h);
static void make_schedule(const std::vector<BufDesc>& descs, uint32_t grid, uint32_t index_base, BufDesc* sorted,
                          uint32_t* ranges);
static int launch_attribution(nmg_engine* h, const uint8_t* data, const BufDesc* sdescs, const uint32_t* ranges,
                              uint32_t nb, uint32_t grid, uint64_t nbytes);
static int stream_append(nmg_engine* h, uint64_t len, uint32_t thread_rank, uint32_t access);

extern "C" int nmg_submit_buffer(nmg_engine* h, const void* bytes, uint64_t len, uint32_t thread_rank,
                                 uint32_t access_type) {
  if (!h || (len && !bytes)) return NMG_ERR_INVALID;
  int rc = check_buffer_args(h, len, thread_rank, access_type);
  if (rc) return rc;
  if (len == 0) return NMG_OK;  // __copy_buffer drops empty segments (mem_sampling.c:680-682)
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

static void run_copies(nmg_engine* h, const std::vector<CopyTask>& tasks) {
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
static int slot_acquire(nmg_engine* h, int s) {
  auto& sl = h->slots[s];
  if (sl.used) HIP_TRY(h, hipEventSynchronize(sl.copied));
  sl.len = 0;
  sl.descs.clear();
  return NMG_OK;
}

// per-buffer count array for `need` buffers; its stride stays fixed while
// chunks are in flight (grown by doubling after draining the engine stream)
static int ensure_bufcnt(nmg_engine* h, size_t need) {
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
static int stream_flush(nmg_engine* h) {
  auto& sl = h->slots[h->cur_slot];
  if (sl.descs.empty()) return NMG_OK;
  const uint32_t nb = (uint32_t)sl.descs.size();
  ensure_occupancy(h);
  const uint32_t grid = std::min<uint32_t>(nb, (uint32_t)(h->num_cus * h->blocks_per_cu));
  int rc = ensure_bufcnt(h, h->descs.size());
  if (rc) return rc;
  const size_t sched_bytes = nb * sizeof(BufDesc) + (grid + 1) * 4;
  if (sched_bytes > sl.hs_cap) {  // (slot acquired: its previous H2D is done)
    if (sl.h_sdescs) (void)hipHostFree(sl.h_sdescs);
    sl.h_sdescs = nullptr;
    sl.hs_cap = std::max<size_t>(sched_bytes * 2, 64 << 10);
    HIP_TRY(h, hipHostMalloc((void**)&sl.h_sdescs, sl.hs_cap, hipHostMallocDefault));
  }
  const uint32_t index_base = (uint32_t)(h->descs.size() - nb);
  uint32_t* h_ranges = reinterpret_cast<uint32_t*>(sl.h_sdescs + nb);
  make_schedule(sl.descs, grid, index_base, sl.h_sdescs, h_ranges);
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
  rc = launch_attribution(h, sl.d_arena, sl.d_sdescs, reinterpret_cast<const uint32_t*>(sl.d_sdescs + nb), nb, grid,
                          sl.len);
  if (rc) return rc;
  HIP_TRY(h, hipEventRecord(sl.done, h->stream));
  sl.used = true;
  // switch halves; the next submit refills the other one once its H2D is done
  h->cur_slot ^= 1;
  return slot_acquire(h, h->cur_slot);
}

// Destination in the open chunk for `len` bytes; flushes the chunk first when
// it is full (running the batch's pending copies into it before the upload).
static int stream_dst(nmg_engine* h, uint64_t len, uint8_t** dst, std::vector<CopyTask>* pending) {
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

static int stream_append(nmg_engine* h, uint64_t len, uint32_t thread_rank, uint32_t access) {
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
  h->buf_bytes.swap(bytes);
  h->d_data = (const uint8_t*)d_data;
  h->external = true;
  h->staged_dirty = false;
  h->descs_dirty = true;
  h->stage_len = 0;
  return NMG_OK;
}

extern "C" int nmg_clear_buffers(nmg_engine* h) {
  if (!h) return NMG_ERR_INVALID;
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
  h->descs.clear();
  h->buf_bytes.clear();
  h->stage_len = 0;
  h->external = false;
  h->d_data = nullptr;
  h->descs_dirty = true;
  h->counts_override = false;
  return NMG_OK;
}

static int upload_buffers(nmg_engine* h) {
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
      HIP_TRY(h, hipMemcpyAsync(h->d_descs, h->descs.data(), n * sizeof(BufDesc), hipMemcpyHostToDevice, h->stream));
      HIP_TRY(h, hipMemsetAsync(h->d_bufcnt, 0, n * 2 * 4, h->stream));
      HIP_TRY(h, hipStreamSynchronize(h->stream));  // descs come from pageable memory
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
static void make_schedule(const std::vector<BufDesc>& descs, uint32_t grid, uint32_t index_base, BufDesc* sorted,
                          uint32_t* ranges) {
  const uint32_t nb = (uint32_t)descs.size();
  std::vector<uint32_t> order(nb);
  for (uint32_t i = 0; i < nb; i++) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
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

static int build_schedule(nmg_engine* h, uint32_t grid) {
  const uint32_t nb = (uint32_t)h->descs.size();
  std::vector<uint32_t> ranges(grid + 1, 0);
  std::vector<BufDesc> sorted(nb);
  make_schedule(h->descs, grid, 0, sorted.data(), ranges.data());
  (void)hipFree(h->d_sdescs);
  (void)hipFree(h->d_ranges);
  h->d_sdescs = nullptr;
  h->d_ranges = nullptr;
  HIP_TRY(h, hipMalloc(&h->d_sdescs, std::max<size_t>(nb, 1) * sizeof(BufDesc)));
  HIP_TRY(h, hipMalloc(&h->d_ranges, (grid + 1) * 4));
  if (nb) HIP_TRY(h, hipMemcpy(h->d_sdescs, sorted.data(), nb * sizeof(BufDesc), hipMemcpyHostToDevice));
  HIP_TRY(h, hipMemcpy(h->d_ranges, ranges.data(), (grid + 1) * 4, hipMemcpyHostToDevice));
  h->sched_grid = grid;
  return NMG_OK;
}

typedef void (*AttributeKernel)(Params);
static AttributeKernel kernel_for(bool timing, int mode) {
  static const AttributeKernel k[2][4] = {
      {attribute_kernel<false, 0>, attribute_kernel<false, 1>, attribute_kernel<false, 2>, attribute_kernel<false, 3>},
      {attribute_kernel<true, 0>, attribute_kernel<true, 1>, attribute_kernel<true, 2>, attribute_kernel<true, 3>}};
  return k[timing ? 1 : 0][mode & 3];
}

static void ensure_occupancy(nmg_engine* h) {
  if (h->blocks_per_cu <= 0) {
    int bpc = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, attribute_kernel<false, 0>, kWG, 0) != hipSuccess || bpc <= 0) bpc = 1;
    h->blocks_per_cu = bpc;
  }
}

// One attribution launch over `nb` buffers whose stream-sorted descriptors and
// per-workgroup ranges are already on the device, on the engine stream,
// bracketed by the launch-timing events.
static int launch_attribution(nmg_engine* h, const uint8_t* data, const BufDesc* sdescs, const uint32_t* ranges,
                              uint32_t nb, uint32_t grid, uint64_t nbytes) {
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
  p.sparse_keys = h->d_sparse_keys;
  p.sparse_vals = h->d_sparse_vals;
  p.sparse_dirty = h->d_sparse_dirty ? h->d_sparse_dirty + (h->nreset & 1) : nullptr;
  p.smatch = (h->flags & NMG_F_SAMPLE_MATCHES) ? h->d_smatch : nullptr;
  // dense LDS tables when the table is small enough (DESIGN.md "Kernels")
  const int mode = (h->E <= kObjSlots ? kModeDenseObj : 0) |
                   (h->hist_cells <= kDensePageCells ? kModeDensePage : 0);
#ifndef NMG_NO_PACK_TAIL
  if (!(mode & kModeDenseObj) && h->d_pk64) {
    // < 2^cbits samples in this launch (a SAMPLE record is 40 B); packed
    // weights < 2^(64 - 2 cbits), so any entry's packed sum < 2^(64 - cbits)
    const uint32_t cbits = 64 - (uint32_t)__builtin_clzll(nbytes / kRecBytes + 1);
    if (2 * cbits < 64) {
      p.pk64 = h->d_pk64;
      p.pk_shift = 64 - cbits;
      p.pk_wlim = 1ull << (64 - 2 * cbits);
    }
  }
#endif
#ifndef NMG_NO_TAIL_LOG
  if (!(mode & kModeDenseObj) && nb && grid <= kLogMaxGrid && (h->flags & NMG_F_MATCH_SAMPLES) &&
      nbytes / kRecBytes < (1ull << 31)) {
    uint32_t rshift = 0;
    while ((((uint64_t)h->E + (1ull << rshift) - 1) >> rshift) > kLogParts) rshift++;
    const uint32_t parts = (uint32_t)(((uint64_t)h->E + (1ull << rshift) - 1) >> rshift);
    // sized for about every sample of the launch spread evenly; a full
    // sub-log only sends its overflow to the atomics
    const uint64_t cap = std::min<uint64_t>(1u << 20, (nbytes / kRecBytes) / ((uint64_t)grid * parts) + 32);
    const size_t need = (size_t)grid * parts * cap * 24;
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
#endif
  const int slot = (int)(h->nlaunch % nmg_engine::kRing);
  if (!h->ring0[slot]) {
    HIP_TRY(h, hipEventCreate(&h->ring0[slot]));
    HIP_TRY(h, hipEventCreate(&h->ring1[slot]));
  }
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
      hipLaunchKernelGGL(kernel_for(true, mode), dim3(grid), dim3(kWG), 0, h->stream, p);
    } else {
      hipLaunchKernelGGL(kernel_for(false, mode), dim3(grid), dim3(kWG), 0, h->stream, p);
    }
    HIP_TRY(h, hipGetLastError());
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
      hipLaunchKernelGGL(tlog_reduce_kernel, dim3(p.tlog_parts), dim3(1024), 0, h->stream, r);
      HIP_TRY(h, hipGetLastError());
    } else if (p.pk64) {
      const uint32_t blocks = (uint32_t)std::min<uint64_t>(2048, (2ull * h->E + 255) / 256);
      hipLaunchKernelGGL(unpack_kernel, dim3(blocks), dim3(256), 0, h->stream, h->d_sum64, p.pk64, h->E,
                         p.pk_shift);
      HIP_TRY(h, hipGetLastError());
    }
  }
  HIP_TRY(h, hipEventRecord(h->ring1[slot], h->stream));
  h->nlaunch++;
  h->launched = true;
  return NMG_OK;
}

static int stream_flush(nmg_engine* h);

extern "C" int nmg_analyze(nmg_engine* h) {
  if (!h) return NMG_ERR_INVALID;
  if (!h->have_table) return fail(h, NMG_ERR_STATE, "nmg_analyze before nmg_set_objects");
  HIP_TRY(h, hipSetDevice(h->device));
  if (h->streaming) return stream_flush(h);  // earlier chunks are already enqueued
  if (h->streamed) return NMG_OK;             // nmg_stream_end flushed everything
  const bool resched = h->descs_dirty;
  int rc = upload_buffers(h);
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
  ensure_occupancy(h);
  // persistent grid: one resident workgroup per slot, each with a byte-balanced range
  const uint32_t grid = nb ? std::min<uint32_t>(nb, (uint32_t)(h->num_cus * h->blocks_per_cu)) : 0;
  if (nb && (resched || grid != h->sched_grid)) {
    rc = build_schedule(h, grid);
    if (rc) return rc;
  }
  uint64_t nbytes = 0;
  for (const BufDesc& d : h->descs) nbytes += d.len;
  return launch_attribution(h, h->d_data, h->d_sdescs, h->d_ranges, nb, grid, nbytes);
}

static int decode_error_word(nmg_engine* h, uint64_t w) {
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
    default: return fail(h, NMG_ERR_RANGE, std::string(msg) + "range error");
  }
}

extern "C" int nmg_synchronize(nmg_engine* h) {
  if (!h) return NMG_ERR_INVALID;
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

extern "C" int nmg_last_analyze_ms(nmg_engine* h, float* ms) {
  if (!h || !ms) return NMG_ERR_INVALID;
  *ms = h->last_ms;
  return NMG_OK;
}

extern "C" uint32_t nmg_get_nb_buffers(nmg_engine* h) {
  if (!h) return 0;
  return h->counts_override ? (uint32_t)h->ov_samples.size() : (uint32_t)h->descs.size();
}

namespace nmg {
int engine_download(nmg_engine* h, HostResults& r) {
  int rc = nmg_synchronize(h);
  if (rc) return rc;
  std::vector<uint64_t> sum(h->n_sum64), mn(h->n_min64), mx(h->n_max64);
  HIP_TRY(h, hipMemcpy(sum.data(), h->d_sum64, h->n_sum64 * 8, hipMemcpyDeviceToHost));
  HIP_TRY(h, hipMemcpy(mn.data(), h->d_min64, h->n_min64 * 8, hipMemcpyDeviceToHost));
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
  const uint64_t E = h->E;
  r.first.assign(mn.begin() + 36, mn.begin() + 36 + E);
  r.count_weight.resize(4 * E);  // SoA [2][2][E] -> [E][2][2]
  for (uint64_t e = 0; e < E; e++)
    for (uint32_t a = 0; a < 2; a++)
      for (uint32_t w = 0; w < 2; w++) r.count_weight[e * 4 + a * 2 + w] = sum[objcw_index(e, a, w, E)];
  if (h->flags & NMG_F_OBJECT_LEVELS)
    r.levels.assign(sum.begin() + 2 * kGlobalSums + 4 * E, sum.end());
  else
    r.levels.clear();
  if (h->counts_override) {
    r.buf_samples = h->ov_samples;
    r.buf_found = h->ov_found;
    r.buf_bytes = h->ov_bytes;
  } else {
    const size_t n = h->descs.size();
    r.buf_samples.assign(n, 0);
    r.buf_found.assign(n, 0);
    if (n) {
      HIP_TRY(h, hipMemcpy(r.buf_samples.data(), h->d_bufcnt, n * 4, hipMemcpyDeviceToHost));
      HIP_TRY(h, hipMemcpy(r.buf_found.data(), h->d_bufcnt + h->bufcnt_stride, n * 4, hipMemcpyDeviceToHost));
    }
    r.buf_bytes = h->buf_bytes;
  }
  // mem_sampling_finalize accumulates the per-buffer int counters (:334-335)
  r.nb_samples_total = 0;
  r.nb_found_total = 0;
  for (size_t b = 0; b < r.buf_samples.size(); b++) {
    r.nb_samples_total += (uint64_t)(int64_t)(int32_t)r.buf_samples[b];
    r.nb_found_total += (uint64_t)(int64_t)(int32_t)r.buf_found[b];
  }
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
  int rc = engine_download(h, r);
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
  int rc = engine_download(h, r);
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
  if (count_weight && h->E) {
    std::vector<uint64_t> soa((size_t)h->E * 4);
    HIP_TRY(h, hipMemcpy(soa.data(), h->d_sum64 + 2 * kGlobalSums, soa.size() * 8, hipMemcpyDeviceToHost));
    for (uint64_t e = 0; e < h->E; e++)
      for (uint32_t a = 0; a < 2; a++)
        for (uint32_t w = 0; w < 2; w++)
          count_weight[e * 4 + a * 2 + w] = soa[objcw_index(e, a, w, h->E) - 2 * kGlobalSums];
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

static int collect_page_cells(nmg_engine* h, std::vector<uint32_t>* rows, int64_t* count) {
  std::vector<uint32_t> cells;
  int rc = engine_download_hist(h, cells);
  if (rc) return rc;
  // sparse cells grouped per entry
  std::vector<std::vector<std::pair<uint64_t, uint32_t>>> sparse(h->sparse_entries.size());
  if (h->d_sparse_keys) {
    std::vector<uint64_t> k(h->sparse_cap);
    std::vector<uint32_t> v(h->sparse_cap);
    HIP_TRY(h, hipMemcpy(k.data(), h->d_sparse_keys, h->sparse_cap * 8, hipMemcpyDeviceToHost));
    HIP_TRY(h, hipMemcpy(v.data(), h->d_sparse_vals, h->sparse_cap * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < k.size(); i++)
      if (k[i] != ~0ull && v[i]) {
        uint32_t s = sparse_key_idx(k[i]);
        // order within an entry: (thread, page)
        sparse[s].push_back({(uint64_t(sparse_key_thread(k[i])) << 32) | sparse_key_page(k[i]), v[i]});
      }
    for (auto& l : sparse) std::sort(l.begin(), l.end());
  }
  std::vector<int64_t> sidx_of(h->E, -1);
  for (size_t s = 0; s < h->sparse_entries.size(); s++) sidx_of[h->sparse_entries[s]] = (int64_t)s;
  int64_t n = 0;
  const uint64_t T = h->T;
  for (uint32_t e = 0; e < h->E; e++) {
    if (h->hist_base[e] != kHistSparse) {
      for (uint32_t th = 0; th < T; th++)
        for (uint64_t pg = 0; pg < h->npages[e]; pg++) {
          uint32_t v = cells[th * h->hist_cells + h->hist_base[e] + pg];
          if (!v) continue;
          if (rows) {
            rows->push_back(e);
            rows->push_back(th);
            rows->push_back((uint32_t)pg);
            rows->push_back(v);
          }
          n++;
        }
    } else if (sidx_of[e] >= 0) {
      for (auto& kv : sparse[sidx_of[e]]) {
        if (rows) {
          rows->push_back(e);
          rows->push_back((uint32_t)(kv.first >> 32));
          rows->push_back((uint32_t)kv.first);
          rows->push_back(kv.second);
        }
        n++;
      }
    }
  }
  *count = n;
  return NMG_OK;
}

extern "C" int64_t nmg_count_page_cells(nmg_engine* h) {
  if (!h || !h->have_table) return NMG_ERR_INVALID;
  int64_t n = 0;
  int rc = collect_page_cells(h, nullptr, &n);
  return rc ? rc : n;
}

extern "C" int nmg_get_page_cells(nmg_engine* h, uint32_t* rows, int64_t n) {
  if (!h || !h->have_table || (n && !rows)) return NMG_ERR_INVALID;
  std::vector<uint32_t> r;
  int64_t cnt = 0;
  int rc = collect_page_cells(h, &r, &cnt);
  if (rc) return rc;
  if (cnt != n) return fail(h, NMG_ERR_INVALID, "row count mismatch");
  if (n) memcpy(rows, r.data(), r.size() * 4);
  return NMG_OK;
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

static void* array_ptr(nmg_engine* h, int which, size_t* bytes) {
  switch (which) {
    case NMG_ARR_SUM64: *bytes = h->n_sum64 * 8; return h->d_sum64;
    case NMG_ARR_MIN64: *bytes = h->n_min64 * 8; return h->d_min64;
    case NMG_ARR_MAX64: *bytes = h->n_max64 * 8; return h->d_max64;
    case NMG_ARR_HIST32: *bytes = h->hist_cells * h->T * 4; return h->d_hist;
    default: *bytes = 0; return nullptr;
  }
}

extern "C" int nmg_export_array(nmg_engine* h, int which, void* d_dst) {
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

static int sparse_download(nmg_engine* h, std::vector<uint64_t>& k, std::vector<uint32_t>& v) {
  int rc = nmg_synchronize(h);
  if (rc) return rc;
  if (!h->d_sparse_keys) {
    k.clear();
    v.clear();
    return NMG_OK;
  }
  std::vector<uint64_t> kk(h->sparse_cap);
  std::vector<uint32_t> vv(h->sparse_cap);
  HIP_TRY(h, hipMemcpy(kk.data(), h->d_sparse_keys, h->sparse_cap * 8, hipMemcpyDeviceToHost));
  HIP_TRY(h, hipMemcpy(vv.data(), h->d_sparse_vals, h->sparse_cap * 4, hipMemcpyDeviceToHost));
  k.clear();
  v.clear();
  for (size_t i = 0; i < kk.size(); i++)
    if (kk[i] != ~0ull && vv[i]) {
      k.push_back(kk[i]);
      v.push_back(vv[i]);
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
  memcpy(keys, k.data(), n * 8);
  memcpy(counts, v.data(), n * 4);
  return NMG_OK;
}

extern "C" int nmg_sparse_import(nmg_engine* h, const uint64_t* keys, const uint32_t* counts, int64_t n) {
  // Re-inserts merged (key, count) pairs into an empty table on this rank.
  if (!h || !h->have_table || (n && (!keys || !counts))) return NMG_ERR_INVALID;
  if (!h->d_sparse_keys) return n ? fail(h, NMG_ERR_STATE, "no sparse table") : NMG_OK;
  if ((uint64_t)n > h->sparse_cap) return fail(h, NMG_ERR_CAPACITY, "sparse table too small");
  std::vector<uint64_t> k(h->sparse_cap, ~0ull);
  std::vector<uint32_t> v(h->sparse_cap, 0);
  for (int64_t i = 0; i < n; i++) {
    uint64_t hh = (keys[i] * 0x9E3779B97F4A7C15ull) >> 20;
    uint64_t slot = hh & (h->sparse_cap - 1);
    while (k[slot] != ~0ull && k[slot] != keys[i]) slot = (slot + 1) & (h->sparse_cap - 1);
    k[slot] = keys[i];
    v[slot] += counts[i];
  }
  HIP_TRY(h, hipSetDevice(h->device));
  HIP_TRY(h, hipMemcpy(h->d_sparse_keys, k.data(), h->sparse_cap * 8, hipMemcpyHostToDevice));
  HIP_TRY(h, hipMemcpy(h->d_sparse_vals, v.data(), h->sparse_cap * 4, hipMemcpyHostToDevice));
  const uint32_t one = 1;  // imported cells: the next reset must clear the table
  HIP_TRY(h, hipMemcpy(h->d_sparse_dirty + (h->nreset & 1), &one, 4, hipMemcpyHostToDevice));
  return NMG_OK;
}

extern "C" int nmg_set_buffer_counts(nmg_engine* h, uint32_t nb_buffers, const uint32_t* nb_samples,
                                     const uint32_t* nb_found, const uint64_t* buffer_bytes) {
  if (!h || (nb_buffers && (!nb_samples || !nb_found || !buffer_bytes))) return NMG_ERR_INVALID;
  h->counts_override = true;
  h->ov_samples.assign(nb_samples, nb_samples + nb_buffers);
  h->ov_found.assign(nb_found, nb_found + nb_buffers);
  h->ov_bytes.assign(buffer_bytes, buffer_bytes + nb_buffers);
  return NMG_OK;
}

extern "C" int nmg_report(nmg_engine* h, const nmg_object_meta* meta, const nmg_report_options* opts,
                          const char* stdout_path) {
  if (!h || (h->E && !meta)) return NMG_ERR_INVALID;
  if (!h->have_table) return fail(h, NMG_ERR_STATE, "nmg_report before nmg_set_objects");
  HostResults r;
  int rc = engine_download(h, r);
  if (rc) return rc;
  std::vector<uint32_t> rows;
  int64_t ncells = 0;
  if ((h->flags & NMG_F_PAGE_HIST) && (!opts || opts->dump_single_items)) {
    rc = collect_page_cells(h, &rows, &ncells);
    if (rc) return rc;
  }
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
  rc = write_report(&res, meta, opts, stdout_path, err, dumps ? &dump : nullptr);
  if (rc && !err.empty()) h->last_error = err;
  return rc;
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
