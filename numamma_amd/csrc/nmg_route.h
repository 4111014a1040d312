// nmg_route.h -- the partition-first path for large object tables (DESIGN.md
// "Partition-first"): what nmg_route.hip and the host engine share.
//
// The reference looks every sample up in one global AVL tree
// (ma_find_mem_info_from_sample, src/mem_analyzer.c:249-306; ht_lower_key,
// tools/hash.c:63-77).  At 10^5..10^6 intervals that is one or two random
// HBM lines per sample on a GPU.  This path first routes the samples by
// address range, then attributes each range with its slice of the table in
// LDS:
//   1. route2_kernel  streams the buffers in analysis order (the byte cursor of
//                     __analyze_buffer, mem_sampling.c:815-927), counts the
//                     SAMPLEs per buffer, and appends a 16 B compact record of
//                     every SAMPLE to a chunk of its partition (partition = a run of
//                     <= kPartKeys consecutive keys; chunks of kChunk records
//                     from the workgroup's private pool);
//      overflow_kernel  the records a full pool turned away, with global lookups;
//   2. count_kernel   chunks per (workgroup, partition), from the chunks' tags,
//                     and the global counters of every routed record from its X
//                     word (update_counters, mem_sampling.c:508-592);
//      plan_kernel    per-partition chunk counts -> list offsets and work items;
//   3. scatter_kernel chunk ids into per-partition lists;
//   4. local_kernel   one work item (<= kItemChunks chunks of one partition) per
//                     workgroup at a time: the partition's keys and node records
//                     in LDS, its object and page counters in LDS, flushed once
//                     per item (__match_sample, :594-673; ma_get_block,
//                     mem_analyzer.c:494-534);
//   5. found_kernel   per-buffer matched-sample counts from the match bits
//                     local_kernel leaves per chunk (on demand: the reference
//                     only sums them, mem_sampling.c:334-335, 357-361).
#pragma once

#include "nmg_kernels.h"

namespace nmg {

constexpr uint32_t kChunk = 64;            // compact records per chunk (one wave processes one chunk)
constexpr uint32_t kPartLevels = 11;
constexpr uint32_t kMaxParts = (1u << kPartLevels) - 1;
// route pass: a sample's partition from a directory over the partition starts
// (RSeg): its segment by comparisons with the segment starts (kernel
// arguments), its slot's entry (u16: last partition starting at or before the
// slot start | starts inside the slot << 11, 31 = to the segment's end), then
// a binary search over those few starts (sorted, in LDS)
constexpr uint32_t kRouteDir = 4096;
constexpr uint32_t kRouteSegs = 8;
constexpr uint32_t kDirCntSat = 31;
struct RSeg {
  uint64_t start;   // first partition start of the segment (~0: unused)
  uint32_t base;    // first directory slot
  uint32_t nslots;  // slots (>= 1)
  uint32_t shift;   // slot j covers [start + (j << shift), + 2^shift); the last slot: to the next segment
  uint32_t qlast;   // last partition of the segment
};
constexpr uint32_t kPartKeys = 1023;       // local pass: keys per partition in LDS (sorted)
constexpr uint32_t kPartSlots = 1024;      // per-partition table stride
constexpr uint32_t kPartDir = 1024;        // directory slots per partition (radix over its key span)
// PartDir, one directory slot (16 B): x = largest key index <= slot start
// (10 bits) | keys inside the slot (11) << 10 | inline (1) << 21; y, z, w =
// the first kDirInline inner keys' offsets from the slot start (u16 pairs,
// 0xffff past the count), valid when `inline` (every listed offset < 2^16):
// a lookup counts the offsets <= its own and reads keys only past them
constexpr uint32_t kDirInline = 6;
// PackedNode, a key's newest entry for the local pass's common path (16 B):
//   x = end - first key, y = alloc_q, z = free_q, w = table position - e0
//   (11 bits) | kPnOlder | kPnExact | kPnOldLds | older entries << kPnOldShift
// with alloc_q / free_q = (date - tbase) >> kPnQShift, saturated to 32 bits
// (an entry freed before tbase: alloc_q = ~0, free_q = 0, no sample
// matches); pe_info.y = buffer_addr - first key.  A sample whose quantised
// timestamp equals either bound, or a key marked exact (its object's start or
// end offset needs more than 32 bits), is decided on the exact node record.
constexpr uint32_t kPnQShift = 8;
constexpr uint32_t kPnOlder = 1u << 11, kPnExact = 1u << 12;
// The older entries of a partition's reused keys (the LIFO chain past the
// newest, tools/hash.c:108-114), in table order, up to kOldLds per partition:
// x = end - first key, y = alloc_q, z = free_q, w = buffer_addr - first key
// (an entry freed before tbase: all zero but y = ~0), and per entry its page
// cell (pe_oinf, as PartInfo's info.x).  A key has them in the list
// (kPnOldLds) when all fit: the list index of its i-th older entry is its
// table position - e0 - key index + i - 1.  Otherwise, or when a quantised
// date is ambiguous, the lookup walks the chain in global memory.
constexpr uint32_t kOldLds = 512;
constexpr uint32_t kPnOldLds = 1u << 13, kPnOldShift = 16;
constexpr uint32_t kPartEntries = 1536;    // entries per partition (LDS object counters)
constexpr uint32_t kPartCells = 28672;     // u16 page cells per partition: nb_threads x cell span
#ifndef NMG_ITEM_CHUNKS
#define NMG_ITEM_CHUNKS 1023
#endif
constexpr uint32_t kItemChunks = NMG_ITEM_CHUNKS;  // chunks per work item (one workgroup): the packed object
                                                   // counters cannot overflow; past 2^16 records a u16 page
                                                   // cell can, and the local pass carries it (kPageCarry)
static_assert((uint64_t)kItemChunks * kChunk < (1ull << (64 - kPackShift)), "packed count per item");
constexpr bool kPageCarry = (uint64_t)kItemChunks * kChunk >= 65536u;
constexpr uint32_t kChunkIdBits = 25;      // route pass LDS: chunk id << 7 | fill
constexpr uint32_t kNoChunk = 0xffffffffu;
constexpr uint32_t kFoundLds = 16384;      // found_kernel: per-buffer LDS counters of one workgroup
// internal switches (tests / A/B only)
constexpr uint32_t kDbgNoRoute = 0x10000;  // large tables: the single-pass attribute_kernel instead
constexpr uint32_t kDbgTinyPool = 0x20000; // route pass: private pools of 2 chunks, so the pool-overflow
                                           // (direct attribution) path runs
// ablation switches (tools/ablate.py; results are wrong with them)
constexpr uint32_t kDbgTinyOvf = 0x80000;  // route pass: an overflow list of 64 records, the rest attributed directly
                                           // (tests, with kDbgTinyPool)
constexpr uint32_t kDbgLapNoWait = 0x100000;   // route pass: a partition's LDS line is given up by a record one
                                                // line ahead of the staged one (tests: the given-up path)
constexpr uint32_t kDbgLocalNoWork = 0x400000;   // local pass: chunk loads only
constexpr uint32_t kDbgRouteTiming = 0x800000;   // route pass: per-wave phase cycles in Params::dbg
constexpr uint32_t kDbgLocalNoObj = 0x1000000;   // local pass: no object counters / first ordinals
constexpr uint32_t kDbgLocalNoPage = 0x2000000;  // local pass: no page cells
constexpr uint32_t kDbgLocalNoGlobal = 0x4000000;  // local pass: no global counters
constexpr uint32_t kDbgLocalNoSearch = 0x8000000;  // local pass: no lookup (nothing matches)
constexpr uint32_t kDbgNoLines = 0x20000000;      // route pass: no LDS line stage (every record stored to its
                                                  // slot; tests and A/B)
constexpr uint32_t kDbgLocalAtomics = 0x80000000u;  // local pass: every flush through atomics (A/B)
constexpr uint32_t kDbgLocalTiming = 0x10000000;  // local pass: per-wave phase cycles in Params::dbg
                                                   // (wait, global, search, match, object, page per chunk;
                                                   // dequeue, setup, flush per item; chunks, items)
constexpr int kRouteTimingWords = 16;            // route2: wait, check+loads, global, search, encode, claim, staged,
                                                 // direct, lap waits, windows, broken, line rounds, stores
                                                 // -, windows, -, -

// One partition: keys [k0, k0 + nk), entries [e0, e0 + ne) (entry ids of the
// offline table are table positions, so a key range owns an id range), dense
// page cells [cb, cb + span) of every thread.
struct PartInfo {
  uint32_t k0, nk, e0, ne;
  uint64_t cb;
  uint32_t span;
  uint32_t dshift;     // directory slot j covers [first key + (j << dshift), + 2^dshift)
  uint32_t pages_lds;  // nb_threads * span <= kPartCells: page cells in LDS, else global atomics
  uint32_t cmap;       // ~0: cells [cb, cb + span); else (online table) span packed cells, the
                       // histogram cell of packed cell j at pe_cmap[cmap + j]
  uint32_t pad[2];
};
static_assert(sizeof(PartInfo) == 48, "PartInfo");

// compact record: 16 B, two u64 words (everything the local pass needs; the
// global counters were done by the route pass)
//   lo = addr - partition start (kAddrBits) | (ts - tbase) << kAddrBits (low 24 bits)
//   hi = (ts - tbase) >> 24 (16 bits) | min(weight, wesc) << 16 (wbits)
//        | location << (16 + wbits): byte offset / 8 (obits), then buffer
//          index g (gbits) -- ordered as the analysis position, so the local
//          pass keeps first matches as locations --
//        | thread rank << (63 - tbits) | access type << 63
// A record whose address, timestamp or weight does not fit carries wesc: the
// local pass re-reads all three from the raw record (rare).
constexpr uint32_t kAddrBits = 40;
// narrowest weight field of a compact record: weights up to 2046 cycles (the
// bulk of PEBS load latencies) never escape; a buffer set whose location
// fields leave fewer bits keeps the single-pass kernel (route_layout)
constexpr uint32_t kMinWeightBits = 11;
constexpr uint32_t kTsBits = 40;
struct XLayout {
  uint32_t gbits, obits, tbits, wbits;  // wbits = min(48 - (gbits + obits + tbits + 1), 16) >= kMinWeightBits
  uint64_t wesc;   // 2^wbits - 1
  uint64_t tbase;  // smallest non-zero alloc_date of the table (earlier samples escape)
};

struct RouteParams {
  Params p;                  // data, sbufs (= descriptors in analysis order, .pad = index), ranges,
                             // global counters, per-buffer counts, and the table for direct attribution
  const uint64_t* pbounds;   // [kMaxParts + 1] partition start keys, ascending, ~0 padding
  const uint16_t* pdir;      // [kRouteDir] directory slots of every segment
  const uint32_t* pdead;     // [(kMaxParts + 1) / 32] bit q: every entry of partition q has free_date 0,
                             // so only a sample with timestamp 0 can match one (alloc <= ts <= free,
                             // is_sample_in_buffer, mem_analyzer.c:148-149): the [stack] range after
                             // warn_non_freed_buffers (Q4), an online table's live objects (Q3)
  RSeg seg[kRouteSegs];      // segments of the partition starts, ascending
  uint32_t nseg;
  uint32_t nparts;
  XLayout xl;
  uint64_t seq0;             // analysis index of descriptor 0 (seq = seq0 + index)
  uint4* rec16;              // [chunks][kChunk] compact records
  uint32_t* cmeta;           // [chunks] partition | fill << 24
  const uint32_t* chunk0;    // [grid + 1] private chunk range of each workgroup
  uint32_t* used;            // [grid] chunks taken
  uint4* ovf16;              // overflow list: records that found no chunk (overflow_kernel)
  unsigned long long* ovfx;  // and their partition's start
  uint32_t* ovf_cnt;         // (= ctl[2]; zeroed by plan_kernel after overflow_kernel read it)
  uint32_t ovf_cap;
};

struct PlanParams {
  uint32_t* pcnt;        // in: [grid][nparts] chunk counts; out: exclusive prefix over workgroups
  uint32_t* pbase;       // out: [nparts] first list slot of each partition (plan_cols_kernel: the totals)
  uint4* items;          // out: {partition, list begin, list end, 0}
  uint32_t* ctl;         // out: [0] number of items, [1] dequeue head (zeroed), [2] overflow records (zeroed), [3] their number for local_kernel
  uint32_t grid, nparts;
};

struct ScatterParams {
  const uint32_t* cmeta;
  const uint32_t* chunk0;
  const uint32_t* used;
  const uint32_t* pcnt;   // exclusive prefixes (plan_kernel)
  const uint32_t* pbase;
  uint32_t* clist;        // [chunks] chunk id | fill << kChunkIdBits, grouped by partition
  uint32_t nparts;
};

struct LocalParams {
  Params p;                  // table (nodes, chain, entries), counters, hist, sparse, flags
  const PartInfo* parts;
  const uint64_t* pe_keys;   // [nparts][kPartSlots] keys, ascending
  const uint4* pe_nodes;     // [nparts][kPartSlots][2] (addr, end), (alloc, free) of each key's newest entry (exact)
  const uint4* pe_pnode;     // [nparts][kPartSlots] the same, packed (PackedNode)
  const uint4* pe_old;       // [nparts][kOldLds] older entries, packed (kOldLds)
  const uint32_t* pe_oinf;   // [nparts][kOldLds] their page cells
  const uint2* pe_info;      // [nparts][kPartSlots] (cell - cb, or packed cell, or ~0 sparse; buffer_addr - first key)
  const uint4* pe_dir;       // [nparts][kPartDir] directory slots (PartDir)
  const uint32_t* pe_ids;    // [table entries] entry id of each table position (an online table,
                             // nmg_update_objects), or null: the id is the position (nmg_set_objects)
  const uint32_t* pe_lrel;   // [table entries] an entry's first packed cell (PartInfo::cmap != ~0)
  const uint32_t* pe_cmap;   // packed cell -> histogram cell
  const uint4* rec16;
  const uint32_t* cmeta;
  const uint32_t* clist;     // chunk id | fill << kChunkIdBits, grouped by partition
  const uint4* items;
  uint32_t* ctl;             // [0] items, [1] dequeue head, [3] records of the overflow path (plan_kernel)
  unsigned long long* cmatch;  // [chunks] match bit per record
  const BufDesc* descs;      // analysis order (escaped weights are re-read from the record)
  XLayout xl;
  uint64_t seq0;
  uint32_t fresh;            // the counters are as the last reset left them (no analysis since): an
                             // item alone on its partition stores its counters without reading them,
                             // unless the overflow path or a large weight wrote to them
};

struct FoundParams {
  const uint32_t* ranges;    // [grid + 1] descriptor range of each route workgroup
  const uint32_t* chunk0;
  const uint32_t* used;
  const uint32_t* cmeta;
  const unsigned long long* cmatch;
  const uint4* rec16;
  uint32_t* bufcnt;          // [2][nb_bufs]
  uint32_t nb_bufs, gbits, gshift;
};

hipError_t launch_route(uint32_t grid, hipStream_t s, const RouteParams& r);
hipError_t launch_overflow(hipStream_t s, const RouteParams& r);
// count_kernel: per route workgroup, chunks per partition (pcnt, from the
// chunks' tags)
struct CountParams {
  ScatterParams sc;
};
hipError_t launch_count(uint32_t grid, hipStream_t s, const CountParams& r);
hipError_t launch_plan(hipStream_t s, const PlanParams& r);
hipError_t launch_scatter(uint32_t grid, hipStream_t s, const ScatterParams& r);
hipError_t launch_local(uint32_t grid, hipStream_t s, const LocalParams& r);
hipError_t launch_found(uint32_t grid, hipStream_t s, const FoundParams& r);

}  // namespace nmg
