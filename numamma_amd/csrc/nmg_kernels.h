// nmg_kernels.h -- what the device code (nmg_kernels.hip) and the host engine
// (nmg_engine.hip) share: layout constants, the kernels' parameter blocks and
// the launchers.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

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
// Long-tail log slots (16 B, one store): a sample (count 1, weight < 2^32)
// is {entry | access << 31, weight, offset, seq}; anything else takes two
// slots, {entry | access << 31, count, kTlogHead, ord >> 32} then
// {weight lo, weight hi, kTlogCont, ord & ~0u}.  Offsets are 8-aligned, so
// the two marks never occur as a sample's offset.
constexpr uint32_t kTlogHead = 0xFFFFFFFFu, kTlogCont = 0xFFFFFFFEu;
constexpr uint32_t kLogChunk = 4096;   // entries per LDS pass of tlog_reduce_kernel
constexpr uint32_t kLogMaxGrid = 1024;  // attribution workgroups a log can serve
constexpr uint32_t kPageBuckets = 896;         // dense page cell -> count: 8-slot buckets
constexpr uint32_t kPageSlots = kPageBuckets * 8;  // 7168 cells (56 KiB)
constexpr uint32_t kObjBuckets = kObjSlots / 8;
// hashed (non-dense) tables are flushed at least every kTableWindows windows:
// u32 counts stay far from overflow and the first-come slots are re-learnt
constexpr uint32_t kTableWindows = 128;  // (256: configs[2] +4 %, 64: c4 +3 %; 128 neutral at c4)
// Dense modes (template flags of attribute_kernel):
//   kModeDenseObj:  nb_entries <= kObjSlots: slot = entry id, no key check;
//   kModeDensePage: dense histogram cells per thread <= kDensePageCells: u16
//                   counts, two per LDS word, flushed at least every
//                   kDensePageWindows windows (<= 1024 samples per cell each,
//                   so a u16 cannot overflow into its neighbour)
constexpr int kModeDenseObj = 1, kModeDensePage = 2;
constexpr int kModeLarge = 4;  // more than kLdsNodes keys: LDS fences + directory + node records in global memory
constexpr uint32_t kDensePageCells = kPageSlots * 4;  // the page table's 56 KiB as u16 cells
constexpr uint32_t kDensePageWindows = 62;
constexpr bool kPackObj = true;
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
constexpr uint32_t kDbgTinyLog = 0x2000;   // long-tail sub-logs of 2 records: exercises the overflow path (tests)
constexpr uint32_t kDbgNoPack = 0x4000;    // overflow through plain atomics, not packed ones (tests)
constexpr uint32_t kDbgNoDir = 0x8000;     // large tables: no fence-bucket directory, binary search only (tests)
constexpr uint32_t kDbgMultiRccl = 0x40000;  // nmg_create: a multi-GPU handle even for nb_gpus <= 1, merged through
                                             // RCCL (a one-rank communicator on a one-GPU box: tests of that branch)
constexpr int kTimingWords = 24;           // per wave: load+check, barrier, process, rest, total, windows, -, -,
                                           // then (wave 0) 8 x 2 words of window trace


// PERF_MEM_LVL_* (/usr/include/linux/perf_event.h:1250-1263)
constexpr uint32_t LVL_NA = 0x01, LVL_HIT = 0x02, LVL_MISS = 0x04;

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
  uint32_t id;     // entry id: the counters' index (node records: of the node's newest entry)
  uint32_t count;  // (node records) entries of the node
  uint32_t first;  // (node records) table position of the newest entry; the older ones follow it
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
  const DevEntry* entries;   // [nb_entries] by entry id (hist, sidx)
  const DevEntry* chain;     // entries in table order (node i's: [first, first + count)); the table
                             // of the last nmg_set_objects / nmg_update_objects
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
  // matched SAMPLEs of every analysis since the last reset (the report's
  // nb_found_samples_total, mem_sampling.c:335, 357-360): added by each kernel
  // that attributes, so that an analysis leaves it final
  unsigned long long* found;
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
  uint4* tlog;               // [grid][tlog_parts][tlog_cap] 16 B slots (kTlogHead layouts); null: off
  uint32_t* tlog_cnt;        // [grid][tlog_parts] records written
  uint32_t tlog_cap, tlog_rshift, tlog_parts;
};

// tlog_reduce_kernel (long-tail log, see Params::tlog)
struct TlogParams {
  const uint4* tlog;
  const uint32_t* tlog_cnt;
  uint64_t* sum64;
  uint64_t* min64;
  unsigned long long* pk64;  // may be null
  uint32_t grid, parts, cap, rshift, nb_entries, pk_shift;
};

// reset_kernel: INIT_COUNTER semantics for every counter array
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
  unsigned long long* found;  // zeroed
};

// Launchers (nmg_kernels.hip).  `mode` = kModeDenseObj | kModeDensePage.
hipError_t launch_attribute(bool timing, int mode, uint32_t grid, hipStream_t s, const Params& p);
int attribute_blocks_per_cu();  // resident attribute_kernel workgroups per CU (>= 1)
hipError_t launch_tlog_reduce(uint32_t grid, hipStream_t s, const TlogParams& r);
hipError_t launch_unpack(uint32_t grid, hipStream_t s, uint64_t* sum64, unsigned long long* pk64,
                         uint32_t nb_entries, uint32_t shift);
hipError_t launch_reset(uint32_t grid, hipStream_t s, const ResetParams& r);
hipError_t launch_merge(hipStream_t s, void* dst, const void* src, uint64_t n, int op);
// packed page histogram (nmg_hist_pack / nmg_hist_unpack); ncells a multiple of 4
// sparse_download: the used slots of the sparse table as (key, count) u64 pairs, *cnt of them
hipError_t launch_sparse_compact(hipStream_t s, const uint64_t* keys, const uint32_t* vals, uint64_t cap,
                                 uint64_t* out, unsigned long long* cnt);
hipError_t launch_sparse_insert(hipStream_t s, uint64_t* keys, uint32_t* vals, uint64_t cap, const uint64_t* pairs,
                                uint64_t n);
hipError_t launch_hist_pack(hipStream_t s, const uint32_t* hist, uint64_t ncells, uint32_t thr, void* u8, void* ovf,
                            uint64_t cap, unsigned long long* cnt, uint32_t* wgcnt);  // wgcnt: [1024] workspace
hipError_t launch_hist_unpack(hipStream_t s, uint32_t* hist, uint64_t ncells, const void* u8, const void* ovf,
                              uint64_t n, unsigned long long* bad);
// packed per-object counters (nmg_objcw_pack / nmg_objcw_unpack): n row words
hipError_t launch_objcw_pack(hipStream_t s, const uint64_t* rows, uint64_t n, uint64_t thr, void* u32, void* ovf,
                             uint64_t cap, unsigned long long* cnt);
hipError_t launch_objcw_unpack(hipStream_t s, uint64_t* rows, uint64_t n, const void* u32, const void* ovf,
                               uint64_t m, unsigned long long* bad);
// per-object counts and weights, SoA rows -> [E][access][w] (aos: E * 32 B)
hipError_t launch_objcw_aos(hipStream_t s, const uint64_t* soa, uint64_t E, void* aos);
// page-cell rows on the device (nmg_get_page_cells / nmg_report): per dense
// entry the number of non-zero cells, then the (entry, thread, page, count)
// rows at each entry's offset, in (thread, page) order
hipError_t launch_cells_sparse_count(hipStream_t s, const uint64_t* ck, const unsigned long long* n_ptr, uint64_t cap,
                                     const uint32_t* sent, uint32_t nsent, const uint64_t* base, uint32_t* cnt);
uint32_t scan_parts(uint64_t n);  // partial sums launch_scan_u32 needs (+ 1)
hipError_t launch_scan_u32(hipStream_t s, const uint32_t* in, uint64_t n, uint64_t* out /* [n + 1] */, uint64_t* part);
hipError_t launch_gather_off(hipStream_t s, const uint64_t* off, const uint32_t* sent, uint32_t nsent, uint64_t* out);
hipError_t launch_copy_rows(hipStream_t s, const void* src, const uint64_t* n_ptr, uint64_t cap, void* dst);
hipError_t launch_cells_count(hipStream_t s, const uint32_t* hist, uint64_t hist_cells, uint32_t T,
                              const uint64_t* base, const uint32_t* np, uint32_t E, uint32_t* cnt);
hipError_t launch_cells_emit(hipStream_t s, const uint32_t* hist, uint64_t hist_cells, uint32_t T,
                             const uint64_t* base, const uint32_t* np, uint32_t E, const uint64_t* off, uint4* rows);

}  // namespace nmg
