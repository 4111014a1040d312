// nmg_big.hip -- MI355X (gfx950) attribution kernel for large object tables
// (more than kLdsNodes keys: BASELINE configs[2] and [3], 100k-1M intervals).
//
// Same work as attribute_kernel (nmg_kernels.hip) -- __analyze_buffer
// (src/mem_sampling.c:815-927) over the stream-sorted buffer list, global
// mem_counters (update_counters, :517-592), lookup
// (ma_find_mem_info_from_sample, src/mem_analyzer.c:249-306), per-object and
// per-page counters (__match_sample :594-673, ma_get_block
// mem_analyzer.c:494-534) -- shaped for tables far larger than LDS:
//
//   * 512-thread workgroups (8 waves, up to 256 VGPRs), one per CU; a window
//     is 1536 stride slots of 40 B and every lane owns kBK = 3 of them
//     (slots tid, tid + 512, tid + 1024), so each stage below runs on three
//     independent records per lane: three LDS fence searches interleaved,
//     three directory loads in flight, then three resolutions (four records
//     per lane need more than 256 VGPRs);
//   * lookup = LDS fence tree (12 levels) -> ONE 64 B load of the bucket's
//     fat directory slot (FatSlot, nmg_kernels.h), which carries the dates,
//     end, size and entry id of both nodes the slot can resolve to.  Slots
//     with several keys inside, reused addresses (older entries), sizes
//     >= 2^30 and buckets without a directory take the node-record path
//     (binary search of the keys, node record, older entries: quirks Q1-Q5);
//   * the next window's record loads are issued after this window's
//     directory loads, so waiting for a directory slot never waits for the
//     record stream;
//   * no device-scope atomics on the per-sample path: per-object counters in
//     an LDS table (first come, 8-way buckets) with the long-tail log behind
//     it (tlog_reduce_kernel); per-page cells in an LDS table keyed by
//     (entry, page) with a page log by entry range behind it
//     (plog16_reduce_kernel adds each range's cells into the histogram with
//     plain coalesced read-modify-writes).
#include "nmg_device.h"

namespace nmg {

#ifndef NMG_BIG_K
#define NMG_BIG_K 2
#endif
constexpr int kBK = NMG_BIG_K;             // records per lane per window
constexpr uint32_t kBWin = kBWG * kBK;     // 1536 stride slots
constexpr uint32_t kBDrain = 64;           // windows between lane-accumulator drains
constexpr uint32_t kBTableWindows = 128;   // hashed LDS tables flushed at least this often
constexpr uint32_t kBPageBuckets = 768;    // LDS page cells: 8-slot buckets
constexpr uint32_t kBPageSlots = kBPageBuckets * 8;
static_assert(kBK * kBDrain <= 256, "lane accumulators: u16 counts, u32 sums of weights < 2^23");

static_assert((uint64_t)kBTableWindows * kBWin < (1u << 20), "flushed slot counts");

struct BigCounters {
  unsigned long long sums[kGlobalSums];
  unsigned long long mins[18];
  unsigned long long maxs[18];
  alignas(16) unsigned int okey[kObjSlots];  // entry id, 8 per bucket
  unsigned int ocnt[kObjSlots];
  unsigned long long ofirst[kObjSlots];
  unsigned long long owt[kObjSlots];
  alignas(16) unsigned int pkey[kBPageSlots];  // entry << pbits | page, 8 per bucket
  unsigned int pcnt[kBPageSlots];
  unsigned int tcur[kLogParts];      // long-tail (object) sub-log cursors
  unsigned int pcur[kPlogMaxParts];  // page sub-log cursors
};

__device__ __forceinline__ int big_obj_slot(BigCounters& bc, uint32_t e) {
  const uint32_t hb = (uint32_t)(((uint64_t)(e * 0x9E3779B1u) * kObjBuckets) >> 32);
  const int j = bucket_slot(&bc.okey[hb * 8], e);
  return j < 0 ? -1 : (int)(hb * 8 + (uint32_t)j);
}

__device__ __forceinline__ int big_page_slot(BigCounters& bc, uint32_t key) {
  const uint32_t hb = (uint32_t)(((uint64_t)(key * 0x9E3779B1u) * kBPageBuckets) >> 32);
  const int j = bucket_slot(&bc.pkey[hb * 8], key);
  return j < 0 ? -1 : (int)(hb * 8 + (uint32_t)j);
}

// one long-tail object contribution (tlog_put, tlog_reduce_kernel)
__device__ __forceinline__ bool big_tlog_append(const Params& p, BigCounters& bc, uint32_t e, uint32_t a, uint32_t cnt,
                                                uint64_t wt, uint64_t ord) {
  return tlog_put(p, bc.tcur, e, a, cnt, wt, ord);
}

// page contribution straight to the histogram (the page log is full or off)
__device__ __forceinline__ void big_page_direct(Params& p, uint32_t e, uint32_t page, uint32_t th, uint32_t cnt,
                                                uint64_t seq, uint32_t off) {
  const uint32_t hb = p.hpre[e];
  if (p.hpre[e + 1] > hb) {
    atomicAdd(p.hist + uint64_t(th) * p.hist_cells + hb + page, cnt);
  } else {
    const uint32_t sidx = p.entries[e].sidx;
    if (sidx != ~0u) sparse_add(p, sparse_key(sidx, th, page), seq, off, cnt);
  }
}

// one page contribution: the workgroup's sub-log of the entry's range, or global
__device__ __forceinline__ void big_page_out(Params& p, BigCounters& bc, uint32_t e, uint32_t page, uint32_t th,
                                             uint32_t cnt, uint64_t seq, uint32_t off) {
  if (p.plog16) {
    const uint32_t part = e >> p.plog_pshift;
    const uint32_t k = atomicAdd(&bc.pcur[part], 1u);
    if (k < p.plog_cap) {
      p.plog16[(uint64_t(blockIdx.x) * p.plog_parts + part) * p.plog_cap + k] = make_uint4(e, page, cnt, th);
      return;
    }
  }
  big_page_direct(p, e, page, th, cnt, seq, off);
}

// Largest key <= addr inside keys [lo, lo + n) given keys[lo] <= addr
// (binary search in global memory: the node-record path only).
__device__ __forceinline__ uint32_t key_search(const Params& p, uint32_t lo, uint32_t n, uint64_t addr) {
  while (n > 1) {
    const uint32_t half = n >> 1;
    const bool le = p.keys[lo + half] <= addr;
    lo = le ? lo + half : lo;
    n = le ? n - half : half;
  }
  return lo;
}

// The node-record path: node k's newest entry, then its older ones (Q2).
__device__ __forceinline__ void match_node(const Params& p, uint32_t k, uint64_t addr, uint64_t ts, Match& m) {
  const uint4* q = reinterpret_cast<const uint4*>(p.nodes + k);
  const uint4 a = q[0], b = q[1], c = q[2];
  if (entry_match(a, b, addr, ts)) {
    m.e = c.w;
    m.baddr = (uint64_t(a.y) << 32) | a.x;
    return;
  }
  const uint4 d = q[3];
  if (d.x > 1) match_older(p, c.w, d.x, addr, ts, m);
}

// lookup state of one record between the stages
struct BLook {
  const FatSlot* slot;  // fat directory slot to load, or null
  uint32_t kind;        // 0 nothing (no key <= addr / no match possible), 1 slot, 2 search bucket, 3 node record
  uint32_t klo, kn;     // kind 2: keys [klo, klo + kn); kind 3: node klo
};

__global__ __launch_bounds__(kBWG, 1) void attribute_big_kernel(Params p) {
  __shared__ uint64_t s_fences[kMaxFences + 1];
  __shared__ uint8_t s_shift[kMaxFences + 1];
  __shared__ uint32_t s_list[kBWin];
  __shared__ BigCounters bc;
  __shared__ uint32_t s_flags[3], s_nlist, s_next, s_err;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const bool match_on = (p.flags & NMG_F_MATCH_SAMPLES) && p.nb_keys;
  const bool pages_on = (p.flags & NMG_F_PAGE_HIST) != 0;
  const bool tables_on = !(p.flags & kDbgNoTables);
  const bool global_on = !(p.flags & kDbgNoGlobal);
  const bool load_only = (p.flags & kDbgLoadOnly) != 0;
  const uint32_t slots = 1u << p.dir_log2;
  const uint32_t pmask = (1u << p.pbits) - 1;

  for (uint32_t i = tid; i <= kMaxFences; i += kBWG) s_fences[i] = p.nb_keys ? p.ffences[i] : ~0ull;
  for (uint32_t i = tid; i < p.nb_fences; i += kBWG) s_shift[i] = p.fatshift[i];
  if (tid < (int)kGlobalSums) bc.sums[tid] = 0;
  if (tid < 18) {
    bc.mins[tid] = ~0ull;  // INIT_COUNTER (mem_analyzer.c:415-420)
    bc.maxs[tid] = 0;
  }
  for (int i = tid; i < (int)kObjSlots; i += kBWG) {
    bc.okey[i] = kEmpty32;
    bc.ocnt[i] = 0;
    bc.ofirst[i] = kEmpty64;
    bc.owt[i] = 0;
  }
  for (int i = tid; i < (int)kBPageSlots; i += kBWG) {
    bc.pkey[i] = kEmpty32;
    bc.pcnt[i] = 0;
  }
  for (int i = tid; i < (int)kLogParts; i += kBWG) bc.tcur[i] = 0;
  for (int i = tid; i < (int)kPlogMaxParts; i += kBWG) bc.pcur[i] = 0;
  if (tid < 3) s_flags[tid] = 0;
  __syncthreads();

  const uint32_t r0 = p.ranges[blockIdx.x], r1 = p.ranges[blockIdx.x + 1];
  if (r0 >= r1) {
    if (p.tlog)
      for (uint32_t i = tid; i < p.tlog_parts; i += kBWG) p.tlog_cnt[uint64_t(blockIdx.x) * p.tlog_parts + i] = 0;
    if (p.plog16)
      for (uint32_t i = tid; i < p.plog_parts; i += kBWG) p.plog_cnt[uint64_t(blockIdx.x) * p.plog_parts + i] = 0;
    return;
  }
  uint32_t idx = r0;
  uint32_t cur = 0;  // byte cursor in buffer idx (`cur_cpt`, mem_sampling.c:836)
  BufDesc d0 = p.sbufs[idx];
  BufDesc d1 = idx + 1 < r1 ? p.sbufs[idx + 1] : d0;
  bool has1 = idx + 1 < r1;
  uint32_t cur_access = d0.access, cur_thread = d0.thread_rank;

  // window geometry: n0 slots in d0 from cur, then n1 slots at the head of d1
  // when d1 continues the same stream (uniform across the workgroup)
  auto geometry = [](uint32_t c, const BufDesc& a, const BufDesc& b, bool hb, uint32_t& n0, uint32_t& n1) {
    const uint32_t left = a.len - c;
    n0 = min(left / kRecBytes + (left % kRecBytes != 0), kBWin);
    n1 = 0;
    if (hb && n0 < kBWin && b.access == a.access && b.thread_rank == a.thread_rank)
      n1 = min(b.len / kRecBytes + (b.len % kRecBytes != 0), kBWin - n0);
  };
  // the records of the window at (i, c): K stride slots per lane
  auto issue = [&](uint32_t i, uint32_t c, RawRec (&raw)[kBK]) {
    BufDesc a, b;
    uint32_t n0 = 0, n1 = 0;
    if (i < r1) {
      a = p.sbufs[i];
      b = i + 1 < r1 ? p.sbufs[i + 1] : a;
      geometry(c, a, b, i + 1 < r1, n0, n1);
    } else {
      a = b = d0;
    }
#pragma unroll
    for (int k = 0; k < kBK; k++) {
      const uint32_t s = uint32_t(k) * kBWG + tid;
      const bool in1 = s >= n0, cand = s < n0 + n1;
      const uint32_t pos = in1 ? (s - n0) * kRecBytes : c + s * kRecBytes;
      load_rec(p.data + (in1 ? b.offset : a.offset), pos, cand ? (in1 ? b.len : a.len) : 0, raw[k]);
    }
  };
  // the position after window (i, c) when that window is regular (the fast
  // path's successor; a slow-path window ends elsewhere, and the records
  // loaded for a mispredicted window are reloaded)
  auto fast_succ = [&](uint32_t i, uint32_t c, const BufDesc& a, const BufDesc& b, bool hb, uint32_t& si, uint32_t& sc) {
    uint32_t n0, n1;
    geometry(c, a, b, hb, n0, n1);
    if (n1) {
      si = i + 1;
      sc = n1 * kRecBytes;
      if (sc >= b.len) {
        si = i + 2;
        sc = 0;
      }
    } else {
      si = i;
      const uint64_t e = uint64_t(c) + uint64_t(n0) * kRecBytes;
      sc = (uint32_t)e;
      if (e >= a.len) {
        si = i + 1;
        sc = 0;
      }
    }
  };
  // two windows of records in flight: window w's records were issued during
  // window w - 2, after its directory loads, so no wait on a directory slot
  // or on the next window's records includes a freshly issued stream load
  RawRec nxA[kBK], nxB[kBK];
  uint32_t pidx, pcur;  // predicted position of the window after the current one
  issue(idx, 0, nxA);
  fast_succ(idx, 0, d0, d1, has1, pidx, pcur);
  issue(pidx, pcur, nxB);
  bool pred_ok = true;  // the current window's records were loaded at its position
  LaneAcc acc;
  lane_acc_clear(acc);
  uint32_t win = 0, acc_windows = 0, last_flush = 0;
  uint32_t ns0 = 0, nf0 = 0, ns1 = 0, nf1 = 0;  // per-buffer tallies: buffers idx, idx + 1

  auto window = [&](RawRec (&craw)[kBK], RawRec (&fraw)[kBK]) -> bool {
    if (!pred_ok) issue(idx, cur, craw);  // mispredicted (after a slow-path window)
    uint32_t n0, n1;
    geometry(cur, d0, d1, has1, n0, n1);
    // ---- decode; fast-path check: every stride slot holds a whole 40 B record
    Rec r[kBK];
    uint32_t pos[kBK];
    bool in1[kBK], cand[kBK];
    bool bad = (cur & 7) != 0;
#pragma unroll
    for (int k = 0; k < kBK; k++) {
      const uint32_t s = uint32_t(k) * kBWG + tid;
      in1[k] = s >= n0;
      cand[k] = s < n0 + n1;
      pos[k] = in1[k] ? (s - n0) * kRecBytes : cur + s * kRecBytes;
      r[k] = decode_rec(craw[k], pos[k]);
      const uint32_t wlen = in1[k] ? d1.len : d0.len;
      bad |= cand[k] && (uint64_t(pos[k]) + kRecBytes > wlen || (r[k].hdr >> 48) != kRecBytes);
    }
    if (__ballot(bad) && lane == 0) atomicOr(&s_flags[win % 3], 1u);
    __syncthreads();
    const uint32_t f = __builtin_amdgcn_readfirstlane(s_flags[win % 3]);
    if (tid == 0) s_flags[(win + 2) % 3] = 0;  // last read before the previous barrier
    win++;

    uint32_t nidx = idx;
    uint64_t ncur;
    bool valid[kBK], shortrec[kBK];
    uint32_t roff[kBK];
    const bool slow = (f & 1) != 0;
    if (!slow) {
#pragma unroll
      for (int k = 0; k < kBK; k++) {
        valid[k] = cand[k] && uint32_t(r[k].hdr) == kSampleType;
        shortrec[k] = false;
        roff[k] = pos[k];
      }
      if (n1) {
        nidx = idx + 1;
        ncur = uint64_t(n1) * kRecBytes;
        if (ncur >= d1.len) {
          nidx = idx + 2;
          ncur = 0;
        }
      } else {
        ncur = cur + uint64_t(n0) * kRecBytes;
        if (ncur >= d0.len) {
          nidx = idx + 1;
          ncur = 0;
        }
      }
    } else {
      // ---- slow path (buffer idx only): wave 0 follows the header chain
      // like the reference's byte cursor (non-SAMPLE records skipped by size,
      // size 0 = abort, truncation), listing up to kBWin SAMPLE offsets
      const uint8_t* base = p.data + d0.offset;
      const uint64_t len = d0.len;
      if (tid < 64) {
        uint64_t q0 = cur;
        uint32_t n = 0, err = 0;
        const uint64_t lim = min(uint64_t(cur) + uint64_t(kBWin) * kRecBytes, len);
        while (q0 < lim && n + 65 <= kBWin) {
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
          if (q0 + 8 > len) { err = kErrTruncated; break; }
          const uint64_t h = (uint64_t)__shfl(hdr, (int)run, 64);
          const uint32_t size = uint32_t(h >> 48);
          if (size == 0) { err = kErrZeroSize; break; }  // mem_sampling.c:857-860
          if (size & 7) { err = kErrUnaligned; break; }
          if (uint32_t(h) == kSampleType) {
            if (q0 + kRecBytes > len || q0 + size > len) { err = kErrTruncated; break; }
            // bit 0: a SAMPLE shorter than 40 B (kept out of the packed counters)
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
      __syncthreads();
      const uint32_t n = __builtin_amdgcn_readfirstlane(s_nlist);
      const uint32_t serr = __builtin_amdgcn_readfirstlane(s_err);
      ncur = serr ? len : __builtin_amdgcn_readfirstlane(s_next);
      if (ncur >= len) {
        nidx = idx + 1;
        ncur = 0;
      }
#pragma unroll
      for (int k = 0; k < kBK; k++) {
        const uint32_t li = uint32_t(k) * kBWG + tid;
        valid[k] = li < n;
        const uint32_t v = valid[k] ? s_list[li] : 0;
        shortrec[k] = (v & 1u) != 0;
        roff[k] = v & ~1u;
        in1[k] = false;
        RawRec rr;
        load_rec(base, roff[k], valid[k] ? len : 0, rr);
        r[k] = decode_rec(rr, roff[k]);
      }
    }
    // next window's descriptors (its loads are issued after this window's
    // directory loads)
    BufDesc nd0 = d0, nd1 = d1;
    if (nidx == idx + 1) {
      nd0 = d1;
      if (nidx + 1 < r1) nd1 = p.sbufs[nidx + 1];
    } else if (nidx == idx + 2) {
      if (nidx < r1) nd0 = p.sbufs[nidx];
      if (nidx + 1 < r1) nd1 = p.sbufs[nidx + 1];
    }
    const bool nhas1 = nidx + 1 < r1;
    const bool stream_end = nidx != idx && (nidx >= r1 || nd0.access != cur_access || nd0.thread_rank != cur_thread);

    // the next window's records (in flight in fraw) were loaded at pidx/pcur;
    // predict the one after it (loaded into craw once this window's
    // directory loads are issued)
    const bool next_ok = nidx == pidx && (uint32_t)ncur == pcur;
    uint32_t qidx = r1, qcur = 0;
    if (nidx < r1) fast_succ(nidx, (uint32_t)ncur, nd0, nd1, nhas1, qidx, qcur);
    bool nxt_issued = false;
    const uint32_t access = d0.access, th = d0.thread_rank;
    uint64_t vm[kBK], fm[kBK];
    int64_t ent[kBK];
    uint64_t baddr[kBK];
#pragma unroll
    for (int k = 0; k < kBK; k++) {
      if (load_only) valid[k] = false;
      vm[k] = __ballot(valid[k]);
      fm[k] = 0;
      ent[k] = -1;
      baddr[k] = 0;
    }
    // ---- global counters: update_counters(global_counters, ...) (mem_sampling.c:882)
    if (global_on) {
#pragma unroll
      for (int k = 0; k < kBK; k++) {
        if (!valid[k]) continue;
        const uint32_t lvl = uint32_t(r[k].dsrc >> 5) & 0x3fff;
        const uint32_t bm = bucket_mask(lvl);
        const uint64_t w = r[k].w;
        if (w < kLaneMaxWeight) {  // register accumulation
          const uint32_t w32 = (uint32_t)w;
          acc.tc += 1;
          acc.tw += w32;
          acc.na += lvl & LVL_NA;
#pragma unroll
          for (int j = 0; j < 5; j++)
            acc.cnt2[j] += ((bm >> (2 * j)) & 1) | ((j < 4 ? (bm >> (2 * j + 1)) & 1 : 0) << 16);
#pragma unroll
          for (int j = 0; j < 9; j++) acc.sum[j] += ((bm >> j) & 1) * w32;
          for (uint32_t m = bm >> 9; m; m &= m - 1) {  // miss buckets
            const uint32_t b = 9 + (uint32_t)__builtin_ctz(m);
            atomicAdd(&bc.sums[3 + 2 * b], 1ull);
            if (w) atomicAdd(&bc.sums[4 + 2 * b], (unsigned long long)w);
          }
        } else {  // weights >= 2^23 cycles: straight to the LDS counters
          atomicAdd(&bc.sums[0], 1ull);
          atomicAdd(&bc.sums[1], (unsigned long long)w);
          if (lvl & LVL_NA) atomicAdd(&bc.sums[2], 1ull);
          for (uint32_t m = bm; m; m &= m - 1) {
            const uint32_t b = (uint32_t)__builtin_ctz(m);
            atomicAdd(&bc.sums[3 + 2 * b], 1ull);
            atomicAdd(&bc.sums[4 + 2 * b], (unsigned long long)w);
          }
        }
        for (uint32_t m = bm; m; m &= m - 1) {  // min / max only move monotonically
          const uint32_t b = (uint32_t)__builtin_ctz(m);
          if (w < bc.mins[b]) atomicMin(&bc.mins[b], (unsigned long long)w);
          if (w > bc.maxs[b]) atomicMax(&bc.maxs[b], (unsigned long long)w);
        }
      }
    }

    if (match_on) {
      // ---- lookup stage 1: LDS fence search for the lane's records, interleaved
      uint32_t ei[kBK];
#pragma unroll
      for (int k = 0; k < kBK; k++) ei[k] = 1;
#pragma unroll
      for (uint32_t lev = 0; lev < kFenceLevels; lev++) {
#pragma unroll
        for (int k = 0; k < kBK; k++) ei[k] = 2 * ei[k] + (s_fences[ei[k]] <= r[k].addr ? 1u : 0u);
      }
      BLook lk[kBK];
#pragma unroll
      for (int k = 0; k < kBK; k++) {
        lk[k].slot = nullptr;
        lk[k].kind = 0;
        lk[k].klo = lk[k].kn = 0;
        const uint32_t node = ei[k] >> (__builtin_ctz(ei[k]) + 1);
        if (!valid[k] || node == 0) continue;  // addr below every key: no match
        const uint32_t b = fence_bucket(node);
        if (b >= p.nb_fences) {  // ~0 padding: addr == UINT64_MAX, the last key is its lower bound
          lk[k].kind = 3;
          lk[k].klo = p.nb_keys - 1;
          continue;
        }
        const uint32_t k0 = b << p.fence_log2;
        const uint32_t sh = s_shift[b];
        if (sh == kShiftSearch) {  // bucket without a directory
          lk[k].kind = 2;
          lk[k].klo = k0;
          lk[k].kn = min(k0 + (1u << p.fence_log2), p.nb_keys) - k0;
          continue;
        }
        const uint64_t rel = r[k].addr - s_fences[node];
        const uint32_t j = (uint32_t)min(rel >> sh, (uint64_t)(slots - 1));
        lk[k].kind = 1;
        lk[k].slot = p.fat + ((uint64_t(b) << p.dir_log2) + j);
      }
      // ---- stage 2: the directory slots (one 64 B line each), in flight together
      uint4 fs[kBK][4];
#pragma unroll
      for (int k = 0; k < kBK; k++) {
        if (lk[k].kind == 1) {
          const uint4* q = reinterpret_cast<const uint4*>(lk[k].slot);
          fs[k][0] = q[0];
          fs[k][1] = q[1];
          fs[k][2] = q[2];
          fs[k][3] = q[3];
        }
      }
      // the records of the window after next: issued after the slot loads,
      // so the wait for a slot never includes them
      issue(qidx, qcur, craw);
      nxt_issued = true;
      // ---- stage 3: resolve from the slot (FatSlot layout, nmg_kernels.h)
#pragma unroll
      for (int k = 0; k < kBK; k++) {
        if (lk[k].kind != 1) continue;
        const uint64_t addr = r[k].addr, ts = r[k].ts;
        // a: end (x,y) alloc (z,w) | free (x,y) eid (z) sz (w); b likewise
        const uint4 a0 = fs[k][0], a1 = fs[k][1], b0 = fs[k][2], b1 = fs[k][3];
        uint64_t cend, calloc, cfree;
        uint32_t ceid, csz;
        if (a1.z & kFatFlag) {  // several keys inside the slot: b holds the first one
          const uint64_t first = u64of(b0.x, b0.y);
          if (addr >= first) {
            lk[k].kind = 2;
            lk[k].klo = b1.z;
            lk[k].kn = b1.w;
            continue;
          }
          cend = u64of(a0.x, a0.y), calloc = u64of(a0.z, a0.w), cfree = u64of(a1.x, a1.y);
          ceid = a1.z & ~kFatFlag, csz = a1.w;
        } else if ((b1.z & kFatFlag) && addr >= u64of(b0.x, b0.y) - b1.w) {  // the key inside, b.end - b.sz
          cend = u64of(b0.x, b0.y), calloc = u64of(b0.z, b0.w), cfree = u64of(b1.x, b1.y);
          ceid = b1.z & ~kFatFlag, csz = b1.w;
        } else {
          cend = u64of(a0.x, a0.y), calloc = u64of(a0.z, a0.w), cfree = u64of(a1.x, a1.y);
          ceid = a1.z & ~kFatFlag, csz = a1.w;
        }
        const bool in_time = calloc <= ts && ts <= cfree;  // is_sample_in_buffer (mem_analyzer.c:148-149)
        if (csz & (kSzBig | kSzOlder)) {
          lk[k].kind = 0;
          // big newest entry out of its time window and no older entries: no match ([stack], Q4)
          if ((csz & kSzOlder) || in_time) {
            lk[k].kind = 3;
            lk[k].klo = csz & kSzMask;
          }
          continue;
        }
        lk[k].kind = 0;
        const uint64_t ba = cend - csz;
        if (ba <= addr && addr < cend && in_time) {
          ent[k] = ceid;
          baddr[k] = ba;
        }
      }
      // ---- the node-record path (rare): binary search, node record, older entries
#pragma unroll
      for (int k = 0; k < kBK; k++) {
        if (lk[k].kind < 2) continue;
        const uint32_t kk = lk[k].kind == 2 ? key_search(p, lk[k].klo, lk[k].kn, r[k].addr) : lk[k].klo;
        Match m;
        m.e = -1;
        m.baddr = 0;
        match_node(p, kk, r[k].addr, r[k].ts, m);
        ent[k] = m.e;
        baddr[k] = m.baddr;
      }
    }
    if (!nxt_issued) issue(qidx, qcur, craw);

    // ---- per-buffer tallies (mem_sampling.c:921-926) and the matched samples' counters
#pragma unroll
    for (int k = 0; k < kBK; k++) {
      fm[k] = __ballot(ent[k] >= 0);
      const uint32_t w0 = uint32_t(k) * kBWG + (uint32_t(tid) & ~63u);
      const uint64_t m1 = (slow || n0 >= w0 + 64) ? 0ull : (n0 <= w0 ? ~0ull : (~0ull << (n0 - w0)));
      ns0 += (uint32_t)__popcll(vm[k] & ~m1);
      nf0 += (uint32_t)__popcll(fm[k] & ~m1);
      ns1 += (uint32_t)__popcll(vm[k] & m1);
      nf1 += (uint32_t)__popcll(fm[k] & m1);
    }
#pragma unroll
    for (int k = 0; k < kBK; k++) {
      const uint64_t seq = in1[k] ? d1.seq : d0.seq;
      if (p.smatch && valid[k])  // dump modes: every SAMPLE record's match at its arena position
        p.smatch[((in1[k] ? d1.offset : d0.offset) + roff[k]) >> 3] = ent[k] >= 0 ? (uint32_t)ent[k] + 1u : 0u;
      if (ent[k] < 0 || !tables_on) continue;
      const uint32_t e = (uint32_t)ent[k];
      const uint64_t w = r[k].w;
      const uint32_t off = roff[k];
      const unsigned long long ord = (seq << 32) | off;  // first match in analysis order (Q7)
      // per-object counters (with packing, a slot only sums packable weights)
      const bool pk = p.pk64 && w < p.pk_wlim && !shortrec[k];
      const int os = (p.pk64 && !pk) ? -1 : big_obj_slot(bc, e);
      if (os >= 0) {
        atomicAdd(&bc.ocnt[os], 1u);
        if (w) atomicAdd(&bc.owt[os], (unsigned long long)w);
        if (ord < bc.ofirst[os]) atomicMin(&bc.ofirst[os], ord);
      } else if (p.tlog && big_tlog_append(p, bc, e, access, 1u, w, ord)) {
      } else if (pk) {
        atomicAdd(p.pk64 + uint64_t(access) * p.nb_entries + e, (1ull << p.pk_shift) | w);
        atomicMin(reinterpret_cast<unsigned long long*>(p.min64 + 36 + e), ord);
      } else {
        atomicAdd(reinterpret_cast<unsigned long long*>(p.sum64 + objcw_index(e, access, 0, p.nb_entries)), 1ull);
        if (w)
          atomicAdd(reinterpret_cast<unsigned long long*>(p.sum64 + objcw_index(e, access, 1, p.nb_entries)),
                    (unsigned long long)w);
        atomicMin(reinterpret_cast<unsigned long long*>(p.min64 + 36 + e), ord);
      }
      if (pages_on) {
        // ma_get_block: page_no = (int)((addr - buffer_addr) / 4096) (mem_analyzer.c:530-531)
        const uint32_t page = uint32_t(int(uint64_t(r[k].addr - baddr[k]) / kPageSize));
        const int ps = page <= pmask ? big_page_slot(bc, (e << p.pbits) | page) : -1;
        if (ps >= 0) atomicAdd(&bc.pcnt[ps], 1u);
        else big_page_out(p, bc, e, page, th, 1u, seq, off);
      }
      if (p.flags & NMG_F_OBJECT_LEVELS) {
        const uint32_t lvl = uint32_t(r[k].dsrc >> 5) & 0x3fff;
        unsigned long long* lv = reinterpret_cast<unsigned long long*>(
            p.sum64 + 2 * kGlobalSums + uint64_t(p.nb_entries) * 4 + (uint64_t(e) * 2 + access) * kLevelWords);
        if (lvl & LVL_NA) atomicAdd(lv, 1ull);
        for (int g = 0; g < 9; g++) {
          if (!(lvl & level_mask(g))) continue;
          const int bucket = (lvl & LVL_HIT) ? g : ((lvl & LVL_MISS) ? 9 + g : -1);
          if (bucket < 0) continue;
          atomicAdd(lv + 1 + 2 * bucket, 1ull);
          if (w) atomicAdd(lv + 2 + 2 * bucket, (unsigned long long)w);
        }
      }
    }

    if (++acc_windows == kBDrain || stream_end) {  // keep the per-lane u32 sums bounded
      lane_acc_drain(acc, bc.sums, lane);
      acc_windows = 0;
    }
    if (nidx != idx) {  // buffer idx (and idx + 1 when skipped over) done
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
    if (stream_end || win - last_flush >= kBTableWindows) {
      __syncthreads();  // every insert and drain of this window is done
      const bool write = !(p.flags & kDbgNoFlush);
      if (stream_end) {
        if (tid < (int)kGlobalSums && write && bc.sums[tid])
          atomicAdd(reinterpret_cast<unsigned long long*>(p.sum64 + gsum_index(cur_access, tid)), bc.sums[tid]);
        if (tid < 18 && write && bc.sums[3 + 2 * tid]) {
          atomicMin(reinterpret_cast<unsigned long long*>(p.min64 + cur_access * 18 + tid), bc.mins[tid]);
          atomicMax(reinterpret_cast<unsigned long long*>(p.max64 + cur_access * 18 + tid), bc.maxs[tid]);
        }
      }
      for (int i = tid; i < (int)kObjSlots; i += kBWG) {
        const uint32_t e = bc.okey[i];
        if (e == kEmpty32) continue;
        const uint64_t cnt = bc.ocnt[i], wt = bc.owt[i];
        if (write && p.tlog && big_tlog_append(p, bc, e, cur_access, (uint32_t)cnt, wt, bc.ofirst[i])) {
        } else if (write && p.pk64) {
          atomicAdd(p.pk64 + uint64_t(cur_access) * p.nb_entries + e, (cnt << p.pk_shift) | wt);
          atomicMin(reinterpret_cast<unsigned long long*>(p.min64 + 36 + e), bc.ofirst[i]);
        } else if (write) {
          atomicAdd(reinterpret_cast<unsigned long long*>(p.sum64 + objcw_index(e, cur_access, 0, p.nb_entries)),
                    (unsigned long long)cnt);
          if (wt)
            atomicAdd(reinterpret_cast<unsigned long long*>(p.sum64 + objcw_index(e, cur_access, 1, p.nb_entries)),
                      (unsigned long long)wt);
          atomicMin(reinterpret_cast<unsigned long long*>(p.min64 + 36 + e), bc.ofirst[i]);
        }
        bc.okey[i] = kEmpty32;
        bc.ocnt[i] = 0;
        bc.ofirst[i] = kEmpty64;
        bc.owt[i] = 0;
      }
      for (int i = tid; i < (int)kBPageSlots; i += kBWG) {
        const uint32_t key = bc.pkey[i];
        if (key == kEmpty32) continue;
        if (write) big_page_out(p, bc, key >> p.pbits, key & pmask, cur_thread, bc.pcnt[i], d0.seq, 0);
        bc.pkey[i] = kEmpty32;
        bc.pcnt[i] = 0;
      }
      last_flush = win;
      __syncthreads();
      if (stream_end) {
        if (tid < (int)kGlobalSums) bc.sums[tid] = 0;
        if (tid < 18) {
          bc.mins[tid] = ~0ull;
          bc.maxs[tid] = 0;
        }
        cur_access = nd0.access;
        cur_thread = nd0.thread_rank;
      }
    }
    idx = nidx;
    cur = (uint32_t)ncur;
    d0 = nd0;
    d1 = nd1;
    has1 = nhas1;
    pred_ok = next_ok;
    pidx = qidx;
    pcur = qcur;
    return idx >= r1;  // the loop's only exit, after the state update
  };
  // unrolled by two: the raw record buffers alternate without register copies
  while (!window(nxA, nxB) && !window(nxB, nxA)) {
  }
  __syncthreads();  // the sub-logs' fill (every append of this workgroup is done)
  if (p.tlog)
    for (uint32_t i = tid; i < p.tlog_parts; i += kBWG)
      p.tlog_cnt[uint64_t(blockIdx.x) * p.tlog_parts + i] = min(bc.tcur[i], p.tlog_cap);
  if (p.plog16)
    for (uint32_t i = tid; i < p.plog_parts; i += kBWG)
      p.plog_cnt[uint64_t(blockIdx.x) * p.plog_parts + i] = min(bc.pcur[i], p.plog_cap);
}

// Sums the page log of one large-table launch: workgroup `part` owns the
// entries [part << pshift, (part + 1) << pshift), whose dense cells are the
// contiguous cells [hpre[e0], hpre[e1]) of every thread's row.  It reads
// that part's sub-log of every attribution workgroup, adds the counts in LDS
// (a window of rows x cells per pass), then adds the window into the
// histogram with plain read-modify-writes: no other writer of those cells
// runs meanwhile, and a row's cells are contiguous, so the update is
// coalesced.  Entries with sparse cells go to the sparse table.
__global__ __launch_bounds__(1024, 1) void plog16_reduce_kernel(Plog16Params rp) {
  __shared__ uint32_t s_cnt[kPlogWin];
  __shared__ uint32_t s_pre[kLogMaxGrid + 1];
  Params& p = rp.p;
  const uint32_t part = blockIdx.x, tid = threadIdx.x;
  for (uint32_t w = tid; w < rp.grid; w += 1024) s_pre[w + 1] = p.plog_cnt[uint64_t(w) * p.plog_parts + part];
  __syncthreads();
  if (tid < 64) {  // prefix over the source workgroups (as in tlog_reduce_kernel)
    const uint32_t per = (rp.grid + 63) / 64, b = min(tid * per, rp.grid), e = min(b + per, rp.grid);
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
  const uint32_t total = s_pre[rp.grid];
  if (total == 0) return;
  const uint32_t e0 = part << p.plog_pshift;
  const uint32_t e1 = (uint32_t)min((uint64_t)e0 + (1ull << p.plog_pshift), (uint64_t)p.nb_entries);
  const uint32_t c0 = p.hpre[e0], span = p.hpre[e1] - c0;
  // windows: cells [w0, w0 + cw) of rows [t0, t0 + tw) per pass
  const uint32_t cw = max(1u, min(span, kPlogWin));
  const uint32_t tw = max(1u, kPlogWin / cw);
  bool first = true;
  for (uint32_t w0 = 0; w0 < max(span, 1u); w0 += cw) {
    for (uint32_t t0 = 0; t0 < p.nb_threads; t0 += tw) {
      const uint32_t t1 = min(t0 + tw, p.nb_threads), wn = min(cw, span - min(w0, span));
      for (uint32_t j = tid; j < (t1 - t0) * cw; j += 1024) s_cnt[j] = 0;
      __syncthreads();
      constexpr int kU = 4;  // records per thread in flight
      for (uint32_t i0 = tid; i0 < total; i0 += kU * 1024) {
        uint4 v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
          const uint32_t i = i0 + u * 1024;
          v[u] = make_uint4(0, 0, 0, 0);
          if (i >= total) continue;
          uint32_t lo = 0, hi = rp.grid;  // source workgroup: s_pre[lo] <= i < s_pre[lo + 1]
          while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_pre[mid] <= i) lo = mid;
            else hi = mid;
          }
          v[u] = p.plog16[(uint64_t(lo) * p.plog_parts + part) * p.plog_cap + (i - s_pre[lo])];
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
          const uint32_t e = v[u].x, page = v[u].y, cnt = v[u].z, th = v[u].w;
          if (cnt == 0) continue;
          const uint32_t hb = p.hpre[e];
          if (p.hpre[e + 1] > hb) {
            const uint32_t c = hb - c0 + page;
            if (th >= t0 && th < t1 && c >= w0 && c < w0 + wn) atomicAdd(&s_cnt[(th - t0) * cw + (c - w0)], cnt);
          } else if (first) {
            const uint32_t sidx = p.entries[e].sidx;
            if (sidx != ~0u) sparse_add(p, sparse_key(sidx, th, page), 0, 0, cnt);
          }
        }
      }
      __syncthreads();
      for (uint32_t t = t0; t < t1; t++) {
        uint32_t* row = p.hist + uint64_t(t) * p.hist_cells + c0 + w0;
        const uint32_t* src = s_cnt + (t - t0) * cw;
        for (uint32_t j = tid; j < wn; j += 1024)
          if (src[j]) row[j] += src[j];
      }
      __syncthreads();
      first = false;
    }
  }
}

hipError_t launch_attribute_big(uint32_t grid, hipStream_t s, const Params& p) {
  hipLaunchKernelGGL(attribute_big_kernel, dim3(grid), dim3(kBWG), 0, s, p);
  return hipGetLastError();
}

int attribute_big_blocks_per_cu() {
  int bpc = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, attribute_big_kernel, kBWG, 0) != hipSuccess || bpc <= 0)
    bpc = 1;
  return bpc;
}

hipError_t launch_plog16_reduce(uint32_t parts, hipStream_t s, const Plog16Params& r) {
  hipLaunchKernelGGL(plog16_reduce_kernel, dim3(parts), dim3(1024), 0, s, r);
  return hipGetLastError();
}

}  // namespace nmg
