// nmg_table.hip -- object tables on the device: the sorted keys and LIFO
// entries of mem_list (FOREACH_HASH order, src/mem_analyzer.c:1820-1823), the
// lookup structures of lower_key (ht_lower_key, tools/hash.c:63-77), the
// partition-first path's partitions, and online table updates.
#include "nmg_engine_impl.h"

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

static void build_big_lookup(const uint64_t* keys, uint32_t K, bool no_dir, BigLookup& bl) {
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
  // bucket-relative indices and counts are 16-bit: S <= 2^16 (larger
  // buckets -- more than 4095 << 16 keys -- are binary-searched)
  if (S == 1 || S > (1u << 16) || no_dir) return;
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

// Lookup structures of a flattened table whose entries, in table order, are
// chain[] (ids in DevEntry::id): node records, then the LDS Eytzinger tree
// (<= kLdsNodes keys) or the fences + directory of the large-table path.
// chain_dev: chain already on the device (the by-id array), else uploaded.
int build_lookup(nmg_engine* h, const uint64_t* keys, const uint32_t* entry_off, uint32_t nb_keys,
                        const std::vector<DevEntry>& chain, DevEntry* chain_dev) {
  h->K = nb_keys;
  std::vector<DevEntry> nodes(nb_keys);
  for (uint32_t k = 0; k < nb_keys; k++) {
    nodes[k] = chain[entry_off[k]];
    nodes[k].first = entry_off[k];
    nodes[k].count = entry_off[k + 1] - entry_off[k];
  }
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_keys, keys, (size_t)nb_keys * 8));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_nodes, nodes.data(), (size_t)nb_keys * sizeof(DevEntry)));
  if (chain_dev) h->d_chain = chain_dev;
  else HIP_TRY(h, alloc_copy(h, (void**)&h->d_chain, chain.data(), chain.size() * sizeof(DevEntry)));
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
    HIP_TRY(h, alloc_copy(h, (void**)&h->d_efences, ef.data(), n * 8));
    HIP_TRY(h, alloc_copy(h, (void**)&h->d_enodes, en.data(), n * sizeof(DevEntry)));
  }
  h->nb_fences = h->fence_log2 = h->dir_log2 = 0;
  if (nb_keys > kLdsNodes) {
    BigLookup bl;
    build_big_lookup(keys, nb_keys, (h->flags & kDbgNoDir) != 0, bl);
    h->nb_fences = bl.nb_fences;
    h->fence_log2 = bl.fence_log2;
    h->dir_log2 = bl.dir_log2;
    HIP_TRY(h, alloc_copy(h, (void**)&h->d_ffences, bl.efences.data(), bl.efences.size() * 8));
    HIP_TRY(h, alloc_copy(h, (void**)&h->d_fshift, bl.shift.data(), bl.shift.size()));
    HIP_TRY(h, alloc_copy(h, (void**)&h->d_dir, bl.dir.data(), bl.dir.size() * sizeof(uint2)));
  }
  return NMG_OK;
}

// The route pass's partition search (route_partition, nmg_route.hip) over
// the P ascending partition starts b: up to kRouteSegs segments, split at the
// gaps between consecutive starts that dwarf the median gap (address spaces
// are clustered: globals, heap, mmap'd regions, the stack), each with
// directory slots in proportion to its partitions.  Slot j of a segment holds
// the last partition starting at or before the slot start, and how many
// starts lie inside the slot (saturated at kDirCntSat: search to the
// segment's last partition).
void route_segments(const uint64_t* b, uint32_t P, RSeg* seg, uint32_t* nseg, std::vector<uint16_t>& dir) {
  std::vector<uint32_t> cuts{0};  // segment k starts at partition cuts[k]
  if (P > 1) {
    std::vector<uint64_t> gaps(P - 1);
    for (uint32_t q = 0; q + 1 < P; q++) gaps[q] = b[q + 1] - b[q];
    std::vector<uint64_t> med(gaps);
    std::nth_element(med.begin(), med.begin() + med.size() / 2, med.end());
    const uint64_t m = std::max<uint64_t>(med[med.size() / 2], 1);
    std::vector<uint32_t> idx(P - 1);
    for (uint32_t q = 0; q + 1 < P; q++) idx[q] = q;
    std::sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) { return gaps[x] > gaps[y]; });
    for (uint32_t i = 0; i < idx.size() && cuts.size() < kRouteSegs; i++) {
      if (gaps[idx[i]] / 64 <= m) break;
      cuts.push_back(idx[i] + 1);
    }
    std::sort(cuts.begin(), cuts.end());
  }
  const uint32_t S = (uint32_t)cuts.size();
  dir.assign(kRouteDir, 0);
  uint32_t used = 0;
  for (uint32_t k = 0; k < kRouteSegs; k++) {
    if (k >= S) {
      seg[k] = RSeg{~0ull, 0, 1, 0, 0};
      continue;
    }
    const uint32_t qa = cuts[k], qb = k + 1 < S ? cuts[k + 1] : P;
    const uint32_t ns = (uint32_t)((uint64_t)(kRouteDir - S) * (qb - qa) / P) + 1;
    const uint64_t span = b[qb - 1] - b[qa];
    uint32_t sh = 0;
    while (sh < 63 && (span >> sh) >= ns) sh++;
    seg[k] = RSeg{b[qa], used, ns, sh, qb - 1};
    uint32_t q = qa;
    for (uint32_t j = 0; j < ns; j++) {
      // slot [s0, s1) relative to the segment start
      const unsigned __int128 s0 = (unsigned __int128)j << sh, s1 = (unsigned __int128)(j + 1) << sh;
      while (q + 1 < qb && (unsigned __int128)(b[q + 1] - b[qa]) <= s0) q++;
      uint32_t c = 0;
      if (j == ns - 1) c = qb - 1 - q;
      else
        while (q + 1 + c < qb && (unsigned __int128)(b[q + 1 + c] - b[qa]) < s1) c++;
      dir[used + j] = (uint16_t)(q | (std::min(c, kDirCntSat) << 11));
    }
    used += ns;
  }
  *nseg = S;
}

// Partitions of the partition-first path (nmg_route.h): runs of consecutive
// keys, each at most kPartKeys keys and kPartEntries entries, and -- where
// the keys allow it -- at most kPartCells dense page cells over all threads,
// so that a partition's lookup tree, node records, object counters and page
// cells fit one workgroup's LDS.  A key range owns a range of table
// positions; `ids` (an online table, nmg_update_objects) maps a position to
// its entry id (null: the id is the position).  An online table's entries
// have their page cells in id order, scattered over the address order, so
// its partitions are not cut by cells (the cells of a partition whose span is
// too wide for LDS take global atomics).  Only for engines that count per
// object (NMG_F_MATCH_SAMPLES) without the dump modes' per-sample output or
// per-object levels; otherwise the table keeps attribute_kernel.
int build_partitions(nmg_engine* h, const uint64_t* keys, const uint32_t* entry_off, uint32_t K,
                            const std::vector<DevEntry>& dev, const uint32_t* ids) {
  free_route_table(h);
  if (K <= kLdsNodes || !(h->flags & NMG_F_MATCH_SAMPLES) || (h->flags & (NMG_F_SAMPLE_MATCHES | NMG_F_OBJECT_LEVELS)))
    return NMG_OK;
  if (ids) {  // the identity map is the offline case
    uint32_t e = 0;
    while (e < entry_off[K] && ids[e] == e) e++;
    if (e == entry_off[K]) ids = nullptr;
  }
  if (ids && h->hist_cells >= (1ull << 31)) return NMG_OK;  // (cell indices of an online table: 32-bit)
  const uint64_t T = h->T;
  std::vector<PartInfo> parts;
  // an online table: the partition's dense cells packed in LDS in table
  // order (lrel: an entry's first LDS cell per table position; cmap: the
  // histogram cell of every packed cell, per partition from PartInfo::cmap)
  std::vector<uint32_t> lrel, cmap;
  if (ids) lrel.assign(entry_off[K], kEmpty32);
  uint32_t k = 0;
  while (k < K) {
    PartInfo pi;
    memset(&pi, 0, sizeof(pi));
    pi.k0 = k;
    pi.e0 = entry_off[k];
    pi.cmap = ~0u;
    uint64_t cb = ~0ull, ce = 0, cc = 0;  // dense cells in [cb, ce), cc of them
    while (k < K && k - pi.k0 < kPartKeys) {
      // a partition's keys span less than 2^(kAddrBits - 1) bytes, so that the
      // compact records' address field (relative to the partition's first key)
      // holds every address its objects cover: a run of keys across a wide gap
      // in the address space (the heap, then the stack) starts a new partition
      if (k > pi.k0 && keys[k] - keys[pi.k0] >= (1ull << (kAddrBits - 1))) break;
      const uint32_t ea = entry_off[k], eb = entry_off[k + 1];
      if (eb - pi.e0 > kPartEntries) {
        if (k == pi.k0) return NMG_OK;  // one address reused more than kPartEntries times: keep attribute_kernel
        break;
      }
      uint64_t ncb = cb, nce = ce, ncc = cc;
      for (uint32_t e = ea; e < eb; e++)
        if (dev[e].hist != kHistSparse) {
          const uint64_t np = h->npages[dev[e].id];
          ncb = std::min<uint64_t>(ncb, dev[e].hist);
          nce = std::max<uint64_t>(nce, dev[e].hist + np);
          ncc += np;
        }
      if (k > pi.k0 && ncb != ~0ull && (ids ? ncc : nce - ncb) * T > kPartCells)
        break;  // (one key alone may exceed: global cells)
      cb = ncb;
      ce = nce;
      cc = ncc;
      k++;
    }
    pi.nk = k - pi.k0;
    pi.ne = entry_off[k] - pi.e0;
    pi.cb = cb == ~0ull ? 0 : cb;
    pi.span = cb == ~0ull ? 0 : (uint32_t)(ce - cb);
    pi.pages_lds = pi.span && (uint64_t)pi.span * T <= kPartCells;
    if (ids && cc && cc * T <= kPartCells) {  // online: the cells packed (cmap), always in LDS
      pi.cmap = (uint32_t)cmap.size();
      pi.span = (uint32_t)cc;
      pi.pages_lds = 1;
      uint32_t off = 0;
      for (uint32_t e = pi.e0; e < pi.e0 + pi.ne; e++)
        if (dev[e].hist != kHistSparse) {
          const uint32_t np = (uint32_t)h->npages[dev[e].id];
          lrel[e] = off;
          for (uint32_t g = 0; g < np; g++) cmap.push_back((uint32_t)(dev[e].hist + g));
          off += np;
        }
    }
    const uint64_t kspan = keys[k - 1] - keys[pi.k0];
    while (pi.dshift < 63 && (kspan >> pi.dshift) >= kPartDir) pi.dshift++;
    parts.push_back(pi);
    if (parts.size() > kMaxParts) return NMG_OK;  // too many partitions for the route pass's LDS tree
  }
  const uint32_t P = (uint32_t)parts.size();
  // the compact records' timestamp base: the earliest allocation (a sample
  // before it can only match objects allocated at time 0, and escapes)
  h->route_tbase = ~0ull;
  for (const DevEntry& d : dev)
    if (d.alloc) h->route_tbase = std::min<uint64_t>(h->route_tbase, d.alloc);
  if (h->route_tbase == ~0ull) h->route_tbase = 0;
  // per partition: keys ascending with their newest entry's node record (the
  // exact one, read by the local pass's rare paths), its packed form and
  // info (the common path), and a directory over the key span: slot j starts
  // at first key + (j << dshift) and holds the index of the largest key <=
  // that start, the number of keys inside the slot (the last slot: every key
  // after its start) and the first kDirInline of those keys' offsets from the
  // slot start when they fit 16 bits (PartDir)
  const uint64_t tb = h->route_tbase;
  std::vector<uint64_t> pk((size_t)P * kPartSlots, ~0ull);
  std::vector<uint4> pn((size_t)P * kPartSlots * 2, make_uint4(0, 0, 0, 0));
  std::vector<uint4> ppn((size_t)P * kPartSlots, make_uint4(0, 0, 0, 0));
  std::vector<uint2> pinf((size_t)P * kPartSlots, make_uint2(kEmpty32, 0));
  std::vector<uint4> pdir((size_t)P * kPartDir, make_uint4(0, 0, 0, 0));
  std::vector<uint4> pold((size_t)P * kOldLds, make_uint4(0, 0, 0, 0));
  std::vector<uint32_t> poinf((size_t)P * kOldLds, kEmpty32);
  // an entry's page cell relative to its partition (as pe_info.x)
  auto cell_rel = [&](const PartInfo& pi, uint32_t e) -> uint32_t {
    const DevEntry& d = dev[e];
    return d.hist == kHistSparse ? kEmpty32 : pi.cmap != ~0u ? lrel[e] : (uint32_t)(d.hist - pi.cb);
  };
  // the quantised dates of an entry (never matching: ~0, 0)
  auto qdates = [&](const DevEntry& d, uint64_t tb, uint32_t& aq, uint32_t& fq) {
    if (d.free < tb) {
      aq = 0xffffffffu;
      fq = 0;
    } else {
      aq = (uint32_t)std::min<uint64_t>((d.alloc > tb ? d.alloc - tb : 0) >> kPnQShift, 0xffffffffull);
      fq = (uint32_t)std::min<uint64_t>((d.free - tb) >> kPnQShift, 0xffffffffull);
    }
  };
  for (uint32_t q = 0; q < P; q++) {
    const PartInfo& pi = parts[q];
    const uint64_t f = keys[pi.k0];
    for (uint32_t r = 0; r < pi.nk; r++) {
      const uint32_t kk = pi.k0 + r;
      const DevEntry& d = dev[entry_off[kk]];
      const size_t o = (size_t)q * kPartSlots + r;
      pk[o] = keys[kk];
      pn[2 * o] = make_uint4((uint32_t)d.addr, (uint32_t)(d.addr >> 32), (uint32_t)d.end, (uint32_t)(d.end >> 32));
      pn[2 * o + 1] = make_uint4((uint32_t)d.alloc, (uint32_t)(d.alloc >> 32), (uint32_t)d.free, (uint32_t)(d.free >> 32));
      const uint32_t older = entry_off[kk + 1] - entry_off[kk] > 1 ? 1u : 0u;
      const uint32_t hrel = cell_rel(pi, entry_off[kk]);
      // packed node (PackedNode): exact where the object's start or end
      // offset from the first key needs more than 32 bits -- unless it was
      // freed before the first allocation (the [stack], Q4): no non-escaped
      // sample can match it, whatever its bounds
      const uint64_t erel = d.end - f, brel = d.addr - f;
      const bool never = d.free < tb;
      const bool exact = !never && (d.addr < f || d.end < d.addr || (erel >> 32) != 0 || (brel >> 32) != 0);
      uint32_t aq, fq;
      qdates(d, tb, aq, fq);
      // the key's older entries in the partition's list (kOldLds) when they fit
      const uint32_t nold = entry_off[kk + 1] - entry_off[kk] - 1, lbase = entry_off[kk] - pi.e0 - r;
      bool old_lds = nold > 0 && nold < 2048 && lbase + nold <= kOldLds;
      for (uint32_t i = 1; old_lds && i <= nold; i++) {
        const uint32_t e = entry_off[kk] + i;
        const DevEntry& od = dev[e];
        uint32_t oa, of;
        qdates(od, tb, oa, of);
        uint4 v = make_uint4(0, oa, of, 0);
        if (od.free >= tb) {  // (else: never matches, bounds irrelevant)
          if (od.addr < f || od.end < od.addr || ((od.end - f) >> 32) != 0) {
            old_lds = false;
            break;
          }
          v.x = (uint32_t)(od.end - f);
          v.w = (uint32_t)(od.addr - f);
        }
        pold[(size_t)q * kOldLds + lbase + i - 1] = v;
        poinf[(size_t)q * kOldLds + lbase + i - 1] = cell_rel(pi, e);
      }
      ppn[o] = make_uint4(exact || never ? 0u : (uint32_t)erel, aq, fq,
                          (entry_off[kk] - pi.e0) | (older ? kPnOlder : 0u) | (exact ? kPnExact : 0u) |
                              (old_lds ? kPnOldLds | (nold << kPnOldShift) : 0u));
      pinf[o] = make_uint2(hrel, exact || never ? 0u : (uint32_t)brel);
    }
    uint32_t lo = 0;
    for (uint32_t j = 0; j < kPartDir; j++) {
      const uint64_t s0 = (uint64_t)j << pi.dshift;  // slot start relative to the first key
      while (lo + 1 < pi.nk && keys[pi.k0 + lo + 1] - f <= s0) lo++;
      uint32_t c = 0;
      while (lo + 1 + c < pi.nk &&
             (j == kPartDir - 1 || keys[pi.k0 + lo + 1 + c] - f < s0 + (1ull << pi.dshift)))
        c++;
      uint32_t off[kDirInline];
      bool inl = true;
      for (uint32_t i = 0; i < kDirInline; i++) {
        off[i] = 0xffffu;
        if (i < c) {
          const uint64_t v = keys[pi.k0 + lo + 1 + i] - f - s0;
          if (v >> 16) inl = false;
          else off[i] = (uint32_t)v;
        }
      }
      pdir[(size_t)q * kPartDir + j] =
          make_uint4(lo | (c << 10) | ((inl && c ? 1u : 0u) << 21), off[0] | (off[1] << 16), off[2] | (off[3] << 16),
                     off[4] | (off[5] << 16));
    }
  }
  // the route pass's partition search: the partitions' first keys ascending,
  // and a directory over them (route_segments)
  std::vector<uint64_t> pb(kMaxParts + 1, ~0ull);
  for (uint32_t q = 0; q < P; q++) pb[q] = keys[parts[q].k0];
  std::vector<uint16_t> rdir;
  route_segments(pb.data(), P, h->rsegs, &h->nrsegs, rdir);
  // partitions whose entries all have free_date 0 (RouteParams::pdead): the
  // route pass keeps only their timestamp-0 samples, the others cannot match
  std::vector<uint32_t> dead((kMaxParts + 1) / 32, 0u);
  for (uint32_t q = 0; q < P; q++) {
    bool d = true;
    for (uint32_t e = parts[q].e0; d && e < parts[q].e0 + parts[q].ne; e++) d = dev[e].free == 0;
    if (d) dead[q >> 5] |= 1u << (q & 31);
  }
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_pdead, dead.data(), dead.size() * 4));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_parts, parts.data(), parts.size() * sizeof(PartInfo)));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_pbounds, pb.data(), pb.size() * 8));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_pdir, rdir.data(), rdir.size() * 2));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_pe_keys, pk.data(), pk.size() * 8));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_pe_nodes, pn.data(), pn.size() * sizeof(uint4)));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_pe_pnode, ppn.data(), ppn.size() * sizeof(uint4)));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_pe_old, pold.data(), pold.size() * sizeof(uint4)));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_pe_oinf, poinf.data(), poinf.size() * 4));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_pe_info, pinf.data(), pinf.size() * sizeof(uint2)));
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_pe_dir, pdir.data(), pdir.size() * sizeof(uint4)));
  if (ids) {
    HIP_TRY(h, alloc_copy(h, (void**)&h->d_pe_ids, ids, (size_t)entry_off[K] * 4));
    HIP_TRY(h, alloc_copy(h, (void**)&h->d_pe_lrel, lrel.data(), lrel.size() * 4));
    if (!cmap.empty()) HIP_TRY(h, alloc_copy(h, (void**)&h->d_pe_cmap, cmap.data(), cmap.size() * 4));
  }
  HIP_TRY(h, hipStreamSynchronize(h->stream));  // (pageable sources)
  h->nparts = P;
  h->route_ok = true;
  return NMG_OK;
}

extern "C" int nmg_set_objects(nmg_engine* h, const uint64_t* keys, const uint32_t* entry_off,
                               uint32_t nb_keys, const nmg_object* entries, uint32_t nb_entries) {
  if (h) h->epoch++;
  if (h) h->counters_fresh = false;
  if (h) h->snap.meta_dirty = h->cprep.meta_dirty = true;
  Range range("nmg_set_objects");
  if (!h || (nb_keys && (!keys || !entry_off)) || (nb_entries && !entries))
    return NMG_ERR_INVALID;
  int rc = check_table(h, keys, entry_off, nb_keys, nb_entries);
  if (rc) return rc;
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
  h->order.clear();
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
    d.id = e;
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
  HIP_TRY(h, alloc_copy(h, (void**)&h->d_entries, dev.data(), (size_t)nb_entries * sizeof(DevEntry)));
  rc = build_lookup(h, keys, entry_off, nb_keys, dev, h->d_entries);
  if (rc) return rc;
  rc = build_partitions(h, keys, entry_off, nb_keys, dev, nullptr);
  if (rc) return rc;
  h->dev_entries = std::move(dev);


  h->n_sum64 = 2 * kGlobalSums + (uint64_t)nb_entries * 4;
  if (h->flags & NMG_F_OBJECT_LEVELS) h->n_sum64 += (uint64_t)nb_entries * 2 * kLevelWords;
  h->n_min64 = 36 + (uint64_t)nb_entries + 1;
  h->n_max64 = 36;
  HIP_TRY(h, hipMalloc(&h->d_sum64, h->n_sum64 * 8));
  HIP_TRY(h, hipMalloc(&h->d_min64, h->n_min64 * 8));
  HIP_TRY(h, hipMalloc(&h->d_max64, h->n_max64 * 8));
  if (!h->d_found) HIP_TRY(h, hipMalloc(&h->d_found, 8));
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
  for (nmg_engine* w : h->workers) {  // multi-GPU: the table on every device
    const int rc = nmg_set_objects(w, keys, entry_off, nb_keys, entries, nb_entries);
    if (rc) return fail(h, rc, w->last_error);
  }
  return nmg_reset_counters(h);
}


// A live --online-analysis table (nmg_update_objects) may hold entries the
// engine has not seen: objects created since the previous alarm (ids E ..
// newE - 1, _init_mem_info's next id, mem_analyzer.c:567-568, with their
// counters from creation, :569-572), and objects whose size at free
// (ma_record_free, :1287) outgrew their page cells.  New entries get page
// cells like nmg_set_objects gives them (dense within the budget, sparse
// otherwise); a dense entry that outgrew its cells moves to a new range with
// its counts.  Every id-indexed counter array is re-laid out on the device
// for the new entry count, counters kept.  (The stream is idle here.)
int grow_entries(nmg_engine* h, uint32_t newE, const uint32_t* ids, const nmg_object* objs, uint32_t n) {
  const uint32_t oldE = h->E;
  const uint64_t T = h->T;
  const bool want_hist = (h->flags & NMG_F_PAGE_HIST) && (h->flags & NMG_F_MATCH_SAMPLES);
  const uint64_t max_cells_per_entry = 1ull << 24, budget_cells = h->hist_budget / 4;
  const uint64_t oldCells = h->hist_cells;
  uint64_t cells = oldCells;
  struct Move {
    uint64_t from, to, np;
  };
  std::vector<Move> moves;
  const size_t nsparse0 = h->sparse_entries.size();
  // Host state is changed in place below; every error return first undoes
  // it (the sizes before the call, and the old fields of the entries that
  // moved), so that a failed update keeps the engine as it was.
  struct Old {
    uint32_t id;
    uint64_t hist, np;
    DevEntry d;
  };
  std::vector<Old> changed;
  auto rollback = [&]() {
    for (auto it = changed.rbegin(); it != changed.rend(); ++it) {
      h->hist_base[it->id] = it->hist;
      h->npages[it->id] = it->np;
      h->dev_entries[it->id] = it->d;
    }
    h->hist_base.resize(oldE);
    h->npages.resize(oldE);
    h->buffer_size.resize(oldE);
    h->entry_addr.resize(oldE);
    h->objects.resize(oldE);
    h->dev_entries.resize(oldE);
    h->sparse_entries.resize(nsparse0);
  };
  auto fail_rb = [&](int code, const std::string& msg) {
    rollback();
    return fail(h, code, msg);
  };
  h->hist_base.resize(newE, kHistSparse);
  h->npages.resize(newE, 1);
  h->buffer_size.resize(newE, 0);
  h->entry_addr.resize(newE, 0);
  h->objects.resize(newE, nmg_object{0, 0, 0, 0});
  h->dev_entries.resize(newE);
  for (uint32_t e = oldE; e < newE; e++) {
    DevEntry& d = h->dev_entries[e];
    memset(&d, 0, sizeof(d));
    d.hist = kHistSparse;
    d.sidx = ~0u;
    d.id = e;
  }
  for (uint32_t j = 0; j < n; j++) {
    const uint32_t id = ids[j];
    const uint64_t np = objs[j].buffer_size / kPageSize + 1;
    DevEntry& d = h->dev_entries[id];
    if (id >= oldE) {
      h->npages[id] = np;
      if (!want_hist) continue;
      if (np * T <= max_cells_per_entry && (cells + np) * T <= budget_cells && cells + np < 0xffffffffull) {
        d.hist = h->hist_base[id] = cells;
        cells += np;
      } else {
        if (h->sparse_entries.size() >= (1u << 22)) return fail_rb(NMG_ERR_CAPACITY, "too many sparse entries");
        d.sidx = (uint32_t)h->sparse_entries.size();
        h->sparse_entries.push_back(id);
      }
    } else if (np > h->npages[id]) {
      changed.push_back({id, h->hist_base[id], h->npages[id], d});
      if (want_hist && h->hist_base[id] != kHistSparse) {
        if (np * T > max_cells_per_entry || (cells + np) * T > budget_cells || cells + np >= 0xffffffffull)
          return fail_rb(NMG_ERR_CAPACITY, "an object outgrew its page cells past the histogram budget");
        moves.push_back({h->hist_base[id], cells, h->npages[id]});
        d.hist = h->hist_base[id] = cells;
        cells += np;
      }
      h->npages[id] = np;
    }
  }
  cells = (cells + 3) & ~uint64_t(3);
  // id-indexed counters, re-laid out for newE entries
  const uint64_t n_sum = 2 * kGlobalSums + (uint64_t)newE * 4 +
                         ((h->flags & NMG_F_OBJECT_LEVELS) ? (uint64_t)newE * 2 * kLevelWords : 0);
  const uint64_t n_min = 36 + (uint64_t)newE + 1;
  uint64_t *sum = nullptr, *mn = nullptr;
  uint32_t* hist = nullptr;
  unsigned long long* pk = nullptr;
  DevEntry* ent = nullptr;
  uint64_t* skeys = nullptr;
  uint32_t *svals = nullptr, *sdirty = nullptr;
  const bool new_sparse = nsparse0 == 0 && !h->sparse_entries.empty() && !h->d_sparse_keys;
  auto undo = [&](hipError_t e, const char* what) {
    (void)hipStreamSynchronize(h->stream);
    (void)hipFree(sum);
    (void)hipFree(mn);
    (void)hipFree(hist);
    (void)hipFree(pk);
    (void)hipFree(ent);
    (void)hipFree(skeys);
    (void)hipFree(svals);
    (void)hipFree(sdirty);
    return fail_rb(NMG_ERR_HIP, std::string("nmg_update_objects: ") + what + ": " + hipGetErrorString(e));
  };
  hipError_t e;
  if ((e = hipMalloc(&sum, n_sum * 8)) != hipSuccess) return undo(e, "counters");
  if ((e = hipMalloc(&mn, n_min * 8)) != hipSuccess) return undo(e, "ordinals");
  if (cells && cells * T != oldCells * T && (e = hipMalloc(&hist, cells * T * 4)) != hipSuccess)
    return undo(e, "page histogram");
  if (newE > kObjSlots && (e = hipMalloc(&pk, (size_t)newE * 2 * 8)) != hipSuccess) return undo(e, "packed counters");
  if ((e = hipMalloc(&ent, (size_t)newE * sizeof(DevEntry))) != hipSuccess) return undo(e, "entries");
  hipStream_t st = h->stream;
  if (new_sparse) {  // the first sparse entry: its table
    if ((e = hipMalloc(&skeys, h->sparse_cap * 8)) != hipSuccess || (e = hipMalloc(&svals, h->sparse_cap * 4)) != hipSuccess ||
        (e = hipMalloc(&sdirty, 2 * 4)) != hipSuccess || (e = hipMemsetAsync(skeys, 0xff, h->sparse_cap * 8, st)) != hipSuccess ||
        (e = hipMemsetAsync(svals, 0, h->sparse_cap * 4, st)) != hipSuccess ||
        (e = hipMemsetAsync(sdirty, 0, 2 * 4, st)) != hipSuccess)
      return undo(e, "sparse page table");
  }
  if ((e = hipMemsetAsync(sum, 0, n_sum * 8, st)) != hipSuccess ||
      (e = hipMemcpyAsync(sum, h->d_sum64, 2 * kGlobalSums * 8, hipMemcpyDeviceToDevice, st)) != hipSuccess ||
      (oldE && (e = hipMemcpy2DAsync(sum + 2 * kGlobalSums, (size_t)newE * 8, h->d_sum64 + 2 * kGlobalSums,
                                     (size_t)oldE * 8, (size_t)oldE * 8, 4, hipMemcpyDeviceToDevice, st)) != hipSuccess) ||
      ((h->flags & NMG_F_OBJECT_LEVELS) && oldE &&
       (e = hipMemcpyAsync(sum + 2 * kGlobalSums + (uint64_t)newE * 4, h->d_sum64 + 2 * kGlobalSums + (uint64_t)oldE * 4,
                           (size_t)oldE * 2 * kLevelWords * 8, hipMemcpyDeviceToDevice, st)) != hipSuccess) ||
      (e = hipMemsetAsync(mn, 0xff, n_min * 8, st)) != hipSuccess ||
      (e = hipMemcpyAsync(mn, h->d_min64, (36 + (size_t)oldE) * 8, hipMemcpyDeviceToDevice, st)) != hipSuccess ||
      (e = hipMemcpyAsync(mn + 36 + newE, h->d_min64 + 36 + oldE, 8, hipMemcpyDeviceToDevice, st)) != hipSuccess ||
      (pk && (e = hipMemsetAsync(pk, 0, (size_t)newE * 2 * 8, st)) != hipSuccess) ||
      (e = hipMemcpyAsync(ent, h->dev_entries.data(), (size_t)newE * sizeof(DevEntry), hipMemcpyHostToDevice, st)) !=
          hipSuccess)
    return undo(e, "re-layout");
  if (hist) {  // [thread][cell] rows with the new stride; moved entries' counts to their new range
    if ((e = hipMemsetAsync(hist, 0, cells * T * 4, st)) != hipSuccess ||
        (oldCells && (e = hipMemcpy2DAsync(hist, cells * 4, h->d_hist, oldCells * 4, oldCells * 4, T,
                                           hipMemcpyDeviceToDevice, st)) != hipSuccess))
      return undo(e, "page histogram re-layout");
    for (const Move& m : moves)
      if ((e = hipMemcpy2DAsync(hist + m.to, cells * 4, hist + m.from, cells * 4, m.np * 4, T, hipMemcpyDeviceToDevice,
                                st)) != hipSuccess ||
          (e = hipMemset2DAsync(hist + m.from, cells * 4, 0, m.np * 4, T, st)) != hipSuccess)
        return undo(e, "page cells of a grown object");
  }
  if ((e = hipStreamSynchronize(st)) != hipSuccess) return undo(e, "re-layout");
  (void)hipFree(h->d_sum64);
  (void)hipFree(h->d_min64);
  (void)hipFree(h->d_pk64);
  if (h->d_chain == h->d_entries) h->d_chain = ent;
  (void)hipFree(h->d_entries);
  h->d_sum64 = sum;
  h->d_min64 = mn;
  h->d_pk64 = pk;
  h->d_entries = ent;
  if (hist) {
    (void)hipFree(h->d_hist);
    h->d_hist = hist;
  }
  h->n_sum64 = n_sum;
  h->n_min64 = n_min;
  h->hist_cells = cells;
  h->E = newE;
  if (new_sparse) {
    h->d_sparse_keys = skeys;
    h->d_sparse_vals = svals;
    h->d_sparse_dirty = sdirty;
  }
  return NMG_OK;
}

// --online-analysis: the table at an alarm, counters kept (mem_sampling.c:953-954
// against the live mem_list).  Entry ids index the counters: ids of the
// nmg_set_objects table, and (live hosts) ids past it for objects created
// since (grow_entries).  The report describes each entry as the latest table
// lists it, in the order of the latest table that lists every entry.
extern "C" int nmg_update_objects(nmg_engine* h, const uint64_t* keys, const uint32_t* entry_off,
                                  uint32_t nb_keys, const uint32_t* entry_ids, const nmg_object* objects) {
  if (h) h->epoch++;
  if (h) h->counters_fresh = false;  // (grown objects' page cells move)
  if (h) h->snap.meta_dirty = h->cprep.meta_dirty = true;
  Range range("nmg_update_objects");
  if (!h || (nb_keys && (!keys || !entry_off || !entry_ids || !objects))) return NMG_ERR_INVALID;
  if (!h->have_table) return fail(h, NMG_ERR_STATE, "nmg_update_objects before nmg_set_objects");
  const uint32_t n = nb_keys ? entry_off[nb_keys] : 0;
  int rc = check_table(h, keys, nb_keys ? entry_off : nullptr, nb_keys, n);
  if (rc) return rc;
  // ids: each at most once; new ones (>= E) consecutive from E
  uint32_t newE = h->E;
  for (uint32_t j = 0; j < n; j++) newE = std::max(newE, entry_ids[j] + 1);
  if (entry_ids && n && (uint64_t)newE > (1ull << 31)) return fail(h, NMG_ERR_RANGE, "too many entries");
  uint64_t nb_grown = 0;
  {
    std::vector<uint8_t> seen(newE, 0);
    for (uint32_t j = 0; j < n; j++) {
      const uint32_t id = entry_ids[j];
      if (seen[id]) return fail(h, NMG_ERR_INVALID, "an entry id listed twice in one table");
      seen[id] = 1;
      if (id < h->E && objects[j].buffer_size / kPageSize + 1 > h->npages[id]) nb_grown++;
    }
    for (uint32_t id = h->E; id < newE; id++)
      if (!seen[id]) return fail(h, NMG_ERR_RANGE, "new entry ids must be consecutive from the current entry count");
  }
  HIP_TRY(h, hipSetDevice(h->device));
  if (h->streaming) {  // the open chunk belongs to the previous alarms' table
    rc = stream_flush(h);
    if (rc) return rc;
  }
  rc = route_settle(h);  // (reads the pool only, not the table)
  if (rc) return rc;
  HIP_TRY(h, hipStreamSynchronize(h->stream));  // launches in flight read the old table and counters
  if (h->multi_pending) {  // merges in flight write the counters being re-laid out
    rc = multi_finish(h);
    if (rc) return rc;
  }
  if (newE > h->E || nb_grown) {
    rc = grow_entries(h, newE, entry_ids, objects, n);
    if (rc) return rc;
  }
  std::vector<DevEntry> chain(n);
  for (uint32_t j = 0; j < n; j++) {
    const uint32_t id = entry_ids[j];
    const nmg_object& o = objects[j];
    DevEntry& d = chain[j];
    d = h->dev_entries[id];  // hist, sidx, id
    d.addr = o.buffer_addr;
    d.end = o.buffer_addr + o.buffer_size;
    d.alloc = o.alloc_date;
    d.free = o.free_date;
    d.count = d.first = 0;
  }
  free_route_table(h);  // (the partitions describe the previous table)
  // build the alarm's lookup beside the current one; keep the current one if that fails
  const LookupSet prev = take_lookup(h);
  rc = build_lookup(h, keys, entry_off, nb_keys, chain, nullptr);
  if (rc == NMG_OK && hipStreamSynchronize(h->stream) != hipSuccess)
    rc = fail(h, NMG_ERR_HIP, "nmg_update_objects: table upload failed");
  if (rc) {
    (void)hipStreamSynchronize(h->stream);
    free_lookup(h);
    put_lookup(h, prev);
    return rc;
  }
  {
    const LookupSet cur = take_lookup(h);
    put_lookup(h, prev);
    free_lookup(h);  // (keeps d_chain when it is the by-id entry array)
    put_lookup(h, cur);
  }
  // the report's view: every listed entry as this table lists it, and this
  // table's order when it lists every entry (ma_finalize walks the table it
  // has at exit, FOREACH_HASH, mem_analyzer.c:1381-1383)
  for (uint32_t j = 0; j < n; j++) {
    const uint32_t id = entry_ids[j];
    h->objects[id] = objects[j];
    h->buffer_size[id] = objects[j].buffer_size;
    h->entry_addr[id] = objects[j].buffer_addr;
  }
  if (n == h->E) {
    bool identity = true;
    for (uint32_t j = 0; j < n && identity; j++) identity = entry_ids[j] == j;
    if (identity) h->order.clear();
    else h->order.assign(entry_ids, entry_ids + n);
  } else if (!h->order.empty()) {
    // a partial table that brought new entries: they follow the known ones,
    // in id order, until a table lists every entry
    for (uint32_t id = (uint32_t)h->order.size(); id < h->E; id++) h->order.push_back(id);
  }
  // the alarm table's partitions.  The new table is committed above, so a
  // failure here is not the update's: the table stays on attribute_kernel
  // (no partitions) and the update goes on to the workers, which must get
  // the same table (a half-applied update would leave them on the old one).
  if (build_partitions(h, keys, entry_off, nb_keys, chain, entry_ids) != NMG_OK) {
    (void)hipGetLastError();
    free_route_table(h);
  }
  for (nmg_engine* w : h->workers) {  // multi-GPU: the table on every device
    rc = nmg_update_objects(w, keys, entry_off, nb_keys, entry_ids, objects);
    if (rc) return fail(h, rc, w->last_error);
  }
  return NMG_OK;
}
