// nmg_cpu_mt.cpp -- TEST INFRASTRUCTURE / CPU BASELINE ONLY.
//
// A second, multi-threaded C++ restatement of NumaMMa's offline sample
// analysis ("the build's bit-exact C++ CPU
// restatement on all host cores"), used by bench.py's cpu_baseline leg and
// checked against the single-threaded oracle (oracle/nmg_oracle.c) by
// tests/test_cpu_mt.py.  It is never part of the product path.
//
// Same semantics as the oracle, with the reference's cost-shaping structures
// replaced by flat ones so that it runs at configs[2]-[3] sizes:
//   * __analyze_buffer's byte cursor (src/mem_sampling.c:815-927): size 0
//     aborts, non-SAMPLE records are skipped by their size, SAMPLE records
//     shorter than 40 B read the 32 B after their header;
//   * update_counters (:517-592) into per-thread global counters;
//   * lookup (mem_analyzer.c:249-286, tools/hash.c:63-77): the largest key
//     <= addr through a fence array (every 64th key) and a search of the
//     fence's 64 keys, then the node's entries newest-first with the
//     inclusive time window (Q1-Q5);
//   * per-entry counters, first-match ordinal and page cells (ma_get_block,
//     mem_analyzer.c:525-534) in per-thread dense arrays (pages of huge
//     objects in per-thread hash maps), merged after the parallel walk.
// Threads take contiguous, byte-balanced ranges of the analysis-ordered
// buffer list; every merge is a sum, min or max, so the result does not
// depend on the split.  Output: the canonical raw-results dump (NMGRES01,
// numamma_amd/results.py).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

constexpr uint32_t kSample = 9;   // PERF_RECORD_SAMPLE
constexpr uint64_t kPage = 4096;  // mem_analyzer.c:471
constexpr uint32_t LVL_NA = 0x01, LVL_HIT = 0x02, LVL_MISS = 0x04;
constexpr uint32_t kGroupMask[9] = {0x08, 0x20, 0x40, 0x10, 0x80, 0x300, 0xC00, 0x1000, 0x2000};
constexpr int kFenceStep = 64;

struct Counters {  // struct mem_counters (mem_analyzer.h:17-41): total, weight, na, 18 x {count, min, max, sum}
  uint64_t total_count = 0, total_weight = 0, na = 0;
  uint64_t b[18][4];
  Counters() {
    for (auto& x : b) {
      x[0] = 0;
      x[1] = ~0ull;  // INIT_COUNTER (mem_analyzer.c:415-420)
      x[2] = 0;
      x[3] = 0;
    }
  }
};

// update_counters (mem_sampling.c:517-592): each level group independently,
// HIT beats MISS, REM_RAM1|2 and REM_CCE1|2 merged (quirk Q12)
inline void update_counters(Counters& c, uint64_t w, uint32_t lvl) {
  c.total_count++;
  c.total_weight += w;
  if (lvl & LVL_NA) c.na++;
  for (int g = 0; g < 9; g++) {
    if (!(lvl & kGroupMask[g])) continue;
    int k = (lvl & LVL_HIT) ? g : ((lvl & LVL_MISS) ? 9 + g : -1);
    if (k < 0) continue;
    uint64_t* x = c.b[k];
    x[0]++;
    if (w < x[1]) x[1] = w;
    if (w > x[2]) x[2] = w;  // (racy compare-then-store in the reference; exact here)
    x[3] += w;
  }
}

struct Entry {
  uint64_t addr, size, alloc, free;
};

struct Table {
  uint32_t nb_threads = 0, nb_keys = 0, nb_entries = 0;
  std::vector<uint64_t> keys, fences;
  std::vector<uint32_t> entry_off;
  std::vector<Entry> ent;
  // page cells: dense [thread][cell] for entries with (size / 4096 + 1) x T <= 2^24 within the budget
  std::vector<uint64_t> hbase;  // per entry, ~0 = sparse
  uint64_t cells = 0;

  // largest key <= addr, or -1 (ht_lower_key, tools/hash.c:63-77)
  int64_t lower_key(uint64_t addr) const {
    if (!nb_keys || addr < keys[0]) return -1;
    const size_t f = std::upper_bound(fences.begin(), fences.end(), addr) - fences.begin() - 1;
    const size_t lo = f * kFenceStep, hi = std::min<size_t>(lo + kFenceStep, nb_keys);
    return (int64_t)(std::upper_bound(keys.begin() + lo, keys.begin() + hi, addr) - keys.begin()) - 1;
  }
  // __ma_find_mem_info_from_sample_generic (mem_analyzer.c:249-286) + is_sample_in_buffer (:141-155)
  int64_t find(uint64_t addr, uint64_t ts) const {
    const int64_t k = lower_key(addr);
    if (k < 0) return -1;
    for (uint32_t e = entry_off[k]; e < entry_off[k + 1]; e++) {
      const Entry& x = ent[e];
      if (x.addr <= addr && addr < x.addr + x.size && x.alloc <= ts && ts <= x.free) return e;
    }
    return -1;
  }
};

struct Buffer {
  uint32_t thread_rank, access;
  std::vector<uint8_t> bytes;  // linearised like __copy_buffer (mem_sampling.c:675-738)
};

struct Local {
  Counters g[2];
  std::vector<uint64_t> cw;     // [E][2][2] count, weight
  std::vector<uint64_t> first;  // [E]
  std::vector<uint64_t> lv;     // [E][2][37] (levels on)
  std::vector<uint32_t> hist;   // [T][cells]
  std::unordered_map<uint64_t, uint32_t> sparse;  // (entry << 40 | thread << 30 | page) for huge objects
  int err = 0;
  uint64_t err_buf = ~0ull;
};

uint64_t rd64(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}
uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}

int load(const char* path, Table& t, std::vector<Buffer>& bufs) {
  FILE* f = fopen(path, "rb");
  if (!f) return -1;
  fseek(f, 0, SEEK_END);
  const long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  std::vector<uint8_t> file(sz > 0 ? (size_t)sz : 0);
  const size_t got = fread(file.data(), 1, file.size(), f);
  fclose(f);
  if (got != file.size() || file.size() < 64 || memcmp(file.data(), "NMGRPLY1", 8) != 0) return -2;
  const uint8_t* p = file.data();
  t.nb_threads = rd32(p + 12);
  t.nb_keys = rd32(p + 16);
  t.nb_entries = rd32(p + 20);
  const uint32_t nb = rd32(p + 24);
  const uint64_t cs_len = rd64(p + 32), str_len = rd64(p + 40);
  size_t off = 64;
  t.keys.assign(reinterpret_cast<const uint64_t*>(p + off), reinterpret_cast<const uint64_t*>(p + off) + t.nb_keys);
  off += 8ull * t.nb_keys;
  t.entry_off.resize(t.nb_keys + 1);
  memcpy(t.entry_off.data(), p + off, 4ull * (t.nb_keys + 1));
  off += (4ull * (t.nb_keys + 1) + 7) & ~7ull;
  t.ent.resize(t.nb_entries);
  for (uint32_t e = 0; e < t.nb_entries; e++) {
    const uint8_t* q = p + off + 72ull * e;
    t.ent[e] = Entry{rd64(q), rd64(q + 8), rd64(q + 24), rd64(q + 32)};
  }
  off += 72ull * t.nb_entries + 8 * cs_len + ((str_len + 7) & ~7ull);
  bufs.resize(nb);
  for (uint32_t b = 0; b < nb; b++) {
    Buffer& B = bufs[b];
    B.thread_rank = rd32(p + off);
    B.access = rd32(p + off + 4);
    const uint64_t tail = rd64(p + off + 8), head = rd64(p + off + 16), ring = rd64(p + off + 24);
    off += 32;
    const uint8_t* r = p + off;
    if (head == tail) {
    } else if (head < tail) {  // two segments (mem_sampling.c:704-713)
      B.bytes.assign(r + tail, r + ring);
      B.bytes.insert(B.bytes.end(), r, r + head);
    } else {
      B.bytes.assign(r + tail, r + head);
    }
    off += (ring + 7) & ~7ull;
  }
  // fences and the dense page-cell layout (the engine's default 4 GiB budget)
  for (uint32_t k = 0; k < t.nb_keys; k += kFenceStep) t.fences.push_back(t.keys[k]);
  t.hbase.assign(t.nb_entries, ~0ull);
  const uint64_t T = std::max<uint32_t>(t.nb_threads, 1), budget = (4ull << 30) / 4;
  for (uint32_t e = 0; e < t.nb_entries; e++) {
    const uint64_t np = t.ent[e].size / kPage + 1;
    if (np * T <= (1ull << 24) && (t.cells + np) * T <= budget) {
      t.hbase[e] = t.cells;
      t.cells += np;
    }
  }
  return 0;
}

// __analyze_buffer over buffers [b0, b1) (mem_sampling.c:815-927)
void walk(const Table& t, const std::vector<Buffer>& bufs, uint32_t b0, uint32_t b1, bool levels, Local& L,
          std::vector<uint32_t>& bs, std::vector<uint32_t>& bf) {
  for (uint32_t b = b0; b < b1; b++) {
    const Buffer& B = bufs[b];
    const uint8_t* d = B.bytes.data();
    const uint64_t len = B.bytes.size();
    const uint32_t a = B.access, th = B.thread_rank;
    uint32_t ns = 0, nf = 0;
    unsigned cur = 0;  // 32-bit cursors (:831-834)
    while (cur < len) {
      if ((uint64_t)cur + 8 > len) {
        L.err = -4;
        break;
      }
      const uint32_t type = rd32(d + cur);
      uint16_t size;
      memcpy(&size, d + cur + 6, 2);
      if (size == 0) {  // :857-860 abort()
        L.err = -3;
        break;
      }
      if (type == kSample) {
        if ((uint64_t)cur + 40 > len || (uint64_t)cur + size > len) {
          L.err = -4;
          break;
        }
        const uint64_t ts = rd64(d + cur + 8), addr = rd64(d + cur + 16), w = rd64(d + cur + 24),
                       dsrc = rd64(d + cur + 32);
        const uint32_t lvl = (uint32_t)(dsrc >> 5) & 0x3fff;
        ns++;
        update_counters(L.g[a], w, lvl);
        const int64_t e = t.find(addr, ts);
        if (e >= 0) {
          nf++;
          const uint64_t ord = ((uint64_t)b << 32) | cur;  // first match in analysis order (Q7)
          if (ord < L.first[e]) L.first[e] = ord;
          L.cw[e * 4 + a * 2] += 1;
          L.cw[e * 4 + a * 2 + 1] += w;
          if (levels) {
            uint64_t* lv = &L.lv[(e * 2 + a) * 37];
            if (lvl & LVL_NA) lv[0]++;
            for (int g = 0; g < 9; g++) {
              if (!(lvl & kGroupMask[g])) continue;
              const int k = (lvl & LVL_HIT) ? g : ((lvl & LVL_MISS) ? 9 + g : -1);
              if (k < 0) continue;
              lv[1 + 2 * k]++;
              lv[2 + 2 * k] += w;
            }
          }
          const uint32_t page = (uint32_t)(int)((addr - t.ent[e].addr) / kPage);  // ma_get_block (:530-531)
          if (t.hbase[e] != ~0ull) L.hist[(uint64_t)th * t.cells + t.hbase[e] + page]++;
          else L.sparse[((uint64_t)e << 40) | ((uint64_t)th << 30) | page]++;
        }
      }
      cur += size;  // :918
    }
    bs[b] = ns;
    bf[b] = nf;
    if (L.err) {
      L.err_buf = b;
      return;
    }
  }
}

}  // namespace

extern "C" {

struct nmo_mt_timing {
  double load_s, analysis_s, merge_s;
  uint64_t nb_samples;
  int threads;
};

// Analyse a replay with `threads` host threads; write the raw dump to raw_path
// (NULL: none).  levels = also the per-entry level buckets (the raw dump holds
// them; the engine's default path does not compute them).
int nmo_mt_run(const char* replay_path, const char* raw_path, int threads, int levels, struct nmo_mt_timing* tm) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  Table t;
  std::vector<Buffer> bufs;
  int rc = load(replay_path, t, bufs);
  if (rc) return rc;
  const uint32_t nb = (uint32_t)bufs.size(), E = t.nb_entries, T = std::max<uint32_t>(t.nb_threads, 1);
  threads = std::max(1, std::min<int>(threads, (int)std::max<uint32_t>(nb, 1)));
  std::vector<Local> loc(threads);
  for (auto& L : loc) {
    L.cw.assign((size_t)E * 4, 0);
    L.first.assign(E, ~0ull);
    if (levels) L.lv.assign((size_t)E * 74, 0);
    L.hist.assign(t.cells * T, 0);
  }
  std::vector<uint32_t> bs(nb, 0), bf(nb, 0);
  // byte-balanced contiguous ranges
  std::vector<uint64_t> csum(nb + 1, 0);
  for (uint32_t b = 0; b < nb; b++) csum[b + 1] = csum[b] + bufs[b].bytes.size() + 64;
  std::vector<uint32_t> cut(threads + 1, nb);
  cut[0] = 0;
  for (int i = 1; i < threads; i++)
    cut[i] = (uint32_t)(std::lower_bound(csum.begin(), csum.end(), csum[nb] * i / threads) - csum.begin());
  const auto t1 = clk::now();
  {
    std::vector<std::thread> pool;
    for (int i = 0; i < threads; i++)
      pool.emplace_back([&, i] { walk(t, bufs, cut[i], cut[i + 1], levels != 0, loc[i], bs, bf); });
    for (auto& th : pool) th.join();
  }
  const auto t2 = clk::now();
  // the first failing buffer in analysis order decides (the reference aborts there)
  uint64_t ebuf = ~0ull;
  for (auto& L : loc)
    if (L.err && L.err_buf < ebuf) {
      ebuf = L.err_buf;
      rc = L.err;
    }
  if (rc) return rc;
  // merge (sums, mins, maxes) -- entries and cells split over the threads
  Local& M = loc[0];
  {
    std::vector<std::thread> pool;
    for (int i = 0; i < threads; i++)
      pool.emplace_back([&, i] {
        const uint64_t e0 = (uint64_t)E * i / threads, e1 = (uint64_t)E * (i + 1) / threads;
        for (int j = 1; j < threads; j++) {
          const Local& L = loc[j];
          for (uint64_t e = e0; e < e1; e++) {
            for (int k = 0; k < 4; k++) M.cw[e * 4 + k] += L.cw[e * 4 + k];
            M.first[e] = std::min(M.first[e], L.first[e]);
            if (levels)
              for (int k = 0; k < 74; k++) M.lv[e * 74 + k] += L.lv[e * 74 + k];
          }
          const uint64_t n = M.hist.size(), c0 = n * i / threads, c1 = n * (i + 1) / threads;
          for (uint64_t c = c0; c < c1; c++) M.hist[c] += L.hist[c];
        }
      });
    for (auto& th : pool) th.join();
  }
  for (int j = 1; j < threads; j++) {
    for (int a = 0; a < 2; a++) {
      Counters& x = M.g[a];
      const Counters& y = loc[j].g[a];
      x.total_count += y.total_count;
      x.total_weight += y.total_weight;
      x.na += y.na;
      for (int k = 0; k < 18; k++) {
        x.b[k][0] += y.b[k][0];
        x.b[k][1] = std::min(x.b[k][1], y.b[k][1]);
        x.b[k][2] = std::max(x.b[k][2], y.b[k][2]);
        x.b[k][3] += y.b[k][3];
      }
    }
    for (auto& kv : loc[j].sparse) M.sparse[kv.first] += kv.second;
  }
  const auto t3 = clk::now();
  uint64_t nsamp = 0, nfound = 0;
  for (uint32_t b = 0; b < nb; b++) {  // int per buffer, summed (mem_sampling.c:334-335)
    nsamp += (uint64_t)(int64_t)(int32_t)bs[b];
    nfound += (uint64_t)(int64_t)(int32_t)bf[b];
  }
  if (raw_path) {
    FILE* f = fopen(raw_path, "wb");
    if (!f) return -5;
    fwrite("NMGRES01", 1, 8, f);
    const uint32_t hdr[4] = {E, nb, t.nb_threads, 0};
    fwrite(hdr, 4, 4, f);
    for (int a = 0; a < 2; a++) {
      const Counters& c = M.g[a];
      fwrite(&c.total_count, 8, 1, f);
      fwrite(&c.total_weight, 8, 1, f);
      fwrite(&c.na, 8, 1, f);
      for (int k = 0; k < 18; k++) fwrite(c.b[k], 8, 4, f);
    }
    fwrite(&nsamp, 8, 1, f);
    fwrite(&nfound, 8, 1, f);
    fwrite(bs.data(), 4, nb, f);
    fwrite(bf.data(), 4, nb, f);
    std::vector<uint64_t> rec(79);
    for (uint32_t e = 0; e < E; e++) {
      std::fill(rec.begin(), rec.end(), 0);
      rec[0] = M.first[e];
      for (int a = 0; a < 2; a++) {
        rec[1 + 39 * a] = M.cw[(uint64_t)e * 4 + a * 2];
        rec[2 + 39 * a] = M.cw[(uint64_t)e * 4 + a * 2 + 1];
        if (levels)
          for (int k = 0; k < 37; k++) rec[3 + 39 * a + k] = M.lv[((uint64_t)e * 2 + a) * 37 + k];
      }
      fwrite(rec.data(), 8, 79, f);
    }
    // cells (entry, thread, page, count) in (entry, thread, page) order, non-zero only
    std::vector<std::vector<std::pair<uint64_t, uint32_t>>> sp(E);
    for (auto& kv : M.sparse) sp[kv.first >> 40].push_back({kv.first & ((1ull << 40) - 1), kv.second});
    for (auto& v : sp) std::sort(v.begin(), v.end());
    uint64_t n = 0;
    const long pos = ftell(f);
    fwrite(&n, 8, 1, f);
    for (uint32_t e = 0; e < E; e++) {
      if (t.hbase[e] != ~0ull) {
        const uint64_t np = t.ent[e].size / kPage + 1;
        for (uint32_t th = 0; th < T; th++)
          for (uint64_t pg = 0; pg < np; pg++) {
            const uint32_t v = M.hist[(uint64_t)th * t.cells + t.hbase[e] + pg];
            if (!v) continue;
            const uint32_t row[4] = {e, th, (uint32_t)pg, v};
            fwrite(row, 4, 4, f);
            n++;
          }
      } else {
        for (auto& kv : sp[e]) {
          if (!kv.second) continue;
          const uint32_t row[4] = {e, (uint32_t)(kv.first >> 30), (uint32_t)(kv.first & ((1u << 30) - 1)), kv.second};
          fwrite(row, 4, 4, f);
          n++;
        }
      }
    }
    fseek(f, pos, SEEK_SET);
    fwrite(&n, 8, 1, f);
    fclose(f);
  }
  if (tm) {
    tm->load_s = std::chrono::duration<double>(t1 - t0).count();
    tm->analysis_s = std::chrono::duration<double>(t2 - t1).count();
    tm->merge_s = std::chrono::duration<double>(t3 - t2).count();
    tm->nb_samples = nsamp;
    tm->threads = threads;
  }
  return 0;
}

}  // extern "C"
