// nmg_report.cpp -- host half of the drop-in: the report part of ma_finalize
// (src/mem_analyzer.c:1802-1884) fed by the engine's device results.
//
//  * call-site registry: sites are created in first-match order (the order
//    __match_sample reaches new_call_site, mem_sampling.c:665-669), then every
//    matched object is re-attached with find_call_site in FOREACH_HASH order
//    (update_call_sites, mem_analyzer.c:1380-1436).  find_call_site's linear
//    scan of the LIFO site list is replaced by two hash maps keyed exactly on
//    its match predicate (callstack-keyed sites / caller_rip-keyed sites);
//    "first in the list" == newest == highest id among the candidates.
//  * __sort_sites (mem_analyzer.c:1531-1557) is reproduced exactly, including
//    its int-truncated running minimum (quirk Q9): a plain sort when every
//    key fits an int, otherwise an O(chain log S) segment-tree simulation of
//    the selection passes.
//  * printf formats are byte-identical to __print_counters (:1438-1487),
//    print_call_site_summary (:1597-1640), __plot_counters (:1559-1583) and
//    mem_sampling_statistics (mem_sampling.c:357-361).
#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <thread>
#include <chrono>
#include <cstdlib>
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <functional>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "nmg_internal.h"

namespace nmg {
namespace {

constexpr uint32_t kMemTypeStack = 2;  // enum mem_type, mem_analyzer.h:58-64

struct Site {
  uint32_t id;
  std::string caller;
  uint64_t caller_rip;
  const uint64_t* callstack;
  int32_t callstack_size;
  uint64_t buffer_size;            // initial_buffer_size of the creating object
  uint32_t mem_type;               // site->mem_info.mem_type
  uint64_t mem_info_buffer_size;   // site->mem_info.buffer_size (:1363)
  uint32_t nb_mallocs = 0;
  uint64_t read_count = 0, read_weight = 0, write_count = 0, write_weight = 0;
  std::vector<uint32_t> objects;   // entries attached at finalize
};

// (the tail points into the caller's callstack pool, alive for the report)
struct CsKey {
  uint64_t size;
  int32_t cs_size;
  uint32_t n;            // tail length
  const uint64_t* tail;  // callstack[3..cs_size)
  uint64_t hash;
  bool operator==(const CsKey& o) const {
    return size == o.size && cs_size == o.cs_size && n == o.n && (n == 0 || !memcmp(tail, o.tail, 8ull * n));
  }
};
struct CsKeyHash {
  size_t operator()(const CsKey& k) const { return (size_t)k.hash; }
};
struct RipKey {
  uint64_t size, rip;
  bool operator==(const RipKey& o) const { return size == o.size && rip == o.rip; }
};
struct RipKeyHash {
  size_t operator()(const RipKey& k) const { return (size_t)(k.size * 0x9E3779B97F4A7C15ull ^ k.rip); }
};

class Registry {
 public:
  explicit Registry(const nmg_object_meta* meta) : meta_(meta) {}

  // find_call_site (mem_analyzer.c:1302-1331)
  int64_t find(uint32_t e) const {
    const nmg_object_meta& m = meta_[e];
    int64_t best = -1;
    auto a = by_cs_.find(cs_key_of(m.initial_buffer_size, m.callstack, m.callstack_size));
    if (a != by_cs_.end()) best = a->second;
    auto b = by_rip_.find(RipKey{m.initial_buffer_size, m.caller_rip});
    if (b != by_rip_.end() && b->second > best) best = b->second;
    return best;  // sites are indexed by creation order == id - 1
  }

  // new_call_site (mem_analyzer.c:1333-1378)
  int64_t create(uint32_t e, uint64_t npages) {
    const nmg_object_meta& m = meta_[e];
    Site s;
    s.id = (uint32_t)sites.size() + 1;  // next_call_site_id starts at 1 (:1339-1340)
    s.caller = caller_string(m);
    s.caller_rip = m.caller_rip;
    s.callstack = m.callstack;
    s.callstack_size = m.callstack_size;
    s.buffer_size = m.initial_buffer_size;
    s.mem_type = m.mem_type;
    // site->mem_info.buffer_size (:1363) is only ever used as buffer_size /
    // 4096 + 1 rows (__plot_counters :1565), i.e. the entry's page count
    s.mem_info_buffer_size = (npages - 1) * kPageSize;
    int64_t idx = (int64_t)sites.size();
    if (m.callstack)
      by_cs_[cs_key_of(m.initial_buffer_size, m.callstack, m.callstack_size)] = idx;
    else
      by_rip_[RipKey{m.initial_buffer_size, m.caller_rip}] = idx;
    sites.push_back(std::move(s));
    return idx;
  }

  std::vector<Site> sites;  // creation order

 private:
  static CsKey cs_key_of(uint64_t size, const uint64_t* cs, int32_t cs_size) {
    CsKey k{size, cs_size, 0, nullptr, 0};
    if (cs && cs_size > 3) {
      k.tail = cs + 3;
      k.n = (uint32_t)(cs_size - 3);
    }
    uint64_t h = size * 0x9E3779B97F4A7C15ull ^ (uint64_t)(uint32_t)cs_size;
    for (uint32_t i = 0; i < k.n; i++) h = (h ^ k.tail[i]) * 0x100000001B3ull;
    k.hash = h;
    return k;
  }
 public:
  // get_caller_function_from_rip (src/mem_tools.c:91-131): "???" for a NULL
  // rip; replays carry the symbolised string; strings live in 1024-byte slots.
  static std::string caller_string(const nmg_object_meta& m) {
    char buf[1024];
    if (m.caller)
      snprintf(buf, sizeof(buf), "%s", m.caller);
    else if (!m.caller_rip)
      snprintf(buf, sizeof(buf), "???");
    else
      snprintf(buf, sizeof(buf), "[0x%" PRIx64 "]", m.caller_rip);
    return buf;
  }

 private:
  const nmg_object_meta* meta_;
  std::unordered_map<CsKey, int64_t, CsKeyHash> by_cs_;
  std::unordered_map<RipKey, int64_t, RipKeyHash> by_rip_;
};

// (uint64_t)(int64_t)(int)x: the comparison in __sort_sites promotes the
// int-truncated running minimum back to uint64_t (mem_analyzer.c:1544-1547)
inline uint64_t trunc_key(uint64_t x) { return (uint64_t)(int64_t)(int32_t)(uint32_t)x; }

// Returns the final list order (indices into sites), head first.
std::vector<int64_t> sort_sites(const std::vector<Site>& sites) {
  const int64_t n = (int64_t)sites.size();
  std::vector<int64_t> out;
  out.reserve(n);
  bool small = true;
  for (const Site& s : sites) small &= s.read_weight < (1ull << 31);
  if (small) {
    // selection of the first minimum in list order (list = id descending),
    // pushed at the head: final = weight descending, ties by id ascending
    for (int64_t i = 0; i < n; i++) out.push_back(i);
    std::stable_sort(out.begin(), out.end(), [&](int64_t a, int64_t b) {
      if (sites[a].read_weight != sites[b].read_weight) return sites[a].read_weight > sites[b].read_weight;
      return a < b;
    });
    return out;
  }
  // general case: simulate the passes.  pos 0 = head of the LIFO list = newest.
  int64_t sz = 1;
  while (sz < n) sz <<= 1;
  const uint64_t kDead = ~0ull;
  std::vector<uint64_t> tree(2 * sz, kDead);
  for (int64_t pos = 0; pos < n; pos++) tree[sz + pos] = sites[n - 1 - pos].read_weight;
  for (int64_t i = sz - 1; i >= 1; i--) tree[i] = std::min(tree[2 * i], tree[2 * i + 1]);
  auto remove = [&](int64_t pos) {
    int64_t i = sz + pos;
    tree[i] = kDead;
    for (i >>= 1; i >= 1; i >>= 1) tree[i] = std::min(tree[2 * i], tree[2 * i + 1]);
  };
  // first position >= from whose value < m, or -1
  std::function<int64_t(int64_t, int64_t, int64_t, int64_t, uint64_t)> first_below;
  first_below = [&](int64_t node, int64_t lo, int64_t hi, int64_t from, uint64_t m) -> int64_t {
    if (hi < from || tree[node] >= m) return -1;
    if (lo == hi) return lo;
    int64_t mid = (lo + hi) / 2;
    int64_t r = first_below(2 * node, lo, mid, from, m);
    if (r >= 0) return r;
    return first_below(2 * node + 1, mid + 1, hi, from, m);
  };
  std::vector<int64_t> removal;
  removal.reserve(n);
  std::vector<char> alive(n, 1);
  int64_t head = 0;
  for (int64_t pass = 0; pass < n; pass++) {
    while (!alive[head]) head++;
    int64_t pick = head;
    uint64_t m = trunc_key(sites[n - 1 - head].read_weight);
    int64_t from = head;  // the head is compared against itself too
    for (;;) {
      int64_t q = first_below(1, 0, sz - 1, from, m);
      if (q < 0) break;
      pick = q;
      m = trunc_key(sites[n - 1 - q].read_weight);
      from = q + 1;
    }
    alive[pick] = 0;
    remove(pick);
    removal.push_back(n - 1 - pick);
  }
  for (int64_t i = n - 1; i >= 0; i--) out.push_back(removal[i]);
  return out;
}

const char* kHitNames[9] = {"L1 Hit",         "L2 Hit",           "L3 Hit",
                            "LFB Hit",        "Local RAM Hit",    "Remote RAM Hit",
                            "Remote cache Hit", "IO memory Hit",  "Uncached memory Hit"};
const char* kMissNames[9] = {nullptr,          nullptr,           nullptr,
                             "LFB Miss",       "Local RAM Miss",  "Remote RAM Miss",
                             "Remote cache Miss", "IO memory Miss", "Uncached memory Miss"};

// __print_counters (mem_analyzer.c:1438-1487)
void print_counters(FILE* f, const nmg_mem_counters* counters) {
  for (int i = 0; i < 2; i++) {
    const nmg_mem_counters& c = counters[i];
    if (i == 0) {
      fprintf(f, "\n");
      fprintf(f, "# --------------------------------------\n");
      fprintf(f, "# Summary of all the read memory access:\n");
    } else {
      fprintf(f, "# --------------------------------------\n");
      fprintf(f, "# Summary of all the write memory access:\n");
    }
    fprintf(f, "# Total count          : \t %" PRIu64 "\n", c.total_count);
    fprintf(f, "# Total weigh          : \t %" PRIu64 "\n", c.total_weight);
    if (c.na_miss_count)
      fprintf(f, "# N/A                  : \t %" PRIu64 " (%f %%)\n", c.na_miss_count,
              100. * c.na_miss_count / c.total_count);
    auto line = [&](int b, const char* name) {
      const nmg_count& k = c.b[b];
      if (!k.count) return;
      double pct = 100. * k.count / c.total_count;
      uint64_t avg = k.count ? k.sum_weight / k.count : 0;
      double wpct = c.total_weight ? 100. * k.sum_weight / c.total_weight : 0;
      fprintf(f,
              "# %s\t: %ld (%f %%) \tmin: %" PRIu64 " cycles\tmax: %" PRIu64 " cycles\t avg: %" PRIu64
              " cycles\ttotal weight: %" PRIu64 " (%f %%)\n",
              name, (long)k.count, pct, k.min_weight, k.max_weight, avg, k.sum_weight, wpct);
    };
    for (int g = 0; g < 9; g++) line(g, kHitNames[g]);
    fprintf(f, "\n");
    for (int g = 3; g < 9; g++) line(9 + g, kMissNames[g]);
  }
}

// Per-site page x thread matrix (__plot_counters input): dense unless huge.
struct SiteHist {
  uint64_t rows = 0;
  uint32_t T = 0;
  bool dense = true;
  std::vector<uint32_t> cells;                    // [page][thread]
  std::unordered_map<uint64_t, uint32_t> sparse;  // page * T + thread
  void init(uint64_t r, uint32_t t) {
    rows = r;
    T = t;
    dense = r * t <= (1ull << 26);
    if (dense) cells.assign(r * t, 0);
  }
  void add(uint64_t page, uint32_t th, uint32_t v) {
    if (page >= rows || th >= T) return;
    if (dense) cells[page * T + th] += v;
    else sparse[page * T + th] += v;
  }
  uint32_t get(uint64_t page, uint32_t th) const {
    if (dense) return cells[page * T + th];
    auto it = sparse.find(page * T + th);
    return it == sparse.end() ? 0 : it->second;
  }
};

// get_data_src_level() belongs to numap (unpinned HEAD, absent here): only
// "L1_Hit", "L2_Hit" and "L3_Hit" are pinned, by README.md:142-147.  The same
// restatement as the oracle's o_data_src_level: the first level bit present
// names the level, then "_Hit" / "_Miss".
std::string data_src_level(uint64_t data_src) {
  const uint32_t lvl = (uint32_t)(data_src >> 5) & 0x3fff;  // union perf_mem_data_src.mem_lvl
  static const struct {
    uint32_t bit;
    const char* name;
  } names[] = {{0x01, "NA"},
               {0x08, "L1"},
               {0x10, "LFB"},
               {0x20, "L2"},
               {0x40, "L3"},
               {0x80, "Local_RAM"},
               {0x100, "Remote_RAM_1_hop"},
               {0x200, "Remote_RAM_2_hops"},
               {0x400, "Remote_Cache_1_hop"},
               {0x800, "Remote_Cache_2_hops"},
               {0x1000, "IO_Memory"},
               {0x2000, "Uncached_Memory"}};
  const char* n = "Unknown";
  for (const auto& x : names)
    if (lvl & x.bit) {
      n = x.name;
      break;
    }
  return std::string(n) + ((lvl & 0x02) ? "_Hit" : ((lvl & 0x04) ? "_Miss" : ""));
}

template <class T>
T load(const uint8_t* p) {
  T v;
  memcpy(&v, p, sizeof(T));
  return v;
}

// The unmatched-sample log header (mem_sampling.c:608-638): the traced
// process's maps file copied by `while (!feof) { fgets(line, 1024); fprintf }`,
// which repeats the last line when the file ends with a newline.
void write_maps_header(FILE* f, const nmg_report_options* opts) {
  fprintf(f, "# %s content:\n", opts->maps_path ? opts->maps_path : "/proc/self/maps");
  const char* t = opts->maps_text ? opts->maps_text : "";
  const size_t len = strlen(t);
  char line[1024];
  line[0] = 0;
  size_t pos = 0;
  bool eof = len == 0;
  while (!eof) {
    if (pos >= len) {
      eof = true;  // fgets returns NULL; line keeps the last line
    } else {
      size_t n = 0;
      while (pos < len && n < sizeof(line) - 1) {
        line[n++] = t[pos++];
        if (line[n - 1] == '\n') break;
      }
      line[n] = 0;
      if (pos >= len && line[n - 1] != '\n') eof = true;  // EOF met inside the last line
    }
    fprintf(f, "# %s", line);
  }
  fprintf(f, "#\n#\n#\n");
  fprintf(f, "#thread_rank timestamp address mem_level access_weight access_type\n");
}

// dladdr() of a callstack frame, from the traced process's module table
const nmg_module* find_module(const std::vector<const nmg_module*>& mods, uint64_t rip) {
  auto it = std::upper_bound(mods.begin(), mods.end(), rip,
                             [](uint64_t x, const nmg_module* m) { return x < m->lo; });
  if (it == mods.begin()) return nullptr;
  const nmg_module* m = *(it - 1);
  return rip < m->hi ? m : nullptr;
}

// print_object_summary (mem_analyzer.c:1728-1748): one row per object of
// mem_list in FOREACH_HASH order (= the table's entry order).  Under
// USE_HASHTABLE (:23) print_object_summary_from_list ignores its list
// argument, so the second call, meant for past_mem_list, prints mem_list
// again (quirk Q20: every row twice).
int write_object_summary(const std::string& path, const nmg_host_results* r, const nmg_object_meta* meta,
                         const nmg_report_options* opts, std::string& err) {
  FILE* f = fopen(path.c_str(), "w");
  if (!f) {
    err = "cannot open " + path;
    return NMG_ERR_IO;
  }
  std::vector<const nmg_module*> mods;
  for (uint32_t i = 0; opts->modules && i < opts->nb_modules; i++) mods.push_back(&opts->modules[i]);
  std::sort(mods.begin(), mods.end(), [](const nmg_module* a, const nmg_module* b) { return a->lo < b->lo; });
  fprintf(f, "#object_id\taddress\tsize\tallocation_date\tdeallocation_date\tcallstack_rip\tcallstack_offsets"
             "\tcallsite_rip\tcallsite\n");
  // _print_object_summary (:1642-1704)
  std::vector<std::string> rows(r->nb_entries);
  std::string rips, offs;
  char buf[64];
  for (uint32_t e = 0; e < r->nb_entries; e++) {
    const nmg_object& o = r->objects[e];
    const nmg_object_meta& m = meta[e];
    rips.clear();
    offs.clear();
    if (m.callstack) {
      for (int32_t i = 3; i < m.callstack_size; i++) {
        const uint64_t rip = m.callstack[i];
        const char* prefix = i == 3 ? "" : ",";
        const nmg_module* mod = find_module(mods, rip);
        const uint64_t fbase = mod ? mod->fbase : 0;
        snprintf(buf, sizeof(buf), "%s0x%" PRIx64, prefix, rip);
        rips += buf;
        offs += prefix;
        offs += mod && mod->fname ? mod->fname : "(null)";
        snprintf(buf, sizeof(buf), ":%td", (ptrdiff_t)(rip - fbase));
        offs += buf;
      }
    } else {
      rips = "NULL";
      offs = "NULL";
    }
    std::string& row = rows[e];
    snprintf(buf, sizeof(buf), "%d\t0x%" PRIx64 "\t%ld\t", (int)m.id, o.buffer_addr, (long)o.buffer_size);
    row = buf;
    snprintf(buf, sizeof(buf), "%" PRIu64 "\t%" PRIu64 "\t", o.alloc_date, o.free_date);
    row += buf;
    row += rips;
    row += '\t';
    row += offs;
    snprintf(buf, sizeof(buf), "\t0x%" PRIx64 "\t", m.caller_rip);
    row += buf;
    row += Registry::caller_string(m);
    row += '\n';
  }
  for (int pass = 0; pass < 2; pass++)
    for (const std::string& row : rows) fwrite(row.data(), 1, row.size(), f);
  fclose(f);
  return NMG_OK;
}

}  // namespace

int write_report(const nmg_host_results* r, const nmg_object_meta* meta, const nmg_report_options* opts,
                 const char* stdout_path, std::string& err, const DumpInput* dump, const uint64_t* found_override) {
  // NMG_REPORT_TIMING=1: phase times on stderr
  const bool timing = getenv("NMG_REPORT_TIMING") != nullptr;
  auto t_last = std::chrono::steady_clock::now();
  auto phase = [&](const char* name) {
    if (!timing) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "nmg_report: %s %.3f s\n", name, std::chrono::duration<double>(t - t_last).count());
    t_last = t;
  };
  const uint32_t E = r->nb_entries;
  const uint32_t T = r->nb_threads;
  FILE* out = stdout;
  if (stdout_path) {
    out = fopen(stdout_path, "w");
    if (!out) {
      err = std::string("cannot open ") + stdout_path;
      return NMG_ERR_IO;
    }
  }
  auto close_out = [&]() {
    if (out != stdout) fclose(out);
    else fflush(out);
  };

  // ---- mem_sampling_finalize's messages (mem_sampling.c:321-344; none online, :313)
  const bool online = opts && opts->online;
  if (online && opts->dump_flags) {  // the reference's _dump_* read the NULL `samples` list online
    close_out();
    err = "dump modes are not available with online analysis (mem_sampling.c:644, 764, 799)";
    return NMG_ERR_INVALID;
  }
  const int nbuf = (int)r->nb_buffers;
  if (!online) fprintf(out, "Analyzing %d sample buffers\n", nbuf);
  uint64_t so_far = 0, found_total = 0;
  size_t total_bytes = 0;
  for (int b = 0; b < nbuf; b++) {
    if (b % 10 == 0 && !online)
      fprintf(out, "\rAnalyzing sample buffer %d/%d. Total samples so far: %zu", b, nbuf, (size_t)so_far);
    so_far += (uint64_t)(int64_t)(int32_t)r->buf_samples[b];  // int nb_samples (:325, :334, :934)
    found_total += (uint64_t)(int64_t)(int32_t)r->buf_found[b];
    total_bytes += r->buf_bytes[b];
  }
  const uint64_t nb_samples_total = so_far;
  if (found_override) found_total = *found_override;
  if (!online) {
    fprintf(out, "\n");
    fprintf(out, "%zu bytes processed\n", total_bytes);
  }
  fprintf(out, "---------------------------------\n");
  fprintf(out, "         MEM ANALYZER\n");
  fprintf(out, "---------------------------------\n");

  // ---- call sites
  phase("buffers");
  Registry reg(meta);
  std::vector<uint32_t> matched;
  if (r->match_samples) {
    for (uint32_t e = 0; e < E; e++)
      if (r->first_ordinal[e] != ~0ull) matched.push_back(e);
    // objects that reach update_call_sites: the matched ones, or every one online
    std::vector<uint32_t> updated;
    if (online)
      for (uint32_t e = 0; e < E; e++) updated.push_back(e);
    else
      updated = matched;
    for (uint32_t e : updated)
      if (meta[e].callstack == nullptr && meta[e].callstack_size > 3) {
        close_out();
        err = "entry with NULL callstack and callstack_size > 3 (the reference dereferences NULL)";
        return NMG_ERR_INVALID;
      }
    // creation: in the analysis order of each object's first matched sample
    std::vector<uint32_t> order(matched);
    std::sort(order.begin(), order.end(),
              [&](uint32_t a, uint32_t b) { return r->first_ordinal[a] < r->first_ordinal[b]; });
    phase("registry: order");
    for (uint32_t e : order)
      if (reg.find(e) < 0) reg.create(e, r->buffer_size[e] / kPageSize + 1);
    phase("registry: create");
    // update_call_sites in FOREACH_HASH order (= flattened order); online, an
    // object never matched finds or creates its site here
    for (uint32_t e : updated) {
      int si = reg.find(e);
      if (si < 0) si = reg.create(e, r->buffer_size[e] / kPageSize + 1);
      Site& site = reg.sites[si];
      site.nb_mallocs++;
      const uint64_t* cw = r->count_weight + (uint64_t)e * 4;
      site.read_count += cw[0];
      site.read_weight += cw[1];
      site.write_count += cw[2];
      site.write_weight += cw[3];
      site.objects.push_back(e);
    }
  }
  std::vector<Site>& sites = reg.sites;
  phase("call-site registry");

  // ---- dump modes (mem_sampling.c:895-914): per SAMPLE record in analysis order
  const char* dir = opts && opts->output_dir ? opts->output_dir : ".";
  const int dflags = opts ? opts->dump_flags : 0;
  const bool dump_single = opts ? opts->dump_single_items != 0 : true;
  mkdir(dir, S_IRWXU);  // get_log_dir (mem_intercept.c:402-409)
  std::vector<FILE*> site_file(sites.size(), nullptr);
  FILE* all_file = nullptr;
  FILE* unmatched_file = nullptr;
  auto open_out = [&](const std::string& base) -> FILE* {
    FILE* f = fopen((std::string(dir) + "/" + base).c_str(), "w");
    if (!f) err = "cannot open " + std::string(dir) + "/" + base;
    return f;
  };
  auto close_dumps = [&]() {
    for (FILE*& f : site_file)
      if (f) fclose(f), f = nullptr;
    if (all_file) fclose(all_file), all_file = nullptr;
    if (unmatched_file) fclose(unmatched_file), unmatched_file = nullptr;
  };
  if (dflags & NMG_DUMP_UNMATCHED) {  // opened at init (mem_intercept.c:528-535)
    unmatched_file = open_out("unmatched_samples.log");
    if (!unmatched_file) {
      close_out();
      return NMG_ERR_IO;
    }
  }
  if (dump && r->match_samples) {
    bool maps_read = false;
    const bool dump_matched = dflags & (NMG_DUMP_CALLSITES | NMG_DUMP_ALL);
    for (const DumpBuffer& b : dump->buffers) {
      const char acc = b.access == NMG_ACCESS_READ ? 'r' : 'w';
      for (uint64_t cur = 0; cur + 8 <= b.len;) {
        const uint32_t type = load<uint32_t>(b.data + cur);
        const uint16_t size = load<uint16_t>(b.data + cur + 6);
        if (size == 0) break;  // (the analysis already reported it)
        if (type == 9 && cur + 40 <= b.len) {
          const uint64_t ts = load<uint64_t>(b.data + cur + 8), addr = load<uint64_t>(b.data + cur + 16);
          const uint64_t w = load<uint64_t>(b.data + cur + 24), dsrc = load<uint64_t>(b.data + cur + 32);
          const uint32_t m = b.match[cur / 8];
          if (!m) {
            if (unmatched_file) {
              if (!maps_read) {
                write_maps_header(unmatched_file, opts);
                maps_read = true;
              }
              fprintf(unmatched_file, "%u %" PRIu64 " 0x%" PRIxPTR " %s %" PRIu64 " %c\n", b.thread_rank, ts,
                      (uintptr_t)addr, data_src_level(dsrc).c_str(), w, acc);
            }
          } else if (dump_matched) {
            const uint32_t e = m - 1;
            const uint64_t offset = addr - dump->entry_addr[e];
            if ((dflags & NMG_DUMP_ALL) && meta[e].mem_type != kMemTypeStack) {  // _dump_mem_info (:740-773)
              if (!all_file) {
                if (!(all_file = open_out("all_memory_accesses.dat"))) break;
                fprintf(all_file, "#thread_rank timestamp object_id offset mem_level access_weight access_type\n");
              }
              fprintf(all_file, "%u %" PRIu64 " %u %" PRIu64 " %s %" PRIu64 " %c\n", b.thread_rank, ts, meta[e].id,
                      offset, data_src_level(dsrc).c_str(), w, acc);
            }
            if (dump_single && meta[e].mem_type != kMemTypeStack) {  // _dump_call_site (:775-808)
              const int64_t si = reg.find(e);
              if (si >= 0) {
                if (!site_file[si]) {
                  char fn[64];
                  snprintf(fn, sizeof(fn), "callsite_dump_%d.dat", (int)sites[si].id);
                  if (!(site_file[si] = open_out(fn))) break;
                  fprintf(site_file[si], "#thread_rank timestamp offset mem_level access_weight access_type\n");
                }
                fprintf(site_file[si], "%u %" PRIu64 " %" PRIuPTR " %s %" PRIu64 " %c\n", b.thread_rank, ts,
                        (uintptr_t)offset, data_src_level(dsrc).c_str(), w, acc);
              }
            }
          }
        }
        cur += size;
      }
      if (!err.empty()) {
        close_dumps();
        close_out();
        return NMG_ERR_IO;
      }
    }
  }

  // ---- ma_finalize prints (mem_analyzer.c:1877-1881)
  phase("dumps");
  print_counters(out, r->global);
  fprintf(out, "Summary of the call sites:\n");
  fprintf(out, "--------------------------\n");
  fprintf(out, "Sorting call sites\n");
  std::vector<int64_t> order = sort_sites(sites);
  phase("sort");
  // __remove_site during the sort (mem_analyzer.c:1506-1528): the site the
  // walk stops at -- the removed one when it heads the list, else its
  // predecessor (quirk Q10) -- gets callsite_summary_<id>.dat and its dump
  // file closed, if it has one.  The list is id-descending; removals run in
  // the reverse of the final order.
  if (dump) {
    std::set<int64_t> remaining;
    for (int64_t i = 0; i < (int64_t)sites.size(); i++) remaining.insert(i);
    for (auto it = order.rbegin(); it != order.rend(); ++it) {
      auto pos = remaining.find(*it);
      auto nxt = std::next(pos);
      const int64_t cur = nxt == remaining.end() ? *it : *nxt;
      remaining.erase(pos);
      if (!site_file[cur]) continue;
      // __print_call_site_stats (:1489-1503): the cumulated counters, whose
      // min / max stay 0 (memset, and ACC_COUNTER's inverted tests: Q8)
      nmg_mem_counters cc[2];
      memset(cc, 0, sizeof(cc));
      for (uint32_t e : sites[cur].objects)
        for (uint32_t a = 0; a < 2; a++) {
          const uint64_t* cw = r->count_weight + (uint64_t)e * 4 + a * 2;
          const uint64_t* lv = dump->levels + ((uint64_t)e * 2 + a) * kLevelWords;
          cc[a].total_count += cw[0];
          cc[a].total_weight += cw[1];
          cc[a].na_miss_count += lv[0];
          for (int k = 0; k < 18; k++) {
            cc[a].b[k].count += lv[1 + 2 * k];
            cc[a].b[k].sum_weight += lv[2 + 2 * k];
          }
        }
      char fn[64];
      snprintf(fn, sizeof(fn), "callsite_summary_%d.dat", (int)sites[cur].id);
      FILE* sf = open_out(fn);
      if (!sf) {
        close_dumps();
        close_out();
        return NMG_ERR_IO;
      }
      print_counters(sf, cc);
      fclose(sf);
      fclose(site_file[cur]);
      site_file[cur] = nullptr;
    }
  }
  close_dumps();  // the rest stay open until exit in the reference
  std::string cs_path = std::string(dir) + "/call_sites.log";
  FILE* cf = fopen(cs_path.c_str(), "w");
  if (!cf) {
    close_out();
    err = "cannot open " + cs_path;
    return NMG_ERR_IO;
  }
  // per-entry ranges of the (entry, thread, page, count) rows
  std::vector<int64_t> cell_begin;
  auto index_cells = [&]() {
    if (!cell_begin.empty()) return;
    cell_begin.assign((size_t)E + 1, 0);
    for (int64_t i = 0; i < r->nb_cells; i++) cell_begin[r->cells[4 * i] + 1]++;
    for (uint32_t e = 0; e < E; e++) cell_begin[e + 1] += cell_begin[e];
  };

  int rc = NMG_OK;
  std::vector<int64_t> jobs;  // sites whose page file is written (in report order)
  for (int64_t idx : order) {
    const Site& s = sites[idx];
    if (!(s.read_count || s.write_count)) continue;
    double avg = 0;
    if (s.read_count) avg = (double)s.read_weight / s.read_count;
    for (int k = 0; k < 2; k++)
      fprintf(k ? out : cf,
              "%d\t%s (size=%zu) - %d buffers. %zu read access (total weight: %" PRIu64
              ", avg weight: %f). %" PRIu64 " wr_access\n",
              (int)s.id, s.caller.c_str(), (size_t)s.buffer_size, (int)s.nb_mallocs, (size_t)s.read_count,
              s.read_weight, avg, s.write_count);
    if (dump_single && s.mem_type != kMemTypeStack) jobs.push_back(idx);
  }
  if (!jobs.empty()) {
    // __plot_counters (mem_analyzer.c:1557-1585): one callsite_counters_<id>.dat
    // per site, (buffer_size / 4096 + 1) rows x next_thread_rank columns.  The
    // files are independent: written by a pool of host threads
    // (NMG_REPORT_THREADS, default min(16, cores)).
    index_cells();
    unsigned nth = std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    if (const char* e = getenv("NMG_REPORT_THREADS")) nth = (unsigned)std::max(1, atoi(e));
    nth = (unsigned)std::min<size_t>(nth, jobs.size());
    std::atomic<size_t> next{0};
    std::mutex mu;
    auto work = [&]() {
      std::string line;
      char cell[16];
      for (size_t j; (j = next.fetch_add(1)) < jobs.size();) {
        const Site& s = sites[jobs[j]];
        SiteHist sh;
        const uint64_t rows = s.mem_info_buffer_size / kPageSize + 1;
        sh.init(rows, T);
        for (uint32_t e : s.objects)
          for (int64_t i = cell_begin[e]; i < cell_begin[e + 1]; i++) {
            const uint32_t* c = r->cells + 4 * i;
            sh.add(c[2], c[1], c[3]);
          }
        char fn[4096];
        snprintf(fn, sizeof(fn), "%s/callsite_counters_%d.dat", dir, (int)s.id);
        FILE* df = fopen(fn, "w");
        if (!df) {
          std::lock_guard<std::mutex> g(mu);
          if (rc == NMG_OK) {
            rc = NMG_ERR_IO;
            err = std::string("cannot open ") + fn;
          }
          next = jobs.size();  // stop the pool
          break;
        }
        for (uint64_t i = 0; i < rows; i++) {
          line.clear();
          for (uint32_t th = 0; th < T; th++) {
            int n = snprintf(cell, sizeof(cell), "\t%d", (int)sh.get(i, th));
            line.append(cell, n);
          }
          line.push_back('\n');
          fwrite(line.data(), 1, line.size(), df);
        }
        fclose(df);
      }
    };
    std::vector<std::thread> pool;
    for (unsigned t = 1; t < nth; t++) pool.emplace_back(work);
    work();
    for (std::thread& t : pool) t.join();
  }
  fclose(cf);
  phase("call_sites.log + page files");
  if (!rc && (dflags & NMG_DUMP_ALL)) {
    if (r->objects)
      rc = write_object_summary(std::string(dir) + "/all_memory_objects.dat", r, meta, opts, err);
    else {
      rc = NMG_ERR_INVALID;
      err = "NMG_DUMP_ALL needs nmg_host_results.objects (all_memory_objects.dat)";
    }
  }
  if (rc) {
    close_out();
    return rc;
  }
  // mem_sampling_statistics (mem_sampling.c:357-361): a float percentage
  float percent = 100.0 * (nb_samples_total - found_total) / nb_samples_total;
  fprintf(out, "%" PRIu64 " samples (including %" PRIu64 " samples that do not match a known memory buffer / %f%%)\n",
          nb_samples_total, nb_samples_total - found_total, percent);
  close_out();
  return NMG_OK;
}

}  // namespace nmg

extern "C" int nmg_report_host(const nmg_host_results* res, const nmg_object_meta* meta,
                               const nmg_report_options* opts, const char* stdout_path) {
  if (!res || (res->nb_entries && (!meta || !res->first_ordinal || !res->count_weight || !res->buffer_size)) ||
      (res->nb_buffers && (!res->buf_samples || !res->buf_found || !res->buf_bytes)) ||
      (res->nb_cells && !res->cells) || res->nb_threads > NMG_MAX_THREADS)
    return NMG_ERR_INVALID;
  for (int64_t i = 0; i < res->nb_cells; i++)
    if (res->cells[4 * i] >= res->nb_entries || (i && res->cells[4 * i] < res->cells[4 * i - 4]))
      return NMG_ERR_INVALID;
  std::string err;
  int rc = nmg::write_report(res, meta, opts, stdout_path, err);
  if (rc && !err.empty()) fprintf(stderr, "nmg_report: %s\n", err.c_str());
  return rc;
}
