// nmg_replay.cpp -- replay-file driver for the engine: the C++ stand-in for
// the reference's LD_PRELOAD host while no live capture is available (no PMU
// in the container, numap absent).  It plays the role of ma_finalize: hands
// the object-table snapshot and every captured buffer (in `samples` order) to
// the engine, then writes the reference's report.  Format: DESIGN.md
// "Replay format".
#include <cerrno>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "nmg_internal.h"

namespace {

constexpr size_t kEntryBytes = 72;

// page-aligned, page-padded storage for the loaded replay (NMG_REPLAY_REGISTER:
// nmg_register_host pins whole pages, which must hold nothing else)
template <class T>
struct PageAlloc {
  using value_type = T;
  PageAlloc() = default;
  template <class U>
  PageAlloc(const PageAlloc<U>&) {}
  T* allocate(size_t n) {
    void* p = nullptr;
    const size_t b = std::max<size_t>((n * sizeof(T) + 4095) & ~size_t(4095), 4096);
    if (posix_memalign(&p, 4096, b)) throw std::bad_alloc();
    return static_cast<T*>(p);
  }
  void deallocate(T* p, size_t) { free(p); }
  template <class U>
  bool operator==(const PageAlloc<U>&) const { return true; }
  template <class U>
  bool operator!=(const PageAlloc<U>&) const { return false; }
};

struct Replay {
  std::vector<uint8_t, PageAlloc<uint8_t>> file;
  uint32_t nb_threads = 0, nb_keys = 0, nb_entries = 0, nb_buffers = 0;
  const uint64_t* keys = nullptr;
  const uint32_t* entry_off = nullptr;
  std::vector<nmg_object> objects;
  std::vector<nmg_object_meta> meta;
  struct Buf {
    uint32_t rank, access;
    uint64_t tail, head, ring;
    const uint8_t* bytes;
  };
  std::vector<Buf> bufs;
  // optional trailing context section (dump modes of the traced process)
  std::vector<nmg_module> modules;  // fname points into `file`
  std::string maps_path, maps_text;
  bool has_maps_path = false;
};

constexpr char kCtxMagic[8] = {'N', 'M', 'G', 'M', 'O', 'D', 'S', '1'};

template <class T>
T get(const uint8_t* p) {
  T v;
  memcpy(&v, p, sizeof(T));
  return v;
}
size_t pad8(size_t x) { return (x + 7) & ~size_t(7); }

int load_replay(const char* path, Replay& r, std::string& err) {
  FILE* f = fopen(path, "rb");
  if (!f) {
    err = std::string("cannot open ") + path + ": " + strerror(errno);
    return NMG_ERR_IO;
  }
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  r.file.resize(sz > 0 ? (size_t)sz : 0);
  size_t got = fread(r.file.data(), 1, r.file.size(), f);
  fclose(f);
  if (got != r.file.size() || r.file.size() < 64) {
    err = "short replay file";
    return NMG_ERR_INVALID;
  }
  const uint8_t* p = r.file.data();
  if (memcmp(p, "NMGRPLY1", 8) != 0 || get<uint32_t>(p + 8) != 1) {
    err = "bad replay magic/version";
    return NMG_ERR_INVALID;
  }
  r.nb_threads = get<uint32_t>(p + 12);
  r.nb_keys = get<uint32_t>(p + 16);
  r.nb_entries = get<uint32_t>(p + 20);
  r.nb_buffers = get<uint32_t>(p + 24);
  uint64_t cs_len = get<uint64_t>(p + 32), str_len = get<uint64_t>(p + 40);
  size_t off = 64;
  // every size is checked against the file before it is added to an offset
  // (header values come from the file and may be anything)
  const uint64_t fsz = r.file.size();
  if (cs_len > fsz / 8 || str_len > fsz) {
    err = "truncated object table";
    return NMG_ERR_INVALID;
  }
  const uint64_t need = off + 8ull * r.nb_keys + pad8(4ull * (r.nb_keys + 1)) + (uint64_t)kEntryBytes * r.nb_entries +
                        8 * cs_len + pad8(str_len);
  if (need > fsz) {
    err = "truncated object table";
    return NMG_ERR_INVALID;
  }
  r.keys = reinterpret_cast<const uint64_t*>(p + off);
  off += 8ull * r.nb_keys;
  r.entry_off = reinterpret_cast<const uint32_t*>(p + off);
  off += pad8(4ull * (r.nb_keys + 1));
  const uint8_t* ent = p + off;
  off += kEntryBytes * r.nb_entries;
  const uint64_t* cs_pool = reinterpret_cast<const uint64_t*>(p + off);
  off += 8 * cs_len;
  const char* str_pool = reinterpret_cast<const char*>(p + off);
  off += pad8(str_len);
  r.objects.resize(r.nb_entries);
  r.meta.resize(r.nb_entries);
  for (uint32_t e = 0; e < r.nb_entries; e++) {
    const uint8_t* q = ent + kEntryBytes * e;
    nmg_object& o = r.objects[e];
    nmg_object_meta& m = r.meta[e];
    o.buffer_addr = get<uint64_t>(q + 0);
    o.buffer_size = get<uint64_t>(q + 8);
    m.initial_buffer_size = get<uint64_t>(q + 16);
    o.alloc_date = get<uint64_t>(q + 24);
    o.free_date = get<uint64_t>(q + 32);
    m.caller_rip = get<uint64_t>(q + 40);
    m.mem_type = get<uint32_t>(q + 48);
    m.id = get<uint32_t>(q + 52);
    uint32_t cs_off = get<uint32_t>(q + 56);
    m.callstack_size = get<int32_t>(q + 60);
    uint32_t caller_off = get<uint32_t>(q + 64);
    uint32_t has_cs = get<uint32_t>(q + 68);
    if (has_cs) {
      if (m.callstack_size < 0 || (uint64_t)cs_off + (uint64_t)m.callstack_size > cs_len) {
        err = "callstack out of range";
        return NMG_ERR_INVALID;
      }
      m.callstack = cs_pool + cs_off;
    } else {
      m.callstack = nullptr;
    }
    if (caller_off != 0xFFFFFFFFu) {
      // the string must end inside the pool (it is printed with %s)
      if (caller_off >= str_len || !memchr(str_pool + caller_off, 0, str_len - caller_off)) {
        err = "caller string out of range";
        return NMG_ERR_INVALID;
      }
      m.caller = str_pool + caller_off;
    } else {
      m.caller = nullptr;
    }
    m.reserved = 0;
  }
  for (uint32_t b = 0; b < r.nb_buffers; b++) {
    if (off + 32 > r.file.size()) {
      err = "truncated buffer header";
      return NMG_ERR_INVALID;
    }
    Replay::Buf B;
    B.rank = get<uint32_t>(p + off);
    B.access = get<uint32_t>(p + off + 4);
    B.tail = get<uint64_t>(p + off + 8);
    B.head = get<uint64_t>(p + off + 16);
    B.ring = get<uint64_t>(p + off + 24);
    off += 32;
    if (B.ring > r.file.size() - off || pad8(B.ring) > r.file.size() - off) {
      err = "truncated ring";
      return NMG_ERR_INVALID;
    }
    B.bytes = p + off;
    off += pad8(B.ring);
    r.bufs.push_back(B);
  }
  // context section: "NMGMODS1", u32 nb_modules, u32 names_bytes, u32
  // maps_path_bytes, u32 maps_text_bytes, u64 0; modules {u64 lo, hi, fbase,
  // u32 name_off, u32 0}; names pool; maps path; maps text (each padded to 8)
  if (off + 32 <= r.file.size() && memcmp(p + off, kCtxMagic, 8) == 0) {
    const uint32_t nm = get<uint32_t>(p + off + 8), nb_names = get<uint32_t>(p + off + 12);
    const uint32_t nb_path = get<uint32_t>(p + off + 16), nb_text = get<uint32_t>(p + off + 20);
    off += 32;
    // (u32 counts: the sums below cannot overflow 64 bits)
    const uint64_t mods_off = off, names_off = mods_off + 32ull * nm, path_off = names_off + pad8(nb_names),
                   text_off = path_off + pad8(nb_path);
    if (text_off + pad8(nb_text) > r.file.size() || (nb_names && p[names_off + nb_names - 1] != 0)) {
      err = "truncated context section";
      return NMG_ERR_INVALID;
    }
    for (uint32_t i = 0; i < nm; i++) {
      const uint8_t* q = p + mods_off + 32ull * i;
      const uint32_t name_off = get<uint32_t>(q + 24);
      if (name_off >= nb_names) {
        err = "module name out of range";
        return NMG_ERR_INVALID;
      }
      r.modules.push_back({get<uint64_t>(q), get<uint64_t>(q + 8), get<uint64_t>(q + 16),
                           reinterpret_cast<const char*>(p + names_off + name_off)});
    }
    r.has_maps_path = nb_path != 0;
    r.maps_path.assign(reinterpret_cast<const char*>(p + path_off), nb_path);
    r.maps_text.assign(reinterpret_cast<const char*>(p + text_off), nb_text);
  }
  return NMG_OK;
}

int write_raw(nmg_engine* h, const Replay& r, const char* path) {
  nmg::HostResults res;
  int rc = nmg::engine_download(h, res);
  if (rc) return rc;
  const uint32_t E = r.nb_entries;
  int64_t ncells = nmg_count_page_cells(h);
  if (ncells < 0) return (int)ncells;
  std::vector<uint32_t> rows(4 * (size_t)ncells);
  rc = nmg_get_page_cells(h, rows.data(), ncells);
  if (rc) return rc;
  FILE* f = fopen(path, "wb");
  if (!f) return NMG_ERR_IO;
  fwrite("NMGRES01", 1, 8, f);
  uint32_t hdr[4] = {E, (uint32_t)res.buf_samples.size(), nmg::engine_nb_threads(h), 0};
  fwrite(hdr, 4, 4, f);
  for (int a = 0; a < 2; a++) {
    const nmg_mem_counters& c = res.global[a];
    fwrite(&c.total_count, 8, 1, f);
    fwrite(&c.total_weight, 8, 1, f);
    fwrite(&c.na_miss_count, 8, 1, f);
    for (int k = 0; k < 18; k++) fwrite(&c.b[k], 8, 4, f);
  }
  fwrite(&res.nb_samples_total, 8, 1, f);
  fwrite(&res.nb_found_total, 8, 1, f);
  fwrite(res.buf_samples.data(), 4, res.buf_samples.size(), f);
  fwrite(res.buf_found.data(), 4, res.buf_found.size(), f);
  const bool lv = !res.levels.empty();
  for (uint32_t e = 0; e < E; e++) {
    uint64_t rec[1 + 2 * 39] = {0};
    rec[0] = res.first[e];
    for (int a = 0; a < 2; a++) {
      uint64_t* q = rec + 1 + 39 * a;
      q[0] = res.count_weight[(uint64_t)e * 4 + a * 2 + 0];
      q[1] = res.count_weight[(uint64_t)e * 4 + a * 2 + 1];
      if (lv) {
        const uint64_t* l = res.levels.data() + ((uint64_t)e * 2 + a) * nmg::kLevelWords;
        q[2] = l[0];
        for (int k = 0; k < 36; k++) q[3 + k] = l[1 + k];
      }
    }
    fwrite(rec, 8, 1 + 2 * 39, f);
  }
  uint64_t n = (uint64_t)ncells;
  fwrite(&n, 8, 1, f);
  fwrite(rows.data(), 4, rows.size(), f);
  fclose(f);
  return NMG_OK;
}

}  // namespace

extern "C" int nmg_run_replay(const char* replay_path, const char* output_dir, const char* stdout_path,
                              const char* raw_path, int device, uint32_t flags) {
  Replay r;
  std::string err;
  int rc = load_replay(replay_path, r, err);
  if (rc) {
    fprintf(stderr, "nmg_replay: %s\n", err.c_str());
    return rc;
  }
  nmg_options opt;
  memset(&opt, 0, sizeof(opt));
  opt.device = device;
  opt.flags = flags | (raw_path ? NMG_F_OBJECT_LEVELS : 0);
  // NMG_REPLAY_DUMP=<NMG_DUMP_* flags>: the dump modes, with the context
  // section's module table and maps file (the -d / -D / -u outputs)
  const char* dump_env = getenv("NMG_REPLAY_DUMP");
  const int dump_flags = dump_env ? atoi(dump_env) : 0;
  if (dump_flags) opt.flags |= NMG_F_SAMPLE_MATCHES | NMG_F_OBJECT_LEVELS;
  opt.nb_threads = r.nb_threads ? r.nb_threads : 1;
  // NMG_REPLAY_STREAM="chunk_bytes[:copy_threads[:batch]]": feed the buffers
  // in nmg_submit_buffers batches (unwrapped ring segments; wrapped ones through
  // nmg_submit_ring), through the streaming path when chunk_bytes > 0
  const char* stream = getenv("NMG_REPLAY_STREAM");
  unsigned long long chunk = 0;
  unsigned threads = 1, batch = 64;
  if (stream && *stream) sscanf(stream, "%llu:%u:%u", &chunk, &threads, &batch);
  opt.copy_threads = threads ? threads : 1;
  nmg_engine* h = nullptr;
  rc = nmg_create(&h, &opt);
  if (rc) {
    fprintf(stderr, "nmg_replay: nmg_create: %s\n", nmg_strerror(rc));
    return rc;
  }
  auto bail = [&](int code) {
    char detail[512];
    nmg_get_last_error_detail(h, detail, sizeof(detail));
    fprintf(stderr, "nmg_replay: %s (%s)\n", nmg_strerror(code), detail);
    nmg_destroy(h);
    return code;
  };
  rc = nmg_set_objects(h, r.keys, r.entry_off, r.nb_keys, r.objects.data(), r.nb_entries);
  if (rc) return bail(rc);
  // NMG_REPLAY_REGISTER=1: the loaded replay (every ring) registered with
  // nmg_register_host, so 16-byte aligned unwrapped buffers are read in place
  const char* reg = getenv("NMG_REPLAY_REGISTER");
  const bool registered = reg && atoi(reg) && !r.file.empty();
  if (registered) {
    rc = nmg_register_host(h, r.file.data(), r.file.size());
    if (rc) return bail(rc);
  }
  if (stream && *stream) {
    if (chunk) {
      rc = nmg_stream_begin(h, chunk, threads ? threads : 1);
      if (rc) return bail(rc);
    }
    std::vector<const void*> ptrs;
    std::vector<uint64_t> lens;
    std::vector<uint32_t> ranks, accs;
    auto drain = [&]() {
      int e = ptrs.empty() ? NMG_OK
                           : nmg_submit_buffers(h, (uint32_t)ptrs.size(), ptrs.data(), lens.data(), ranks.data(),
                                                accs.data());
      ptrs.clear();
      lens.clear();
      ranks.clear();
      accs.clear();
      return e;
    };
    for (const auto& b : r.bufs) {
      if (b.head < b.tail) {  // wrapped: linearised by the engine (__copy_buffer)
        rc = drain();
        if (!rc) rc = nmg_submit_ring(h, b.bytes, b.ring, b.tail, b.head, b.rank, b.access);
      } else {
        ptrs.push_back(b.bytes + b.tail);
        lens.push_back(b.head - b.tail);
        ranks.push_back(b.rank);
        accs.push_back(b.access);
        rc = ptrs.size() >= (batch ? batch : 1) ? drain() : NMG_OK;
      }
      if (rc) return bail(rc);
    }
    rc = drain();
    if (rc) return bail(rc);
  } else {
    for (const auto& b : r.bufs) {
      rc = nmg_submit_ring(h, b.bytes, b.ring, b.tail, b.head, b.rank, b.access);
      if (rc) return bail(rc);
    }
  }
  rc = nmg_analyze(h);
  if (rc) return bail(rc);
  rc = nmg_synchronize(h);
  if (rc) return bail(rc);
  nmg_report_options ro;
  memset(&ro, 0, sizeof(ro));
  ro.output_dir = output_dir;
  ro.dump_single_items = 1;
  ro.dump_flags = dump_flags;
  ro.maps_path = r.has_maps_path ? r.maps_path.c_str() : nullptr;
  ro.maps_text = r.maps_text.empty() ? nullptr : r.maps_text.c_str();
  ro.modules = r.modules.data();
  ro.nb_modules = (uint32_t)r.modules.size();
  rc = nmg_report(h, r.meta.data(), &ro, stdout_path);
  if (rc) return bail(rc);
  if (raw_path) {
    rc = write_raw(h, r, raw_path);
    if (rc) return bail(rc);
  }
  nmg_destroy(h);
  return NMG_OK;
}

// ---------------------------------------------------------------------------
// capture side of the bridge: the replay writer (format: DESIGN.md §4,
// numamma_amd/replay.py).  Host-only; every write is checked.

struct nmg_replay_writer {
  FILE* f = nullptr;
  uint32_t nb_buffers = 0;
  uint32_t nb_threads = 0;
  bool ok = true;
  std::vector<uint8_t> ctx;  // context section, written by nmg_replay_close
};

namespace {

template <class T>
void put(std::vector<uint8_t>& out, T v) {
  const size_t n = out.size();
  out.resize(n + sizeof(T));
  memcpy(out.data() + n, &v, sizeof(T));
}
void pad_to8(std::vector<uint8_t>& out) { out.resize(pad8(out.size()), 0); }

}  // namespace

extern "C" int nmg_replay_open(nmg_replay_writer** out, const char* path, uint32_t nb_threads, const uint64_t* keys,
                               const uint32_t* entry_off, uint32_t nb_keys, const nmg_object* entries,
                               const nmg_object_meta* meta, uint32_t nb_entries) {
  if (!out || !path || (nb_keys && (!keys || !entry_off)) || (nb_entries && (!entries || !meta)))
    return NMG_ERR_INVALID;
  *out = nullptr;
  if (nb_threads > NMG_MAX_THREADS) return NMG_ERR_RANGE;
  if (entry_off && (entry_off[0] != 0 || entry_off[nb_keys] != nb_entries)) return NMG_ERR_INVALID;
  // pools: callstacks (u64) and caller strings (NUL-terminated), in entry order
  std::vector<uint64_t> cs_pool;
  std::string str_pool;
  std::vector<uint8_t> ent;
  ent.reserve((size_t)nb_entries * kEntryBytes);
  for (uint32_t e = 0; e < nb_entries; e++) {
    const nmg_object& o = entries[e];
    const nmg_object_meta& m = meta[e];
    uint32_t cs_off = 0, has_cs = 0, caller_off = 0xFFFFFFFFu;
    if (m.callstack) {
      if (m.callstack_size < 0) return NMG_ERR_INVALID;
      cs_off = (uint32_t)cs_pool.size();
      cs_pool.insert(cs_pool.end(), m.callstack, m.callstack + m.callstack_size);
      has_cs = 1;
    }
    if (m.caller) {
      caller_off = (uint32_t)str_pool.size();
      str_pool.append(m.caller);
      str_pool.push_back('\0');
    }
    put<uint64_t>(ent, o.buffer_addr);
    put<uint64_t>(ent, o.buffer_size);
    put<uint64_t>(ent, m.initial_buffer_size);
    put<uint64_t>(ent, o.alloc_date);
    put<uint64_t>(ent, o.free_date);
    put<uint64_t>(ent, m.caller_rip);
    put<uint32_t>(ent, m.mem_type);
    put<uint32_t>(ent, m.id);
    put<uint32_t>(ent, cs_off);
    put<int32_t>(ent, m.callstack_size);
    put<uint32_t>(ent, caller_off);
    put<uint32_t>(ent, has_cs);
  }
  std::vector<uint8_t> hdr;
  hdr.insert(hdr.end(), {'N', 'M', 'G', 'R', 'P', 'L', 'Y', '1'});
  put<uint32_t>(hdr, 1);
  put<uint32_t>(hdr, nb_threads);
  put<uint32_t>(hdr, nb_keys);
  put<uint32_t>(hdr, nb_entries);
  put<uint32_t>(hdr, 0);  // nb_buffers, patched by nmg_replay_close
  put<uint32_t>(hdr, 0);
  put<uint64_t>(hdr, cs_pool.size());
  put<uint64_t>(hdr, str_pool.size());
  put<uint64_t>(hdr, 0);
  put<uint64_t>(hdr, 0);
  for (uint32_t k = 0; k < nb_keys; k++) put<uint64_t>(hdr, keys[k]);
  for (uint32_t k = 0; k <= nb_keys; k++) put<uint32_t>(hdr, entry_off ? entry_off[k] : 0);
  pad_to8(hdr);
  hdr.insert(hdr.end(), ent.begin(), ent.end());
  for (uint64_t v : cs_pool) put<uint64_t>(hdr, v);
  hdr.insert(hdr.end(), str_pool.begin(), str_pool.end());
  pad_to8(hdr);
  nmg_replay_writer* w = new (std::nothrow) nmg_replay_writer();
  if (!w) return NMG_ERR_NOMEM;
  w->f = fopen(path, "wb");
  if (!w->f) {
    delete w;
    return NMG_ERR_IO;
  }
  w->nb_threads = nb_threads;
  if (fwrite(hdr.data(), 1, hdr.size(), w->f) != hdr.size()) {
    fclose(w->f);
    delete w;
    return NMG_ERR_IO;
  }
  *out = w;
  return NMG_OK;
}

extern "C" int nmg_replay_add_ring(nmg_replay_writer* w, const void* ring, uint64_t ring_size, uint64_t data_tail,
                                   uint64_t data_head, uint32_t thread_rank, uint32_t access_type) {
  if (!w || !w->f || (ring_size && !ring) || data_tail > ring_size || data_head > ring_size || access_type > 1)
    return NMG_ERR_INVALID;
  if (thread_rank >= NMG_MAX_THREADS || (w->nb_threads && thread_rank >= w->nb_threads)) return NMG_ERR_RANGE;
  std::vector<uint8_t> h;
  put<uint32_t>(h, thread_rank);
  put<uint32_t>(h, access_type);
  put<uint64_t>(h, data_tail);
  put<uint64_t>(h, data_head);
  put<uint64_t>(h, ring_size);
  static const uint8_t zeros[8] = {0};
  const size_t padn = pad8(ring_size) - ring_size;
  if (fwrite(h.data(), 1, h.size(), w->f) != h.size() || fwrite(ring, 1, ring_size, w->f) != ring_size ||
      fwrite(zeros, 1, padn, w->f) != padn) {
    w->ok = false;
    return NMG_ERR_IO;
  }
  w->nb_buffers++;
  return NMG_OK;
}

extern "C" int nmg_replay_set_context(nmg_replay_writer* w, const nmg_module* modules, uint32_t nb_modules,
                                      const char* maps_path, const char* maps_text) {
  if (!w || !w->f || (nb_modules && !modules)) return NMG_ERR_INVALID;
  std::string names;
  std::vector<uint8_t> mods;
  for (uint32_t i = 0; i < nb_modules; i++) {
    const nmg_module& m = modules[i];
    if (m.hi < m.lo) return NMG_ERR_INVALID;
    put<uint64_t>(mods, m.lo);
    put<uint64_t>(mods, m.hi);
    put<uint64_t>(mods, m.fbase);
    put<uint32_t>(mods, (uint32_t)names.size());
    put<uint32_t>(mods, 0);
    names.append(m.fname ? m.fname : "(null)");
    names.push_back('\0');
  }
  const std::string path = maps_path ? maps_path : "", text = maps_text ? maps_text : "";
  std::vector<uint8_t>& c = w->ctx;
  c.clear();
  c.insert(c.end(), kCtxMagic, kCtxMagic + 8);
  put<uint32_t>(c, nb_modules);
  put<uint32_t>(c, (uint32_t)names.size());
  put<uint32_t>(c, (uint32_t)path.size());
  put<uint32_t>(c, (uint32_t)text.size());
  put<uint64_t>(c, 0);
  c.insert(c.end(), mods.begin(), mods.end());
  c.insert(c.end(), names.begin(), names.end());
  pad_to8(c);
  c.insert(c.end(), path.begin(), path.end());
  pad_to8(c);
  c.insert(c.end(), text.begin(), text.end());
  pad_to8(c);
  return NMG_OK;
}

extern "C" int nmg_replay_close(nmg_replay_writer* w) {
  if (!w) return NMG_ERR_INVALID;
  bool ok = w->ok && w->f;
  if (ok && !w->ctx.empty()) ok = fwrite(w->ctx.data(), 1, w->ctx.size(), w->f) == w->ctx.size();
  if (w->f) {
    ok = ok && fseek(w->f, 24, SEEK_SET) == 0 && fwrite(&w->nb_buffers, 4, 1, w->f) == 1;
    ok = (fclose(w->f) == 0) && ok;
  }
  delete w;
  return ok ? NMG_OK : NMG_ERR_IO;
}
