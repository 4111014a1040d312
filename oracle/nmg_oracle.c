/*
 * nmg_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of NumaMMa's offline PEBS sample-analysis path, used as the
 * parity checker for the MI355X engine.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load or run this code, and only as the
 * checker / CPU baseline -- never as part of the product path.
 *
 * Parity status (see DESIGN.md "Oracle"):
 *   - object lookup (ht_lower_key + LIFO entry scan) is PINNED against the
 *     reference's own tools/hash.c compiled into oracle/_ref/ (randomised
 *     differential tests in tests/test_oracle_ref.py);
 *   - report formats are pinned against the reference README example outputs
 *     (tests/golden/readme_*.txt, whitespace-normalised);
 *   - counter / page-block / call-site semantics: the reference's
 *     mem_sampling.c and mem_analyzer.c cannot be built here (they need the
 *     absent numap + libpfm headers and a cmake-generated numamma.h), so these
 *     are restated from source, line by line, and are "parity unpinned"
 *     beyond the README examples.
 *
 * The restatement deliberately keeps the reference's data structures where
 * they shape the cost (sorted singly-linked per-thread page-block lists,
 * linear LIFO call-site list, O(S^2) selection sort) so that it doubles as a
 * faithful single-core CPU baseline.
 *
 * Citations are path:line in numamma/numamma (reference @ v2).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <inttypes.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>

#include "nmg_oracle.h"

#define MAX_THREADS 1024 /* src/numamma.h.in:9 */
#define PAGE_SIZE 4096   /* src/mem_analyzer.c:471 */
#define PERF_RECORD_SAMPLE 9
#define ACCESS_READ 0
#define ACCESS_WRITE 1
#define ACCESS_MAX 2

/* PERF_MEM_LVL_* -- /usr/include/linux/perf_event.h:1250-1263 */
#define LVL_NA 0x01
#define LVL_HIT 0x02
#define LVL_MISS 0x04
#define LVL_L1 0x08
#define LVL_LFB 0x10
#define LVL_L2 0x20
#define LVL_L3 0x40
#define LVL_LOC_RAM 0x80
#define LVL_REM_RAM1 0x100
#define LVL_REM_RAM2 0x200
#define LVL_REM_CCE1 0x400
#define LVL_REM_CCE2 0x800
#define LVL_IO 0x1000
#define LVL_UNC 0x2000

/* mem_type values -- src/mem_analyzer.h:58-64 */
#define MEM_TYPE_STACK 2

/* struct count / struct mem_counters -- src/mem_analyzer.h:10-41 */
struct o_count {
  uint64_t count, min_weight, max_weight, sum_weight;
};
struct o_counters {
  uint64_t total_count, total_weight, na_miss_count;
  struct o_count b[18]; /* 9 hit buckets then 9 miss buckets, header order */
};
enum {
  B_L1, B_L2, B_L3, B_LFB, B_LOC_RAM, B_REM_RAM, B_REM_CCE, B_IO, B_UNC
};

/* struct block_info -- src/mem_analyzer.h:52-56 */
struct o_block {
  unsigned block_id;
  struct o_counters counters[ACCESS_MAX];
  struct o_block *next;
};

/* flattened struct memory_info -- src/mem_analyzer.h:68-86 */
struct o_mem {
  uint64_t buffer_addr, buffer_size, initial_buffer_size;
  uint64_t alloc_date, free_date, caller_rip;
  uint32_t mem_type, id;
  const uint64_t *callstack; /* NULL == callstack_rip NULL */
  int callstack_size;
  const char *caller; /* NULL == not symbolised */
  struct o_block **blocks; /* NULL until first match (mem_sampling.c:654-658) */
  struct o_site *call_site;
  uint64_t first_ordinal; /* oracle bookkeeping for the raw-results dump */
};

/* struct call_site -- src/mem_analyzer.h:140-152 */
struct o_site {
  uint32_t id;
  char caller[1024];
  uint64_t caller_rip;
  const uint64_t *callstack;
  int callstack_size;
  uint64_t buffer_size; /* initial_buffer_size of the creating object */
  unsigned nb_mallocs;
  uint32_t mem_type;             /* site->mem_info.mem_type */
  uint64_t mem_info_buffer_size; /* site->mem_info.buffer_size (:1363) */
  struct o_block **blocks;       /* site->mem_info.blocks */
  struct o_block cumulated;      /* site->cumulated_counters */
  FILE *dump_file;               /* site->dump_file: callsite_dump_<id>.dat (dump modes) */
  struct o_site *next;
};

struct o_buffer {
  uint32_t thread_rank, access_type;
  uint8_t *data; /* linearised copy, as produced by __copy_buffer */
  uint64_t size;
};

struct o_state {
  /* object table (the AVL tree, flattened: sorted unique keys + LIFO entries) */
  uint32_t nb_keys, nb_entries, nb_threads;
  uint64_t *keys;
  uint32_t *entry_off;
  struct o_mem *mems;
  /* sample_list in analysis order */
  uint32_t nb_buffers;
  struct o_buffer *buffers;
  /* global state */
  struct o_counters global_counters[2]; /* mem_sampling.c:35 */
  uint64_t nb_samples_total, nb_found_samples_total;
  uint32_t *buf_samples, *buf_found;
  struct o_site *call_sites; /* mem_analyzer.c:1300 */
  uint32_t next_call_site_id;
  /* online analysis: the table at the current alarm (NULL: the replay's) */
  const struct nmo_alarm *snap;
  /* dump modes (settings.dump / dump_all / dump_unmatched) */
  const struct nmo_settings *set;
  const char *outdir;
  FILE *dump_all_file;       /* mem_sampling.c:24 */
  FILE *dump_unmatched_file; /* mem_intercept.c:26, opened at init (:528-535) */
  int maps_read;             /* mem_sampling.c:608 */
  int dump_err;
  /* raw file bytes */
  uint8_t *file;
  size_t file_size;
};

/* ------------------------------------------------------------------ */
/* replay file reader (format: DESIGN.md "Replay format")              */

static int rd_fail(const char *msg) {
  fprintf(stderr, "nmg_oracle: invalid replay: %s\n", msg);
  return NMO_ERR_FORMAT;
}

static uint64_t rd_u64(const uint8_t *p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}
static uint32_t rd_u32(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
static size_t pad8(size_t x) { return (x + 7) & ~(size_t)7; }

/*
 * Linearise a ring segment [tail, head) exactly like __copy_buffer
 * (src/mem_sampling.c:675-738).  Returns 0 when the ring is empty (the
 * reference never pushes such a buffer onto `samples`, :680-682).
 */
static uint64_t o_copy_buffer(const uint8_t *ring, uint64_t ring_size,
                              uint64_t tail, uint64_t head, uint8_t **out) {
  if (head == tail) return 0;
  uint64_t size = head - tail;
  if (head < tail) size = ring_size - tail + head; /* :687-694 */
  uint8_t *copy = malloc(size ? size : 1);
  if (head < tail) {
    uint64_t first = ring_size - tail; /* :704-713 */
    memcpy(copy, ring + tail, first);
    memcpy(copy + first, ring, head);
  } else {
    memcpy(copy, ring + tail, size); /* :714-718 */
  }
  *out = copy;
  return size;
}

static int o_load(struct o_state *st, const char *path) {
  FILE *f = fopen(path, "rb");
  if (!f) {
    fprintf(stderr, "nmg_oracle: cannot open %s: %s\n", path, strerror(errno));
    return NMO_ERR_IO;
  }
  fseek(f, 0, SEEK_END);
  long sz = ftell(f);
  fseek(f, 0, SEEK_SET);
  if (sz < 64) {
    fclose(f);
    return rd_fail("short header");
  }
  st->file = malloc((size_t)sz);
  st->file_size = (size_t)sz;
  if (fread(st->file, 1, (size_t)sz, f) != (size_t)sz) {
    fclose(f);
    return NMO_ERR_IO;
  }
  fclose(f);
  const uint8_t *p = st->file;
  if (memcmp(p, "NMGRPLY1", 8) != 0) return rd_fail("bad magic");
  if (rd_u32(p + 8) != 1) return rd_fail("bad version");
  st->nb_threads = rd_u32(p + 12);
  st->nb_keys = rd_u32(p + 16);
  st->nb_entries = rd_u32(p + 20);
  st->nb_buffers = rd_u32(p + 24);
  uint64_t cs_len = rd_u64(p + 32);
  uint64_t str_len = rd_u64(p + 40);
  size_t off = 64;
  size_t need = off + 8ull * st->nb_keys + pad8(4ull * (st->nb_keys + 1)) +
                72ull * st->nb_entries + 8 * cs_len + pad8(str_len);
  if (need > st->file_size) return rd_fail("truncated table");
  st->keys = (uint64_t *)(st->file + off);
  off += 8ull * st->nb_keys;
  st->entry_off = (uint32_t *)(st->file + off);
  off += pad8(4ull * (st->nb_keys + 1));
  const uint8_t *ent = st->file + off;
  off += 72ull * st->nb_entries;
  const uint64_t *cs_pool = (const uint64_t *)(st->file + off);
  off += 8 * cs_len;
  const char *str_pool = (const char *)(st->file + off);
  off += pad8(str_len);

  if (st->entry_off[0] != 0 || st->entry_off[st->nb_keys] != st->nb_entries)
    return rd_fail("entry offsets");
  for (uint32_t i = 0; i < st->nb_keys; i++) {
    if (st->entry_off[i + 1] <= st->entry_off[i]) return rd_fail("empty key");
    if (i && st->keys[i] <= st->keys[i - 1]) return rd_fail("keys not sorted");
  }
  st->mems = calloc(st->nb_entries ? st->nb_entries : 1, sizeof(struct o_mem));
  for (uint32_t e = 0; e < st->nb_entries; e++) {
    const uint8_t *r = ent + 72ull * e;
    struct o_mem *m = &st->mems[e];
    m->buffer_addr = rd_u64(r + 0);
    m->buffer_size = rd_u64(r + 8);
    m->initial_buffer_size = rd_u64(r + 16);
    m->alloc_date = rd_u64(r + 24);
    m->free_date = rd_u64(r + 32);
    m->caller_rip = rd_u64(r + 40);
    m->mem_type = rd_u32(r + 48);
    m->id = rd_u32(r + 52);
    uint32_t cs_off = rd_u32(r + 56);
    int32_t cs_size = (int32_t)rd_u32(r + 60);
    uint32_t caller_off = rd_u32(r + 64);
    uint32_t has_cs = rd_u32(r + 68);
    m->callstack_size = cs_size;
    if (has_cs) {
      if (cs_size < 0 || (uint64_t)cs_off + (uint64_t)cs_size > cs_len)
        return rd_fail("callstack range");
      m->callstack = cs_pool + cs_off;
    } else {
      /* a NULL callstack with size > 3 would be dereferenced by
       * find_call_site (mem_analyzer.c:1312-1313) and crash the reference */
      if (cs_size > 3) return rd_fail("NULL callstack with size > 3");
      m->callstack = NULL;
    }
    if (caller_off != 0xFFFFFFFFu) {
      if (caller_off >= str_len) return rd_fail("caller offset");
      m->caller = str_pool + caller_off;
    }
    m->first_ordinal = UINT64_MAX;
  }
  /* buffers */
  st->buffers = calloc(st->nb_buffers ? st->nb_buffers : 1, sizeof(struct o_buffer));
  uint32_t kept = 0;
  for (uint32_t b = 0; b < st->nb_buffers; b++) {
    if (off + 32 > st->file_size) return rd_fail("truncated buffer header");
    const uint8_t *h = st->file + off;
    uint32_t rank = rd_u32(h), access = rd_u32(h + 4);
    uint64_t tail = rd_u64(h + 8), head = rd_u64(h + 16), ring = rd_u64(h + 24);
    off += 32;
    if (off + pad8(ring) > st->file_size) return rd_fail("truncated ring");
    if (tail > ring || head > ring) return rd_fail("cursor beyond ring");
    if (rank >= MAX_THREADS) return rd_fail("thread rank >= MAX_THREADS");
    if (access >= ACCESS_MAX) return rd_fail("access type");
    uint8_t *copy = NULL;
    uint64_t size = o_copy_buffer(st->file + off, ring, tail, head, &copy);
    off += pad8(ring);
    if (!size) continue; /* empty ring: never pushed (mem_sampling.c:680-682) */
    if (size >= (1ull << 32)) return rd_fail("buffer >= 4 GiB (unsigned cursors, mem_sampling.c:831-834)");
    st->buffers[kept].thread_rank = rank;
    st->buffers[kept].access_type = access;
    st->buffers[kept].data = copy;
    st->buffers[kept].size = size;
    kept++;
  }
  st->nb_buffers = kept;
  return 0;
}

/* ------------------------------------------------------------------ */
/* counters                                                            */

/* INIT_COUNTER / init_mem_counter -- src/mem_analyzer.c:415-446 */
static void o_init_counters(struct o_counters *c) {
  c->total_count = c->total_weight = c->na_miss_count = 0;
  for (int i = 0; i < 18; i++) {
    c->b[i].count = 0;
    c->b[i].min_weight = UINT64_MAX;
    c->b[i].max_weight = 0;
    c->b[i].sum_weight = 0;
  }
}

/* UPDATE_COUNTER -- src/mem_sampling.c:508-515 */
static void o_update_count(struct o_count *c, uint64_t w) {
  c->count++;
  if (w < c->min_weight) c->min_weight = w;
  if (w > c->max_weight) c->max_weight = w;
  c->sum_weight += w;
}

/* update_counters -- src/mem_sampling.c:517-592 */
static void o_update_counters(struct o_counters *counters, uint64_t weight,
                              uint64_t data_src, int access) {
  struct o_counters *c = &counters[access];
  unsigned lvl = (unsigned)((data_src >> 5) & 0x3fff); /* mem_lvl:14 at bit 5 */
  c->total_count++;
  c->total_weight += weight;
  if (lvl & LVL_NA) c->na_miss_count++;
#define LEVEL(mask, idx)                                             \
  if (lvl & (mask)) {                                               \
    if (lvl & LVL_HIT) o_update_count(&c->b[idx], weight);          \
    else if (lvl & LVL_MISS) o_update_count(&c->b[9 + idx], weight); \
  }
  LEVEL(LVL_L1, B_L1)
  LEVEL(LVL_L2, B_L2)
  LEVEL(LVL_L3, B_L3)
  LEVEL(LVL_LFB, B_LFB)
  LEVEL(LVL_LOC_RAM, B_LOC_RAM)
  LEVEL(LVL_REM_RAM1 | LVL_REM_RAM2, B_REM_RAM)
  LEVEL(LVL_REM_CCE1 | LVL_REM_CCE2, B_REM_CCE)
  LEVEL(LVL_IO, B_IO)
  LEVEL(LVL_UNC, B_UNC)
#undef LEVEL
}

/* ------------------------------------------------------------------ */
/* object lookup                                                       */

/* ht_lower_key (tools/hash.c:63-77) on the flattened key array:
 * index of the largest key <= addr, or -1. */
static int64_t o_lower_key(const struct o_state *st, uint64_t addr) {
  int64_t lo = 0, hi = (int64_t)st->nb_keys - 1, best = -1;
  while (lo <= hi) {
    int64_t mid = lo + (hi - lo) / 2;
    if (st->keys[mid] <= addr) {
      best = mid;
      lo = mid + 1;
    } else {
      hi = mid - 1;
    }
  }
  return best;
}

/* is_sample_in_buffer -- src/mem_analyzer.c:141-155 (void* arithmetic wraps) */
static int o_in_buffer(const struct o_mem *m, uint64_t addr, uint64_t ts) {
  if (m->buffer_addr <= addr && addr < m->buffer_addr + m->buffer_size)
    if (m->alloc_date <= ts && ts <= m->free_date) return 1;
  return 0;
}

/* __ma_find_mem_info_from_sample_generic -- src/mem_analyzer.c:249-286:
 * only the lower-bound node is examined (no fallback to smaller keys); its
 * entries are scanned newest-first and the first hit wins. */
static int64_t o_find(const struct o_state *st, uint64_t addr, uint64_t ts, uint64_t *baddr) {
  if (st->snap) { /* online: the live mem_list at this alarm */
    const struct nmo_alarm *a = st->snap;
    int64_t lo = 0, hi = (int64_t)a->nb_keys - 1, k = -1;
    while (lo <= hi) {
      int64_t mid = lo + (hi - lo) / 2;
      if (a->keys[mid] <= addr) {
        k = mid;
        lo = mid + 1;
      } else {
        hi = mid - 1;
      }
    }
    if (k < 0) return -1;
    for (uint32_t j = a->entry_off[k]; j < a->entry_off[k + 1]; j++) {
      struct o_mem m;
      memset(&m, 0, sizeof(m));
      m.buffer_addr = a->ent4[4 * j];
      m.buffer_size = a->ent4[4 * j + 1];
      m.alloc_date = a->ent4[4 * j + 2];
      m.free_date = a->ent4[4 * j + 3];
      if (o_in_buffer(&m, addr, ts)) {
        *baddr = m.buffer_addr;
        return a->entry_ids[j];
      }
    }
    return -1;
  }
  int64_t k = o_lower_key(st, addr);
  if (k < 0) return -1;
  for (uint32_t e = st->entry_off[k]; e < st->entry_off[k + 1]; e++)
    if (o_in_buffer(&st->mems[e], addr, ts)) {
      *baddr = st->mems[e].buffer_addr;
      return e;
    }
  return -1;
}

/* ------------------------------------------------------------------ */
/* page blocks                                                         */

static struct o_block *o_new_block(unsigned id) {
  struct o_block *b = malloc(sizeof(*b));
  b->block_id = id;
  o_init_counters(&b->counters[0]);
  o_init_counters(&b->counters[1]);
  b->next = NULL;
  return b;
}

/* __allocate_counters + __init_counters -- src/mem_analyzer.c:406-460.
 * The reference mallocs 1024 head blocks per object up front; the oracle
 * materialises a head lazily on first use, which has identical semantics
 * (every head is block 0 with freshly initialised counters). */
static struct o_block **o_allocate_counters(void) {
  return calloc(MAX_THREADS, sizeof(struct o_block *));
}
static struct o_block *o_head(struct o_block **blocks, unsigned th) {
  if (!blocks[th]) blocks[th] = o_new_block(0);
  return blocks[th];
}

/* __ma_search_block -- src/mem_analyzer.c:474-489 */
static struct o_block *o_search_block(struct o_block *block, unsigned page) {
  while (block) {
    if (block->block_id == page) return block;
    if (!block->next || block->next->block_id > page) return NULL;
    block = block->next;
  }
  return NULL;
}

/* __ma_get_block -- src/mem_analyzer.c:494-523: walk the sorted list,
 * inserting a zeroed block after the last smaller one. */
static struct o_block *o_get_block(struct o_block *block, unsigned page) {
  while (block) {
    if (block->block_id == page) return block;
    if (!block->next || block->next->block_id > page) {
      struct o_block *nb = o_new_block(page);
      nb->next = block->next;
      block->next = nb;
    }
    block = block->next;
  }
  return NULL;
}

/* ma_get_block -- src/mem_analyzer.c:525-534 (page_no is an int); baddr =
 * the object's buffer_addr when the sample was matched */
static struct o_block *o_ma_get_block(struct o_mem *m, unsigned th, uint64_t addr, uint64_t baddr) {
  uint64_t offset = addr - baddr;
  int page_no = (int)(offset / PAGE_SIZE);
  return o_get_block(o_head(m->blocks, th), (unsigned)page_no);
}

/* ------------------------------------------------------------------ */
/* call sites                                                          */

/* find_call_site -- src/mem_analyzer.c:1302-1331 */
static struct o_site *o_find_call_site(struct o_state *st, const struct o_mem *m) {
  for (struct o_site *s = st->call_sites; s; s = s->next) {
    if (s->buffer_size != m->initial_buffer_size) continue;
    if (s->callstack) {
      if (s->callstack_size == m->callstack_size) {
        int match = 1;
        for (int i = 3; i < s->callstack_size; i++)
          if (s->callstack[i] != m->callstack[i]) {
            match = 0;
            break;
          }
        if (match) return s;
      }
    } else if (s->caller_rip == m->caller_rip) {
      return s;
    }
  }
  return NULL;
}

/* caller string of an object; get_caller_function_from_rip
 * (src/mem_tools.c:91-131) returns "???" for a NULL rip.  Replays carry the
 * symbolised string; an unsymbolised non-NULL rip is rendered "[0x<rip>]". */
static void o_caller_string(const struct o_mem *m, char *out) {
  if (m->caller) {
    snprintf(out, 1024, "%s", m->caller);
  } else if (!m->caller_rip) {
    snprintf(out, 1024, "???");
  } else {
    snprintf(out, 1024, "[0x%" PRIx64 "]", m->caller_rip);
  }
}

/* new_call_site -- src/mem_analyzer.c:1333-1378 (pushed at the list head) */
static struct o_site *o_new_call_site(struct o_state *st, const struct o_mem *m) {
  struct o_site *s = calloc(1, sizeof(*s));
  s->id = st->next_call_site_id++;
  s->callstack = m->callstack;
  s->callstack_size = m->callstack_size;
  s->caller_rip = m->caller_rip;
  o_caller_string(m, s->caller);
  s->buffer_size = m->initial_buffer_size;
  s->nb_mallocs = 0;
  s->mem_type = m->mem_type;
  s->mem_info_buffer_size = m->buffer_size;
  s->blocks = o_allocate_counters();
  s->cumulated.block_id = 0;
  s->cumulated.next = NULL;
  memset(&s->cumulated.counters, 0, sizeof(s->cumulated.counters)); /* :1370-1372 */
  s->next = st->call_sites;
  st->call_sites = s;
  return s;
}

/* ACC_COUNTER / ACC_COUNTERS -- src/mem_analyzer.c:1396-1427.  Note the
 * reference's max update uses '>' and so never raises max (quirk Q8). */
static void o_acc_counters(struct o_counters *to, const struct o_counters *from) {
  to->total_count += from->total_count;
  to->total_weight += from->total_weight;
  to->na_miss_count += from->na_miss_count;
  for (int i = 0; i < 18; i++) {
    to->b[i].count += from->b[i].count;
    to->b[i].sum_weight += from->b[i].sum_weight;
    if (to->b[i].min_weight > from->b[i].min_weight) to->b[i].min_weight = from->b[i].min_weight;
    if (to->b[i].max_weight > from->b[i].max_weight) to->b[i].max_weight = from->b[i].max_weight;
  }
}

/* update_call_sites -- src/mem_analyzer.c:1380-1436 */
static void o_update_call_sites(struct o_state *st, struct o_mem *m) {
  struct o_site *s = o_find_call_site(st, m);
  if (!s) s = o_new_call_site(st, m);
  s->nb_mallocs++;
  for (unsigned i = 0; i < MAX_THREADS; i++) {
    struct o_block *block = m->blocks[i];
    while (block) {
      struct o_block *mem_block = o_get_block(o_head(s->blocks, i), block->block_id);
      struct o_block *site_block = o_get_block(&s->cumulated, 0);
      for (int j = 0; j < ACCESS_MAX; j++) {
        o_acc_counters(&mem_block->counters[j], &block->counters[j]);
        o_acc_counters(&site_block->counters[j], &block->counters[j]);
      }
      block = block->next;
    }
  }
}

/* ------------------------------------------------------------------ */
/* analysis                                                            */

/* __match_sample -- src/mem_sampling.c:594-673 */
static int64_t o_match_sample(struct o_state *st, uint64_t addr, uint64_t ts,
                              uint64_t weight, uint64_t data_src, int access,
                              unsigned th, uint64_t ordinal) {
  uint64_t baddr = 0;
  int64_t e = o_find(st, addr, ts, &baddr);
  if (e < 0) return -1;
  struct o_mem *m = &st->mems[e];
  if (!m->blocks) m->blocks = o_allocate_counters();
  if (ordinal < m->first_ordinal) m->first_ordinal = ordinal;
  struct o_block *block = o_ma_get_block(m, th, addr, baddr);
  o_update_counters(block->counters, weight, data_src, access);
  if (!m->call_site) {
    m->call_site = o_find_call_site(st, m);
    if (!m->call_site) m->call_site = o_new_call_site(st, m);
  }
  return e;
}

/* ------------------------------------------------------------------ */
/* dump modes -- src/mem_sampling.c:599-650, 740-808, 895-914          */

/* get_data_src_level() belongs to numap (unpinned HEAD, absent here): only
 * "L1_Hit", "L2_Hit" and "L3_Hit" are pinned, by the reference's README
 * (README.md:142-147).  Restated: the first level bit present names the
 * level, then "_Hit" / "_Miss"; the engine's report writer uses the same
 * restatement (parity unpinned beyond those three strings). */
static void o_data_src_level(uint64_t data_src, char *out) {
  const uint32_t lvl = (uint32_t)(data_src >> 5) & 0x3fff; /* union perf_mem_data_src.mem_lvl */
  static const struct { uint32_t bit; const char *name; } names[] = {
      {LVL_NA, "NA"}, {LVL_L1, "L1"}, {LVL_LFB, "LFB"}, {LVL_L2, "L2"}, {LVL_L3, "L3"},
      {LVL_LOC_RAM, "Local_RAM"}, {LVL_REM_RAM1, "Remote_RAM_1_hop"}, {LVL_REM_RAM2, "Remote_RAM_2_hops"},
      {LVL_REM_CCE1, "Remote_Cache_1_hop"}, {LVL_REM_CCE2, "Remote_Cache_2_hops"}, {LVL_IO, "IO_Memory"},
      {LVL_UNC, "Uncached_Memory"}};
  const char *n = "Unknown";
  for (unsigned i = 0; i < sizeof(names) / sizeof(names[0]); i++)
    if (lvl & names[i].bit) {
      n = names[i].name;
      break;
    }
  sprintf(out, "%s%s", n, (lvl & LVL_HIT) ? "_Hit" : ((lvl & LVL_MISS) ? "_Miss" : ""));
}

static FILE *o_open_out(struct o_state *st, const char *base) {
  char fn[4096];
  snprintf(fn, sizeof(fn), "%s/%s", st->outdir ? st->outdir : ".", base);
  FILE *f = fopen(fn, "w");
  if (!f) st->dump_err = NMO_ERR_IO;
  return f;
}

/* the unmatched branch of __match_sample (:602-650).  The header copies the
 * traced process's /proc/<pid>/maps with `while(!feof) { fgets; fprintf }`,
 * which prints the last line twice when the file ends with a newline. */
static void o_dump_unmatched(struct o_state *st, const struct o_buffer *buf, uint64_t ts, uint64_t addr,
                             uint64_t weight, uint64_t dsrc) {
  FILE *f = st->dump_unmatched_file;
  if (!f) return;
  if (!st->maps_read) {
    fprintf(f, "# %s content:\n", st->set->maps_path ? st->set->maps_path : "/proc/self/maps");
    const char *t = st->set->maps_text ? st->set->maps_text : "";
    char line[1024];
    line[0] = 0;
    size_t pos = 0, len = strlen(t);
    int eof = len == 0;
    while (!eof) { /* fgets(line, 1024, maps) over the captured text */
      if (pos >= len) {
        eof = 1; /* fgets returns NULL, line unchanged */
      } else {
        size_t n = 0;
        while (pos < len && n < sizeof(line) - 1) {
          line[n++] = t[pos++];
          if (line[n - 1] == '\n') break;
        }
        line[n] = 0;
        if (pos >= len && line[n - 1] != '\n') eof = 1; /* EOF hit while reading */
      }
      fprintf(f, "# %s", line);
    }
    fprintf(f, "#\n#\n#\n");
    st->maps_read = 1;
    fprintf(f, "#thread_rank timestamp address mem_level access_weight access_type\n");
  }
  char lvl[64];
  o_data_src_level(dsrc, lvl);
  fprintf(f, "%u %" PRIu64 " 0x%" PRIxPTR " %s %" PRIu64 " %c\n", buf->thread_rank, ts, (uintptr_t)addr, lvl,
          weight, buf->access_type == ACCESS_READ ? 'r' : 'w');
}

/* _dump_mem_info (:740-773) and _dump_call_site (:775-808) */
static void o_dump_matched(struct o_state *st, const struct o_buffer *buf, struct o_mem *m, uint64_t ts,
                           uint64_t offset, uint64_t weight, uint64_t dsrc) {
  char lvl[64];
  o_data_src_level(dsrc, lvl);
  const char acc = buf->access_type == ACCESS_READ ? 'r' : 'w';
  if (st->set->dump_all && m->mem_type != MEM_TYPE_STACK) {
    if (!st->dump_all_file) {
      st->dump_all_file = o_open_out(st, "all_memory_accesses.dat");
      if (!st->dump_all_file) return;
      fprintf(st->dump_all_file, "#thread_rank timestamp object_id offset mem_level access_weight access_type\n");
    }
    fprintf(st->dump_all_file, "%u %" PRIu64 " %u %" PRIu64 " %s %" PRIu64 " %c\n", buf->thread_rank, ts, m->id,
            offset, lvl, weight, acc);
  }
  if (st->set->dump_single_items && m->call_site && m->mem_type != MEM_TYPE_STACK) {
    struct o_site *site = m->call_site;
    if (!site->dump_file) {
      char base[64];
      snprintf(base, sizeof(base), "callsite_dump_%d.dat", (int)site->id);
      site->dump_file = o_open_out(st, base);
      if (!site->dump_file) return;
      fprintf(site->dump_file, "#thread_rank timestamp offset mem_level access_weight access_type\n");
    }
    fprintf(site->dump_file, "%u %" PRIu64 " %" PRIuPTR " %s %" PRIu64 " %c\n", buf->thread_rank, ts,
            (uintptr_t)offset, lvl, weight, acc);
  }
}

/* __analyze_buffer -- src/mem_sampling.c:815-927 on a linearised copy
 * (data_tail = 0, data_head = buffer_size; the wrap branch never fires). */
static int o_analyze_buffer(struct o_state *st, uint32_t bidx, int match_samples,
                            uint32_t *nb_samples, uint32_t *found) {
  struct o_buffer *buf = &st->buffers[bidx];
  unsigned cur = 0, stop = (unsigned)buf->size;
  while (cur < stop) {
    const uint8_t *ev = buf->data + cur;
    if ((uint64_t)cur + 8 > buf->size) return NMO_ERR_TRUNCATED;
    uint32_t type = rd_u32(ev);
    uint16_t size;
    memcpy(&size, ev + 6, 2);
    if (size == 0) return NMO_ERR_ZERO_SIZE; /* :857-860 abort() */
    if (type == PERF_RECORD_SAMPLE) {
      /* a record that runs past the end of the copy would be read through
       * frontier_buffer past the allocation (:865-879): undefined in the
       * reference, rejected here */
      if ((uint64_t)cur + 40 > buf->size || (uint64_t)cur + size > buf->size)
        return NMO_ERR_TRUNCATED;
      uint64_t ts = rd_u64(ev + 8), addr = rd_u64(ev + 16);
      uint64_t weight = rd_u64(ev + 24), dsrc = rd_u64(ev + 32);
      (*nb_samples)++;
      o_update_counters(st->global_counters, weight, dsrc, (int)buf->access_type);
      int64_t e = -1;
      if (match_samples) {
        uint64_t ordinal = ((uint64_t)bidx << 32) | cur;
        e = o_match_sample(st, addr, ts, weight, dsrc, (int)buf->access_type, buf->thread_rank, ordinal);
        if (e >= 0)
          (*found)++;
        else if (st->set && st->set->dump_unmatched)
          o_dump_unmatched(st, buf, ts, addr, weight, dsrc);
      }
      if (st->set && (st->set->dump || st->set->dump_all) && e >= 0) {
        struct o_mem *m = &st->mems[e];
        o_dump_matched(st, buf, m, ts, addr - m->buffer_addr, weight, dsrc);
      }
    }
    cur += size; /* :918 */
  }
  return 0;
}

/* ------------------------------------------------------------------ */
/* reports                                                             */

static const char *o_level_names_hit[9] = {
    "L1 Hit", "L2 Hit", "L3 Hit", "LFB Hit", "Local RAM Hit", "Remote RAM Hit",
    "Remote cache Hit", "IO memory Hit", "Uncached memory Hit"};
static const char *o_level_names_miss[9] = {
    NULL, NULL, NULL, "LFB Miss", "Local RAM Miss", "Remote RAM Miss",
    "Remote cache Miss", "IO memory Miss", "Uncached memory Miss"};

/* __print_counters -- src/mem_analyzer.c:1438-1487 */
static void o_print_counters(FILE *f, const struct o_counters *counters) {
  for (int i = 0; i < ACCESS_MAX; i++) {
    const struct o_counters *c = &counters[i];
    if (i == ACCESS_READ) {
      fprintf(f, "\n");
      fprintf(f, "# --------------------------------------\n");
      fprintf(f, "# Summary of all the read memory access:\n");
    } else {
      fprintf(f, "# --------------------------------------\n");
      fprintf(f, "# Summary of all the write memory access:\n");
    }
    fprintf(f, "# Total count          : \t %" PRIu64 "\n", c->total_count);
    fprintf(f, "# Total weigh          : \t %" PRIu64 "\n", c->total_weight);
    if (c->na_miss_count)
      fprintf(f, "# N/A                  : \t %" PRIu64 " (%f %%)\n", c->na_miss_count,
              (100. * c->na_miss_count / c->total_count));
#define PRINT_ONE(idx, str)                                                              \
  if (c->b[idx].count)                                                                   \
    fprintf(f,                                                                           \
            "# %s\t: %ld (%f %%) \tmin: %" PRIu64 " cycles\tmax: %" PRIu64              \
            " cycles\t avg: %" PRIu64 " cycles\ttotal weight: %" PRIu64 " (%f %%)\n",   \
            str, (long)c->b[idx].count, (100. * c->b[idx].count / c->total_count),       \
            c->b[idx].min_weight, c->b[idx].max_weight,                                   \
            (c->b[idx].count ? c->b[idx].sum_weight / c->b[idx].count : 0),              \
            c->b[idx].sum_weight,                                                        \
            (c->total_weight ? 100. * c->b[idx].sum_weight / c->total_weight : 0))
    for (int k = 0; k < 9; k++) PRINT_ONE(k, o_level_names_hit[k]);
    fprintf(f, "\n");
    for (int k = 3; k < 9; k++) PRINT_ONE(9 + k, o_level_names_miss[k]);
#undef PRINT_ONE
  }
}

/* __print_call_site_stats -- src/mem_analyzer.c:1489-1503 */
static void o_print_call_site_stats(struct o_state *st, struct o_site *site) {
  char base[64];
  snprintf(base, sizeof(base), "callsite_summary_%d.dat", (int)site->id);
  FILE *f = o_open_out(st, base);
  if (!f) return;
  o_print_counters(f, site->cumulated.counters);
  fclose(f);
}

/* __remove_site -- src/mem_analyzer.c:1506-1528.  On leaving, the site the
 * walk stopped at -- the removed site itself when it was the head, else its
 * predecessor (quirk Q10) -- has its summary written and its dump file closed
 * when it has one (dump modes). */
static void o_remove_site(struct o_state *st, struct o_site *site) {
  struct o_site *cur = st->call_sites;
  if (cur == site) {
    st->call_sites = cur->next;
    goto out;
  }
  while (cur->next) {
    if (cur->next == site) {
      cur->next = site->next;
      goto out;
    }
    cur = cur->next;
  }
out:
  if (cur && cur->dump_file) {
    o_print_call_site_stats(st, cur);
    fclose(cur->dump_file);
    cur->dump_file = NULL;
  }
}

/* __sort_sites -- src/mem_analyzer.c:1531-1557: repeated selection of the
 * first site whose read total_weight is below an *int*-truncated running
 * minimum (quirk Q9), each pushed at the head of the result. */
static void o_sort_sites(struct o_state *st, FILE *out) {
  struct o_site *head = NULL;
  fprintf(out, "Sorting call sites\n");
  while (st->call_sites) {
    struct o_site *cur = st->call_sites, *min_site = cur;
    int min_weight = (int)cur->cumulated.counters[ACCESS_READ].total_weight;
    while (cur) {
      if (cur->cumulated.counters[ACCESS_READ].total_weight < (uint64_t)(int64_t)min_weight) {
        min_weight = (int)cur->cumulated.counters[ACCESS_READ].total_weight;
        min_site = cur;
      }
      cur = cur->next;
    }
    o_remove_site(st, min_site);
    min_site->next = head;
    head = min_site;
  }
  st->call_sites = head;
}

/* __plot_counters -- src/mem_analyzer.c:1559-1583 */
static int o_plot_counters(struct o_site *s, int nb_threads, const char *filename) {
  FILE *file = fopen(filename, "w");
  if (!file) return NMO_ERR_IO;
  int nb_pages = (int)((s->mem_info_buffer_size / PAGE_SIZE) + 1);
  for (int i = 0; i < nb_pages; i++) {
    for (int th = 0; th < nb_threads; th++) {
      /* an unmaterialised head is a zero block 0: searching it finds nothing
       * non-zero either way */
      struct o_block *block = s->blocks[th] ? o_search_block(s->blocks[th], (unsigned)i) : NULL;
      int total_access = 0;
      if (block) {
        total_access += block->counters[ACCESS_READ].total_count;
        total_access += block->counters[ACCESS_WRITE].total_count;
      }
      fprintf(file, "\t%d", total_access);
    }
    fprintf(file, "\n");
  }
  fclose(file);
  return 0;
}

/* print_call_site_summary -- src/mem_analyzer.c:1597-1640 */
static int o_print_call_site_summary(struct o_state *st, FILE *out, const char *outdir,
                                     int dump_single_items) {
  fprintf(out, "Summary of the call sites:\n");
  fprintf(out, "--------------------------\n");
  o_sort_sites(st, out);
  char path[4096];
  snprintf(path, sizeof(path), "%s/call_sites.log", outdir);
  FILE *cf = fopen(path, "w");
  if (!cf) return NMO_ERR_IO;
  for (struct o_site *s = st->call_sites; s; s = s->next) {
    const struct o_counters *cc = s->cumulated.counters;
    if (cc[ACCESS_READ].total_count || cc[ACCESS_WRITE].total_count) {
      double avg = 0;
      if (cc[ACCESS_READ].total_count)
        avg = (double)cc[ACCESS_READ].total_weight / cc[ACCESS_READ].total_count;
      for (int k = 0; k < 2; k++)
        fprintf(k ? out : cf,
                "%d\t%s (size=%zu) - %d buffers. %zu read access (total weight: %" PRIu64
                ", avg weight: %f). %" PRIu64 " wr_access\n",
                (int)s->id, s->caller, (size_t)s->buffer_size, (int)s->nb_mallocs,
                (size_t)cc[ACCESS_READ].total_count, cc[ACCESS_READ].total_weight, avg,
                cc[ACCESS_WRITE].total_count);
      if (dump_single_items && s->mem_type != MEM_TYPE_STACK) {
        char fn[4096];
        snprintf(fn, sizeof(fn), "%s/callsite_counters_%d.dat", outdir, (int)s->id);
        int rc = o_plot_counters(s, (int)st->nb_threads, fn);
        if (rc) {
          fclose(cf);
          return rc;
        }
      }
    }
  }
  fclose(cf);
  return 0;
}

/* ------------------------------------------------------------------ */
/* all_memory_objects.dat -- src/mem_analyzer.c:1642-1748             */

/* dladdr(): the module holding rip (linear scan: test sizes) */
static const struct nmo_module *o_dladdr(const struct nmo_settings *set, uint64_t rip) {
  for (uint32_t i = 0; set->modules && i < set->nb_modules; i++)
    if (set->modules[i].lo <= rip && rip < set->modules[i].hi) return &set->modules[i];
  return NULL;
}

/* _print_object_summary -- mem_analyzer.c:1642-1704 */
static void o_print_object_row(struct o_state *st, FILE *f, const struct o_mem *m) {
  char caller[1024];
  o_caller_string(m, caller);
  size_t cap = 64 + (m->callstack_size > 0 ? (size_t)m->callstack_size : 0) * 32;
  char *rips = malloc(cap), *offs;
  size_t ocap = 64;
  for (int i = 3; m->callstack && i < m->callstack_size; i++) {
    const struct nmo_module *mod = o_dladdr(st->set, m->callstack[i]);
    ocap += 32 + (mod && mod->fname ? strlen(mod->fname) : 8);
  }
  offs = malloc(ocap);
  rips[0] = offs[0] = '\0';
  if (m->callstack) {
    size_t rl = 0, ol = 0;
    for (int i = 3; i < m->callstack_size; i++) {
      uint64_t rip = m->callstack[i];
      const struct nmo_module *mod = o_dladdr(st->set, rip);
      uint64_t fbase = mod ? mod->fbase : 0;
      const char *prefix = i == 3 ? "" : ",";
      rl += (size_t)sprintf(rips + rl, "%s0x%" PRIx64, prefix, rip);
      ol += (size_t)sprintf(offs + ol, "%s%s:%td", prefix, mod && mod->fname ? mod->fname : "(null)",
                            (ptrdiff_t)(rip - fbase));
    }
  } else {
    strcpy(rips, "NULL");
    strcpy(offs, "NULL");
  }
  fprintf(f, "%d\t0x%" PRIx64 "\t%ld\t%" PRIu64 "\t%" PRIu64 "\t%s\t%s\t0x%" PRIx64 "\t%s\n", (int)m->id,
          m->buffer_addr, (long)m->buffer_size, m->alloc_date, m->free_date, rips, offs, m->caller_rip, caller);
  free(rips);
  free(offs);
}

/* print_object_summary -- mem_analyzer.c:1728-1748.  With USE_HASHTABLE
 * (:23) print_object_summary_from_list walks mem_list whatever list it is
 * given (:1706-1716), so the past_mem_list call prints mem_list again (Q20). */
static int o_print_object_summary(struct o_state *st) {
  FILE *f = o_open_out(st, "all_memory_objects.dat");
  if (!f) return NMO_ERR_IO;
  fprintf(f, "#object_id\taddress\tsize\tallocation_date\tdeallocation_date\tcallstack_rip\tcallstack_offsets"
             "\tcallsite_rip\tcallsite\n");
  for (int pass = 0; pass < 2; pass++)
    for (uint32_t e = 0; e < st->nb_entries; e++) o_print_object_row(st, f, &st->mems[e]);
  fclose(f);
  return 0;
}

/* ------------------------------------------------------------------ */
/* raw-results dump (canonical format shared with the engine tests)    */

static int o_write_raw(struct o_state *st, const char *path) {
  FILE *f = fopen(path, "wb");
  if (!f) return NMO_ERR_IO;
  const char magic[8] = {'N', 'M', 'G', 'R', 'E', 'S', '0', '1'};
  fwrite(magic, 1, 8, f);
  uint32_t hdr[4] = {st->nb_entries, st->nb_buffers, st->nb_threads, 0};
  fwrite(hdr, 4, 4, f);
  for (int a = 0; a < 2; a++) {
    const struct o_counters *c = &st->global_counters[a];
    fwrite(&c->total_count, 8, 1, f);
    fwrite(&c->total_weight, 8, 1, f);
    fwrite(&c->na_miss_count, 8, 1, f);
    for (int k = 0; k < 18; k++) fwrite(&c->b[k], 8, 4, f);
  }
  fwrite(&st->nb_samples_total, 8, 1, f);
  fwrite(&st->nb_found_samples_total, 8, 1, f);
  fwrite(st->buf_samples, 4, st->nb_buffers, f);
  fwrite(st->buf_found, 4, st->nb_buffers, f);
  /* per entry: first ordinal, then per access: count, weight, na, 18 x (count, sum) */
  for (uint32_t e = 0; e < st->nb_entries; e++) {
    struct o_mem *m = &st->mems[e];
    uint64_t rec[1 + 2 * 39];
    memset(rec, 0, sizeof(rec));
    rec[0] = m->first_ordinal;
    if (m->blocks) {
      for (unsigned th = 0; th < MAX_THREADS; th++)
        for (struct o_block *b = m->blocks[th]; b; b = b->next)
          for (int a = 0; a < 2; a++) {
            uint64_t *r = rec + 1 + 39 * a;
            const struct o_counters *c = &b->counters[a];
            r[0] += c->total_count;
            r[1] += c->total_weight;
            r[2] += c->na_miss_count;
            for (int k = 0; k < 18; k++) {
              r[3 + 2 * k] += c->b[k].count;
              r[4 + 2 * k] += c->b[k].sum_weight;
            }
          }
    }
    fwrite(rec, 8, 1 + 2 * 39, f);
  }
  /* page histogram: (entry, thread, page, read+write count) for every
   * block with a non-zero count, in (entry, thread, page) order */
  uint64_t n = 0;
  long pos = ftell(f);
  fwrite(&n, 8, 1, f);
  for (uint32_t e = 0; e < st->nb_entries; e++) {
    struct o_mem *m = &st->mems[e];
    if (!m->blocks) continue;
    for (unsigned th = 0; th < MAX_THREADS; th++)
      for (struct o_block *b = m->blocks[th]; b; b = b->next) {
        uint32_t cnt = (uint32_t)(b->counters[0].total_count + b->counters[1].total_count);
        if (!cnt) continue;
        uint32_t row[4] = {e, th, b->block_id, cnt};
        fwrite(row, 4, 4, f);
        n++;
      }
  }
  fseek(f, pos, SEEK_SET);
  fwrite(&n, 8, 1, f);
  fclose(f);
  return 0;
}

/* ------------------------------------------------------------------ */
/* driver: mem_sampling_finalize + ma_finalize (report part)           */

static void o_free(struct o_state *st) {
  if (st->mems) {
    for (uint32_t e = 0; e < st->nb_entries; e++) {
      struct o_block **bl = st->mems[e].blocks;
      if (!bl) continue;
      for (unsigned th = 0; th < MAX_THREADS; th++) {
        struct o_block *b = bl[th];
        while (b) {
          struct o_block *n = b->next;
          free(b);
          b = n;
        }
      }
      free(bl);
    }
  }
  struct o_site *s = st->call_sites;
  while (s) {
    struct o_site *n = s->next;
    for (unsigned th = 0; th < MAX_THREADS; th++) {
      struct o_block *b = s->blocks[th];
      while (b) {
        struct o_block *nn = b->next;
        free(b);
        b = nn;
      }
    }
    struct o_block *b = s->cumulated.next;
    while (b) {
      struct o_block *nn = b->next;
      free(b);
      b = nn;
    }
    free(s->blocks);
    free(s);
    s = n;
  }
  for (uint32_t b = 0; b < st->nb_buffers; b++) free(st->buffers[b].data);
  free(st->buffers);
  free(st->mems);
  free(st->buf_samples);
  free(st->buf_found);
  free(st->file);
}

static double o_now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

int nmo_run(const char *replay_path, const char *outdir, const char *stdout_path,
            const char *raw_path, const struct nmo_settings *settings,
            struct nmo_timing *timing) {
  struct o_state st;
  memset(&st, 0, sizeof(st));
  st.next_call_site_id = 1; /* mem_analyzer.c:1339 */
  int rc = o_load(&st, replay_path);
  if (rc) {
    o_free(&st);
    return rc;
  }
  int match = settings ? settings->match_samples : 1;
  int dump_single = settings ? settings->dump_single_items : 1;
  FILE *out = stdout;
  if (stdout_path) {
    out = fopen(stdout_path, "w");
    if (!out) {
      o_free(&st);
      return NMO_ERR_IO;
    }
  }
  if (outdir) mkdir(outdir, 0700);
  struct nmo_settings defaults = {1, 1, 0, 0, 0, 0, NULL, NULL, NULL, 0, 0};
  st.set = settings ? settings : &defaults;
  st.outdir = outdir;
  if (st.set->dump_unmatched) { /* opened at init, mem_intercept.c:528-535 */
    st.dump_unmatched_file = o_open_out(&st, "unmatched_samples.log");
    if (!st.dump_unmatched_file) {
      if (out != stdout) fclose(out);
      o_free(&st);
      return NMO_ERR_IO;
    }
  }
  o_init_counters(&st.global_counters[0]); /* mem_sampling.c:212-213 */
  o_init_counters(&st.global_counters[1]);
  st.buf_samples = calloc(st.nb_buffers ? st.nb_buffers : 1, 4);
  st.buf_found = calloc(st.nb_buffers ? st.nb_buffers : 1, 4);

  /* mem_sampling_finalize -- src/mem_sampling.c:311-346; online, the
   * buffers were analysed at the alarms (__process_samples, :929-966) and
   * finalize prints nothing (:313) */
  const int online = st.set->nb_alarms > 0;
  if (online && st.set->alarms[st.set->nb_alarms - 1].buf_end != st.nb_buffers) {
    if (out != stdout) fclose(out);
    o_free(&st);
    return NMO_ERR_FORMAT;
  }
  double t0 = o_now();
  if (!online) fprintf(out, "Analyzing %d sample buffers\n", (int)st.nb_buffers);
  int nb_blocks = 0;
  size_t total_buffer_size = 0;
  uint32_t alarm = 0;
  for (uint32_t b = 0; b < st.nb_buffers; b++) {
    uint32_t nb = 0, found = 0;
    if (online) {
      while (b >= st.set->alarms[alarm].buf_end) alarm++;
      st.snap = &st.set->alarms[alarm];
    } else if (nb_blocks % 10 == 0) {
      fprintf(out, "\rAnalyzing sample buffer %d/%d. Total samples so far: %zu", nb_blocks,
              (int)st.nb_buffers, (size_t)st.nb_samples_total);
    }
    rc = o_analyze_buffer(&st, b, match, &nb, &found);
    if (rc) break;
    st.buf_samples[b] = nb;
    st.buf_found[b] = found;
    st.nb_samples_total += (uint64_t)(int)nb;
    st.nb_found_samples_total += (uint64_t)(int)found;
    total_buffer_size += st.buffers[b].size;
    nb_blocks++;
  }
  double t1 = o_now();
  if (rc) {
    if (out != stdout) fclose(out);
    o_free(&st);
    return rc;
  }
  st.snap = NULL;
  if (!online) {
    fprintf(out, "\n");
    fprintf(out, "%zu bytes processed\n", total_buffer_size);
  }

  /* ma_finalize -- src/mem_analyzer.c:1809-1881 */
  fprintf(out, "---------------------------------\n");
  fprintf(out, "         MEM ANALYZER\n");
  fprintf(out, "---------------------------------\n");
  /* FOREACH_HASH: keys ascending, each node's entries newest-first */
  for (uint32_t e = 0; e < st.nb_entries; e++) {
    /* online, every object has counters since _init_mem_info (:569-572) */
    if (online && match && !st.mems[e].blocks) st.mems[e].blocks = o_allocate_counters();
    if (st.mems[e].blocks) o_update_call_sites(&st, &st.mems[e]);
  }
  o_print_counters(out, st.global_counters);
  if (outdir) rc = o_print_call_site_summary(&st, out, outdir, dump_single);
  if (!rc && outdir && st.set->dump_all) rc = o_print_object_summary(&st);
  /* mem_sampling_statistics -- src/mem_sampling.c:357-361 */
  float percent = 100.0 * (st.nb_samples_total - st.nb_found_samples_total) / st.nb_samples_total;
  fprintf(out,
          "%" PRIu64 " samples (including %" PRIu64
          " samples that do not match a known memory buffer / %f%%)\n",
          st.nb_samples_total, st.nb_samples_total - st.nb_found_samples_total, percent);
  double t2 = o_now();
  if (out != stdout) fclose(out);
  /* files still open at exit are flushed by the C runtime in the reference */
  for (struct o_site *s = st.call_sites; s; s = s->next)
    if (s->dump_file) fclose(s->dump_file), s->dump_file = NULL;
  if (st.dump_all_file) fclose(st.dump_all_file);
  if (st.dump_unmatched_file) fclose(st.dump_unmatched_file); /* mem_intercept.c:582-584 */
  if (!rc && st.dump_err) rc = st.dump_err;
  if (!rc && raw_path) rc = o_write_raw(&st, raw_path);
  if (timing) {
    timing->analysis_s = t1 - t0;
    timing->total_s = t2 - t0;
    timing->nb_samples = st.nb_samples_total;
  }
  o_free(&st);
  return rc;
}

/* Direct lookup on a caller-provided flattened table (tests pin this against
 * the reference's own AVL tree in oracle/_ref).  ent4 = [E][4] of
 * (buffer_addr, buffer_size, alloc_date, free_date). */
int64_t nmo_lookup(const uint64_t *keys, const uint32_t *entry_off, uint32_t nb_keys,
                   const uint64_t *ent4, uint64_t addr, uint64_t ts) {
  struct o_state st;
  memset(&st, 0, sizeof(st));
  st.keys = (uint64_t *)keys;
  st.entry_off = (uint32_t *)entry_off;
  st.nb_keys = nb_keys;
  int64_t k = o_lower_key(&st, addr);
  if (k < 0) return -1;
  for (uint32_t e = entry_off[k]; e < entry_off[k + 1]; e++) {
    struct o_mem m;
    memset(&m, 0, sizeof(m));
    m.buffer_addr = ent4[4 * e];
    m.buffer_size = ent4[4 * e + 1];
    m.alloc_date = ent4[4 * e + 2];
    m.free_date = ent4[4 * e + 3];
    if (o_in_buffer(&m, addr, ts)) return e;
  }
  return -1;
}

const char *nmo_strerror(int rc) {
  switch (rc) {
    case 0: return "ok";
    case NMO_ERR_IO: return "i/o error";
    case NMO_ERR_FORMAT: return "invalid replay file";
    case NMO_ERR_ZERO_SIZE: return "record with size 0 (reference aborts, mem_sampling.c:857)";
    case NMO_ERR_TRUNCATED: return "truncated record at buffer end";
    default: return "unknown error";
  }
}

#ifdef NMO_MAIN
int main(int argc, char **argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s replay.bin outdir [raw.bin] [--no-match]\n", argv[0]);
    return 2;
  }
  struct nmo_settings s = {1, 1, 0, 0, 0, 0, NULL, NULL};
  const char *raw = NULL;
  for (int i = 3; i < argc; i++) {
    if (!strcmp(argv[i], "--no-match")) s.match_samples = 0;
    else raw = argv[i];
  }
  struct nmo_timing t;
  int rc = nmo_run(argv[1], argv[2], NULL, raw, &s, &t);
  if (rc) {
    fprintf(stderr, "nmg_oracle: %s\n", nmo_strerror(rc));
    return 1;
  }
  fprintf(stderr, "oracle: %" PRIu64 " samples analysed in %.3f s (%.3f Msamples/s)\n",
          t.nb_samples, t.analysis_s, t.nb_samples / t.analysis_s / 1e6);
  return 0;
}
#endif
