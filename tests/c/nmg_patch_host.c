/*
 * nmg_patch_host.c -- runs INTEGRATION.md section 1's patch as written
 * (test program; the patch's two translation units are cut out of the
 * document by tests/c/extract_patch.py and linked with this file).
 *
 * This file plays the unchanged rest of NumaMMa: it fills the reference's
 * data structures from a replay file -- `mem_list` (keys ascending, each with
 * its memory_info entries newest first) and the `samples` list in analysis
 * order, every buffer a linear copy as __copy_buffer makes it
 * (src/mem_sampling.c:675-738: data_tail = 0, data_head = buffer_size) --
 * then calls the patched ma_finalize() (src/mem_analyzer.c:1802-1884), which
 * must print the reference's whole stdout once.
 *
 *   nmg_patch_host replay.bin output_dir        (report on stdout)
 */
#define _POSIX_C_SOURCE 200809L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ref_stubs.h"

#define ENTRY_BYTES 72

/* ---- the reference globals the patch reads (mem_intercept.c, mem_analyzer.c, mem_sampling.c) */
struct numamma_settings settings;
struct ht_node *mem_list;
struct sample_list *samples;
unsigned next_thread_rank;
int do_get_at_analysis;
struct mem_allocator *sample_mem;
int is_record_safe = 1;
static void *plain_malloc(size_t n) { return malloc(n); }
void *(*libmalloc)(size_t size) = plain_malloc;

char *get_log_dir(void) { return settings.output_dir; }
/* replays carry symbolised callers; an entry without one stays without one */
char *get_caller_function_from_rip(void *rip) {
  (void)rip;
  return NULL;
}
void mem_allocator_free(struct mem_allocator *mem, void *ptr) {
  (void)mem;
  free(ptr);
}
void ma_get_variables(void) {}
/* the replay's table is the post-finalize one: free dates stamped, [stack] registered */
void ma_register_stack(void) {}
void ma_thread_finalize(void) {}
void warn_non_freed_buffers(void) {}
void print_object_summary(void) {} /* settings.dump_all == 0 */

static uint32_t rd32(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
static uint64_t rd64(const uint8_t *p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}
static size_t pad8(size_t x) { return (x + 7) & ~(size_t)7; }

static uint8_t *slurp(const char *path, size_t *len) {
  FILE *f = fopen(path, "rb");
  uint8_t *buf;
  long sz;
  if (!f) return NULL;
  if (fseek(f, 0, SEEK_END) != 0 || (sz = ftell(f)) < 0 || fseek(f, 0, SEEK_SET) != 0) {
    fclose(f);
    return NULL;
  }
  buf = (uint8_t *)malloc((size_t)sz + 1);
  if (buf && fread(buf, 1, (size_t)sz, f) != (size_t)sz) {
    free(buf);
    buf = NULL;
  }
  fclose(f);
  *len = (size_t)sz;
  return buf;
}

int main(int argc, char **argv) {
  size_t len = 0, off;
  uint8_t *file;
  uint32_t nthreads, nkeys, nent, nbufs, k, b;
  uint64_t cs_len, str_len;
  const uint8_t *ent, *cs;
  const char *strs;
  uint32_t *entry_off;
  struct memory_info *info;
  struct ht_node *nodes;
  struct ht_entry *entries;
  struct sample_list **tail = &samples;

  if (argc != 3) {
    fprintf(stderr, "usage: %s replay.bin output_dir\n", argv[0]);
    return 2;
  }
  file = slurp(argv[1], &len);
  if (!file || len < 64 || memcmp(file, "NMGRPLY1", 8) != 0) {
    fprintf(stderr, "cannot read replay %s\n", argv[1]);
    return 2;
  }
  nthreads = rd32(file + 12);
  nkeys = rd32(file + 16);
  nent = rd32(file + 20);
  nbufs = rd32(file + 24);
  cs_len = rd64(file + 32);
  str_len = rd64(file + 40);
  off = 64;
  settings.sampling_rate = 10000;
  settings.match_samples = 1;
  settings.dump_single_items = 1;
  settings.output_dir = argv[2];
  next_thread_rank = nthreads;

  /* mem_list: one node per key, ascending; entries newest first */
  nodes = (struct ht_node *)calloc((size_t)nkeys + 1, sizeof *nodes);
  entries = (struct ht_entry *)calloc((size_t)nent + 1, sizeof *entries);
  info = (struct memory_info *)calloc((size_t)nent + 1, sizeof *info);
  entry_off = (uint32_t *)malloc(4 * ((size_t)nkeys + 1));
  if (!nodes || !entries || !info || !entry_off) return 2;
  memcpy(entry_off, file + off + 8 * (size_t)nkeys, 4 * ((size_t)nkeys + 1));
  ent = file + off + 8 * (size_t)nkeys + pad8(4 * ((size_t)nkeys + 1));
  cs = ent + (size_t)ENTRY_BYTES * nent;
  strs = (const char *)(cs + 8 * (size_t)cs_len);
  for (k = 0; k < nkeys; k++) {
    uint32_t e;
    nodes[k].key = rd64(file + off + 8 * (size_t)k);
    nodes[k].next_in_order = k + 1 < nkeys ? &nodes[k + 1] : NULL;
    nodes[k].entries = entry_off[k] < entry_off[k + 1] ? &entries[entry_off[k]] : NULL;
    for (e = entry_off[k]; e < entry_off[k + 1]; e++) {
      const uint8_t *q = ent + (size_t)ENTRY_BYTES * e;
      struct memory_info *m = &info[e];
      uint32_t caller_off = rd32(q + 64);
      m->buffer_addr = (void *)(uintptr_t)rd64(q + 0);
      m->buffer_size = rd64(q + 8);
      m->initial_buffer_size = rd64(q + 16);
      m->alloc_date = rd64(q + 24);
      m->free_date = rd64(q + 32);
      m->caller_rip = (void *)(uintptr_t)rd64(q + 40);
      m->mem_type = (enum mem_type)rd32(q + 48);
      m->id = rd32(q + 52);
      m->callstack_size = (int)rd32(q + 60);
      m->callstack_rip = rd32(q + 68) ? (void **)(cs + 8 * (size_t)rd32(q + 56)) : NULL;
      m->caller = caller_off != 0xFFFFFFFFu ? (char *)(strs + caller_off) : NULL;
      entries[e].value = m;
      entries[e].next = e + 1 < entry_off[k + 1] ? &entries[e + 1] : NULL;
    }
  }
  mem_list = nkeys ? &nodes[0] : NULL;
  off = (size_t)(strs - (const char *)file) + pad8((size_t)str_len);

  /* samples: analysis order, each ring segment linearised like __copy_buffer */
  for (b = 0; b < nbufs; b++) {
    uint32_t rank = rd32(file + off), acc = rd32(file + off + 4);
    uint64_t t = rd64(file + off + 8), h = rd64(file + off + 16), ring = rd64(file + off + 24);
    const uint8_t *r = file + off + 32;
    uint64_t n = h >= t ? h - t : ring - t + h;
    off += 32 + pad8((size_t)ring);
    if (n == 0) continue; /* data_head == data_tail: nothing is pushed (:680-682) */
    {
      struct sample_list *s = (struct sample_list *)calloc(1, sizeof *s);
      uint8_t *copy = (uint8_t *)malloc((size_t)n);
      if (!s || !copy) return 2;
      if (h >= t) {
        memcpy(copy, r + t, (size_t)n);
      } else {
        memcpy(copy, r + t, (size_t)(ring - t));
        memcpy(copy + (ring - t), r, (size_t)h);
      }
      s->buffer = (struct perf_event_header *)copy;
      s->data_tail = 0;
      s->data_head = n;
      s->buffer_size = (size_t)n;
      s->access_type = (enum access_type)acc;
      s->thread_rank = rank;
      *tail = s;
      tail = &s->next;
    }
  }

  ma_finalize();
  fflush(stdout);
  free(file);
  return 0;
}
