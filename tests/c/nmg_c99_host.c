/*
 * nmg_c99_host.c -- a C99 consumer of include/numamma_gpu.h (test program).
 *
 * Runs the sequence INTEGRATION.md section 1 patches into NumaMMa's
 * mem_sampling_finalize / ma_finalize (src/mem_sampling.c:311-346,
 * src/mem_analyzer.c:1802-1884): nmg_create -> nmg_set_objects (the
 * flattened object table, FOREACH_HASH order, entries newest-first) ->
 * nmg_submit_ring for every `samples` element in analysis order (ring
 * segments, wrapped ones included, linearised by the engine like
 * __copy_buffer, :675-738) -> nmg_analyze -> nmg_synchronize -> nmg_report ->
 * nmg_destroy.  Its input is a replay file (replay format), read
 * here with plain C stdio so that no part of the product's own loader is
 * involved.
 *
 *   nmg_c99_host replay.bin output_dir stdout_path
 *
 * Exit status 0 on success; otherwise the failing call and nmg_strerror().
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "numamma_gpu.h"

#define ENTRY_BYTES 72

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

static int fail(const char *what, int rc, nmg_engine *h) {
  char detail[512];
  detail[0] = 0;
  nmg_get_last_error_detail(h, detail, sizeof detail);
  fprintf(stderr, "%s: %s (%s)\n", what, nmg_strerror(rc), detail);
  return 1;
}

int main(int argc, char **argv) {
  size_t len = 0, off;
  uint8_t *file;
  uint32_t nthreads, nkeys, nent, nbufs, e, b;
  uint64_t cs_len, str_len;
  uint64_t *keys, *pool;
  uint32_t *entry_off;
  const char *strs;
  struct nmg_object *obj;
  struct nmg_object_meta *meta;
  struct nmg_options opt;
  struct nmg_report_options ro;
  nmg_engine *h = NULL;
  int rc;

  if (argc != 4) {
    fprintf(stderr, "usage: %s replay.bin output_dir stdout_path\n", argv[0]);
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
  keys = (uint64_t *)malloc(8 * (size_t)nkeys + 8);
  entry_off = (uint32_t *)malloc(4 * ((size_t)nkeys + 1));
  obj = (struct nmg_object *)malloc(sizeof *obj * ((size_t)nent + 1));
  meta = (struct nmg_object_meta *)calloc((size_t)nent + 1, sizeof *meta);
  pool = (uint64_t *)malloc(8 * (size_t)cs_len + 8);
  if (!keys || !entry_off || !obj || !meta || !pool) return 2;
  memcpy(keys, file + off, 8 * (size_t)nkeys);
  off += 8 * (size_t)nkeys;
  memcpy(entry_off, file + off, 4 * ((size_t)nkeys + 1));
  off += pad8(4 * ((size_t)nkeys + 1));
  {
    const uint8_t *ent = file + off;
    const uint8_t *cs = ent + (size_t)ENTRY_BYTES * nent;
    memcpy(pool, cs, 8 * (size_t)cs_len);
    strs = (const char *)(cs + 8 * (size_t)cs_len);
    for (e = 0; e < nent; e++) {
      const uint8_t *q = ent + (size_t)ENTRY_BYTES * e;
      uint32_t caller_off = rd32(q + 64);
      obj[e].buffer_addr = rd64(q + 0);
      obj[e].buffer_size = rd64(q + 8);
      obj[e].alloc_date = rd64(q + 24);
      obj[e].free_date = rd64(q + 32);
      meta[e].initial_buffer_size = rd64(q + 16);
      meta[e].caller_rip = rd64(q + 40);
      meta[e].mem_type = rd32(q + 48);
      meta[e].id = rd32(q + 52);
      meta[e].callstack_size = (int32_t)rd32(q + 60);
      meta[e].callstack = rd32(q + 68) ? pool + rd32(q + 56) : NULL;
      meta[e].caller = caller_off != 0xFFFFFFFFu ? strs + caller_off : NULL;
    }
    off += (size_t)ENTRY_BYTES * nent + 8 * (size_t)cs_len + pad8((size_t)str_len);
  }

  memset(&opt, 0, sizeof opt);
  opt.device = 0;
  opt.flags = NMG_F_MATCH_SAMPLES | NMG_F_PAGE_HIST;
  opt.nb_threads = nthreads;
  rc = nmg_create(&h, &opt);
  if (rc) return fail("nmg_create", rc, NULL);
  rc = nmg_set_objects(h, keys, entry_off, nkeys, obj, nent);
  if (rc) return fail("nmg_set_objects", rc, h);
  for (b = 0; b < nbufs; b++) { /* `samples` list order (mem_sampling.c:324) */
    uint32_t rank = rd32(file + off), acc = rd32(file + off + 4);
    uint64_t tail = rd64(file + off + 8), head = rd64(file + off + 16), ring = rd64(file + off + 24);
    off += 32;
    rc = nmg_submit_ring(h, file + off, ring, tail, head, rank, acc);
    if (rc) return fail("nmg_submit_ring", rc, h);
    off += pad8((size_t)ring);
  }
  rc = nmg_analyze(h);
  if (!rc) rc = nmg_synchronize(h);
  if (rc) return fail("nmg_analyze", rc, h);
  memset(&ro, 0, sizeof ro);
  ro.output_dir = argv[2];
  ro.dump_single_items = 1;
  rc = nmg_report(h, meta, &ro, argv[3]);
  if (rc) return fail("nmg_report", rc, h);
  nmg_destroy(h);
  free(file);
  free(keys);
  free(entry_off);
  free(obj);
  free(meta);
  free(pool);
  return 0;
}
