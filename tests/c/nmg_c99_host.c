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
 *   nmg_c99_host --bridge replay.bin output_dir stdout_path
 *
 * Under an LD_PRELOAD allocator interposer (tests/c/nmg_interpose.c, the
 * hazards of INTEGRATION.md section 2):
 *  - NMG_HOST_PROTECT=1 raises the interposer's thread-local recursion
 *    counter (`nmg_interpose_unsafe`, found through dlopen(NULL)) around every
 *    engine call, as NumaMMa's analysis code runs with is_recurse_unsafe
 *    raised (numamma.h.in:60-74); unset, the engine's allocations are
 *    recorded like the application's;
 *  - --bridge runs the out-of-process fallback instead: the replay is
 *    recorded through the host-only capture bridge (nmg_replay_open /
 *    add_ring / close: no HIP call in this process), then LD_PRELOAD is set
 *    to $NMG_BRIDGE_PRELOAD (the value without the interposer; unset when
 *    empty, like unset_ld_preload, mem_intercept.c:472-502) and the helper
 *    $NMG_BRIDGE_HELPER (numamma_amd/bin/nmg_replay) analyses and reports
 *    it.
 *
 * Exit status 0 on success; otherwise the failing call and nmg_strerror().
 */
#define _POSIX_C_SOURCE 200809L
#include <dlfcn.h>
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

static volatile int *unsafe_flag; /* the interposer's recursion counter (NMG_HOST_PROTECT=1) */
#define ENGINE(call)            \
  do {                          \
    if (unsafe_flag) ++*unsafe_flag; \
    rc = (call);                \
    if (unsafe_flag) --*unsafe_flag; \
  } while (0)

/* --bridge: the capture bridge, then the helper without the interposer */
static int bridge(const uint8_t *file, size_t off, uint32_t nthreads, const uint64_t *keys, const uint32_t *entry_off,
                  uint32_t nkeys, const struct nmg_object *obj, const struct nmg_object_meta *meta, uint32_t nent,
                  uint32_t nbufs, const char *outdir, const char *stdout_path) {
  char path[4096], cmd[16384];
  const char *helper = getenv("NMG_BRIDGE_HELPER"), *pre = getenv("NMG_BRIDGE_PRELOAD");
  nmg_replay_writer *w = NULL;
  uint32_t b;
  int rc;
  if (!helper) {
    fprintf(stderr, "--bridge needs NMG_BRIDGE_HELPER\n");
    return 2;
  }
  snprintf(path, sizeof path, "%s.replay.bin", outdir);
  rc = nmg_replay_open(&w, path, nthreads, keys, entry_off, nkeys, obj, meta, nent);
  if (rc) return fail("nmg_replay_open", rc, NULL);
  for (b = 0; b < nbufs; b++) {
    uint32_t rank = rd32(file + off), acc = rd32(file + off + 4);
    uint64_t tail = rd64(file + off + 8), head = rd64(file + off + 16), ring = rd64(file + off + 24);
    off += 32;
    rc = nmg_replay_add_ring(w, file + off, ring, tail, head, rank, acc);
    if (rc) return fail("nmg_replay_add_ring", rc, NULL);
    off += pad8((size_t)ring);
  }
  rc = nmg_replay_close(w);
  if (rc) return fail("nmg_replay_close", rc, NULL);
  if (pre && *pre)
    setenv("LD_PRELOAD", pre, 1);
  else
    unsetenv("LD_PRELOAD");
  snprintf(cmd, sizeof cmd, "'%s' '%s' '%s' > '%s'", helper, path, outdir, stdout_path);
  rc = system(cmd);
  remove(path);
  if (rc != 0) {
    fprintf(stderr, "helper failed (%d): %s\n", rc, cmd);
    return 1;
  }
  return 0;
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

  int use_bridge = argc == 5 && strcmp(argv[1], "--bridge") == 0;
  const char *prot = getenv("NMG_HOST_PROTECT");

  if (use_bridge) {
    argv++;
    argc--;
  }
  if (argc != 4) {
    fprintf(stderr, "usage: %s [--bridge] replay.bin output_dir stdout_path\n", argv[0]);
    return 2;
  }
  if (prot && strcmp(prot, "1") == 0) {
    void *self = dlopen(NULL, RTLD_LAZY);
    unsafe_flag = self ? (volatile int *)dlsym(self, "nmg_interpose_unsafe") : NULL;
    if (!unsafe_flag) {
      fprintf(stderr, "NMG_HOST_PROTECT=1 but no interposer is loaded\n");
      return 2;
    }
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

  if (use_bridge)
    return bridge(file, off, nthreads, keys, entry_off, nkeys, obj, meta, nent, nbufs, argv[2], argv[3]);

  memset(&opt, 0, sizeof opt);
  opt.device = 0;
  opt.flags = NMG_F_MATCH_SAMPLES | NMG_F_PAGE_HIST;
  opt.nb_threads = nthreads;
  ENGINE(nmg_create(&h, &opt));
  if (rc) return fail("nmg_create", rc, NULL);
  ENGINE(nmg_set_objects(h, keys, entry_off, nkeys, obj, nent));
  if (rc) return fail("nmg_set_objects", rc, h);
  for (b = 0; b < nbufs; b++) { /* `samples` list order (mem_sampling.c:324) */
    uint32_t rank = rd32(file + off), acc = rd32(file + off + 4);
    uint64_t tail = rd64(file + off + 8), head = rd64(file + off + 16), ring = rd64(file + off + 24);
    off += 32;
    ENGINE(nmg_submit_ring(h, file + off, ring, tail, head, rank, acc));
    if (rc) return fail("nmg_submit_ring", rc, h);
    off += pad8((size_t)ring);
  }
  ENGINE(nmg_analyze(h));
  if (!rc) ENGINE(nmg_synchronize(h));
  if (rc) return fail("nmg_analyze", rc, h);
  memset(&ro, 0, sizeof ro);
  ro.output_dir = argv[2];
  ro.dump_single_items = 1;
  ENGINE(nmg_report(h, meta, &ro, argv[3]));
  if (rc) return fail("nmg_report", rc, h);
  if (unsafe_flag) ++*unsafe_flag;
  nmg_destroy(h);
  if (unsafe_flag) --*unsafe_flag;
  free(file);
  free(keys);
  free(entry_off);
  free(obj);
  free(meta);
  free(pool);
  return 0;
}
