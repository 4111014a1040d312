/*
 * nmg_interpose.c -- a minimal LD_PRELOAD interposer for tests: it wraps the
 * allocator and pthread_create the way NumaMMa's libnumamma.so does, so that
 * the engine (HIP runtime threads, pinned allocations, copy pool, report
 * writer threads) and the capture bridge can be run under the same hazards
 * (INTEGRATION.md section 2).  Written for this repository; what it mimics:
 *
 *  - every malloc / calloc / realloc / operator new block carries a 64-byte
 *    header right before the user pointer, ending with a canary, and a tail
 *    canary right after the user bytes (the layout of mem_block_info,
 *    src/mem_intercept.h:44-61, 103-121); free() checks the head canary and
 *    hands a pointer it did not allocate straight to libc (mem_intercept.c:
 *    246-299), and aborts on a damaged tail canary;
 *  - the libc entry points are found with dlsym(RTLD_NEXT); allocations made
 *    while dlsym itself runs come from a static bump arena ("hand made"
 *    blocks, never freed, mem_intercept.c:46-71, 75-104);
 *  - a thread-local recursion counter (`nmg_interpose_unsafe`, numamma.h.in:
 *    60-74): while it is raised nothing is recorded.  A host that calls the
 *    engine with it raised finds the symbol with dlsym(RTLD_DEFAULT, ...);
 *  - a safe malloc is recorded like ma_record_malloc (mem_analyzer.c:1122-):
 *    a global mutex, a backtrace of the caller, an insert into a hash table
 *    (allocated outside the wrapped allocator); a free is looked up there and
 *    stamped;
 *  - pthread_create runs the new thread through a trampoline that does a
 *    per-thread init first (a 64 KiB per-thread buffer, like
 *    mem_sampling_thread_init's sample rings; mem_intercept.c:325-387).
 *
 *  - NMG_INTERPOSE_CANARY_CHECK=0 reproduces NumaMMa's default setting
 *    (settings.canary_check = 0, numamma.h.in:41): CANARY_OK is then always
 *    true (mem_intercept.h:68), so free() and realloc() take every pointer
 *    for one of theirs and read its header (mem_intercept.c:266-298,
 *    159-183) -- a block the interposer did not allocate (memalign & co,
 *    which it does not wrap either) would hand a garbage pointer to libc;
 *    this interposer stops at the first such block instead (exit code 86,
 *    after its counters; see canary_ok).  With
 *    the check on (the default here, NumaMMa's --canary-check), free() passes
 *    such a block to libc, and realloc() aborts on it like the reference.
 *
 * At exit it prints one line on stderr:
 *   nmg_interpose: {"recorded": R, "freed": F, "foreign_frees": X, "hand_made": H,
 *                   "threads": T, "unsafe_skips": S}
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

#define CANARY 0xdeadbeefdeadbeefull
#define KIND_MALLOC 0
#define KIND_NEW 1
#define KIND_HAND 2
#define KIND_INTERNAL 3

struct blk_head {      /* 64 bytes, 16-aligned: the user pointer stays 16-aligned */
  void *user;
  void *raw;           /* what libc returned */
  uint32_t kind, pad;
  size_t total;
  size_t size;
  uint64_t *tail;
  void *record;
  uint64_t canary;     /* last field: user - 8 */
} __attribute__((aligned(16)));

#define HEAD ((size_t)sizeof(struct blk_head))
#define TAIL ((size_t)sizeof(uint64_t))

__thread volatile int nmg_interpose_unsafe;

static void *(*real_malloc)(size_t);
static void *(*real_calloc)(size_t, size_t);
static void *(*real_realloc)(void *, size_t);
static void (*real_free)(void *);
static int (*real_pthread_create)(pthread_t *, const pthread_attr_t *, void *(*)(void *), void *);

/* bump arena for allocations made while dlsym runs */
static unsigned char hand_arena[1 << 20] __attribute__((aligned(64)));
static size_t hand_next;
static __thread int in_dlsym;

static unsigned long n_recorded, n_freed, n_foreign, n_hand, n_threads, n_skips;
static int canary_check = 1; /* NMG_INTERPOSE_CANARY_CHECK (read once, in resolve) */

/* records: open addressing on the user pointer, mmap'ed (not the wrapped allocator) */
struct rec {
  void *ptr;
  size_t size;
  unsigned long alloc_seq, free_seq;
  void *frames[6];
  int nframes;
};
#define REC_SLOTS (1u << 22)
static struct rec *recs;
static unsigned long seq;
static pthread_mutex_t rec_lock = PTHREAD_MUTEX_INITIALIZER;

static void resolve(void) {
  if (real_malloc) return;
  in_dlsym++;
  real_malloc = (void *(*)(size_t))dlsym(RTLD_NEXT, "malloc");
  real_calloc = (void *(*)(size_t, size_t))dlsym(RTLD_NEXT, "calloc");
  real_realloc = (void *(*)(void *, size_t))dlsym(RTLD_NEXT, "realloc");
  real_free = (void (*)(void *))dlsym(RTLD_NEXT, "free");
  real_pthread_create = (int (*)(pthread_t *, const pthread_attr_t *, void *(*)(void *), void *))dlsym(
      RTLD_NEXT, "pthread_create");
  in_dlsym--;
  {
    const char *e = getenv("NMG_INTERPOSE_CANARY_CHECK");
    canary_check = !(e && e[0] == '0');
  }
  if (!real_malloc || !real_free || !real_calloc || !real_realloc) {
    static const char m[] = "nmg_interpose: dlsym failed\n";
    (void)!write(2, m, sizeof m - 1);
    abort();
  }
}

static struct blk_head *fill_head(void *raw, size_t size, uint32_t kind) {
  struct blk_head *h = (struct blk_head *)raw;
  h->user = (unsigned char *)raw + HEAD;
  h->raw = raw;
  h->kind = kind;
  h->total = size + HEAD + TAIL;
  h->size = size;
  h->tail = (uint64_t *)((unsigned char *)h->user + size);
  memcpy(h->tail, &(uint64_t){CANARY}, 8);  /* (the tail may be unaligned) */
  h->record = NULL;
  h->canary = CANARY;
  return h;
}

static void *hand_made(size_t size) {
  size_t need = (size + HEAD + TAIL + 63) & ~(size_t)63;
  size_t at = __atomic_fetch_add(&hand_next, need, __ATOMIC_RELAXED);
  if (at + need > sizeof hand_arena) return NULL;
  __atomic_fetch_add(&n_hand, 1, __ATOMIC_RELAXED);
  return fill_head(hand_arena + at, size, KIND_HAND)->user;
}

static int ours(void *user) {
  if (!user || ((uintptr_t)user & 15)) return 0;
  return ((struct blk_head *)((unsigned char *)user - HEAD))->canary == CANARY;
}

static void print_stats(void);

/* CANARY_OK (mem_intercept.h:68): always true without the canary check, so
 * NumaMMa would read this block's header from the bytes before it and hand
 * libc a pointer taken from them.  The test interposer stops there instead:
 * it counts the block, prints its counters and a line naming the pointer,
 * and ends the process with NMG_INTERPOSE_FOREIGN_EXIT -- the outcome is
 * asserted precisely and no process that holds the GPU frees garbage. */
#define NMG_INTERPOSE_FOREIGN_EXIT 86
static int canary_ok(void *user) {
  if (!canary_check) {
    if (!ours(user)) {
      char line[160];
      int n;
      __atomic_fetch_add(&n_foreign, 1, __ATOMIC_RELAXED);
      n = snprintf(line, sizeof line,
                   "nmg_interpose: foreign block %p under canary_check=0 (its header would be trusted)\n", user);
      if (n > 0) (void)!write(2, line, (size_t)n);
      print_stats();
      _exit(NMG_INTERPOSE_FOREIGN_EXIT);
    }
    return 1;
  }
  return ours(user);
}

static size_t slot_of(void *p) { return (size_t)(((uintptr_t)p >> 4) * 0x9E3779B97F4A7C15ull >> 42) & (REC_SLOTS - 1); }

static void record_alloc(struct blk_head *h) {
  void *frames[9];
  int n;
  nmg_interpose_unsafe++;
  n = backtrace(frames, 9); /* (the first call dlopens the unwinder: recursion-protected) */
  pthread_mutex_lock(&rec_lock);
  if (!recs) {
    void *m = mmap(NULL, (size_t)REC_SLOTS * sizeof(struct rec), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS,
                   -1, 0);
    recs = m == MAP_FAILED ? NULL : (struct rec *)m;
  }
  if (recs) {
    size_t s = slot_of(h->user);
    for (unsigned probe = 0; probe < 64; probe++, s = (s + 1) & (REC_SLOTS - 1)) {
      struct rec *r = &recs[s];
      if (r->ptr && r->free_seq == 0) continue; /* live block in this slot */
      r->ptr = h->user;
      r->size = h->size;
      r->alloc_seq = ++seq;
      r->free_seq = 0;
      r->nframes = n > 3 ? (n - 3 < 6 ? n - 3 : 6) : 0;
      if (r->nframes) memcpy(r->frames, frames + 3, sizeof(void *) * (size_t)r->nframes);
      h->record = r;
      n_recorded++;
      break;
    }
  }
  pthread_mutex_unlock(&rec_lock);
  nmg_interpose_unsafe--;
}

static void record_free(struct blk_head *h) {
  struct rec *r = (struct rec *)h->record;
  if (!r) return;
  nmg_interpose_unsafe++;
  pthread_mutex_lock(&rec_lock);
  if (r->ptr == h->user && r->free_seq == 0) {
    r->free_seq = ++seq;
    n_freed++;
  }
  pthread_mutex_unlock(&rec_lock);
  nmg_interpose_unsafe--;
}

static void *wrapped_alloc(size_t size, uint32_t kind) {
  void *raw;
  struct blk_head *h;
  if (in_dlsym) return hand_made(size);
  resolve();
  nmg_interpose_unsafe++;
  raw = real_malloc(size + HEAD + TAIL);
  nmg_interpose_unsafe--;
  if (!raw) return NULL;
  h = fill_head(raw, size, kind);
  if (nmg_interpose_unsafe == 0)
    record_alloc(h);
  else {
    h->kind = KIND_INTERNAL;
    __atomic_fetch_add(&n_skips, 1, __ATOMIC_RELAXED);
  }
  return h->user;
}

void *malloc(size_t size) { return wrapped_alloc(size, KIND_MALLOC); }
void *_Znwm(size_t size) {
  void *p = wrapped_alloc(size, KIND_NEW);
  if (!p) abort();
  return p;
}
void *_Znam(size_t size) { return _Znwm(size); }

void *calloc(size_t n, size_t size) {
  size_t bytes;
  void *p;
  if (size && n > (size_t)-1 / size) return NULL;
  bytes = n * size;
  if (in_dlsym) {
    p = hand_made(bytes);
    if (p) memset(p, 0, bytes);
    return p;
  }
  p = wrapped_alloc(bytes, KIND_MALLOC);
  if (p) memset(p, 0, bytes);
  return p;
}

void free(void *ptr) {
  struct blk_head *h;
  if (!ptr) return;
  resolve();
  if (!canary_ok(ptr)) { /* not ours (memalign & co): libc's */
    __atomic_fetch_add(&n_foreign, 1, __ATOMIC_RELAXED);
    real_free(ptr);
    return;
  }
  h = (struct blk_head *)((unsigned char *)ptr - HEAD);
  if (canary_check && memcmp(h->tail, &(uint64_t){CANARY}, 8) != 0) {
    static const char m[] = "nmg_interpose: tail canary erased\n";
    (void)!write(2, m, sizeof m - 1);
    abort();
  }
  if (h->kind == KIND_HAND) return;
  if (nmg_interpose_unsafe == 0 && (h->kind == KIND_MALLOC || h->kind == KIND_NEW)) record_free(h);
  h->canary = 0;
  real_free(h->raw);
}
void _ZdlPv(void *p) { free(p); }
void _ZdaPv(void *p) { free(p); }
void _ZdlPvm(void *p, size_t n) {
  (void)n;
  free(p);
}
void _ZdaPvm(void *p, size_t n) {
  (void)n;
  free(p);
}

void *realloc(void *ptr, size_t size) {
  struct blk_head *h;
  void *raw;
  if (!ptr) return malloc(size);
  if (!size) {
    free(ptr);
    return NULL;
  }
  resolve();
  if (!canary_ok(ptr)) { /* mem_intercept.c:159-166: "I can't find this pointer !" */
    static const char m[] = "nmg_interpose: realloc of a block it did not allocate\n";
    (void)!write(2, m, sizeof m - 1);
    abort();
  }
  h = (struct blk_head *)((unsigned char *)ptr - HEAD);
  if (h->kind == KIND_HAND) { /* emulate: copy out of the arena */
    void *p = malloc(size);
    if (p) memcpy(p, ptr, h->size < size ? h->size : size);
    return p;
  }
  if (nmg_interpose_unsafe == 0) record_free(h);
  nmg_interpose_unsafe++;
  raw = real_realloc(h->raw, size + HEAD + TAIL);
  nmg_interpose_unsafe--;
  if (!raw) return NULL;
  h = fill_head(raw, size, KIND_MALLOC);
  if (nmg_interpose_unsafe == 0) record_alloc(h);
  return h->user;
}

/* memalign & co are not wrapped (nor are they in the reference): their blocks
 * reach free() without our header and go back to libc.  malloc_usable_size
 * must see through the header (libc's would read it as a chunk). */
size_t malloc_usable_size(void *ptr) {
  static size_t (*real_mus)(void *);
  if (!ptr) return 0;
  if (ours(ptr)) return ((struct blk_head *)((unsigned char *)ptr - HEAD))->size;
  if (!real_mus) real_mus = (size_t(*)(void *))dlsym(RTLD_NEXT, "malloc_usable_size");
  return real_mus ? real_mus(ptr) : 0;
}

struct tramp {
  void *(*fn)(void *);
  void *arg;
};

static void *thread_start(void *a) {
  struct tramp t = *(struct tramp *)a;
  void *ring;
  void *res;
  nmg_interpose_unsafe++;
  real_free(a);
  __atomic_fetch_add(&n_threads, 1, __ATOMIC_RELAXED);
  ring = real_malloc(64 << 10); /* the thread's sample ring */
  if (ring) memset(ring, 0, 64 << 10);
  nmg_interpose_unsafe--;
  res = t.fn(t.arg);
  nmg_interpose_unsafe++;
  real_free(ring);
  nmg_interpose_unsafe--;
  return res;
}

int pthread_create(pthread_t *th, const pthread_attr_t *attr, void *(*fn)(void *), void *arg) {
  struct tramp *t;
  resolve();
  t = (struct tramp *)real_malloc(sizeof *t);
  if (!t) return 11; /* EAGAIN */
  t->fn = fn;
  t->arg = arg;
  return real_pthread_create(th, attr, thread_start, t);
}

__attribute__((destructor)) static void report(void) { print_stats(); }

static void print_stats(void) {
  char line[256];
  int n = snprintf(line, sizeof line,
                   "nmg_interpose: {\"recorded\": %lu, \"freed\": %lu, \"foreign_frees\": %lu, \"hand_made\": %lu, "
                   "\"threads\": %lu, \"unsafe_skips\": %lu}\n",
                   n_recorded, n_freed, n_foreign, n_hand, n_threads, n_skips);
  if (n > 0) (void)!write(2, line, (size_t)n);
}
