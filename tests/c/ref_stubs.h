/*
 * ref_stubs.h -- the reference declarations INTEGRATION.md section 1's patch
 * uses, restated for the test harness (tests/c/nmg_patch_host.c).  Test
 * infrastructure only: no reference source is included or copied.
 *
 * Field names and types follow the reference so the patch compiles as a
 * maintainer would paste it:
 *   struct numamma_settings      src/numamma.h.in:12-34
 *   struct memory_info, date_t   src/mem_analyzer.h:8, 58-86
 *   struct ht_node / ht_entry    tools/hash.h:10-23 (here an in-order list:
 *                                FOREACH_HASH, hash.h:75-78, walks keys ascending)
 *   struct sample_list, samples  src/mem_sampling.c:61-72
 *   libmalloc                    src/mem_intercept.h:9
 *   PROTECT_RECORD               src/mem_analyzer.c:49-60
 */
#ifndef NMG_REF_STUBS_H
#define NMG_REF_STUBS_H

#include <linux/perf_event.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint64_t date_t;

struct numamma_settings {
  int verbose;
  int sampling_rate;
  int alarm;
  int flush;
  size_t buffer_size;
  int canary_check;
  char *output_dir;
  int match_samples;
  int online_analysis;
  int dump_all;
  int dump;
  int dump_unmatched;
  int dump_single_items;
};
extern struct numamma_settings settings;
char *get_log_dir(void);

enum access_type { ACCESS_READ, ACCESS_WRITE, ACCESS_MAX };
enum mem_type { none, global_symbol, stack, dynamic_allocation, lib };

struct call_site;
struct block_info;
struct memory_info {
  enum mem_type mem_type;
  date_t alloc_date;
  date_t free_date;
  size_t initial_buffer_size;
  size_t buffer_size;
  void *buffer_addr;
  void **callstack_rip;
  int callstack_size;
  void *caller_rip;
  char *caller;
  struct call_site *call_site;
  struct block_info **blocks;
  unsigned int id;
};

struct ht_entry {
  void *value;
  struct ht_entry *next;
};
struct ht_node {
  uint64_t key;
  struct ht_node *next_in_order; /* stands in for the AVL links */
  struct ht_entry *entries;      /* newest first (hash.c:108-114) */
};
#define FOREACH_HASH(root, iter) for (iter = (root); iter; iter = iter->next_in_order)
extern struct ht_node *mem_list;

struct sample_list {
  struct sample_list *next;
  struct perf_event_header *buffer;
  uint64_t data_tail;
  uint64_t data_head;
  size_t buffer_size;
  enum access_type access_type;
  date_t start_date;
  date_t stop_date;
  unsigned thread_rank;
};
extern struct sample_list *samples;
extern unsigned next_thread_rank;
extern int do_get_at_analysis;

struct mem_allocator;
extern struct mem_allocator *sample_mem;
void mem_allocator_free(struct mem_allocator *mem, void *ptr);

extern void *(*libmalloc)(size_t size);
char *get_caller_function_from_rip(void *rip);

void ma_get_variables(void);
void ma_register_stack(void);
void ma_thread_finalize(void);
void warn_non_freed_buffers(void);
void print_object_summary(void);
void mem_sampling_finalize(void);
void ma_finalize(void);

extern int is_record_safe;
#define PROTECT_RECORD do { is_record_safe = 0; } while (0)
#define UNPROTECT_RECORD do { is_record_safe = 1; } while (0)

#endif
