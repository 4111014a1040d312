/*
 * numamma_gpu.h -- C-ABI of the MI355X-native PEBS sample-analysis engine.
 *
 * Drop-in replacement for NumaMMa's offline buffer-processing loop:
 *   - the body of mem_sampling_finalize()'s `while(samples)` loop
 *     (src/mem_sampling.c:324-342) and everything it reaches
 *     (__analyze_buffer :815-927, update_counters :517-592,
 *      __match_sample :594-673, ma_find_mem_info_from_sample
 *      src/mem_analyzer.c:249-306, ma_get_block :494-534,
 *      ht_lower_key tools/hash.c:63-77);
 *   - the report half of ma_finalize() (src/mem_analyzer.c:1813-1881:
 *     update_call_sites, __print_counters, print_call_site_summary,
 *     mem_sampling_statistics src/mem_sampling.c:357-361).
 *
 * Plain C, opaque handle, int status (0 = ok, < 0 = NMG_ERR_*), no exceptions
 * and no HIP/torch types across the boundary.  The reference aborts on every
 * error (e.g. mem_sampling.c:857-860); the engine returns a code instead and
 * nmg_strerror() names it.
 *
 * Threading: one engine per calling thread; calls on one handle are not
 * re-entrant.  The online/alarm path (SIGALRM, mem_sampling.c:130-139) must
 * not call into the engine from a signal handler: enqueue there and call from
 * a worker thread.
 */
#ifndef NUMAMMA_GPU_H
#define NUMAMMA_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NMG_MAX_THREADS 1024 /* MAX_THREADS, src/numamma.h.in:9 */
#define NMG_ACCESS_READ 0    /* enum access_type, src/mem_analyzer.h:43-47 */
#define NMG_ACCESS_WRITE 1
#define NMG_NB_BUCKETS 18 /* 9 hit + 9 miss levels of struct mem_counters */

/* status codes */
#define NMG_OK 0
#define NMG_ERR_INVALID -1      /* bad argument / inconsistent table */
#define NMG_ERR_HIP -2          /* HIP runtime failure (no GPU, OOM, ...) */
#define NMG_ERR_NOMEM -3        /* host allocation failure */
#define NMG_ERR_ZERO_SIZE -4    /* record with header.size == 0 (reference abort(), mem_sampling.c:857-860) */
#define NMG_ERR_TRUNCATED -5    /* SAMPLE record running past the buffer end (reference reads out of bounds, :865-879) */
#define NMG_ERR_STATE -6        /* call out of order (e.g. analyze before set_objects) */
#define NMG_ERR_RANGE -7        /* thread rank >= nb_threads, buffer >= 4 GiB (unsigned cursors, :831-834) */
#define NMG_ERR_CAPACITY -8     /* sparse page-histogram table full (raise nmg_options.sparse_capacity) */
#define NMG_ERR_UNALIGNED -9    /* record size not a multiple of 8 (perf ABI guarantees 8-byte records) */
#define NMG_ERR_IO -10          /* report file could not be written */

/* engine flags */
#define NMG_F_MATCH_SAMPLES 0x1  /* settings.match_samples (numamma.h.in:27) */
#define NMG_F_PAGE_HIST 0x2      /* per-(object, page, thread) counts for callsite_counters_<id>.dat */
#define NMG_F_OBJECT_LEVELS 0x4  /* per-object level buckets (count, sum) for callsite_summary_<id>.dat */
#define NMG_F_SAMPLE_MATCHES 0x8 /* keep every SAMPLE record's match (object or none) for the dump modes */
#define NMG_F_SINGLE_PASS 0x10   /* large tables (> 1023 keys): one attribution pass with global lookups instead of
                                    the partition-first passes; same results (A/B and tests) */
#define NMG_F_DEFAULT (NMG_F_MATCH_SAMPLES | NMG_F_PAGE_HIST)
/* every public flag: nmg_create rejects any other bit with NMG_ERR_INVALID */
#define NMG_F_ALL (NMG_F_MATCH_SAMPLES | NMG_F_PAGE_HIST | NMG_F_OBJECT_LEVELS | NMG_F_SAMPLE_MATCHES | NMG_F_SINGLE_PASS)

/* struct count, src/mem_analyzer.h:10-15 */
struct nmg_count {
  uint64_t count, min_weight, max_weight, sum_weight;
};

/* struct mem_counters, src/mem_analyzer.h:17-41 (same 600-byte layout);
 * b[0..8] = L1, L2, L3, LFB, local RAM, remote RAM, remote cache, IO,
 * uncached hits; b[9..17] = the same levels' misses. */
struct nmg_mem_counters {
  uint64_t total_count, total_weight, na_miss_count;
  struct nmg_count b[NMG_NB_BUCKETS];
};

/* One entry of the object table: the fields of struct memory_info
 * (src/mem_analyzer.h:68-86) that sample attribution reads. */
struct nmg_object {
  uint64_t buffer_addr; /* current address (realloc rewrites it, quirk Q5) */
  uint64_t buffer_size; /* size at free (ma_record_free, mem_analyzer.c:1287) */
  uint64_t alloc_date;  /* 0 for globals / libs / [stack] */
  uint64_t free_date;   /* after warn_non_freed_buffers (mem_analyzer.c:1751-1799) */
};

/* Host-only metadata of an entry, consumed by the call-site registry
 * (find_call_site / new_call_site, mem_analyzer.c:1302-1378). */
struct nmg_object_meta {
  uint64_t initial_buffer_size;
  uint64_t caller_rip;
  const uint64_t *callstack; /* NULL == callstack_rip NULL */
  int32_t callstack_size;
  uint32_t mem_type; /* enum mem_type, mem_analyzer.h:58-64 (2 == stack) */
  const char *caller; /* symbolised call site; NULL -> "???" for a NULL rip */
  uint32_t id;
  uint32_t reserved;
};

struct nmg_options {
  int32_t device;            /* HIP device ordinal */
  uint32_t flags;            /* NMG_F_* */
  uint32_t nb_threads;       /* next_thread_rank: page-histogram columns (<= 1024) */
  uint32_t copy_threads;     /* host threads for nmg_submit_buffers copies (0 = 1) */
  uint64_t hist_budget_bytes; /* dense page-histogram arena cap (0 = default 4 GiB) */
  uint64_t sparse_capacity;   /* sparse (object, page, thread) slots (0 = default 1<<22) */
  /* Multi-GPU from one host process: nb_gpus > 1 shards the
   * submitted buffer list over the GPUs devices[0..nb_gpus) (NULL: device,
   * device + 1, ...) in contiguous byte-balanced ranges, replicates the
   * object table, and merges the per-GPU counters into this handle at
   * nmg_analyze -- RCCL reduces over xGMI (sum / min / max) when the devices
   * are distinct, a device-side merge when they are one device (testing).
   * Results, getters and nmg_report read the merged counters.  Such an engine
   * takes host buffers (nmg_submit_*); device-resident buffers and streaming
   * stay single-GPU.  0 or 1: one GPU, `device`.
   * The three fields below were added after the first version of this
   * struct (which ended at sparse_capacity, NMG_OPTIONS_V1_SIZE bytes).
   * nmg_create reads the whole current struct: zero-initialise it.  A
   * caller built against the first version passes its own struct size to
   * nmg_create_ex, which reads only that many bytes.  nb_gpus / devices are
   * used only with abi_version == NMG_OPTIONS_ABI.  Without it they are
   * ignored by nmg_create (a first-version binary's bytes past its struct),
   * and nmg_create_ex(..., sizeof(struct nmg_options)) rejects nb_gpus > 1
   * with NMG_ERR_INVALID (not a silent one-GPU engine). */
  uint32_t nb_gpus;
  uint32_t abi_version;      /* NMG_OPTIONS_ABI to use nb_gpus / devices */
  const int32_t *devices;
};
#define NMG_OPTIONS_ABI 0x4e4d4702u /* "NMG" v2: nmg_options with nb_gpus / abi_version / devices */
#define NMG_OPTIONS_V1_SIZE 32      /* bytes of the first struct version: device .. sparse_capacity */

struct nmg_report_options {
  const char *output_dir;  /* settings.output_dir; call_sites.log etc. land here */
  int32_t dump_single_items; /* write callsite_counters_<id>.dat (default 1) */
  int32_t dump_flags;        /* NMG_DUMP_*: the dump modes (engine created with
                                NMG_F_SAMPLE_MATCHES | NMG_F_OBJECT_LEVELS) */
  const char *maps_path;     /* NMG_DUMP_UNMATCHED header: the traced process's "/proc/<pid>/maps" */
  const char *maps_text;     /* ... and that file's content, captured with the run (NULL: none) */
  /* NMG_DUMP_ALL: all_memory_objects.dat's callstack_offsets column resolves
   * each frame as dladdr() did in the traced process (_print_object_summary,
   * mem_analyzer.c:1660-1690): the module whose [lo, hi) holds the rip gives
   * dli_fname and dli_fbase.  A frame outside every module prints
   * "(null):<rip>" (dladdr failed; the reference reads an uninitialised
   * Dl_info there -- unpinned). */
  const struct nmg_module *modules;
  uint32_t nb_modules;
  /* --online-analysis (mem_sampling.c:313, :953-954): the counters were
   * accumulated alarm by alarm (nmg_update_objects), so mem_sampling_finalize
   * prints nothing, and every object has counters from its creation
   * (_init_mem_info, mem_analyzer.c:569-572), so ma_finalize passes each one
   * to update_call_sites (:1832-1834), matched or not. */
  uint32_t online;
};

struct nmg_module {
  uint64_t lo, hi;   /* text range of the loaded object */
  uint64_t fbase;    /* Dl_info.dli_fbase */
  const char *fname; /* Dl_info.dli_fname */
};
/* dump modes (settings.dump / dump_all / dump_unmatched, numamma.h.in:28-31;
 * mem_sampling.c:599-650, 740-808, 895-914; mem_analyzer.c:1489-1528):
 * callsite_dump_<id>.dat and callsite_summary_<id>.dat, all_memory_accesses.dat,
 * unmatched_samples.log.  get_data_src_level() strings are numap's (unpinned
 * beyond "L1_Hit", "L2_Hit", "L3_Hit", README.md:142-147). */
#define NMG_DUMP_CALLSITES 0x1 /* -d */
#define NMG_DUMP_ALL 0x2       /* -D; also all_memory_objects.dat (mem_analyzer.c:1728-1748) */
#define NMG_DUMP_UNMATCHED 0x4 /* -u */

struct nmg_engine;
typedef struct nmg_engine nmg_engine;

const char *nmg_strerror(int status);
/* text of the last error on h (h == NULL: the calling thread's last failed nmg_create) */
int nmg_get_last_error_detail(nmg_engine *h, char *buf, size_t len);

/* opt == NULL: defaults.  Flags outside NMG_F_ALL are NMG_ERR_INVALID. */
int nmg_create(nmg_engine **out, const struct nmg_options *opt);
/* The same, reading only the first opt_size bytes of *opt (the rest as
 * zero): NMG_OPTIONS_V1_SIZE for a caller of the first struct version. */
int nmg_create_ex(nmg_engine **out, const struct nmg_options *opt, size_t opt_size);
void nmg_destroy(nmg_engine *h);

/*
 * Object table snapshot: the AVL tree of mem_analyzer.c after
 * warn_non_freed_buffers + ma_register_stack, flattened.  keys[] are the
 * node keys in ascending order (unique); node i owns entries
 * [entry_off[i], entry_off[i+1]) listed newest-first (the LIFO entry list of
 * tools/hash.c:108-114).  Copied; the caller keeps ownership.
 */
int nmg_set_objects(nmg_engine *h, const uint64_t *keys, const uint32_t *entry_off,
                    uint32_t nb_keys, const struct nmg_object *entries, uint32_t nb_entries);

/*
 * Online analysis (--online-analysis: __process_samples analyses each alarm's
 * rings in place, mem_sampling.c:953-954, against the object table as it is
 * at that alarm): replace the lookup table, keeping every counter.  The
 * table is flattened like nmg_set_objects': keys[] ascending, key i's entries
 * [entry_off[i], entry_off[i+1]) of objects[] newest-first, and entry_ids[j]
 * the id of objects[j] -- the index of its counters.  Objects still alive at
 * the alarm carry free_date 0 (they never match, quirk Q3); objects not yet
 * allocated are absent.
 *   Live hosts (mem_info->id - 1 as the id): nmg_set_objects may start empty
 * (or with the table of the first alarm); an update may list new ids, which
 * must run consecutively from the current entry count: their counters start
 * at zero, as _init_mem_info gives a new object counters at creation
 * (mem_analyzer.c:567-572).  An object whose size grew (ma_record_free,
 * :1287) keeps its page counts in a larger range.
 *   Recorded runs: nmg_set_objects with the final table, and alarm tables
 * listing subsets of its ids.
 *   The report describes each entry as the latest table listed it, walking
 * the entries in the order of the latest table that listed every one (at
 * exit, pass the table ma_finalize walks: nmg_update_objects with the final
 * table; nmg_report's meta[] then follows that table's order).  In streaming
 * mode the open chunk is analysed with the previous table first.  Copied; the
 * caller keeps ownership.
 */
int nmg_update_objects(nmg_engine *h, const uint64_t *keys, const uint32_t *entry_off, uint32_t nb_keys,
                       const uint32_t *entry_ids, const struct nmg_object *objects);

/*
 * Append one captured buffer to the analysis list, in analysis order (the
 * reference analyses `samples` head-first, i.e. newest capture first).
 * nmg_submit_ring() linearises a perf ring segment [data_tail, data_head)
 * exactly like __copy_buffer (mem_sampling.c:675-738); an empty segment is
 * dropped, as the reference never pushes it.  Bytes are copied to pinned
 * staging memory; the caller keeps ownership.
 */
int nmg_submit_ring(nmg_engine *h, const void *ring, uint64_t ring_size, uint64_t data_tail,
                    uint64_t data_head, uint32_t thread_rank, uint32_t access_type);
int nmg_submit_buffer(nmg_engine *h, const void *bytes, uint64_t len, uint32_t thread_rank,
                      uint32_t access_type);

/*
 * Batch form of nmg_submit_buffer: n linearised buffers (host pointers, e.g.
 * the malloc'd __copy_buffer copies of the `samples` list, mem_sampling.c:696),
 * in analysis order.  The copies into pinned staging are split over the
 * engine's copy threads (nmg_options.copy_threads / nmg_stream_begin).  Empty buffers are
 * dropped like in nmg_submit_buffer.
 */
int nmg_submit_buffers(nmg_engine *h, uint32_t n, const void *const *bytes, const uint64_t *lens,
                       const uint32_t *thread_ranks, const uint32_t *access_types);

/*
 * Host memory the kernels read in place: [ptr, ptr + bytes) is pinned and
 * mapped for the device (hipHostRegister) once -- e.g. a thread's mmap'd
 * perf ring (numap; the ring nmg_submit_ring reads at every alarm,
 * mem_sampling.c:675-738).  A buffer later given to nmg_submit_buffer(s) or
 * nmg_submit_ring (unwrapped segment) that lies inside such a range and
 * starts 16-byte aligned is not copied: nmg_analyze's kernels read it over
 * PCIe, so it must stay unchanged until nmg_synchronize.  Batch path of a
 * single-GPU engine without the dump modes only (streaming, dump modes and
 * multi-GPU handles copy as before).  ptr must be page-aligned (4 KiB) and
 * the pages up to ptr + bytes rounded up belong to the caller alone: whole
 * pages are registered.  Ranges must not overlap.
 * nmg_unregister_host takes the ptr given at registration; buffers inside
 * the range must have been dropped (nmg_clear_buffers) first.
 */
int nmg_register_host(nmg_engine *h, void *ptr, uint64_t bytes);
int nmg_unregister_host(nmg_engine *h, void *ptr);

/*
 * Streaming (BASELINE configs[4]; the online branch of __process_samples,
 * mem_sampling.c:953-957, fed at each alarm, :130-177): buffers submitted
 * after nmg_stream_begin are uploaded and analysed in chunks of about
 * chunk_bytes while the caller keeps submitting -- double-buffered pinned
 * staging, hipMemcpyAsync on a copy stream, the attribution kernel on the
 * engine stream as soon as its chunk has landed.  A submit blocks only when
 * both staging halves are still in flight.  nmg_analyze() flushes the last
 * partial chunk; results accumulate exactly as for one nmg_analyze over all
 * buffers (analysis order = submission order across chunks).  copy_threads
 * (>= 1) host threads copy each nmg_submit_buffers batch.  Attribution uses
 * the table of the last nmg_set_objects (online semantics).
 * Not combinable with nmg_set_device_buffers.
 */
int nmg_stream_begin(nmg_engine *h, uint64_t chunk_bytes, uint32_t copy_threads);
/* Flush the open chunk and leave streaming mode (buffers stay counted). */
int nmg_stream_end(nmg_engine *h);

/*
 * Device-resident variant: linearised buffers already in HBM (caller-owned).
 * offsets[] must be 16-byte aligned.  seq_base = analysis-order index of
 * buffer 0 (non-zero when the buffer list is sharded over GPUs).  Replaces any
 * previously submitted buffers.
 */
int nmg_set_device_buffers(nmg_engine *h, const void *d_data, const uint64_t *offsets,
                           const uint64_t *lengths, const uint32_t *thread_ranks,
                           const uint32_t *access_types, uint32_t nb_buffers, uint64_t seq_base);

/* Enqueue attribution of every submitted buffer (stages host buffers H2D
 * first).  Asynchronous; counters accumulate across calls. */
int nmg_analyze(nmg_engine *h);
int nmg_synchronize(nmg_engine *h);
/* Zero every counter (global, per buffer, per object, page histogram); per
 * buffer counts replaced by nmg_set_buffer_counts are dropped (the engine's own
 * buffers again). */
int nmg_reset_counters(nmg_engine *h);
/* Drop every submitted buffer (staging memory is kept for reuse). */
int nmg_clear_buffers(nmg_engine *h);

/* ---- results (synchronising, copied to host) ---- */
int nmg_get_global_counters(nmg_engine *h, struct nmg_mem_counters out[2],
                            uint64_t *nb_samples, uint64_t *nb_found);
uint32_t nmg_get_nb_buffers(nmg_engine *h);
/* per analysed buffer: SAMPLE records and matched samples */
int nmg_get_buffer_counts(nmg_engine *h, uint32_t *nb_samples, uint32_t *nb_found);
/* per entry: first-match ordinal ((analysis seq << 32) | byte offset,
 * UINT64_MAX if never matched), and per access (count, weight) */
int nmg_get_object_counters(nmg_engine *h, uint64_t *first_ordinal, uint64_t *count_weight /* [E][2][2] */);
/* per entry and access: na_miss_count then 18 x (count, sum) [E][2][37] (NMG_F_OBJECT_LEVELS) */
int nmg_get_object_levels(nmg_engine *h, uint64_t *levels);
/* number of non-zero (entry, thread, page) cells */
int64_t nmg_count_page_cells(nmg_engine *h);
/* non-zero cells as (entry, thread, page, count) rows in (entry, thread, page) order */
int nmg_get_page_cells(nmg_engine *h, uint32_t *rows /* [n][4] */, int64_t n);

/* ---- results snapshot: the getters' results copied to host memory while
 * the next analysis runs (one engine of one GPU; not a multi-GPU handle, not
 * after nmg_set_buffer_counts).
 * nmg_results_begin enqueues, behind the analyses already enqueued, a device
 * copy of every result (the per-buffer matched counts and the page-cell rows
 * built there) and their copy to pinned host memory on a stream of their
 * own, and returns: the engine may be reset and analyse again at once.
 * nmg_results_end waits for that copy and describes it; the arrays are the
 * engine's and stay valid until the next nmg_results_begin or
 * nmg_destroy.  Their content equals what nmg_get_global_counters,
 * nmg_get_buffer_counts, nmg_get_object_counters and nmg_get_page_cells
 * returned at the time of nmg_results_begin. */
struct nmg_results_view {
  struct nmg_mem_counters global[2];
  uint64_t nb_samples, nb_found;
  uint32_t nb_buffers, nb_entries;
  const uint32_t *buffer_samples, *buffer_found; /* [nb_buffers] */
  const uint64_t *first_ordinal;                 /* [nb_entries] */
  const uint64_t *count_weight;                  /* [nb_entries][2][2] */
  int64_t nb_cells;
  const uint32_t *cells;                         /* [nb_cells][4] as nmg_get_page_cells */
};
int nmg_results_begin(nmg_engine *h);
int nmg_results_end(nmg_engine *h, struct nmg_results_view *out);

/* ---- multi-GPU merge (sharded buffer lists, one engine per rank) ----
 * Arrays are exposed as flat u64 / u32 vectors so a caller can reduce them
 * with RCCL (torch.distributed) over xGMI:
 *   NMG_ARR_SUM64  : u64 sums   (global sums, per-object counts/weights/levels)
 *   NMG_ARR_MIN64  : u64 mins   (global bucket mins, first-match ordinals, error word)
 *   NMG_ARR_MAX64  : u64 maxes  (global bucket maxes)
 *   NMG_ARR_HIST32 : u32 sums   (dense page histogram)
 * nmg_export_array copies device -> device (dst is a device pointer),
 * nmg_import_array copies back.  Sizes in elements. */
#define NMG_ARR_SUM64 0
#define NMG_ARR_MIN64 1
#define NMG_ARR_MAX64 2
#define NMG_ARR_HIST32 3
uint64_t nmg_array_size(nmg_engine *h, int which);
int nmg_export_array(nmg_engine *h, int which, void *d_dst);
int nmg_import_array(nmg_engine *h, int which, const void *d_src);
/* The page histogram packed for the merge (NMG_ARR_HIST32 is most of the
 * payload: 98 of 140 MB per rank at 1M intervals).  nmg_hist_pack writes
 * every cell of at most `threshold` (<= 255) as one byte to d_u8 (device,
 * nmg_array_size(HIST32) bytes; larger cells as 0) and each larger cell as
 * (cell << 32 | count) to d_ovf (device, ovf_cap u64); *n_ovf = their number
 * (> ovf_cap: the list is incomplete -- merge NMG_ARR_HIST32 instead).  With
 * threshold <= 255 / ranks the byte arrays of all ranks add up without
 * overflow (a u8 SUM reduce); the root then calls nmg_hist_unpack with the
 * summed bytes and every rank's overflow entries (entries with count 0 are
 * padding): histogram = bytes + overflow, exactly the u32 sum. */
int nmg_hist_pack(nmg_engine *h, uint32_t threshold, void *d_u8, void *d_ovf, uint64_t ovf_cap, uint64_t *n_ovf);
int nmg_hist_unpack(nmg_engine *h, const void *d_u8, const void *d_ovf, uint64_t n_ovf);
/* Packed per-object counters for the merge: the count and
 * weight rows of a sum64 image (nmg_export_array(NMG_ARR_SUM64) into d_sum64)
 * as u32 words where a value is below `threshold` (2^32 / ranks: the sum over
 * the ranks fits), 0 where it is not, and those values listed as (row word,
 * value) u64 pairs in d_ovf (up to ovf_cap pairs; *n_ovf = the full length).
 * d_u32 holds 4 * nb_entries words.  After a u32 SUM reduce of d_u32 and a
 * gather of the lists, nmg_objcw_unpack writes the rows of d_sum64 (then
 * nmg_import_array) from the summed words plus every listed value. */
int nmg_objcw_pack(nmg_engine *h, const void *d_sum64, uint64_t threshold, void *d_u32, void *d_ovf,
                   uint64_t ovf_cap, uint64_t *n_ovf);
int nmg_objcw_unpack(nmg_engine *h, void *d_sum64, const void *d_u32, const void *d_ovf, uint64_t n_ovf);
/* sparse (object, page, thread) cells: export as (key, count) pairs on host,
 * in ascending key order (keys are unique) */
int64_t nmg_sparse_count(nmg_engine *h);
int nmg_sparse_export(nmg_engine *h, uint64_t *keys, uint32_t *counts, int64_t n);
int nmg_sparse_import(nmg_engine *h, const uint64_t *keys, const uint32_t *counts, int64_t n);
/* replace per-buffer counts with the whole job's (rank 0 before reporting) */
int nmg_set_buffer_counts(nmg_engine *h, uint32_t nb_buffers, const uint32_t *nb_samples,
                          const uint32_t *nb_found, const uint64_t *buffer_bytes);

/* ---- device timing of the last nmg_analyze (HIP events on the engine stream) ---- */
int nmg_last_analyze_ms(nmg_engine *h, float *ms);
/* durations of up to n most recent launches (oldest first, max 64); returns the count */
int nmg_get_launch_times(nmg_engine *h, float *ms, int n);
/* the same launches split: the attribution kernel alone (attribute_ms) and the
 * whole launch including the long-tail reduce (total_ms); returns the count */
int nmg_get_kernel_times(nmg_engine *h, float *attribute_ms, float *total_ms, int n);
/* a multi-GPU handle's last nmg_analyze: GPU time of the counter merge on the
 * root device (from the end of worker 0's analysis to the end of the reduces
 * into the handle, waiting for the other workers included) and the counter
 * bytes each worker contributes to it (sum64, min64, max64, page histogram);
 * 0 and 0 for a single-GPU engine */
int nmg_get_merge_stats(nmg_engine *h, float *merge_ms, uint64_t *payload_bytes);

/*
 * Report: the stdout text of mem_sampling_finalize + ma_finalize from
 * "Analyzing %d sample buffers" to the final statistics line, written to
 * stdout_path (NULL = process stdout), plus call_sites.log and
 * callsite_counters_<id>.dat in opts->output_dir -- byte-identical formats
 * (mem_analyzer.c:1438-1640, mem_sampling.c:321-361).
 * meta[] parallels the entries passed to nmg_set_objects.
 * The per-site files are written by up to 16 host threads (environment:
 * NMG_REPORT_THREADS=n sets the count, NMG_REPORT_TIMING=1 prints phase times
 * on stderr); the output does not depend on the count.
 */
int nmg_report(nmg_engine *h, const struct nmg_object_meta *meta,
               const struct nmg_report_options *opts, const char *stdout_path);

/*
 * Host-only report from plain result arrays (no GPU needed): what rank 0 runs
 * after a multi-GPU merge, and what nmg_report() calls internally.
 * cells[] = (entry, thread, page, count) rows sorted by entry.
 */
struct nmg_host_results {
  struct nmg_mem_counters global[2];
  uint32_t nb_buffers;
  uint32_t nb_entries;
  const uint32_t *buf_samples; /* per analysed buffer (int in the reference) */
  const uint32_t *buf_found;
  const uint64_t *buf_bytes;
  const uint64_t *buffer_size;   /* per entry: struct memory_info.buffer_size */
  const uint64_t *first_ordinal; /* per entry, UINT64_MAX = never matched */
  const uint64_t *count_weight;  /* [E][2][2] */
  const uint32_t *cells;
  int64_t nb_cells;
  uint32_t nb_threads;    /* next_thread_rank */
  uint32_t match_samples; /* settings.match_samples */
  /* per entry (the nmg_set_objects table): all_memory_objects.dat rows
   * (NMG_DUMP_ALL); may be NULL otherwise */
  const struct nmg_object *objects;
};
int nmg_report_host(const struct nmg_host_results *res, const struct nmg_object_meta *meta,
                    const struct nmg_report_options *opts, const char *stdout_path);

/* Convenience driver used by the nmg_replay CLI and the tests: load a replay
 * file (DESIGN.md "Replay format"), analyse it on `device`, report. */
int nmg_run_replay(const char *replay_path, const char *output_dir, const char *stdout_path,
                   const char *raw_path, int device, uint32_t flags);

/*
 * Capture/replay bridge: record a live run's analysis input
 * in the replay format, host-only (no GPU), so that it can be analysed later,
 * elsewhere, or by an out-of-process helper (`nmg_replay` CLI) when HIP must
 * not run inside the LD_PRELOAD'ed process.
 *   nmg_replay_open: the object-table snapshot, with the same arrays as
 *     nmg_set_objects plus the call-site metadata (taken where ma_finalize
 *     walks mem_list, src/mem_analyzer.c:1813); callstacks and caller strings
 *     are copied into the file's pools;
 *   nmg_replay_add_ring: one `samples` list element in analysis order
 *     (mem_sampling.c:324), stored as given (the ring segment [data_tail,
 *     data_head) is linearised at analysis time, like nmg_submit_ring);
 *   nmg_replay_close: patches the buffer count and closes the file.
 */
typedef struct nmg_replay_writer nmg_replay_writer;
int nmg_replay_open(nmg_replay_writer **out, const char *path, uint32_t nb_threads, const uint64_t *keys,
                    const uint32_t *entry_off, uint32_t nb_keys, const struct nmg_object *entries,
                    const struct nmg_object_meta *meta, uint32_t nb_entries);
int nmg_replay_add_ring(nmg_replay_writer *w, const void *ring, uint64_t ring_size, uint64_t data_tail,
                        uint64_t data_head, uint32_t thread_rank, uint32_t access_type);
/* The dump modes' context of the traced process, stored in the replay's
 * optional trailing section and used by nmg_run_replay when NMG_REPLAY_DUMP
 * is set: the module table (dladdr, all_memory_objects.dat) and
 * /proc/<pid>/maps (unmatched_samples.log header).  Call before close. */
int nmg_replay_set_context(nmg_replay_writer *w, const struct nmg_module *modules, uint32_t nb_modules,
                           const char *maps_path, const char *maps_text);
int nmg_replay_close(nmg_replay_writer *w);

#ifdef __cplusplus
}
#endif
#endif /* NUMAMMA_GPU_H */
