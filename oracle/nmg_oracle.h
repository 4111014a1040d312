/*
 * nmg_oracle.h -- TEST INFRASTRUCTURE ONLY (see nmg_oracle.c header).
 * CPU restatement of NumaMMa's offline sample-analysis path.
 */
#ifndef NMG_ORACLE_H
#define NMG_ORACLE_H
#include <stdint.h>

#define NMO_ERR_IO -1
#define NMO_ERR_FORMAT -2
#define NMO_ERR_ZERO_SIZE -3
#define NMO_ERR_TRUNCATED -4

struct nmo_settings {
  int match_samples;     /* settings.match_samples (numamma.h.in:27) */
  int dump_single_items; /* settings.dump_single_items (numamma.h.in:32) */
  int dump;              /* settings.dump, -d (numamma.h.in:28) */
  int dump_all;          /* settings.dump_all, -D (numamma.h.in:29) */
  int dump_unmatched;    /* settings.dump_unmatched, -u (numamma.h.in:31) */
  int reserved;
  const char *maps_path; /* "/proc/<pid>/maps" of the traced process (unmatched_samples.log header) */
  const char *maps_text; /* that file's content, captured with the run (NULL: empty) */
  const struct nmo_module *modules; /* dladdr() of the traced process (all_memory_objects.dat) */
  uint32_t nb_modules;
  uint32_t reserved2;
  /* --online-analysis (mem_sampling.c:953-954): nb_alarms > 0 analyses the
   * buffers alarm by alarm, each against the object table as it stands at
   * that alarm, and reports as ma_finalize does online */
  const struct nmo_alarm *alarms;
  uint32_t nb_alarms;
  uint32_t reserved3;
};

/* The object table at one alarm, flattened like the replay's (keys
 * ascending, entries newest-first), and the buffers analysed with it:
 * [previous alarm's buf_end, buf_end).  entry_ids[j] = index of entry j in
 * the replay's (final) table, whose counters it updates; ent4[j] = its
 * (buffer_addr, buffer_size, alloc_date, free_date) at the alarm. */
struct nmo_alarm {
  uint32_t buf_end;
  uint32_t nb_keys;
  const uint64_t *keys;
  const uint32_t *entry_off; /* [nb_keys + 1] */
  const uint32_t *entry_ids;
  const uint64_t *ent4;
};

/* Dl_info of the frames in [lo, hi): dli_fbase, dli_fname */
struct nmo_module {
  uint64_t lo, hi, fbase;
  const char *fname;
};

struct nmo_timing {
  double analysis_s; /* mem_sampling_finalize() loop */
  double total_s;    /* analysis + report */
  uint64_t nb_samples;
};

/* Run the whole offline analysis of a replay file: writes the reference's
 * stdout report to stdout_path (or stdout), call_sites.log and
 * callsite_counters_<id>.dat into outdir, and (optionally) the canonical
 * raw-results dump to raw_path.  Returns 0 or a NMO_ERR_* code. */
int nmo_run(const char *replay_path, const char *outdir, const char *stdout_path,
            const char *raw_path, const struct nmo_settings *settings,
            struct nmo_timing *timing);
const char *nmo_strerror(int rc);
int64_t nmo_lookup(const uint64_t *keys, const uint32_t *entry_off, uint32_t nb_keys,
                   const uint64_t *ent4, uint64_t addr, uint64_t ts);

#endif
