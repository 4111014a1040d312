// report_threads.cpp -- ThreadSanitizer driver of the report writer's threads
// (tools/sanitize.sh).
//
// nmg_report_host (numamma_amd/csrc/nmg_report.cpp) writes the
// callsite_counters_<id>.dat files from a pool of up to 16 threads
// (NMG_REPORT_THREADS).  This program builds a seeded synthetic result set --
// 4000 entries in ~1300 call sites, a few pages each, 8 threads, cells for
// most matched entries -- reports it once with one writer thread and once
// with seven, under -fsanitize=thread, and requires the two output trees to
// be byte-identical.
//
//   report_threads OUT_DIR
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "numamma_gpu.h"

static std::string slurp(const std::string& p) {
  std::string s;
  if (FILE* f = fopen(p.c_str(), "rb")) {
    char buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
    fclose(f);
  }
  return s;
}

int main(int argc, char** argv) {
  if (argc != 2) {
    fprintf(stderr, "usage: %s OUT_DIR\n", argv[0]);
    return 2;
  }
  const std::string out = argv[1];
  const uint32_t E = 4000, T = 8;
  std::mt19937_64 rng(12345);
  std::vector<uint64_t> size(E), first(E, ~0ull), cw(4 * E, 0);
  std::vector<nmg_object_meta> meta(E);
  std::vector<uint64_t> stacks(E * 6);
  std::vector<std::string> callers(E / 3 + 1);
  for (size_t i = 0; i < callers.size(); i++) callers[i] = "site_" + std::to_string(i);
  std::vector<uint32_t> cells;
  for (uint32_t e = 0; e < E; e++) {
    const uint32_t site = (uint32_t)(rng() % callers.size());
    size[e] = 64 + 4096 * (site % 5) + (site % 97);
    meta[e] = nmg_object_meta{};
    meta[e].initial_buffer_size = size[e];
    meta[e].caller_rip = 0x400000 + site;
    for (int k = 0; k < 6; k++) stacks[e * 6 + k] = 0x400000 + site * 7 + (uint64_t)k;
    meta[e].callstack = &stacks[e * 6];
    meta[e].callstack_size = 6;
    meta[e].mem_type = 3;
    meta[e].caller = callers[site].c_str();
    meta[e].id = e + 1;
    if (rng() % 4 == 0) continue;  // never matched
    first[e] = ((uint64_t)(rng() % 5000) << 32) | (rng() % 100000);
    for (int a = 0; a < 2; a++) {
      cw[(e * 2 + a) * 2 + 0] = rng() % 1000;
      cw[(e * 2 + a) * 2 + 1] = rng() % 200000;
    }
    const uint32_t np = (uint32_t)(size[e] / 4096 + 1);
    for (uint32_t t = 0; t < T; t++)
      for (uint32_t pg = 0; pg < np; pg++)
        if (rng() % 3) cells.insert(cells.end(), {e, t, pg, (uint32_t)(1 + rng() % 50)});
  }
  std::vector<uint32_t> bs(100, 1000), bf(100, 700);
  std::vector<uint64_t> bb(100, 40000);
  nmg_host_results r;
  memset(&r, 0, sizeof r);
  r.global[0].total_count = 100000;
  r.global[0].total_weight = 1234567;
  r.nb_buffers = 100;
  r.nb_entries = E;
  r.buf_samples = bs.data();
  r.buf_found = bf.data();
  r.buf_bytes = bb.data();
  r.buffer_size = size.data();
  r.first_ordinal = first.data();
  r.count_weight = cw.data();
  r.cells = cells.data();
  r.nb_cells = (int64_t)(cells.size() / 4);
  r.nb_threads = T;
  r.match_samples = 1;
  std::string trees[2];
  for (int k = 0; k < 2; k++) {
    const char* nth = k ? "7" : "1";
    setenv("NMG_REPORT_THREADS", nth, 1);
    const std::string dir = out + "/threads_" + nth;
    nmg_report_options ro;
    memset(&ro, 0, sizeof ro);
    ro.output_dir = dir.c_str();
    ro.dump_single_items = 1;
    const std::string so = dir + ".stdout";
    const int rc = nmg_report_host(&r, meta.data(), &ro, so.c_str());
    if (rc) {
      fprintf(stderr, "nmg_report_host (%s threads): %d\n", nth, rc);
      return 1;
    }
    trees[k] = slurp(so) + slurp(dir + "/call_sites.log");
    for (uint32_t id = 1; id < 2000; id++) trees[k] += slurp(dir + "/callsite_counters_" + std::to_string(id) + ".dat");
  }
  if (trees[0] != trees[1] || trees[0].size() < 10000) {
    fprintf(stderr, "report trees differ between 1 and 7 writer threads (%zu vs %zu bytes)\n", trees[0].size(),
            trees[1].size());
    return 1;
  }
  printf("report_threads: 1 and 7 writer threads give the same %zu bytes\n", trees[0].size());
  return 0;
}
