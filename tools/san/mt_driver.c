/* mt_driver.c -- ThreadSanitizer driver of the multi-threaded CPU restatement
 * (oracle/nmg_cpu_mt.cpp, test infrastructure): analyses a replay with one
 * and with eight host threads and requires byte-identical raw results.
 *   mt_driver replay.bin raw_prefix */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

struct nmo_mt_timing {
  double load_s, analysis_s, merge_s;
  unsigned long long nb_samples;
  int threads;
};
int nmo_mt_run(const char *replay_path, const char *raw_path, int threads, int levels, struct nmo_mt_timing *tm);

static char *slurp(const char *p, long *n) {
  FILE *f = fopen(p, "rb");
  char *b;
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  *n = ftell(f);
  fseek(f, 0, SEEK_SET);
  b = malloc((size_t)*n + 1);
  if (b && fread(b, 1, (size_t)*n, f) != (size_t)*n) {
    free(b);
    b = NULL;
  }
  fclose(f);
  return b;
}

int main(int argc, char **argv) {
  char p1[4096], p8[4096];
  struct nmo_mt_timing t;
  long n1 = 0, n8 = 0;
  char *a, *b;
  if (argc != 3) {
    fprintf(stderr, "usage: %s replay.bin raw_prefix\n", argv[0]);
    return 2;
  }
  snprintf(p1, sizeof p1, "%s_1.bin", argv[2]);
  snprintf(p8, sizeof p8, "%s_8.bin", argv[2]);
  if (nmo_mt_run(argv[1], p1, 1, 1, &t) || nmo_mt_run(argv[1], p8, 8, 1, &t)) {
    fprintf(stderr, "nmo_mt_run failed\n");
    return 1;
  }
  a = slurp(p1, &n1);
  b = slurp(p8, &n8);
  if (!a || !b || n1 != n8 || memcmp(a, b, (size_t)n1) != 0) {
    fprintf(stderr, "raw results differ between 1 and 8 threads\n");
    return 1;
  }
  printf("mt_driver: 1 and 8 threads give the same %ld-byte raw results (%llu samples)\n", n1, t.nb_samples);
  return 0;
}
