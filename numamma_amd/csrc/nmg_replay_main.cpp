// nmg_replay CLI: analyse a replay file on the GPU and write NumaMMa's report.
//   nmg_replay replay.bin outdir [--raw raw.bin] [--device N] [--no-match]
// Environment: NMG_REPLAY_DUMP=<NMG_DUMP_* flags> (the -d / -D / -u outputs,
// with the replay's context section), NMG_REPLAY_STREAM=chunk[:threads[:batch]].
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "numamma_gpu.h"

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr,
            "usage: %s replay.bin outdir [--raw raw.bin] [--device N] [--no-match]\n"
            "  env NMG_REPLAY_DUMP=<1 -d | 2 -D | 4 -u>, NMG_REPLAY_STREAM=chunk[:threads[:batch]]\n",
            argv[0]);
    return 2;
  }
  const char* raw = nullptr;
  int device = 0;
  uint32_t flags = NMG_F_DEFAULT;
  for (int i = 3; i < argc; i++) {
    if (!strcmp(argv[i], "--raw") && i + 1 < argc) raw = argv[++i];
    else if (!strcmp(argv[i], "--device") && i + 1 < argc) device = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--no-match")) flags &= ~NMG_F_MATCH_SAMPLES;
    else {
      fprintf(stderr, "unknown argument %s\n", argv[i]);
      return 2;
    }
  }
  int rc = nmg_run_replay(argv[1], argv[2], nullptr, raw, device, flags);
  return rc ? 1 : 0;
}
