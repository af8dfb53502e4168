/*
 * gen_synth <kind> <nbases> <out-file> [seed]
 * Writes the synthetic genome of csrc/synth.h (kind 0 uniform, 1 tandem) as a
 * single line of lowercase bases, no header, no trailing newline.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>

#include "synth.h"

typedef struct { char *buf; int kind; uint64_t seed, begin, end; } job_t;

static void *run(void *p) {
  job_t *j = (job_t *)p;
  gcz_synth_fill_range(j->buf + j->begin, j->kind, j->seed, j->begin, j->end);
  return NULL;
}

int main(int argc, char **argv) {
  if (argc < 4) { fprintf(stderr, "usage: gen_synth kind nbases out [seed]\n"); return 2; }
  int kind = atoi(argv[1]);
  uint64_t n = strtoull(argv[2], NULL, 10);
  uint64_t seed = argc > 4 ? strtoull(argv[4], NULL, 0) : GCZ_SYNTH_SEED;
  char *buf = malloc(n ? n : 1);
  if (!buf) { perror("malloc"); return 1; }
  enum { T = 8 };
  pthread_t th[T];
  job_t jobs[T];
  for (int t = 0; t < T; ++t) {
    jobs[t] = (job_t){buf, kind, seed, n * t / T, n * (t + 1) / T};
    pthread_create(&th[t], NULL, run, &jobs[t]);
  }
  for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);
  FILE *f = fopen(argv[3], "wb");
  if (!f || fwrite(buf, 1, n, f) != n) { perror("write"); return 1; }
  fclose(f);
  free(buf);
  return 0;
}
