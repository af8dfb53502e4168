/*
 * Synthetic genome generator shared by the bench, the tests and the oracle
 * harness.  Deterministic and random-access: any byte range can be produced
 * independently, so hosts fill large genomes in parallel and the GPU box
 * regenerates exactly the bytes the goldens were computed on.
 *
 *  kind 0 (uniform): base j = "acgt"[(splitmix64_at(seed, j/32) >> 2*(j%32)) & 3]
 *  kind 1 (tandem):  alternating regions of U[1000, 100000] bases; each region
 *                    is, with probability 1/2, a tandem repeat of a random ACGT
 *                    unit of period U[2, 200], otherwise uniform (the uniform
 *                    bytes of kind 0 at the same absolute positions).
 *
 * SURVEY.md §8(d) configs 4 and 5.  Plain C so that C, C++ and HIP hosts can
 * include it.
 */
#ifndef GCZ_SYNTH_H
#define GCZ_SYNTH_H

#include <stdint.h>

#define GCZ_SYNTH_SEED (0x9E3779B97F4A7C15ull ^ 42ull)
#define GCZ_GAMMA 0x9E3779B97F4A7C15ull

static inline uint64_t gcz_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* i-th output of a splitmix64 stream started at `seed` (0-based). */
static inline uint64_t gcz_splitmix_at(uint64_t seed, uint64_t i) {
  return gcz_mix64(seed + (i + 1) * GCZ_GAMMA);
}

static inline char gcz_uniform_base(uint64_t seed, uint64_t j) {
  return "acgt"[(gcz_splitmix_at(seed, j >> 5) >> (2 * (j & 31))) & 3];
}

static inline void gcz_synth_uniform(char *out, uint64_t seed, uint64_t begin, uint64_t end) {
  uint64_t j = begin;
  while (j < end) {
    uint64_t x = gcz_splitmix_at(seed, j >> 5) >> (2 * (j & 31));
    uint64_t stop = ((j >> 5) + 1) << 5;
    if (stop > end) stop = end;
    for (; j < stop; ++j, x >>= 2) out[j - begin] = "acgt"[x & 3];
  }
}

/* Region walk for kind 1: calls fill for every region overlapping [begin,end). */
static inline void gcz_synth_tandem(char *out, uint64_t seed, uint64_t begin, uint64_t end) {
  uint64_t rs = seed ^ 0xA5A5A5A5A5A5A5A5ull;  /* region stream */
  uint64_t ri = 0, start = 0;
  while (start < end) {
    uint64_t len = 1000 + gcz_splitmix_at(rs, ri++) % 99001;
    uint64_t kind = gcz_splitmix_at(rs, ri++) & 1;
    uint64_t period = 2 + gcz_splitmix_at(rs, ri++) % 199;
    uint64_t useed = gcz_splitmix_at(rs, ri++);
    uint64_t stop = start + len;
    if (stop > begin) {
      uint64_t a = start > begin ? start : begin;
      uint64_t b = stop < end ? stop : end;
      if (kind == 0) {
        gcz_synth_uniform(out + (a - begin), seed, a, b);
      } else {
        char unit[200];
        gcz_synth_uniform(unit, useed, 0, period);
        for (uint64_t j = a; j < b; ++j) out[j - begin] = unit[(j - start) % period];
      }
    }
    start = stop;
  }
}

static inline void gcz_synth_fill_range(char *out, int kind, uint64_t seed, uint64_t begin, uint64_t end) {
  if (kind == 1) gcz_synth_tandem(out, seed, begin, end);
  else gcz_synth_uniform(out, seed, begin, end);
}

#endif
