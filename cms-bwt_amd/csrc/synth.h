// synth.h — deterministic synthetic DNA workload.
//
// Counter-based: every byte is a pure function of (seed, stream, index), so
// the host generator (tools/gen_synth, tests) and the on-device generator
// used by bench.py produce byte-identical collections without sharing state.
//
//   reference  : ref[k]      = "ACGT"[h(seed, 0, k) >> 62]
//   copy c>=1  : u = h(seed, c, k); if (u >> 11) < p * 2^53 the base at k is
//                replaced by one of the other three: (b + 1 + (u & 0x7ff) % 3) & 3
//
// FASTA layout: ">ref\n<seq>\n" and ">copy_c\n<seq>\n" x C,
// single-line sequences unless a line width is given.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SYNTH_HD __host__ __device__ __forceinline__
#else
#define SYNTH_HD static inline
#endif

SYNTH_HD uint64_t synth_mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

SYNTH_HD uint64_t synth_hash(uint64_t seed, uint64_t stream, uint64_t k) {
  return synth_mix64(synth_mix64(seed + 0xD1B54A32D192ED03ull * (stream + 1)) ^ k);
}

SYNTH_HD uint8_t synth_base_code(uint64_t seed, uint64_t k) {
  return (uint8_t)(synth_hash(seed, 0, k) >> 62);
}

// p_threshold = (uint64_t)(p * 2^53)
SYNTH_HD uint8_t synth_copy_code(uint64_t seed, uint64_t copy, uint64_t k,
                                 uint64_t p_threshold) {
  uint8_t b = synth_base_code(seed, k);
  uint64_t u = synth_hash(seed, copy, k);
  if ((u >> 11) < p_threshold) b = (uint8_t)((b + 1 + (u & 0x7ff) % 3) & 3);
  return b;
}

SYNTH_HD char synth_acgt(uint8_t code) {
  return code == 0 ? 'A' : code == 1 ? 'C' : code == 2 ? 'G' : 'T';
}

static inline uint64_t synth_threshold(double p) {
  if (p <= 0) return 0;
  if (p >= 1) return (1ull << 53);
  return (uint64_t)(p * 9007199254740992.0);
}
