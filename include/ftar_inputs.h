/*
 * ftar_inputs.h — portable seeded synthetic inputs (header-only, C/C++).
 *
 * One generator shared by the oracle, the reference golden driver, the
 * product benchmark and the Python tests (tests/ftar_inputs.py mirrors it in
 * numpy), so every consumer sees bit-identical buffers for (seed, stream).
 * splitmix64 -> fp32 uniform in [-1, 1); bf16 by RNE from it.
 *
 *   mix(z)        = splitmix64 finaliser
 *   state(seed,s) = mix(seed ^ (0xD1B54A32D192ED03 * (s + 1)))
 *   next()        = mix(state += 0x9E3779B97F4A7C15)
 *   f32           = ((z >> 40) - 2^23) * 2^-23          exact, in [-1, 1)
 *   f64           = ((z >> 11) - 2^52) * 2^-52          exact, in [-1, 1)
 *   bf16          = round-to-nearest-even(f32)
 *   bool          = z >> 63
 *   integer types = low bytes of z
 */
#ifndef FTAR_INPUTS_H
#define FTAR_INPUTS_H

#include <stdint.h>
#include <stddef.h>
#include <string.h>

enum {
  FTI_U8 = 0, FTI_I8 = 1, FTI_U16 = 2, FTI_I16 = 3, FTI_I32 = 4, FTI_I64 = 5,
  FTI_F32 = 6, FTI_F64 = 7, FTI_BOOL = 8, FTI_BF16 = 9
};

static inline size_t fti_dtype_size(int dt) {
  static const size_t sz[] = {1, 1, 2, 2, 4, 8, 4, 8, 1, 2};
  return (dt >= 0 && dt <= 9) ? sz[dt] : 0;
}

static inline uint64_t fti_mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static inline uint16_t fti_f32_to_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

/* Fill n elements of dtype dt for stream `stream` (e.g. the rank) of `seed`. */
static inline void fti_fill(int dt, uint64_t seed, uint64_t stream, void* out, size_t n) {
  uint64_t st = fti_mix(seed ^ (0xD1B54A32D192ED03ull * (stream + 1)));
  for (size_t i = 0; i < n; ++i) {
    st += 0x9E3779B97F4A7C15ull;
    uint64_t z = fti_mix(st);
    switch (dt) {
      case FTI_U8: case FTI_I8: ((uint8_t*)out)[i] = (uint8_t)z; break;
      case FTI_U16: case FTI_I16: ((uint16_t*)out)[i] = (uint16_t)z; break;
      case FTI_I32: ((uint32_t*)out)[i] = (uint32_t)z; break;
      case FTI_I64: ((uint64_t*)out)[i] = z; break;
      case FTI_F32: ((float*)out)[i] = (float)((int64_t)(z >> 40) - (1ll << 23)) * (1.0f / 8388608.0f); break;
      case FTI_F64: ((double*)out)[i] = (double)((int64_t)(z >> 11) - (1ll << 52)) * (1.0 / 4503599627370496.0); break;
      case FTI_BOOL: ((uint8_t*)out)[i] = (uint8_t)(z >> 63); break;
      case FTI_BF16: {
        float f = (float)((int64_t)(z >> 40) - (1ll << 23)) * (1.0f / 8388608.0f);
        ((uint16_t*)out)[i] = fti_f32_to_bf16(f);
        break;
      }
    }
  }
}

#endif /* FTAR_INPUTS_H */
