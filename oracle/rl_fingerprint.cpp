// rl_fingerprint.cpp — independent restatement of the product's key fingerprint
//  so tests can check the fingerprint kernel bit-for-bit.
// TEST INFRASTRUCTURE ONLY. Decisions in rl_oracle.cpp use exact key strings, never this.
#include <cstring>

#include "rl_oracle.h"

namespace {
inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t fmix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xFF51AFD7ED558CCDull;
  x ^= x >> 33;
  x *= 0xC4CEB9FE1A85EC53ull;
  x ^= x >> 33;
  return x;
}
}  // namespace

// Prefix lanes (a, b) before the window is folded in: also the routed record's key identity.
// Unit-independent: one prefix + window start is one Redis key string whatever the rule.
extern "C" void rlo_prefix_lanes(const uint8_t* prefix, uint32_t len, uint64_t seed, uint64_t* a_out, uint64_t* b_out) {
  uint64_t a = seed ^ 0x9E3779B97F4A7C15ull;
  uint64_t b = (seed + 0xC2B2AE3D27D4EB4Full) ^ ((uint64_t)len << 32);
  for (uint32_t o = 0; o < len; o += 8) {
    uint64_t w = 0;
    for (uint32_t k = 0; k < 8 && o + k < len; ++k) w |= (uint64_t)prefix[o + k] << (8 * k);
    a = rotl((a ^ w) * 0x165667B19E3779F9ull, 31);
    b = (b + w) * 0xD6E8FEB86659FD93ull;
    b ^= b >> 29;
  }
  *a_out = a;
  *b_out = b;
}

// Multi-GPU owner of a key (the product's route_owner): multiply-shift of a lane mix.
extern "C" uint32_t rlo_route_owner(uint64_t a, uint64_t b, uint32_t n_shards) {
  const uint64_t x = fmix(a ^ rotl(b, 29));
  return (uint32_t)(((x >> 32) * (uint64_t)n_shards) >> 32);
}

extern "C" void rlo_fingerprint(const uint8_t* prefix, uint32_t len, uint64_t window_start, uint64_t seed,
                                uint64_t* hi, uint64_t* lo) {
  uint64_t a, b;
  rlo_prefix_lanes(prefix, len, seed, &a, &b);
  a ^= window_start * 0xC2B2AE3D27D4EB4Full;
  b = (b ^ window_start) * 0x165667B19E3779F9ull;
  *hi = fmix(a + rotl(b, 23));
  *lo = fmix(b ^ (a * 0xC4CEB9FE1A85EC53ull)) & 0xFFFFFFFFull;
}

// Home unit of a key string: the largest unit whose divider divides its window start; region
// = (home - 1) * 2 + parity of the home window, gen = home window index + 1.
extern "C" void rlo_place(uint32_t ws, uint32_t* region, uint32_t* gen) {
  const uint32_t home = ws % 86400u == 0 ? 4u : ws % 3600u == 0 ? 3u : ws % 60u == 0 ? 2u : 1u;
  const uint32_t div = home == 4u ? 86400u : home == 3u ? 3600u : home == 2u ? 60u : 1u;
  *region = (home - 1u) * 2u + ((ws / div) & 1u);
  *gen = ws / div + 1u;
}

// Batch form over a prefix blob (test-fixture generation: searching fingerprint collisions).
extern "C" void rlo_fingerprint_many(const uint8_t* blob, const uint32_t* off, uint32_t n, uint64_t window_start,
                                     uint64_t seed, uint64_t* hi, uint64_t* lo) {
  for (uint32_t i = 0; i < n; ++i) rlo_fingerprint(blob + off[i], off[i + 1] - off[i], window_start, seed, hi + i, lo + i);
}
