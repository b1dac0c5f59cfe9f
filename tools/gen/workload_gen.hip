// workload_gen.hip — device-side generator of BASELINE config-2/3/4/5 batches for bench.py
// (measurement tooling, not product; SURVEY.md §8d workload definitions).
//
// The same construction as api-ratelimit_amd/workload.py — bounded Zipf(s) ranks by
// rejection-inversion (Hörmann & Derflinger 1996) from a counter-based splitmix64 stream,
// ranks through the fixed bijective permutation rank*a + 0x2545F491 mod N, rule = rank % 3,
// key prefix "bench_k_<decimal key>_" — so the bench can run the thousands of distinct
// 1e6-descriptor batches one second of traffic holds without generating them on the host.
// The draws are not bit-identical to numpy's (independent retries per descriptor, device
// libm), only identically distributed; parity tests use workload.py's host batches.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ double u01(uint64_t x) { return (double)(splitmix64(x) >> 11) * (1.0 / 9007199254740992.0); }

struct ZipfC {
  double s, hx1, hN, sq;
  uint64_t N;
};
__device__ __forceinline__ double zh(const ZipfC& z, double x) { return exp(-z.s * log(x)); }
__device__ __forceinline__ double zH(const ZipfC& z, double x) {
  const double lx = log(x), t = (1.0 - z.s) * lx;
  return lx * (fabs(t) > 1e-8 ? expm1(t) / t : 1.0 + t / 2.0);
}
__device__ __forceinline__ double zHinv(const ZipfC& z, double x) {
  double t = x * (1.0 - z.s);
  t = t > -1.0 + 1e-16 ? t : -1.0 + 1e-16;
  return exp((fabs(t) > 1e-8 ? log1p(t) / t : 1.0 - t / 2.0) * x);
}

__device__ __forceinline__ uint32_t ndigits(uint64_t v) {
  uint32_t d = 1;
  while (v >= 10) {
    v /= 10;
    ++d;
  }
  return d;
}

// mode 0: Zipf ranks (config 3: rule = rank % 3); mode 1: uniform ranks (config 2: rule 0);
// mode 2: Zipf ranks, rule = rank % 3, and hits_addend ~ U{1..8} per request (config 5); mode 3:
// Zipf ranks of config 4's 4-entry descriptors (no rule: the device resolves it). plen: the
// prefix's length before the key's decimal digits.
__global__ void k_keys(ZipfC z, int mode, uint64_t ctr0, uint64_t mult, uint32_t n, uint64_t* __restrict__ key,
                       uint32_t* __restrict__ rule, uint32_t* __restrict__ len, uint32_t* __restrict__ hits,
                       uint32_t plen) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t rank = 0;
  if (mode == 1) {
    rank = (uint64_t)(u01(ctr0 + i) * (double)z.N);
    if (rank >= z.N) rank = z.N - 1;
  } else {
    for (uint32_t a = 0;; ++a) {
      const double u = z.hN + u01(ctr0 + (uint64_t)a * 0x100000000ull + i) * (z.hx1 - z.hN);
      const double x = zHinv(z, u);
      double k = floor(x + 0.5);
      k = k < 1.0 ? 1.0 : (k > (double)z.N ? (double)z.N : k);
      if (k - x <= z.sq || u >= zH(z, k + 0.5) - zh(z, k) || a >= 64) {
        rank = (uint64_t)k - 1;
        break;
      }
    }
  }
  const uint64_t kv = (rank * mult + 0x2545F491ull) % z.N;  // rank, mult < 2^32: no overflow
  key[i] = kv;
  if (mode == 3) {  // "bench4_a_<d0>_b_<d1>_c_<d2>_d_<kv / 1000>_"
    len[i] = 22u + ndigits(kv / 1000u);
    return;
  }
  rule[i] = mode == 1 ? 0u : (uint32_t)(rank % 3);
  len[i] = plen + ndigits(kv) + 1u;  // prefix + decimal + "_"
  if (mode == 2 && hits) hits[i] = (uint32_t)(splitmix64(ctr0 ^ 0x5A5A5A5A00000000ull ^ i) % 8u) + 1u;
}

struct Prefix {
  char p[16];
  uint32_t n;
};
// Config 4 (BASELINE: 1e9 keys, nested 4-entry descriptors resolved by the tree): the key's
// digits pick the entries' values, so the tree's key/value nodes (values 0..5) and its
// key-only defaults are both taken; the prefix bytes double as the resolve batch's strings:
// domain "bench4" and each entry's key and value are ranges of the prefix.
__global__ void k_bytes4(uint32_t n, const uint64_t* __restrict__ key, const uint32_t* __restrict__ off,
                         uint8_t* __restrict__ blob, uint32_t* __restrict__ req_of, uint32_t* __restrict__ domain,
                         uint32_t* __restrict__ entry_first, uint32_t* __restrict__ entry) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i > n) return;
  entry_first[i] = 4u * i;
  if (i == n) return;
  const uint32_t o = off[i];
  uint8_t* p = blob + o;
  const char pre[7] = {'b', 'e', 'n', 'c', 'h', '4', '_'};
  for (int k = 0; k < 7; ++k) p[k] = (uint8_t)pre[k];
  const uint64_t kv = key[i];
  const uint32_t dg[3] = {(uint32_t)(kv % 10u), (uint32_t)(kv / 10u % 10u), (uint32_t)(kv / 100u % 10u)};
  const char names[4] = {'a', 'b', 'c', 'd'};
  for (int e = 0; e < 3; ++e) {
    p[7 + 4 * e] = (uint8_t)names[e];
    p[8 + 4 * e] = '_';
    p[9 + 4 * e] = (uint8_t)('0' + dg[e]);
    p[10 + 4 * e] = '_';
  }
  p[19] = 'd';
  p[20] = '_';
  uint64_t v = kv / 1000u;
  const uint32_t nd = off[i + 1] - o - 22u;
  for (int k = (int)nd - 1; k >= 0; --k) {
    p[21 + k] = (uint8_t)('0' + v % 10);
    v /= 10;
  }
  p[21 + nd] = '_';
  req_of[i] = i;
  domain[2 * i] = o;
  domain[2 * i + 1] = 6u;
  for (int e = 0; e < 4; ++e) {
    uint32_t* x = entry + 16u * i + 4u * e;
    x[0] = o + 7u + 4u * e;  // key
    x[1] = 1u;
    x[2] = o + 9u + 4u * e;  // value
    x[3] = e < 3 ? 1u : nd;
  }
}

__global__ void k_bytes(uint32_t n, const uint64_t* __restrict__ key, const uint32_t* __restrict__ off,
                        uint8_t* __restrict__ blob, uint32_t* __restrict__ req_of, Prefix pre) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t* p = blob + off[i];
  for (uint32_t k = 0; k < pre.n; ++k) p[k] = (uint8_t)pre.p[k];
  uint64_t v = key[i];
  const uint32_t nd = off[i + 1] - off[i] - pre.n - 1u;
  for (int k = (int)nd - 1; k >= 0; --k) {
    p[pre.n + k] = (uint8_t)('0' + v % 10);
    v /= 10;
  }
  p[pre.n + nd] = '_';
  req_of[i] = i;
}

}  // namespace

extern "C" {

// Keys, rules and prefix lengths of one batch. stream = batch index (counter stream).
int rlw_keys(int mode, uint64_t N, double s, double hx1, double hN, double sq, uint64_t seed, uint64_t stream,
             uint64_t mult, uint32_t n, uint64_t* key, uint32_t* rule, uint32_t* len, void* hip_stream) {
  ZipfC z{s, hx1, hN, sq, N};
  const uint64_t ctr0 = ((seed * 1000003ull + stream) & 0xFFFFFFull) << 40;
  hipLaunchKernelGGL(k_keys, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)hip_stream, z, mode, ctr0, mult, n, key,
                     rule, len, (uint32_t*)nullptr, 8u);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
// The same with the per-request hits (mode 2) and the prefix length before the digits.
int rlw_keys2(int mode, uint64_t N, double s, double hx1, double hN, double sq, uint64_t seed, uint64_t stream,
              uint64_t mult, uint32_t n, uint64_t* key, uint32_t* rule, uint32_t* len, uint32_t* hits,
              uint32_t plen, void* hip_stream) {
  ZipfC z{s, hx1, hN, sq, N};
  const uint64_t ctr0 = ((seed * 1000003ull + stream) & 0xFFFFFFull) << 40;
  hipLaunchKernelGGL(k_keys, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)hip_stream, z, mode, ctr0, mult, n, key,
                     rule, len, hits, plen);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Prefix bytes at the given offsets (off[n + 1], exclusive scan of the lengths) and req_of = i.
int rlw_bytes(uint32_t n, const uint64_t* key, const uint32_t* off, uint8_t* blob, uint32_t* req_of,
              void* hip_stream) {
  Prefix pre{{'b', 'e', 'n', 'c', 'h', '_', 'k', '_'}, 8u};
  hipLaunchKernelGGL(k_bytes, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)hip_stream, n, key, off, blob, req_of,
                     pre);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int rlw_bytes2(uint32_t n, const uint64_t* key, const uint32_t* off, uint8_t* blob, uint32_t* req_of,
               const char* prefix, uint32_t plen, void* hip_stream) {
  Prefix pre{};
  if (plen > sizeof pre.p) return -1;
  for (uint32_t k = 0; k < plen; ++k) pre.p[k] = prefix[k];
  pre.n = plen;
  hipLaunchKernelGGL(k_bytes, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)hip_stream, n, key, off, blob, req_of,
                     pre);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
// Config 4: prefix bytes, req_of, and the resolve batch's domain / entry_first / entry arrays.
int rlw_bytes4(uint32_t n, const uint64_t* key, const uint32_t* off, uint8_t* blob, uint32_t* req_of,
               uint32_t* domain, uint32_t* entry_first, uint32_t* entry, void* hip_stream) {
  hipLaunchKernelGGL(k_bytes4, dim3((n + 256) / 256), dim3(256), 0, (hipStream_t)hip_stream, n, key, off, blob, req_of,
                     domain, entry_first, entry);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
