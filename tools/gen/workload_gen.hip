// workload_gen.hip — device-side generator of BASELINE config-2/3 batches for bench.py
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

// mode 0: Zipf ranks (config 3: rule = rank % 3); mode 1: uniform ranks (config 2: rule 0).
__global__ void k_keys(ZipfC z, int mode, uint64_t ctr0, uint64_t mult, uint32_t n, uint64_t* __restrict__ key,
                       uint32_t* __restrict__ rule, uint32_t* __restrict__ len) {
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
  rule[i] = mode == 1 ? 0u : (uint32_t)(rank % 3);
  len[i] = 8u + ndigits(kv) + 1u;  // "bench_k_" + decimal + "_"
}

__global__ void k_bytes(uint32_t n, const uint64_t* __restrict__ key, const uint32_t* __restrict__ off,
                        uint8_t* __restrict__ blob, uint32_t* __restrict__ req_of) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint8_t* p = blob + off[i];
  const char pre[8] = {'b', 'e', 'n', 'c', 'h', '_', 'k', '_'};
  for (int k = 0; k < 8; ++k) p[k] = (uint8_t)pre[k];
  uint64_t v = key[i];
  const uint32_t nd = off[i + 1] - off[i] - 9u;
  for (int k = (int)nd - 1; k >= 0; --k) {
    p[8 + k] = (uint8_t)('0' + v % 10);
    v /= 10;
  }
  p[8 + nd] = '_';
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
                     rule, len);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Prefix bytes at the given offsets (off[n + 1], exclusive scan of the lengths) and req_of = i.
int rlw_bytes(uint32_t n, const uint64_t* key, const uint32_t* off, uint8_t* blob, uint32_t* req_of,
              void* hip_stream) {
  hipLaunchKernelGGL(k_bytes, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)hip_stream, n, key, off, blob, req_of);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
