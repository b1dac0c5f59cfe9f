// Roofline denominators of SURVEY.md §8d, measured on the box bench.py runs on
// (measurement tooling: loaded by bench.py, never by the product path).
//   streaming: 1 GiB device copy (float4, grid-stride) -> read+write GB/s
//   random:    U random 32-B slot RMWs (two 16-B loads + one returning 64-bit atomicAdd on
//              the slot's counter) on a table of the engine's size -> slot RMWs/s
// t_roof = streaming_bytes / copy_GBps + U / rmw_rate (bench.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

namespace {
struct __attribute__((aligned(16))) Slot { uint64_t ctrl, key, lo, cnt; };

__global__ void k_copy(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) b[i] = a[i];
}

__global__ void k_slot_rmw(Slot* t, size_t mask, uint32_t n, uint64_t seed, uint64_t* sink) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t z = seed + (uint64_t)i * 0x9E3779B97F4A7C15ull;  // splitmix64 slot index
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  Slot* s = t + (z & mask);
  const uint4 lo = *reinterpret_cast<const uint4*>(s);
  const uint4 hi = *(reinterpret_cast<const uint4*>(s) + 1);
  const unsigned long long old = atomicAdd(reinterpret_cast<unsigned long long*>(&s->cnt), 1ull);
  if ((old ^ lo.x ^ hi.y) == 0xdeadbeefcafeull) sink[0] = old;
}

template <class F>
float best_ms(F f, int reps) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < reps; ++r) {
    hipEventRecord(a);
    f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    best = std::min(best, ms);
  }
  hipEventDestroy(a);
  hipEventDestroy(b);
  return best;
}
}  // namespace

// Returns 0 on success. table_slots is rounded down to a power of two.
extern "C" int rl_probe_roofline(uint64_t table_slots, uint32_t U, double* copy_gbs, double* rmw_per_s,
                                 double* rmw_us) {
  size_t S = 1;
  while (S * 2 <= table_slots) S *= 2;
  const size_t nb = (size_t)1 << 30;
  float4 *ca = nullptr, *cb = nullptr;
  Slot* t = nullptr;
  uint64_t* sink = nullptr;
  if (hipMalloc(&ca, nb) != hipSuccess || hipMalloc(&cb, nb) != hipSuccess ||
      hipMalloc(&t, S * sizeof(Slot)) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess)
    return -1;
  hipMemset(ca, 1, nb);
  hipMemset(t, 0, S * sizeof(Slot));
  const float cms = best_ms([&] { hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, ca, cb, nb / 16); }, 10);
  *copy_gbs = 2.0 * nb / (cms * 1e-3) / 1e9;
  uint64_t seed = 1;
  const float rms = best_ms(
      [&] {
        hipLaunchKernelGGL(k_slot_rmw, dim3((U + 255) / 256), dim3(256), 0, 0, t, S - 1, U, seed, sink);
        seed += 0x1234567ull;  // fresh slots each rep: no L2 reuse across reps
      },
      20);
  *rmw_us = rms * 1e3;
  *rmw_per_s = U / (rms * 1e-3);
  hipFree(ca);
  hipFree(cb);
  hipFree(t);
  hipFree(sink);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}
