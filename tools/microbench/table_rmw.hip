// Random-access roofline microbenchmarks for the counter table (MI355X / gfx950).
//
// Measures, on a table of 32-B slots resident in HBM:
//   (1) streaming copy bandwidth (float4),
//   (2) U random 32-B slot read-modify-writes by plain load + plain store,
//   (3) U random 64-bit atomicCAS on slot ctrl words,
//   (4) U random 64-bit atomicAdd (returning) on slot counters,
//   (5) (2) again with the slot indices sorted ascending (the order the leader
//       pass visits the table after the radix sort).
// Output: one line per test, "name ns_per_launch G_ops_per_s GB_per_s".
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

struct __attribute__((aligned(16))) Slot { uint64_t ctrl, fp, cnt, misc; };

__global__ void k_copy(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) b[i] = a[i];
}

__global__ void k_rmw(Slot* t, const uint32_t* __restrict__ idx, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Slot* s = t + idx[i];
  uint4 lo = *reinterpret_cast<const uint4*>(s);
  uint4 hi = *(reinterpret_cast<const uint4*>(s) + 1);
  hi.x += 1u; lo.y ^= i;
  *reinterpret_cast<uint4*>(s) = lo;
  *(reinterpret_cast<uint4*>(s) + 1) = hi;
}

__global__ void k_cas(Slot* t, const uint32_t* __restrict__ idx, uint32_t n, uint64_t* sink) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Slot* s = t + idx[i];
  unsigned long long old = atomicCAS((unsigned long long*)&s->ctrl, 0ull, (unsigned long long)(i + 1));
  if (old == 0xdeadbeefull) sink[0] = old;
}

__global__ void k_add(Slot* t, const uint32_t* __restrict__ idx, uint32_t n, uint64_t* sink) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Slot* s = t + idx[i];
  unsigned long long old = atomicAdd((unsigned long long*)&s->cnt, 1ull);
  if (old == 0xdeadbeefull) sink[0] = old;
}

__global__ void k_probe_read(const Slot* __restrict__ t, const uint32_t* __restrict__ idx, uint32_t n, uint64_t* sink) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Slot* s = t + idx[i];
  uint4 lo = *reinterpret_cast<const uint4*>(s);
  if (lo.x == 0xdeadbeefu) sink[0] = lo.y;
}

static uint64_t sm(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <class F>
static float time_it(F f, int reps) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  int log2slots = argc > 1 ? atoi(argv[1]) : 25;
  uint32_t U = argc > 2 ? (uint32_t)atoi(argv[2]) : 632000;
  size_t S = (size_t)1 << log2slots;
  Slot* t; CK(hipMalloc(&t, S * sizeof(Slot))); CK(hipMemset(t, 0, S * sizeof(Slot)));
  uint64_t* sink; CK(hipMalloc(&sink, 64));
  std::vector<uint32_t> h(U); uint64_t x = 12345;
  for (uint32_t i = 0; i < U; ++i) h[i] = (uint32_t)(sm(x) & (S - 1));
  uint32_t* d; CK(hipMalloc(&d, U * 4)); CK(hipMemcpy(d, h.data(), U * 4, hipMemcpyHostToDevice));
  std::vector<uint32_t> hs = h; std::sort(hs.begin(), hs.end());
  uint32_t* ds; CK(hipMalloc(&ds, U * 4)); CK(hipMemcpy(ds, hs.data(), U * 4, hipMemcpyHostToDevice));

  size_t nb = (size_t)1 << 30;  // 1 GiB copy
  float4 *ca, *cb; CK(hipMalloc(&ca, nb)); CK(hipMalloc(&cb, nb)); CK(hipMemset(ca, 1, nb));
  int reps = 20;
  float ms = time_it([&] { k_copy<<<2048 * 4, 256>>>(ca, cb, nb / 16); }, 5);
  printf("copy_1GiB %.1f us  %.0f GB/s\n", ms * 1e3, 2.0 * nb / (ms * 1e-3) / 1e9);
  dim3 g((U + 255) / 256);
  auto rep = [&](const char* nm, float m, double bytes_per) {
    printf("%-22s %8.2f us  %7.2f Gops/s  %7.1f GB/s(algo %g B/op)\n", nm, m * 1e3, U / (m * 1e-3) / 1e9,
           U * bytes_per / (m * 1e-3) / 1e9, bytes_per);
  };
  rep("probe_read_random", time_it([&] { k_probe_read<<<g, 256>>>(t, d, U, sink); }, reps), 32);
  rep("rmw32_random", time_it([&] { k_rmw<<<g, 256>>>(t, d, U); }, reps), 64);
  rep("rmw32_sorted", time_it([&] { k_rmw<<<g, 256>>>(t, ds, U); }, reps), 64);
  CK(hipMemset(t, 0, S * sizeof(Slot)));
  rep("cas64_random", time_it([&] { k_cas<<<g, 256>>>(t, d, U, sink); }, reps), 8);
  rep("cas64_sorted", time_it([&] { k_cas<<<g, 256>>>(t, ds, U, sink); }, reps), 8);
  rep("atomadd64_random", time_it([&] { k_add<<<g, 256>>>(t, d, U, sink); }, reps), 8);
  rep("atomadd64_sorted", time_it([&] { k_add<<<g, 256>>>(t, ds, U, sink); }, reps), 8);
  printf("table_bytes %zu U %u\n", S * sizeof(Slot), U);
  return 0;
}
