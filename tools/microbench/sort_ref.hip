// Reference timing of rocPRIM's tuned radix sort on the batch shape (tooling only:
// a yardstick for the hand-written sort in api-ratelimit_amd/csrc, never linked into it).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 1000000;
  std::vector<uint64_t> hk(n); std::vector<uint32_t> hv(n);
  uint64_t x = 7;
  for (int i = 0; i < n; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; hk[i] = x; hv[i] = i; }
  uint64_t *k0, *k1; uint32_t *v0, *v1;
  CK(hipMalloc(&k0, n * 8)); CK(hipMalloc(&k1, n * 8)); CK(hipMalloc(&v0, n * 4)); CK(hipMalloc(&v1, n * 4));
  CK(hipMemcpy(k0, hk.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(v0, hv.data(), n * 4, hipMemcpyHostToDevice));
  for (int bits : {64, 48, 32}) {
    size_t tmp = 0; void* dt = nullptr;
    CK(hipcub::DeviceRadixSort::SortPairs(dt, tmp, k0, k1, v0, v1, n, 64 - bits, 64));
    CK(hipMalloc(&dt, tmp));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipcub::DeviceRadixSort::SortPairs(dt, tmp, k0, k1, v0, v1, n, 64 - bits, 64));
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < 20; ++r) CK(hipcub::DeviceRadixSort::SortPairs(dt, tmp, k0, k1, v0, v1, n, 64 - bits, 64));
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b));
    printf("hipcub_sortpairs n=%d bits=%d  %.2f us\n", n, bits, ms * 1e3 / 20);
    CK(hipFree(dt));
  }
  return 0;
}
