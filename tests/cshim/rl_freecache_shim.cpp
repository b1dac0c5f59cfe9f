// rl_freecache_shim.cpp — ctypes access to the host freecache model (api-ratelimit_amd/csrc/
// rl_freecache.hpp, HIP_LOCAL_CACHE=freecache) for tests/test_freecache_model.py. Test
// infrastructure only; host code, no GPU.
#include <string>

#include "rl_freecache.hpp"

using ratelimit::FreeCacheModel;

extern "C" {
void* fcm_create(int64_t bytes) { return new FreeCacheModel(bytes); }
void fcm_destroy(void* p) { delete static_cast<FreeCacheModel*>(p); }
int fcm_get(void* p, const char* key, uint32_t len, uint32_t now) {
  return static_cast<FreeCacheModel*>(p)->Get(std::string(key, len), now) ? 1 : 0;
}
int fcm_set(void* p, const char* key, uint32_t len, int64_t ttl, uint32_t now) {
  return static_cast<FreeCacheModel*>(p)->Set(std::string(key, len), ttl, now) ? 1 : 0;
}
void fcm_stats(void* p, uint64_t* out) { static_cast<FreeCacheModel*>(p)->stats(out); }
uint64_t fcm_xxh64(const char* data, uint32_t len) { return ratelimit::xxh64(data, len); }
}
