// rl_freecache.hpp — a bounded local over-limit cache with freecache's eviction, for
// LOCAL_CACHE_SIZE_IN_BYTES caches too small to hold every over-limit key of a window.
//
// The reference's local cache is github.com/coocood/freecache v1.1.0 (go.mod:9), created with
// freecache.NewCache(LOCAL_CACHE_SIZE_IN_BYTES) (src/service_cmd/runner/runner.go:85-88) and
// used by BaseRateLimiter: Get before a key's INCRBY (base_limiter.go:57-66), Set(key, "",
// TTL = the unit's divider) when the reply passes the limit (base_limiter.go:94-106).
// freecache is not in this image, so this is a restatement of its published algorithm and
// PARITY-UNPINNED:
//   * max(size, 512 KiB) bytes split into 256 segments (xxhash64(key) & 255), each a ring
//     buffer of size/256 bytes; an entry takes 24 B of header + the key + its value capacity
//     (1 B for the empty value); a Set whose entry passes a quarter of the segment is refused;
//   * Get misses when the entry's expireAt <= now (and deletes it), else bumps its accessTime;
//     a Set of a key present overwrites it in place (new TTL and accessTime);
//   * a Set that does not fit evacuates from the ring's oldest end: deleted entries are
//     dropped, an expired entry (expireAt < now) or a least-recently-used one (accessTime *
//     totalCount <= totalTime, the segment's sums over its live ring entries) is evicted, any
//     other entry is moved to the ring's newest end — at most five moves in a row, the sixth
//     oldest entry is evicted regardless.
// freecache stamps entries with its own clock (wall-clock seconds); this model takes the
// request's time (TimeSource.UnixNow), which is the same second in a deployment whose time
// source is the wall clock.
#pragma once
#include <cstdint>
#include <cstring>
#include <list>
#include <string>
#include <unordered_map>
#include <vector>

namespace ratelimit {

// xxHash64 with seed 0 (freecache's hashFunc: cespare/xxhash Sum64).
inline uint64_t xxh64(const void* data, size_t len) {
  constexpr uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                     P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
  auto rotl = [](uint64_t x, int r) { return (x << r) | (x >> (64 - r)); };
  auto rd64 = [](const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; };
  auto rd32 = [](const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; };
  auto round = [&](uint64_t acc, uint64_t in) { return rotl(acc + in * P2, 31) * P1; };
  const uint8_t* p = static_cast<const uint8_t*>(data);
  const uint8_t* const end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
    for (; p + 32 <= end; p += 32) {
      v1 = round(v1, rd64(p));
      v2 = round(v2, rd64(p + 8));
      v3 = round(v3, rd64(p + 16));
      v4 = round(v4, rd64(p + 24));
    }
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    for (uint64_t v : {v1, v2, v3, v4}) h = (h ^ round(0, v)) * P1 + P4;
  } else {
    h = P5;
  }
  h += (uint64_t)len;
  for (; p + 8 <= end; p += 8) h = rotl(h ^ round(0, rd64(p)), 27) * P1 + P4;
  if (p + 4 <= end) {
    h = rotl(h ^ (uint64_t)rd32(p) * P1, 23) * P2 + P3;
    p += 4;
  }
  for (; p < end; ++p) h = rotl(h ^ (uint64_t)*p * P5, 11) * P1;
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

class FreeCacheModel {
 public:
  static constexpr int SEGMENTS = 256;
  static constexpr int64_t MIN_BYTES = 512 * 1024;
  static constexpr int64_t ENTRY_HDR = 24;

  explicit FreeCacheModel(int64_t size_bytes) {
    const int64_t size = size_bytes < MIN_BYTES ? MIN_BYTES : size_bytes;
    for (auto& s : seg_) {
      s.cap = size / SEGMENTS;
      s.vacuum = s.cap;
    }
  }

  // Get(key) == nil error (the value is always empty here). now: unix seconds.
  bool Get(const std::string& key, uint32_t now) {
    Seg& s = seg_[xxh64(key.data(), key.size()) & (SEGMENTS - 1)];
    ++lookups_;
    auto it = s.idx.find(key);
    if (it == s.idx.end()) {
      ++misses_;
      return false;
    }
    Ent& e = *it->second;
    if (e.expire_at != 0 && e.expire_at <= now) {  // expired: deleted, counted a miss
      e.deleted = true;
      s.idx.erase(it);
      ++expired_;
      ++misses_;
      return false;
    }
    s.total_time += (int64_t)(uint32_t)(now - e.access_time);
    e.access_time = now;
    ++hits_;
    return true;
  }

  // Set(key, "", ttl_seconds); false when freecache refuses it (ErrLargeKey / ErrLargeEntry).
  bool Set(const std::string& key, int64_t ttl_seconds, uint32_t now) {
    Seg& s = seg_[xxh64(key.data(), key.size()) & (SEGMENTS - 1)];
    if (key.size() > 65535) return false;
    if ((int64_t)key.size() + ENTRY_HDR > s.cap / 4) return false;
    const uint32_t expire_at = ttl_seconds > 0 ? now + (uint32_t)ttl_seconds : 0u;
    auto it = s.idx.find(key);
    if (it != s.idx.end()) {  // value capacity 1 >= 0: overwritten in place
      Ent& e = *it->second;
      s.total_time += (int64_t)now - (int64_t)e.access_time;
      e.access_time = now;
      e.expire_at = expire_at;
      ++overwrites_;
      return true;
    }
    const int64_t len = ENTRY_HDR + (int64_t)key.size() + 1;
    evacuate(s, len, now);
    s.ring.push_back(Ent{key, now, expire_at, len, false});
    s.idx[key] = std::prev(s.ring.end());
    s.total_time += now;
    s.total_count += 1;
    s.vacuum -= len;
    return true;
  }

  uint64_t entry_count() const {
    uint64_t n = 0;
    for (const auto& s : seg_) n += s.idx.size();
    return n;
  }
  // hits, misses, lookups, live entries, evicted (LRU or forced), expired (at Get or eviction)
  void stats(uint64_t* out) const {
    out[0] = hits_;
    out[1] = misses_;
    out[2] = lookups_;
    out[3] = entry_count();
    out[4] = evacuated_;
    out[5] = expired_;
  }

 private:
  struct Ent {
    std::string key;
    uint32_t access_time, expire_at;
    int64_t len;
    bool deleted;
  };
  struct Seg {
    std::list<Ent> ring;  // oldest first
    std::unordered_map<std::string, std::list<Ent>::iterator> idx;
    int64_t cap = 0, vacuum = 0, total_count = 0, total_time = 0;
  };

  void evacuate(Seg& s, int64_t len, uint32_t now) {
    int moved = 0;
    while (s.vacuum < len) {
      auto it = s.ring.begin();
      Ent& o = *it;
      if (o.deleted) {
        moved = 0;
        s.total_time -= o.access_time;
        s.total_count -= 1;
        s.vacuum += o.len;
        s.ring.erase(it);
        continue;
      }
      const bool expired = o.expire_at != 0 && o.expire_at < now;
      const bool lru = (int64_t)o.access_time * s.total_count <= s.total_time;
      if (expired || lru || moved > 5) {
        moved = 0;
        s.total_time -= o.access_time;
        s.total_count -= 1;
        s.vacuum += o.len;
        if (expired) ++expired_; else ++evacuated_;
        s.idx.erase(o.key);
        s.ring.erase(it);
      } else {  // recently used: moved to the newest end (same bytes, vacuum unchanged)
        s.ring.splice(s.ring.end(), s.ring, it);
        ++moved;
      }
    }
  }

  Seg seg_[SEGMENTS];
  uint64_t hits_ = 0, misses_ = 0, lookups_ = 0, evacuated_ = 0, expired_ = 0, overwrites_ = 0;
};

}  // namespace ratelimit
