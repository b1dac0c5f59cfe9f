// rl_resolve.h — device layout of the descriptor tree (GetLimit, rl_resolve.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "rl_hip.h"

namespace rlhip {

constexpr uint32_t TREE_EMPTY = 0xFFFFFFFFu;  // empty edge-table slot
constexpr uint32_t TREE_NONE = 0xFFFFFFFFu;   // lookup miss

struct TreeNodeDev {
  uint32_t parent;      // node id or RL_TREE_ROOT (a domain)
  uint32_t name_off;    // map key: domain name, or finalKey = key["_" value]
  uint32_t name_len;
  uint32_t rule;        // rule id of the node's limit, RL_NIL_RULE if none
  uint32_t n_children;  // len(descriptors) (config_impl.go:320)
  uint32_t hash;        // tree_hash(parent, name)
  uint32_t pad[2];
};
static_assert(sizeof(TreeNodeDev) == 32, "tree node layout");

struct TreeDesc2 {
  const TreeNodeDev* nodes;
  const uint32_t* slots;  // (parent, name) edge table: node id or TREE_EMPTY
  const uint8_t* names;
  uint32_t mask;          // slots - 1 (power of two)
};

struct ResolveIn {
  uint32_t n_desc;
  const uint8_t* bytes;
  const uint32_t* domain;         // [2 n_desc] (off, len)
  const uint32_t* entry_first;    // [n_desc + 1]
  const uint32_t* entry;          // [4 n_entries] (key off, key len, value off, value len)
  const uint32_t* override_rule;  // [n_desc] or null
};

// FNV-1a over (parent, name bytes) with a final avalanche; host and device agree.
__host__ __device__ inline uint32_t tree_hash_init(uint32_t parent) { return 2166136261u ^ (parent * 0x9E3779B1u); }
__host__ __device__ inline uint32_t tree_hash_step(uint32_t h, uint32_t byte) { return (h ^ byte) * 16777619u; }
__host__ __device__ inline uint32_t tree_hash_final(uint32_t h) {
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  h *= 0x297A2D39u;
  h ^= h >> 15;
  return h;
}

int build_tree(const rl_tree_node* nodes, uint32_t n, const uint8_t* names, uint32_t names_len,
               std::vector<TreeNodeDev>& out_nodes, std::vector<uint32_t>& out_slots, std::string& err);
void launch_resolve(hipStream_t st, const ResolveIn& in, const TreeDesc2& t, uint32_t* rule_out);

}  // namespace rlhip
