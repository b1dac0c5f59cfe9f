// rl_resolve.h — device layout of the descriptor tree (GetLimit, rl_resolve.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "rl_hip.h"

namespace rlhip {

constexpr uint32_t TREE_EMPTY = 0xFFFFFFFFu;  // empty edge-table slot (node id half)
constexpr uint32_t TREE_NONE = 0xFFFFFFFFu;   // lookup miss
constexpr int TREE_INLINE = 32;               // name bytes held in the node itself
constexpr int TREE_PROBE = 4;                 // edge slots read per probe round (one round trip)

// 64 B: the header and the first TREE_INLINE name bytes arrive in one load pair, so a lookup
// whose name fits compares it without a third round trip.
struct __attribute__((aligned(64))) TreeNodeDev {
  uint32_t parent;      // node id or RL_TREE_ROOT (a domain)
  uint32_t name_len;    // map key: domain name, or finalKey = key["_" value]
  uint32_t rule;        // rule id of the node's limit, RL_NIL_RULE if none
  uint32_t n_children;  // len(descriptors) (config_impl.go:320)
  uint32_t hash;        // tree_hash(parent, fold(name))
  uint32_t name_off;    // the whole name in the names blob (bytes past TREE_INLINE)
  uint32_t pad[2];
  uint32_t name[TREE_INLINE / 4];  // first bytes of the name, little-endian, zero-padded
};
static_assert(sizeof(TreeNodeDev) == 64, "tree node layout");

// The first pass's copy of the tree (k_resolve): nodes renumbered breadth-first so that a
// node's children have consecutive ids, and each node carries its children's edge hashes, so
// ONE 64-B load of a node both confirms it (parent, name) and looks the next level's names up
// among its children. A node with more than FAST_CHILDREN children, or two children whose hashes
// are equal, keeps its children in the fast edge table instead (FAST_OVERFLOW), as the domains
// (the root's children) always are.
constexpr int FAST_CHILDREN = 8;
constexpr uint32_t FAST_OVERFLOW = 0x80000000u;  // len_flags: children in the fast edge table
constexpr uint32_t FAST_NO_CHILD = 0xFFFFFFFFu;  // chash of an unused child slot (fast hashes are even)
struct __attribute__((aligned(64))) FastNode {
  uint32_t parent;       // fast id of the parent, or RL_TREE_ROOT
  uint32_t len_flags;    // name length (low 24 bits, saturated), FAST_OVERFLOW
  uint32_t rule;         // RL_NIL_RULE if none
  uint32_t first_child;  // fast id of child 0 (children k = first_child + k)
  uint32_t name[4];      // first 16 name bytes, little-endian, zero-padded
  uint32_t chash[FAST_CHILDREN];  // fast_hash(this id, child k's name), or FAST_NO_CHILD
};
static_assert(sizeof(FastNode) == 64, "fast node layout");

struct TreeDesc2 {
  const TreeNodeDev* nodes;
  const uint64_t* slots;  // (parent, name) edge table: hash << 32 | node id, or ~0; mask + TREE_PROBE entries
                          // (the first TREE_PROBE - 1 repeated at the end, so a probe round never wraps)
  const uint8_t* names;
  uint32_t mask;          // power-of-two table size - 1 (load <= 1/8)
  // the first pass's tree (fast ids; same edge-table layout over fast_hash, for the domains and
  // the children of overflow nodes)
  const FastNode* fnodes;
  const uint64_t* fslots;
  uint32_t fmask, n_fnodes;
};

struct ResolveIn {
  uint32_t n_desc, n_entries, bytes_len;
  const uint8_t* bytes;
  const uint32_t* domain;         // [2 n_desc] (off, len)
  const uint32_t* entry_first;    // [n_desc + 1]
  const uint32_t* entry;          // [4 n_entries] (key off, key len, value off, value len)
  const uint32_t* override_rule;  // [n_desc] or null
};

// The name folded four bytes at a time (little-endian words, the last one zero-padded), then
// the length and the parent and an avalanche: a name's fold does not depend on where in the
// tree it is looked up, and a word step is a few instructions where a byte step was one per
// byte. Host and device agree.
constexpr uint32_t TREE_FOLD0 = 2166136261u;
__host__ __device__ inline uint32_t tree_fold_word(uint32_t h, uint32_t w) {
  h ^= w;
  h = (h << 13) | (h >> 19);
  return h * 0x85EBCA77u + 0xC2B2AE3Du;
}
__host__ __device__ inline uint32_t tree_hash(uint32_t parent, uint32_t fold, uint32_t len) {
  uint32_t h = fold ^ (parent * 0x9E3779B1u + 0x7F4A7C15u) ^ (len * 0x27D4EB2Fu);
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  h *= 0x297A2D39u;
  h ^= h >> 15;
  return h;
}

int build_tree(const rl_tree_node* nodes, uint32_t n, const uint8_t* names, uint32_t names_len,
               std::vector<TreeNodeDev>& out_nodes, std::vector<uint64_t>& out_slots, uint32_t& mask, std::string& err);
// The edge hash of the first pass's tree: tree_hash over fast ids, bit 0 clear (so no hash equals
// FAST_NO_CHILD or the slots' empty word).
__host__ __device__ inline uint32_t fast_hash(uint32_t parent, uint32_t fold, uint32_t len) {
  return tree_hash(parent, fold, len) & ~1u;
}
// The first pass's tree from build_tree's nodes (and fast_id[original id] = fast id, for tests).
void build_fast_tree(const std::vector<TreeNodeDev>& nodes, const uint8_t* names, std::vector<FastNode>& out_nodes,
                     std::vector<uint64_t>& out_slots, uint32_t& mask, std::vector<uint32_t>* fast_id = nullptr);
// Two launches: the level-pipelined walk, then the exact walk for the descriptors it leaves
// (flags: resolve_flag_words(n_desc) words of scratch, never holding `seq` (non-zero, this
// launch's number) before the launch: zeroed once, then numbered launches).
void launch_resolve(hipStream_t st, const ResolveIn& in, const TreeDesc2& t, uint32_t* rule_out, uint32_t* flags,
                    uint32_t seq);
uint32_t resolve_flag_words(uint32_t n_desc);
// k_resolve's code on the host (tests/cshim): both passes, *exact = the exact walk decided
uint32_t resolve_one_host(const ResolveIn& in, const TreeDesc2& t, uint32_t i, bool* exact = nullptr);
uint32_t resolve_exact_host(const ResolveIn& in, const TreeDesc2& t, uint32_t i);

}  // namespace rlhip
