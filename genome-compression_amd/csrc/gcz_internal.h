// Internal definitions shared by the libgcz translation units.
#pragma once

#include <cstdint>
#include <vector>

#define GCZ_BUILDING 1
#include "../../include/gcz.h"

namespace gcz {

constexpr uint32_t kNullWord = 0x9fffffffu;   // pointer(nullptr), src/shared_tree.cpp:96-97
constexpr uint32_t kNullIndex = 0x1fffffffu;
constexpr uint32_t kIndexMask = 0x1fffffffu;
constexpr uint32_t kFlagMask = 0xe0000000u;

inline uint32_t ul(uint32_t w) { return w & 0x7fffffffu; }   // pointer::to_ulong, :103-107

}  // namespace gcz

// Host-resident shared tree: the three members of the reference's shared_tree
// (include/shared_tree.h:221-223) in the raw word layout.
struct gcz_tree {
  int L = 12;
  std::vector<uint64_t> leaves;
  std::vector<std::vector<uint32_t>> layers;   // 2 words (left,right) per node
  uint32_t root = gcz::kNullWord;
};
