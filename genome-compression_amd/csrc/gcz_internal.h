// Internal definitions shared by the libgcz translation units.
#pragma once

#include <cstddef>
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

// Data bytes per fasta_reader buffer (src/fasta_reader.cpp:22-31): the buffer
// holds min(file_size/L + 1, buffer_strands) strands; 0 = default 1 << 22
// (include/fasta_reader.h:23).
inline uint64_t reader_buffer_bytes(uint64_t file_size, int L, uint64_t buffer_strands) {
  if (!buffer_strands) buffer_strands = uint64_t(1) << 22;
  const uint64_t fs = file_size / uint64_t(L) + 1;
  return (fs < buffer_strands ? fs : buffer_strands) * uint64_t(L);
}

}  // namespace gcz

namespace gcz {
// Raw view of a shared tree (used by both the C ABI's gcz_tree and the C++
// shared_tree): leaves, per-layer node words (2 per node), root.
struct TreeView {
  int L = 12;
  uint64_t* leaves = nullptr;
  size_t n_leaves = 0;
  std::vector<uint32_t*> layer;
  std::vector<size_t> layer_n;
  uint32_t root = kNullWord;
};
void view_sort(TreeView& t);
uint64_t view_bytes(const TreeView& t);
uint64_t view_serialize(const TreeView& t, uint8_t* buf, uint64_t cap);
uint64_t view_width(const TreeView& t);
}  // namespace gcz

// Host-resident shared tree: the three members of the reference's shared_tree
// (include/shared_tree.h:221-223) in the raw word layout.
struct gcz_tree {
  int L = 12;
  std::vector<uint64_t> leaves;
  std::vector<std::vector<uint32_t>> layers;   // 2 words (left,right) per node
  uint32_t root = gcz::kNullWord;
};
