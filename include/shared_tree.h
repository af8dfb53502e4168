/*
 * shared_tree.h — balanced shared tree (node DAG) built on MI355X.
 *
 * Drop-in for the reference's include/shared_tree.h.  Same classes, names,
 * member functions and semantics:
 *   pointer   29-bit index + mirror/transpose/invariant bits (:36-77); the
 *             in-memory word layout bits 0-28 / 29 / 30 / 31 is also libgcz's
 *   node      two pointers (:99-134)
 *   shared_tree  constructors, accessors, frequency sort, bytes/serialize/
 *             deserialize/save, DFS iterator (:154-237)
 * The construction engine (the reference's tree_constructor, :245-316) is
 * replaced by the libgcz HIP build (include/gcz.h): the constructors hand the
 * genome to the GPU and copy the finished DAG back into the containers.
 *   tree_constructor  the reference's class, same members: reduce() (whole
 *             genomes) runs the HIP build; the element-at-a-time members
 *             (emplace_*, reduce_leaves/nodes/segment/roots) keep the reference's
 *             incremental dictionaries on the host for code that assembles a
 *             tree piece by piece -- they are not the build path.
 *
 * Device selection: GCZ_DEVICE (default 0).  Errors behave like the
 * reference: an unknown nucleotide prints "Encountered unknown symbol: ..."
 * and exits(1); a device failure prints the libgcz error and exits(1).
 * Implementation: genome-compression_amd/csrc/cxx/shared_tree.cpp.
 */
#pragma once

#include <array>
#include <cassert>
#include <cstddef>
#include <cstdint>
#include <filesystem>
#include <iostream>
#include <memory>
#include <new>
#include <tuple>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

#include "dna.h"
#include "fasta_reader.h"
#include "utility.h"   // the reference's shared_tree.h:24 includes it too

class pointer {
 public:
  static constexpr auto address_bits = std::array{4, 12, 20, 28};

  pointer(std::nullptr_t = nullptr) noexcept : word{0x9fffffffu} {}
  pointer(const pointer& other, bool mirror = false, bool transpose = false) noexcept;
  pointer(std::size_t index, bool mirror, bool transpose, bool invariant) noexcept
      : word{std::uint32_t(index) | (std::uint32_t(mirror && !invariant) << 29) | (std::uint32_t(transpose) << 30) |
             (std::uint32_t(invariant) << 31)} {}
  pointer(pointer&&) noexcept = default;
  pointer& operator=(const pointer&) noexcept = default;
  pointer& operator=(pointer&&) noexcept = default;

  static auto from_word(std::uint32_t w) noexcept -> pointer {
    pointer p;
    p.word = w;
    return p;
  }
  auto raw() const noexcept -> std::uint32_t { return word; }

  bool empty() const noexcept { return *this == nullptr; }
  auto canonical() const noexcept { return word & 0x1fffffffu; }
  auto index() const noexcept -> std::size_t {
    assert(!empty());
    return word & 0x1fffffffu;
  }

  bool operator==(const pointer& o) const noexcept { return to_ulong() == o.to_ulong(); }
  bool operator!=(const pointer& o) const noexcept { return to_ulong() != o.to_ulong(); }
  bool operator<(const pointer& o) const noexcept { return to_ulong() < o.to_ulong(); }
  auto to_ulong() const noexcept -> unsigned long { return word & 0x7fffffffu; }
  operator bool() const noexcept { return *this != nullptr; }

  auto bytes() const noexcept -> std::size_t;
  void serialize(std::ostream& os) const;
  static auto deserialize(std::istream& is) -> pointer;

  bool is_mirrored() const noexcept { return (word >> 29) & 1u; }
  bool is_transposed() const noexcept { return (word >> 30) & 1u; }
  bool is_inverted() const noexcept { return is_mirrored() && is_transposed(); }
  bool is_invariant() const noexcept { return word >> 31; }

  auto mirrored() const noexcept { return pointer{*this, true, false}; }
  auto transposed() const noexcept { return pointer{*this, false, true}; }
  auto inverted() const noexcept { return pointer{*this, true, true}; }

 private:
  std::uint32_t word;
};
static_assert(sizeof(pointer) == 4, "pointer is one 32-bit word");

inline auto& operator<<(std::ostream& os, const pointer& p) {
  if (p.empty()) return os << "empty";
  return os << '(' << p.index() << ": " << p.is_mirrored() << p.is_transposed() << p.is_invariant() << ')';
}

namespace std {
template <>
struct hash<pointer> {
  auto operator()(const pointer& p) const noexcept -> std::size_t {
    std::uint64_t x = p.to_ulong() * 0x9E3779B97F4A7C15ull;
    return std::size_t(x ^ (x >> 29));
  }
};
}  // namespace std

class node {
 public:
  node(pointer left, pointer right = nullptr) : children{left, right} {}
  node(const node&) noexcept = default;
  node(node&&) noexcept = default;
  node& operator=(const node&) noexcept = default;
  node& operator=(node&&) noexcept = default;

  bool operator==(const node& o) const noexcept { return children == o.children; }
  bool operator!=(const node& o) const noexcept { return !(*this == o); }
  bool operator<(const node& o) const noexcept { return children < o.children; }

  auto left() const noexcept { return children[0]; }
  auto right() const noexcept { return children[1]; }

  auto mirrored() const noexcept { return node{children[1].mirrored(), children[0].mirrored()}; }
  auto transposed() const noexcept { return node{children[0].transposed(), children[1].transposed()}; }
  auto inverted() const noexcept { return node{children[1].inverted(), children[0].inverted()}; }
  auto canonical() const noexcept -> std::tuple<node, bool, bool>;

  auto bytes() const noexcept { return left().bytes() + right().bytes(); }
  void serialize(std::ostream& os) const;
  static auto deserialize(std::istream& is) -> node;

 private:
  std::array<pointer, 2> children;
};
static_assert(sizeof(node) == 8, "node is two 32-bit words");

inline auto& operator<<(std::ostream& os, const node& n) {
  return os << "node<" << n.left() << ", " << n.right() << '>';
}

namespace std {
template <>
struct hash<node> {
  auto operator()(const node& n) const noexcept -> std::size_t {
    auto h = std::hash<pointer>();
    return 5 * h(n.left()) + 3 * h(n.right());
  }
};
}  // namespace std

// Allocator of the tree's containers: resize() without a value leaves the
// elements (plain 32/64-bit words with trivial destructors) uninitialised,
// because a device copy or a full permutation fills them right after -- 0.6 GB
// of value-initialisation and page faults otherwise; large arrays are huge-page
// mappings (gcz_host_alloc, include/gcz.h).
extern "C" void* gcz_host_alloc(std::uint64_t bytes);              // libgcz (include/gcz.h)
extern "C" void gcz_host_free(void* p, std::uint64_t bytes);

template <class T>
struct gcz_uninit_allocator : std::allocator<T> {
  template <class U>
  struct rebind {
    using other = gcz_uninit_allocator<U>;
  };
  gcz_uninit_allocator() = default;
  template <class U>
  gcz_uninit_allocator(const gcz_uninit_allocator<U>&) noexcept {}
  T* allocate(std::size_t n) {   // (the C entry point returns nullptr; the container throws)
    void* p = gcz_host_alloc(n * sizeof(T));
    if (!p) throw std::bad_alloc();
    return static_cast<T*>(p);
  }
  void deallocate(T* p, std::size_t n) noexcept { gcz_host_free(p, n * sizeof(T)); }
  template <class U>
  void construct(U*) noexcept {
    static_assert(std::is_trivially_destructible_v<U> && std::is_standard_layout_v<U>,
                  "uninitialised construction needs a plain word type");
  }
  template <class U, class... A>
  void construct(U* p, A&&... a) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
};

// The sorted arrays of a device sort, not yet copied into a tree's containers (shared_tree.cpp).
struct gcz_lazy_copy;

class shared_tree {
 public:
  shared_tree() = default;
  // (explicit for the lazy host copy after a device sort: a copy reads the sorted arrays first, a
  // destroyed or overwritten tree cancels its pending copy)
  ~shared_tree();
  shared_tree(const shared_tree& other);
  shared_tree(shared_tree&& other) noexcept;
  auto operator=(const shared_tree& other) -> shared_tree&;
  auto operator=(shared_tree&& other) noexcept -> shared_tree&;
  shared_tree(std::filesystem::path path);
  shared_tree(fasta_reader file, bool verbose = false);
  shared_tree(std::vector<dna>& data, bool verbose = false);

  auto depth() const { return nodes.size() + 1; }
  auto width() const -> std::size_t;

  auto children(std::size_t layer, pointer p) const -> std::size_t;
  auto node_count() const -> std::size_t;
  auto node_count(std::size_t layer) const { return nodes[layer].size(); }
  auto leaf_count() const noexcept { return leaves.size(); }

  auto access_leaf(pointer p) const -> dna;
  auto access_node(std::size_t layer, pointer p) const -> node {
    materialize();
    return nodes[layer][p.index()];
  }
  auto operator[](std::uint64_t index) const -> dna;

  void add_layer() {
    materialize();   // (a pending copy's destination must not move)
    nodes.emplace_back();
  }
  void emplace_node(std::size_t layer, node n) {
    materialize();
    nodes[layer].emplace_back(n);
  }
  void emplace_leaf(dna leaf) {
    materialize();
    leaves.emplace_back(leaf);
  }

  auto histogram(std::size_t layer) const -> std::vector<std::size_t>;
  void store_histogram(std::filesystem::path) const;

  void rewire_nodes(std::size_t layer, const std::vector<std::size_t>& indices);
  void sort_leaves();
  void sort_nodes(std::size_t layer);
  void sort_tree(bool verbose = false);

  auto bytes() const noexcept -> std::size_t;
  void serialize(std::ostream& os) const;
  static auto deserialize(std::istream& is) -> shared_tree;
  void save(std::filesystem::path) const;

  auto root_pointer() const noexcept -> pointer { return root; }

  friend inline auto operator<<(std::ostream& os, const shared_tree& tree) -> std::ostream&;

  struct iterator {
    struct status {
      status(std::size_t layer, pointer current) : layer{layer}, current{current} {}
      std::size_t layer;  // leaf level is the maximum std::size_t value
      pointer current;
    };

    iterator(const shared_tree& nodes, std::size_t layer, pointer root);

    auto operator*() const noexcept -> dna;
    auto operator++() -> iterator&;
    auto operator!=(const iterator&) const { return !stack.empty(); }
    void next_leaf();

    const shared_tree& parent;
    std::vector<status> stack;
  };
  using const_iterator = iterator;

  auto begin() const { return iterator{*this, nodes.size() - 1, root}; }
  auto end() const { return iterator{*this, 0, nullptr}; }

 private:
  friend class tree_constructor;
  friend auto shared_tree_on_gpus(const std::filesystem::path& path, int gpus) -> shared_tree;
  void build_from_gpu();   // copies the last libgcz build of this thread into the containers
  bool on_device() const;  // the engine's device arrays still hold exactly this tree
  // After a device sort the containers keep their sizes but not yet the sorted contents: those
  // stay in HBM (compress writes its .dag from there and never reads them on the host) and are
  // copied in by the first host read (materialize), or before the engine's next build or sort.
  std::shared_ptr<gcz_lazy_copy> lazy;
  void materialize() const;
  void drop_lazy();        // the containers are about to be replaced: no copy

  using layer_vector = std::vector<node, gcz_uninit_allocator<node>>;
  using leaf_vector = std::vector<dna, gcz_uninit_allocator<dna>>;
  std::vector<layer_vector> nodes;
  leaf_vector leaves;
  pointer root;
  std::uint64_t device_gen = 0;   // engine build generation mirrored here (0: host only)
};

inline auto operator<<(std::ostream& os, const shared_tree& tree) -> std::ostream& {
  tree.materialize();
  os << "Leaves (" << tree.leaves.size() << "):";
  for (const auto& leaf : tree.leaves) os << ' ' << leaf;
  os << '\n';
  for (const auto& layer : tree.nodes) {
    os << "Layer (" << layer.size() << "):";
    for (const auto& n : layer) os << ' ' << n;
    os << '\n';
  }
  return os;
}

/* Beyond the reference surface (compress --gpus=N): the construction of a FASTA file
 * spread over `gpus` devices GCZ_DEVICE .. GCZ_DEVICE + gpus - 1, one process per GPU
 * (this process and gpus - 1 children forked before any device work), strand ranges per
 * rank and owner-hashed exchanges over RCCL; the slices meet in
 * shared memory and the result equals shared_tree{path}.  GCZ_MULTI_TRANSPORT=shm runs
 * every rank on GCZ_DEVICE with host-staged exchanges (testing on one GPU). */
auto shared_tree_on_gpus(const std::filesystem::path& path, int gpus) -> shared_tree;

/******************************************************************************
 * tree_constructor (reference include/shared_tree.h:245-316, src/shared_tree.cpp:617-763).
 *
 * reduce(data) / reduce(file): the whole genome through the libgcz HIP build; the
 * parent receives the finished DAG (leaves, layers, root) and the root is returned.
 * It expects a constructor that has not emplaced anything yet (as the shared_tree
 * constructors use it); the GPU build is global, which equals the reference's
 * segmented reduce for its power-of-two segments.
 *
 * The element-at-a-time members keep the reference's dictionaries on the host:
 * emplace_leaf / emplace_leaves / emplace_node hash-cons one element (first
 * occurrence = next index of the parent's layer), reduce_leaves / reduce_nodes
 * pair up one layer, reduce_segment reduces a segment to one root, reduce_roots
 * combines the roots.  Same results as the reference's, element for element.
 */
class tree_constructor {
 public:
  tree_constructor(shared_tree& parent);

  auto emplace_node(std::size_t layer_index, pointer left, pointer right = nullptr) -> pointer;
  auto emplace_leaves(dna left, dna right) -> pointer;
  auto emplace_leaves(dna last) -> pointer;
  auto emplace_leaf(dna leaf) -> pointer;

  template <typename Iterable>
  auto reduce_leaves(Iterable&& layer) -> std::vector<pointer>;
  auto reduce_nodes(const std::vector<pointer>& segment, std::size_t index) -> std::vector<pointer>;
  auto reduce_roots(bool verbose = false) -> pointer;
  auto reduce(const std::vector<dna>& data, bool verbose = false) -> pointer;
  auto reduce(fasta_reader& file, bool verbose = false) -> pointer;

  template <typename Iterable>
  void reduce_segment(Iterable&& layer);

 private:
  shared_tree& parent;
  std::vector<std::unordered_map<node, std::size_t>> nodes;
  std::unordered_map<dna, std::size_t> leaves;
  std::vector<pointer> roots;
};

// reduce_leaves (src/shared_tree.h:287-302): pairs of strands -> layer-0 pointers
// (foreach_pair, include/utility.h:17-29: an odd last strand pairs with null)
template <typename Iterable>
auto tree_constructor::reduce_leaves(Iterable&& iterable) -> std::vector<pointer> {
  auto layer = std::vector<pointer>{};
  const std::size_t n = std::size(iterable);
  layer.reserve(n / 2 + n % 2);
  if (parent.depth() == 1) {
    parent.add_layer();
    nodes.emplace_back();
  }
  auto it = std::begin(iterable);
  for (std::size_t i = 0; i + 1 < n; i += 2) {
    const dna left = *it++;
    const dna right = *it++;
    layer.emplace_back(emplace_leaves(left, right));
  }
  if (n % 2) layer.emplace_back(emplace_leaves(dna{*it}));
  return layer;
}

// reduce_segment (:308-319): a segment down to one root, appended to the roots
template <typename Iterable>
void tree_constructor::reduce_segment(Iterable&& segment) {
  auto layer = reduce_leaves(segment);
  for (auto index = 1u; layer.size() > 1 || index < nodes.size(); ++index) layer = reduce_nodes(layer, index);
  roots.emplace_back(layer.front());
}
