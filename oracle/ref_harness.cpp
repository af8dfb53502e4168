// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// Harness around the *compiled reference* (Quinten-van-Woerkom/genome-compression,
// sources under /root/reference, built by oracle/Makefile into oracle/_ref/).
// It is our own driver code: it includes the reference's headers and links the
// reference's src/*.cpp unmodified, and dumps what the reference computes so the
// C restatement (oracle/gcz_oracle.c) and the MI355X path can be pinned to it.
//
// Modes
//   dump <fasta> <L> <prefix>        shared_tree{fasta_reader{path}} (compress.cpp:183)
//   dumpleaves <u64.bin> <L> <prefix> shared_tree(std::vector<dna>&)  (shared_tree.cpp:212)
//   dumpbuf <fasta> <L> <buffer> <prefix>  shared_tree{fasta_reader{path, buffer}}: the tree of
//                                    reader buffers of `buffer` strands (shared_tree.cpp:719-736)
//   time <kind> <nbases> <L> [reps]  synthetic genome (csrc/synth.h) -> vector<dna> -> build
//   random <seed>                    prints dna::random(seed) (dna.cpp:92-96) as u64
//   reader <fasta> <L> <buffer> <out> fasta_reader{path, buffer} (fasta_reader.cpp:13-35) read_into
//                                    loop (:92-106): u64 strands to out, one u64 buffer size per
//                                    read_into call to out.bufs (pins the per-buffer line contract)
//
// dump outputs (all little-endian):
//   prefix.leaves.bin   u64 per leaf (first-occurrence order, before sort)
//   prefix.layers.bin   per layer: u64 count, then count x (u32 left, u32 right) raw
//                       words incl. the invariant bit 31 (layout SURVEY §8 notation)
//   prefix.unsorted.dag shared_tree::serialize before sort_tree
//   prefix.dag          shared_tree::serialize after sort_tree  (== compress output)
//   prefix.json         counts, root word, width, bytes
#include <algorithm>
#include <array>
#include <cassert>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <filesystem>
#include <fstream>
#include <functional>
#include <future>
#include <iostream>
#include <limits>
#include <memory>
#include <mutex>
#include <new>
#include <numeric>
#include <random>
#include <sstream>
#include <string>
#include <string_view>
#include <thread>
#include <tuple>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

#include "robin_hood.h"
#include "parallel_hashmap/phmap.h"

// shared_tree keeps nodes/leaves/root private (shared_tree.h:220-223); the dump
// needs the raw words including the in-memory-only invariant bit.
#define private public
#include "shared_tree.h"
#include "dna.h"
#include "fasta_reader.h"
#undef private

#include "../genome-compression_amd/csrc/synth.h"

// fasta_reader::load_buffer passes getline a count of char_buffer.size() - position + 1
// (fasta_reader.cpp:52), so a getline that fills the buffer stores its '\0' one byte past
// the vector.  At the default 2^22-strand buffer that byte lands in the slack of the
// page-rounded mmap chunk; at the small buffer sizes the reader tests use, it lands in
// the next heap chunk's header.  Every allocation gets 16 bytes of slack so the
// reference's behaviour is defined at every buffer size (the reference is unmodified).
void* operator new(std::size_t n) {
  if (void* p = std::malloc(n + 16)) return p;
  throw std::bad_alloc{};
}
void operator delete(void* p) noexcept { std::free(p); }
void operator delete(void* p, std::size_t) noexcept { std::free(p); }

static uint32_t word(const pointer& p) {
  return (uint32_t)p.data | ((uint32_t)p.mirror << 29) | ((uint32_t)p.transpose << 30) |
         ((uint32_t)p.invariant << 31);
}

static void dump_tree(shared_tree& tree, const std::string& prefix, std::uintmax_t file_size,
                      double build_ms) {
  {
    std::ofstream f(prefix + ".leaves.bin", std::ios::binary);
    for (const auto& l : tree.leaves) {
      uint64_t v = l.to_ullong();
      f.write((const char*)&v, 8);
    }
  }
  {
    std::ofstream f(prefix + ".layers.bin", std::ios::binary);
    for (const auto& layer : tree.nodes) {
      uint64_t n = layer.size();
      f.write((const char*)&n, 8);
      for (const auto& nd : layer) {
        uint32_t w[2] = {word(nd.left()), word(nd.right())};
        f.write((const char*)w, 8);
      }
    }
  }
  {
    std::ofstream f(prefix + ".unsorted.dag", std::ios::binary);
    tree.serialize(f);
  }
  const auto width = tree.width();
  const auto unsorted_bytes = tree.bytes();
  tree.sort_tree();
  {
    std::ofstream f(prefix + ".dag", std::ios::binary);
    tree.serialize(f);
  }
  const auto bytes = tree.bytes();
  std::ostringstream ratio;
  ratio << double(file_size) / double(bytes);   // compress.cpp:74 formatting
  std::ofstream j(prefix + ".json");
  j << "{\"L\": " << dna::size() << ", \"width\": " << width << ", \"depth\": " << tree.depth()
    << ", \"n_leaves\": " << tree.leaf_count() << ", \"n_nodes\": " << tree.node_count()
    << ", \"root\": " << word(tree.root) << ", \"bytes\": " << bytes
    << ", \"unsorted_bytes\": " << unsorted_bytes << ", \"file_size\": " << file_size
    << ", \"ratio\": \"" << ratio.str() << "\", \"build_ms\": " << build_ms << ", \"layer_sizes\": [";
  for (size_t i = 0; i < tree.nodes.size(); ++i) j << (i ? ", " : "") << tree.nodes[i].size();
  j << "]}\n";
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::cerr << "usage: ref_harness dump|dumpleaves|time|random ...\n";
    return 2;
  }
  std::string mode = argv[1];
  if (mode == "dump" && argc == 5) {
    dna::size(std::atoi(argv[3]));
    auto t0 = std::chrono::high_resolution_clock::now();
    shared_tree tree{std::filesystem::path{argv[2]}};
    auto t1 = std::chrono::high_resolution_clock::now();
    dump_tree(tree, argv[4], std::filesystem::file_size(argv[2]),
              std::chrono::duration<double, std::milli>(t1 - t0).count());
    return 0;
  }
  if (mode == "dumpbuf" && argc == 6) {
    dna::size(std::atoi(argv[3]));
    auto t0 = std::chrono::high_resolution_clock::now();
    shared_tree tree{fasta_reader{std::filesystem::path{argv[2]}, std::strtoull(argv[4], nullptr, 10)}};
    auto t1 = std::chrono::high_resolution_clock::now();
    dump_tree(tree, argv[5], std::filesystem::file_size(argv[2]),
              std::chrono::duration<double, std::milli>(t1 - t0).count());
    return 0;
  }
  if (mode == "dumpleaves" && argc == 5) {
    dna::size(std::atoi(argv[3]));
    std::ifstream f(argv[2], std::ios::binary);
    std::vector<dna> data;
    uint64_t v;
    while (f.read((char*)&v, 8)) data.emplace_back(dna{(unsigned long long)v});
    auto t0 = std::chrono::high_resolution_clock::now();
    shared_tree tree{data};
    auto t1 = std::chrono::high_resolution_clock::now();
    dump_tree(tree, argv[4], 8 * data.size(), std::chrono::duration<double, std::milli>(t1 - t0).count());
    return 0;
  }
  if (mode == "time" && argc >= 5) {
    // CPU baseline: reference pack (dna ctor, dna.cpp:79-84) + build (shared_tree.cpp:212-215)
    int kind = std::atoi(argv[2]);
    uint64_t nbases = std::strtoull(argv[3], nullptr, 10);
    dna::size(std::atoi(argv[4]));
    int reps = argc > 5 ? std::atoi(argv[5]) : 1;
    std::vector<char> ascii(nbases);
    gcz_synth_fill_range(ascii.data(), kind, GCZ_SYNTH_SEED, 0, nbases);
    const uint64_t L = dna::size();
    const uint64_t S = nbases / L;
    double best_pack = 1e30, best_build = 1e30;
    uint64_t nodes = 0, leaves = 0;
    for (int r = 0; r < reps; ++r) {
      auto t0 = std::chrono::high_resolution_clock::now();
      std::vector<dna> data;
      data.reserve(S);
      for (uint64_t i = 0; i < S; ++i) data.emplace_back(dna{std::string_view{&ascii[i * L], L}});
      auto t1 = std::chrono::high_resolution_clock::now();
      shared_tree tree{data};
      auto t2 = std::chrono::high_resolution_clock::now();
      best_pack = std::min(best_pack, std::chrono::duration<double, std::milli>(t1 - t0).count());
      best_build = std::min(best_build, std::chrono::duration<double, std::milli>(t2 - t1).count());
      nodes = tree.node_count();
      leaves = tree.leaf_count();
    }
    double bases = double(S * L);
    std::printf("{\"bases\": %.0f, \"pack_ms\": %.3f, \"build_ms\": %.3f, \"bases_per_s\": %.6e, "
                "\"n_leaves\": %llu, \"n_nodes\": %llu, \"threads\": 1}\n",
                bases, best_pack, best_build, bases / ((best_pack + best_build) * 1e-3),
                (unsigned long long)leaves, (unsigned long long)nodes);
    return 0;
  }
  if (mode == "reader" && argc == 6) {
    dna::size(std::atoi(argv[3]));
    fasta_reader file{std::filesystem::path{argv[2]}, std::strtoull(argv[4], nullptr, 10)};
    std::ofstream f(argv[5], std::ios::binary), fb(std::string(argv[5]) + ".bufs", std::ios::binary);
    std::vector<dna> buffer;
    while (file.read_into(buffer)) {
      uint64_t n = buffer.size();
      fb.write((const char*)&n, 8);
      for (const auto& d : buffer) {
        uint64_t v = d.to_ullong();
        f.write((const char*)&v, 8);
      }
    }
    return 0;
  }
  if (mode == "random" && argc == 3) {
    std::printf("%llu\n", (unsigned long long)dna::random(std::atoi(argv[2])).to_ullong());
    return 0;
  }
  std::cerr << "bad arguments\n";
  return 2;
}
