// Host-side paths of the drop-in surface, for the sanitizer builds (Makefile.san):
// FASTA reading, the element-at-a-time tree_constructor, the host frequency sort,
// bytes(), serialize / save / deserialize and decompression -- no device involved.
//
// usage: test_host <fasta> <out.dag> [L]
//   writes the sorted .dag of <fasta> to <out.dag> (the caller compares its sha256
//   with the reference golden) and checks round trips on the way.
#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "dna.h"
#include "fasta_reader.h"
#include "gcz.h"
#include "shared_tree.h"

static int failures = 0;
#define CHECK(cond, msg)                                   \
  do {                                                     \
    if (!(cond)) {                                         \
      ++failures;                                          \
      std::cout << "FAIL: " << msg << '\n';                \
    }                                                      \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 3) {
    std::cerr << "usage: test_host <fasta> <out.dag> [L]\n";
    return 2;
  }
  if (argc > 3) dna::size(std::size_t(std::atoi(argv[3])));
  const std::string path = argv[1];
  const auto genome = read_genome(path);
  // the host extractor behind fasta_reader equals the C-ABI one
  {
    std::ifstream f(path, std::ios::binary);
    std::vector<std::uint8_t> raw((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    std::vector<std::uint8_t> bases(raw.size() + 1);
    const auto nb = gcz_fasta_extract(raw.data(), raw.size(), int(dna::size()), 0, bases.data());
    CHECK(nb / dna::size() == genome.size(), "gcz_fasta_extract strand count");
  }
  // element-at-a-time construction in 2^22-strand segments (tree_constructor::reduce(fasta_reader&))
  shared_tree tree;
  tree_constructor c{tree};
  const std::size_t seg = std::size_t(1) << 22;
  for (std::size_t i = 0; i < genome.size(); i += seg)
    c.reduce_segment(std::vector<dna>(genome.begin() + i, genome.begin() + std::min(genome.size(), i + seg)));
  const pointer root = c.reduce_roots();
  CHECK(root == tree.root_pointer(), "reduce_roots sets the tree root");
  for (std::size_t i = 0; i < genome.size(); i += 997) CHECK(tree[i] == genome[i], "decompression at " << i);
  tree.sort_tree();
  for (std::size_t i = 0; i < genome.size(); i += 991) CHECK(tree[i] == genome[i], "decompression after sort at " << i);
  std::ostringstream a;
  tree.serialize(a);
  CHECK(a.str().size() == tree.bytes(), "bytes() equals the serialized size");
  std::istringstream in(a.str());
  const auto back = shared_tree::deserialize(in);
  std::ostringstream b;
  back.serialize(b);
  CHECK(a.str() == b.str(), "deserialize + serialize round trip");
  gcz_tree* t = gcz_tree_new();
  CHECK(gcz_tree_deserialize(t, int(dna::size()), reinterpret_cast<const std::uint8_t*>(a.str().data()), a.str().size()) ==
            GCZ_OK,
        "C-ABI deserialize");
  std::vector<std::uint8_t> buf(a.str().size());
  CHECK(gcz_tree_serialize(t, buf.data(), buf.size()) == buf.size() && std::string(buf.begin(), buf.end()) == a.str(),
        "C-ABI serialize round trip");
  gcz_tree_free(t);
  tree.save(argv[2]);
  std::cout << (failures ? "FAILED " : "OK ") << failures << '\n';
  return failures ? 1 : 0;
}
