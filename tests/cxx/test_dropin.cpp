// C++ drop-in surface tests (include/dna.h, fasta_reader.h, shared_tree.h).
// Mirrors the behaviours the reference's own tests pin (tests/test.cpp:33-409):
// symmetry ops, pointer bits, FASTA reading, canonical invariance, round-trip
// decompression after build / sort / (de)serialization.
//
// usage: test_dropin <golden-dir> [gpu]
//   without "gpu" only host-side groups run (no device needed)
#include <cstdio>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "dna.h"
#include "fasta_reader.h"
#include "shared_tree.h"

static int failures = 0;
#define CHECK(cond, msg)                                                   \
  do {                                                                     \
    if (!(cond)) {                                                         \
      ++failures;                                                          \
      std::cout << "FAIL " << __func__ << ": " << msg << '\n';             \
    }                                                                      \
  } while (0)

static std::string dir;

static void dna_ops() {
  const dna a{std::string_view{"AAAAAAAAAAAA"}};
  const dna t{std::string_view{"TTTTTTTTTTTT"}};
  CHECK(a.transposed() == t, "A transposes to T");
  const dna p{std::string_view{"ACTGACTGACTG"}};
  const dna q{std::string_view{"GTCAGTCAGTCA"}};
  CHECK(p.mirrored() == q, "mirror reverses");
  CHECK(p.inverted() == p.transposed().mirrored(), "inverted = mirrored(transposed)");
  const dna pal{std::string_view{"ACGTTAATTGCA"}};
  CHECK(pal.invariant(), "palindrome is mirror invariant");
  std::ostringstream os;
  os << dna{std::string_view{"acgtrykmbvdh"}};
  CHECK(os.str() == "ACGTRYKMBVDH", "case-insensitive parse + print: " << os.str());
  // canonical is the minimum over the four variants
  const auto [c, m, tr, inv] = p.canonical();
  CHECK(!(p.transposed() < c) && !(p.mirrored() < c) && !(p.inverted() < c) && !(p < c), "canonical is min");
  (void)m; (void)tr; (void)inv;
  std::stringstream ss;
  p.serialize(ss);
  CHECK(dna::deserialize(ss) == p, "dna serialize round trip");
}

static void pointer_ops() {
  const pointer basis{3280, false, false, false};
  CHECK(basis != basis.transposed(), "transposed non-null pointer differs");
  CHECK(basis != basis.mirrored(), "mirrored non-invariant pointer differs");
  CHECK(basis.index() == 3280, "index round trip");
  const pointer inv{7, true, false, true};
  CHECK(!inv.is_mirrored(), "mirror bit cleared for invariant pointers");
  CHECK(inv.mirrored() == inv, "invariant pointer is its own mirror");
  const pointer null{};
  CHECK(null.empty() && null.transposed().empty() && null.inverted().empty(), "null stays null");
  for (std::size_t idx : {0ul, 15ul, 16ul, 4111ul, 4112ul, 1052687ul, 1052688ul, 123456789ul}) {
    const pointer p{idx, bool(idx & 1), bool(idx & 2), false};
    std::stringstream ss;
    p.serialize(ss);
    CHECK(std::size_t(ss.str().size()) == p.bytes(), "bytes() = serialized size");
    CHECK(pointer::deserialize(ss) == p, "pointer round trip " << idx);
  }
  std::stringstream ss;
  null.serialize(ss);
  CHECK(pointer::deserialize(ss).empty(), "null round trip");
}

static void canonical_invariance() {
  const pointer l{0, false, false, false}, r{1, true, false, false};
  const auto a = std::get<0>(node{l, r}.canonical());
  CHECK(a == std::get<0>(a.mirrored().canonical()), "mirror");
  CHECK(a == std::get<0>(a.transposed().canonical()), "transpose");
  CHECK(a == std::get<0>(a.inverted().canonical()), "invert");
}

static void file_reader() {
  // multi-line file with blank lines reads like the single-line original
  fasta_reader edited{dir + "/data/edited"};
  std::ifstream f(dir + "/data/chmpxx", std::ios::binary);
  std::string direct((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  std::vector<dna> buf;
  std::size_t i = 0;
  bool same = true;
  while (edited.read_into(buf))
    for (const auto& b : buf) {
      same &= b == dna{std::string_view{&direct[i * dna::size()], dna::size()}};
      ++i;
    }
  CHECK(same, "edited == chmpxx strand by strand");
  CHECK(i == direct.size() / dna::size(), "strand count " << i);
  CHECK(read_genome(dir + "/data/chmpxx").size() == i, "read_genome");
}

template <class T>
static bool same_sequence(const shared_tree& tree, const T& data) {
  std::size_t i = 0;
  bool ok = true;
  for (auto it = tree.begin(); it != tree.end(); ++it) ok &= i < data.size() && *it == data[i++];
  for (std::size_t k = 0; k < data.size() && ok; k += 97) ok &= tree[k] == data[k];
  return ok && i == data.size();
}

static void gpu_transposition() {
  const auto a = dna::random(0);
  const auto t = a.transposed();
  std::vector<dna> data{a, a, t, a, a, t, t, t};
  shared_tree tree{data};
  CHECK(tree.width() == data.size(), "width");
  CHECK(tree.leaf_count() == 1, "a and its transpose share one leaf");
  CHECK(same_sequence(tree, data), "decompression");
}

static void gpu_frequency_sort() {
  const auto a = dna::random(1), b = dna::random(2), c = dna::random(3);
  std::vector<dna> data;
  for (char x : std::string("bbbacbacbabacacacabcaaaaaaaaaaaaaa")) data.push_back(x == 'a' ? a : x == 'b' ? b : c);
  shared_tree tree{data};
  shared_tree old = tree;
  tree.sort_tree();
  CHECK(same_sequence(tree, data) && same_sequence(old, data), "sort keeps the sequence");
}

static void gpu_file_build() {
  const auto data = read_genome(dir + "/data/chmpxx");
  shared_tree from_vector{const_cast<std::vector<dna>&>(data)};
  shared_tree from_file{std::filesystem::path{dir + "/data/chmpxx"}};
  CHECK(from_vector.width() == data.size(), "width");
  CHECK(same_sequence(from_file, data), "file build decompresses");
  CHECK(same_sequence(from_vector, data), "vector build decompresses");
  std::stringstream a, b;
  from_vector.serialize(a);
  from_file.serialize(b);
  CHECK(a.str() == b.str(), "file and vector builds serialize identically");
  from_file.sort_tree();
  CHECK(from_file.bytes() == 104990, "sorted bytes() = reference 104990, got " << from_file.bytes());
  std::stringstream s;
  from_file.serialize(s);
  auto load = shared_tree::deserialize(s);
  CHECK(load.width() == from_file.width() && load.leaf_count() == from_file.leaf_count(), "deserialize dims");
  CHECK(same_sequence(load, data), "deserialized tree decompresses");
}

// The host copy a device sort defers to the first host read (shared_tree::materialize): every
// way a pending tree can be read, copied, moved, overwritten or outlived by the engine's next
// build gives the sorted tree -- the one the host-only sort of the same build produces.
static void gpu_lazy_sorted_copy() {
  const auto data = read_genome(dir + "/data/hehcmv");
  const auto other = read_genome(dir + "/data/chmpxx");
  auto reference_sorted = [&] {   // the host frequency sort of a copy (no device sort)
    shared_tree t{const_cast<std::vector<dna>&>(data)};
    shared_tree h = t;        // a copy: on the device too, but the sort below is the host's
    shared_tree unrelated{const_cast<std::vector<dna>&>(other)};   // the engine moves on: h is host-only
    h.sort_tree();
    std::stringstream s;
    h.serialize(s);
    return s.str();
  }();
  auto dump = [](const shared_tree& t) {
    std::stringstream s;
    t.serialize(s);
    return s.str();
  };
  {   // read right after the sort (iterator, operator[], access_node via width's traversal)
    shared_tree t{const_cast<std::vector<dna>&>(data)};
    t.sort_tree();
    CHECK(same_sequence(t, data), "pending tree decompresses");
    CHECK(dump(t) == reference_sorted, "pending tree serializes as the host sort");
  }
  {   // the engine's next build copies the pending arrays in first
    shared_tree t{const_cast<std::vector<dna>&>(data)};
    t.sort_tree();
    shared_tree u{const_cast<std::vector<dna>&>(other)};
    CHECK(same_sequence(t, data), "pending tree read after another build");
    CHECK(dump(t) == reference_sorted, "pending tree after another build: sorted contents");
    CHECK(same_sequence(u, other), "the other build");
  }
  {   // moved, then copied, while pending; a pending tree destroyed before the next build
    shared_tree t{const_cast<std::vector<dna>&>(data)};
    t.sort_tree();
    shared_tree m{std::move(t)};
    shared_tree c = m;
    CHECK(dump(c) == reference_sorted, "copy of a moved pending tree");
    CHECK(dump(m) == reference_sorted, "moved pending tree");
    {
      shared_tree gone{const_cast<std::vector<dna>&>(other)};
      gone.sort_tree();
    }
    shared_tree next{const_cast<std::vector<dna>&>(data)};
    CHECK(same_sequence(next, data), "a build after a destroyed pending tree");
  }
  {   // sorted twice on the device, then assigned over while pending
    shared_tree t{const_cast<std::vector<dna>&>(data)};
    t.sort_tree();
    t.sort_tree();
    CHECK(dump(t) == reference_sorted, "sorted twice");
    shared_tree a{const_cast<std::vector<dna>&>(other)};
    a.sort_tree();
    a = shared_tree{const_cast<std::vector<dna>&>(data)};
    CHECK(same_sequence(a, data), "assigned over a pending tree");
    tree_constructor tc{a};
    tc.reduce(data);
    CHECK(same_sequence(a, data), "tree_constructor::reduce into a tree");
  }
}

// fasta_reader's buffer API (include/fasta_reader.h:31-33): load_buffer + read_into
// hand out the same strands as read_genome; swap_buffers exchanges the buffers.
static void buffer_api() {
  const auto path = dir + "/data/chmpxx";
  const auto all = read_genome(path);
  fasta_reader f{path, 1000};
  std::vector<dna> got, buf;
  f.load_buffer();
  CHECK(!f.eof(), "a loaded buffer is not eof");
  while (f.read_into(buf)) {
    CHECK(buf.size() <= 1000, "buffer size bound");
    got.insert(got.end(), buf.begin(), buf.end());
  }
  CHECK(f.eof(), "eof after the last buffer");
  CHECK(got == all, "buffers concatenate to read_genome: " << got.size() << " vs " << all.size());
  fasta_reader g{path, 64};
  g.load_buffer();          // back = strands [0, 64)
  g.swap_buffers();         // front = [0, 64), back empty
  g.load_buffer();          // back = [64, 128)
  std::vector<dna> b;
  CHECK(g.read_into(b) && b.size() == 64 && b.front() == all[64], "read_into after swap_buffers hands out the back buffer");
  g.swap_buffers();         // back = [0, 64) again
  CHECK(g.read_into(b) && b.front() == all[0], "swap_buffers brings the front buffer back");
}

static std::string dump(const shared_tree& t) {
  std::ostringstream os;
  os << t;
  return os.str();
}

// tree_constructor (include/shared_tree.h:245-316): the element-at-a-time members build
// the same DAG as the GPU build, reduce() runs the GPU build into the parent.
static void gpu_tree_constructor() {
  auto data = read_genome(dir + "/data/chmpxx");
  const shared_tree gpu{data};
  shared_tree a;
  tree_constructor ca{a};
  ca.reduce_segment(data);
  const pointer ra = ca.reduce_roots();
  CHECK(ra == gpu.root_pointer(), "element-wise root equals the GPU root");
  CHECK(dump(a) == dump(gpu), "element-wise DAG equals the GPU DAG");
  // segments of 2^12 strands (the last one shorter) then reduce_roots: the reference's
  // segmented build, equal to the global one
  shared_tree b;
  tree_constructor cb{b};
  const std::size_t seg = 4096;
  for (std::size_t i = 0; i < data.size(); i += seg)
    cb.reduce_segment(std::vector<dna>(data.begin() + i, data.begin() + std::min(data.size(), i + seg)));
  CHECK(cb.reduce_roots() == gpu.root_pointer() && dump(b) == dump(gpu), "segmented reduce equals the global build");
  shared_tree c;
  tree_constructor cc{c};
  CHECK(cc.reduce(data) == gpu.root_pointer(), "reduce(data) root");
  CHECK(dump(c) == dump(gpu), "reduce(data) DAG");
  CHECK(c[5000] == data[5000], "reduce(data) tree decompresses");
  shared_tree d;
  tree_constructor cd{d};
  fasta_reader f{dir + "/data/chmpxx"};
  CHECK(cd.reduce(f) == gpu.root_pointer() && dump(d) == dump(gpu), "reduce(fasta_reader)");
}

// fasta_reader{path, B} with B not a power of two: every reader buffer is its own subtree
// (src/shared_tree.cpp:719-736).  The GPU build (shared_tree{reader}, tree_constructor::
// reduce(reader)) equals the element-wise constructor fed buffer by buffer; a reader whose
// first buffers were already read out builds the rest.
static void gpu_reader_segments() {
  for (const std::size_t B : {std::size_t(1000), std::size_t(7), std::size_t(4095)}) {
    shared_tree host;
    tree_constructor ch{host};
    fasta_reader hr{dir + "/data/chmpxx", B};
    std::vector<dna> buf;
    while (hr.read_into(buf)) ch.reduce_segment(buf);
    const pointer root = ch.reduce_roots();
    const shared_tree gpu{fasta_reader{dir + "/data/chmpxx", B}};
    CHECK(gpu.root_pointer() == root && dump(gpu) == dump(host), "shared_tree{fasta_reader{path, B}} = buffer subtrees");
    shared_tree d;
    tree_constructor cd{d};
    fasta_reader f{dir + "/data/chmpxx", B};
    CHECK(cd.reduce(f) == root && dump(d) == dump(host), "tree_constructor::reduce(fasta_reader{path, B})");
  }
  // two buffers handed out before reduce(): the tree of the remaining ones
  const std::size_t B = 1000;
  fasta_reader hr{dir + "/data/chmpxx", B};
  std::vector<dna> buf;
  hr.read_into(buf);
  hr.read_into(buf);
  shared_tree host;
  tree_constructor ch{host};
  while (hr.read_into(buf)) ch.reduce_segment(buf);
  const pointer root = ch.reduce_roots();
  fasta_reader f{dir + "/data/chmpxx", B};
  f.read_into(buf);
  f.read_into(buf);
  shared_tree d;
  tree_constructor cd{d};
  CHECK(cd.reduce(f) == root && dump(d) == dump(host), "reduce(reader) after two read_into calls");
}

// every buffer handed out before reduce(): nothing is left to build (the reference reduces an
// empty root list, undefined); the drop-in prints libgcz's error and exits(1) like its other
// build failures -- run as its own process ("exhausted"), the exit is the expected outcome
static int gpu_reader_exhausted() {
  fasta_reader f{dir + "/data/chmpxx", 1000};
  std::vector<dna> buf;
  while (f.read_into(buf)) {}
  shared_tree d;
  tree_constructor cd{d};
  cd.reduce(f);
  std::cout << "reduce() of an exhausted reader returned\n";
  return 3;
}

int main(int argc, char** argv) {
  dir = argc > 1 ? argv[1] : "tests/golden";
  const bool gpu = argc > 2 && std::string(argv[2]) == "gpu";
  if (argc > 2 && std::string(argv[2]) == "exhausted") return gpu_reader_exhausted();
  dna_ops();
  pointer_ops();
  canonical_invariance();
  file_reader();
  buffer_api();
  if (gpu) {
    gpu_tree_constructor();
    gpu_reader_segments();
    gpu_transposition();
    gpu_frequency_sort();
    gpu_file_build();
    gpu_lazy_sorted_copy();
  }
  std::cout << (failures ? "FAILED " : "OK ") << failures << '\n';
  return failures ? 1 : 0;
}
