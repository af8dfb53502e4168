// shared_tree container (include/shared_tree.h) on top of libgcz.
// Construction: the HIP build (gcz_build.hip) replaces tree_constructor
// (reference src/shared_tree.cpp:621-763); everything after the build restates
// the reference container: pointer compression :25-67,122-163, node :169-196,
// access/indexing :231-291, histogram/sort :316-483, bytes/serialize/deserialize
// :488-546, iterator :553-614.
#include "shared_tree.h"

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <mutex>
#include <numeric>
#include <sstream>
#include <thread>

#include <signal.h>
#include <sys/mman.h>
#include <sys/prctl.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <string_view>

#include "gcz.h"
#include "../gcz_internal.h"

namespace {

// One libgcz context per process (device GCZ_DEVICE, default 0), created on
// first use.  Builds are serialised, matching the reference's single build thread.
std::atomic<bool> engine_alive{false};

struct Engine {
  gcz_ctx* ctx = nullptr;
  std::mutex mu;
  std::uint64_t gen = 0;   // generation of the tree the device arrays hold (bumped by builds and device sorts)
  // the device sort whose sorted arrays no tree has copied in yet (at most one: the device holds one tree)
  std::shared_ptr<gcz_lazy_copy> pending;
  Engine() {
    const char* d = std::getenv("GCZ_DEVICE");
    const int rc = gcz_ctx_create(d ? std::atoi(d) : 0, &ctx);
    if (rc != GCZ_OK) {
      std::cerr << "libgcz: no usable MI355X device (code " << rc << "), aborting...\n";
      std::exit(1);
    }
    engine_alive.store(true);
  }
  ~Engine() {
    engine_alive.store(false);
    gcz_ctx_destroy(ctx);
  }
};

Engine& engine() {
  static Engine e;
  return e;
}

// GCZ_TIMING=1: host wall-clock of the construction phases on stderr ("gcz-time phase ms").
struct PhaseTimer {
  const char* name;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  explicit PhaseTimer(const char* n) : name{n} {}
  ~PhaseTimer() {
    static const bool on = std::getenv("GCZ_TIMING") != nullptr;
    if (on)
      std::cerr << "gcz-time " << name << ' '
                << std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() << '\n';
  }
};

void check_build(int rc, gcz_ctx* ctx) {
  if (rc == GCZ_OK) return;
  gcz_host_pool_release(0);   // (a pre-faulted pool no fetch will use)
  gcz_info info{};
  gcz_info_get(ctx, &info);
  if (rc == GCZ_ERR_SYMBOL) {   // to_nac, src/dna.cpp:44-47
    int c = info.error_symbol;
    if (c >= 'a' && c <= 'z') c -= 32;
    std::cerr << "Encountered unknown symbol: " << c << " (ASCII code " << c << ")\n";
  } else if (rc == GCZ_ERR_EMPTY) {
    std::cerr << "Genome shorter than one strand of " << dna::size() << " nucleotides, aborting...\n";
  } else {
    std::cerr << "libgcz build failed (code " << rc << "): " << gcz_ctx_last_error(ctx) << '\n';
  }
  std::exit(1);
}

}  // namespace

// The destination of a device sort's arrays (shared_tree::lazy): the tree's containers keep their
// sizes across the sort (a permutation), so raw pointers to their storage stay valid while the
// tree lives -- also across a move, which takes the storage along.  Flags under the engine mutex.
struct gcz_lazy_copy {
  std::atomic<bool> pending{true};
  bool dead = false;   // the tree went away or its containers are being replaced
  std::uint64_t* leaves = nullptr;
  std::vector<std::uint32_t*> layers;
};

namespace {
// Before the engine's device arrays change (a build, a sort, a gather into its context): the
// pending sorted arrays into their tree.  (e.mu held)
void flush_pending(Engine& e) {
  std::shared_ptr<gcz_lazy_copy> p = std::move(e.pending);
  if (!p || !p->pending.load() || p->dead) return;
  PhaseTimer t{"fetch-sorted"};
  check_build(gcz_fetch_host(e.ctx, p->leaves, p->layers.data()), e.ctx);
  p->pending.store(false);
}

// pointer compression, src/shared_tree.cpp:25-67
int segment(std::uint32_t idx) {
  if (idx == 0x1fffffffu) return 3;
  if (idx < 16u) return 0;
  if (idx < 16u + 4096u) return 1;
  if (idx < 16u + 4096u + 1048576u) return 2;
  return 3;
}
constexpr std::uint32_t kSegStart[4] = {0, 16, 16 + 4096, 16 + 4096 + 1048576};

template <class Layers, class Leaves>
gcz::TreeView view(const Layers& nodes, const Leaves& leaves, pointer root) {
  gcz::TreeView v;
  v.L = int(dna::size());
  v.leaves = const_cast<std::uint64_t*>(reinterpret_cast<const std::uint64_t*>(leaves.data()));
  v.n_leaves = leaves.size();
  for (const auto& layer : nodes) {
    v.layer.push_back(const_cast<std::uint32_t*>(reinterpret_cast<const std::uint32_t*>(layer.data())));
    v.layer_n.push_back(layer.size());
  }
  v.root = root.raw();
  return v;
}

}  // namespace

// ---- pointer -----------------------------------------------------------------
// transform ctor, src/shared_tree.cpp:76-80
pointer::pointer(const pointer& other, bool mirror, bool transpose) noexcept {
  const std::uint32_t w = other.word;
  const bool m = (w >> 29) & 1u, t = (w >> 30) & 1u, v = w >> 31;
  const bool nm = (mirror != m) && !v;
  const bool nt = (transpose != t) && other != nullptr;
  word = (w & 0x9fffffffu) | (std::uint32_t(nm) << 29) | (std::uint32_t(nt) << 30);
}

auto pointer::bytes() const noexcept -> std::size_t {
  return (4 + address_bits[segment(word & 0x1fffffffu)]) / 8;
}

void pointer::serialize(std::ostream& os) const {
  const std::uint32_t idx = word & 0x1fffffffu;
  const int seg = segment(idx);
  const std::uint32_t off = idx == 0x1fffffffu ? 0xfffffffu : idx - kSegStart[seg];
  int sh = address_bits[seg] - 4;
  os.put(char((off >> sh) | (((word >> 29) & 1u) << 4) | (((word >> 30) & 1u) << 5) | (seg << 6)));
  for (sh -= 8; sh >= 0; sh -= 8) os.put(char(off >> sh));
}

auto pointer::deserialize(std::istream& is) -> pointer {
  const std::uint32_t first = static_cast<unsigned char>(is.get());
  const int seg = (first >> 6) & 3;
  std::uint64_t off = std::uint64_t(first & 0xf) << (address_bits[seg] - 4);
  for (int sh = address_bits[seg] - 12; sh >= 0; sh -= 8) off |= std::uint64_t(static_cast<unsigned char>(is.get())) << sh;
  const std::size_t idx = (seg == 3 && off == 0xfffffff) ? 0x1fffffffu : kSegStart[seg] + off;
  return pointer{idx, bool((first >> 4) & 1), bool((first >> 5) & 1), false};
}

// ---- node ----------------------------------------------------------------------
// node::canonical, include/shared_tree.h:119-126 (lexicographic min of (node, m, t))
auto node::canonical() const noexcept -> std::tuple<node, bool, bool> {
  std::tuple<node, bool, bool> best{*this, false, false};
  const std::tuple<node, bool, bool> cand[3] = {{mirrored(), true, false}, {transposed(), false, true},
                                                {inverted(), true, true}};
  for (const auto& c : cand)
    if (c < best) best = c;
  return best;
}

void node::serialize(std::ostream& os) const {
  children[0].serialize(os);
  children[1].serialize(os);
}

auto node::deserialize(std::istream& is) -> node {
  auto l = pointer::deserialize(is);
  auto r = pointer::deserialize(is);
  return node{l, r};
}

// ---- construction (libgcz) -------------------------------------------------------
namespace {
// The device context comes up (HIP runtime + code objects, ~0.1 s) while the file is mapped.
fasta_reader open_with_engine(const std::filesystem::path& path) {
  if (::access(path.c_str(), R_OK) != 0) return fasta_reader{path};   // prints the reference's error
  PhaseTimer t{"open"};
  std::error_code ec;
  const auto fsize = std::filesystem::file_size(path, ec);
  std::thread init([fsize] {   // the context, the input buffer and a warm upload path, while the file maps
    PhaseTimer t{"context"};
    auto& e = engine();
    std::lock_guard<std::mutex> lock(e.mu);
    flush_pending(e);   // (another tree's sorted arrays still in HBM, before the reservations)
    (void)gcz_upload_reserve(e.ctx, fsize);
    if (fsize >= (std::uint64_t(64) << 20)) (void)gcz_fetch_reserve(e.ctx, fsize);   // the fetch's ring
  });
  fasta_reader f = [&] { PhaseTimer t{"map"}; return fasta_reader{path}; }();
  if (!ec && fsize >= (std::uint64_t(64) << 20)) {
    // ... and the tree's host storage is faulted in meanwhile (the runtime start leaves the
    // host idle for ~0.1-0.25 s): a bound of the fetched arrays -- <= S nodes over all
    // layers and <= S leaves, 8 B each, S <= file bytes / L -- capped at 2 GB; the fetch
    // then copies into present pages (gcz_host_prefault, include/gcz.h)
    PhaseTimer t{"prefault"};
    const std::uint64_t S = fsize / std::max<std::size_t>(1, dna::size());
    (void)gcz_host_prefault(std::min<std::uint64_t>(16 * S + (std::uint64_t(96) << 20), std::uint64_t(2) << 30), 8);
  }
  init.join();
  return f;
}
}  // namespace

shared_tree::shared_tree(std::filesystem::path path) : shared_tree{open_with_engine(path)} {}

shared_tree::shared_tree(fasta_reader file, bool verbose) {
  auto& e = engine();
  std::lock_guard<std::mutex> lock(e.mu);
  flush_pending(e);
  struct PoolGuard {   // the pool open_with_engine faulted in goes whichever way this ends
    ~PoolGuard() { gcz_host_pool_release(1); }
  } pool_guard;
  {
    PhaseTimer t{"upload+build"};
    check_build(gcz_build_host_fasta_buffered(e.ctx, file.raw_data(), file.raw_size(), int(dna::size()),
                                              file.buffer_strands(), file.strands_read()),
                e.ctx);
  }
  build_from_gpu();
  if (verbose) std::cout << "\rConstructing subtrees: done.\n\rCombining subtrees: done.\n";
}

shared_tree::shared_tree(std::vector<dna>& data, bool verbose) {
  static_assert(sizeof(dna) == 8, "dna is one 64-bit word");
  auto& e = engine();
  std::lock_guard<std::mutex> lock(e.mu);
  flush_pending(e);
  check_build(gcz_build_host_leaves(e.ctx, reinterpret_cast<const std::uint64_t*>(data.data()), data.size(),
                                    int(dna::size())),
              e.ctx);
  build_from_gpu();
  if (verbose) std::cout << "\rConstructing subtrees: done.\n\rCombining subtrees: done.\n";
}

// ---- tree_constructor (src/shared_tree.cpp:617-763) ---------------------------------
tree_constructor::tree_constructor(shared_tree& parent) : parent{parent} { nodes.reserve(64); }

auto tree_constructor::emplace_leaf(dna leaf) -> pointer {   // :630-637
  const auto [canonical, mirror, transpose, invariant] = leaf.canonical();
  const auto ins = leaves.emplace(canonical, parent.leaf_count());
  if (ins.second) parent.emplace_leaf(canonical);
  return pointer{ins.first->second, mirror, transpose, invariant};
}

auto tree_constructor::emplace_leaves(dna left, dna right) -> pointer {   // :643-647
  const auto l = emplace_leaf(left);
  const auto r = emplace_leaf(right);
  return emplace_node(0, l, r);
}

auto tree_constructor::emplace_leaves(dna last) -> pointer { return emplace_node(0, emplace_leaf(last)); }   // :653-656

auto tree_constructor::emplace_node(std::size_t layer, pointer left, pointer right) -> pointer {   // :662-672
  const auto [canonical, mirror, transpose] = node{left, right}.canonical();
  const auto ins = nodes[layer].emplace(canonical, parent.node_count(layer));
  if (ins.second) parent.emplace_node(layer, canonical);
  const bool invariant = left == right.mirrored();
  return pointer{ins.first->second, mirror, transpose, invariant};
}

auto tree_constructor::reduce_roots(bool verbose) -> pointer {   // :677-692
  for (auto index = nodes.size(); roots.size() > 1; ++index) roots = reduce_nodes(roots, index);
  if (verbose) std::cout << "\rCombining subtrees: done.\n";
  parent.root = roots.front();   // (the reference's callers assign it; a tree built outside one needs it too)
  return roots.front();
}

auto tree_constructor::reduce_nodes(const std::vector<pointer>& iterable, std::size_t index)
    -> std::vector<pointer> {   // :697-712
  auto layer = std::vector<pointer>{};
  layer.reserve(iterable.size() / 2 + iterable.size() % 2);
  if (parent.depth() - 2 < index) {
    parent.add_layer();
    nodes.emplace_back();
  }
  for (std::size_t i = 0; i + 1 < iterable.size(); i += 2) layer.emplace_back(emplace_node(index, iterable[i], iterable[i + 1]));
  if (iterable.size() % 2) layer.emplace_back(emplace_node(index, iterable.back()));
  return layer;
}

auto tree_constructor::reduce(const std::vector<dna>& data, bool verbose) -> pointer {   // :743-763, on the GPU
  static_assert(sizeof(dna) == 8, "dna is one 64-bit word");
  auto& e = engine();
  {
    std::lock_guard<std::mutex> lock(e.mu);
    parent.drop_lazy();
    flush_pending(e);
    check_build(gcz_build_host_leaves(e.ctx, reinterpret_cast<const std::uint64_t*>(data.data()), data.size(),
                                      int(dna::size())),
                e.ctx);
    parent.build_from_gpu();
  }
  if (verbose) std::cout << "\rConstructing subtrees: done.\n\rCombining subtrees: done.\n";
  roots.assign(1, parent.root);
  return parent.root;
}

// every reader buffer of file.buffer_strands() strands its own subtree, the roots combined
// (one global level loop for the default power-of-two buffers: the same tree)
auto tree_constructor::reduce(fasta_reader& file, bool verbose) -> pointer {   // :719-736, on the GPU
  auto& e = engine();
  {
    std::lock_guard<std::mutex> lock(e.mu);
    parent.drop_lazy();
    flush_pending(e);
    check_build(gcz_build_host_fasta_buffered(e.ctx, file.raw_data(), file.raw_size(), int(dna::size()),
                                              file.buffer_strands(), file.strands_read()),
                e.ctx);
    parent.build_from_gpu();
  }
  if (verbose) std::cout << "\rConstructing subtrees: done.\n\rCombining subtrees: done.\n";
  roots.assign(1, parent.root);
  return parent.root;
}

// ---- multi-GPU construction (compress --gpus=N) ------------------------------------
namespace {

constexpr int kMaxGpus = 31;    // the multi-rank build's rank limit (gcz_dist_device.h kMaxRanks)

struct MultiShared {            // head of the shared result region
  std::atomic<int> status[kMaxGpus];  // per rank: 0 running, 1 done, 2 failed (read by rank 0's watcher)
  gcz_info info;                // rank 0's whole-tree summary
};

// Rank 0's watcher: a rank that fails (its status, or an exit that is not a clean 0) ends
// the whole job at once -- the other ranks may be blocked in an RCCL collective or in
// communicator creation, which has no timeout -- by killing every child and exiting 1.
// Children die with the parent (PR_SET_PDEATHSIG), so a failure of rank 0 ends them too.
class RankWatcher {
 public:
  RankWatcher(MultiShared* ms, std::vector<pid_t> kids) : ms_{ms}, kids_{std::move(kids)}, st_(kids_.size(), -1) {
    thread_ = std::thread([this] { run(); });
  }
  // Stops watching and reaps the children that are left: true iff every rank exited 0.
  bool finish() {
    done_.store(true);
    thread_.join();
    bool ok = true;
    for (std::size_t i = 0; i < kids_.size(); ++i) {
      if (st_[i] < 0) {
        int st = 0;
        st_[i] = ::waitpid(kids_[i], &st, 0) == kids_[i] && WIFEXITED(st) ? WEXITSTATUS(st) : 255;
      }
      ok = ok && st_[i] == 0;
    }
    return ok;
  }

 private:
  void run() {
    while (!done_.load()) {
      for (std::size_t i = 0; i < kids_.size(); ++i) {
        const int r = int(i) + 1;
        bool failed = ms_->status[r].load() == 2;
        if (st_[i] < 0) {
          int st = 0;
          if (::waitpid(kids_[i], &st, WNOHANG) == kids_[i]) {
            st_[i] = WIFEXITED(st) ? WEXITSTATUS(st) : 255;
            failed = failed || st_[i] != 0;
          }
        }
        if (failed) {
          for (pid_t p : kids_) ::kill(p, SIGKILL);
          std::cerr << "libgcz: rank " << r << " of the multi-GPU build failed, stopping every rank\n";
          std::_Exit(1);
        }
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
  }
  MultiShared* ms_;
  std::vector<pid_t> kids_;
  std::vector<int> st_;   // exit status of a reaped child, -1 while running
  std::atomic<bool> done_{false};
  std::thread thread_;
};

// first byte of [0, n) that is not one of the 16 symbols (any case), or n; threads
std::uint64_t first_unknown(const std::uint8_t* b, std::uint64_t n) {
  static const auto ok = [] {
    std::array<bool, 256> t{};
    for (char c : std::string_view{"SACRGBNKTWVDYHM-"}) {
      t[static_cast<unsigned char>(c)] = true;
      t[static_cast<unsigned char>(std::tolower(c))] = true;
    }
    return t;
  }();
  const unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<std::uint64_t> first(T, n);
  std::vector<std::thread> th;
  for (unsigned t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      const std::uint64_t a = n * t / T, e = n * (t + 1) / T;
      for (std::uint64_t i = a; i < e; ++i)
        if (!ok[b[i]]) { first[t] = i; return; }
    });
  for (auto& x : th) x.join();
  return *std::min_element(first.begin(), first.end());
}

[[noreturn]] void rank_fail(MultiShared* ms, int rank, const char* what, int rc, gcz_ctx* c) {
  std::cerr << "libgcz rank " << rank << ": " << what << " failed (code " << rc << ")"
            << (c ? std::string(": ") + gcz_ctx_last_error(c) : std::string()) << '\n';
  ms->status[rank].store(2);
  std::_Exit(1);
}

}  // namespace

auto shared_tree_on_gpus(const std::filesystem::path& path, int gpus) -> shared_tree {
  const int L = int(dna::size());
  fasta_reader f{path};
  // the FASTA contract on the host (gcz_fasta_extract), into memory the ranks share
  const std::uint64_t fsz = f.raw_size();
  auto* bases = static_cast<std::uint8_t*>(
      ::mmap(nullptr, fsz + 16, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0));
  if (bases == MAP_FAILED) { std::cerr << "libgcz: no memory for the bases\n"; std::exit(1); }
  const std::uint64_t nb = fsz ? gcz_fasta_extract(f.raw_data(), fsz, L, 0, bases) : 0;
  const std::uint64_t S = nb / std::uint64_t(L);
  if (S == 0) {
    std::cerr << "Genome shorter than one strand of " << dna::size() << " nucleotides, aborting...\n";
    std::exit(1);
  }
  if (const auto bad = first_unknown(bases, S * L); bad < S * L)   // to_nac's message and exit(1)
    (void)dna{std::string_view{reinterpret_cast<const char*>(bases + bad), 1}};
  if (gpus > kMaxGpus) {
    std::cerr << "compress: --gpus=" << gpus << " is more than the " << kMaxGpus
              << " ranks the multi-GPU build supports, aborting...\n";
    std::exit(1);
  }
  gpus = std::max(1, gpus);
  // the ranks' status words, shared across the fork (the tree itself is gathered on the device)
  const std::size_t rbytes = (sizeof(MultiShared) + 4095) / 4096 * 4096;
  auto* region = static_cast<char*>(::mmap(nullptr, rbytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0));
  if (region == MAP_FAILED) { std::cerr << "libgcz: no memory for the rank status\n"; std::exit(1); }
  auto* ms = new (region) MultiShared{};
  const bool shm = [] {
    const char* t = std::getenv("GCZ_MULTI_TRANSPORT");
    return t && std::string_view{t} == "shm";
  }();
  const char* dv = std::getenv("GCZ_DEVICE");
  const int dev0 = dv ? std::atoi(dv) : 0;
  const std::string shm_name = "/gcz_compress_" + std::to_string(::getpid());
  // ranks 1.. are forked before this process touches the device; the RCCL id goes over pipes
  std::vector<int> wr(gpus, -1);
  std::vector<pid_t> kids;
  int rank = 0, rd = -1;
  for (int r = 1; r < gpus; ++r) {
    int fd[2];
    if (::pipe(fd) != 0) { std::cerr << "libgcz: pipe failed\n"; std::exit(1); }
    const pid_t pid = ::fork();
    if (pid < 0) { std::cerr << "libgcz: fork failed\n"; std::exit(1); }
    if (pid == 0) {
      ::prctl(PR_SET_PDEATHSIG, SIGKILL);   // never outlive rank 0
      if (::getppid() == 1) std::_Exit(1);
      rank = r;
      rd = fd[0];
      ::close(fd[1]);
      for (int q = 1; q < r; ++q) ::close(wr[q]);
      break;
    }
    ::close(fd[0]);
    wr[r] = fd[1];
    kids.push_back(pid);
  }
  std::unique_ptr<RankWatcher> watch;
  if (rank == 0 && !kids.empty()) watch = std::make_unique<RankWatcher>(ms, kids);
  gcz_ctx* ctx = nullptr;
  int rc = gcz_ctx_create(shm ? dev0 : dev0 + rank, &ctx);
  if (rc) rank_fail(ms, rank, "device context", rc, nullptr);
  gcz_group* g = nullptr;
  if (shm) {
    rc = gcz_group_create_shm(ctx, rank, gpus, shm_name.c_str(), (S / std::uint64_t(gpus) + 1) * 64 + (64u << 20), &g);
  } else {
    unsigned char id[128] = {};
    if (rank == 0) {
      if ((rc = gcz_dist_unique_id(id, sizeof id))) rank_fail(ms, 0, "RCCL unique id", rc, ctx);
      // (a rank that already died closed its pipe: EPIPE, not SIGPIPE)
      struct sigaction ign {}, old {};
      ign.sa_handler = SIG_IGN;
      ::sigaction(SIGPIPE, &ign, &old);
      for (int r = 1; r < gpus; ++r)
        if (::write(wr[r], id, sizeof id) != ssize_t(sizeof id)) rank_fail(ms, 0, "id pipe", -1, ctx);
      ::sigaction(SIGPIPE, &old, nullptr);
    } else if (::read(rd, id, sizeof id) != ssize_t(sizeof id)) {
      rank_fail(ms, rank, "id pipe", -1, ctx);
    }
    rc = gcz_group_create_rccl(ctx, rank, gpus, id, &g);
  }
  if (rc) rank_fail(ms, rank, "group", rc, ctx);
  std::uint64_t s0 = 0, s1 = 0;
  if ((rc = gcz_dist_plan(S, gpus, rank, &s0, &s1, nullptr))) rank_fail(ms, rank, "partition plan", rc, ctx);
  void* d = gcz_dev_alloc(ctx, (s1 - s0) * std::uint64_t(L) + 16);
  if (!d) rank_fail(ms, rank, "device allocation", GCZ_ERR_DEVICE, ctx);
  if ((rc = gcz_memcpy_h2d(ctx, d, bases + s0 * std::uint64_t(L), (s1 - s0) * std::uint64_t(L))))
    rank_fail(ms, rank, "upload", rc, ctx);
  const void* dp = d;
  if ((rc = gcz_group_build_device_bases(g, &dp, S, L))) rank_fail(ms, rank, "build", rc, ctx);
  // the whole tree gathered device to device into rank 0's engine context (gcz_group_assemble):
  // there it is a device-resident tree like a one-GPU build's, so the frequency sort, bytes()
  // and the .dag writer run on the GPU (sort_tree / serialize above)
  gcz_ctx* dst = rank == 0 ? engine().ctx : nullptr;
  if (rank == 0) {   // (another tree's sorted arrays still in HBM: the gather overwrites them)
    auto& e = engine();
    std::lock_guard<std::mutex> lock(e.mu);
    flush_pending(e);
  }
  if ((rc = gcz_group_assemble(g, dst))) rank_fail(ms, rank, "tree gather", rc, ctx);
  gcz_dev_free(ctx, d);
  gcz_group_destroy(g);
  gcz_ctx_destroy(ctx);
  ms->status[rank].store(1);
  if (rank != 0) std::_Exit(0);
  const bool ok = !watch || watch->finish();
  for (int r = 1; r < gpus; ++r) ::close(wr[r]);
  if (!ok) { std::cerr << "libgcz: a rank of the multi-GPU build failed\n"; std::exit(1); }
  shared_tree t;
  {
    auto& e = engine();
    std::lock_guard<std::mutex> lock(e.mu);
    t.build_from_gpu();
  }
  ::munmap(region, rbytes);
  ::munmap(bases, fsz + 16);
  return t;
}

void shared_tree::build_from_gpu() {
  PhaseTimer t{"fetch"};
  drop_lazy();   // (the containers are refilled)
  gcz_ctx* ctx = engine().ctx;
  gcz_info info{};
  gcz_info_get(ctx, &info);
  std::vector<std::uint32_t*> outs(info.n_layers);
  {
    PhaseTimer t2{"fetch-alloc"};
    leaves.resize(info.n_leaves);
    nodes.resize(info.n_layers);   // keeps each layer's storage when a device sort refetches the same sizes
    for (int k = 0; k < info.n_layers; ++k) {
      nodes[k].resize(info.layer_size[k]);
      outs[k] = reinterpret_cast<std::uint32_t*>(nodes[k].data());
    }
  }
  {
    PhaseTimer t2{"fetch-copy"};
    // a large tree's frequency-sort buffers are allocated beside the copy (compress sorts next;
    // its first device sort at 1 Gbase otherwise starts with ~40 ms of allocation)
    std::uint64_t total = info.n_leaves;
    for (int k = 0; k < info.n_layers; ++k) total += info.layer_size[k];
    std::thread reserve;
    if (total >= (std::uint64_t(1) << 22)) reserve = std::thread([ctx] { (void)gcz_sort_reserve(ctx); });
    const int rc = gcz_fetch_host(ctx, reinterpret_cast<std::uint64_t*>(leaves.data()), outs.data());
    if (reserve.joinable()) reserve.join();
    check_build(rc, ctx);
  }
  // what the pre-faulted pool did not hold goes back on a side thread (unmapping ~0.6 GB of
  // present pages takes ~25 ms)
  gcz_host_pool_release(1);
  root = pointer::from_word(info.root);
  device_gen = ++engine().gen;
}

bool shared_tree::on_device() const { return device_gen != 0 && device_gen == engine().gen; }

// ---- the lazy host copy of a device sort -----------------------------------------------
void shared_tree::materialize() const {
  if (!lazy || !lazy->pending.load(std::memory_order_acquire)) return;
  auto& e = engine();
  std::lock_guard<std::mutex> lock(e.mu);
  if (!lazy->pending.load() || lazy->dead) return;
  PhaseTimer t{"fetch-sorted"};
  check_build(gcz_fetch_host(e.ctx, lazy->leaves, lazy->layers.data()), e.ctx);
  lazy->pending.store(false, std::memory_order_release);
  if (e.pending == lazy) e.pending.reset();
}

void shared_tree::drop_lazy() {   // (e.mu held by every caller but the destructor / assignments)
  if (lazy) lazy->dead = true;
  lazy.reset();
}

shared_tree::~shared_tree() {
  if (lazy && engine_alive.load()) {
    auto& e = engine();
    std::lock_guard<std::mutex> lock(e.mu);
    lazy->dead = true;
  }
}

shared_tree::shared_tree(const shared_tree& o) {
  o.materialize();
  nodes = o.nodes;
  leaves = o.leaves;
  root = o.root;
  device_gen = o.device_gen;
}

shared_tree::shared_tree(shared_tree&& o) noexcept
    : lazy(std::move(o.lazy)), nodes(std::move(o.nodes)), leaves(std::move(o.leaves)), root(o.root),
      device_gen(o.device_gen) {}

auto shared_tree::operator=(const shared_tree& o) -> shared_tree& {
  if (this == &o) return *this;
  o.materialize();
  if (lazy && engine_alive.load()) {
    std::lock_guard<std::mutex> lock(engine().mu);
    drop_lazy();
  }
  nodes = o.nodes;
  leaves = o.leaves;
  root = o.root;
  device_gen = o.device_gen;
  return *this;
}

auto shared_tree::operator=(shared_tree&& o) noexcept -> shared_tree& {
  if (this == &o) return *this;
  if (lazy && engine_alive.load()) {
    std::lock_guard<std::mutex> lock(engine().mu);
    drop_lazy();
  }
  nodes = std::move(o.nodes);
  leaves = std::move(o.leaves);
  root = o.root;
  device_gen = o.device_gen;
  lazy = std::move(o.lazy);
  return *this;
}

// ---- accessors -----------------------------------------------------------------
auto shared_tree::width() const -> std::size_t {
  assert(nodes.back().size() == 1);
  if (on_device()) {   // a tree of the device build: the strands it was built from (gcz_info)
    gcz_info info{};
    if (gcz_info_get(engine().ctx, &info) == GCZ_OK) return std::size_t(info.n_strands);
  }
  materialize();
  return gcz::view_width(view(nodes, leaves, root));
}

auto shared_tree::children(std::size_t layer, pointer p) const -> std::size_t {   // :252-259
  if (p.empty()) return 0;
  const auto n = access_node(layer, p);
  if (layer == 0) return !n.left().empty() + !n.right().empty();
  return children(layer - 1, n.left()) + children(layer - 1, n.right());
}

auto shared_tree::node_count() const -> std::size_t {
  std::size_t sum = 0;
  for (const auto& layer : nodes) sum += layer.size();
  return sum;
}

auto shared_tree::access_leaf(pointer p) const -> dna {   // :231-236
  materialize();
  auto leaf = leaves[p.index()];
  if (p.is_mirrored()) leaf = leaf.mirrored();
  if (p.is_transposed()) leaf = leaf.transposed();
  return leaf;
}

auto shared_tree::operator[](std::uint64_t index) const -> dna {   // :268-291
  auto current = root;
  for (int layer = int(nodes.size()) - 1; layer >= 0; --layer) {
    const auto n = access_node(std::size_t(layer), current);
    const auto size = std::uint64_t(1) << layer;
    const bool mirror = current.is_mirrored(), transpose = current.is_transposed();
    const pointer first = mirror ? n.right() : n.left();
    const pointer second = mirror ? n.left() : n.right();
    if (index < size) {
      current = pointer{first, mirror, transpose};
    } else {
      index -= size;
      current = pointer{second, mirror, transpose};
    }
  }
  return access_leaf(current);
}

// ---- frequency sort (:316-483) ------------------------------------------------------
auto shared_tree::histogram(std::size_t layer) const -> std::vector<std::size_t> {
  assert(layer < nodes.size());
  materialize();
  std::vector<std::size_t> result(layer == 0 ? leaves.size() : nodes[layer - 1].size(), 0);
  for (const auto& n : nodes[layer]) {
    if (auto l = n.left(); l) ++result[l.index()];
    if (auto r = n.right(); r) ++result[r.index()];
  }
  return result;
}

void shared_tree::store_histogram(std::filesystem::path path) const {
  std::ofstream file{path};
  for (std::size_t layer = 0; layer < nodes.size(); ++layer) {
    auto freq = histogram(layer);
    std::sort(freq.begin(), freq.end(), std::greater<>());
    for (std::size_t i = 0; i < freq.size(); i += 1000) {
      for (std::size_t j = i; j < std::min(freq.size(), i + 1000); ++j) file << freq[j] << ',';
      file << '\n';
    }
    file << '\n';
  }
}

void shared_tree::rewire_nodes(std::size_t layer, const std::vector<std::size_t>& indices) {
  materialize();
  device_gen = 0;
  auto rewire = [&](pointer old) {
    if (old.empty()) return old;
    return pointer{indices[old.index()], old.is_mirrored(), old.is_transposed(), old.is_invariant()};
  };
  for (auto& n : nodes[layer]) n = node{rewire(n.left()), rewire(n.right())};
}

namespace {
std::vector<std::size_t> sorted_positions(const std::vector<std::size_t>& freq) {
  std::vector<std::size_t> idx(freq.size());
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](auto a, auto b) { return freq[a] > freq[b]; });
  std::vector<std::size_t> inv(idx.size());
  for (std::size_t i = 0; i < idx.size(); ++i) inv[idx[i]] = i;
  return inv;
}
}  // namespace

void shared_tree::sort_leaves() {
  const auto pos = sorted_positions(histogram(0));
  leaf_vector r(leaves.size());
  for (std::size_t i = 0; i < pos.size(); ++i) r[pos[i]] = leaves[i];
  leaves.swap(r);
  rewire_nodes(0, pos);
}

void shared_tree::sort_nodes(std::size_t layer) {
  const auto pos = sorted_positions(histogram(layer + 1));
  layer_vector r(nodes[layer].size());
  for (std::size_t i = 0; i < pos.size(); ++i) r[pos[i]] = nodes[layer][i];
  nodes[layer].swap(r);
  rewire_nodes(layer + 1, pos);
}

void shared_tree::sort_tree(bool verbose) {
  if (on_device()) {   // the arrays are still in HBM: sort there; the host copy waits for its first read
    auto& e = engine();
    std::lock_guard<std::mutex> lock(e.mu);
    if (e.pending != lazy) flush_pending(e);   // (another tree's sorted arrays: none while this one is on the device)
    {
      PhaseTimer t{"device-sort"};
      check_build(gcz_sort_device(e.ctx), e.ctx);
    }
    if (!lazy) {   // (sorting again a tree whose copy is still pending: the same destination)
      gcz_info info{};
      gcz_info_get(e.ctx, &info);
      auto lz = std::make_shared<gcz_lazy_copy>();
      lz->leaves = reinterpret_cast<std::uint64_t*>(leaves.data());
      for (int k = 0; k < info.n_layers; ++k) lz->layers.push_back(reinterpret_cast<std::uint32_t*>(nodes[k].data()));
      lazy = std::move(lz);
    }
    e.pending = lazy;
    root = [&] {
      gcz_info info{};
      gcz_info_get(e.ctx, &info);
      return pointer::from_word(info.root);
    }();
    device_gen = ++e.gen;
  } else {
    materialize();
    auto v = view(nodes, leaves, root);   // all layers at once, in parallel (same net effect)
    gcz::view_sort(v);
  }
  if (verbose) std::cout << "\rSorting nodes: done.\n";
}

// ---- persistence (:488-546) ------------------------------------------------------------
auto shared_tree::bytes() const noexcept -> std::size_t {
  if (on_device()) {
    std::uint64_t b = 0;
    if (gcz_bytes_device(engine().ctx, &b) == GCZ_OK) return b;
  }
  materialize();
  return gcz::view_bytes(view(nodes, leaves, root));
}

void shared_tree::serialize(std::ostream& os) const {
  if (on_device()) {   // the .dag is written on the device
    std::uint64_t n = 0;
    if (gcz_bytes_device(engine().ctx, &n) == GCZ_OK) {
      std::unique_ptr<std::uint8_t[]> buf(new std::uint8_t[n]);   // left uninitialised: the D2H copy fills it
      if (gcz_serialize_device(engine().ctx, buf.get(), n, &n) == GCZ_OK) {
        os.write(reinterpret_cast<const char*>(buf.get()), std::streamsize(n));
        return;
      }
    }
  }
  materialize();
  const auto v = view(nodes, leaves, root);
  std::vector<std::uint8_t> buf(gcz::view_bytes(v));
  gcz::view_serialize(v, buf.data(), buf.size());
  os.write(reinterpret_cast<const char*>(buf.data()), std::streamsize(buf.size()));
}

auto shared_tree::deserialize(std::istream& is) -> shared_tree {
  shared_tree result;
  result.root = pointer::deserialize(is);
  std::uint64_t size = 0;
  auto read_u64 = [&](std::uint64_t& v) {
    v = 0;
    for (int i = 0; i < 8; ++i) {
      const int c = is.get();
      if (c == EOF) return false;
      v = (v << 8) | std::uint64_t(c);
    }
    return true;
  };
  read_u64(size);
  for (std::uint64_t i = 0; i < size; ++i) result.leaves.emplace_back(dna::deserialize(is));
  while (read_u64(size)) {
    result.nodes.emplace_back();
    result.nodes.back().reserve(size);
    for (std::uint64_t i = 0; i < size; ++i) result.nodes.back().emplace_back(node::deserialize(is));
  }
  return result;
}

void shared_tree::save(std::filesystem::path path) const {
  PhaseTimer t{"save"};
  std::ofstream file{path, std::ios::binary};
  serialize(file);
}

// ---- iterator (:553-614) ----------------------------------------------------------------
shared_tree::iterator::iterator(const shared_tree& parent, std::size_t layer, pointer root) : parent{parent} {
  if (root) {
    stack.emplace_back(layer, root);
    next_leaf();
  }
}

auto shared_tree::iterator::operator*() const noexcept -> dna { return parent.access_leaf(stack.back().current); }

auto shared_tree::iterator::operator++() -> iterator& {
  stack.pop_back();
  next_leaf();
  return *this;
}

void shared_tree::iterator::next_leaf() {
  while (!stack.empty()) {
    const auto st = stack.back();
    if (st.layer == std::size_t(-1)) return;
    const auto top = st.current;
    const auto n = parent.access_node(st.layer, top);
    stack.pop_back();
    auto push = [&](pointer next) { stack.emplace_back(st.layer - 1, pointer{next, top.is_mirrored(), top.is_transposed()}); };
    if (top.is_mirrored()) {
      if (n.left()) push(n.left());
      if (n.right()) push(n.right());
    } else {
      if (n.right()) push(n.right());
      if (n.left()) push(n.left());
    }
  }
}
