// Host-side build context shared by the single-device build (gcz_build.hip)
// and the multi-rank build (gcz_dist.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gcz_device.h"
#include "gcz_dense.h"

#define HIP_TRY(x)                                                                    \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) return fail(GCZ_ERR_DEVICE, #x, hipGetErrorString(e_));    \
  } while (0)

namespace gcz_host {

using gcz_dev::u32;
using gcz_dev::u64;

inline u64 next_pow2(u64 x) {
  u64 p = 1;
  while (p < x) p <<= 1;
  return p;
}

inline u64 inv64(u64 a) {                 // inverse of an odd number mod 2^64 (Newton)
  u64 x = a;
  for (int i = 0; i < 6; ++i) x *= 2 - a * x;
  return x;
}

inline u32 bit_width(u64 x) {
  u32 b = 0;
  while (x) { ++b; x >>= 1; }
  return b;
}

inline u32 log2_exact(u64 x) { return bit_width(x) - 1; }

constexpr u32 kAdaptiveProbeLimit = 256;
constexpr u64 kMixC1 = 0x9E3779B97F4A7C15ull;
constexpr u64 kMixC2 = 0xD6E8FEB86659FD93ull;

struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  template <class T> T* as() const { return static_cast<T*>(ptr); }
};

// A level's table: packed 8-B words when quotient+displacement+position fit
// in 64 bits, else 16-B wide slots.
struct LevelTab {
  bool packed = false;
  gcz_dev::PackedTab pt{};
  gcz_dev::WideTab wt{};
  u64 cap = 0;
  u64 bytes() const { return cap * (packed ? 8 : 16); }
};

inline LevelTab plan_table(void* buf, u64 cap, u32 K, u64 npos, u32 B, bool allow_packed, u32 wide_limit) {
  LevelTab lt;
  lt.cap = cap;
  const u32 c = log2_exact(cap);
  const u32 Q = K > c ? K - c : 0;
  const u32 P = std::max<u32>(1, bit_width(npos - 1));
  const int room = 64 - int(Q) - int(P);
  if (allow_packed && K <= 64 && room >= 6) {
    lt.packed = true;
    gcz_dev::PackedTab& t = lt.pt;
    t.tab = static_cast<u64*>(buf);
    t.mask = u32(cap - 1);
    t.D = u32(std::min(room, 16));   // displacement bits: probe limit 2^D - 2
    t.limit = (1u << t.D) - 2;
    t.B = B;
    t.c = c;
    t.P = P;
    t.sh = (K + 1) / 2;
    t.kmask = K >= 64 ? ~0ull : ((1ull << K) - 1);
    t.c1 = kMixC1; t.c2 = kMixC2;
    t.c1i = inv64(kMixC1); t.c2i = inv64(kMixC2);
  } else {
    lt.wt.tab = static_cast<gcz_dev::Slot*>(buf);
    lt.wt.mask = u32(cap - 1);
    lt.wt.limit = wide_limit;
    lt.wt.B = B;
  }
  return lt;
}

enum KernelId {
  KID_LEAF, KID_NODE, KID_FLAGSCAN_LEAF, KID_FLAGSCAN_NODE, KID_RESOLVE_LEAF, KID_RESOLVE_NODE, KID_MEMSET,
  KID_EXCHANGE, KID_DIST, KID_OWNER, KID_IDS, KID_REMAP, KID_TAIL, KID_SORT, KID_DAG, KID_DIRECT,
  KID_BKT_COUNT, KID_BKT_SCAN, KID_BKT_SCATTER, KID_BKT_DEDUPE, KID_BKT_FINE,
  KID_DL_PACK, KID_DL_SCAN, KID_DL_SCATTER, KID_DL_FIRST, KID_DL_FBSCAN, KID_DL_IDS, KID_DL_WORDS, KID_L0, KID_MARK,
  KID_DL_PROBE,
  KID_COUNT
};
inline const char* kernel_name(int k) {
  static const char* names[KID_COUNT] = {"leaf_insert", "node_insert", "flagscan_leaf", "flagscan_node",
                                         "resolve_leaf", "resolve_node", "clear", "exchange", "dist_bucket",
                                         "dist_owner", "dist_ids", "dist_remap", "tail", "sort", "dag_write", "direct_levels",
                                         "bucket_count", "bucket_scan", "bucket_scatter", "bucket_dedupe", "bucket_fine",
                                         "dl_pack", "dl_scan", "dl_scatter", "dl_first", "dl_fbscan", "dl_ids",
                                         "dl_words", "dist_l0", "mark", "dl_probe"};
  return names[k];
}

// Leaf chunk plan (strands [chunk_start[c], chunk_start[c+1])): a first chunk of
// S >> first_log2 strands, then one of the same size, then doubling.
std::vector<u64> leaf_chunks(u64 S, int first_log2 = 6);

// One node level of the build.
struct NodeLevel {
  int k = 0;                        // layer index (marks parity)
  const u32* in = nullptr;          // n final words of the previous level
  u64 n = 0, p = 0;                 // p = ceil(n / 2) pairs
  u32* words = nullptr;             // p output words
  uint2* out = nullptr;             // unique nodes, indexed by id
  u64* count = nullptr;             // unique count (device)
  u64 bound = 0;                    // child ids < bound
  bool prev_marks = false;          // previous level's marks valid (singleton propagation)
  const u64* pcount = nullptr;      // direct iff *pcount == n
  u32 id_off = 0;                   // direct ids are id_off + j
  bool direct_known = false;        // host knows the level is direct: launch the insert only
  u64* desc = nullptr;              // look-back descriptors (ceil(p / kTile))
  u32* ticket = nullptr;
  u32* hashed_next = nullptr;       // single-device build: look ahead for the next level (null: off)
  u64* gate = nullptr;              // ... and open its gate (the next level's pcount)
  bool allow_bucket = false;        // single-device build: bucketed insert allowed (overflow -> rebuild)
  bool repetitive = false;          // ... the host knows the data is repetitive (no single-pass buckets)
  // fused small-build levels (k_node_insert with a resolver, gcz_device.h): this level's
  // table lives in ftab region k % 3, its repeats are settled by the next level's insert
  // unless it is the last one before the tail (resolve launched here)
  bool fused = false, fused_last = false;
  bool tail_settles = false;        // fused_last and the tail follows: it settles this level's repeats
  u64 p_next = 0;                   // the next level's pairs (its table is cleared here)
  void* ftab = nullptr;             // region base of this level's table
  void* ftab_next = nullptr;        // ... and of the next level's
  gcz_host::u32* sid = nullptr;     // ids of this level's repeated keys by slot (flag scan -> next insert)
  const gcz_host::u32* sid_prev = nullptr;   // ... of the previous level
  // reader-buffer segments: the previous level's marks as expanded with the input (k_seg_expand)
  const unsigned char* prev_nf = nullptr;
  const unsigned char* prev_multi = nullptr;
};

// One leaf level (all chunks).
struct LeafLevel {
  const void* bases = nullptr;      // ASCII (4-B aligned) or null
  const u64* leaves = nullptr;      // packed strands or null
  u64 S = 0;
  int L = 12;
  u64 cap = 0;                      // table slots
  bool adaptive = false;            // probe-limited: overflow -> grow and rebuild
  u32* words = nullptr;             // S words (local ids)
  u64* out = nullptr;               // unique leaves, indexed by id
  std::vector<u64> chunk_start;
  u64* desc = nullptr;              // descriptors, chunk c at desc + desc_off[c]
  std::vector<u64> desc_off;
  u64* count = nullptr;             // count[c] = uniques after chunk c (cumulative, device)
  u32* ticket = nullptr;            // one per chunk
  // multi-rank: chunks [c_begin, c_end) only (c_end < 0: all; table and marks are cleared
  // when c_begin == 0), and a dictionary of seed_n keys whose ids are their indices
  int c_begin = 0, c_end = -1;
  const u64* seed = nullptr;
  u64 seed_n = 0;
  bool precleared = false;          // table and marks already cleared (k_build_init)
  bool defer_resolve = false;       // fused small build: level 0's insert settles the repeats
  u64* lkey = nullptr;              // ... through ids by slot (lsid) the flag scan leaves, emitting
  u32* lsid = nullptr;              //     first occurrences from the keys the insert stored (lkey)
};

}  // namespace gcz_host

// What a captured build graph depends on (gcz_ctx::build): replayed only on a match.
struct GraphKey {
  const void* bases;
  const void* leaves;
  gcz_host::u64 nbases, S;
  int L;
  gcz_host::u64 leaf_cap;
  bool packed, bucket;
  hipStream_t stream;
  void *tab, *wa, *wb, *nodes, *leaves_out, *nf, *desc, *ftab, *fsid, *flkey, *flsid;
  bool fused;
  bool operator==(const GraphKey& o) const {
    return bases == o.bases && leaves == o.leaves && nbases == o.nbases && S == o.S && L == o.L &&
           leaf_cap == o.leaf_cap && packed == o.packed && bucket == o.bucket && stream == o.stream && tab == o.tab &&
           wa == o.wa && wb == o.wb && nodes == o.nodes && leaves_out == o.leaves_out && nf == o.nf && desc == o.desc &&
           ftab == o.ftab && fsid == o.fsid && flkey == o.flkey && flsid == o.flsid && fused == o.fused;
  }
};

struct gcz_dist_state;   // gcz_dist.hip
struct gcz_sort_state;   // gcz_sort.hip
struct gcz_ingest_state; // gcz_ingest.hip
// Builds of more than 2^29 - 1 strands on one device (gcz_ctx::build): virtual ranks
// whose slices are concatenated into the context's arrays (gcz_dist.hip).
int gcz_split_build(struct gcz_ctx* c, const void* d_bases, const gcz_host::u64* d_leaves, gcz_host::u64 S, int L);
// GCZ_CANARY=1: the overwritten guard bands of c's buffers, described into `out` (gcz_build.hip)
int gcz_canary_scan(struct gcz_ctx* c, std::string& out);

struct gcz_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string last_error;
  gcz_host::DevBuf wa, wb, grp, desc, tab, leaves_out, nodes_out, hdr, input, nf, multi;
  gcz_host::DevBuf stats;   // hashed-pair counter shards (k_node_insert), summed into hdr->hashed[0]
  gcz_host::DevBuf bkt_key, bkt_cnt, bkt_off, bkt_tmp, bkt_rec2;   // bucketed node insert (k_bkt_*)
  gcz_host::DevBuf dl_pw, dl_rec, dl_idrec, dl_cnt, dl_off, dl_offt, dl_fpg, dl_fb, dl_wpre, dl_desc, dl_fl, dl_fo;   // dense leaf level
  gcz_host::DevBuf dl_fbw;   // ... the bitmap interleaved with its prefix (k_dl_fbw; single device)
  // ... multi-rank: rfc (dl_lh), presence bitmaps (own, gathered), bucket counts + exchange vector (dl_pos),
  // gathered exchange vectors (dl_lower), G (dl_list), relay table (dl_gid), relay buffers, status words
  gcz_host::DevBuf dl_lh, dl_pb, dl_pbs, dl_lower, dl_pos, dl_list, dl_gid, dl_recv, dl_stage, dl_seg;
  gcz_dev::DensePlan dl_plan{};
  unsigned probe_ranks = 1;   // ranks sharing the repetitive-data probe (multi-rank dense leaf level)
  gcz_dev::Header* h_hdr = nullptr;   // pinned
  unsigned char* h_ring = nullptr;    // pinned D2H staging ring of the host fetch (gcz_fetch_host)
  gcz_host::u64 h_ring_bytes = 0;
  hipEvent_t ring_ev[4] = {};         // its slots' D2H completions
  unsigned char* nf_set[2] = {nullptr, nullptr};      // marks, even / odd layers
  unsigned char* multi_set[2] = {nullptr, nullptr};
  // last build
  gcz_info info{};
  std::vector<gcz_host::u64> layer_off;  // node offsets (in nodes) per layer within nodes_out
  bool allow_packed = true;
  // profiling
  bool profile = false;
  bool force_wide = false;   // GCZ_TABLE=wide: always use 16-B slots (testing)
  int node_cap_shift = 1;    // node table capacity = next_pow2(p << shift)   (GCZ_NODE_CAP_SHIFT)
  int leaf_cap_log2 = 0;     // force the adaptive leaf table size            (GCZ_LEAF_CAP_LOG2)
  bool use_tail = true;      // fuse the top levels into one launch           (GCZ_TAIL=0 disables)
  bool use_direct = true;    // direct subtrees after a host check at layer 1 (GCZ_DIRECT=0 disables)
  int leaf_first_log2 = 6;   // first leaf chunk = S >> this                 (GCZ_LEAF_FIRST_LOG2)
  int predup_mode = 0;       // node-insert LDS pre-dedupe: 0 auto, 1 on, 2 off  (GCZ_PREDUP)
  bool use_bucket = true;    // bucketed LDS node insert on non-repetitive data  (GCZ_BUCKET=0 disables)
  gcz_host::u64 bucket_min = 1ull << 20;   // ... on levels of at least this many pairs (GCZ_BUCKET_MIN)
  bool two_pass = true;      // ... as the two-pass partition where records fit (GCZ_BUCKET_TWO=0: one pass)
  bool part_words_off = true;   // ... and, without the block collapse, writes no provisional word (the dedupe
                                // takes a repeat's bits from its pair; GCZ_PART_WORDS=1: the words are written;
                                // measured part 0.291 -> 0.273 ms uniform_1g, tandem unchanged)
  gcz_host::u32 bkt_xcd = 3;   // ... whose bitmap dedupe (bit 1) and fine pass (bit 2) take XCD-contiguous
                               // workgroup runs (GCZ_BKT_XCD; measured dedupe -5 us, fine -11 us uniform_1g)
  bool part_marks = true;    // ... whose partition writes every mark (no clearing pass; GCZ_PART_MARKS=0)
  bool sparse_scan = true;   // ... and whose few repeats are ranked without a look-back scan (GCZ_SPARSE_SCAN=0)
  bool part_wave = false;    // ... and whose collapse inserts a one-key wave once (GCZ_PART_WAVE=1;
                             // measured 0.14 ms slower on tandem_3g2, off)
  gcz_host::DevBuf nf_list;  // ... those repeats' positions (k_bkt_dedupe2)
  gcz_host::DevBuf bkt_redo; // ... the buckets the bitmap dedupe hands to k_bkt_dedupe2 (k_bkt_dedupe_bm)
  bool tile_count = false;   // large flag scans: tile prefixes counted ahead, no look-back (GCZ_TILE_COUNT=1;
                             // measured 0.75 ms slower on tandem_3g2, neutral on uniform_1g: off)
  unsigned resolve_grid = 2048;   // node resolve: at most this many workgroups, striding (GCZ_RESOLVE_GRID;
                                 // 0: p / 256; 2048 measured -32 us uniform_1g, -0.25 ms tandem_3g2)
  gcz_host::DevBuf tcount;   // ... done counter (zeroed once: the last block resets it) + the prefixes
  bool bucket_now = true;    // this build (cleared after a bucket overflow: rebuild with the table)
  int dense_mode = 1;        // dense leaf level (gcz_dense.h): 0 off, 1 on large pure-ACGT inputs, 2 any size (GCZ_DENSE)
  gcz_host::u64 dense_min = 1ull << 21;   // ... from this many strands (mode 1)
  bool dense_used = false;   // the last build's leaf level ran dense
  bool dedupe_bm = true;     // two-pass levels: the bitmap dedupe k_bkt_dedupe_bm (+ k_bkt_dedupe2 for the
                             // buckets it hands back; GCZ_DEDUPE_BM=0: k_bkt_dedupe2 alone)
  // ... its code buckets (GCZ_DENSE_NB): 512 at L = 12 -- 2^14 codes per bucket (64 KB LDS tables,
  // two workgroups per CU) and runs of ~64 records per (chunk, bucket); 1024 measured 2.576 vs
  // 2.460 ms per 1 Gbase build (words 0.336 -> 0.308, first 0.257 -> 0.214, scatter 0.239 -> 0.208)
  gcz_host::u32 dense_nb = 512;
  // ... its chunk kernels walking XCD-contiguous chunk runs (GCZ_DL_XCD: DensePlan::xcd bits): the
  // scatter only -- measured 0.193 against 0.207 ms; words 0.488 against 0.307 and first (whose
  // input the scatter writes) 0.296 against 0.213 ms with every chunk kernel mapped
  gcz_host::u32 dl_xcd = 2;
  bool dl_fbw_on = true;      // k_dl_ids ranks through the interleaved bitmap (GCZ_DL_FBW=0: two lines a rank;
                              // measured ids 0.182 -> 0.164 ms for +7 us of interleaving)
  bool use_graph = true;     // small builds as a replayed HIP graph       (GCZ_GRAPH=0 disables)
  bool use_fused = true;     // small builds: two launches per node level  (GCZ_FUSED=0 disables)
  int small_cap_shift = 2;   // ... and tables 2^this times the usual size: short probe chains (GCZ_SMALL_CAP_SHIFT)
  int small_leaf_shift = -1; // ... the leaf table's own (GCZ_SMALL_LEAF_SHIFT; -1: small_cap_shift)
  int cap_boost = 0;         // (this build's node-table boost)
  // builds of more strands than this run as virtual ranks (always above 2^29 - 1;
  // GCZ_SPLIT_MIN lowers it for testing the split path on small genomes)
  gcz_host::u64 split_min_strands = ~0ull;
  gcz_host::u64 split_share = 1ull << 28;   // strands per virtual rank (GCZ_SPLIT_SHARE)
  // the next build's reader buffers of this many strands (gcz_build_*_fasta_buffered; 0: one
  // global level loop, which equals any power-of-two buffer)
  gcz_host::u64 segment_strands = 0;
  gcz_host::DevBuf seg_w, seg_nf, seg_mu;   // a level's input expanded at the segment ends
  gcz_host::DevBuf seg_in;                  // realigned bases after skipped reader buffers
  gcz_host::DevBuf ftab;     // ... their node tables, three rotating regions
  gcz_host::DevBuf fsid;     // ... and slot -> id of each table's repeated keys, three regions
  gcz_host::DevBuf flkey, flsid;   // ... the leaf level's canonical keys by position, ids by slot
  bool upload_warm = false;   // the runtime's host -> device path has run once (upload_reserve)
  int upload_reserve(size_t bytes);                     // input buffer of `bytes`, touched; the copy path warmed
  int upload(void* d_dst, const void* h_src, size_t n); // stream-ordered before later work on `stream`
  hipGraphExec_t graph_exec = nullptr;
  GraphKey graph_key{}, graph_seen{};
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
  std::vector<hipEvent_t> event_pool;
  size_t event_used = 0;
  gcz_host::u64 prof_launches[gcz_host::KID_COUNT] = {};
  double prof_ms[gcz_host::KID_COUNT] = {};
  std::vector<float> prof_trace;   // (kid, start ms after ev_start, duration ms) per profiled scope
  hipEvent_t ev_start = nullptr, ev_stop = nullptr;
  hipEvent_t ev_dfail = nullptr;   // the dense pack's verdict copied to the pinned header
  gcz_dist_state* dist = nullptr;   // multi-rank build state (gcz_dist.hip)
  gcz_sort_state* sortst = nullptr; // device sort / .dag writer state (gcz_sort.hip)
  gcz_ingest_state* ingest = nullptr; // device FASTA ingest state (gcz_ingest.hip)
  gcz_group* split = nullptr;         // virtual ranks of builds beyond 2^29 - 1 strands (gcz_dist.hip)

  int fail(int code, const char* what, const char* detail) {
    last_error = std::string(what) + ": " + detail;
    info.status = code;
    return code;
  }

  // GCZ_CANARY=1 (testing): every ensure()d buffer is allocated kCanaryBytes longer and the
  // extra bytes hold kCanaryByte; gcz_ctx_canary_check finds the bands a kernel overwrote (a GPU
  // store past a buffer's size, which faults only past the allocation's granule otherwise).
  static constexpr size_t kCanaryBytes = 4096;
  static constexpr unsigned char kCanaryByte = 0xA5;
  bool canary = false;
  std::vector<gcz_host::DevBuf*> canary_bufs;
  int ensure(gcz_host::DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes && b.ptr) return GCZ_OK;
    if (b.ptr) {
      HIP_TRY(hipStreamSynchronize(stream));
      HIP_TRY(hipFree(b.ptr));
      b.ptr = nullptr; b.bytes = 0;
    }
    const size_t n = bytes ? bytes : 16;
    HIP_TRY(hipMalloc(&b.ptr, n + (canary ? kCanaryBytes : 0)));
    b.bytes = n;
    if (canary) {
      HIP_TRY(hipMemsetAsync(static_cast<char*>(b.ptr) + n, kCanaryByte, kCanaryBytes, stream));
      if (std::find(canary_bufs.begin(), canary_bufs.end(), &b) == canary_bufs.end()) canary_bufs.push_back(&b);
    }
    return GCZ_OK;
  }
  // ensure() that leaves last_error / info.status alone: for work on a side thread beside
  // another call on this context (gcz_sort_reserve during gcz_fetch_host)
  hipError_t ensure_quiet(gcz_host::DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes && b.ptr) return hipSuccess;
    if (b.ptr) {
      if (hipError_t e = hipStreamSynchronize(stream)) return e;
      if (hipError_t e = hipFree(b.ptr)) return e;
      b.ptr = nullptr; b.bytes = 0;
    }
    if (hipError_t e = hipMalloc(&b.ptr, bytes ? bytes : 16)) return e;
    b.bytes = bytes ? bytes : 16;
    return hipSuccess;
  }

  hipEvent_t next_event() {
    if (event_used == event_pool.size()) {
      hipEvent_t e;
      (void)hipEventCreate(&e);
      event_pool.push_back(e);
    }
    return event_pool[event_used++];
  }
  void prof_begin(int, hipEvent_t& a) {
    if (!profile) return;
    a = next_event();
    (void)hipEventRecord(a, stream);
  }
  void prof_end(int kid, hipEvent_t a) {
    if (!profile) return;
    hipEvent_t b = next_event();
    (void)hipEventRecord(b, stream);
    pending.push_back({kid, {a, b}});
  }
  void prof_collect() {
    static const bool verbose = std::getenv("GCZ_PROFILE_VERBOSE") != nullptr;
    for (auto& pe : pending) {
      float ms = 0.f, t0 = -1.f;
      (void)hipEventElapsedTime(&ms, pe.second.first, pe.second.second);
      if (ev_start && hipEventElapsedTime(&t0, ev_start, pe.second.first) != hipSuccess) t0 = -1.f;
      if (prof_trace.size() < (1u << 16) * 3) {
        prof_trace.push_back(float(pe.first));
        prof_trace.push_back(t0);
        prof_trace.push_back(ms);
      }
      if (verbose) std::fprintf(stderr, "gcz-prof %s %.4f\n", gcz_host::kernel_name(pe.first), double(ms));
      prof_ms[pe.first] += ms;
      prof_launches[pe.first] += 1;
    }
    pending.clear();
    event_used = 0;
  }

  gcz_host::u64 node_cap(gcz_host::u64 p) const {   // load <= 2/3 (shift 0), 1/2 (1, default), 1/4 (2)
    using gcz_host::next_pow2;
    return std::max<gcz_host::u64>(256, next_pow2(node_cap_shift <= 0 ? p + p / 2 + 1 : p << node_cap_shift))
           << cap_boost;
  }
  // Marks buffers for levels of up to S elements (sets aligned for uchar2 loads).
  int ensure_marks(gcz_host::u64 S);
  int ensure_marks(gcz_host::u64 n0, gcz_host::u64 n1);   // set 0 / set 1 element counts

  int leaf_level(const gcz_host::LeafLevel& a, gcz_dev::Header* d_hdr);
  // The dense leaf level (pure-ACGT strands, L <= 12); *used = false when a strand is
  // not pure ACGT (the caller then runs leaf_level).  Writes a.words, a.out and the
  // unique count to *ucount.
  int leaf_level_dense(const gcz_host::LeafLevel& a, gcz_dev::Header* d_hdr, gcz_host::u64* ucount, bool* used);
  // ... in two phases (gcz_dist.hip exchanges in between): A = local first occurrences
  // (check: read the pure-ACGT flag on the host; list: first positions by code, the presence
  // bitmap and the status words vec only), B = ids (gid: by hashed code, null: local;
  // ids_done: the multi-rank ids kernel already wrote them) and words (leaves: write the
  // unique leaves, or null).
  int dense_phase_a(const gcz_host::LeafLevel& a, gcz_dev::Header* d_hdr, gcz_host::u64* ucount, bool check, bool list,
                    bool* used, gcz_host::u64* vec = nullptr,    // vec (list): the first exchange's status words
                    bool pack_only = false);                     // ... stop after the pack (dense_phase_a2 goes on)
  // the rest of phase A after a pack_only call: scan + scatter (a2), first positions (a3; list:
  // the presence bitmap and status words instead of the first bitmap and its scan)
  int dense_phase_a2(const gcz_host::LeafLevel& a);
  // (rfc / bcnt: the fused schedule's rank 0 -- its r-first lists straight from the first pass)
  int dense_phase_a3(gcz_dev::Header* d_hdr, gcz_host::u64* ucount, bool list, gcz_host::u64* vec,
                     gcz_host::u32* rfc = nullptr, gcz_host::u32* bcnt = nullptr);
  int dense_phase_b(const gcz_host::LeafLevel& a, gcz_dev::Header* d_hdr, const gcz_host::u32* gid,
                    gcz_host::u64* leaves, bool ids_done = false);
  int node_level(const gcz_host::NodeLevel& a, gcz_dev::Header* d_hdr);
  // Known-direct levels k0..k0+nlev-1 in one launch (gcz_device.h k_direct_levels).
  int direct_levels(const gcz_host::u32* in, int k0, int nlev, const gcz_dev::DirectPlan& dp, gcz_host::u32* out,
                    gcz_dev::Header* d_hdr, const gcz_dev::DirectRemap& rm = {},
                    const gcz_host::u64* guard = nullptr, gcz_host::u64 expect = 0);
  // Levels k0..D-1 in one launch (n0 <= kTailMaxN input words); writes counts and the root
  // (and, given the statistics shards, sums them: the build's last launch).
  int tail_levels(const gcz_host::u32* in, gcz_host::u64 n0, const gcz_host::u64* pcount, int k0, int D,
                  const std::vector<gcz_host::u64>& layer_off, gcz_dev::Header* d_hdr,
                  const gcz_host::u64* shards = nullptr, const gcz_dev::TailSettle& st = {});
  int build(const void* d_bases, const gcz_host::u64* d_leaves, gcz_host::u64 nbases, gcz_host::u64 S, int L);
};

// Times the launches of one scope on the context's stream (when profiling).
struct ProfScope {
  gcz_ctx* c;
  int kid;
  hipEvent_t e{};
  ProfScope(gcz_ctx* c_, int kid_) : c(c_), kid(kid_) { c->prof_begin(kid, e); }
  ~ProfScope() { c->prof_end(kid, e); }
};
