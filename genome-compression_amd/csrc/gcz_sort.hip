// Frequency sort, bytes() and the .dag writer on the device (SURVEY §8(f)
// rows 1-2).  Reference: shared_tree::histogram / sort_leaves / sort_nodes /
// sort_tree / rewire_nodes (src/shared_tree.cpp:316-483), bytes (:488-496),
// serialize (:504-513), pointer::serialize (:122-142); spec: SURVEY App. C.
//
// Net effect of sort_tree: every child layer (the leaves and node layers
// 0..D-2) is permuted independently by the reference counts its parent layer
// holds, descending, ties by the old index (std::stable_sort); parents are
// rewired with the m/t/v bits kept; the top layer and the root stay.  On the
// device:
//  * histogram per parent layer: a large layer that references each child many
//    times (the leaves) is partitioned by child-id range (2^15 ids per bucket: count
//    matrix, look-back scan, a scatter of 2-B records) and every bucket is counted by
//    one workgroup in LDS, which also reduces the layer's min / max count; other
//    layers count with global atomics (their references come in near id order);
//  * per child layer whose counts are not all equal (else the order is the
//    identity), a stable LSD counting sort of (hi - count) in passes of <= 8 bits:
//    per-tile digit counts, a scan, and a scatter whose in-tile ranks come from
//    wave ballots (a match mask per digit, so equal digits keep their order); the
//    last pass writes each element's new position directly;
//  * one pass over every node layer that rewires children and permutes the layer.
// The .dag is written by an exclusive scan of per-node byte sizes and one
// byte-scatter pass.
#include "gcz_ctx.h"
#include "gcz_scan.h"

using namespace gcz_dev;
using namespace gcz_host;

struct gcz_sort_state {
  DevBuf cnt, keys, keys2, vals, vals2, newpos, mm, tmp, sizes, pos, acc, dag, nodes2, leaves2, dw1, dw2, text;
  DevBuf hmat, hoff, hrec, desc;   // partitioned histogram; scan descriptors
  u32* h_mm = nullptr;
};

void gcz_sort_state_free(gcz_ctx* c) {
  gcz_sort_state* s = c->sortst;
  if (!s) return;
  for (DevBuf* b : {&s->cnt, &s->keys, &s->keys2, &s->vals, &s->vals2, &s->newpos, &s->mm, &s->tmp, &s->sizes,
                    &s->pos, &s->acc, &s->dag, &s->nodes2, &s->leaves2, &s->dw1, &s->dw2, &s->text, &s->hmat,
                    &s->hoff, &s->hrec, &s->desc})
    if (b->ptr) (void)hipFree(b->ptr);
  if (s->h_mm) (void)hipHostFree(s->h_mm);
  delete s;
  c->sortst = nullptr;
}

namespace {

constexpr u32 kSegStart1 = 16, kSegStart2 = 16 + 4096, kSegStart3 = 16 + 4096 + 1048576;

__device__ __forceinline__ bool is_null(u32 w) { return ulw(w) == kIdx; }

__device__ __forceinline__ u32 ptr_bytes(u32 w) {   // pointer::bytes, src/shared_tree.cpp:122-125
  const u32 i = w & kIdx;
  if (i == kIdx) return 4;
  return i < kSegStart1 ? 1 : i < kSegStart2 ? 2 : i < kSegStart3 ? 3 : 4;
}

// pointer::serialize (src/shared_tree.cpp:133-142)
__device__ __forceinline__ void put_ptr(unsigned char* o, u32 w) {
  const u32 idx = w & kIdx;
  u32 seg, off;
  if (idx == kIdx) { seg = 3; off = 0xfffffffu; }
  else if (idx < kSegStart1) { seg = 0; off = idx; }
  else if (idx < kSegStart2) { seg = 1; off = idx - kSegStart1; }
  else if (idx < kSegStart3) { seg = 2; off = idx - kSegStart2; }
  else { seg = 3; off = idx - kSegStart3; }
  const int bits = 4 + 8 * int(seg);
  int sh = bits - 4;
  *o++ = (unsigned char)((off >> sh) | (((w >> 29) & 1u) << 4) | (((w >> 30) & 1u) << 5) | (seg << 6));
  for (sh -= 8; sh >= 0; sh -= 8) *o++ = (unsigned char)(off >> sh);
}

__device__ __forceinline__ void put_be(unsigned char* o, u64 v, int nbytes) {   // binary_write, utility.h:178-184
  for (int i = nbytes - 1; i >= 0; --i) *o++ = (unsigned char)(v >> (8 * i));
}

// histogram (src/shared_tree.cpp:316-326): references of each child from the parent layer
__global__ __launch_bounds__(kBlock) void k_hist(const u32* __restrict__ parent, u64 nwords, u32* __restrict__ cnt) {
  const u64 i = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= nwords) return;
  const u32 w = parent[i];
  if (!is_null(w)) atomicAdd(&cnt[w & kIdx], 1u);
}

// ---- partitioned histogram (parent layers of >= 2^20 words) ----
// Buckets of 2^kHB child ids; chunks of kHChunk parent words (one count-matrix
// column each, dealt to XCDs in contiguous runs like the build's bucket chunks).
constexpr int kHThreads = 1024;
constexpr int kHItems = 64;
constexpr u64 kHChunk = u64(kHThreads) * kHItems;
constexpr u32 kHB = 15;                 // ids per bucket: 2^15 (LDS counters, 128 KB)
constexpr u32 kHMaxBuckets = 4096;      // child layers of <= 2^27 nodes (LDS cursors, 16 KB)

__device__ __forceinline__ u64 h_chunk(u64 G) {
  const u64 b = blockIdx.x, per = G / 8;
  return b < 8 * per ? (b % 8) * per + b / 8 : b;
}

__global__ __launch_bounds__(kHThreads) void k_hcount(const u32* __restrict__ words, u64 nw, u32 nb, u64 G,
                                                      u32* __restrict__ mat) {
  __shared__ u32 hist[kHMaxBuckets];
  for (u32 q = threadIdx.x; q < nb; q += kHThreads) hist[q] = 0;
  __syncthreads();
  const u64 g = h_chunk(G), j0 = g * kHChunk;
#pragma unroll 8
  for (int e = 0; e < kHItems; ++e) {
    const u64 j = j0 + u64(e) * kHThreads + threadIdx.x;
    if (j >= nw) break;
    const u32 w = words[j];
    if (!is_null(w)) atomicAdd(&hist[(w & kIdx) >> kHB], 1u);
  }
  __syncthreads();
  for (u32 q = threadIdx.x; q < nb; q += kHThreads) mat[u64(q) * G + g] = hist[q];
}

__global__ __launch_bounds__(kHThreads) void k_hscatter(const u32* __restrict__ words, u64 nw, u32 nb, u64 G,
                                                        const u32* __restrict__ off,
                                                        unsigned short* __restrict__ rec) {
  __shared__ u32 cur[kHMaxBuckets];
  const u64 g = h_chunk(G), j0 = g * kHChunk;
  for (u32 q = threadIdx.x; q < nb; q += kHThreads) cur[q] = off[u64(q) * G + g];
  __syncthreads();
#pragma unroll 8
  for (int e = 0; e < kHItems; ++e) {
    const u64 j = j0 + u64(e) * kHThreads + threadIdx.x;
    if (j >= nw) break;
    const u32 w = words[j];
    if (is_null(w)) continue;
    const u32 id = w & kIdx;
    const u32 d = atomicAdd(&cur[id >> kHB], 1u);
    rec[d] = (unsigned short)(id & ((1u << kHB) - 1));
  }
}

// One workgroup per bucket: LDS counters for its 2^kHB ids, written coalesced, and
// the block's min / max folded into mm[0..1].
__global__ __launch_bounds__(kHThreads) void k_hbucket(const unsigned short* __restrict__ rec,
                                                       const u32* __restrict__ off, u64 G, u64 nc,
                                                       u32* __restrict__ cnt, u32* __restrict__ mm) {
  extern __shared__ u32 c32[];   // 2^kHB counters (dynamic: 128 KB)
  __shared__ u32 smin[kHThreads / 64], smax[kHThreads / 64];
  const u64 b = blockIdx.x;
  for (u32 q = threadIdx.x; q < (1u << kHB); q += kHThreads) c32[q] = 0;
  __syncthreads();
  const u32 r0 = off[b * G], r1 = off[(b + 1) * G];
  for (u32 i = r0 + threadIdx.x; i < r1; i += kHThreads) atomicAdd(&c32[rec[i]], 1u);
  __syncthreads();
  u32 lo = ~0u, hi = 0;
  const u64 id0 = b << kHB;
  for (u32 q = threadIdx.x; q < (1u << kHB); q += kHThreads) {
    if (id0 + q >= nc) break;
    const u32 v = c32[q];
    cnt[id0 + q] = v;
    lo = min(lo, v);
    hi = max(hi, v);
  }
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, u32(__shfl_xor(int(lo), o, 64)));
    hi = max(hi, u32(__shfl_xor(int(hi), o, 64)));
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) { smin[wave] = lo; smax[wave] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kHThreads / 64; ++w) { lo = min(lo, smin[w]); hi = max(hi, smax[w]); }
    atomicMin(&mm[0], lo);
    atomicMax(&mm[1], hi);
  }
}

// ---- stable counting sort by count, descending (LSD passes of <= 8 bits) ----
// key = hi - count (ascending order <=> descending counts); a tile of kCsTile
// elements, each wave taking 1024 consecutive ones (item e of lane l: element
// e * 64 + l, in order), so ranks follow positions.
constexpr int kCsThreads = 256;
constexpr int kCsItems = 16;
constexpr u64 kCsWaveSpan = 64 * kCsItems;
constexpr u64 kCsTile = u64(kCsThreads) * kCsItems;

struct CsPass {
  const u32* cnt;      // first pass: counts (key = hi - cnt[i], value = i)
  const u32* keys;     // later passes: keys / values of the previous pass
  const u32* vals;
  u32 hi;
  u32 shift, bits;     // digit = (key >> shift) & (2^bits - 1)
  u64 n;
  __device__ __forceinline__ u32 key(u64 i) const { return cnt ? hi - cnt[i] : keys[i]; }
  __device__ __forceinline__ u32 val(u64 i) const { return cnt ? u32(i) : vals[i]; }
  __device__ __forceinline__ u32 digit(u32 k) const { return (k >> shift) & ((1u << bits) - 1u); }
};

__global__ __launch_bounds__(kCsThreads) void k_cs_count(CsPass P, u64 ntiles, u32* __restrict__ mat) {
  __shared__ u32 hist[256];
  const u32 R = 1u << P.bits;
  for (u32 q = threadIdx.x; q < R; q += kCsThreads) hist[q] = 0;
  __syncthreads();
  const u64 t = blockIdx.x, i0 = t * kCsTile;
#pragma unroll
  for (int e = 0; e < kCsItems; ++e) {
    const u64 i = i0 + u64(e) * kCsThreads + threadIdx.x;
    if (i < P.n) atomicAdd(&hist[P.digit(P.key(i))], 1u);
  }
  __syncthreads();
  for (u32 q = threadIdx.x; q < R; q += kCsThreads) mat[u64(q) * ntiles + t] = hist[q];
}

// off = exclusive scan of the digit-major matrix.  last pass: newpos[value] = rank;
// else keys_out / vals_out at the rank.
__global__ __launch_bounds__(kCsThreads) void k_cs_scatter(CsPass P, u64 ntiles, const u32* __restrict__ off,
                                                           u32* __restrict__ keys_out, u32* __restrict__ vals_out,
                                                           u32* __restrict__ newpos) {
  __shared__ u32 wc[kCsThreads / 64][256];
  const u32 R = 1u << P.bits;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (u32 q = threadIdx.x; q < R * (kCsThreads / 64); q += kCsThreads) wc[q / R][q % R] = 0;
  __syncthreads();
  const u64 t = blockIdx.x;
  const u64 w0 = t * kCsTile + u64(wave) * kCsWaveSpan;
  const u64 lt = (1ull << lane) - 1;
  u32 key[kCsItems], rank[kCsItems];
#pragma unroll
  for (int e = 0; e < kCsItems; ++e) {
    const u64 i = w0 + u64(e) * 64 + lane;
    const bool ok = i < P.n;
    key[e] = ok ? P.key(i) : 0u;
    const u32 d = P.digit(key[e]);
    u64 m = __ballot(ok);
    for (u32 b = 0; b < P.bits; ++b) {
      const u64 bal = __ballot((d >> b) & 1u);
      m &= ((d >> b) & 1u) ? bal : ~bal;
    }
    const u32 base = ok ? wc[wave][d] : 0u;
    rank[e] = base + u32(__popcll(m & lt));
    if (ok && (m & lt) == 0) wc[wave][d] = base + u32(__popcll(m));   // the lowest lane of the match
  }
  __syncthreads();
  for (u32 q = threadIdx.x; q < R; q += kCsThreads) {   // exclusive prefix over the waves, per digit
    u32 run = off[u64(q) * ntiles + t];
    for (int w = 0; w < kCsThreads / 64; ++w) {
      const u32 v = wc[w][q];
      wc[w][q] = run;
      run += v;
    }
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kCsItems; ++e) {
    const u64 i = w0 + u64(e) * 64 + lane;
    if (i >= P.n) continue;
    const u32 dst = wc[wave][P.digit(key[e])] + rank[e];
    if (newpos) newpos[P.val(i)] = dst;
    else {
      keys_out[dst] = key[e];
      vals_out[dst] = P.val(i);
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_minmax(const u32* __restrict__ cnt, u64 n, u32* __restrict__ mm) {
  __shared__ u32 smin[kBlock / 64], smax[kBlock / 64];
  u32 lo = ~0u, hi = 0;
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < n; i += u64(gridDim.x) * kBlock) {
    const u32 c = cnt[i];
    lo = min(lo, c);
    hi = max(hi, c);
  }
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, u32(__shfl_xor(int(lo), o, 64)));
    hi = max(hi, u32(__shfl_xor(int(hi), o, 64)));
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) { smin[wave] = lo; smax[wave] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kBlock / 64; ++w) { lo = min(lo, smin[w]); hi = max(hi, smax[w]); }
    atomicMin(&mm[0], lo);
    atomicMax(&mm[1], hi);
  }
}

__global__ void k_mm_init(u32* mm, int D) {
  for (int i = threadIdx.x; i < D; i += blockDim.x) { mm[2 * i] = ~0u; mm[2 * i + 1] = 0u; }
}

__global__ __launch_bounds__(kBlock) void k_perm_leaves(const u64* __restrict__ in, u64 n,
                                                        const u32* __restrict__ newpos, u64* __restrict__ out) {
  const u64 i = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) out[newpos[i]] = in[i];
}

// rewire_nodes (:383-403) with the child permutation and reorder_layer (:371-377) with
// the own one, for every node layer in one launch (storage slot g of layer k).
struct PermPlan {
  u64 node[GCZ_MAX_LAYERS + 1];     // storage start of each layer (+ the end)
  u64 count[GCZ_MAX_LAYERS];
  long long child[GCZ_MAX_LAYERS];  // offset of the child layer's newpos, -1: identity
  long long own[GCZ_MAX_LAYERS];    // offset of the layer's own newpos, -1: identity
};

__global__ __launch_bounds__(kBlock) void k_perm_nodes(const uint2* __restrict__ in, u64 N, int D, PermPlan pp,
                                                       const u32* __restrict__ newpos, uint2* __restrict__ out) {
  const u64 g = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= N) return;
  int k = 0;
  while (k + 1 < D && g >= pp.node[k + 1]) ++k;
  const u64 i = g - pp.node[k];
  if (i >= pp.count[k]) return;
  uint2 w = in[g];
  if (pp.child[k] >= 0) {
    const u32* cn = newpos + pp.child[k];
    if (!is_null(w.x)) w.x = (w.x & kBits) | cn[w.x & kIdx];
    if (!is_null(w.y)) w.y = (w.y & kBits) | cn[w.y & kIdx];
  }
  out[pp.node[k] + (pp.own[k] >= 0 ? newpos[pp.own[k] + i] : i)] = w;
}

struct LayerStarts {
  u64 node[GCZ_MAX_LAYERS + 1];   // storage start of each layer within the node buffer (+ the end)
  u64 count[GCZ_MAX_LAYERS];      // nodes of each layer (storage holds ceil(n/2) slots, count <= that)
};

__device__ __forceinline__ int layer_of(const LayerStarts& ls, int D, u64 g) {
  int k = 0;
  while (k + 1 < D && g >= ls.node[k + 1]) ++k;
  return k;
}

// Byte size of every storage slot (0 past a layer's node count) and their sum.
__global__ __launch_bounds__(kBlock) void k_node_sizes(const uint2* __restrict__ nodes, u64 n, LayerStarts ls, int D,
                                                       u32* __restrict__ sz, unsigned long long* __restrict__ acc) {
  __shared__ u32 part[kBlock / 64];
  const u64 i = u64(blockIdx.x) * kBlock + threadIdx.x;
  u32 b = 0;
  if (i < n) {
    const int k = layer_of(ls, D, i);
    if (i - ls.node[k] < ls.count[k]) {
      const uint2 w = nodes[i];
      b = ptr_bytes(w.x) + ptr_bytes(w.y);
    }
    if (sz) sz[i] = b;
  }
  for (int o = 32; o > 0; o >>= 1) b += u32(__shfl_xor(int(b), o, 64));
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = b;
  __syncthreads();
  if (threadIdx.x == 0) {   // line-padded shards (k_stats_sum): a few shared addresses would serialise
    u32 t = 0;
    for (int w = 0; w < kBlock / 64; ++w) t += part[w];
    if (t) atomicAdd(&acc[(blockIdx.x & (kStatShards - 1)) * kStatStride], (unsigned long long)t);
  }
}

__global__ __launch_bounds__(kBlock) void k_write_nodes(const uint2* __restrict__ nodes, u64 n,
                                                        const u64* __restrict__ pos, LayerStarts ls, int D, u64 hdr,
                                                        unsigned char* __restrict__ out) {
  const u64 g = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (g >= n) return;
  const int k = layer_of(ls, D, g);
  if (g - ls.node[k] >= ls.count[k]) return;
  unsigned char* o = out + hdr + 8 * u64(k + 1) + pos[g];
  const uint2 w = nodes[g];
  put_ptr(o, w.x);
  put_ptr(o + ptr_bytes(w.x), w.y);
}

__global__ __launch_bounds__(kBlock) void k_write_leaves(const u64* __restrict__ leaves, u64 n, int lb, u64 base,
                                                         unsigned char* __restrict__ out) {
  const u64 i = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) put_be(out + base + i * u64(lb), leaves[i], lb);
}

// root pointer, leaf count and every layer's count (its position needs the scan)
__global__ void k_write_headers(u32 root, u64 n_leaves, LayerStarts ls, int D, u64 hdr,
                                const u64* __restrict__ pos, const u32* __restrict__ sz, unsigned char* __restrict__ out) {
  put_ptr(out, root);
  put_be(out + ptr_bytes(root), n_leaves, 8);
  for (int k = 0; k < D; ++k) {
    const u64 g = ls.node[k];
    const u64 before = g < ls.node[D] ? pos[g] : (pos[ls.node[D] - 1] + sz[ls.node[D] - 1]);
    put_be(out + hdr + 8 * u64(k) + before, ls.count[k], 8);
  }
}

// ---- decompression ---------------------------------------------
// shared_tree::operator[] (src/shared_tree.cpp:268-291) for every index at once,
// top-down one layer per launch: a word w referencing node (l, r) of layer k
// stands for (M(r), M(l)) with w's transpose bit applied when w is mirrored,
// else (l, r) with it (the transform ctor, :76-80); access_leaf (:230-235)
// applies mirror / transpose to the canonical leaf.
__global__ __launch_bounds__(kBlock) void k_expand(const u32* __restrict__ w_in, u64 pw,
                                                   const uint2* __restrict__ layer, u32* __restrict__ w_out,
                                                   u64 nout) {
  const u64 j = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= pw) return;
  const u32 w = w_in[j];
  const uint2 nd = layer[w & kIdx];
  const u32 m = (w >> 29) & 1u, t = (w >> 30) & 1u;
  const u32 a = m ? xf(nd.y, 1, t) : xf(nd.x, 0, t);
  const u32 b = m ? xf(nd.x, 1, t) : xf(nd.y, 0, t);
  w_out[2 * j] = a;
  if (2 * j + 1 < nout) w_out[2 * j + 1] = b;
}

__constant__ char kSym[16] = {'S', 'A', 'C', 'R', 'G', 'B', 'N', 'K', 'T', 'W', 'V', 'D', 'Y', 'H', 'M', '-'};

// One strand per thread, staged through LDS so the text is stored coalesced.
__global__ __launch_bounds__(kBlock) void k_leaves_text(const u32* __restrict__ words, u64 S,
                                                        const u64* __restrict__ leaves, int L,
                                                        unsigned char* __restrict__ out) {
  __shared__ unsigned char buf[kBlock * 16];
  const u64 s0 = u64(blockIdx.x) * kBlock;
  const u64 s = s0 + threadIdx.x;
  if (s < S) {
    const u32 w = words[s];
    u64 v = leaves[w & kIdx];
    if ((w >> 29) & 1u) v = leaf_mirrored(v, L);
    if ((w >> 30) & 1u) v = leaf_transposed(v);
    for (int i = 0; i < L; ++i) buf[threadIdx.x * L + i] = (unsigned char)kSym[(v >> (4 * i)) & 15];
  }
  __syncthreads();
  const u64 nstr = S - s0 < u64(kBlock) ? S - s0 : u64(kBlock);
  for (u64 b = threadIdx.x; b < nstr * u64(L); b += kBlock) out[s0 * L + b] = buf[b];
}

dim3 grid_of(u64 n) { return dim3(unsigned(std::max<u64>(1, (n + kBlock - 1) / kBlock))); }

LayerStarts layer_starts(const gcz_ctx* c) {
  LayerStarts ls{};
  const int D = c->info.n_layers;
  for (int k = 0; k <= D; ++k) ls.node[k] = c->layer_off[k];
  for (int k = 0; k < D; ++k) ls.count[k] = c->info.layer_size[k];
  return ls;
}

u32 host_ptr_bytes(u32 w) {
  const u32 i = w & kIdx;
  if (i == kIdx) return 4;
  return i < kSegStart1 ? 1 : i < kSegStart2 ? 2 : i < kSegStart3 ? 3 : 4;
}

}  // namespace

#define S_HIP(x)                                                                         \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) return c->fail(GCZ_ERR_DEVICE, #x, hipGetErrorString(e_));     \
  } while (0)

extern "C" {

int gcz_sort_device(gcz_ctx* c) {
  if (!c || c->info.status != GCZ_OK || c->info.n_layers < 1) return GCZ_ERR_ARG;
  S_HIP(hipSetDevice(c->device));
  if (!c->sortst) c->sortst = new gcz_sort_state();
  gcz_sort_state& s = *c->sortst;
  const int D = c->info.n_layers;
  const u64 nl = c->info.n_leaves;
  // child layer cl: 0 = leaves (parent: node layer 0), cl = k + 1 = node layer k (parent: layer k + 1)
  std::vector<u64> n_of(D), coff(D + 1, 0);
  for (int cl = 0; cl < D; ++cl) {
    n_of[cl] = cl == 0 ? nl : c->info.layer_size[cl - 1];
    coff[cl + 1] = coff[cl] + n_of[cl];
  }
  u64 nmax = 0, nwmax = 0, matmax = 0, tilemax = 0;
  // per parent layer: partitioned histogram (nb buckets x G chunks) or global atomics (nb = 0)
  std::vector<u32> hnb(D, 0);
  std::vector<u64> hG(D, 0);
  for (int cl = 0; cl < D; ++cl) {
    nmax = std::max(nmax, n_of[cl]);
    const u64 nw = 2 * c->info.layer_size[cl];
    const u64 nb = (n_of[cl] + (1ull << kHB) - 1) >> kHB;
    // partition when parents reference their children many times over in random order (the
    // leaves: ~20 references each at 1 Gbase); a layer whose children are referenced about once
    // is referenced in near position order (ids are first occurrences), where atomics coalesce
    if (nw >= (1ull << 20) && nw >= 4 * n_of[cl] && nb >= 1 && nb <= kHMaxBuckets) {
      hnb[cl] = u32(nb);
      hG[cl] = (nw + kHChunk - 1) / kHChunk;
      nwmax = std::max(nwmax, nw);
      matmax = std::max(matmax, nb * hG[cl] + 1);
    }
  }
  const u64 cs_tiles = (nmax + kCsTile - 1) / kCsTile;
  matmax = std::max(matmax, 256 * cs_tiles + 1);
  tilemax = scan_tiles(matmax);
  const u64 N = c->layer_off[D];
  int rc;
  if ((rc = c->ensure(s.cnt, coff[D] * 4 + 16)) || (rc = c->ensure(s.newpos, coff[D] * 4 + 16)) ||
      (rc = c->ensure(s.keys, nmax * 4 + 16)) || (rc = c->ensure(s.keys2, nmax * 4 + 16)) ||
      (rc = c->ensure(s.vals, nmax * 4 + 16)) || (rc = c->ensure(s.vals2, nmax * 4 + 16)) ||
      (rc = c->ensure(s.mm, size_t(D) * 8 + 16)) || (rc = c->ensure(s.nodes2, N * 8 + 16)) ||
      (rc = c->ensure(s.leaves2, nl * 8 + 16)) || (rc = c->ensure(s.hmat, matmax * 4 + 16)) ||
      (rc = c->ensure(s.hoff, matmax * 4 + 16)) || (rc = c->ensure(s.hrec, nwmax * 2 + 16)) ||
      (rc = c->ensure(s.desc, tilemax * 8 + 16)))
    return rc;
  if (!s.h_mm) S_HIP(hipHostMalloc((void**)&s.h_mm, size_t(GCZ_MAX_LAYERS) * 8, hipHostMallocDefault));
  S_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_hbucket), hipFuncAttributeMaxDynamicSharedMemorySize,
                            int((1u << kHB) * 4)));
  hipEvent_t e0{};
  c->prof_begin(KID_SORT, e0);
  u32* cnt = s.cnt.as<u32>();
  u32* mm = s.mm.as<u32>();
  u32* mat = s.hmat.as<u32>();
  u32* off = s.hoff.as<u32>();
  u64* sdesc = s.desc.as<u64>();
  // exclusive scan of m matrix entries (+ the total at off[m])
  auto scan = [&](u64 m) -> int {
    const u64 t = scan_tiles(m + 1);
    S_HIP(hipMemsetAsync(sdesc, 0, t * 8 + 16, c->stream));
    hipLaunchKernelGGL(k_scan_excl<ScanU32>, dim3(unsigned(t)), dim3(kScanThreads), 0, c->stream, ScanU32{mat, m},
                       m + 1, off, sdesc, reinterpret_cast<u32*>(sdesc + t), static_cast<u64*>(nullptr));
    S_HIP(hipGetLastError());
    return GCZ_OK;
  };
  hipLaunchKernelGGL(k_mm_init, dim3(1), dim3(64), 0, c->stream, mm, D);   // [min, max] per child layer
  const uint2* nodes = c->nodes_out.as<uint2>();
  for (int cl = 0; cl < D; ++cl) {
    const u64 nw = 2 * c->info.layer_size[cl];   // words of parent layer cl
    const u32* words = reinterpret_cast<const u32*>(nodes + c->layer_off[cl]);
    if (hnb[cl]) {
      const u32 nb = hnb[cl];
      const u64 G = hG[cl];
      hipLaunchKernelGGL(k_hcount, dim3(unsigned(G)), dim3(kHThreads), 0, c->stream, words, nw, nb, G, mat);
      if ((rc = scan(u64(nb) * G))) return rc;
      hipLaunchKernelGGL(k_hscatter, dim3(unsigned(G)), dim3(kHThreads), 0, c->stream, words, nw, nb, G, off,
                         s.hrec.as<unsigned short>());
      hipLaunchKernelGGL(k_hbucket, dim3(nb), dim3(kHThreads), (1u << kHB) * 4, c->stream,
                         s.hrec.as<unsigned short>(), off, G, n_of[cl], cnt + coff[cl], mm + 2 * cl);
    } else {
      if (n_of[cl]) S_HIP(hipMemsetAsync(cnt + coff[cl], 0, n_of[cl] * 4, c->stream));
      if (nw)
        hipLaunchKernelGGL(k_hist, grid_of(nw), dim3(kBlock), 0, c->stream, words, nw, cnt + coff[cl]);
      if (n_of[cl])
        hipLaunchKernelGGL(k_minmax, dim3(unsigned(std::min<u64>(1024, (n_of[cl] + kBlock - 1) / kBlock))),
                           dim3(kBlock), 0, c->stream, cnt + coff[cl], n_of[cl], mm + 2 * cl);
    }
    S_HIP(hipGetLastError());
  }
  S_HIP(hipMemcpyAsync(s.h_mm, mm, size_t(D) * 8, hipMemcpyDeviceToHost, c->stream));
  S_HIP(hipStreamSynchronize(c->stream));
  std::vector<bool> ident(D);
  for (int cl = 0; cl < D; ++cl) ident[cl] = n_of[cl] <= 1 || s.h_mm[2 * cl] == s.h_mm[2 * cl + 1];
  // stable descending sort of (count, index) per non-trivial child layer: newpos[old] = new
  for (int cl = 0; cl < D; ++cl) {
    if (ident[cl]) continue;
    const u64 n = n_of[cl];
    const u32 lo = s.h_mm[2 * cl], hi = s.h_mm[2 * cl + 1];
    const u32 bits = bit_width(u64(hi - lo));
    const u32 npass = (bits + 7) / 8, db = (bits + npass - 1) / npass;
    const u64 nt = (n + kCsTile - 1) / kCsTile;
    u32 *kin = nullptr, *vin = nullptr, *kout = s.keys.as<u32>(), *vout = s.vals.as<u32>();
    for (u32 ps = 0; ps < npass; ++ps) {
      CsPass P{};
      P.cnt = ps == 0 ? cnt + coff[cl] : nullptr;
      P.keys = kin;
      P.vals = vin;
      P.hi = hi;
      P.shift = ps * db;
      P.bits = std::min(db, bits - ps * db);
      P.n = n;
      hipLaunchKernelGGL(k_cs_count, dim3(unsigned(nt)), dim3(kCsThreads), 0, c->stream, P, nt, mat);
      if ((rc = scan(u64(1u << P.bits) * nt))) return rc;
      const bool last = ps + 1 == npass;
      hipLaunchKernelGGL(k_cs_scatter, dim3(unsigned(nt)), dim3(kCsThreads), 0, c->stream, P, nt, off, kout, vout,
                         last ? s.newpos.as<u32>() + coff[cl] : nullptr);
      S_HIP(hipGetLastError());
      kin = kout;
      vin = vout;
      kout = kout == s.keys.as<u32>() ? s.keys2.as<u32>() : s.keys.as<u32>();
      vout = vout == s.vals.as<u32>() ? s.vals2.as<u32>() : s.vals.as<u32>();
    }
  }
  // apply: leaves, then every node layer (rewire children, permute itself)
  if (!ident[0] && nl) {
    hipLaunchKernelGGL(k_perm_leaves, grid_of(nl), dim3(kBlock), 0, c->stream, c->leaves_out.as<u64>(), nl,
                       s.newpos.as<u32>(), s.leaves2.as<u64>());
    std::swap(c->leaves_out, s.leaves2);
  }
  PermPlan pp{};
  for (int k = 0; k <= D; ++k) pp.node[k] = c->layer_off[k];
  for (int k = 0; k < D; ++k) {
    pp.count[k] = c->info.layer_size[k];
    pp.child[k] = ident[k] ? -1 : (long long)coff[k];
    pp.own[k] = (k + 1 < D && !ident[k + 1]) ? (long long)coff[k + 1] : -1;
  }
  hipLaunchKernelGGL(k_perm_nodes, grid_of(N), dim3(kBlock), 0, c->stream, nodes, N, D, pp, s.newpos.as<u32>(),
                     s.nodes2.as<uint2>());
  S_HIP(hipGetLastError());
  std::swap(c->nodes_out, s.nodes2);
  c->prof_end(KID_SORT, e0);
  S_HIP(hipStreamSynchronize(c->stream));
  return GCZ_OK;
}

int gcz_bytes_device(gcz_ctx* c, uint64_t* out) {
  if (!c || !out || c->info.status != GCZ_OK) return GCZ_ERR_ARG;
  S_HIP(hipSetDevice(c->device));
  if (!c->sortst) c->sortst = new gcz_sort_state();
  gcz_sort_state& s = *c->sortst;
  if (int rc = c->ensure(s.acc, kStatBytes + 8)) return rc;
  S_HIP(hipMemsetAsync(s.acc.ptr, 0, kStatBytes, c->stream));
  const int D = c->info.n_layers;
  const u64 N = c->layer_off[D];
  const LayerStarts ls = layer_starts(c);
  hipLaunchKernelGGL(k_node_sizes, grid_of(N), dim3(kBlock), 0, c->stream, c->nodes_out.as<uint2>(), N, ls, D,
                     nullptr, s.acc.as<unsigned long long>());
  u64* total = s.acc.as<u64>() + kStatBytes / 8;
  hipLaunchKernelGGL(k_stats_sum, dim3(1), dim3(1024), 0, c->stream, s.acc.as<u64>(), total);
  S_HIP(hipGetLastError());
  u64 nb = 0;
  S_HIP(hipMemcpyAsync(&nb, total, 8, hipMemcpyDeviceToHost, c->stream));
  S_HIP(hipStreamSynchronize(c->stream));
  *out = host_ptr_bytes(c->info.root) + 8 + c->info.n_leaves * u64((c->info.L + 1) / 2) +
         8 * u64(c->info.n_layers) + nb;
  return GCZ_OK;
}

// The .dag bytes into device memory (d_out == null: a context buffer); *written = size.
static int serialize_on_device(gcz_ctx* c, unsigned char** d_dag, uint64_t* written) {
  if (!c->sortst) c->sortst = new gcz_sort_state();
  gcz_sort_state& s = *c->sortst;
  uint64_t total = 0;
  if (int rc = gcz_bytes_device(c, &total)) return rc;
  const int D = c->info.n_layers;
  const u64 N = c->layer_off[D];
  int rc;
  if ((rc = c->ensure(s.sizes, N * 4 + 16)) || (rc = c->ensure(s.pos, N * 8 + 16)) ||
      (rc = c->ensure(s.dag, total + 16)))
    return rc;
  hipEvent_t e0{};
  c->prof_begin(KID_DAG, e0);
  S_HIP(hipMemsetAsync(s.acc.ptr, 0, kStatBytes, c->stream));
  const LayerStarts ls = layer_starts(c);
  hipLaunchKernelGGL(k_node_sizes, grid_of(N), dim3(kBlock), 0, c->stream, c->nodes_out.as<uint2>(), N, ls, D,
                     s.sizes.as<u32>(), s.acc.as<unsigned long long>());
  const u64 t = scan_tiles(N);   // u64 byte offsets (tile sums <= 8 * kScanTile)
  if ((rc = c->ensure(s.desc, std::max<u64>(s.desc.bytes, t * 8 + 16)))) return rc;
  S_HIP(hipMemsetAsync(s.desc.ptr, 0, t * 8 + 16, c->stream));
  hipLaunchKernelGGL((k_scan_excl<ScanU32, u64>), dim3(unsigned(std::max<u64>(t, 1))), dim3(kScanThreads), 0,
                     c->stream, ScanU32{s.sizes.as<u32>(), N}, N, s.pos.as<u64>(), s.desc.as<u64>(),
                     reinterpret_cast<u32*>(s.desc.as<u64>() + t), static_cast<u64*>(nullptr));
  S_HIP(hipGetLastError());
  const int lb = (c->info.L + 1) / 2;
  const u64 hdr = host_ptr_bytes(c->info.root) + 8 + c->info.n_leaves * u64(lb);
  unsigned char* out = s.dag.as<unsigned char>();
  hipLaunchKernelGGL(k_write_headers, dim3(1), dim3(1), 0, c->stream, c->info.root, c->info.n_leaves, ls, D, hdr,
                     s.pos.as<u64>(), s.sizes.as<u32>(), out);
  hipLaunchKernelGGL(k_write_leaves, grid_of(c->info.n_leaves), dim3(kBlock), 0, c->stream,
                     c->leaves_out.as<u64>(), c->info.n_leaves, lb, host_ptr_bytes(c->info.root) + 8, out);
  hipLaunchKernelGGL(k_write_nodes, grid_of(N), dim3(kBlock), 0, c->stream, c->nodes_out.as<uint2>(), N,
                     s.pos.as<u64>(), ls, D, hdr, out);
  S_HIP(hipGetLastError());
  c->prof_end(KID_DAG, e0);
  *d_dag = out;
  *written = total;
  return GCZ_OK;
}

int gcz_serialize_device(gcz_ctx* c, uint8_t* host_buf, uint64_t cap, uint64_t* written) {
  if (!c || !written || c->info.status != GCZ_OK) return GCZ_ERR_ARG;
  S_HIP(hipSetDevice(c->device));
  unsigned char* d = nullptr;
  uint64_t n = 0;
  if (int rc = serialize_on_device(c, &d, &n)) return rc;
  *written = n;
  if (!host_buf || cap < n) {
    S_HIP(hipStreamSynchronize(c->stream));
    return GCZ_ERR_ARG;
  }
  S_HIP(hipMemcpyAsync(host_buf, d, n, hipMemcpyDeviceToHost, c->stream));
  S_HIP(hipStreamSynchronize(c->stream));
  return GCZ_OK;
}

int gcz_decompress_device(gcz_ctx* c, void* d_out, uint64_t cap) {
  if (!c || !d_out || c->info.status != GCZ_OK || c->info.n_layers < 1) return GCZ_ERR_ARG;
  const u64 S = c->info.n_strands;
  const int L = c->info.L;
  if (cap < S * u64(L)) return GCZ_ERR_ARG;
  S_HIP(hipSetDevice(c->device));
  if (!c->sortst) c->sortst = new gcz_sort_state();
  gcz_sort_state& s = *c->sortst;
  if (int rc = c->ensure(s.dw1, S * 4 + 16)) return rc;
  if (int rc = c->ensure(s.dw2, S * 4 + 16)) return rc;
  const int D = c->info.n_layers;
  // element counts: the input of node layer k has n[k] words (n[0] = S), its output n[k + 1]
  std::vector<u64> n(D + 1);
  n[0] = S;
  for (int k = 0; k < D; ++k) n[k + 1] = (n[k] + 1) / 2;
  u32* cur = s.dw1.as<u32>();
  u32* nxt = s.dw2.as<u32>();
  S_HIP(hipMemcpyAsync(cur, &c->info.root, 4, hipMemcpyHostToDevice, c->stream));
  S_HIP(hipStreamSynchronize(c->stream));   // the root came from a host variable
  for (int k = D - 1; k >= 0; --k) {
    hipLaunchKernelGGL(k_expand, grid_of(n[k + 1]), dim3(kBlock), 0, c->stream, cur, n[k + 1],
                       c->nodes_out.as<uint2>() + c->layer_off[k], nxt, n[k]);
    std::swap(cur, nxt);
  }
  hipLaunchKernelGGL(k_leaves_text, grid_of(S), dim3(kBlock), 0, c->stream, cur, S, c->leaves_out.as<u64>(), L,
                     static_cast<unsigned char*>(d_out));
  S_HIP(hipGetLastError());
  S_HIP(hipStreamSynchronize(c->stream));
  return GCZ_OK;
}

int gcz_decompress(gcz_ctx* c, uint8_t* host_out, uint64_t cap) {
  if (!c || !host_out || c->info.status != GCZ_OK) return GCZ_ERR_ARG;
  const u64 n = c->info.n_strands * u64(c->info.L);
  if (cap < n) return GCZ_ERR_ARG;
  S_HIP(hipSetDevice(c->device));
  if (!c->sortst) c->sortst = new gcz_sort_state();
  if (int rc = c->ensure(c->sortst->text, n + 16)) return rc;
  if (int rc = gcz_decompress_device(c, c->sortst->text.ptr, n)) return rc;
  S_HIP(hipMemcpy(host_out, c->sortst->text.ptr, n, hipMemcpyDeviceToHost));
  return GCZ_OK;
}

const uint8_t* gcz_device_dag(gcz_ctx* c, uint64_t* written) {
  if (!c || !written || c->info.status != GCZ_OK || hipSetDevice(c->device) != hipSuccess) return nullptr;
  unsigned char* d = nullptr;
  if (serialize_on_device(c, &d, written)) return nullptr;
  return hipStreamSynchronize(c->stream) == hipSuccess ? d : nullptr;
}

}  // extern "C"
