// Dense leaf level: tree_constructor::emplace_leaf (src/shared_tree.cpp:630-637)
// for genomes whose strands are all A/C/G/T and L <= 12, without a hash table.
//
// A pure-ACGT strand is a 2L-bit code (A,C,G,T -> 0..3 keeps the numeric order
// of the nibble codes 1,2,4,8, so transposition is `x ^ mask`, mirroring a
// 2-bit-group reverse, and the canonical choice is the same as dna::canonical,
// src/dna.cpp:135-143).  Canonical codes live in [0, 4^L): the level is a
// bucketed sort, all LDS-resident, with no random HBM access per strand:
//
//   pack     one pass over the bases: canonical code c, m/t/v, hashed code
//            h = c*K mod 4^L (a bijection, balances the buckets); writes the
//            pre-word (h | m t v) per strand and a per-chunk histogram of the
//            NB buckets (h's top bits) -> count matrix, bucket-major.
//   scan     exclusive sum of the count matrix (gcz_scan.h), and its chunk-major
//            copy (k_dl_tr) for the per-chunk kernels.
//   scatter  per chunk of 32 Ki strands: records (h's low bits, position in
//            the chunk) staged in LDS by bucket, written as contiguous runs.
//   first    one workgroup per bucket: LDS table of the bucket's RB codes,
//            atomicMin of the position -> each key's first occurrence; sets
//            that position's bit in the first-occurrence bitmap FB.
//   fbscan   popcount prefix of FB words: ids = first-occurrence ranks
//            (the reference's parent.leaf_count() at emplace time).
//   ids      per bucket: the id of every present key (FB rank of its first
//            position) in LDS -> one id per record, bucket order.
//   words    per chunk: the chunk's records' ids back into position order in
//            LDS, + the pre-word's m/t/v -> final words; first occurrences
//            (FB bit) write their leaf, whose ids are consecutive in position order.
//
// Strands that are not pure ACGT (IUPAC, invalid symbols, L > 12) set
// hdr->dense_fail in the pack; the host then runs the hash-table leaf level.
#pragma once

#include <hip/hip_runtime.h>

#include "gcz_device.h"

namespace gcz_dev {

constexpr int kDLog = 15;
constexpr u32 kDC = 1u << kDLog;     // strands per chunk (positions in a chunk fit 15 bits)
constexpr int kDThreads = 1024;
constexpr u32 kDNBMax = 1024;        // buckets (h's top bits)

// Bits of the level's code space: a canonical 2-bit code is the minimum of an orbit that holds
// the code and its complement (x ^ cmask), which differ in the top bit, so its top bit is 0.
__host__ __device__ __forceinline__ u32 dense_code_bits(u32 L) { return 2 * L - 1; }

struct DensePlan {
  u64 S;
  u32 nch;     // chunks of kDC strands
  u32 L;
  u32 cmask;   // 4^L - 1 (the complement's mask)
  u32 hmask;   // 2^(2L-1) - 1: hashed codes (a canonical code's top bit is 0, dense_code_bits)
  u32 NB;      // buckets, power of two <= kDNBMax
  u32 IB;      // log2(codes per bucket) <= kDLog
  u32 K, Kinv; // odd multiplier mod 4^L and its inverse
  // the fused multi-rank schedule's sort and first pass, queued before its mid-build read: they
  // return at once when the pack found repetitive or non-ACGT data (that attempt is discarded)
  const Header* gate;
  u32 xcd;     // chunk kernels taking the XCD-contiguous chunk order (dl_chunk): bit 0 pack,
               // 1 scatter, 2 fb, 3 words; clear: chunk = block
};

// Chunk of a chunk kernel's workgroup (grid = nch).  Workgroups are dealt round-robin over the
// 8 XCDs, so with P.xcd each XCD takes a contiguous run of chunks, walked in order: the runs
// (chunk, bucket) and (chunk + 1, bucket) that share a line at their boundary, and the pack's
// count-matrix entries of neighbouring chunks, meet in one XCD's L2 instead of two.
template <u32 kBit>
__device__ __forceinline__ u32 dl_chunk(const DensePlan& P) {
  const u32 b = blockIdx.x, per = P.nch / 8;
  return (P.xcd & kBit) && b < 8 * per ? (b % 8) * per + b / 8 : b;
}

// The fused schedule's 6-byte layer-0 records (gcz_dist_fast.h): the canonical pair re-labelled
// by the children's canonical 2-bit codes -- a dna::canonical code is the minimum of its orbit,
// which holds a code and its complement (x ^ mask), so its top bit is 0: Bc = 2L - 1 bits --
// left child code | m, right child code | m | t (a canonical node's left child never carries t,
// include/shared_tree.h:119-126) = K = 2 Bc + 3 bits, mixed by a K-bit bijection h;
// owner = h's top lgR bits, record = the K - lgR bits below (<= 48).
struct PreKey {
  u32 on;                            // 0: 8-B raw keys
  u32 Kinv, cmask;                   // hashed code -> code
  u32 Bc, K, lgR;
  u32 sh;
  u64 kmask, c1, c2;                 // the mix (PackedTab::mix's form)
  __device__ __forceinline__ u64 mix(u64 x) const {   // (one multiply round: a bijection on K bits
    x ^= x >> sh; x = (x * c1) & kmask;                // that spreads the owner and partition bits;
    x ^= x >> sh;                                      // the owner's table mixes again on its own)
    return x;
  }
  __device__ __forceinline__ u64 label(u32 w) const {   // a child word -> code << 2 | m << 1 | t
    const u32 c = ((w & kIdx) * Kinv) & cmask;
    return (u64(c) << 2) | (((w >> 29) & 1u) << 1) | ((w >> 30) & 1u);   // (bit 29 mirror, 30 transpose)
  }
};

// the record key of a canonical pair (cl, cr) of pre-words: owner << 48 | the K - lgR bits
__device__ __forceinline__ void pre_key_of(const PreKey& pk, u32 cl, u32 cr, u64& key) {
  const u64 k = ((pk.label(cl) >> 1) << (pk.Bc + 2)) | pk.label(cr);   // (cl's t bit is 0)
  const u64 h = pk.mix(k);
  const u32 sh = pk.K - pk.lgR;
  key = ((h >> sh) << 48) | (h & ((1ull << sh) - 1ull));
}

// ACGT (any case) -> 0..3; other valid IUPAC symbols -> 4; unknown -> 5
static __device__ __forceinline__ int acgt_code(int c) {
  const int u = (c >= 'a' && c <= 'z') ? c - 32 : c;
  switch (u) {
    case 'A': return 0; case 'C': return 1; case 'G': return 2; case 'T': return 3;
    default: return nac_code(c) >= 0 ? 4 : 5;
  }
}

// reverse the L 2-bit groups of x (dna::mirrored on the 2-bit code, dna.cpp:116-121)
static __device__ __forceinline__ u32 rev2(u32 x, u32 L) {
  u32 r = __brev(x);
  r = ((r >> 1) & 0x55555555u) | ((r & 0x55555555u) << 1);
  return r >> (32 - 2 * L);
}

// dna::canonical on a 2-bit code: min over (x,F,F) (T,F,T) (M,T,F) (I,T,T) (dna.cpp:135-143)
static __device__ __forceinline__ u32 canon2(u32 x, u32 L, u32 cmask, u32& m, u32& t, u32& v) {
  const u32 tx = x ^ cmask, mx = rev2(x, L), ix = mx ^ cmask;
  v = x == mx;
  u32 best = x;
  m = 0; t = 0;
  if (tx < best) { best = tx; m = 0; t = 1; }
  if (mx < best) { best = mx; m = 1; t = 0; }
  if (ix < best) { best = ix; m = 1; t = 1; }
  return best;
}

// 2-bit code -> nibble-packed dna value (A,C,G,T = 1,2,4,8 at bits 4i, include/dna.h:20-32)
// (branch-free: the 2-bit groups spread to 4-bit slots, then one-hot per slot -- a loop over
// the L bases inside the words passes' divergent first-leaf branch cost ~30 us per launch)
static __device__ __forceinline__ u64 code2_leaf(u32 c, u32 L) {
  u64 x = c;
  x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
  x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
  x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x << 2)) & 0x3333333333333333ull;   // base i's 2 bits at bits 4i, 4i + 1
  const u64 M = 0x1111111111111111ull, lo = x & M, hi = (x >> 1) & M;
  const u64 v = (~hi & ~lo & M) | ((~hi & lo & M) << 1) | ((hi & ~lo & M) << 2) | ((hi & lo & M) << 3);
  return L >= 16 ? v : v & ((1ull << (4 * L)) - 1ull);
}

// Block-wide exclusive scan of one u32 per thread (kDThreads threads); returns
// the thread's exclusive prefix, *total = the block sum.  s_tmp: 16 u32.
static __device__ __forceinline__ u32 block_excl(u32 x, u32* s_tmp, u32* total) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  u32 incl = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u32 y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) s_tmp[wave] = incl;
  __syncthreads();
  u32 before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kDThreads / 64; ++w) {
    const u32 v = s_tmp[w];
    before += w < wave ? v : 0u;
    all += v;
  }
  *total = all;
  __syncthreads();
  return before + incl - x;
}

// The runs (b, ch) of one chunk: s_base[b] = local exclusive offset (s_base[NB] = the
// chunk's strands), s_dst[b] = the run's start in the record array.  offt: the run starts
// chunk-major (k_dl_tr), so a chunk reads two contiguous rows of NB words instead of a
// strided column of the bucket-major scan output.
static __device__ __forceinline__ void chunk_runs(const u32* __restrict__ offt, const DensePlan& P, u32 ch, u32* s_base,
                                           u32* s_dst, u32* s_tmp) {
  const u32 b = threadIdx.x;   // NB <= kDThreads
  u32 c = 0, d = 0;
  if (b < P.NB) {
    d = offt[u64(ch) * P.NB + b];
    c = offt[u64(ch + 1) * P.NB + b] - d;
  }
  u32 total;
  const u32 e = block_excl(c, s_tmp, &total);
  if (b < P.NB) {
    s_base[b] = e;
    s_dst[b] = d;
  }
  if (b == 0) s_base[P.NB] = total;
  __syncthreads();
}

// dst[c * rows + r] = src[r * stride + c] (r < rows, c < cols): a 32 x 32 tiled transpose
// through LDS, coalesced on both sides: the run starts, chunk-major copy of the scan's
// bucket-major output (rows = NB, cols = nch + 1, stride = nch -- column nch is a bucket's end
// = the next bucket's start).  (Tried for the pack's count matrix and k_dl_first's chunk
// offsets too: neutral, not kept.)
[[maybe_unused]] static __global__ __launch_bounds__(256) void k_dl_tr(const u32* __restrict__ src, u32 rows, u32 cols,
                                               u64 stride, u32* __restrict__ dst) {
  __shared__ u32 t[32][33];
  const u32 c0 = blockIdx.x * 32, r0 = blockIdx.y * 32, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (u32 i = ty; i < 32; i += 8) {
    const u32 r = r0 + i, c = c0 + tx;
    if (r < rows && c < cols) t[i][tx] = src[u64(r) * stride + c];
  }
  __syncthreads();
  for (u32 i = ty; i < 32; i += 8) {
    const u32 c = c0 + i, r = r0 + tx;
    if (r < rows && c < cols) dst[u64(c) * rows + r] = t[tx][i];
  }
}

constexpr int kDBatch = 8;   // strands / records in flight per thread

// L bytes of strand s from 4-B aligned loads (no LDS staging)
template <int L>
static __device__ __forceinline__ void load_strand(const unsigned char* __restrict__ bases, u64 s, u32 (&w)[4]) {
  const u64 a = s * L;
  const u32* p = reinterpret_cast<const u32*>(bases + (a & ~3ull));
  constexpr int NW = L % 4 == 0 ? L / 4 : (L + 3 + 3) / 4;   // (L % 4 == 0: every strand is 4-B aligned)
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = i < NW ? p[i] : 0u;
}

// Pack: the strand's pre-word make_word(h, m, t, v) and the chunk's bucket histogram.
// Bases: L bytes per strand (dna::dna(string_view), src/dna.cpp:79-84); leaves: u64.
// (zdesc / nz16: the dense level's scan descriptors, cleared here -- no memset launch)
template <int L, bool kBases>
[[maybe_unused]] static __global__ __launch_bounds__(kDThreads) void k_dl_pack(const unsigned char* __restrict__ bases,
                                                       const u64* __restrict__ leaves, DensePlan P,
                                                       u32* __restrict__ pw, u32* __restrict__ cnt,
                                                       Header* __restrict__ hdr, uint4* __restrict__ zdesc,
                                                       u64 nz16) {
  __shared__ u32 s_hist[kDNBMax];
  __shared__ signed char s_lut[256];
  const int tid = threadIdx.x;
  for (u64 i = u64(blockIdx.x) * kDThreads + tid; i < nz16; i += u64(gridDim.x) * kDThreads)
    zdesc[i] = make_uint4(0, 0, 0, 0);
  if (tid < 256) s_lut[tid] = (signed char)acgt_code(tid);
  for (u32 b = tid; b < P.NB; b += kDThreads) s_hist[b] = 0;
  const u32 ch = dl_chunk<1>(P);
  const u64 c0 = u64(ch) * kDC;
  const u32 ib = P.IB;
  bool fail = false;
  __syncthreads();
  for (u32 it = 0; it < kDC / kDThreads; it += kDBatch) {
    u32 w[kDBatch][4];
    u64 lv[kDBatch];
#pragma unroll
    for (int j = 0; j < kDBatch; ++j) {
      const u64 s = c0 + u64(it + j) * kDThreads + tid;
      if constexpr (kBases) {
        if (s < P.S) load_strand<L>(bases, s, w[j]);
      } else {
        lv[j] = s < P.S ? leaves[s] : 0ull;
      }
    }
#pragma unroll
    for (int j = 0; j < kDBatch; ++j) {
      const u64 s = c0 + u64(it + j) * kDThreads + tid;
      if (s >= P.S) continue;
      u32 x = 0;
      bool ok = true;
      if constexpr (kBases && L % 4 == 0) {
        // four bases a word in registers: code = ((b >> 1) ^ (b >> 2)) & 3 maps A C G T (either
        // case) to 0 1 2 3; the byte is ACGT iff (b | 0x20) is the lower-case letter of its code
        // (one byte permute of "acgt" by the codes)
#pragma unroll
        for (int q = 0; q < L / 4; ++q) {
          const u32 b = w[j][q];
          const u32 k = ((b >> 1) ^ (b >> 2)) & 0x03030303u;
          ok &= (b | 0x20202020u) == __builtin_amdgcn_perm(0u, 0x74676361u, k);
          const u32 t = k | (k >> 6);
          x |= ((t & 0xfu) | ((t >> 12) & 0xf0u)) << (8 * q);
        }
      } else if constexpr (kBases) {
        const u32 sh = u32(s * L) & 3u;
#pragma unroll
        for (int c = 0; c < L; ++c) {
          const u32 byte_i = sh + u32(c);
          const u32 ch = (w[j][byte_i >> 2] >> (8 * (byte_i & 3))) & 0xffu;
          const int k = s_lut[ch];
          ok &= k < 4;
          x |= u32(k & 3) << (2 * c);
        }
      } else {
        const u64 v = lv[j];
        if (L < 16 && (v >> (4 * L))) ok = false;
#pragma unroll
        for (int c = 0; c < L; ++c) {
          const u32 nib = u32(v >> (4 * c)) & 15u;
          ok &= nib != 0 && (nib & (nib - 1)) == 0;
          x |= u32(__ffs(nib) - 1) << (2 * c);
        }
      }
      fail |= !ok;
      if (ok) {
        u32 m, t, v;
        const u32 cc = canon2(x, L, P.cmask, m, t, v);
        const u32 h = (cc * P.K) & P.hmask;
        pw[s] = make_word(h, m, t, v);
        atomicAdd(&s_hist[h >> ib], 1u);
      } else {
        pw[s] = ~0u;   // (no pre-word is all ones: h < 2^24; the multi-rank scatter skips it)
      }
    }
  }
  if (__ballot(fail) && (tid & 63) == 0) atomicOr(&hdr->dense_fail, 1u);
  __syncthreads();
  for (u32 b = tid; b < P.NB; b += kDThreads) cnt[u64(b) * P.nch + ch] = s_hist[b];
}

// Scatter: records (h's low IB bits << kDLog | position in chunk, the pre-word's m/t/v in
// bits 29-31) in runs
// (chunk, bucket) at off[b * nch + chunk] of the bucket-ordered record array,
// staged in LDS so every run is written contiguously.
[[maybe_unused]] static __global__ __launch_bounds__(kDThreads) void k_dl_scatter(const u32* __restrict__ pw, DensePlan P,
                                                          const u32* __restrict__ offt, u32* __restrict__ rec) {
  if (P.gate && (P.gate->predup | P.gate->dense_fail)) return;
  extern __shared__ u32 s_dyn[];
  u32* s_stage = s_dyn;                 // kDC records
  u32* s_base = s_dyn + kDC;            // NB + 1: local exclusive offsets of the runs
  u32* s_cur = s_base + kDNBMax + 1;    // NB: cursors
  u32* s_dst = s_cur + kDNBMax;         // NB: global run starts
  u32* s_tmp = s_dst + kDNBMax;         // 16
  const int tid = threadIdx.x;
  const u32 ch = dl_chunk<2>(P);
  const u64 c0 = u64(ch) * kDC;
  const u32 n = u32(P.S - c0 < u64(kDC) ? P.S - c0 : u64(kDC));
  u32 h[kDC / kDThreads];   // pre-words: hashed code | m/t/v
#pragma unroll
  for (u32 j = 0; j < kDC / kDThreads; ++j) {   // every pre-word load in flight at once
    const u32 q = j * kDThreads + tid;
    h[j] = q < n ? pw[c0 + q] : 0u;
  }
  chunk_runs(offt, P, ch, s_base, s_dst, s_tmp);
  if (u32(tid) < P.NB) s_cur[tid] = s_base[tid];
  __syncthreads();
  const u32 imask = (1u << P.IB) - 1u;
#pragma unroll
  for (u32 j = 0; j < kDC / kDThreads; ++j) {
    const u32 q = j * kDThreads + tid;
    if (q < n && h[j] != ~0u) {   // (a strand the pack rejected: the multi-rank build runs on to the exchange)
      const u32 hc = h[j] & kIdx;
      const u32 slot = atomicAdd(&s_cur[hc >> P.IB], 1u);
      s_stage[slot] = ((hc & imask) << kDLog) | q | (h[j] & kBits);   // (IB + 15 <= 29 bits, then m/t/v)
    }
  }
  const int lane = tid & 63, wave = tid >> 6;
  // the staged runs written as flat 64-record groups (k_dl_words' walk), every lane busy
  {
    u32* s_gs = s_tmp + 16;   // group g -> the run holding record 64 g
    const u32 nrec = s_base[P.NB];
    for (u32 b = u32(tid); b < P.NB; b += kDThreads) {
      const u32 s1 = s_base[b + 1];
      for (u32 g = (s_base[b] + 63) >> 6; (g << 6) < s1; ++g) s_gs[g] = b;
    }
    __syncthreads();
    const u32 ng = (nrec + 63) >> 6;
    for (u32 g = wave; g < ng; g += kDThreads / 64) {
      const u32 k = (g << 6) + u32(lane);
      if (k >= nrec) continue;
      u32 b = s_gs[g];
      while (s_base[b + 1] <= k) ++b;
      rec[s_dst[b] + (k - s_base[b])] = s_stage[k];
    }
  }
}

// The records of bucket b, [off[b*nch], off[(b+1)*nch]), visited kDBatch per
// thread at a time; f(record, position).  Each group of consecutive chunks'
// runs is contiguous, so the chunk of a record is found among the group's run
// starts held in registers (broadcast by shuffles).
template <class F>
static __device__ __forceinline__ void bucket_records(const u32* __restrict__ rec, const u32* __restrict__ off,
                                               const DensePlan& P, u32 b, F f) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int G = 16;   // chunks per wave step
  const u64 row = u64(b) * P.nch;
  // run starts of chunks ch0.., and the end; the next step's are loaded with this step's records
  auto starts = [&](u32 ch0) {
    const u32 nc = P.nch - ch0 < u32(G) ? P.nch - ch0 : u32(G);
    return lane <= int(nc) ? off[row + ch0 + lane] : 0u;
  };
  u32 bnd = u32(wave) * G < P.nch ? starts(u32(wave) * G) : 0u;
  for (u32 ch0 = u32(wave) * G; ch0 < P.nch; ch0 += (kDThreads / 64) * G) {
    const u32 nc = P.nch - ch0 < u32(G) ? P.nch - ch0 : u32(G);
    const u32 r0 = __shfl(bnd, 0, 64), r1 = __shfl(bnd, int(nc), 64);
    const u32 nxt = ch0 + (kDThreads / 64) * G;
    const u32 bnd_next = nxt < P.nch ? starts(nxt) : 0u;
    u32 st[G];   // run starts of the group's chunks (past nc: never <= a record index)
#pragma unroll
    for (int g = 1; g < G; ++g) {
      const u32 v = __shfl(bnd, g, 64);
      st[g] = g < int(nc) ? v : ~0u;
    }
    for (u32 r = r0 + lane; r < r1; r += 64 * kDBatch) {
      u32 x[kDBatch];
#pragma unroll
      for (int j = 0; j < kDBatch; ++j) {
        const u32 rj = r + 64u * j;
        x[j] = rj < r1 ? rec[rj] : 0u;
      }
#pragma unroll
      for (int j = 0; j < kDBatch; ++j) {
        const u32 rj = r + 64u * j;
        if (rj >= r1) continue;
        u32 c = 0;   // chunks of the group whose run starts at or before rj, minus one
#pragma unroll
        for (int g = 1; g < G; ++g) c += st[g] <= rj ? 1u : 0u;
        f(x[j], rj, ((ch0 + c) << kDLog) | (x[j] & (kDC - 1)));
      }
    }
    bnd = bnd_next;
  }
}

// First occurrences: one workgroup per bucket; LDS table of its 2^IB codes.
// Writes each code's first position to fpg (~0 if absent), and the bucket's
// first positions sorted by chunk: fl[b * RB + ...], with fo[ch * NB + b] the start
// of chunk ch's (a counting sort in LDS; k_dl_fb gathers them per chunk).  pb
// (multi-rank build, else null): the presence bitmap, bit h set iff hashed code h occurs.
// fl null (multi-rank phase A): first positions and the presence bitmap only; block 0 also
// writes the status words vec = {pure-ACGT failure, 0, repetitive data} (settled by the pack
// and the probe before this launch).
// rfc (rank 0 of the fused multi-rank schedule, whose r-first codes are all its codes): also
// k_dl_rfirst's code-order list and per-bucket count (rfc[b * RB + j], bcnt[b]); fpg may be null.
[[maybe_unused]] static __global__ __launch_bounds__(kDThreads) __attribute__((amdgpu_waves_per_eu(8))) void k_dl_first(const u32* __restrict__ rec, const u32* __restrict__ off,
                                                        DensePlan P, u32* __restrict__ fpg, u32* __restrict__ fl,
                                                        u32* __restrict__ fo, unsigned long long* __restrict__ pb,
                                                        const Header* __restrict__ hdr = nullptr,
                                                        u64* __restrict__ vec = nullptr, u32* __restrict__ rfc = nullptr,
                                                        u32* __restrict__ bcnt = nullptr) {
  if (P.gate && (P.gate->predup | P.gate->dense_fail)) return;
  extern __shared__ u32 s_dyn[];
  u32* s_fp = s_dyn;                    // RB codes
  u32* s_cnt = s_dyn + (1u << P.IB);    // nch + 1 chunk counters
  __shared__ u32 s_tmp[16];
  const int tid = threadIdx.x;
  const u32 b = blockIdx.x, RB = 1u << P.IB;
  if (vec && b == 0 && tid == 0) {
    vec[0] = hdr->dense_fail;
    vec[1] = 0;
    vec[2] = hdr->predup;
  }
  for (u32 i = tid; i < RB; i += kDThreads) s_fp[i] = ~0u;
  for (u32 c = tid; c <= P.nch; c += kDThreads) s_cnt[c] = 0;
  __syncthreads();
  bucket_records(rec, off, P, b, [&](u32 x, u32, u32 pos) {
    const u32 idx = (x & kIdx) >> kDLog;
    if (s_fp[idx] > pos) atomicMin(&s_fp[idx], pos);
  });
  __syncthreads();
  // 16 codes per thread (RB <= 16 Ki).  The first positions stay in LDS (s_fp is only read from
  // here on) and each code's rank among the bucket's first positions of its chunk (< kDC) takes
  // half a register: the kernel fits 64 VGPRs, two workgroups per CU (fp[16] and rk[16] in
  // registers took 78, one per CU; measured the same 0.210 ms at 1 Gbase either way)
  constexpr int PER = 16;
  auto fp_of = [&](int k) { const u32 i = u32(k) * kDThreads + tid; return i < RB ? s_fp[i] : ~0u; };
  u32 rk2[PER / 2];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const u32 i = u32(k) * kDThreads + tid;
    const u32 fp = fp_of(k);
    if (fpg && i < RB) fpg[u64(b) * RB + i] = fp;
    const u32 rk = fl && fp != ~0u ? atomicAdd(&s_cnt[fp >> kDLog], 1u) : 0u;
    if (k & 1) rk2[k >> 1] |= rk << 16;
    else rk2[k >> 1] = rk;
    if (pb) {
      const u32 h = (b << P.IB) | i;
      if (RB >= 64) {
        const u64 m = __ballot(fp != ~0u);
        if ((tid & 63) == 0 && i < RB) pb[h >> 6] = m;
      } else if (fp != ~0u) {
        atomicOr(&pb[h >> 6], 1ull << (h & 63));
      }
    }
  }
  if (rfc) {   // code order = (k, wave, lane): exclusive prefix of the 256 (k, wave) counts
    __shared__ u32 s_wc[16 * (kDThreads / 64)];
    const int lane = tid & 63, wave = tid >> 6;
    u64 m[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      m[k] = __ballot(fp_of(k) != ~0u);
      if (lane == 0) s_wc[k * (kDThreads / 64) + wave] = u32(__popcll(m[k]));
    }
    __syncthreads();
    u32 total;
    const u32 e = block_excl(u32(tid) < 16u * (kDThreads / 64) ? s_wc[tid] : 0u, s_tmp, &total);
    if (u32(tid) < 16u * (kDThreads / 64)) s_wc[tid] = e;
    __syncthreads();
    const u64 lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const u32 fp = fp_of(k);
      if (fp != ~0u) rfc[u64(b) * RB + s_wc[k * (kDThreads / 64) + wave] + u32(__popcll(m[k] & lt))] = fp;
    }
    if (tid == 0) bcnt[b] = total;
  }
  if (!fl) return;
  __syncthreads();
  // exclusive scan of the nch + 1 counters (a few per thread, in order)
  const u32 n1 = P.nch + 1, per = (n1 + kDThreads - 1) / kDThreads, c0 = tid * per;
  u32 loc = 0;
  for (u32 c = c0; c < c0 + per && c < n1; ++c) loc += s_cnt[c];
  u32 total;
  u32 run = block_excl(loc, s_tmp, &total);
  for (u32 c = c0; c < c0 + per && c < n1; ++c) {
    const u32 v = s_cnt[c];
    s_cnt[c] = run;
    fo[u64(c) * P.NB + b] = run;
    run += v;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const u32 fp = fp_of(k);
    if (fp != ~0u) fl[u64(b) * RB + s_cnt[fp >> kDLog] + ((rk2[k >> 1] >> (16 * (k & 1))) & 0xffffu)] = fp;
  }
}

// First-occurrence bitmap of one chunk: its first positions from every bucket's
// sorted list (k_dl_first), set in LDS, written as the chunk's 512 bitmap words.
[[maybe_unused]] static __global__ __launch_bounds__(kDThreads) void k_dl_fb(const u32* __restrict__ fl, const u32* __restrict__ fo,
                                                     DensePlan P, unsigned long long* __restrict__ fb) {
  __shared__ u32 s_bits[kDC / 32];
  const int tid = threadIdx.x;
  const u32 ch = dl_chunk<4>(P), RB = 1u << P.IB;
  for (u32 w = tid; w < kDC / 32; w += kDThreads) s_bits[w] = 0;
  __syncthreads();
  for (u32 b = tid; b < P.NB; b += kDThreads) {
    const u32 o0 = fo[u64(ch) * P.NB + b], o1 = fo[u64(ch + 1) * P.NB + b];
    for (u32 k0 = o0; k0 < o1; k0 += 8) {   // 8 loads in flight
      u32 q[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) q[j] = k0 + j < o1 ? fl[u64(b) * RB + k0 + j] & (kDC - 1) : ~0u;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (q[j] != ~0u) atomicOr(&s_bits[q[j] >> 5], 1u << (q[j] & 31));
    }
  }
  __syncthreads();
  for (u32 w = tid; w < kDC / 64; w += kDThreads)
    fb[u64(ch) * (kDC / 64) + w] = u64(s_bits[2 * w]) | (u64(s_bits[2 * w + 1]) << 32);
}

struct ScanPopc {   // popcount of each first-occurrence bitmap word
  const unsigned long long* fb;
  __device__ __forceinline__ u32 operator()(u64 i) const { return u32(__popcll(fb[i])); }
};

static __device__ __forceinline__ u32 fb_rank(const unsigned long long* __restrict__ fb, const u32* __restrict__ wpre, u32 p) {
  const unsigned long long w = fb[p >> 6];
  return wpre[p >> 6] + u32(__popcll(w & ((1ull << (p & 63)) - 1ull)));
}

// The first-occurrence bitmap word and its popcount prefix side by side (16 B per 64 positions:
// {word lo, word hi, prefix, 0}), so a rank is one random line instead of two (k_dl_ids).
[[maybe_unused]] static __global__ __launch_bounds__(256) void k_dl_fbw(const unsigned long long* __restrict__ fb,
                                                                       const u32* __restrict__ wpre, u64 nfb,
                                                                       uint4* __restrict__ fbw) {
  const u64 w = u64(blockIdx.x) * 256 + threadIdx.x;
  if (w >= nfb) return;
  const unsigned long long b = fb[w];
  fbw[w] = make_uint4(u32(b), u32(b >> 32), wpre[w], 0u);
}
static __device__ __forceinline__ u32 fbw_rank(const uint4* __restrict__ fbw, u32 p) {
  const uint4 v = fbw[p >> 6];
  const unsigned long long w = (u64(v.y) << 32) | v.x;
  return v.z + u32(__popcll(w & ((1ull << (p & 63)) - 1ull)));
}

// Ids: per bucket, the id of each present code (rank of its first position)
// in LDS, then one final word (id | the record's m/t/v) per record in bucket order.
// gid (multi-rank build): the GLOBAL id of every code present on this rank,
// indexed by hashed code; null: ids are this build's first-occurrence ranks.
[[maybe_unused]] static __global__ __launch_bounds__(kDThreads) void k_dl_ids(const u32* __restrict__ rec, const u32* __restrict__ off,
                                                      DensePlan P, const u32* __restrict__ fpg,
                                                      const unsigned long long* __restrict__ fb,
                                                      const u32* __restrict__ wpre, const u32* __restrict__ gid,
                                                      u32* __restrict__ idrec, const uint4* __restrict__ fbw = nullptr) {
  extern __shared__ u32 s_id[];
  const int tid = threadIdx.x;
  const u32 b = blockIdx.x, RB = 1u << P.IB;
  constexpr int kFill = 16;   // codes per thread in flight (RB <= 16 Ki: one step)
  for (u32 i0 = 0; i0 < RB; i0 += kDThreads * kFill) {
    u32 fp[kFill];
#pragma unroll
    for (int j = 0; j < kFill; ++j) {
      const u32 i = i0 + u32(j) * kDThreads + tid;
      fp[j] = i < RB ? (gid ? gid : fpg)[u64(b) * RB + i] : ~0u;
    }
    if (fbw && !gid) {   // 8 ranks' lines in flight before the first is used (absent: line 0, unused)
#pragma unroll
      for (int h = 0; h < kFill; h += 8) {
        uint4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fbw[fp[h + j] == ~0u ? 0u : fp[h + j] >> 6];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const u32 i = i0 + u32(h + j) * kDThreads + tid, p = fp[h + j];
          const unsigned long long w = (u64(v[j].y) << 32) | v[j].x;
          if (i < RB) s_id[i] = p == ~0u ? 0u : v[j].z + u32(__popcll(w & ((1ull << (p & 63)) - 1ull)));
        }
      }
      continue;
    }
#pragma unroll
    for (int j = 0; j < kFill; ++j) {
      const u32 i = i0 + u32(j) * kDThreads + tid;
      if (i < RB) s_id[i] = gid ? fp[j] : fp[j] == ~0u ? 0u : fb_rank(fb, wpre, fp[j]);
    }
  }
  __syncthreads();
  const u64 row = u64(b) * P.nch;
  const u32 r0 = off[row], r1 = off[row + P.nch];
  for (u32 r = r0 + tid; r < r1; r += kDThreads * kDBatch) {
    u32 x[kDBatch];
#pragma unroll
    for (int j = 0; j < kDBatch; ++j) {
      const u32 rj = r + u32(j) * kDThreads;
      x[j] = rj < r1 ? rec[rj] : 0u;
    }
#pragma unroll
    for (int j = 0; j < kDBatch; ++j) {
      const u32 rj = r + u32(j) * kDThreads;
      if (rj < r1) idrec[rj] = s_id[(x[j] & kIdx) >> kDLog] | (x[j] & kBits);   // the final word
    }
  }
}

// Words: per chunk, the final words of its records (k_dl_ids, bucket order) back into
// position order in LDS, written out coalesced.  A record at a first occurrence (the
// chunk's first-occurrence bitmap, staged in LDS) emits its leaf from the record's code
// (bucket | the record's low code bits) at leaves_out[id - leaf_off]; leaf ids are the
// first-occurrence ranks (the multi-rank build: rank r's r-first positions, ids from off_r).
// dl_words_chunk does it all but the write-out: emit(s_w, n, c0) gets the chunk's n words in
// position order in LDS (after a barrier).
template <class Emit>
static __device__ __forceinline__ void dl_words_chunk(const u32* __restrict__ rec, const u32* __restrict__ idrec,
                                               const u32* __restrict__ offt, const DensePlan& P,
                                               const unsigned long long* __restrict__ fb, u64* __restrict__ leaves_out,
                                               u32 leaf_off, u32* s_dyn, Emit emit) {
  u32* s_w = s_dyn;                  // kDC final words by position in the chunk
  u32* s_base = s_dyn + kDC;         // NB + 1
  u32* s_dst = s_base + kDNBMax + 1; // NB
  u32* s_tmp = s_dst + kDNBMax;      // 16
  u32* s_fb = s_tmp + 16;            // kDC / 32 first-occurrence bits of the chunk
  u32* s_ex = s_fb + kDC / 32;       // kDC / 64: the run of each 64-record group's first record
  const int tid = threadIdx.x;
  const u32 ch = dl_chunk<8>(P);
  const u64 c0 = u64(ch) * kDC;
  const u32 n = u32(P.S - c0 < u64(kDC) ? P.S - c0 : u64(kDC));
  if (leaves_out)
    for (u32 w = tid; w < kDC / 64; w += kDThreads) {
      const u64 m = (c0 + u64(w) * 64 < P.S) ? fb[(c0 >> 6) + w] : 0ull;
      s_fb[2 * w] = u32(m);
      s_fb[2 * w + 1] = u32(m >> 32);
    }
  chunk_runs(offt, P, ch, s_base, s_dst, s_tmp);
  const int lane = tid & 63, wave = tid >> 6;
  const u32 IB = P.IB, imask = (1u << IB) - 1u;
  auto leaf = [&](u32 b, u32 xr, u32 wr) {   // one record at a first occurrence: its leaf
    const u32 q = xr & (kDC - 1);
    if ((s_fb[q >> 5] >> (q & 31)) & 1u) {
      const u32 h = (b << IB) | (((xr & kIdx) >> kDLog) & imask);
      leaves_out[(wr & kIdx) - leaf_off] = code2_leaf((h * P.Kinv) & P.hmask, P.L);
    }
  };
  // the chunk's records walked as one flat sequence of 64-record groups over the runs (every
  // lane busy: a group spans 2-3 runs of ~32 records), a group's first run looked up in LDS
  {
    u32* s_gs = s_ex;   // group g -> the run holding record 64 g
    const u32 nrec = s_base[P.NB];
    for (u32 b = u32(tid); b < P.NB; b += kDThreads) {
      const u32 s1 = s_base[b + 1];
      for (u32 g = (s_base[b] + 63) >> 6; (g << 6) < s1; ++g) s_gs[g] = b;
    }
    __syncthreads();
    const u32 ng = (nrec + 63) >> 6;
    constexpr int GW = 8;   // groups per wave step (2 loads each in flight per lane; 16: -4 us, 32: +14 us)
    for (u32 g0 = wave; g0 < ng; g0 += (kDThreads / 64) * GW) {
      u32 x[GW], w[GW], bq[GW];
#pragma unroll
      for (int q = 0; q < GW; ++q) {
        const u32 g = g0 + u32(q) * (kDThreads / 64), k = (g << 6) + u32(lane);
        bq[q] = ~0u;
        x[q] = w[q] = 0;
        if (g < ng && k < nrec) {
          u32 b = s_gs[g];
          while (s_base[b + 1] <= k) ++b;
          const u32 at = s_dst[b] + (k - s_base[b]);
          x[q] = rec[at];
          w[q] = idrec[at];
          bq[q] = b;
        }
      }
      // the loads waited for once, unconditionally: waits inside the per-record branches below
      // also waited for the leaf stores issued before them (one vmcnt for loads and stores)
#pragma unroll
      for (int q = 0; q < GW; ++q) asm volatile("" ::"v"(x[q]), "v"(w[q]));
#pragma unroll
      for (int q = 0; q < GW; ++q)
        if (bq[q] != ~0u) s_w[x[q] & (kDC - 1)] = w[q];
      if (leaves_out)
#pragma unroll
        for (int q = 0; q < GW; ++q)
          if (bq[q] != ~0u) leaf(bq[q], x[q], w[q]);
    }
    __syncthreads();
    emit(s_w, n, c0);
  }
}

[[maybe_unused]] static __global__ __launch_bounds__(kDThreads) void k_dl_words(const u32* __restrict__ rec,
                                                        const u32* __restrict__ idrec, const u32* __restrict__ offt,
                                                        DensePlan P, const unsigned long long* __restrict__ fb,
                                                        u32* __restrict__ words, u64* __restrict__ leaves_out,
                                                        u32 leaf_off = 0) {
  extern __shared__ u32 s_dyn[];
  dl_words_chunk(rec, idrec, offt, P, fb, leaves_out, leaf_off, s_dyn, [&](const u32* s_w, u32 n, u64 c0) {
    for (u32 q = threadIdx.x; q < n; q += kDThreads) words[c0 + q] = s_w[q];
  });
}

// ---- multi-rank build (gcz_dist.hip): the leaf level of one rank ----------------
//
// A key's global first occurrence is on the lowest rank holding it (rank order = position
// order), so with every rank's presence bitmap (one allgather) rank r knows its "r-first"
// keys (held by no lower rank); their global ids are off_r + their rank among rank r's
// r-first positions, off_r = the r-first counts of lower ranks.  Per code bucket:
//
//   phase A  pack, scan, scatter, first (local first position per code, presence bitmap)
//   -- allgather the presence bitmaps (+ status words) --
//   rfirst   per bucket: the r-first codes (present here, in no lower rank's bitmap), their
//            first positions by chunk (fl/fo, as the single-device first) and in code order
//            (rfc), and the bucket's count
//   fb, scan the r-first position bitmap and its popcount prefix: local r-first ranks
//   gq       per bucket: G[bucket prefix + j] = the local rank of the bucket's j-th r-first
//            code in CODE order; the bucket prefixes ride in the exchange vector
//   -- allgather the exchange vectors (r-first count + bucket prefixes); relay the G arrays --
//            (a rank with few r-first codes writes its leaves here too)
//   ids      per bucket: the global id of every code present here in LDS -- for each lower
//            rank q (and r itself) the codes q holds first are present_q & ~(present_0 | ..
//            | present_{q-1}); a code's index among them in the bucket is a popcount prefix of
//            those bitmap words, so its id is off_q + G_q[prefix_q(b) + index]: no code-indexed
//            id table, no list in id order -- then one final word per record
//   words    as single-device; leaves: rank r's r-first codes in position order.

// Bits [64 lw, 64 lw + 64) of bucket b's codes in bitmap bm (RB < 64: the bucket's RB bits).
static __device__ __forceinline__ u64 bucket_word(const unsigned long long* __restrict__ bm, u32 b, u32 IB, u32 lw) {
  const u64 h0 = u64(b) << IB;
  if (IB >= 6) return bm[(h0 >> 6) + lw];
  return (bm[h0 >> 6] >> (h0 & 63)) & ((1ull << (1u << IB)) - 1ull);
}

// r-first codes of each bucket: fl/fo by chunk (k_dl_fb builds the position bitmap), rfc in
// code order (rfc[b * RB + j]), bcnt[b].  pbs: the R gathered presence bitmaps (stride words).
[[maybe_unused]] static __global__ __launch_bounds__(kDThreads) void k_dl_rfirst(const u32* __restrict__ fpg, DensePlan P,
                                                         const unsigned long long* __restrict__ pbs, u64 stride, int r,
                                                         u32* __restrict__ fl, u32* __restrict__ fo,
                                                         u32* __restrict__ rfc, u32* __restrict__ bcnt) {
  extern __shared__ u32 s_cnt[];   // nch + 1 chunk counters
  __shared__ u64 s_low[256];       // OR of the lower ranks' words of this bucket
  __shared__ u32 s_wc[16 * (kDThreads / 64)];   // r-first codes per (k, wave), then their prefix
  __shared__ u32 s_tmp[16];
  constexpr int PER = 16;          // codes per thread: i = k * kDThreads + tid (coalesced loads, RB <= 16 Ki)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const u32 b = blockIdx.x, RB = 1u << P.IB, NW = RB >= 64 ? RB / 64 : 1u;
  for (u32 c = tid; c <= P.nch; c += kDThreads) s_cnt[c] = 0;
  for (u32 lw = tid; lw < NW; lw += kDThreads) {
    u64 x = 0;
    for (int q = 0; q < r; ++q) x |= bucket_word(pbs + u64(q) * stride, b, P.IB, lw);
    s_low[lw] = x;
  }
  u32 fp[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const u32 i = u32(k) * kDThreads + tid;
    fp[k] = i < RB ? fpg[u64(b) * RB + i] : ~0u;
  }
  __syncthreads();
  u32 rk[PER];
  u64 m[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const u32 i = u32(k) * kDThreads + tid;
    if (fp[k] != ~0u && ((s_low[i >> 6] >> (i & 63)) & 1ull)) fp[k] = ~0u;   // held by a lower rank
    rk[k] = fp[k] != ~0u ? atomicAdd(&s_cnt[fp[k] >> kDLog], 1u) : 0u;
    m[k] = __ballot(fp[k] != ~0u);
    if (lane == 0) s_wc[k * (kDThreads / 64) + wave] = u32(__popcll(m[k]));
  }
  __syncthreads();
  u32 total;   // code order = (k, wave, lane): exclusive prefix of the 256 (k, wave) counts
  const u32 e = block_excl(u32(tid) < 16u * (kDThreads / 64) ? s_wc[tid] : 0u, s_tmp, &total);
  if (u32(tid) < 16u * (kDThreads / 64)) s_wc[tid] = e;
  __syncthreads();
  const u64 lt = (1ull << lane) - 1ull;
#pragma unroll
  for (int k = 0; k < PER; ++k)
    if (fp[k] != ~0u) rfc[u64(b) * RB + s_wc[k * (kDThreads / 64) + wave] + u32(__popcll(m[k] & lt))] = fp[k];
  if (tid == 0) bcnt[b] = total;
  // exclusive scan of the nch + 1 chunk counters (a few per thread, in order)
  const u32 n1 = P.nch + 1, per = (n1 + kDThreads - 1) / kDThreads, c0 = tid * per;
  u32 loc = 0;
  for (u32 c = c0; c < c0 + per && c < n1; ++c) loc += s_cnt[c];
  u32 run = block_excl(loc, s_tmp, &total);
  for (u32 c = c0; c < c0 + per && c < n1; ++c) {
    const u32 v = s_cnt[c];
    s_cnt[c] = run;
    fo[u64(c) * P.NB + b] = run;
    run += v;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PER; ++k)
    if (fp[k] != ~0u) fl[u64(b) * RB + s_cnt[fp[k] >> kDLog] + rk[k]] = fp[k];
}

// G: per bucket, the local r-first rank of each r-first code in code order, at the bucket's
// prefix; xv = the rank's exchange vector {r-first count, status, prefix of bucket 0, 1, ...}
// (status: bit 0 a non-ACGT strand, bit 1 repetitive data; the host adds bit 2, failed).
// A rank with few r-first codes (dl_rleaves_sparse: count * 4 < S) writes its leaves here,
// by rank (random stores of few entries), instead of a pass over every position (k_dl_rleaves;
// at 1 Gbase over 8 ranks rank 1 first-holds ~0.7 M of its 10.9 M strands' codes: 41 us there).
__host__ __device__ __forceinline__ bool dl_rleaves_sparse(u64 count, u64 S) { return count * 4 < S; }
[[maybe_unused]] static __global__ __launch_bounds__(kDThreads) void k_dl_gq(const u32* __restrict__ rfc, const u32* __restrict__ bcnt,
                                                     DensePlan P, const unsigned long long* __restrict__ rfb,
                                                     const u32* __restrict__ wpre, const u64* __restrict__ ucount,
                                                     u32* __restrict__ G, u32* __restrict__ xv,
                                                     const u32* __restrict__ pw, u64* __restrict__ leaves_out,
                                                     const u64* __restrict__ status) {
  __shared__ u32 s_tmp[16];
  const int tid = threadIdx.x;
  const u32 b = blockIdx.x, RB = 1u << P.IB;
  u32 pre;   // sum over the buckets before b (NB <= kDThreads)
  (void)block_excl(u32(tid) < b ? bcnt[tid] : 0u, s_tmp, &pre);
  if (tid == 0) {
    xv[2 + b] = pre;
    if (b == 0) {   // the r-first count and the phase-A status words (k_dl_first's vec)
      xv[0] = u32(*ucount);
      xv[1] = (status[0] ? 1u : 0u) | (status[2] ? 2u : 0u);
    }
  }
  const u32 n = bcnt[b];
  const bool lv = leaves_out && dl_rleaves_sparse(*ucount, P.S);
  constexpr int kQ = 4;   // codes per thread in flight (the rank lookups are random L2 reads)
  for (u32 j0 = tid; j0 < n; j0 += kQ * kDThreads) {
    u32 fp[kQ];
    unsigned long long w[kQ];
    u32 wp[kQ];
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      const u32 j = j0 + u32(q) * kDThreads;
      fp[q] = j < n ? rfc[u64(b) * RB + j] : 0u;
    }
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      const u32 j = j0 + u32(q) * kDThreads;
      w[q] = j < n ? rfb[fp[q] >> 6] : 0ull;
      wp[q] = j < n ? wpre[fp[q] >> 6] : 0u;
    }
#pragma unroll
    for (int q = 0; q < kQ; ++q) {
      const u32 j = j0 + u32(q) * kDThreads;
      if (j >= n) continue;
      const u32 k = wp[q] + u32(__popcll(w[q] & ((1ull << (fp[q] & 63)) - 1ull)));   // fb_rank
      G[pre + j] = k;
      if (lv) leaves_out[k] = code2_leaf(((pw[fp[q]] & kIdx) * P.Kinv) & P.hmask, P.L);
    }
  }
}

// The relay (gcz_dist.hip) leaves piece p = [c_q p / R, c_q (p+1) / R) of every list q at
// seg_src[q R + p] of the receive buffer; in global id order that piece starts at
// seg_dst[q R + p] = off_q + c_q p / R.
constexpr int kDlMaxRanks = 31;
struct DlRelay {
  u64 off[kDlMaxRanks + 1];                     // global id offsets (r-first counts of lower ranks)
  u64 seg_src[kDlMaxRanks * kDlMaxRanks];       // piece starts in the relay's receive buffer
  u64 seg_dst[kDlMaxRanks * kDlMaxRanks];       // ... and by global id
  u64 seg_len[kDlMaxRanks * kDlMaxRanks];
};

// Global ids of every code present on rank r (LDS), then one final word per record.  pbs /
// xvs: the gathered presence bitmaps (stride words) and exchange vectors (xstride u32); gl: the
// relay's receive buffer.  Codes: 16 contiguous per thread (a quarter word).
// The G arrays are read where the relay left them (T's pieces: list q's element at global id
// position off_q + k lies in the piece p with seg_dst <= off_q + k < seg_dst + seg_len).
// (dl_ids_mr_block: one workgroup's bucket b; k_dl_ids_mr launches one per bucket)
static __device__ __forceinline__ void dl_ids_mr_block(const u32* __restrict__ rec, const u32* __restrict__ off,
                                                       const DensePlan& P, const unsigned long long* __restrict__ pbs,
                                                       u64 stride, const u32* __restrict__ xvs, u64 xstride,
                                                       const u32* __restrict__ gl, const DlRelay* __restrict__ T,
                                                       int R, int r, u32* __restrict__ idrec, u32 b) {
  extern __shared__ u32 s_id[];    // RB
  // ranks q <= r in rounds of QB: their words, first-held words and prefixes loaded and
  // scanned together (one load round trip and two barriers per round, not per rank)
  constexpr int QB = 4;
  __shared__ u64 s_rf[QB][256];
  __shared__ u32 s_pf[QB][256];
  __shared__ u64 s_sdst[QB][kDlMaxRanks + 1], s_ssrc[QB][kDlMaxRanks], s_base[QB];
  __shared__ u32 s_wt[QB][4];
  __shared__ u64 s_mine[256];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const u32 RB = 1u << P.IB, NW = RB >= 64 ? RB / 64 : 1u;
  u64 acc = 0;   // (threads < NW: the OR of the words of the ranks before this round)
  if (u32(tid) < NW) s_mine[tid] = bucket_word(pbs + u64(r) * stride, b, P.IB, tid);
  const u32 lw = u32(tid) >> 2, sh = (u32(tid) & 3u) * 16u;   // this thread's codes: 16 tid .. 16 tid + 15
  for (int q0 = 0; q0 <= r; q0 += QB) {
    const int nq = r + 1 - q0 < QB ? r + 1 - q0 : QB;
    if (tid < nq * R) {   // the lists' pieces, by global id position
      const int i = tid / R, pp = tid % R;
      s_sdst[i][pp] = T->seg_dst[u64(q0 + i) * R + pp];
      s_ssrc[i][pp] = T->seg_src[u64(q0 + i) * R + pp];
    }
    if (tid < nq) {
      s_sdst[tid][R] = T->off[q0 + tid + 1];
      s_base[tid] = T->off[q0 + tid] + xvs[u64(q0 + tid) * xstride + 2 + b];
    }
    u32 pc[QB], inc[QB];
    if (u32(tid) < NW) {
      u64 w[QB];
#pragma unroll
      for (int i = 0; i < QB; ++i) w[i] = i < nq ? bucket_word(pbs + u64(q0 + i) * stride, b, P.IB, tid) : 0ull;
#pragma unroll
      for (int i = 0; i < QB; ++i) {
        const u64 rf = w[i] & ~acc;
        acc |= w[i];
        s_rf[i][tid] = rf;
        pc[i] = u32(__popcll(rf));
      }
    } else {
#pragma unroll
      for (int i = 0; i < QB; ++i) pc[i] = 0;
    }
    if (wave < 4) {   // (NW <= 256: the first four waves) inclusive wave scans, wave totals
#pragma unroll
      for (int i = 0; i < QB; ++i) {
        u32 v = pc[i];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const u32 y = __shfl_up(v, o, 64);
          if (lane >= o) v += y;
        }
        inc[i] = v;
        if (lane == 63) s_wt[i][wave] = v;
      }
    }
    __syncthreads();
    if (u32(tid) < NW) {
#pragma unroll
      for (int i = 0; i < QB; ++i) {
        u32 pre = inc[i] - pc[i];
        for (int w2 = 0; w2 < wave; ++w2) pre += s_wt[i][w2];
        s_pf[i][tid] = pre;
      }
    }
    __syncthreads();
    if (16u * u32(tid) < RB) {   // codes first held by q: id = off_q + G_q[prefix_q(b) + index]
      const u32 mw = u32(s_mine[lw] >> sh) & 0xffffu;   // (codes not held here need no id)
      for (int i = 0; i < nq; ++i) {
        const u64 rfw = s_rf[i][lw];
        u32 win = u32(rfw >> sh) & mw;
        if (!win) continue;
        const u64 base = s_base[i] + s_pf[i][lw];
        const u32 qo = u32(T->off[q0 + i]);
        int pc2 = 0;   // the piece holding the window's first id position, then onwards
        while (win) {
          const u32 j = u32(__ffs(int(win))) - 1u;
          win &= win - 1u;
          const u64 g = base + u64(__popcll(rfw & ((1ull << (sh + j)) - 1ull)));
          while (pc2 + 1 < R && s_sdst[i][pc2 + 1] <= g) ++pc2;
          s_id[16u * u32(tid) + j] = qo + gl[s_ssrc[i][pc2] + (g - s_sdst[i][pc2])];
        }
      }
    }
    __syncthreads();
  }
  const u64 row = u64(b) * P.nch;
  const u32 r0 = off[row], r1 = off[row + P.nch];
  for (u32 x0 = r0 + tid; x0 < r1; x0 += kDThreads * kDBatch) {
    u32 x[kDBatch];
#pragma unroll
    for (int j = 0; j < kDBatch; ++j) {
      const u32 rj = x0 + u32(j) * kDThreads;
      x[j] = rj < r1 ? rec[rj] : 0u;
    }
#pragma unroll
    for (int j = 0; j < kDBatch; ++j) {
      const u32 rj = x0 + u32(j) * kDThreads;
      if (rj < r1) idrec[rj] = s_id[(x[j] & kIdx) >> kDLog] | (x[j] & kBits);
    }
  }
}

[[maybe_unused]] static __global__ __launch_bounds__(kDThreads) void k_dl_ids_mr(const u32* __restrict__ rec, const u32* __restrict__ off,
                                                         DensePlan P, const unsigned long long* __restrict__ pbs,
                                                         u64 stride, const u32* __restrict__ xvs, u64 xstride,
                                                         const u32* __restrict__ gl, const DlRelay* __restrict__ T,
                                                         int R, int r, u32* __restrict__ idrec) {
  dl_ids_mr_block(rec, off, P, pbs, stride, xvs, xstride, gl, T, R, r, idrec, blockIdx.x);
}

// This rank's slice of the unique leaves: its r-first codes in position order (= id order),
// one thread per position of the r-first position bitmap (a wave shares one bitmap word).
[[maybe_unused]] static __global__ __launch_bounds__(256) void k_dl_rleaves(const unsigned long long* __restrict__ rfb,
                                                    const u32* __restrict__ wpre, const u32* __restrict__ pw,
                                                    DensePlan P, u64* __restrict__ out) {
  const u64 p = u64(blockIdx.x) * 256 + threadIdx.x;
  if (p >= P.S) return;
  const unsigned long long m = rfb[p >> 6];
  if (!((m >> (p & 63)) & 1ull)) return;
  const u32 k = wpre[p >> 6] + u32(__popcll(m & ((1ull << (p & 63)) - 1ull)));
  const u32 h = pw[p] & kIdx;
  out[k] = code2_leaf((h * P.Kinv) & P.hmask, P.L);
}

}  // namespace gcz_dev
