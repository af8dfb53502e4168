// Device code of the multi-rank build's fused leaf + layer-0 round schedule (gcz_dist.hip,
// gcz_group::build_fast): pure-ACGT genomes (the dense leaf level, L <= 12) whose node levels
// take no local dedupe (non-repetitive data) and whose layer 1 turns out direct -- the
// synthetic 1 Gbase uniform genome of the benchmark.
//
// The idea: the reference's node identity (`node::operator==` on canonical nodes,
// include/shared_tree.h:119-126, src/shared_tree.cpp:175-177) depends on the children's
// pointers only through equality and the per-pointer transforms (pointer(other, m, t),
// src/shared_tree.cpp:76-80), never through the index VALUE.  Relabelling the leaves by any
// bijection maps node classes onto node classes, so layer 0 can be hash-consed across ranks
// with the leaves' hashed 2-bit codes as labels (the dense pack's pre-words, gcz_dense.h)
// BEFORE the leaves' global ids exist.  The layer-0 key exchange therefore rides in the same
// collective groups as the leaf-id exchange instead of after it:
//
//   R1a allgather: status words + layer-0 owner counts (right after the pack and the keys'
//       one-pass scatter into owner regions, k_fl_scatter: the one mid-build host read --
//       the path, the keys' all-to-all sizes)
//   K2  keys to owners (code labels): one all-to-all on a second stream and communicator, so
//       it runs beside the leaf level's sort and the next collectives (RCCL; the testing
//       transports run it in line)
//   R1b allgather: presence bitmaps
//   R2  leaf G arrays, relay 1 (fixed-capacity pieces: no host read of the r-first counts)
//   R3  owner replies (2 bits per record) | leaf G arrays, relay 2 | allgather of the owners'
//       not-first counts per source (-> every rank's layer-0 id offset, no count round)
//   R4  C: first holders' ids to owners (fixed-capacity slots) | allgather: look-ahead, status
//   R5  D: owners forward them to the other holders (fixed-capacity slots)
//   R6  top words to rank 0 (gather)              R7  final vectors (allgather, host sync)
//
// Only then are the layer-0 nodes written, canonicalised with the global leaf ids
// (k_fl_words_l0).  Any surprise (a non-ACGT strand or repetitive data at R1a -- the scatter and
// the dense sort then return at once on the device --, an owner region overflow, an owner that
// cannot take the two-pass dedupe, a C/D slot overflow, a look-ahead that finds layer 1 not
// direct, an owner bucket overflow) makes every rank discard the attempt together and run the
// general schedule (gcz_group::build's exchange loop), which handles every input.
#pragma once

#include "gcz_dist_device.h"

namespace gcz_dev {

// C / D records per (sender, receiver) pair in the fixed-capacity slots: a segment is
// [count, records...] of kFlCap + 1 u64 (a count above kFlCap = overflow: the attempt is
// discarded).  1 Gbase uniform: C/D carry ~1 record at R = 8 (strong), ~100 per rank weak.
constexpr u32 kFlCap = 4096;
constexpr u32 kFlSeg = kFlCap + 1;

// Per (bucket, rank q): the codes rank q holds first (present_q & ~(present_0 | ... |
// present_{q-1})), counted from the gathered presence bitmaps -- every rank derives every
// rank's r-first counts itself (the general schedule allgathers them).  One block per bucket;
// k_fl_prefix_relay then writes, per rank q, the exclusive prefix of its per-bucket counts into
// the layout of the general schedule's gathered exchange vectors (xvs[q * xw + 2 + b],
// k_dl_ids_mr reads them) with the total, c_q, at xvs[q * xw], and the leaf relay's table
// (fl_relay_table).
// the leaf relay's piece q of a list of c elements: [c q / R, c (q + 1) / R) (see below)
__device__ __forceinline__ u64 fl_piece(u64 c, u32 q, u32 R) { return c * q / R; }

struct FlRelayOut {
  u32* xvs;
  u64 xw;
  u32 me;
  u64 cap2;
  DlRelay* T;
  u64* leaf;      // {leaf offset, r-first count, total}
};

// one block: the relay table from the r-first totals c[0, R) (LDS)
static __device__ void fl_relay_table(const u64* s_c, u32 R, const FlRelayOut& o) {
  __shared__ u64 s_off[kDlMaxRanks + 1];
  __shared__ u64 s_len[kDlMaxRanks * kDlMaxRanks];
  const u32 t0 = threadIdx.x;
  if (t0 == 0) {
    u64 x = 0;
    for (u32 s = 0; s < R; ++s) {
      s_off[s] = x;
      x += s_c[s];
    }
    s_off[R] = x;
  }
  for (u32 t = t0; t < R * R; t += blockDim.x) {   // piece q of list s
    const u32 q = t / R, s = t % R;
    s_len[t] = fl_piece(s_c[s], q + 1, R) - fl_piece(s_c[s], q, R);
  }
  __syncthreads();
  if (t0 <= R) o.T->off[t0] = s_off[t0];
  if (t0 == 0) {
    o.leaf[0] = s_off[o.me];
    o.leaf[1] = s_c[o.me];
    o.leaf[2] = s_off[R];
  }
  for (u32 t = t0; t < R * R; t += blockDim.x) {
    const u32 q = t / R, s = t % R;
    u64 at = u64(q) * o.cap2;   // rank q's block of the relay-2 buffer: lists 0 .. s-1's pieces q first
    for (u32 s2 = 0; s2 < s; ++s2) at += s_len[q * R + s2];
    const u64 sg = u64(s) * R + q;
    o.T->seg_src[sg] = at;
    o.T->seg_dst[sg] = s_off[s] + fl_piece(s_c[s], q, R);
    o.T->seg_len[sg] = s_len[t];
  }
}

[[maybe_unused]] static __global__ __launch_bounds__(256) void k_fl_counts(const unsigned long long* __restrict__ pbs,
                                                       u64 stride, int R, DensePlan P, u32* __restrict__ cntb) {
  __shared__ u32 s_c[kMaxRanks];
  const int tid = threadIdx.x, lane = tid & 63;
  const u32 b = blockIdx.x, RB = 1u << P.IB, NW = RB >= 64 ? RB / 64 : 1u;
  if (tid < R) s_c[tid] = 0;
  __syncthreads();
  u32 c[kMaxRanks];
#pragma unroll
  for (int q = 0; q < kMaxRanks; ++q) c[q] = 0;
  for (u32 lw = tid; lw < NW; lw += 256) {
    u64 acc = 0;
#pragma unroll
    for (int q = 0; q < kMaxRanks; ++q)
      if (q < R) {
        const u64 w = bucket_word(pbs + u64(q) * stride, b, P.IB, lw);
        c[q] += u32(__popcll(w & ~acc));
        acc |= w;
      }
  }
#pragma unroll
  for (int q = 0; q < kMaxRanks; ++q)
    if (q < R) {
      const u32 v = u32(wave_sum(u64(c[q])));
      if (lane == 0 && v) atomicAdd(&s_c[q], v);
    }
  __syncthreads();
  if (tid < R) cntb[u64(tid) * P.NB + b] = s_c[tid];
}

// One block of kDThreads (NB <= 1024 buckets): the prefixes and totals into xvs, then the relay
// table.  (A separate launch: a last-block ticket in k_fl_counts needs a device-scope fence per
// block, an L2 write-back on this part.)
[[maybe_unused]] static __global__ __launch_bounds__(kDThreads) void k_fl_prefix_relay(const u32* __restrict__ cntb, int R,
                                                               DensePlan P, FlRelayOut o) {
  __shared__ u32 s_tmp[16];
  __shared__ u64 s_tot[kDlMaxRanks];
  const int tid = threadIdx.x;
  for (int q = 0; q < R; ++q) {
    u32 total;
    const u32 x = u32(tid) < P.NB ? cntb[u64(q) * P.NB + tid] : 0u;
    const u32 e = block_excl(x, s_tmp, &total);
    if (u32(tid) < P.NB) o.xvs[u64(q) * o.xw + 2 + tid] = e;
    if (tid == 0) {
      o.xvs[u64(q) * o.xw] = total;
      o.xvs[u64(q) * o.xw + 1] = 0;
      s_tot[q] = total;
    }
  }
  __syncthreads();
  fl_relay_table(s_tot, u32(R), o);
}

// The owner's not-first records counted per source rank (its dedupe's list): a source's
// globally-first layer-0 pairs are its pairs minus the not-first ones at every owner.
// (C5's device functions take their workgroup's index and count within the launch: k_fl_c5)
static __device__ __forceinline__ void fl_ownnf(const u32* __restrict__ olist, const u32* __restrict__ ocnt,
                                                const Displ& D, u32 R, u64* __restrict__ onf, u32 bx, u32 gx) {
  __shared__ u32 s_c[kMaxRanks];
  if (threadIdx.x < R) s_c[threadIdx.x] = 0;
  __syncthreads();
  const u32 n = *ocnt;
  for (u32 i = bx * 256 + threadIdx.x; i < n; i += gx * 256) atomicAdd(&s_c[seg_of(D, R, olist[i])], 1u);
  __syncthreads();
  if (threadIdx.x < R && s_c[threadIdx.x])
    atomicAdd(reinterpret_cast<unsigned long long*>(&onf[threadIdx.x]), (unsigned long long)s_c[threadIdx.x]);
}

// The owner's replies (k_bkt_dedupe2<true>: 0, 6 first of a repeated key, 7 not first) packed
// 2 bits per record, segment by segment (k_dist_flags' reply_code2 reads them): one thread per output byte.
static __device__ __forceinline__ void fl_pack2(const unsigned char* __restrict__ rflag, const Displ& D,
                                                const Displ& P4, u32 R, unsigned char* __restrict__ out, u32 bx) {
  const u64 t = u64(bx) * 256 + threadIdx.x;
  if (t >= P4.d[R]) return;
  const u32 s = seg_of(P4, R, t);
  const u64 i0 = (t - P4.d[s]) * 4, n = D.d[s + 1] - D.d[s];
  u32 b = 0;
#pragma unroll
  for (u32 j = 0; j < 4; ++j)
    if (i0 + j < n) {
      const unsigned char f = rflag[D.d[s] + i0 + j];
      b |= u32(f == 0 ? 0 : f == 6 ? 1 : 2) << (2 * j);
    }
  out[t] = (unsigned char)b;
}

// ---- the leaf relay with fixed-capacity pieces --------------------------------------------
// Rank s's G list (c_s elements, k_dl_gq) is cut into R pieces, piece q = [c_s q / R,
// c_s (q + 1) / R) -> rank q (relay 1: slot s of rank q's buffer, cap1 elements per slot); rank
// q concatenates the pieces it got (relay 2: cap2 elements to every rank, slot q).  The c_s come
// from the gathered bitmaps (k_fl_counts: xvs[s * xw]), so every rank computes the layout and
// k_dl_ids_mr's table itself.

// relay 1, sender side: the rank's G list into slot q of the staging buffer, piece by piece
// (the piece bounds in LDS: no division per element)
[[maybe_unused]] static __global__ __launch_bounds__(256) void k_fl_relay_out(const u32* __restrict__ G,
                                                          const u64* __restrict__ leaf, u32 R, u64 cap1,
                                                          u32* __restrict__ stage) {
  __shared__ u64 s_b[kDlMaxRanks + 1];
  const u64 c = leaf[1];
  if (threadIdx.x <= R) s_b[threadIdx.x] = fl_piece(c, threadIdx.x, R);
  __syncthreads();
  for (u64 j = u64(blockIdx.x) * 256 + threadIdx.x; j < c; j += u64(gridDim.x) * 256) {
    u32 q = 0;
    while (q + 1 < R && s_b[q + 1] <= j) ++q;
    stage[u64(q) * cap1 + (j - s_b[q])] = G[j];
  }
}

// relay 2, sender side (rank me): the pieces it received (slot s: piece me of list s) back to back
static __device__ __forceinline__ void fl_relay_mid(const u32* __restrict__ got, const u32* __restrict__ xvs, u64 xw,
                                                    u32 R, u32 me, u64 cap1, u32* __restrict__ out, u32 bx, u32 gx) {
  __shared__ u64 s_len[kDlMaxRanks + 1];
  if (threadIdx.x == 0) {
    u64 o = 0;
    for (u32 s = 0; s < R; ++s) {
      s_len[s] = o;
      const u64 c = xvs[u64(s) * xw];
      o += fl_piece(c, me + 1, R) - fl_piece(c, me, R);
    }
    s_len[R] = o;
  }
  __syncthreads();
  for (u64 j = u64(bx) * 256 + threadIdx.x; j < s_len[R]; j += u64(gx) * 256) {
    u32 s = 0;
    while (s + 1 < R && s_len[s + 1] <= j) ++s;
    out[j] = got[u64(s) * cap1 + (j - s_len[s])];
  }
}

// C5's tail in one launch (after the owner's dedupe): workgroups [0, npack) pack the replies,
// the next 64 count the not-first records per source, the last 256 stage relay 2
struct FlC5 {
  const u32* olist;
  const u32* ocnt;
  Displ D, P4;
  u64* onf;
  const unsigned char* rflag;
  unsigned char* packed;
  u32 npack;
  const u32* got;
  const u32* xvs;
  u64 xw, cap1;
  u32 me;
  u32* relay2;
};
[[maybe_unused]] static __global__ __launch_bounds__(256) void k_fl_c5(FlC5 a, u32 R) {
  const u32 b = blockIdx.x;
  if (b < a.npack) {
    fl_pack2(a.rflag, a.D, a.P4, R, a.packed, b);
  } else if (b < a.npack + 64) {
    fl_ownnf(a.olist, a.ocnt, a.D, R, a.onf, b - a.npack, 64);
  } else {
    fl_relay_mid(a.got, a.xvs, a.xw, R, a.me, a.cap1, a.relay2, b - a.npack - 64, 256);
  }
}

struct FlPairs {   // layer-0 pairs of every rank (host-known from the plan)
  u64 p[kMaxRanks];
};

// This rank's layer-0 id offset (and its unique count) from R3's gathered not-first counts
// (gonf[o * R + s] = owner o's not-first records of source s): u_s = p_s - sum_o gonf[o R + s].
// R^2 loads (L2-resident): recomputed where it is needed rather than a launch of its own.
__device__ __forceinline__ u64 fl_offset(const u64* __restrict__ gonf, u32 R, const FlPairs& pp, u32 me, u64* u_me) {
  u64 o = 0;
  for (u32 s = 0; s <= me; ++s) {
    u64 nf = 0;
    for (u32 q = 0; q < R; ++q) nf += gonf[u64(q) * R + s];
    const u64 u = pp.p[s] - nf;
    if (s == me) {
      if (u_me) *u_me = u;
      return o;
    }
    o += u;
  }
  return o;
}

// R4's gathered {look-ahead pairs, failure} of every rank -> 0 when layer 1 is direct on
// every rank and none failed (the direct subtrees' guard)
__device__ __forceinline__ u64 fl_guard(const u64* __restrict__ g4, u32 R) {
  u64 t = 0;
  for (u32 s = 0; s < R; ++s) t += g4[2 * s] + g4[2 * s + 1];
  return t;
}

// Layer 0's records bucketed by owner in ONE pass over the pre-words (no count pass, no scan):
// owner q's records go to the fixed-capacity region [q cap, (q + 1) cap) of the send buffer,
// each tile's place in it found by a decoupled look-back over the tiles' per-owner counts
// (tiles taken in dispatch order by a ticket, so a tile waits only on tiles already running).
// Stable: within a region the records keep position order, so owners see each source's records
// in order (the first record of a key is its first occurrence).  A thread takes kFsItems
// consecutive pairs, counts them per owner in 16-bit fields of two registers (owners 0-3 | 4-7:
// a tile's count fits), one block scan of those gives every record its place in the tile's
// owner-sorted copy in LDS, and the tile leaves LDS as R contiguous runs (coalesced stores).
// A region that would overflow drops its surplus (never written out of bounds) and the status
// word R gets bit 4: every rank then runs the general schedule (the mid-build read).  The last
// tile writes the owner totals and the status words (R1a's vector, as k_bscan_small does).  Also
// what the exchange expects zeroed: the global flags and the rank scan's look-back words;
// count_out = the pairs.
struct FlScatter {
  u64* skey;               // low 32 bits of the 6-byte records (split) or 8-byte keys
  u32* sidx;
  unsigned short* skey_hi; // (split) the high 16 bits
  u64 cap;                 // records per owner region
  u64* desc;               // R x nb look-back descriptors (owner-major: a poll reads 512 B), zeroed, then the ticket
  u32 nb;
  u64* tot;                // [0, R): owner totals, [R, R + 6): status words
  const Header* h;
  unsigned char* gnf;
  unsigned char* gmul;
  u64* ddesc;
  u64* count_out;
  u32 spin_cap;            // look-back polls before a tile gives up (kFlSpinCap; 0: at once, testing)
};
constexpr u32 kFlSpinCap = 1u << 22;   // look-back polls before a tile gives up (status bit 8)
constexpr int kFsThreads = 512, kFsItems = kTile / kFsThreads;   // 16 consecutive pairs a thread
constexpr u32 kFsGrid = 512;     // persistent blocks: two per CU (80 KB of LDS each) on 256 CUs
constexpr int kFlMaxRanks = 8;   // the fused schedule's ranks at most (one node)
static_assert(kFlMaxRanks <= kFsThreads / 64 && kTile <= 65535, "one look-back wave per owner, 16-bit fields");

__device__ __forceinline__ u32 fs_field(u64 lo, u64 hi, u32 d) {
  return u32(((d < 4 ? lo : hi) >> (16 * (d & 3))) & 0xffffu);
}

// this thread's kFsItems pairs of tile `tile` (pairs past the level: null words)
__device__ __forceinline__ void fs_load(const RecSrc& s, u32 tile, uint4 (&w)[kFsItems / 2]) {
  const u64 j0 = u64(tile) * kTile + u64(threadIdx.x) * kFsItems;
  if (2 * (j0 + kFsItems) <= s.n) {   // every pair whole: 16-byte loads
    const uint4* w4 = reinterpret_cast<const uint4*>(s.pre) + j0 / 2;
#pragma unroll
    for (int k = 0; k < kFsItems / 2; ++k) w[k] = w4[k];
  } else {
#pragma unroll
    for (int k = 0; k < kFsItems / 2; ++k) {
      u32 l0 = kNullWord, r0 = kNullWord, l1 = kNullWord, r1 = kNullWord;
      if (j0 + 2 * k < s.p) load_pair(s.pre, s.n, j0 + 2 * k, l0, r0);
      if (j0 + 2 * k + 1 < s.p) load_pair(s.pre, s.n, j0 + 2 * k + 1, l1, r1);
      w[k] = make_uint4(l0, r0, l1, r1);
    }
  }
}

// Persistent: a block takes tiles by the ticket until none is left; the next tile's pre-words
// are in flight while the block waits on its look-back and writes the current tile out.
[[maybe_unused]] static __global__ __launch_bounds__(kFsThreads) void k_fl_scatter(RecSrc s, FlScatter a) {
  constexpr int kW = kFsThreads / 64;
  __shared__ u64 s_key[kTile];
  __shared__ unsigned short s_pos[kTile];
  __shared__ u64 s_wl[kW], s_wh[kW];
  __shared__ u32 s_start[kMaxRanks + 1];
  __shared__ u64 s_base[kMaxRanks];
  __shared__ u32 s_tile[2], s_bad;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const u32 R = s.R;
  if (a.h->predup | a.h->dense_fail) {   // repetitive or not pure ACGT (the pack said so): the
    // general schedule runs instead, so only R1a's vector is written (no scatter to waste)
    if (blockIdx.x == 0 && tid <= int(R) + 5)
      a.tot[tid] = tid < int(R) ? 0ull
                 : tid == int(R)     ? u64(a.h->overflow | a.h->leaf_overflow)
                 : tid == int(R) + 2 ? a.h->err_offset
                 : tid == int(R) + 4 ? u64(a.h->predup)
                 : tid == int(R) + 5 ? u64(a.h->dense_fail)
                                     : 0ull;
    return;
  }
  u32* ticket = reinterpret_cast<u32*>(a.desc + u64(a.nb) * R);
  if (tid == 0) {
    s_tile[0] = atomicAdd(ticket, 1u);
    s_bad = 0;
  }
  __syncthreads();
  u32 tile = s_tile[0];
  uint4 w[kFsItems / 2];
  if (tile < a.nb) fs_load(s, tile, w);
  for (int it = 0; tile < a.nb; ++it) {
    const u64 p = s.p, e_base = u64(tile) * kTile;
    {   // the flags and the look-back word of this tile's pairs, zeroed for the exchange
      const u64 end = tile + 1 == a.nb ? p + 1 : std::min<u64>(e_base + kTile, p + 1);
      for (u64 q = e_base / 16 + tid; q < (end + 15) / 16; q += kFsThreads) {
        reinterpret_cast<uint4*>(a.gnf)[q] = make_uint4(0, 0, 0, 0);
        reinterpret_cast<uint4*>(a.gmul)[q] = make_uint4(0, 0, 0, 0);
      }
      if (tid == 0) {
        a.ddesc[tile] = 0;
        if (tile == 0) *a.count_out = p;
        s_tile[(it + 1) & 1] = atomicAdd(ticket, 1u);   // (read after the next barrier)
      }
    }
    // keys, owners, counts per owner
    const u64 j0 = e_base + u64(tid) * kFsItems;
    u64 key[kFsItems];
    u32 okm = 0;
#pragma unroll
    for (int k = 0; k < kFsItems / 2; ++k) {
      if (pre_rec(s, w[k].x, w[k].y, j0 + 2 * k < p, key[2 * k])) okm |= 1u << (2 * k);
      if (pre_rec(s, w[k].z, w[k].w, j0 + 2 * k + 1 < p, key[2 * k + 1])) okm |= 2u << (2 * k);
    }
    u64 cl = 0, ch = 0;
    u32 dst[kFsItems / 8];   // owners, 4 bits each
#pragma unroll
    for (int k = 0; k < kFsItems / 8; ++k) dst[k] = 0;
#pragma unroll
    for (int e = 0; e < kFsItems; ++e) {
      const u32 d = rec_dest(s, key[e]);
      dst[e / 8] |= d << (4 * (e % 8));
      const u64 inc = ((okm >> e) & 1u) ? 1ull << (16 * (d & 3)) : 0ull;
      if (d < 4) cl += inc; else ch += inc;
    }
    // the block scan of the packed counts: this thread's first place per owner
    u64 il = cl, ih = ch;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u64 tl = __shfl_up(il, o, 64), th = __shfl_up(ih, o, 64);
      if (lane >= o) { il += tl; ih += th; }
    }
    if (lane == 63) { s_wl[wave] = il; s_wh[wave] = ih; }
    __syncthreads();
    const u32 next = s_tile[(it + 1) & 1];
    u64 bl = 0, bh = 0, tl = 0, th = 0;
#pragma unroll
    for (int w2 = 0; w2 < kW; ++w2) {
      const u64 vl = s_wl[w2], vh = s_wh[w2];
      if (w2 < wave) { bl += vl; bh += vh; }
      tl += vl; th += vh;
    }
    // tile totals per owner -> bucket starts; every owner's aggregate published at once
    u64 sl = 0, sh = 0;   // the buckets' starts, packed
    {
      u32 run = 0;
      for (u32 q = 0; q < R; ++q) {
        if (q < 4) sl |= u64(run) << (16 * q); else sh |= u64(run) << (16 * (q - 4));
        run += fs_field(tl, th, q);
      }
      if (tid <= int(R)) {
        u32 st = 0;
        for (u32 q = 0; q < u32(tid); ++q) st += fs_field(tl, th, q);
        s_start[tid] = st;
      }
    }
    if (tid < int(R))
      __hip_atomic_store(&a.desc[u64(tid) * a.nb + tile], (tile == 0 ? kStP : kStA) | u64(fs_field(tl, th, u32(tid))),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the records into the owner-sorted copy
    u64 curl = sl + bl + il - cl, curh = sh + bh + ih - ch;
#pragma unroll
    for (int e = 0; e < kFsItems; ++e) {
      const u32 d = (dst[e / 8] >> (4 * (e % 8))) & 15u;
      if ((okm >> e) & 1u) {
        const u32 at = fs_field(curl, curh, d);
        s_key[at] = key[e];
        s_pos[at] = (unsigned short)(tid * kFsItems + e);
        const u64 inc = 1ull << (16 * (d & 3));
        if (d < 4) curl += inc; else curh += inc;
      }
    }
    if (next < a.nb) fs_load(s, next, w);   // (in flight through the look-back and the write-out)
    // the look-back: owner q by wave q (64 predecessors per poll)
    if (u32(wave) < R) {
      const u32 q = u32(wave);
      const u64 agg = fs_field(tl, th, q);
      u64 prefix = 0;
      if (tile > 0) {
        long long look = (long long)tile - 1;
        u32 polls = 0;
        for (;;) {
          const long long idx = look - lane;
          const u64 dv = idx >= 0 ? __hip_atomic_load(&a.desc[u64(q) * a.nb + u64(idx)], __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT)
                                  : 0ull;
          const u64 st = dv >> 62;
          const u64 pm = __ballot(st == 2);
          const u64 zm = __ballot(idx >= 0 && st == 0);
          const int firstP = pm ? __ffsll((long long)pm) - 1 : 64;
          const u64 need = firstP >= 63 ? ~0ull : ((1ull << (firstP + 1)) - 1);
          if ((zm & need) || a.spin_cap == 0) {
            if (++polls > a.spin_cap) {   // (bounded: a tile never waits forever)
              if (lane == 0) {   // (any block: the status word, OR-ed -- the last tile may be another's)
                s_bad = 1;
                atomicOr(reinterpret_cast<unsigned long long*>(&a.tot[R]), 256ull);
              }
              break;
            }
            // back off (the polls are uncached loads: a tight spin of every waiting tile costs
            // the chip's memory bandwidth)
            for (u32 z = 0; z < std::min<u32>(polls, 8u); ++z) __builtin_amdgcn_s_sleep(16);
            continue;
          }
          prefix += wave_sum(lane <= firstP && idx >= 0 ? (dv & kValMask) : 0ull);
          if (firstP < 64 || look < 64) break;
          look -= 64;
        }
        if (lane == 0)
          __hip_atomic_store(&a.desc[u64(q) * a.nb + tile], kStP | (prefix + agg), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
      if (lane == 0) s_base[q] = prefix;
    }
    __syncthreads();
    if (tile + 1 == a.nb && tid <= int(R) + 5) {   // the last tile: owner totals and status words
      if (tid < int(R)) {
        const u64 t = s_base[tid] + fs_field(tl, th, u32(tid));
        a.tot[tid] = t > a.cap ? a.cap : t;
      } else {
        const u32 w2 = u32(tid) - R;
        u64 v = 0;
        if (w2 == 0) {
          u32 over = 0;
          for (u32 q = 0; q < R; ++q) over |= s_base[q] + fs_field(tl, th, q) > a.cap ? 1u : 0u;
          v = u64(a.h->overflow | a.h->leaf_overflow) | (over ? 16ull : 0ull) | (s_bad ? 256ull : 0ull);
        } else if (w2 == 2) {
          v = a.h->err_offset;
        } else if (w2 == 4) {
          v = u64(a.h->predup);
        } else if (w2 == 5) {
          v = u64(a.h->dense_fail);
        }
        if (w2 == 0)
          atomicOr(reinterpret_cast<unsigned long long*>(&a.tot[tid]), (unsigned long long)v);   // (R1a's word: zeroed)
        else
          a.tot[tid] = v;
      }
    }
    // the owner-sorted copy out: R contiguous runs
    u32 st[kFlMaxRanks + 1];
#pragma unroll
    for (int q = 0; q <= kFlMaxRanks; ++q) st[q] = s_start[q <= int(R) ? q : int(R)];
    const u32 nt = st[kFlMaxRanks];
    for (u32 i = u32(tid); i < nt; i += kFsThreads) {
      u32 q = 0;
#pragma unroll
      for (int k = 1; k < kFlMaxRanks; ++k) q += i >= st[k] ? 1u : 0u;   // (empty buckets: equal starts)
      const u64 o = s_base[q] + (i - s_start[q]);
      if (o < a.cap) {   // (a surplus record is dropped: status bit 4, the general schedule)
        const u64 at = u64(q) * a.cap + o;
        const u64 k = s_key[i];
        if (a.skey_hi) {
          reinterpret_cast<u32*>(a.skey)[at] = u32(k);
          a.skey_hi[at] = (unsigned short)(k >> 32);
        } else {
          a.skey[at] = k;
        }
        a.sidx[at] = u32(e_base + s_pos[i]);
      }
    }
    __syncthreads();   // (the copy, the starts and the bases are the next tile's)
    tile = next;
  }
}

// C and D at the owner, one block: the first holders' ids into the keys' id slots, then every
// not-first record's id into the slot of its source (the C / D counts of this schedule are
// bounded by the slots: kFlCap per pair).
// (one workgroup of 1024 threads; k_fl_ids_cd runs it beside the leaf ids' buckets)
static __device__ __forceinline__ void fl_cd_block(const u64* __restrict__ rc, const Displ& D, u32 R,
                                                   const u32* __restrict__ oslot, const OwnTab& T,
                                                   const u32* __restrict__ olist, const u32* __restrict__ ocnt,
                                                   u64* __restrict__ dbuf, u32* __restrict__ bad) {
  for (u32 s = 0; s < R; ++s) {
    const u64 n = rc[u64(s) * kFlSeg];
    if (n > kFlCap) {
      if (threadIdx.x == 0) atomicOr(bad, 1u);
      continue;
    }
    for (u64 i = threadIdx.x; i < n; i += 1024) {
      const u64 v = rc[u64(s) * kFlSeg + 1 + i];
      own_set_id(T, oslot[D.d[s] + u32(v)], u32(v >> 32));
    }
  }
  __syncthreads();
  const u32 n = *ocnt;
  for (u32 i = threadIdx.x; i < n; i += 1024) {
    const u32 k = olist[i];
    const u32 s = seg_of(D, R, k);
    const u64 slot = atomicAdd(reinterpret_cast<unsigned long long*>(&dbuf[u64(s) * kFlSeg]), 1ull);
    if (slot >= kFlCap) {
      atomicOr(bad, 1u);
      continue;
    }
    dbuf[u64(s) * kFlSeg + 1 + slot] = u64(k - D.d[s]) | (u64(own_id(T, oslot[k])) << 32);
  }
}

// C7 in one launch: blocks [0, NB) the leaf level's global ids (dl_ids_mr_block, gcz_dense.h),
// block NB the owner's C -> D records (fl_cd_block)
struct FlCd {
  const u64* rc;
  Displ D;
  const u32* oslot;
  OwnTab T;
  const u32* olist;
  const u32* ocnt;
  u64* dbuf;
  u32* bad;
};
[[maybe_unused]] static __global__ __launch_bounds__(kDThreads) void k_fl_ids_cd(const u32* __restrict__ rec, const u32* __restrict__ off,
                                                         DensePlan P, const unsigned long long* __restrict__ pbs,
                                                         u64 stride, const u32* __restrict__ xvs, u64 xstride,
                                                         const u32* __restrict__ gl, const DlRelay* __restrict__ T,
                                                         int R, int r, u32* __restrict__ idrec, FlCd c) {
  if (blockIdx.x < P.NB) {
    dl_ids_mr_block(rec, off, P, pbs, stride, xvs, xstride, gl, T, R, r, idrec, blockIdx.x);
    return;
  }
  fl_cd_block(c.rc, c.D, u32(R), c.oslot, c.T, c.olist, c.ocnt, c.dbuf, c.bad);
}

// C at a first holder: (index within its segment to owner q, global id) into q's slot.
// (a slot overflow goes straight into this rank's R4 vector: r4[1])
[[maybe_unused]] static __global__ __launch_bounds__(256) void k_fl_cvals(const u32* __restrict__ clist,
                                                      const u32* __restrict__ ccount, const u32* __restrict__ sidx,
                                                      Displ SD, u32 R, const u32* __restrict__ gid,
                                                      const u64* __restrict__ gonf, FlPairs pp, u32 me,
                                                      u64* __restrict__ cbuf, u64* __restrict__ r4) {
  const u32 n = *ccount;
  if (n == 0) return;
  const u64 off = fl_offset(gonf, R, pp, me, nullptr);
  for (u32 i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const u32 k = clist[i];
    const u32 q = seg_of(SD, R, k);
    const u64 slot = atomicAdd(reinterpret_cast<unsigned long long*>(&cbuf[u64(q) * kFlSeg]), 1ull);
    if (slot >= kFlCap) {
      atomicOr(reinterpret_cast<unsigned long long*>(&r4[1]), 1ull);
      continue;
    }
    const u32 id = u32(off + (gid[sidx[k]] & ~kLocalId));
    cbuf[u64(q) * kFlSeg + 1 + slot] = u64(k - SD.d[q]) | (u64(id) << 32);
  }
}

// The final vector of a fast-schedule rank: the general one (k_dist_final) plus failure bit 2
// (a C/D overflow, a look-ahead that found layer 1 not direct), [2] = this rank's r-first
// leaves and [3] = its layer-0 uniques.
// (one wave: lane k < GCZ_MAX_LAYERS copies layer k's count, lane s < R sums source s's
// not-first counts and its look-ahead / status words)
[[maybe_unused]] static __global__ __launch_bounds__(64) void k_fl_final(const Header* __restrict__ h,
                                                         DistHdr* __restrict__ dh, int tail0, int D, int has_tail,
                                                         const u32* __restrict__ bad, const u64* __restrict__ g4,
                                                         const u64* __restrict__ gonf, FlPairs pp, u32 R, u32 me) {
  const u32 t = threadIdx.x;
  for (u32 k = t; k < GCZ_MAX_LAYERS; k += 64)
    dh->final_vec[4 + k] = (has_tail && int(k) >= tail0 && int(k) < D) ? h->count[kLayerSlot + k] : 0ull;
  u64 nf = 0, gv = 0;
  if (t < R) {
    for (u32 q = 0; q < R; ++q) nf += gonf[u64(q) * R + t];
    gv = g4[2 * t] + g4[2 * t + 1];
  }
  const u64 gsum = wave_sum(gv);
  if (t == me) dh->final_vec[3] = pp.p[t] - nf;   // this rank's layer-0 uniques
  if (t == 0) {
    dh->final_vec[0] = u64(h->overflow | h->leaf_overflow) | ((*bad || gsum) ? 2ull : 0ull);
    dh->final_vec[1] = has_tail ? u64(h->root) : 0ull;
    dh->final_vec[2] = dh->fl_leaf[1];   // this rank's r-first leaves
  }
}

}  // namespace gcz_dev

namespace gcz_dev {

// Layer 0 with the global leaf ids (emplace_node, src/shared_tree.cpp:662-672), fused into the
// dense level's words pass (k_dl_words): the chunk's leaf words never leave LDS.  Each pair of
// the chunk gets its canonical node and bits; a globally-first pair takes id off + its local
// rank and writes its node at that rank of the rank's slice, the others take the id D
// delivered.  The chunk's first positions (the rank's r-first codes) write their leaves.
// Block 0 also settles the direct subtrees' guard from R4's vectors.
struct FlL0 {
  const unsigned char* gnf;   // per pair: not globally first
  u32* gid;                   // per pair: local rank | kLocalId (first), else the global id
  const u64* gonf;            // R3's gathered not-first counts
  const u64* g4;              // R4's gathered {look-ahead, failure}
  FlPairs pp;
  u32 R, me;
  const u64* leaf;            // k_fl_counts' {leaf offset, r-first count, total}
  uint2* nodes;               // the rank's slice of layer 0
  u32* words0;                // layer-0 words (the direct subtrees' input)
  u64* guard;
};

// R5's D records (the owners' ids of this rank's not-first pairs whose first holder is another
// rank) into gid, one thread a slot, before k_fl_words_l0 reads them (a few hundred records: in
// every words block, the R dependent segment reads cost each workgroup several microseconds)
[[maybe_unused]] static __global__ __launch_bounds__(256) void k_fl_dpatch(const u64* __restrict__ rd, Displ SD, u32 R,
                                                                          const u32* __restrict__ sidx,
                                                                          u32* __restrict__ gid, u32* __restrict__ bad) {
  const u64 t = u64(blockIdx.x) * 256 + threadIdx.x;
  const u32 q = u32(t / kFlCap), i = u32(t % kFlCap);
  if (q >= R) return;
  const u64 n = rd[u64(q) * kFlSeg];
  if (n > kFlCap) {
    if (i == 0) atomicOr(bad, 1u);
    return;
  }
  if (i < n) {
    const u64 v = rd[u64(q) * kFlSeg + 1 + i];
    gid[sidx[SD.d[q] + u32(v)]] = u32(v >> 32);
  }
}
// Rank 0's leaves and those of a rank whose r-first positions are dense go out here in
// position order (= id order) from the pre-words: coalesced stores, where k_dl_words'
// record-order stores scatter (at 1 Gbase over 8 ranks rank 0 first-holds ~47 % of its strands'
// codes); k_dl_gq writes the others'.
[[maybe_unused]] static __global__ __launch_bounds__(kDThreads) void k_fl_words_l0(const u32* __restrict__ rec,
                                                           const u32* __restrict__ idrec, const u32* __restrict__ offt,
                                                           DensePlan P, const unsigned long long* __restrict__ fb,
                                                           const u32* __restrict__ pw, u64* __restrict__ leaves_out,
                                                           FlL0 a) {
  extern __shared__ u32 s_dyn[];
  __shared__ u32 s_off, s_loff;
  if (threadIdx.x == 0) {
    s_off = u32(fl_offset(a.gonf, a.R, a.pp, a.me, nullptr));
    s_loff = u32(a.leaf[0]);
    if (blockIdx.x == 0) *a.guard = fl_guard(a.g4, a.R);
  }
  dl_words_chunk(rec, idrec, offt, P, fb, nullptr, 0, s_dyn, [&](const u32* s_w, u32 n, u64 c0) {
    const u64 j0 = c0 / 2;
    const u32 np = (n + 1) / 2, off = s_off;
    // a rank > 0 whose r-first positions are sparse had k_dl_gq write its leaves (by rank, in
    // the segment where rank 0's r-first work sets the pace): measured at 1 Gbase over 8 ranks,
    // rank 1's 0.67 M leaves cost ~50 us here against ~27 us there; rank 0 writes here, where it
    // is the lightest rank (its 4.2 M leaves over 8 Gbase: ~60 us here, ~140 us there)
    const bool dense = a.me == 0 || !dl_rleaves_sparse(a.leaf[1], P.S);
#pragma unroll 4
    for (u32 jj = threadIdx.x; jj < np; jj += kDThreads) {
      const u64 j = j0 + jj;
      const unsigned char f = a.gnf[j];
      const u32 g = a.gid[j];
      const u64 fw = dense ? fb[(c0 + 2 * jj) >> 6] : 0ull;   // (the pair's two positions share a word)
      const u32 sh = u32(c0 + 2 * jj) & 63u;
      const u32 l = s_w[2 * jj], r = 2 * jj + 1 < n ? s_w[2 * jj + 1] : kNullWord;
      if ((fw >> sh) & 1ull)
        leaves_out[(l & kIdx) - s_loff] = code2_leaf(((pw[c0 + 2 * jj] & kIdx) * P.Kinv) & P.hmask, P.L);
      if (2 * jj + 1 < n && ((fw >> (sh + 1)) & 1ull))
        leaves_out[(r & kIdx) - s_loff] = code2_leaf(((pw[c0 + 2 * jj + 1] & kIdx) * P.Kinv) & P.hmask, P.L);
      u32 cl, cr, m, t;
      node_canonical(l, r, cl, cr, m, t);
      const u32 v = ulw(l) == ulw(xf(r, 1, 0));
      u32 id = g;
      if (!f) {
        const u32 lr = g & ~kLocalId;
        a.nodes[lr] = make_uint2(cl, cr);
        id = off + lr;
      }
      a.words0[j] = make_word(id, m, t, v);
    }
  });
}

}  // namespace gcz_dev
