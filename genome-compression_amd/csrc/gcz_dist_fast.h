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
//       count: the one mid-build host read -- the path, the keys' all-to-all sizes)
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
// Only then are the layer-0 nodes written, canonicalised with the global leaf ids (k_fl_l0).
// Any surprise (a non-ACGT strand or repetitive data at R1, an owner that cannot take the
// two-pass dedupe, a C/D slot overflow, a look-ahead that finds layer 1 not direct, an owner
// bucket overflow) makes every rank discard the attempt together and run the general schedule
// (gcz_group::build's exchange loop), which handles every input.
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

// Layer 0's records per owner, per tile of kTile pairs (the bucketing's count pass over the
// pre-words: k_bucket_scatter with RecSrc::pre follows and reads the keys this pass leaves in
// rs.pkey), and what the exchange expects zeroed: the global flags and the rank scan's
// look-back words; count_out = the pairs.
[[maybe_unused]] static __global__ __launch_bounds__(kBlock) void k_fl_count(RecSrc rs, u32* __restrict__ blockcnt, u32 nb,
                                                         unsigned char* __restrict__ gnf,
                                                         unsigned char* __restrict__ gmul, u64* __restrict__ ddesc,
                                                         u64* __restrict__ count_out) {
  __shared__ u32 h[kMaxRanks];
  const int tid = threadIdx.x;
  const u64 p = rs.p;
  {
    const u64 end = blockIdx.x + 1 == gridDim.x ? p + 1 : std::min<u64>(u64(blockIdx.x + 1) * kTile, p + 1);
    const u64 e0 = u64(blockIdx.x) * kTile / 16, e1 = (end + 15) / 16;
    for (u64 e = e0 + tid; e < e1; e += kBlock) {
      reinterpret_cast<uint4*>(gnf)[e] = make_uint4(0, 0, 0, 0);
      reinterpret_cast<uint4*>(gmul)[e] = make_uint4(0, 0, 0, 0);
    }
    if (tid == 0) ddesc[blockIdx.x] = 0;
  }
  if (tid < int(rs.R)) h[tid] = 0;
  if (blockIdx.x == 0 && tid == 0) *count_out = p;
  __syncthreads();
  // one LDS atomic per (wave, item, destination): the lanes sharing a destination found by a
  // ballot per destination bit (R <= 8 addresses: per-lane atomics would serialize on them)
  constexpr int kB = 8;
  const u32 dbits = rs.R > 1 ? 32u - u32(__clz(int(rs.R - 1))) : 0u;
  const u64 lt = (1ull << (tid & 63)) - 1ull;
  for (int e0 = 0; e0 < kItems; e0 += kB) {
    u64 key[kB];
    u32 lid[kB];
    bool ok[kB];
#pragma unroll
    for (int q = 0; q < kB; ++q) {
      const u64 e = u64(blockIdx.x) * kTile + u64(e0 + q) * kBlock + tid;
      ok[q] = rec_get_canon(rs, e, key[q], lid[q]);
      if (e < p) rs.pkey[e] = ok[q] ? key[q] : ~0ull;
    }
#pragma unroll
    for (int q = 0; q < kB; ++q) {
      const u32 d = ok[q] ? rec_dest(rs, key[q]) : 0u;
      u64 m = __ballot(ok[q]);
      for (u32 bit = 0; bit < dbits; ++bit) {
        const bool set = (d >> bit) & 1u;
        const u64 bb = __ballot(ok[q] && set);
        m &= set ? bb : ~bb;
      }
      if (ok[q] && (m & lt) == 0) atomicAdd(&h[d], u32(__popcll(m)));
    }
  }
  __syncthreads();
  if (tid < int(rs.R)) blockcnt[u64(tid) * nb + blockIdx.x] = h[tid];
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
  // R5's D records (the owners' ids of this rank's not-first pairs): each
  // block writes the ones of its own pairs into gid before reading them
  const u64* rd;
  Displ SD;
  const u32* sidx;
  u32* bad;
};
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
  const u64 cc0 = u64(blockIdx.x) * kDC;
  const u32 npp = u32((std::min<u64>(P.S - cc0, kDC) + 1) / 2);
  {   // D: the ids of this chunk's not-first pairs whose first holder is another rank
    const u64 j0 = cc0 / 2, j1 = j0 + npp;
    for (u32 q = 0; q < a.R; ++q) {
      const u64 n = a.rd[u64(q) * kFlSeg];
      if (n > kFlCap) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.bad, 1u);
        continue;
      }
      for (u64 i = threadIdx.x; i < n; i += kDThreads) {
        const u64 v = a.rd[u64(q) * kFlSeg + 1 + i];
        const u32 j = a.sidx[a.SD.d[q] + u32(v)];
        if (j >= j0 && j < j1) a.gid[j] = u32(v >> 32);
      }
    }
    __threadfence_block();   // (this workgroup reads them back: no device-scope fence, an L2 write-back)
    __syncthreads();
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
