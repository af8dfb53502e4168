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
//   R1  allgather: presence bitmaps + status words + layer-0 owner counts
//       (the one mid-build host read: status -> path, counts -> exact all-to-all sizes)
//   R2  keys to owners (code labels) | leaf G arrays, relay 1
//   R3  owner replies | leaf G arrays, relay 2 | allgather of the owners' not-first counts
//       per source (-> every rank's layer-0 id offset, no count round of its own)
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
// rank's r-first counts itself (the general schedule allgathers them).  One block per bucket.
[[maybe_unused]] static __global__ __launch_bounds__(256) void k_fl_counts(const unsigned long long* __restrict__ pbs,
                                                       u64 stride, int R, DensePlan P, u32* __restrict__ cntb) {
  __shared__ u32 s_c[kMaxRanks];
  const int tid = threadIdx.x;
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
      if ((tid & 63) == 0 && v) atomicAdd(&s_c[q], v);
    }
  __syncthreads();
  if (tid < R) cntb[u64(tid) * P.NB + b] = s_c[tid];
}

// One block: per rank q the exclusive prefix of its per-bucket counts into the layout of the
// general schedule's gathered exchange vectors (xvs[q * xw + 2 + b], k_dl_ids_mr reads them)
// with the total at xvs[q * xw]; and the compact vector the host reads at the mid-build sync:
// mid[q * (4 + R) + j] = rank q's status words and owner counts (behind its bitmap in pbs),
// mid[R * (4 + R) + q] = c_q.
[[maybe_unused]] static __global__ __launch_bounds__(kDThreads) void k_fl_prefix(const u32* __restrict__ cntb, int R, DensePlan P,
                                                         u64 xw, u32* __restrict__ xvs,
                                                         const unsigned long long* __restrict__ pbs, u64 stride,
                                                         u64 nw, u64* __restrict__ mid) {
  __shared__ u32 s_tmp[16];
  const int tid = threadIdx.x;
  for (int q = 0; q < R; ++q) {
    u32 total;
    const u32 x = u32(tid) < P.NB ? cntb[u64(q) * P.NB + tid] : 0u;
    const u32 e = block_excl(x, s_tmp, &total);
    if (u32(tid) < P.NB) xvs[u64(q) * xw + 2 + tid] = e;
    if (tid == 0) {
      xvs[u64(q) * xw] = total;
      xvs[u64(q) * xw + 1] = 0;
      mid[u64(R) * (4 + R) + q] = total;
    }
    if (tid < 4 + R) mid[u64(q) * (4 + R) + tid] = pbs[u64(q) * stride + nw + tid];
  }
}

// The owner's not-first records counted per source rank (its dedupe's list): a source's
// globally-first layer-0 pairs are its pairs minus the not-first ones at every owner.
[[maybe_unused]] static __global__ __launch_bounds__(256) void k_fl_ownnf(const u32* __restrict__ olist,
                                                      const u32* __restrict__ ocnt, Displ D, u32 R,
                                                      u64* __restrict__ onf) {
  __shared__ u32 s_c[kMaxRanks];
  if (threadIdx.x < R) s_c[threadIdx.x] = 0;
  __syncthreads();
  const u32 n = *ocnt;
  for (u32 i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) atomicAdd(&s_c[seg_of(D, R, olist[i])], 1u);
  __syncthreads();
  if (threadIdx.x < R && s_c[threadIdx.x])
    atomicAdd(reinterpret_cast<unsigned long long*>(&onf[threadIdx.x]), (unsigned long long)s_c[threadIdx.x]);
}

struct FlPairs {   // layer-0 pairs of every rank (host-known from the plan)
  u64 p[kMaxRanks];
};

// Layer-0 id offsets from the gathered not-first counts (gonf[o * R + s] = owner o's
// not-first records of source s): u_s = p_s - sum_o gonf[o R + s], off[s] = u_0 + .. + u_{s-1};
// offs[R + 1] = this rank's u.
[[maybe_unused]] static __global__ void k_fl_offs(const u64* __restrict__ gonf, u32 R, FlPairs pp, u32 me,
                                                  u64* __restrict__ offs) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  u64 o = 0;
  for (u32 s = 0; s < R; ++s) {
    u64 nf = 0;
    for (u32 q = 0; q < R; ++q) nf += gonf[u64(q) * R + s];
    const u64 u = pp.p[s] - nf;
    offs[s] = o;
    if (s == me) offs[R + 1] = u;
    o += u;
  }
  offs[R] = o;
}

// C at a first holder: (index within its segment to owner q, global id) into q's slot.
[[maybe_unused]] static __global__ __launch_bounds__(256) void k_fl_cvals(const u32* __restrict__ clist,
                                                      const u32* __restrict__ ccount, const u32* __restrict__ sidx,
                                                      Displ SD, u32 R, const u32* __restrict__ gid,
                                                      const u64* __restrict__ offs, u32 me, u64* __restrict__ cbuf,
                                                      u32* __restrict__ bad) {
  const u32 n = *ccount;
  for (u32 i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const u32 k = clist[i];
    const u32 q = seg_of(SD, R, k);
    const u64 slot = atomicAdd(reinterpret_cast<unsigned long long*>(&cbuf[u64(q) * kFlSeg]), 1ull);
    if (slot >= kFlCap) {
      atomicOr(bad, 1u);
      continue;
    }
    const u32 id = u32(offs[me] + (gid[sidx[k]] & ~kLocalId));
    cbuf[u64(q) * kFlSeg + 1 + slot] = u64(k - SD.d[q]) | (u64(id) << 32);
  }
}

// C at the owner: the first holder's global id of each shared key into the key's id slot.
[[maybe_unused]] static __global__ __launch_bounds__(256) void k_fl_setid(const u64* __restrict__ rc, Displ D, u32 R,
                                                      const u32* __restrict__ oslot, OwnTab T,
                                                      u32* __restrict__ bad) {
  for (u32 s = 0; s < R; ++s) {
    const u64 n = rc[u64(s) * kFlSeg];
    if (n > kFlCap) {
      if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(bad, 1u);
      continue;
    }
    for (u64 i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
      const u64 v = rc[u64(s) * kFlSeg + 1 + i];
      own_set_id(T, oslot[D.d[s] + u32(v)], u32(v >> 32));
    }
  }
}

// D at the owner: every not-first record (the dedupe's list) gets its key's id back, into the
// slot of the record's source.
[[maybe_unused]] static __global__ __launch_bounds__(256) void k_fl_getid(const u32* __restrict__ olist,
                                                      const u32* __restrict__ ocnt, const u32* __restrict__ oslot,
                                                      Displ D, u32 R, OwnTab T, u64* __restrict__ dbuf,
                                                      u32* __restrict__ bad) {
  const u32 n = *ocnt;
  for (u32 i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
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

// D at a holder: the global id of each of its not-first pairs.
[[maybe_unused]] static __global__ __launch_bounds__(256) void k_fl_dvals(const u64* __restrict__ rd, Displ SD, u32 R,
                                                      const u32* __restrict__ sidx, u32* __restrict__ gid,
                                                      u32* __restrict__ bad) {
  for (u32 q = 0; q < R; ++q) {
    const u64 n = rd[u64(q) * kFlSeg];
    if (n > kFlCap) {
      if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(bad, 1u);
      continue;
    }
    for (u64 i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
      const u64 v = rd[u64(q) * kFlSeg + 1 + i];
      gid[sidx[SD.d[q] + u32(v)]] = u32(v >> 32);
    }
  }
}

// R4's vector of this rank: {look-ahead pairs (k_lookahead added them), failure so far}
[[maybe_unused]] static __global__ void k_fl_r4pack(DistHdr* __restrict__ dh) { dh->fl_r4[1] = dh->fl_bad; }

// R4's gathered vectors {look-ahead pairs, failure flags} of every rank -> one word: 0 when
// layer 1 is direct everywhere and no rank failed (the direct subtrees' guard).
[[maybe_unused]] static __global__ void k_fl_guard(const u64* __restrict__ g4, u32 R, u64* __restrict__ guard) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  u64 t = 0;
  for (u32 s = 0; s < R; ++s) t += g4[2 * s] + g4[2 * s + 1];
  *guard = t;
}

// Layer 0 with the global leaf ids (emplace_node, src/shared_tree.cpp:662-672): the pair's
// canonical node and bits; a globally-first pair takes id off + its local rank and writes its
// node at that rank in the rank's slice; the others take the id D delivered.  Four pairs per
// thread, their loads issued together.
[[maybe_unused]] static __global__ __launch_bounds__(kBlock) void k_fl_l0(const u32* __restrict__ in, u64 n, u64 p,
                                                      const unsigned char* __restrict__ gnf,
                                                      const u32* __restrict__ gid, const u64* __restrict__ offs,
                                                      u32 me, uint2* __restrict__ nodes, u32* __restrict__ words) {
  constexpr int kB = 4;
  const u64 j0 = (u64(blockIdx.x) * kBlock * kB) + threadIdx.x;
  u32 l[kB], r[kB], g[kB];
  unsigned char f[kB];
#pragma unroll
  for (int q = 0; q < kB; ++q) {
    const u64 j = j0 + u64(q) * kBlock;
    l[q] = r[q] = kNullWord;
    g[q] = 0;
    f[q] = 0;
    if (j < p) {
      load_pair(in, n, j, l[q], r[q]);
      g[q] = gid[j];
      f[q] = gnf[j];
    }
  }
  const u32 off = u32(offs[me]);
#pragma unroll
  for (int q = 0; q < kB; ++q) {
    const u64 j = j0 + u64(q) * kBlock;
    if (j >= p) continue;
    u32 cl, cr, m, t;
    node_canonical(l[q], r[q], cl, cr, m, t);
    const u32 v = ulw(l[q]) == ulw(xf(r[q], 1, 0));
    u32 id = g[q];
    if (!f[q]) {
      const u32 lr = g[q] & ~kLocalId;
      nodes[lr] = make_uint2(cl, cr);
      id = off + lr;
    }
    words[j] = make_word(id, m, t, v);
  }
}

// The final vector of a fast-schedule rank: the general one (k_dist_final) plus failure bit 2
// (a C/D overflow, a look-ahead that found layer 1 not direct) and [3] = this rank's layer-0
// uniques.
[[maybe_unused]] static __global__ void k_fl_final(const Header* __restrict__ h, DistHdr* __restrict__ dh, int tail0,
                                                   int D, int has_tail, const u32* __restrict__ bad,
                                                   const u64* __restrict__ guard, const u64* __restrict__ offs,
                                                   u32 R) {
  dh->final_vec[0] = u64(h->overflow | h->leaf_overflow) | ((*bad || *guard) ? 2ull : 0ull);
  dh->final_vec[1] = has_tail ? u64(h->root) : 0ull;
  dh->final_vec[2] = u64(tail0);
  dh->final_vec[3] = offs[R + 1];
  for (int k = 0; k < GCZ_MAX_LAYERS; ++k)
    dh->final_vec[4 + k] = (has_tail && k >= tail0 && k < D) ? h->count[kLayerSlot + k] : 0ull;
}

}  // namespace gcz_dev
