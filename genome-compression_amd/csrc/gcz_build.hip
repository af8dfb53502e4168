// MI355X (gfx950) shared_tree construction: host orchestration and the C ABI.
// Device code and the algorithm description: gcz_device.h; the multi-rank
// build: gcz_dist.hip.
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>

#include "gcz_ctx.h"
#include "gcz_dense.h"
#include "gcz_scan.h"

using namespace gcz_dev;
using namespace gcz_host;

void gcz_dist_state_free(gcz_ctx* c);   // gcz_dist.hip
void gcz_sort_state_free(gcz_ctx* c);   // gcz_sort.hip
void gcz_ingest_state_free(gcz_ctx* c); // gcz_ingest.hip

namespace {

template <class Tab>
void launch_leaf_bases(int L, dim3 g, hipStream_t st, const unsigned char* b, u64 i0, u64 i1, const Tab& T,
                       u32* rec, unsigned char* nf, Header* hdr, u64* lkey) {
  switch (L) {
#define GCZ_CASE(X) \
  case X: hipLaunchKernelGGL((k_leaf_bases<X, Tab>), g, dim3(kBlock), 0, st, b, i0, i1, T, rec, nf, hdr, lkey); break;
    GCZ_CASE(1) GCZ_CASE(2) GCZ_CASE(3) GCZ_CASE(4) GCZ_CASE(5) GCZ_CASE(6) GCZ_CASE(7) GCZ_CASE(8)
    GCZ_CASE(9) GCZ_CASE(10) GCZ_CASE(11) GCZ_CASE(12) GCZ_CASE(13) GCZ_CASE(14) GCZ_CASE(15) GCZ_CASE(16)
#undef GCZ_CASE
    default: break;
  }
}

}  // namespace

// leaf chunks, geometric: S/64, S/64, S/32, ... S/2 (multiples of the leaf tile);
// the first small chunks discover most keys, the big later ones mostly hit
// settled slots.  Small inputs are one chunk.
std::vector<u64> gcz_host::leaf_chunks(u64 S, int first_log2) {
  std::vector<u64> chunk_start{0};
  const u64 tile = kLeafTile;
  u64 next = std::max<u64>(tile, ((S >> first_log2) + tile - 1) / tile * tile);
  // one chunk up to 2^21 strands (GCZ_LEAF_CHUNKS_FROM overrides: tests chunk small inputs)
  const char* env = std::getenv("GCZ_LEAF_CHUNKS_FROM");
  if (S <= (env ? u64(std::atoll(env)) : (1ull << 21))) next = S;
  bool first = true;
  while (chunk_start.back() < S && int(chunk_start.size()) < kMaxChunks) {
    const u64 c0 = chunk_start.back();
    u64 c1 = std::min(S, c0 + next);
    if (S - c1 < tile) c1 = S;
    chunk_start.push_back(c1);
    if (!first) next *= 2;
    first = false;
  }
  chunk_start.back() = S;
  if (chunk_start.size() == 1) chunk_start.push_back(S);   // S == 0: one empty chunk
  return chunk_start;
}

int gcz_ctx::ensure_marks(u64 S) { return ensure_marks(S, (S + 1) / 2); }

// Set 0: the leaves and the outputs of odd node levels (n0 elements at most); set 1: the
// outputs of even node levels (n1).  A global level loop has n1 = ceil(S / 2); reader-buffer
// segments can make layer 0 longer (up to S pairs for one-strand buffers).
int gcz_ctx::ensure_marks(u64 n0, u64 n1) {
  const u64 b0 = (n0 + 16 + 255) / 256 * 256, b1 = (n1 + 16 + 255) / 256 * 256;
  if (int rc = ensure(nf, b0 + b1)) return rc;             // [leaf / outputs of odd layers][of even layers]
  if (int rc = ensure(multi, b0 + b1)) return rc;
  nf_set[0] = nf.as<unsigned char>();
  nf_set[1] = nf.as<unsigned char>() + b0;
  multi_set[0] = multi.as<unsigned char>();
  multi_set[1] = multi.as<unsigned char>() + b0;
  return GCZ_OK;
}

int gcz_ctx::leaf_level(const LeafLevel& a, Header* d_hdr) {
  if (a.S == 0) return GCZ_OK;
  const u32 limit = a.adaptive ? kAdaptiveProbeLimit : kMaxProbe;
  const int L = a.L;
  // packed leaves only from bases (< 2^4L by construction); user leaves may carry any bits.
  // Chunked settling needs one spare bit in the packed word, hence K + 1.
  // Chunked settling needs two spare bits in the packed word (settled, seeded-global), hence K + 2.
  LevelTab lt = plan_table(tab.ptr, a.cap, a.bases ? 4 * u32(L) + 2 : 64, std::max(a.S, a.seed_n + 1), 0,
                           allow_packed && a.bases, limit);
  if (lt.packed) {
    lt.pt.limit = std::min(lt.pt.limit, limit);
    lt.pt.kmask >>= 2;                   // the key itself has 4L bits
    lt.pt.sh = (4 * u32(L) + 1) / 2;
    lt.pt.cas_first = cap_boost > 0;   // sparse small-build table: the home slot is mostly free
  }
  unsigned char* d_nf = nf_set[0];
  hipEvent_t e0{};
  if (a.c_begin == 0 && !a.precleared) {
    prof_begin(KID_MEMSET, e0);
    HIP_TRY(hipMemsetAsync(tab.ptr, 0xff, lt.bytes(), stream));
    HIP_TRY(hipMemsetAsync(d_nf, 0, a.S, stream));
    prof_end(KID_MEMSET, e0);
  }
  if (a.seed && a.seed_n && lt.packed) {   // (a wide table just goes without: seeding only saves work)
    prof_begin(KID_LEAF, e0);
    hipLaunchKernelGGL(k_leaf_seed, dim3(unsigned((a.seed_n + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream,
                       a.seed, a.seed_n, lt.pt, &d_hdr->leaf_overflow);
    HIP_TRY(hipGetLastError());
    prof_end(KID_LEAF, e0);
  }
  u32* A = a.words;
  const int C = a.c_end >= 0 ? a.c_end : int(a.chunk_start.size()) - 1;
  for (int c = a.c_begin; c < C; ++c) {
    const u64 i0 = a.chunk_start[c], i1 = a.chunk_start[c + 1];
    const dim3 g(unsigned((i1 - i0 + kBlock - 1) / kBlock));
    prof_begin(KID_LEAF, e0);
    if (a.bases) {
      const auto* b = static_cast<const unsigned char*>(a.bases);
      if (lt.packed) launch_leaf_bases(L, g, stream, b, i0, i1, lt.pt, A, d_nf, d_hdr, a.lkey);
      else launch_leaf_bases(L, g, stream, b, i0, i1, lt.wt, A, d_nf, d_hdr, a.lkey);
    } else {
      hipLaunchKernelGGL((k_leaf_packed<WideTab>), g, dim3(kBlock), 0, stream, a.leaves, i0, i1, L, lt.wt, A,
                         d_nf, d_hdr, a.lkey);
    }
    HIP_TRY(hipGetLastError());
    // repetitive data? (switches the node inserts' LDS pre-dedupe; a small build's node
    // levels gain nothing from it: no probe there, predup stays off unless forced)
    if (c == 0 && (predup_mode != 0 || a.S >= kDupProbeMin)) {
      const u64 ip = std::min(i1, i0 + (u64(1) << 21));   // a sample of up to 2^21 strands is enough
      if (predup_mode == 0)
        hipLaunchKernelGGL(k_dup_probe, dim3(unsigned((ip - i0 + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream,
                           A, i0, ip, d_hdr);
      hipLaunchKernelGGL(k_dup_decide, dim3(1), dim3(1), 0, stream, d_hdr, ip - i0, u32(predup_mode));
    }
    prof_end(KID_LEAF, e0);
    const u64 tile = scan_tile(i1 - i0);
    const dim3 gs(unsigned((i1 - i0 + tile - 1) / tile));
    const u64* id0 = c == 0 ? nullptr : &a.count[c - 1];
    prof_begin(KID_FLAGSCAN_LEAF, e0);
    u64* ldesc = i1 - i0 <= kSmallScanMax && i0 % 256 == 0 ? nullptr : a.desc + a.desc_off[c];
#define GCZ_FLAGSCAN_LEAF(TAB, TV, IT)                                                                   \
  hipLaunchKernelGGL((k_flagscan_leaf<TAB, IT>), gs, dim3(kBlock), 0, stream, A, i0, i1, TV, d_nf,      \
                     ldesc, &a.ticket[c], a.out, id0, &a.count[c], a.lkey, a.lsid)
    if (lt.packed) {
      if (tile == u64(kTile)) GCZ_FLAGSCAN_LEAF(PackedTab, lt.pt, kItems);
      else if (tile == u64(kTileSmall)) GCZ_FLAGSCAN_LEAF(PackedTab, lt.pt, kItemsSmall);
      else GCZ_FLAGSCAN_LEAF(PackedTab, lt.pt, kItemsTiny);
    } else {
      if (tile == u64(kTile)) GCZ_FLAGSCAN_LEAF(WideTab, lt.wt, kItems);
      else if (tile == u64(kTileSmall)) GCZ_FLAGSCAN_LEAF(WideTab, lt.wt, kItemsSmall);
      else GCZ_FLAGSCAN_LEAF(WideTab, lt.wt, kItemsTiny);
    }
#undef GCZ_FLAGSCAN_LEAF
    HIP_TRY(hipGetLastError());
    prof_end(KID_FLAGSCAN_LEAF, e0);
    if (a.defer_resolve && c + 1 == C) break;   // settled by level 0's insert (fused small build)
    prof_begin(KID_RESOLVE_LEAF, e0);
    if (lt.packed)
      hipLaunchKernelGGL((k_resolve_leaf<PackedTab>), g, dim3(kBlock), 0, stream, A, i0, i1, lt.pt, d_nf);
    else
      hipLaunchKernelGGL((k_resolve_leaf<WideTab>), g, dim3(kBlock), 0, stream, A, i0, i1, lt.wt, d_nf);
    HIP_TRY(hipGetLastError());
    prof_end(KID_RESOLVE_LEAF, e0);
  }
  return GCZ_OK;
}

namespace {

template <bool kBases>
void launch_dl_pack(int L, dim3 g, hipStream_t st, const unsigned char* b, const u64* lv, const DensePlan& P,
                    u32* pw, u32* cnt, Header* hdr, uint4* zdesc, u64 nz16) {
  switch (L) {
#define GCZ_CASE(X)                                                                                          \
  case X:                                                                                                    \
    hipLaunchKernelGGL((k_dl_pack<X, kBases>), g, dim3(kDThreads), 0, st, b, lv, P, pw, cnt, hdr, zdesc,   \
                       nz16);                                                                                \
    break;
    GCZ_CASE(1) GCZ_CASE(2) GCZ_CASE(3) GCZ_CASE(4) GCZ_CASE(5) GCZ_CASE(6) GCZ_CASE(7) GCZ_CASE(8)
    GCZ_CASE(9) GCZ_CASE(10) GCZ_CASE(11) GCZ_CASE(12)
#undef GCZ_CASE
    default: break;
  }
}

template <class F>
hipError_t allow_lds(F f, int bytes) {   // dynamic LDS above the default 64 KB
  return hipFuncSetAttribute(reinterpret_cast<const void*>(f), hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

}  // namespace

int gcz_ctx::dense_phase_a(const LeafLevel& a, Header* d_hdr, u64* ucount, bool check, bool list, bool* used,
                           u64* vec, bool pack_only) {
  *used = false;
  const u64 S = a.S;
  const u32 L = u32(a.L);
  if (L < 1 || L > 12 || S == 0) return GCZ_OK;
  DensePlan& P = dl_plan;
  P = DensePlan{};
  P.S = S;
  P.L = L;
  P.xcd = dl_xcd;
  P.nch = u32((S + kDC - 1) / kDC);
  P.cmask = u32((1ull << (2 * L)) - 1);
  const u32 cbits = dense_code_bits(L);
  P.hmask = u32((1ull << cbits) - 1);
  // dense_nb buckets (GCZ_DENSE_NB; a power of two <= kDNBMax), at least enough that a bucket's
  // LDS table holds at most 2^14 codes (k_dl_first's 16 codes per thread)
  P.NB = u32(std::min<u64>(std::max<u64>({u64(dense_nb), (1ull << cbits) >> 14, 1}), 1ull << cbits));
  P.NB = std::min<u32>(1u << log2_exact(P.NB), kDNBMax);
  P.IB = cbits - log2_exact(P.NB);
  const u32 kmul = 0x5bd1e995u;                     // odd: a bijection mod 4^L
  u32 Ki = kmul;
  for (int i = 0; i < 5; ++i) Ki *= 2u - kmul * Ki;   // inverse mod 2^32 (hence mod 4^L)
  P.K = kmul & P.hmask;   // (odd: a bijection mod 2^cbits)
  P.Kinv = Ki & P.hmask;
  const u64 ncnt = u64(P.NB) * P.nch;
  const u64 nfb = (S + 63) / 64;
  const u64 t_cnt = scan_tiles(ncnt + 1), t_fb = scan_tiles(nfb + 1);
  const u64 ncodes = u64(1) << cbits;
  int rc;
  if ((rc = ensure(dl_pw, S * 4 + 16)) || (rc = ensure(dl_rec, S * 4 + 16)) || (rc = ensure(dl_idrec, S * 4 + 16)) ||
      (rc = ensure(dl_cnt, ncnt * 4 + 16)) || (rc = ensure(dl_off, (ncnt + 1) * 4 + 16)) ||
      (rc = ensure(dl_offt, (ncnt + P.NB) * 4 + 16)) ||
      (rc = ensure(dl_fpg, ncodes * 4 + 16)) || (rc = ensure(dl_fb, u64(P.nch) * (kDC / 64) * 8 + 16)) ||
      (rc = ensure(dl_wpre, (nfb + 1) * 4 + 16)) || (rc = ensure(dl_desc, (t_cnt + t_fb) * 8 + 32)) ||
      (rc = ensure(dl_fl, ncodes * 4 + 16)) || (rc = ensure(dl_fo, u64(P.NB) * (P.nch + 1) * 4 + 16)))
    return rc;
  if (list && (rc = ensure(dl_pb, (ncodes / 64 + 1) * 8))) return rc;
  const int first_bytes = int(((1u << P.IB) + P.nch + 1) * 4);
  if (first_bytes > 160 * 1024) return GCZ_OK;   // (never at L <= 12, S < 2^29)
  const int scat_bytes = int((kDC + 3 * kDNBMax + 1 + 16 + kDC / 64) * 4);
  HIP_TRY(allow_lds(k_dl_scatter, scat_bytes));
  HIP_TRY(allow_lds(k_dl_first, first_bytes));
  hipEvent_t e0{};
  prof_begin(KID_DL_PACK, e0);
  const u64 nz16 = ((t_cnt + t_fb) * 8 + 16 + 15) / 16;   // (the descriptors and the two tickets; dl_desc holds 16 B more)
  if (a.bases)
    launch_dl_pack<true>(int(L), dim3(P.nch), stream, static_cast<const unsigned char*>(a.bases), nullptr, P,
                         dl_pw.as<u32>(), dl_cnt.as<u32>(), d_hdr, static_cast<uint4*>(dl_desc.ptr), nz16);
  else
    launch_dl_pack<false>(int(L), dim3(P.nch), stream, nullptr, a.leaves, P, dl_pw.as<u32>(), dl_cnt.as<u32>(),
                          d_hdr, static_cast<uint4*>(dl_desc.ptr), nz16);
  HIP_TRY(hipGetLastError());
  prof_end(KID_DL_PACK, e0);
  prof_begin(KID_DL_PROBE, e0);
  // repetitive data? (the node inserts' LDS pre-dedupe): in-block repeats of a sample's
  // hashed codes (equal codes <=> equal keys)
  // (a rank of an R-rank build samples the first 1/R of that, at least 2^18, of its own
  // slice: R prefixes, not a spread over the genome; the decision is OR-ed over the ranks
  // and written back into every rank's header before the node levels, gcz_dist.hip)
  const u64 ip = std::min<u64>(S, std::max<u64>(u64(1) << 18, (u64(1) << 21) / std::max(1u, probe_ranks)));
  hipLaunchKernelGGL(k_dup_probe, dim3(unsigned((ip + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream,
                     dl_pw.as<u32>(), u64(0), ip, d_hdr);
  hipLaunchKernelGGL(k_dup_decide, dim3(1), dim3(1), 0, stream, d_hdr, ip, u32(predup_mode));
  HIP_TRY(hipGetLastError());
  if (check) {   // single device: the pure-ACGT verdict, read after the scatter is queued (below)
    if (!ev_dfail) HIP_TRY(hipEventCreateWithFlags(&ev_dfail, hipEventDisableTiming));
    HIP_TRY(hipMemcpyAsync(&h_hdr->dense_fail, &d_hdr->dense_fail, 4, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipEventRecord(ev_dfail, stream));
  }
  prof_end(KID_DL_PROBE, e0);
  if (pack_only) {   // (the fused multi-rank schedule queues its own work before the rest)
    *used = true;
    return GCZ_OK;
  }
  if (int rc2 = dense_phase_a2(a)) return rc2;
  if (check) {
    // the host waits for the pack's verdict only, while the scan and scatter (harmless on a
    // failed pack: rejected strands carry no record) keep the device busy
    HIP_TRY(hipEventSynchronize(ev_dfail));
    if (h_hdr->dense_fail) {   // the hash-table leaf level follows: no repetitive-data verdict from here
      // (the probe's counts too: they were taken over the rejected pack's pre-words, and the
      // hash-table level's own probe adds into the same shards; dupstat sits right before predup)
      static_assert(offsetof(Header, predup) == offsetof(Header, dupstat) + sizeof(Header::dupstat),
                    "dupstat and predup are cleared as one range");
      HIP_TRY(hipMemsetAsync(&d_hdr->dupstat[0], 0, sizeof(d_hdr->dupstat) + sizeof(d_hdr->predup), stream));
      return GCZ_OK;
    }
  }
  *used = true;
  return dense_phase_a3(d_hdr, ucount, list, vec);
}

// scan of the (bucket, chunk) counts and the records' scatter into bucket order
int gcz_ctx::dense_phase_a2(const LeafLevel& a) {
  (void)a;
  const DensePlan& P = dl_plan;
  const u64 ncnt = u64(P.NB) * P.nch, nfb = (P.S + 63) / 64;
  const u64 t_cnt = scan_tiles(ncnt + 1), t_fb = scan_tiles(nfb + 1);
  u64* sdesc = dl_desc.as<u64>();
  u32* tickets = reinterpret_cast<u32*>(sdesc + t_cnt + t_fb);
  const int scat_bytes = int((kDC + 3 * kDNBMax + 1 + 16 + kDC / 64) * 4);
  hipEvent_t e0{};
  prof_begin(KID_DL_SCAN, e0);
  hipLaunchKernelGGL(k_scan_excl<ScanU32>, dim3(unsigned(t_cnt)), dim3(kScanThreads), 0, stream,
                     ScanU32{dl_cnt.as<u32>(), ncnt}, ncnt + 1, dl_off.as<u32>(), sdesc, &tickets[0],
                     static_cast<u64*>(nullptr));
  hipLaunchKernelGGL(k_dl_tr, dim3((P.nch + 1 + 31) / 32, (P.NB + 31) / 32), dim3(256), 0, stream, dl_off.as<u32>(),
                     P.NB, P.nch + 1, u64(P.nch), dl_offt.as<u32>());
  HIP_TRY(hipGetLastError());
  prof_end(KID_DL_SCAN, e0);
  prof_begin(KID_DL_SCATTER, e0);
  hipLaunchKernelGGL(k_dl_scatter, dim3(P.nch), dim3(kDThreads), scat_bytes, stream, dl_pw.as<u32>(), P,
                     dl_offt.as<u32>(), dl_rec.as<u32>());
  HIP_TRY(hipGetLastError());
  prof_end(KID_DL_SCATTER, e0);
  return GCZ_OK;
}

// first positions; single device: + the first bitmap and its popcount scan (the unique count);
// multi-rank (list): + the presence bitmap and the status words only -- the r-first filter,
// position bitmap and ranks follow the bitmap exchange (gcz_dist.hip)
int gcz_ctx::dense_phase_a3(Header* d_hdr, u64* ucount, bool list, u64* vec, u32* rfc, u32* bcnt) {
  const DensePlan& P = dl_plan;
  const u64 ncnt = u64(P.NB) * P.nch, nfb = (P.S + 63) / 64;
  const u64 t_cnt = scan_tiles(ncnt + 1), t_fb = scan_tiles(nfb + 1);
  const u64 ncodes = u64(1) << dense_code_bits(P.L);
  u64* sdesc = dl_desc.as<u64>();
  u32* tickets = reinterpret_cast<u32*>(sdesc + t_cnt + t_fb);
  const int first_bytes = int(((1u << P.IB) + P.nch + 1) * 4);
  hipEvent_t e0{};
  prof_begin(KID_DL_FIRST, e0);
  if (list && (1u << P.IB) < 64) HIP_TRY(hipMemsetAsync(dl_pb.ptr, 0, (ncodes / 64 + 1) * 8, stream));
  hipLaunchKernelGGL(k_dl_first, dim3(P.NB), dim3(kDThreads), first_bytes, stream, dl_rec.as<u32>(), dl_off.as<u32>(),
                     P, rfc ? nullptr : dl_fpg.as<u32>(), (list && !rfc) ? nullptr : dl_fl.as<u32>(), dl_fo.as<u32>(),
                     list ? dl_pb.as<unsigned long long>() : nullptr, static_cast<const Header*>(d_hdr),
                     list ? vec : nullptr, rfc, bcnt);
  HIP_TRY(hipGetLastError());
  if (list) {
    prof_end(KID_DL_FIRST, e0);
    return GCZ_OK;
  }
  hipLaunchKernelGGL(k_dl_fb, dim3(P.nch), dim3(kDThreads), 0, stream, dl_fl.as<u32>(), dl_fo.as<u32>(), P,
                     dl_fb.as<unsigned long long>());
  HIP_TRY(hipGetLastError());
  prof_end(KID_DL_FIRST, e0);
  prof_begin(KID_DL_FBSCAN, e0);
  hipLaunchKernelGGL(k_scan_excl<ScanPopc>, dim3(unsigned(t_fb)), dim3(kScanThreads), 0, stream,
                     ScanPopc{dl_fb.as<unsigned long long>()}, nfb, dl_wpre.as<u32>(), sdesc + t_cnt, &tickets[1],
                     ucount);
  HIP_TRY(hipGetLastError());
  if (dl_fbw_on) {
    if (int rc = ensure(dl_fbw, nfb * 16 + 16)) return rc;
    hipLaunchKernelGGL(k_dl_fbw, dim3(unsigned((nfb + 255) / 256)), dim3(256), 0, stream, dl_fb.as<unsigned long long>(),
                       dl_wpre.as<u32>(), nfb, static_cast<uint4*>(dl_fbw.ptr));
    HIP_TRY(hipGetLastError());
  }
  prof_end(KID_DL_FBSCAN, e0);
  return GCZ_OK;
}

int gcz_ctx::dense_phase_b(const LeafLevel& a, Header* d_hdr, const u32* gid, u64* leaves, bool ids_done) {
  (void)d_hdr;
  const DensePlan& P = dl_plan;
  const int RBbytes = int((1u << P.IB) * 4);
  const int words_bytes = int((kDC + 2 * kDNBMax + 1 + 16 + kDC / 32 + kDC / 64) * 4);
  HIP_TRY(allow_lds(k_dl_ids, RBbytes));
  HIP_TRY(allow_lds(k_dl_words, words_bytes));
  hipEvent_t e0{};
  if (!ids_done) {   // (multi-rank: k_dl_ids_mr wrote the final words per record)
    prof_begin(KID_DL_IDS, e0);
    hipLaunchKernelGGL(k_dl_ids, dim3(P.NB), dim3(kDThreads), RBbytes, stream, dl_rec.as<u32>(), dl_off.as<u32>(), P,
                       dl_fpg.as<u32>(), dl_fb.as<unsigned long long>(), dl_wpre.as<u32>(), gid, dl_idrec.as<u32>(),
                       dl_fbw_on && !gid ? static_cast<const uint4*>(dl_fbw.ptr) : nullptr);
    HIP_TRY(hipGetLastError());
    prof_end(KID_DL_IDS, e0);
  }
  prof_begin(KID_DL_WORDS, e0);
  hipLaunchKernelGGL(k_dl_words, dim3(P.nch), dim3(kDThreads), words_bytes, stream, dl_rec.as<u32>(),
                     dl_idrec.as<u32>(), dl_offt.as<u32>(), P, dl_fb.as<unsigned long long>(), a.words, leaves);
  HIP_TRY(hipGetLastError());
  prof_end(KID_DL_WORDS, e0);
  return GCZ_OK;
}

int gcz_ctx::leaf_level_dense(const LeafLevel& a, Header* d_hdr, u64* ucount, bool* used) {
  if (int rc = dense_phase_a(a, d_hdr, ucount, true, false, used)) return rc;
  if (!*used) return GCZ_OK;
  return dense_phase_b(a, d_hdr, nullptr, a.out);
}

int gcz_ctx::node_level(const NodeLevel& a, Header* d_hdr) {
  const u64 p = a.p, n = a.n;
  if (p == 0) return GCZ_OK;
  const u64 cap = node_cap(p);
  const u32 Bk = std::max<u32>(1, bit_width(a.bound));
  LevelTab nt = plan_table(a.fused ? a.ftab : tab.ptr, cap, 2 * (Bk + 2), p, Bk, allow_packed, kMaxProbe);
  nt.pt.cas_first = cap_boost > 0;
  const int cur = (a.k + 1) & 1, prev = a.k & 1;
  unsigned char* knf = nf_set[cur];
  u32* in = const_cast<u32*>(a.in);   // (written only by a fused insert, which settles it)
  if (a.direct_known) {   // *pcount == n is set: the insert writes words and nodes, nothing else runs
    hipEvent_t e0{};
    prof_begin(KID_NODE, e0);
    const dim3 gi(unsigned((p + kBlock - 1) / kBlock));
    hipLaunchKernelGGL((k_node_insert<WideTab, NoRes>), gi, dim3(kBlock), 0, stream, in, n, p, WideTab{}, nullptr,
                       nullptr, a.words, Marks{knf, multi_set[cur]}, d_hdr, a.pcount, a.out, a.count, a.id_off,
                       stats.as<u64>(), 0u, NoRes{}, FuseIn{});
    HIP_TRY(hipGetLastError());
    prof_end(KID_NODE, e0);
    return GCZ_OK;
  }
  const Marks mk{knf, multi_set[cur]};
  const unsigned char* pnf = a.prev_nf ? a.prev_nf : a.prev_marks ? nf_set[prev] : nullptr;
  const unsigned char* pmu = a.prev_nf ? a.prev_multi : a.prev_marks ? multi_set[prev] : nullptr;
  Group* d_grp = grp.as<Group>();
  // bucketed insert (decided on the device: hdr->predup == 0) when the buckets average
  // <= 2560 pairs (the LDS dedupe holds 4608) and a record fits 8 bytes
  BktPlan bp{};
  bp.T = nt.pt;
  bp.K = 2 * (Bk + 2);
  // (up to 2^16 buckets through the two-pass partition: 256 coarse x 256 fine, e.g. 133 M pairs
  // on layer 0 of a 3.2 Gbase genome; the single pass counts at most 2^14 in LDS)
  const u32 bb_max = two_pass ? kPartMaxB1 + kFineMaxB2 : u32(kBktMaxLog);
  while (bp.bb < bb_max && (p >> bp.bb) > 2560) ++bp.bb;
  u32 bkt = a.allow_bucket && bucket_now && nt.packed && p >= bucket_min && (p >> bp.bb) <= 2560 &&
            bp.K >= bp.bb && bp.K - bp.bb + kBktRP <= 64 &&
            p <= u64(kBktMaxG) * kBktChunk ? 1u : 0u;
  const u32 bb = bp.bb;
  const u64 G = (p + kBktChunk - 1) / kBktChunk;
  const u64 ncnt = (u64(1) << bb) * G + 1;
  const u64 t_scan = scan_tiles(ncnt);   // look-back scan of the count matrix: descriptors + ticket
  // two-pass partition (k_bkt_part / fine / dedupe2) when a record holds the key's low
  // K - bb bits and its position in a fine slice
  Bkt2Plan b2{};
  b2.T = nt.pt;
  b2.K = bp.K;
  b2.b1 = std::min<u32>(bb, kPartMaxB1);
  b2.b2 = bb - b2.b1;
  b2.G = (p + kPartChunk - 1) / kPartChunk;
  const u64 mean_run = std::max<u64>(1, std::min<u64>(p, kPartChunk) >> b2.b1);   // records per (chunk, coarse)
  b2.SC = u32(std::max<u64>(1, std::min<u64>(128, u64(kFineCap / 2) / mean_run)));
  b2.SC = 1u << log2_exact(b2.SC);   // a power of two
  b2.P = kPartLog + log2_exact(b2.SC);
  b2.nslice = u32((b2.G + b2.SC - 1) / b2.SC);
  const bool two = bkt && two_pass && b2.b2 <= u32(kFineMaxB2) && bp.K - b2.b1 + kPartLog <= 64 &&
                   bp.K - bb + b2.P <= 64 && mean_run * b2.SC <= u64(kFineCap) / 2 && b2.nslice <= 512;
  if (two) bkt = 2;   // (the two-pass partition also takes repetitive data: kernels see bkt 2)
  else if (a.repetitive || bb > u32(kBktMaxLog)) bkt = 0;   // (the single pass would skip on the device)
  if (two) {
    int rc;
    const u64 nfine = (u64(1) << b2.b1) * b2.nslice;
    if ((rc = ensure(bkt_key, b2.G * kPartChunk * 8)) ||
        (rc = ensure(bkt_cnt, b2.G * ((u64(1) << b2.b1) + 1) * 4 + 16)) ||
        (rc = ensure(bkt_rec2, nfine * kFineCap * 8)) ||
        (rc = ensure(bkt_off, nfine * ((u64(1) << b2.b2) + 1) * 4 + 16)))
      return rc;
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(k_bkt_part),
                                hipFuncAttributeMaxDynamicSharedMemorySize, int(kPartChunk * 8)));
    HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(k_bkt_fine),
                                hipFuncAttributeMaxDynamicSharedMemorySize, int(kFineCap * 8)));
  } else if (bkt) {
    int rc;
    if ((rc = ensure(bkt_key, p * 8)) || (rc = ensure(bkt_cnt, ncnt * 4)) ||
        (rc = ensure(bkt_off, ncnt * 4)) || (rc = ensure(bkt_tmp, t_scan * 8 + 16)))
      return rc;
    HIP_TRY(hipMemsetAsync(bkt_tmp.ptr, 0, t_scan * 8 + 16, stream));
  }
  // two-pass levels: k_bkt_part writes every mark itself (the clear only zeroed marks there),
  // and the dedupe lists the level's not-first positions for the sparse flag scan
  b2.wmarks = two && part_marks ? 1u : 0u;
  b2.wave1 = part_wave ? 1u : 0u;
  b2.xcd = bkt_xcd;
  if (two && !a.fused && part_words_off) {   // (no provisional words on collapse-free levels)
    b2.in = a.in;
    b2.n = n;
  }
  if (two && sparse_scan) {
    if (int rc = ensure(nf_list, kNfListCap * 4 + 16)) return rc;
    b2.nfl = nf_list.as<u32>();
  }
  hipEvent_t e0{};
  if (!a.fused && !b2.wmarks) {
    prof_begin(KID_MEMSET, e0);
    const u64 tab16 = nt.bytes() / 16, p16 = (p + 15) / 16;
    const u64 blocks = std::min<u64>(4096, (std::max(tab16, p16) + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_clear, dim3(unsigned(blocks)), dim3(kBlock), 0, stream, static_cast<uint4*>(tab.ptr),
                       tab16, reinterpret_cast<uint4*>(knf), reinterpret_cast<uint4*>(mk.multi), p16, a.pcount, n,
                       d_hdr, bkt);
    HIP_TRY(hipGetLastError());
    prof_end(KID_MEMSET, e0);
  }
  const dim3 gi(unsigned((p + kBlock - 1) / kBlock));
  if (two) {
    prof_begin(KID_BKT_SCATTER, e0);
    hipLaunchKernelGGL(k_bkt_part, dim3(unsigned(b2.G)), dim3(kBktThreads), size_t(kPartChunk) * 8, stream, a.in,
                       n, p, pnf, pmu, b2, bkt_key.as<u64>(), bkt_cnt.as<u32>(), a.words, mk, d_hdr, a.pcount,
                       stats.as<u64>(), a.out, a.count, a.id_off);
    HIP_TRY(hipGetLastError());
    prof_end(KID_BKT_SCATTER, e0);
    prof_begin(KID_BKT_FINE, e0);
    hipLaunchKernelGGL(k_bkt_fine, dim3(unsigned((u64(1) << b2.b1) * b2.nslice)), dim3(kBktThreads),
                       size_t(kFineCap) * 8, stream, bkt_key.as<u64>(), bkt_cnt.as<u32>(), b2, bkt_rec2.as<u64>(),
                       bkt_off.as<u32>(), d_hdr, a.pcount, n, &d_hdr->bkt_overflow);
    HIP_TRY(hipGetLastError());
    prof_end(KID_BKT_FINE, e0);
    prof_begin(KID_BKT_DEDUPE, e0);
    if (dedupe_bm) {
      // the bitmap dedupe; buckets over its capacity (hot keys of repetitive data) go to
      // k_bkt_dedupe2 in a second launch of a few workgroups that takes them from a list (empty:
      // they exit at once)
      if (int rc = ensure(bkt_redo, (u64(1) << kBktMaxLog) * 4 + 16)) return rc;
      Bkt2Plan bm = b2;
      bm.redo = bkt_redo.as<u32>();
      bm.redo_cnt = &d_hdr->redo[a.k];
      hipLaunchKernelGGL(k_bkt_dedupe_bm<false>, dim3(1u << bb), dim3(kBmThreads), 0, stream, bkt_rec2.as<u64>(),
                         bkt_off.as<u32>(), bm, a.words, mk, d_hdr, a.pcount, n, &d_hdr->bkt_overflow);
      hipLaunchKernelGGL(k_bkt_dedupe2_redo, dim3(64), dim3(kBktThreads), 0, stream, bkt_rec2.as<u64>(),
                         bkt_off.as<u32>(), bm, a.words, mk, d_hdr, a.pcount, n, &d_hdr->bkt_overflow);
    } else
      hipLaunchKernelGGL(k_bkt_dedupe2<false>, dim3(1u << bb), dim3(kBktThreads), 0, stream, bkt_rec2.as<u64>(),
                         bkt_off.as<u32>(), b2, a.words, mk, d_hdr, a.pcount, n, &d_hdr->bkt_overflow);
    HIP_TRY(hipGetLastError());
    prof_end(KID_BKT_DEDUPE, e0);
  } else if (bkt) {
    prof_begin(KID_BKT_COUNT, e0);
    hipLaunchKernelGGL(k_bkt_count, dim3(unsigned(G)), dim3(kBktThreads), 0, stream, a.in, n, p, pnf, pmu, bp,
                       bkt_cnt.as<u32>(), G, d_hdr, a.pcount, stats.as<u64>());
    HIP_TRY(hipGetLastError());
    prof_end(KID_BKT_COUNT, e0);
    prof_begin(KID_BKT_SCAN, e0);
    hipLaunchKernelGGL(k_scan_excl<ScanU32>, dim3(unsigned(t_scan)), dim3(kScanThreads), 0, stream,
                       ScanU32{bkt_cnt.as<u32>(), ncnt - 1}, ncnt, bkt_off.as<u32>(), bkt_tmp.as<u64>(),
                       reinterpret_cast<u32*>(bkt_tmp.as<u64>() + t_scan), static_cast<u64*>(nullptr));
    HIP_TRY(hipGetLastError());
    prof_end(KID_BKT_SCAN, e0);
    prof_begin(KID_BKT_SCATTER, e0);
    hipLaunchKernelGGL(k_bkt_scatter, dim3(unsigned(G)), dim3(kBktThreads), 0, stream, a.in, n, p, pnf, pmu, bp,
                       bkt_off.as<u32>(), G, bkt_key.as<u64>(), a.words, d_hdr, a.pcount);
    HIP_TRY(hipGetLastError());
    prof_end(KID_BKT_SCATTER, e0);
    prof_begin(KID_BKT_DEDUPE, e0);
    hipLaunchKernelGGL(k_bkt_dedupe, dim3(1u << bb), dim3(kBktThreads), size_t(G) * 4, stream, bkt_off.as<u32>(), G,
                       bkt_key.as<u64>(), a.words, mk, d_hdr, a.pcount, n);
    HIP_TRY(hipGetLastError());
    prof_end(KID_BKT_DEDUPE, e0);
  }
  prof_begin(KID_NODE, e0);
  FuseIn fz{};
  u64 clr16 = 0;   // fused: marks of the next level, cleared by the flag scan
  if (a.fused) {
    if (a.k > 0) {
      fz.pcount = &d_hdr->count[kLayerSlot + a.k - 1];
      fz.phashed = &d_hdr->hashed_next[a.k - 1];
      fz.gate_out = &d_hdr->gate[a.k - 1];
    }
    if (a.p_next) {
      const u32 Bn = std::max<u32>(1, bit_width(p));
      fz.clear = static_cast<uint4*>(a.ftab_next);
      fz.clear16 = plan_table(a.ftab_next, node_cap(a.p_next), 2 * (Bn + 2), a.p_next, Bn, allow_packed, kMaxProbe)
                       .bytes() / 16;
      clr16 = (a.p_next + 15) / 16;
    }
  }
  auto insert = [&](auto T, auto res) {
    hipLaunchKernelGGL((k_node_insert<decltype(T), decltype(res)>), gi, dim3(kBlock), 0, stream, in, n, p, T, pnf,
                       pmu, a.words, mk, d_hdr, a.pcount, a.out, a.count, a.id_off, stats.as<u64>(), bkt, res, fz);
  };
  auto insert_settling = [&](auto T) {   // the resolver of the previous level (fused builds)
    if (!a.fused) insert(T, NoRes{});
    else insert(T, SlotRes{nf_set[prev], a.sid_prev});   // (k = 0: the leaves' ids by slot)
  };
  if (two && !a.fused) {
    // two-pass levels: k_bkt_part inserts (or, on a level that turned out direct, writes the
    // words and nodes itself), so the insert would only launch p / 256 empty workgroups
  } else if (nt.packed) {
    insert_settling(nt.pt);
  } else {
    insert_settling(nt.wt);
  }
  HIP_TRY(hipGetLastError());
  prof_end(KID_NODE, e0);
  uint4* clr_nf = reinterpret_cast<uint4*>(nf_set[prev]);
  uint4* clr_mu = reinterpret_cast<uint4*>(multi_set[prev]);
  prof_begin(KID_FLAGSCAN_NODE, e0);
  const u64 tile = scan_tile(p);
  const dim3 gs(unsigned((p + tile - 1) / tile));
  u64* ndesc = p <= kSmallScanMax ? nullptr : a.desc;   // small levels: no look-back chain
  // large levels: the tiles' prefixes counted ahead instead of the look-back (GCZ_TILE_COUNT)
  u32* tpre = nullptr;
  if (ndesc && tile_count && !a.fused) {
    const u64 nt = (p + tile - 1) / tile;
    const void* had = tcount.ptr;
    if (int rc = ensure(tcount, nt * 4 + 64)) return rc;
    if (tcount.ptr != had) HIP_TRY(hipMemsetAsync(tcount.ptr, 0, 64, stream));   // (the done counter, once)
    tpre = tcount.as<u32>() + 16;
    auto count = [&](auto items) {
      hipLaunchKernelGGL((k_tile_count<decltype(items)::value>), gs, dim3(kBlock), 0, stream, knf, p, a.pcount, n,
                         tpre, tcount.as<u32>(), static_cast<const u32*>(b2.nfl), static_cast<const u32*>(&d_hdr->nnf),
                         bkt == 2 ? static_cast<const u32*>(&d_hdr->predup) : nullptr);
    };
    if (tile == u64(kTile)) count(std::integral_constant<int, kItems>{});
    else count(std::integral_constant<int, kItemsSmall>{});
  }
  auto flagscan = [&](auto items) {
    hipLaunchKernelGGL((k_flagscan_node<decltype(items)::value>), gs, dim3(kBlock), 0, stream, a.words, p, a.in, n,
                       knf, d_grp, ndesc, a.ticket, a.out, a.count, a.pcount, mk.multi, a.hashed_next, clr_nf, clr_mu,
                       clr16, a.fused && (!a.fused_last || a.tail_settles) ? a.sid : nullptr,
                       bkt == 2 ? static_cast<const u32*>(&d_hdr->predup) : nullptr, b2.nfl,
                       static_cast<const u32*>(&d_hdr->nnf), static_cast<const u32*>(tpre));
  };
  if (tile == u64(kTile)) flagscan(std::integral_constant<int, kItems>{});
  else if (tile == u64(kTileSmall)) flagscan(std::integral_constant<int, kItemsSmall>{});
  else flagscan(std::integral_constant<int, kItemsTiny>{});
  HIP_TRY(hipGetLastError());
  prof_end(KID_FLAGSCAN_NODE, e0);
  // the next level's insert (or the tail) settles the repeats
  if (a.fused && (!a.fused_last || a.tail_settles)) return GCZ_OK;
  prof_begin(KID_RESOLVE_NODE, e0);
  const dim3 gr(resolve_grid ? unsigned(std::min<u64>(gi.x, resolve_grid)) : gi.x);
  if (nt.packed)
    hipLaunchKernelGGL((k_resolve_node<PackedTab>), gr, dim3(kBlock), 0, stream, a.words, p, nt.pt, knf, d_grp,
                       a.pcount, n, a.count, a.hashed_next, a.gate, d_hdr, bkt, b2.nfl ? 1u : 0u);
  else
    hipLaunchKernelGGL((k_resolve_node<WideTab>), gr, dim3(kBlock), 0, stream, a.words, p, nt.wt, knf, d_grp,
                       a.pcount, n, a.count, a.hashed_next, a.gate, d_hdr, bkt, b2.nfl ? 1u : 0u);
  HIP_TRY(hipGetLastError());
  prof_end(KID_RESOLVE_NODE, e0);
  return GCZ_OK;
}

int gcz_ctx::direct_levels(const u32* in, int k0, int nlev, const DirectPlan& dp, u32* out, Header* d_hdr,
                           const DirectRemap& rm, const u64* guard, u64 expect) {
  hipEvent_t e0{};
  prof_begin(KID_DIRECT, e0);
  const u64 blocks = (dp.n[0] + kDirectChunk - 1) / kDirectChunk;
  hipLaunchKernelGGL(k_direct_levels, dim3(unsigned(blocks)), dim3(kBlock), 0, stream, in, k0, nlev,
                     nodes_out.as<uint2>(), dp, out, d_hdr, rm, guard, expect);
  HIP_TRY(hipGetLastError());
  prof_end(KID_DIRECT, e0);
  return GCZ_OK;
}

int gcz_ctx::tail_levels(const u32* in, u64 n0, const u64* pcount, int k0, int D, const std::vector<u64>& layer_off_,
                         Header* d_hdr, const u64* shards, const TailSettle& st) {
  TailOut to{};
  for (int k = k0; k < D; ++k) to.layer_off[k] = layer_off_[k];
  hipEvent_t e0{};
  prof_begin(KID_TAIL, e0);
  HIP_TRY(hipFuncSetAttribute(reinterpret_cast<const void*>(k_tail), hipFuncAttributeMaxDynamicSharedMemorySize,
                              int(kTailLds)));
  hipLaunchKernelGGL(k_tail, dim3(1), dim3(kTailThreads), kTailLds, stream, in, n0, pcount, k0, D, nodes_out.as<uint2>(), to,
                     d_hdr, shards, st);
  HIP_TRY(hipGetLastError());
  prof_end(KID_TAIL, e0);
  return GCZ_OK;
}

int gcz_ctx::build(const void* d_bases, const u64* d_leaves, u64 nbases, u64 S, int L) {
  info = gcz_info{};
  info.L = L;
  info.status = GCZ_OK;
  if (L < 1 || L > 16) return fail(GCZ_ERR_ARG, "build", "leaf length L must be in 1..16");
  if (d_bases) S = nbases / u64(L);
  if (S == 0) return fail(GCZ_ERR_EMPTY, "build", "fewer than L bases: nothing to build");
  // reader-buffer segments of segB strands (one build only); a single buffer or a power of
  // two >= 2 pairs exactly like the global level loop.  (Buffers of one strand
  // are not: each strand becomes a unary layer-0 node of its own.)
  u64 segB = segment_strands;
  segment_strands = 0;
  if (segB >= S || (segB >= 2 && (segB & (segB - 1)) == 0)) segB = 0;
  // positions are 29-bit fields of the words: longer genomes run as virtual ranks
  if (S > u64(kIdx) || split_min_strands < S) {
    if (segB)
      return fail(GCZ_ERR_CAPACITY, "build", "reader buffers that are not a power of two need at most 2^29-1 strands");
    return gcz_split_build(this, d_bases, d_leaves, S, L);
  }
  info.n_strands = S;

  // ---- plan: node layers, leaf chunks, scan descriptor regions ----
  // Segmented levels k < seg_d (the depth of one full buffer's subtree): full segments hold
  // seg_bk[k] input elements; where that is odd the input is expanded to seg_ne[k] elements
  // (k_seg_expand), one null after every segment but the last.
  int seg_d = 0;
  u64 nseg = 0;
  std::vector<u64> seg_bk, seg_ne;
  if (segB) {
    seg_d = std::max<int>(1, int(bit_width(segB - 1)));
    nseg = (S + segB - 1) / segB;
  }
  std::vector<u64> pk;                     // pairs per node layer
  for (u64 n = S;;) {
    u64 ne = n;
    if (int(pk.size()) < seg_d) {
      const int k = int(pk.size());
      const u64 bk = (segB + (u64(1) << k) - 1) >> k;
      if (bk & 1) ne = n + nseg - 1;
      seg_bk.push_back(bk);
      seg_ne.push_back(ne);
    }
    const u64 p = (ne + 1) / 2;
    pk.push_back(p);
    if (p == 1) break;
    n = p;
  }
  if (pk.size() > GCZ_MAX_LAYERS) return fail(GCZ_ERR_CAPACITY, "build", "too many layers");
  const int D = int(pk.size());
  layer_off.assign(D + 1, 0);
  for (int k = 0; k < D; ++k) layer_off[k + 1] = layer_off[k] + pk[k];
  const std::vector<u64> chunk_start = leaf_chunks(S, leaf_first_log2);
  const int C = int(chunk_start.size()) - 1;
  std::vector<u64> desc_off;
  u64 ntiles_total = 0;
  for (int c = 0; c < C; ++c) {
    desc_off.push_back(ntiles_total);
    const u64 len = chunk_start[c + 1] - chunk_start[c];
    ntiles_total += (len + scan_tile(len) - 1) / scan_tile(len);
  }
  for (int k = 0; k < D; ++k) {
    desc_off.push_back(ntiles_total);
    ntiles_total += (pk[k] + scan_tile(pk[k]) - 1) / scan_tile(pk[k]);
  }

  // leaf table: big enough for S when S is small; otherwise start at 2^24 slots
  // (every ACGT 12-mer class fits) and grow after an overflow.
  const u64 full_cap = std::max<u64>(256, next_pow2(2 * S));
  u64 leaf_cap = full_cap;
  // (each call starts here: no state carries over between builds; a probe overflow
  // grows the table and rebuilds, counted in info.attempts)
  if (S > (1ull << 22)) leaf_cap = std::min(full_cap, u64(1) << 24);
  if (leaf_cap_log2 > 0 && S > (1ull << 22)) leaf_cap = std::min(full_cap, 1ull << leaf_cap_log2);
  // small builds: a launch lasts as long as its longest probe chain, so their tables are
  // sparser (a few MB at most)
  const bool small = S <= 2 * kDirectCheckMin;
  if (small) leaf_cap = full_cap << (small_leaf_shift >= 0 ? small_leaf_shift : small_cap_shift);
  cap_boost = small ? small_cap_shift : 0;
  const u64 node_cap0 = node_cap(pk[0]);

  int rc;
  if ((rc = ensure(wa, S * 4 + 16))) return rc;
  if ((rc = ensure(wb, (seg_d ? S : (S + 1) / 2) * 4 + 16))) return rc;
  if (seg_d) {
    const u64 ne_max = *std::max_element(seg_ne.begin(), seg_ne.end());
    if ((rc = ensure(seg_w, ne_max * 4 + 16)) || (rc = ensure(seg_nf, ne_max + 16)) || (rc = ensure(seg_mu, ne_max + 16)))
      return rc;
  }
  if ((rc = ensure(grp, ((S + 63) / 64 + kGroupsPerTile) * sizeof(Group)))) return rc;
  if ((rc = ensure(desc, ntiles_total * 8 + 64))) return rc;
  if ((rc = ensure(leaves_out, S * 8 + 16))) return rc;
  if ((rc = ensure(nodes_out, layer_off[D] * 8 + 16))) return rc;
  if ((rc = ensure(hdr, sizeof(Header)))) return rc;
  if ((rc = ensure(stats, kStatBytes))) return rc;
  {   // marks of every level's output, by parity (k_clear / the flag scans write pk[k] of set (k + 1) & 1)
    u64 n0 = S, n1 = 0;
    for (int k = 0; k < D; ++k) (k & 1 ? n0 : n1) = std::max(k & 1 ? n0 : n1, pk[k]);
    if ((rc = ensure_marks(n0, n1))) return rc;
  }
  if (!h_hdr) HIP_TRY(hipHostMalloc((void**)&h_hdr, sizeof(Header), hipHostMallocDefault));

  Header* d_hdr = hdr.as<Header>();
  u32* A = wa.as<u32>();
  u32* Bw = wb.as<u32>();
  u64* d_desc = desc.as<u64>();

  if (!ev_start) {
    HIP_TRY(hipEventCreate(&ev_start));
    HIP_TRY(hipEventCreate(&ev_stop));
  }

  allow_packed = !force_wide;
  bucket_now = use_bucket;
  const bool try_dense = dense_mode != 0 && L <= 12 && (S >= dense_min || dense_mode == 2);
  for (;;) {
    if ((rc = ensure(tab, std::max(leaf_cap, node_cap0) * 16))) return rc;
    // small build, one leaf chunk, no bucketed level, no host look at a gate: two launches
    // per node level (FuseIn, gcz_device.h), the node tables in three regions of ftab
    const bool fused = use_fused && !seg_d && !try_dense && C == 1 && pk[0] < kDirectCheckMin &&
                       !(bucket_now && pk[0] >= bucket_min) && (S > u64(kTailMaxN) || !use_tail);
    const u64 fregion = node_cap0 * 16;
    if (fused && ((rc = ensure(ftab, 3 * fregion)) || (rc = ensure(fsid, 3 * node_cap0 * 4)) ||
                  (rc = ensure(flkey, S * 8 + 16)) || (rc = ensure(flsid, leaf_cap * 4)))) return rc;
    auto fregion_ptr = [&](int k) { return static_cast<void*>(ftab.as<unsigned char>() + u64(k % 3) * fregion); };
    // One build's launches, start event to header copy.  A build whose launch sequence
    // has no host decision inside (no dense-level fallback check, no look at the direct
    // gate: small genomes) is captured once as a HIP graph and replayed while the shape
    // and buffers stay the same -- its ~30 short kernels are otherwise bound by the
    // host's per-launch cost.
    auto enqueue = [&]() -> int {
      HIP_TRY(hipEventRecord(ev_start, stream));
      {   // header, descriptors, statistics and (hash-table leaf level) its table and marks: one launch
        InitPlan ip{};
        ip.hdr = d_hdr;
        ip.desc = static_cast<uint4*>(desc.ptr);
        ip.ndesc16 = (ntiles_total * 8 + 15) / 16;
        ip.stats = static_cast<uint4*>(stats.ptr);
        ip.nstats16 = kStatBytes / 16;
        if (!try_dense) {
          const LevelTab lt = plan_table(tab.ptr, leaf_cap, d_bases ? 4 * u32(L) + 2 : 64, S, 0,
                                         allow_packed && d_bases, leaf_cap < 2 * S ? kAdaptiveProbeLimit : kMaxProbe);
          ip.tab = static_cast<uint4*>(tab.ptr);
          ip.ntab16 = lt.bytes() / 16;
          ip.nf = reinterpret_cast<uint4*>(nf_set[0]);
          ip.nnf16 = (S + 15) / 16;
        }
        if (fused) {   // level 0's table and marks
          const u32 B0 = std::max<u32>(1, bit_width(std::min(S, leaf_cap)));
          ip.ftab = static_cast<uint4*>(fregion_ptr(0));
          ip.nftab16 = plan_table(ip.ftab, node_cap0, 2 * (B0 + 2), pk[0], B0, allow_packed, kMaxProbe).bytes() / 16;
          ip.fnf = reinterpret_cast<uint4*>(nf_set[1]);
          ip.fmulti = reinterpret_cast<uint4*>(multi_set[1]);
          ip.nfm16 = (pk[0] + 15) / 16;
        }
        const u64 big = std::max<u64>({ip.ndesc16, ip.nstats16, ip.ntab16, ip.nnf16, ip.nftab16, ip.nfm16});
        hipLaunchKernelGGL(k_build_init, dim3(unsigned(std::min<u64>(4096, (big + kBlock - 1) / kBlock))),
                           dim3(kBlock), 0, stream, ip);
        HIP_TRY(hipGetLastError());
      }

      // ---- leaf level, in chunks ----
      LeafLevel la;
      la.bases = d_bases; la.leaves = d_leaves; la.S = S; la.L = L;
      la.cap = leaf_cap;
      la.adaptive = leaf_cap < 2 * S;
      la.words = A;
      la.out = leaves_out.as<u64>();
      la.chunk_start = chunk_start;
      la.desc = d_desc;
      la.desc_off = desc_off;
      la.count = d_hdr->count;
      la.ticket = d_hdr->ticket;
      dense_used = false;
      la.precleared = !try_dense;
      la.defer_resolve = fused;
      la.lkey = fused ? flkey.as<u64>() : nullptr;
      la.lsid = fused ? flsid.as<u32>() : nullptr;
      if (try_dense) {
        if ((rc = leaf_level_dense(la, d_hdr, &d_hdr->count[C - 1], &dense_used))) return rc;
        if (!dense_used) HIP_TRY(hipMemsetAsync(&d_hdr->dense_fail, 0, 4, stream));
      }
      if (!dense_used && (rc = leaf_level(la, d_hdr))) return rc;

      // ---- node layers ----
      u32* in = A;
      u32* outw = Bw;
      u64 n = S;
      u64 bound = std::min(S, leaf_cap);        // child ids of layer 0 are leaf ids < #slots
      bool tail_done = false, direct = false;
      bool prev_regular = false;   // the previous level ran node_level (its gate is written)
      bool table_only = false;     // hdr->predup seen on the host: no bucketed levels
      for (int k = 0; k < D; ++k) {
        const bool segmented = k < seg_d;   // pairing inside reader buffers
        if (n <= u64(kTailMaxN) && use_tail && !segmented) {   // the rest fits one workgroup: one launch
          const u64* pc = k == 0 ? &d_hdr->count[C - 1] : prev_regular ? &d_hdr->gate[k - 1]
                                                                         : &d_hdr->count[kLayerSlot + k - 1];
          TailSettle st{};
          if (fused && k > 0) {   // the last fused level's repeats and gate
            st.nf = nf_set[k & 1];
            st.sid = fsid.as<u32>() + u64((k - 1) % 3) * node_cap0;
            st.pcount = &d_hdr->count[kLayerSlot + k - 1];
            st.phashed = &d_hdr->hashed_next[k - 1];
            st.gate_out = &d_hdr->gate[k - 1];
          }
          if ((rc = tail_levels(in, n, pc, k, D, layer_off, d_hdr, stats.as<u64>(), st))) return rc;
          tail_done = true;
          break;
        }
        if (direct) {   // host-known: up to kDirectLog levels per launch, ids = positions
          DirectPlan dp{};
          int nlev = 0;
          u64 m = n;
          dp.n[0] = n;
          while (nlev < kDirectLog && k + nlev < D && (m > u64(kTailMaxN) || !use_tail)) {
            dp.layer_off[k + nlev] = layer_off[k + nlev];
            m = pk[k + nlev];
            dp.n[++nlev] = m;
          }
          if (nlev == 0) return fail(GCZ_ERR_ARG, "build", "internal: empty direct step");
          if ((rc = direct_levels(in, k, nlev, dp, outw, d_hdr))) return rc;
          prev_regular = false;
          std::swap(in, outw);
          n = m;
          bound = m;
          k += nlev - 1;
          continue;
        }
        NodeLevel na;
        na.k = k;
        na.in = in; na.n = n; na.p = pk[k];
        if (segmented && seg_ne[k] != n) {   // a null after every odd segment (and its marks)
          const bool marks = k > 0;
          hipLaunchKernelGGL(k_seg_expand, dim3(unsigned((seg_ne[k] + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream,
                             in, marks ? nf_set[k & 1] : nullptr, marks ? multi_set[k & 1] : nullptr, seg_bk[k],
                             seg_ne[k], seg_w.as<u32>(), marks ? seg_nf.as<unsigned char>() : nullptr,
                             marks ? seg_mu.as<unsigned char>() : nullptr);
          HIP_TRY(hipGetLastError());
          na.in = seg_w.as<u32>();
          na.n = seg_ne[k];
          if (marks) {
            na.prev_nf = seg_nf.as<unsigned char>();
            na.prev_multi = seg_mu.as<unsigned char>();
          }
        }
        na.words = outw;
        na.out = nodes_out.as<uint2>() + layer_off[k];
        na.count = &d_hdr->count[kLayerSlot + k];
        na.bound = bound;
        na.prev_marks = k > 0;
        na.pcount = k == 0 ? &d_hdr->count[C - 1] : &d_hdr->gate[k - 1];
        na.desc = d_desc + desc_off[C + k];
        na.ticket = &d_hdr->ticket[kLayerSlot + k];
        // look-ahead for layer k + 1 (its pairs' children are here; not where that layer pairs
        // inside reader buffers)
        na.hashed_next = k + 1 < seg_d ? nullptr : &d_hdr->hashed_next[k];
        na.gate = &d_hdr->gate[k];
        na.allow_bucket = !fused;
        na.repetitive = table_only;
        if (fused) {
          na.fused = true;
          na.ftab = fregion_ptr(k);
          na.ftab_next = fregion_ptr(k + 1);
          na.sid = fsid.as<u32>() + u64(k % 3) * node_cap0;
          na.sid_prev = k > 0 ? fsid.as<u32>() + u64((k - 1) % 3) * node_cap0 : flsid.as<u32>();
          na.p_next = k + 1 < D ? pk[k + 1] : 0;
          na.fused_last = k + 1 == D || (pk[k] <= u64(kTailMaxN) && use_tail);
          na.tail_settles = k + 1 < D && pk[k] <= u64(kTailMaxN) && use_tail;
        }
        if ((rc = node_level(na, d_hdr))) return rc;
        prev_regular = true;
        std::swap(in, outw);
        n = pk[k];
        bound = pk[k];
        // a look at the device after layers 0 and 1: once a gate is open every later
        // level is direct and runs as direct subtrees (saves ~4 launches per level)
        if (k <= 1 && use_direct && n >= kDirectCheckMin && k + 1 >= seg_d) {   // (a host round trip: only where levels are big)
          // the next direct step is launched before the round trip, guarded on the device by
          // the gate (all unique data: the wait overlaps it; otherwise it exits at once)
          DirectPlan sdp{};
          int snlev = 0;
          u64 sm = n;
          if (k + 1 < D && (n > u64(kTailMaxN) || !use_tail)) {
            sdp.n[0] = n;
            while (snlev < kDirectLog && k + 1 + snlev < D && (sm > u64(kTailMaxN) || !use_tail)) {
              sdp.layer_off[k + 1 + snlev] = layer_off[k + 1 + snlev];
              sm = pk[k + 1 + snlev];
              sdp.n[++snlev] = sm;
            }
            if (snlev > 0 && (rc = direct_levels(in, k + 1, snlev, sdp, outw, d_hdr, DirectRemap{}, &d_hdr->gate[k], n)))
              return rc;
          }
          HIP_TRY(hipMemcpyAsync(&h_hdr->gate[k], &d_hdr->gate[k], 8, hipMemcpyDeviceToHost, stream));
          HIP_TRY(hipMemcpyAsync(&h_hdr->predup, &d_hdr->predup, 4, hipMemcpyDeviceToHost, stream));
          HIP_TRY(hipStreamSynchronize(stream));
          direct = h_hdr->gate[k] == n;
          table_only = h_hdr->predup != 0;   // repetitive data: later levels skip the single-pass bucket launches
          if (direct && snlev > 0) {   // the speculative step ran: continue after it
            prev_regular = false;
            std::swap(in, outw);
            n = sm;
            bound = sm;
            k += snlev;
          }
        }
      }
      if (!tail_done) {   // (the tail sums the statistics itself)
        hipLaunchKernelGGL(k_build_finish, dim3(1), dim3(1024), 0, stream, in, stats.as<u64>(), d_hdr);
        HIP_TRY(hipGetLastError());
      }
      HIP_TRY(hipEventRecord(ev_stop, stream));
      HIP_TRY(hipMemcpyAsync(h_hdr, d_hdr, sizeof(Header), hipMemcpyDeviceToHost, stream));
      return GCZ_OK;
    };
    // (a level that may take the bucketed path can allocate inside: never captured; a
    // shape is captured on its second build, once every buffer has its size)
    const bool static_seq = use_graph && !profile && !seg_d && !try_dense && pk[0] < kDirectCheckMin &&
                            !(use_bucket && pk[0] >= bucket_min);
    bool launched = false;
    if (static_seq) {
      const GraphKey key{d_bases, d_leaves, nbases, S, L, leaf_cap, allow_packed, bucket_now, stream,
                         tab.ptr, wa.ptr, wb.ptr, nodes_out.ptr, leaves_out.ptr, nf.ptr, desc.ptr,
                         fused ? ftab.ptr : nullptr, fused ? fsid.ptr : nullptr, fused ? flkey.ptr : nullptr,
                         fused ? flsid.ptr : nullptr, fused};
      if (graph_exec && key == graph_key) {
        launched = hipGraphLaunch(graph_exec, stream) == hipSuccess;
      } else if (!(key == graph_seen)) {
        graph_seen = key;   // first build of this shape: eager
      } else {
        if (graph_exec) (void)hipGraphExecDestroy(graph_exec);
        graph_exec = nullptr;
        if (hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal) == hipSuccess) {
          const int crc = enqueue();
          hipGraph_t g = nullptr;
          const hipError_t ce = hipStreamEndCapture(stream, &g);
          if (crc == GCZ_OK && ce == hipSuccess && g &&
              hipGraphInstantiate(&graph_exec, g, nullptr, nullptr, 0) == hipSuccess) {
            graph_key = key;
            launched = hipGraphLaunch(graph_exec, stream) == hipSuccess;
          }
          if (g) (void)hipGraphDestroy(g);
          if (!launched) {   // capture refused something: run it eagerly
            if (graph_exec) (void)hipGraphExecDestroy(graph_exec);
            graph_exec = nullptr;
            (void)hipGetLastError();
            info.status = GCZ_OK;
            last_error.clear();
          }
        }
      }
    }
    if (!launched && (rc = enqueue())) return rc;
    HIP_TRY(hipStreamSynchronize(stream));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, ev_start, ev_stop));
    info.build_ms = ms;
    info.build_ms_all += ms;
    info.attempts += 1;
    if (profile) prof_collect();
    if (h_hdr->bkt_overflow && bucket_now) {      // a hot key overflowed a bucket: rebuild with the table
      bucket_now = false;
      continue;
    }
    if (h_hdr->leaf_overflow && leaf_cap < 2 * S) {    // leaf table too small: grow and rebuild
      leaf_cap = std::min(full_cap, leaf_cap * 8);
      continue;
    }
    if ((h_hdr->overflow || h_hdr->leaf_overflow) && allow_packed) {   // displacement field overflow
      allow_packed = false;
      continue;
    }
    break;
  }

  if (h_hdr->err_offset != ~0ull) {
    info.error_offset = h_hdr->err_offset;
    unsigned char sym = 0;
    if (d_bases) HIP_TRY(hipMemcpy(&sym, static_cast<const unsigned char*>(d_bases) + h_hdr->err_offset, 1,
                                   hipMemcpyDeviceToHost));
    info.error_symbol = sym;
    return fail(GCZ_ERR_SYMBOL, "build", "unknown nucleotide symbol");
  }
  if (h_hdr->overflow || h_hdr->leaf_overflow)
    return fail(GCZ_ERR_CAPACITY, "build", "hash table probe limit exceeded");
  info.n_layers = D;
  info.n_leaves = h_hdr->count[C - 1];
  for (int k = 0; k < D; ++k) info.layer_size[k] = h_hdr->count[kLayerSlot + k];
  info.root = h_hdr->root;
  for (int i = 0; i < 64; ++i) info.hashed_pairs += h_hdr->hashed[i];
  info.bucketed_pairs = h_hdr->hashed[1];
  info.leaf_path = dense_used ? 1u : 0u;
  info.repetitive = h_hdr->predup;
  info.handed_back = 0;
  for (int k = 0; k < GCZ_MAX_LAYERS; ++k) info.handed_back += h_hdr->redo[k];
  return GCZ_OK;
}

// ---- host -> device upload ----------------------------------------------------------
// The runtime's pageable copy reaches the link's ~56 GB/s once warm (a pinned staging
// ring of 1-8 worker threads measured 30-54 GB/s: tools/microbench/upload.hip,
// profiles/r02/microbench_upload.jsonl).  What costs on a cold process is the first copy
// (~32 GB/s: the runtime's staging path and the destination's first DMA touch), so
// upload_reserve() warms the path with a small copy (the C++ surface runs it while the
// file is mapped) and upload() touches a destination with a memset before the DMA.
int gcz_ctx::upload_reserve(size_t bytes) {
  if (int rc = ensure(input, std::max<size_t>(bytes, size_t(8) << 20) + 16)) return rc;
  HIP_TRY(hipMemsetAsync(input.ptr, 0, input.bytes, stream));
  if (!upload_warm) {
    const size_t n = size_t(8) << 20;
    std::vector<char> h(n, 0);
    HIP_TRY(hipMemcpyAsync(input.ptr, h.data(), n, hipMemcpyHostToDevice, stream));
    upload_warm = true;
  }
  HIP_TRY(hipStreamSynchronize(stream));
  return GCZ_OK;
}

int gcz_ctx::upload(void* d_dst, const void* h_src, size_t n) {
  if (n == 0) return GCZ_OK;
  if (n >= (size_t(64) << 20)) HIP_TRY(hipMemsetAsync(d_dst, 0, n, stream));   // first DMA touch, ~0.2 ms/GB
  HIP_TRY(hipMemcpyAsync(d_dst, h_src, n, hipMemcpyHostToDevice, stream));
  return GCZ_OK;
}

extern "C" {

int gcz_ctx_create(int device, gcz_ctx** out) {
  if (!out) return GCZ_ERR_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return GCZ_ERR_DEVICE;
  if (device < 0 || device >= ndev) return GCZ_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return GCZ_ERR_DEVICE;
  auto* c = new gcz_ctx();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return GCZ_ERR_DEVICE;
  }
  c->stream = c->own_stream;
  if (const char* t = std::getenv("GCZ_CANARY")) c->canary = std::atoi(t) != 0;
  if (const char* t = std::getenv("GCZ_DEDUPE_BM")) c->dedupe_bm = std::atoi(t) != 0;
  if (const char* t = std::getenv("GCZ_DL_FBW")) c->dl_fbw_on = std::atoi(t) != 0;
  if (const char* t = std::getenv("GCZ_PART_WORDS")) c->part_words_off = std::atoi(t) == 0;
  if (const char* t = std::getenv("GCZ_BKT_XCD")) c->bkt_xcd = u32(std::strtoul(t, nullptr, 10));
  if (const char* t = std::getenv("GCZ_DL_XCD")) c->dl_xcd = u32(std::strtoul(t, nullptr, 10));
  if (const char* t = std::getenv("GCZ_DENSE_NB")) c->dense_nb = u32(std::strtoul(t, nullptr, 10));
  if (const char* t = std::getenv("GCZ_TABLE")) c->force_wide = std::strcmp(t, "wide") == 0;
  if (const char* t = std::getenv("GCZ_NODE_CAP_SHIFT")) c->node_cap_shift = std::atoi(t);
  if (const char* t = std::getenv("GCZ_LEAF_CAP_LOG2")) c->leaf_cap_log2 = std::atoi(t);
  if (const char* t = std::getenv("GCZ_TAIL")) c->use_tail = std::atoi(t) != 0;
  if (const char* t = std::getenv("GCZ_DIRECT")) c->use_direct = std::atoi(t) != 0;
  if (const char* t = std::getenv("GCZ_PREDUP")) c->predup_mode = std::atoi(t);   // 1 on, 2 off, 0 auto
  if (const char* t = std::getenv("GCZ_BUCKET")) c->use_bucket = std::atoi(t) != 0;
  if (const char* t = std::getenv("GCZ_BUCKET_MIN")) c->bucket_min = std::strtoull(t, nullptr, 10);
  if (const char* t = std::getenv("GCZ_BUCKET_TWO")) c->two_pass = std::atoi(t) != 0;
  if (const char* t = std::getenv("GCZ_PART_MARKS")) c->part_marks = std::atoi(t) != 0;
  if (const char* t = std::getenv("GCZ_SPARSE_SCAN")) c->sparse_scan = std::atoi(t) != 0;
  if (const char* t = std::getenv("GCZ_PART_WAVE")) c->part_wave = std::atoi(t) != 0;
  if (const char* t = std::getenv("GCZ_TILE_COUNT")) c->tile_count = std::atoi(t) != 0;
  if (const char* t = std::getenv("GCZ_RESOLVE_GRID")) c->resolve_grid = u32(std::strtoul(t, nullptr, 10));
  if (const char* t = std::getenv("GCZ_DENSE")) c->dense_mode = std::atoi(t);
  if (const char* t = std::getenv("GCZ_GRAPH")) c->use_graph = std::atoi(t) != 0;
  if (const char* t = std::getenv("GCZ_FUSED")) c->use_fused = std::atoi(t) != 0;
  if (const char* t = std::getenv("GCZ_SMALL_CAP_SHIFT")) c->small_cap_shift = std::max(0, std::min(4, std::atoi(t)));
  if (const char* t = std::getenv("GCZ_SMALL_LEAF_SHIFT")) c->small_leaf_shift = std::max(0, std::min(4, std::atoi(t)));
  if (const char* t = std::getenv("GCZ_SPLIT_MIN")) c->split_min_strands = std::strtoull(t, nullptr, 10);
  if (const char* t = std::getenv("GCZ_SPLIT_SHARE")) c->split_share = std::max<u64>(1024, std::strtoull(t, nullptr, 10));
  if (const char* t = std::getenv("GCZ_LEAF_FIRST_LOG2")) c->leaf_first_log2 = std::max(1, std::min(20, std::atoi(t)));
  *out = c;
  return GCZ_OK;
}

void gcz_ctx_destroy(gcz_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  gcz_dist_state_free(c);
  gcz_sort_state_free(c);
  gcz_ingest_state_free(c);
  for (DevBuf* b : {&c->wa, &c->wb, &c->grp, &c->desc, &c->tab, &c->leaves_out, &c->nodes_out, &c->hdr, &c->input,
                    &c->nf, &c->multi, &c->stats, &c->bkt_key, &c->bkt_cnt, &c->bkt_off, &c->bkt_tmp, &c->bkt_rec2, &c->dl_pw,
                    &c->dl_rec, &c->dl_idrec, &c->dl_cnt, &c->dl_off, &c->dl_offt, &c->dl_fpg, &c->dl_fb, &c->dl_wpre, &c->dl_fbw,
                    &c->dl_desc, &c->dl_fl, &c->dl_fo, &c->dl_lh, &c->dl_pb, &c->dl_pbs, &c->dl_lower,
                    &c->dl_pos, &c->dl_list, &c->dl_gid, &c->dl_recv, &c->dl_stage, &c->dl_seg, &c->seg_w,
                    &c->seg_nf, &c->seg_mu, &c->seg_in, &c->nf_list, &c->tcount, &c->bkt_redo})
    if (b->ptr) (void)hipFree(b->ptr);
  if (c->h_hdr) (void)hipHostFree(c->h_hdr);
  if (c->h_ring) (void)hipHostFree(c->h_ring);
  for (hipEvent_t e : c->ring_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->graph_exec) (void)hipGraphExecDestroy(c->graph_exec);
  for (auto e : c->event_pool) (void)hipEventDestroy(e);
  if (c->ev_dfail) (void)hipEventDestroy(c->ev_dfail);
  if (c->ev_start) (void)hipEventDestroy(c->ev_start);
  if (c->ev_stop) (void)hipEventDestroy(c->ev_stop);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
}

// The guard bands of GCZ_CANARY=1 (gcz_ctx::ensure): the buffers whose band is not all
// kCanaryByte any more, named where they are context members.
extern "C++" int gcz_canary_scan(gcz_ctx* c, std::string& out) {
  if (!c->canary) return -1;
  if (hipStreamSynchronize(c->stream) != hipSuccess) {
    out += "stream synchronisation failed; ";
    return 1;
  }
  static const std::pair<DevBuf gcz_ctx::*, const char*> names[] = {
      {&gcz_ctx::wa, "wa"}, {&gcz_ctx::wb, "wb"}, {&gcz_ctx::grp, "grp"}, {&gcz_ctx::desc, "desc"},
      {&gcz_ctx::tab, "tab"}, {&gcz_ctx::leaves_out, "leaves_out"}, {&gcz_ctx::nodes_out, "nodes_out"},
      {&gcz_ctx::hdr, "hdr"}, {&gcz_ctx::input, "input"}, {&gcz_ctx::nf, "nf"}, {&gcz_ctx::multi, "multi"},
      {&gcz_ctx::stats, "stats"}, {&gcz_ctx::bkt_key, "bkt_key"}, {&gcz_ctx::bkt_cnt, "bkt_cnt"},
      {&gcz_ctx::bkt_off, "bkt_off"}, {&gcz_ctx::bkt_tmp, "bkt_tmp"}, {&gcz_ctx::bkt_rec2, "bkt_rec2"},
      {&gcz_ctx::dl_pw, "dl_pw"}, {&gcz_ctx::dl_rec, "dl_rec"}, {&gcz_ctx::dl_idrec, "dl_idrec"},
      {&gcz_ctx::dl_cnt, "dl_cnt"}, {&gcz_ctx::dl_off, "dl_off"}, {&gcz_ctx::dl_offt, "dl_offt"},
      {&gcz_ctx::dl_fpg, "dl_fpg"}, {&gcz_ctx::dl_fb, "dl_fb"}, {&gcz_ctx::dl_wpre, "dl_wpre"}, {&gcz_ctx::dl_fbw, "dl_fbw"},
      {&gcz_ctx::dl_desc, "dl_desc"}, {&gcz_ctx::dl_fl, "dl_fl"}, {&gcz_ctx::dl_fo, "dl_fo"},
      {&gcz_ctx::dl_lh, "dl_lh"}, {&gcz_ctx::dl_pb, "dl_pb"}, {&gcz_ctx::dl_pbs, "dl_pbs"},
      {&gcz_ctx::dl_lower, "dl_lower"}, {&gcz_ctx::dl_pos, "dl_pos"}, {&gcz_ctx::dl_list, "dl_list"},
      {&gcz_ctx::dl_gid, "dl_gid"}, {&gcz_ctx::dl_recv, "dl_recv"}, {&gcz_ctx::dl_stage, "dl_stage"},
      {&gcz_ctx::dl_seg, "dl_seg"}, {&gcz_ctx::seg_w, "seg_w"}, {&gcz_ctx::seg_nf, "seg_nf"},
      {&gcz_ctx::seg_mu, "seg_mu"}, {&gcz_ctx::seg_in, "seg_in"}, {&gcz_ctx::nf_list, "nf_list"},
      {&gcz_ctx::tcount, "tcount"}, {&gcz_ctx::bkt_redo, "bkt_redo"}, {&gcz_ctx::ftab, "ftab"}, {&gcz_ctx::fsid, "fsid"},
      {&gcz_ctx::flkey, "flkey"}, {&gcz_ctx::flsid, "flsid"}};
  std::vector<unsigned char> band(gcz_ctx::kCanaryBytes);
  int bad = 0;
  for (size_t k = 0; k < c->canary_bufs.size(); ++k) {
    DevBuf* b = c->canary_bufs[k];
    if (!b->ptr) continue;
    if (hipMemcpy(band.data(), static_cast<char*>(b->ptr) + b->bytes, band.size(), hipMemcpyDeviceToHost) != hipSuccess) {
      out += "band copy failed; ";
      return bad + 1;
    }
    size_t first = band.size();
    for (size_t j = 0; j < band.size(); ++j)
      if (band[j] != gcz_ctx::kCanaryByte) {
        first = j;
        break;
      }
    if (first == band.size()) continue;
    ++bad;
    std::string name = "buffer #" + std::to_string(k) + " (not a context member: multi-rank / sort / ingest state)";
    for (const auto& nm : names)
      if (&(c->*(nm.first)) == b) name = nm.second;
    out += name + " of " + std::to_string(b->bytes) + " B: guard byte +" + std::to_string(first) + " overwritten; ";
  }
  return bad;
}

int gcz_ctx_canary_check(gcz_ctx* c, char* msg, uint64_t cap) {
  if (!c) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  std::string out;
  const int n = gcz_canary_scan(c, out);
  if (msg && cap) std::snprintf(msg, size_t(cap), "%s", out.c_str());
  return n;
}

// The check itself (tests): a scratch buffer of 1000 bytes sized by ensure(), one byte stored
// right past it; returns 0 when the scan reports exactly that buffer.
int gcz_ctx_canary_selftest(gcz_ctx* c) {
  if (!c) return GCZ_ERR_ARG;
  if (!c->canary) return -1;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  DevBuf b;
  if (c->ensure(b, 1000)) return GCZ_ERR_DEVICE;
  std::string out;
  int rc = gcz_canary_scan(c, out) == 0 ? 0 : 1;   // (nothing overwritten yet)
  if (!rc && hipMemsetAsync(static_cast<char*>(b.ptr) + 1000, 0x5A, 1, c->stream) != hipSuccess) rc = 2;
  out.clear();
  if (!rc) rc = gcz_canary_scan(c, out) == 1 && out.find("+0 overwritten") != std::string::npos ? 0 : 3;
  c->canary_bufs.erase(std::remove(c->canary_bufs.begin(), c->canary_bufs.end(), &b), c->canary_bufs.end());
  (void)hipFree(b.ptr);
  return rc;
}

int gcz_ctx_set_stream(gcz_ctx* c, void* s) {
  if (!c) return GCZ_ERR_ARG;
  c->stream = s ? static_cast<hipStream_t>(s) : c->own_stream;
  return GCZ_OK;
}
void* gcz_ctx_stream(gcz_ctx* c) { return c ? c->stream : nullptr; }
const char* gcz_ctx_last_error(gcz_ctx* c) { return c ? c->last_error.c_str() : "null context"; }

void* gcz_dev_alloc(gcz_ctx* c, uint64_t bytes) {
  if (!c || hipSetDevice(c->device) != hipSuccess) return nullptr;
  void* p = nullptr;
  return hipMalloc(&p, bytes ? bytes : 1) == hipSuccess ? p : nullptr;
}

int gcz_dev_free(gcz_ctx* c, void* p) {
  if (!c) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  (void)hipStreamSynchronize(c->stream);
  return hipFree(p) == hipSuccess ? GCZ_OK : GCZ_ERR_DEVICE;
}

int gcz_memcpy_h2d(gcz_ctx* c, void* dst, const void* src, uint64_t bytes) {
  if (!c) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  if (int rc = c->upload(dst, src, bytes)) return rc;
  return hipStreamSynchronize(c->stream) == hipSuccess ? GCZ_OK : GCZ_ERR_DEVICE;
}

int gcz_upload_reserve(gcz_ctx* c, uint64_t bytes) {
  if (!c) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  return c->upload_reserve(bytes);
}

int gcz_memcpy_d2h(gcz_ctx* c, void* dst, const void* src, uint64_t bytes) {
  if (!c) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  if (hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream) != hipSuccess) return GCZ_ERR_DEVICE;
  return hipStreamSynchronize(c->stream) == hipSuccess ? GCZ_OK : GCZ_ERR_DEVICE;
}

int gcz_ctx_sync(gcz_ctx* c) {
  if (!c) return GCZ_ERR_ARG;
  return hipStreamSynchronize(c->stream) == hipSuccess ? GCZ_OK : GCZ_ERR_DEVICE;
}

int gcz_build_device_bases(gcz_ctx* c, const void* d_bases, uint64_t nbases, int L) {
  if (!c || (!d_bases && nbases)) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  if (reinterpret_cast<uintptr_t>(d_bases) & 3) {   // the leaf kernel stages with 4-B loads
    if (int rc = c->ensure(c->input, nbases + 16)) return rc;
    if (hipMemcpyAsync(c->input.ptr, d_bases, nbases, hipMemcpyDeviceToDevice, c->stream) != hipSuccess)
      return c->fail(GCZ_ERR_DEVICE, "gcz_build_device_bases", "realign copy failed");
    d_bases = c->input.ptr;
  }
  return c->build(d_bases, nullptr, nbases, 0, L);
}

int gcz_build_device_leaves(gcz_ctx* c, const uint64_t* d_leaves, uint64_t S, int L) {
  if (!c || (!d_leaves && S)) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  return c->build(nullptr, reinterpret_cast<const u64*>(d_leaves), 0, S, L);
}

int gcz_build_host_leaves(gcz_ctx* c, const uint64_t* leaves, uint64_t S, int L) {
  if (!c || (!leaves && S)) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  if (int rc = c->ensure(c->input, S * 8 + 16)) return rc;
  if (S && c->upload(c->input.ptr, leaves, S * 8)) return c->fail(GCZ_ERR_DEVICE, "gcz_build_host_leaves", "H2D copy failed");
  return c->build(nullptr, static_cast<const u64*>(c->input.ptr), 0, S, L);
}

int gcz_build_host_fasta(gcz_ctx* c, const void* fasta, uint64_t nbytes, int L) {
  if (!c || (!fasta && nbytes)) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  // the raw file goes to the device; headers / line breaks are removed there (gcz_ingest.hip:
  // a file of one unbroken line is built in place, without a host scan for line breaks)
  if (int rc = c->ensure(c->input, nbytes + 16)) return rc;
  if (nbytes && c->upload(c->input.ptr, fasta, nbytes))
    return c->fail(GCZ_ERR_DEVICE, "gcz_build_host_fasta", "H2D copy failed");
  return gcz_build_device_fasta(c, c->input.ptr, nbytes, L);
}

int gcz_info_get(gcz_ctx* c, gcz_info* out) {
  if (!c || !out) return GCZ_ERR_ARG;
  *out = c->info;
  return GCZ_OK;
}

int gcz_copy_leaves(gcz_ctx* c, uint64_t* host_out) {
  if (!c || !host_out || c->info.status != GCZ_OK) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  if (c->info.n_leaves &&
      hipMemcpyAsync(host_out, c->leaves_out.ptr, c->info.n_leaves * 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
    return GCZ_ERR_DEVICE;
  return hipStreamSynchronize(c->stream) == hipSuccess ? GCZ_OK : GCZ_ERR_DEVICE;
}

int gcz_copy_layer(gcz_ctx* c, int k, uint32_t* host_out) {
  if (!c || !host_out || c->info.status != GCZ_OK || k < 0 || k >= c->info.n_layers) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  const u64 n = c->info.layer_size[k];
  if (n && hipMemcpyAsync(host_out, static_cast<uint2*>(c->nodes_out.ptr) + c->layer_off[k], n * 8,
                          hipMemcpyDeviceToHost, c->stream) != hipSuccess)
    return GCZ_ERR_DEVICE;
  return hipStreamSynchronize(c->stream) == hipSuccess ? GCZ_OK : GCZ_ERR_DEVICE;
}

const uint64_t* gcz_device_leaves(gcz_ctx* c) {
  return c && c->info.status == GCZ_OK ? static_cast<const uint64_t*>(c->leaves_out.ptr) : nullptr;
}
const uint32_t* gcz_device_layer(gcz_ctx* c, int k) {
  if (!c || c->info.status != GCZ_OK || k < 0 || k >= c->info.n_layers) return nullptr;
  return reinterpret_cast<const uint32_t*>(static_cast<uint2*>(c->nodes_out.ptr) + c->layer_off[k]);
}

// The whole DAG of the last build into caller-owned host memory (fresh, unpinned pages):
// DMA into a pinned staging ring (kRingSlots slots of kRingChunk bytes, allocated once per
// context) while host threads copy the previous slot out, each a slice -- the page faults of
// the destination are taken by several threads at once and the DMA never waits for them.
// The runtime's pageable D2H path copies and faults on one thread (~10 GB/s at 1 Gbase).
namespace {
constexpr u64 kRingChunk = u64(16) << 20;
constexpr int kRingSlots = 4;

// A small DAG (one ring slot) is gathered into the pinned ring by a kernel of this library's
// own instead of one runtime D2H copy per layer: the runtime's first device-to-host copy in a
// process pays a one-time start-up of its copy path (~17 ms measured on merged's 1.2 MB tree,
// profiles/r03 and r04 compress_e2e), a kernel launch from an already loaded module does not.
// Stores go to host memory directly (vector stores; the ring is pinned and device-visible).
constexpr int kGatherMax = 64;
struct HostGather {
  const u64* src[kGatherMax];
  u64 off[kGatherMax];   // destination word offset in the ring
  u64 len[kGatherMax];   // words (pieces are whole u64 / uint2 arrays)
  u32 n;
};
static __global__ __launch_bounds__(256) void k_gather_host(HostGather g, u64* __restrict__ ring) {
  const u32 i = blockIdx.y;
  if (i >= g.n) return;
  const u64* __restrict__ s = g.src[i];
  u64* d = ring + g.off[i];
  for (u64 k = u64(blockIdx.x) * 256 + threadIdx.x; k < g.len[i]; k += u64(gridDim.x) * 256) d[k] = s[k];
}

struct CopyPool {   // T - 1 workers + the calling thread copy one chunk's slices, then meet
  int T;
  std::vector<std::thread> th;
  std::mutex m;
  std::condition_variable cv, done_cv;
  const unsigned char* src = nullptr;
  unsigned char* dst = nullptr;
  u64 len = 0;
  u64 gen = 0;
  int pending = 0;
  bool stop = false;
  explicit CopyPool(int t) : T(t) {
    for (int i = 1; i < T; ++i) th.emplace_back([this, i] { work(i); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(m);
      stop = true;
    }
    cv.notify_all();
    for (auto& x : th) x.join();
  }
  void slice(int i) {
    const u64 a = len * u64(i) / u64(T), b = len * u64(i + 1) / u64(T);
    if (b > a) std::memcpy(dst + a, src + a, b - a);
  }
  void work(int i) {
    u64 seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> lk(m);
      cv.wait(lk, [&] { return stop || gen != seen; });
      if (stop) return;
      seen = gen;
      lk.unlock();
      slice(i);
      lk.lock();
      if (--pending == 0) done_cv.notify_one();
    }
  }
  void copy(const unsigned char* s, unsigned char* d, u64 n) {
    if (T == 1 || n < (u64(1) << 20)) {
      std::memcpy(d, s, n);
      return;
    }
    {
      std::lock_guard<std::mutex> g(m);
      src = s; dst = d; len = n;
      pending = T - 1;
      ++gen;
    }
    cv.notify_all();
    slice(0);
    std::unique_lock<std::mutex> lk(m);
    done_cv.wait(lk, [&] { return pending == 0; });
  }
};
}  // namespace

// The staging ring for a fetch of `total` bytes: one slot holding a small DAG, else kRingSlots
// slots of kRingChunk; pinned once per context (~16 ms for 64 MB on the box: the drop-in
// reserves it while the context comes up; two slots or 8 MB ones were measured slower).
int gcz_fetch_reserve(gcz_ctx* c, uint64_t total) {
  if (!c) return GCZ_ERR_ARG;
  const u64 need = total > kRingChunk ? u64(kRingSlots) * kRingChunk : (total + 4095) & ~u64(4095);
  if (c->h_ring_bytes < need) {
    const auto t0 = std::chrono::steady_clock::now();
    if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
    if (c->h_ring) (void)hipHostFree(c->h_ring);
    c->h_ring = nullptr;
    c->h_ring_bytes = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&c->h_ring), need, hipHostMallocDefault) != hipSuccess)
      return GCZ_ERR_DEVICE;
    c->h_ring_bytes = need;
    if (std::getenv("GCZ_TIMING"))
      std::fprintf(stderr, "gcz-time ring-alloc %g\n",
                   std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
  }
  for (hipEvent_t& e : c->ring_ev)
    if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return GCZ_ERR_DEVICE;
  return GCZ_OK;
}

int gcz_fetch_host(gcz_ctx* c, uint64_t* leaves_out, uint32_t* const* layers_out) {
  if (!c || c->info.status != GCZ_OK) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  struct Piece { const unsigned char* src; unsigned char* dst; u64 len; };
  std::vector<Piece> pieces;   // <= kRingChunk each
  u64 total = 0;
  auto add = [&](const void* src, void* dst, u64 len) {
    if (len && !dst) return false;
    for (u64 o = 0; o < len; o += kRingChunk)
      pieces.push_back({static_cast<const unsigned char*>(src) + o, static_cast<unsigned char*>(dst) + o,
                        std::min<u64>(kRingChunk, len - o)});
    total += len;
    return true;
  };
  if (!add(c->leaves_out.ptr, leaves_out, c->info.n_leaves * 8)) return GCZ_ERR_ARG;
  for (int k = 0; k < c->info.n_layers; ++k)
    if (!add(static_cast<uint2*>(c->nodes_out.ptr) + c->layer_off[k], layers_out ? layers_out[k] : nullptr,
             c->info.layer_size[k] * 8))
      return GCZ_ERR_ARG;
  if (pieces.empty()) return GCZ_OK;
  if (int rc = gcz_fetch_reserve(c, total)) return rc;
  const unsigned hc = std::thread::hardware_concurrency();
  CopyPool pool(total >= (u64(8) << 20) ? int(std::min<unsigned>(8, std::max(1u, hc))) : 1);
  if (total <= kRingChunk) {   // one D2H batch, then the host copies
    u64 at = 0;
    if (pieces.size() <= size_t(kGatherMax)) {   // one gather kernel into the ring (see k_gather_host)
      HostGather g{};
      u64 mx = 0;
      for (const Piece& p : pieces) {
        g.src[g.n] = reinterpret_cast<const u64*>(p.src);
        g.off[g.n] = at / 8;
        g.len[g.n] = p.len / 8;
        mx = std::max(mx, p.len / 8);
        ++g.n;
        at += p.len;
      }
      const dim3 grid(unsigned(std::min<u64>(64, (mx + 255) / 256)), g.n);
      hipLaunchKernelGGL(k_gather_host, grid, dim3(256), 0, c->stream, g, reinterpret_cast<u64*>(c->h_ring));
      if (hipGetLastError() != hipSuccess) return GCZ_ERR_DEVICE;
    } else {
      for (const Piece& p : pieces) {
        if (hipMemcpyAsync(c->h_ring + at, p.src, p.len, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
          return GCZ_ERR_DEVICE;
        at += p.len;
      }
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess) return GCZ_ERR_DEVICE;
    at = 0;
    for (const Piece& p : pieces) {
      pool.copy(c->h_ring + at, p.dst, p.len);
      at += p.len;
    }
    return GCZ_OK;
  }
  const size_t slots = kRingSlots;
  auto stage_of = [&](size_t i) { return c->h_ring + (i % slots) * kRingChunk; };
  auto issue = [&](size_t i) {
    return hipMemcpyAsync(stage_of(i), pieces[i].src, pieces[i].len, hipMemcpyDeviceToHost, c->stream) ==
               hipSuccess &&
           hipEventRecord(c->ring_ev[i % slots], c->stream) == hipSuccess;
  };
  for (size_t i = 0; i < pieces.size() && i < slots; ++i)
    if (!issue(i)) return GCZ_ERR_DEVICE;
  for (size_t i = 0; i < pieces.size(); ++i) {
    if (hipEventSynchronize(c->ring_ev[i % slots]) != hipSuccess) return GCZ_ERR_DEVICE;
    pool.copy(stage_of(i), pieces[i].dst, pieces[i].len);
    if (i + slots < pieces.size() && !issue(i + slots)) return GCZ_ERR_DEVICE;
  }
  return GCZ_OK;
}

int gcz_tree_fetch(gcz_ctx* c, gcz_tree* t) {
  if (!c || !t || c->info.status != GCZ_OK) return GCZ_ERR_ARG;
  t->L = c->info.L;
  t->root = c->info.root;
  t->leaves.resize(c->info.n_leaves);
  t->layers.assign(c->info.n_layers, {});
  std::vector<uint32_t*> outs(c->info.n_layers);
  for (int k = 0; k < c->info.n_layers; ++k) {
    t->layers[k].resize(2 * c->info.layer_size[k]);
    outs[k] = t->layers[k].data();
  }
  return gcz_fetch_host(c, t->leaves.data(), outs.data());
}

int gcz_profile_enable(gcz_ctx* c, int on) {
  if (!c) return GCZ_ERR_ARG;
  c->profile = on != 0;
  return GCZ_OK;
}
int gcz_profile_entry(gcz_ctx* c, int k, const char** name, uint64_t* launches, double* total_ms) {
  if (!c || k < 0 || k >= KID_COUNT) return -1;
  if (name) *name = kernel_name(k);
  if (launches) *launches = c->prof_launches[k];
  if (total_ms) *total_ms = c->prof_ms[k];
  return 0;
}
void gcz_profile_reset(gcz_ctx* c) {
  if (!c) return;
  for (int k = 0; k < KID_COUNT; ++k) { c->prof_launches[k] = 0; c->prof_ms[k] = 0; }
  c->prof_trace.clear();
}
uint64_t gcz_profile_trace(gcz_ctx* c, float* out, uint64_t cap) {
  if (!c) return 0;
  const uint64_t n = c->prof_trace.size() / 3;
  for (uint64_t i = 0; out && i < std::min(n, cap) * 3; ++i) out[i] = c->prof_trace[i];
  return n;
}

}  // extern "C"
