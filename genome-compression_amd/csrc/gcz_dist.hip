// Multi-rank shared_tree construction: one rank per GPU (RCCL over xGMI), or R
// virtual ranks sharing one device (testing).  Algorithm: gcz_dist_device.h.
//
// Partition: rank r owns strands [r*B, (r+1)*B) clipped to S,
// where B = ceil(S/R) rounded up to a multiple of 2^G.  Node level k < G pairs
// elements (2j, 2j+1) that then lie on one rank, so levels 0..G-1 run
// distributed; the n_G < ~R*1024 words left are gathered to rank 0, which
// finishes the top layers alone.  Rank r's uniques of every distributed level
// are the contiguous id range [off_r, off_r + c_r) of that layer, so the
// layers are the rank-ordered concatenation of the slices — byte-identical to
// the single-device (and the reference's) build.
#include <dlfcn.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <rccl/rccl.h>   // types only: the functions are resolved with dlsym

#include "gcz_ctx.h"
#include "gcz_dist_device.h"
#include "gcz_dist_fast.h"
#include "gcz_scan.h"

using namespace gcz_dev;
using namespace gcz_host;

struct gcz_dist_state {
  DevBuf scratch, gnf, gmul, gid, blockcnt, bchunk, skey, sidx, sflag, scval, sdval, clist;   // sender side
  DevBuf dict;                                                                // rank 0's leaf dictionary
  DevBuf rkey, oslot, rflag, rcval, rdval, owntab, oids, omin, olist;         // owner side
  DevBuf ob_cnt, ob_off, ob_desc, ob_rec;                                      // owner bucketed dedupe
  DevBuf ob_seg, ob_rt, ob_rec2, ob_fo;                                        // ... as the two-pass partition
  DevBuf dhdr, gath, gath2, gathf, ddesc, tail_in, nfl;
  u64* h_gath = nullptr;    // pinned mirrors of the gathered vectors
  u64* h_gath2 = nullptr;
  u64* h_gathf = nullptr;
  DlRelay* h_relay = nullptr;   // pinned staging of the dense leaf relay table (H2D, stream-ordered)
  DevBuf skey_hi, rkey_hi;   // fused schedule: the 6-byte records' high 16 bits
  DevBuf fl_desc;            // fused schedule: k_fl_scatter's look-back descriptors + ticket
  DevBuf fl_cntb, fl_mid, fl_g3, fl_g4;   // fused schedule: r-first counts per bucket, the mid-build
  u64* h_mid = nullptr;                   // vector (+ pinned mirror), R3's / R4's gathered vectors
};

void gcz_dist_state_free(gcz_ctx* c) {
  if (c->split) {
    gcz_group_destroy(c->split);
    c->split = nullptr;
  }
  gcz_dist_state* d = c->dist;
  if (!d) return;
  for (DevBuf* b : {&d->dict, &d->scratch, &d->gnf, &d->gmul, &d->gid, &d->blockcnt, &d->bchunk, &d->skey, &d->sidx, &d->sflag,
                    &d->scval, &d->sdval, &d->clist, &d->olist, &d->rkey, &d->oslot, &d->rflag, &d->rcval, &d->rdval, &d->owntab, &d->oids,
                    &d->omin, &d->ob_cnt, &d->ob_off, &d->ob_desc, &d->ob_rec, &d->ob_seg, &d->ob_rt,
                    &d->ob_rec2, &d->ob_fo, &d->fl_cntb, &d->fl_mid, &d->fl_g3, &d->fl_g4, &d->skey_hi,
                    &d->rkey_hi, &d->fl_desc,
                    &d->dhdr, &d->gath, &d->gath2, &d->gathf, &d->ddesc, &d->tail_in, &d->nfl})
    if (b->ptr) (void)hipFree(b->ptr);
  for (u64* h : {d->h_gath, d->h_gath2, d->h_gathf})
    if (h) (void)hipHostFree(h);
  if (d->h_relay) (void)hipHostFree(d->h_relay);
  if (d->h_mid) (void)hipHostFree(d->h_mid);
  delete d;
  c->dist = nullptr;
}

namespace {

// Limit on one exchange (GCZ_DIST_TIMEOUT_S, default 180 s): the shm transport's barrier, the
// RCCL watchdog (gcz_group::Watch).
long dist_timeout_s() {
  const char* e = std::getenv("GCZ_DIST_TIMEOUT_S");
  const long v = e ? std::atol(e) : 180;
  return v > 0 ? v : 180;
}

// ---- transports ------------------------------------------------------------------

struct Transport {
  int world = 1;
  std::string err;
  virtual ~Transport() = default;
  // counts: M[s * world + d] elements from rank s to rank d (reverse: from d to s).
  // send[i]: local rank i's buffer, segments in destination order; recv[i]: segments in source order.
  virtual int alltoallv(const std::vector<u64>& M, bool reverse, size_t elem, const std::vector<const void*>& send,
                        const std::vector<void*>& recv) = 0;
  // Same counts, explicit element displacements: sd[s * world + d] in rank s's send buffer,
  // rd[d * world + s] in rank d's receive buffer.
  virtual int alltoallv_at(const std::vector<u64>& M, bool reverse, size_t elem, const std::vector<u64>& sd,
                           const std::vector<u64>& rd, const std::vector<const void*>& send,
                           const std::vector<void*>& recv) = 0;
  virtual int allgather(size_t bytes, const std::vector<const void*>& send, const std::vector<void*>& recv) = 0;
  // Several exchanges as ONE group (RCCL: one ncclGroupStart/End, a single launch whose
  // transfers proceed together; the other transports run them one after the other).  Each op
  // is an alltoallv_at; an allgather is the op whose every count is its size, every send
  // displacement 0 and receive displacement s * size (XOp::allgather).
  struct XOp {
    std::vector<u64> M, sd, rd;
    bool rev = false;
    size_t elem = 1;
    std::vector<const void*> send;
    std::vector<void*> recv;
  };
  virtual int group(const std::vector<XOp>& ops) {
    for (const XOp& o : ops)
      if (int rc = alltoallv_at(o.M, o.rev, o.elem, o.sd, o.rd, o.send, o.recv)) return rc;
    return 0;
  }
  // A bulk group on the transport's second stream (and communicator), beside the build's own:
  // bulk_stream() null = the build's stream (the testing transports run bulk groups in line).
  virtual hipStream_t bulk_stream() { return nullptr; }
  virtual int group_bulk(const std::vector<XOp>& ops) { return group(ops); }
  // rank 0's `bytes` at send[i of rank 0] to recv[i] of every other rank
  virtual int bcast0(size_t bytes, const std::vector<const void*>& send, const std::vector<void*>& recv) = 0;
  // rank 0 receives cnt[r] elements from every rank r, concatenated in rank order
  virtual int gather0(const std::vector<u64>& cnt, size_t elem, const std::vector<const void*>& send,
                      void* recv0) = 0;
};

u64 mcount(const std::vector<u64>& M, int R, bool reverse, int s, int d) {
  return reverse ? M[size_t(d) * R + s] : M[size_t(s) * R + d];
}
u64 send_displ(const std::vector<u64>& M, int R, bool rev, int s, int d) {
  u64 o = 0;
  for (int q = 0; q < d; ++q) o += mcount(M, R, rev, s, q);
  return o;
}
u64 recv_displ(const std::vector<u64>& M, int R, bool rev, int d, int s) {
  u64 o = 0;
  for (int q = 0; q < s; ++q) o += mcount(M, R, rev, q, d);
  return o;
}

// One peer's share of rank `me`'s all-to-all, in bytes: what the point-to-point transport
// (RcclTransport) sends to and receives from `peer` (peer == me: the local copy).  The counts
// M[s * R + d] (reverse: transposed) place the segments back to back in peer order, or at
// the explicit element displacements sd[s * R + d] (sender s) / rd[d * R + s] (receiver d).
// Host tests drive this arithmetic through gcz_dist_p2p_plan against the transport contract.
struct P2POp {
  int peer;
  u64 send_off, send_bytes, recv_off, recv_bytes;
};
std::vector<P2POp> p2p_plan(const std::vector<u64>& M, int R, int me, bool rev, size_t elem, const u64* sd,
                            const u64* rd) {
  std::vector<P2POp> ops;
  ops.resize(size_t(R));
  for (int q = 0; q < R; ++q) {
    P2POp& o = ops[size_t(q)];
    o.peer = q;
    o.send_bytes = mcount(M, R, rev, me, q) * elem;
    o.recv_bytes = mcount(M, R, rev, q, me) * elem;
    o.send_off = (sd ? sd[size_t(me) * R + q] : send_displ(M, R, rev, me, q)) * elem;
    o.recv_off = (rd ? rd[size_t(me) * R + q] : recv_displ(M, R, rev, me, q)) * elem;
  }
  return ops;
}
// gather to rank 0 = the all-to-all whose only nonzero column is rank 0's
std::vector<u64> gather_matrix(const std::vector<u64>& cnt, int R) {
  std::vector<u64> M(size_t(R) * R, 0);
  for (int s = 0; s < R; ++s) M[size_t(s) * R] = cnt[size_t(s)];
  return M;
}

// All ranks in this process on one stream: exchanges are device copies.  GCZ_LOCAL_BULK=1 gives
// it a second stream for bulk groups (RcclTransport's second stream and communicator): their
// copies then run there, ordered only by the schedule's bulk events (gcz_group::x_group_bulk /
// bulk_done), as K2 runs beside the build on RCCL.
struct LocalTransport : Transport {
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;   // (GCZ_LOCAL_BULK=1)
  hipStream_t cur = nullptr;       // the copies' stream: `stream`, or stream2 inside group_bulk
  ~LocalTransport() override {
    if (stream2) (void)hipStreamDestroy(stream2);
  }
  hipStream_t bulk_stream() override { return stream2; }
  int group_bulk(const std::vector<XOp>& ops) override {
    cur = stream2;
    const int rc = group(ops);
    cur = nullptr;
    return rc;
  }
  int copy(void* dst, const void* src, size_t bytes) {
    if (!bytes) return GCZ_OK;
    if (hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, cur ? cur : stream) != hipSuccess) {
      err = "local transport copy failed";
      return GCZ_ERR_DEVICE;
    }
    return GCZ_OK;
  }
  int alltoallv(const std::vector<u64>& M, bool rev, size_t elem, const std::vector<const void*>& send,
                const std::vector<void*>& recv) override {
    for (int s = 0; s < world; ++s)
      for (int d = 0; d < world; ++d)
        if (int rc = copy(static_cast<char*>(recv[d]) + recv_displ(M, world, rev, d, s) * elem,
                          static_cast<const char*>(send[s]) + send_displ(M, world, rev, s, d) * elem,
                          mcount(M, world, rev, s, d) * elem))
          return rc;
    return GCZ_OK;
  }
  int alltoallv_at(const std::vector<u64>& M, bool rev, size_t elem, const std::vector<u64>& sd,
                   const std::vector<u64>& rd, const std::vector<const void*>& send,
                   const std::vector<void*>& recv) override {
    for (int s = 0; s < world; ++s)
      for (int d = 0; d < world; ++d)
        if (int rc = copy(static_cast<char*>(recv[d]) + rd[size_t(d) * world + s] * elem,
                          static_cast<const char*>(send[s]) + sd[size_t(s) * world + d] * elem,
                          mcount(M, world, rev, s, d) * elem))
          return rc;
    return GCZ_OK;
  }
  int allgather(size_t bytes, const std::vector<const void*>& send, const std::vector<void*>& recv) override {
    for (int s = 0; s < world; ++s)
      for (int d = 0; d < world; ++d)
        if (int rc = copy(static_cast<char*>(recv[d]) + size_t(s) * bytes, send[s], bytes)) return rc;
    return GCZ_OK;
  }
  int bcast0(size_t bytes, const std::vector<const void*>& send, const std::vector<void*>& recv) override {
    for (int d = 1; d < world; ++d)
      if (int rc = copy(recv[d], send[0], bytes)) return rc;
    return GCZ_OK;
  }
  int gather0(const std::vector<u64>& cnt, size_t elem, const std::vector<const void*>& send,
              void* recv0) override {
    u64 o = 0;
    for (int s = 0; s < world; ++s) {
      if (int rc = copy(static_cast<char*>(recv0) + o * elem, send[s], cnt[s] * elem)) return rc;
      o += cnt[s];
    }
    return GCZ_OK;
  }
};

struct RcclApi {
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*CommSplit)(ncclComm_t, int, int, ncclComm_t*, ncclConfig_t*) = nullptr;   // (optional)
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  bool ok = false;
};

// RCCL is loaded on first use; a process that already holds torch's RCCL
// (same SONAME) shares it.  RTLD_LOCAL: a copy torch loads LATER (its own
// librccl.so) must not bind its globals to ours -- with RTLD_GLOBAL both
// copies' static destructors ran on one set of objects at exit (double free).
RcclApi& rccl() {
  static RcclApi api = [] {
    RcclApi a;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return a;
#define GCZ_SYM(field, name) a.field = reinterpret_cast<decltype(a.field)>(dlsym(h, name))
    GCZ_SYM(GetUniqueId, "ncclGetUniqueId");
    GCZ_SYM(CommInitRank, "ncclCommInitRank");
    GCZ_SYM(CommDestroy, "ncclCommDestroy");
    GCZ_SYM(CommAbort, "ncclCommAbort");
    GCZ_SYM(GroupStart, "ncclGroupStart");
    GCZ_SYM(GroupEnd, "ncclGroupEnd");
    GCZ_SYM(Send, "ncclSend");
    GCZ_SYM(Recv, "ncclRecv");
    GCZ_SYM(AllGather, "ncclAllGather");
    GCZ_SYM(Broadcast, "ncclBroadcast");
    GCZ_SYM(GetErrorString, "ncclGetErrorString");
    GCZ_SYM(CommSplit, "ncclCommSplit");
#undef GCZ_SYM
    a.ok = a.GetUniqueId && a.CommInitRank && a.CommDestroy && a.CommAbort && a.GroupStart && a.GroupEnd && a.Send && a.Recv &&
           a.AllGather && a.Broadcast && a.GetErrorString;
    return a;
  }();
  return api;
}

// One rank of this process on its own GPU; peers are other processes.  Every exchange is
// one group of ncclSend / ncclRecv (or an ncclAllGather / ncclBroadcast) on the build stream,
// its transfers planned by p2p_plan.  A collective that does not complete is bounded by the
// group's watchdog (gcz_group::Watch), which aborts the communicator.
struct RcclTransport : Transport {
  int me = 0;
  std::atomic<ncclComm_t> comm{nullptr};
  hipStream_t stream = nullptr;
  // bulk groups: a second communicator (ncclCommSplit of the first: its own channels) on its own
  // stream, so a large all-to-all runs beside the build's kernels and small collectives
  std::atomic<ncclComm_t> comm2{nullptr};
  hipStream_t stream2 = nullptr;
  ~RcclTransport() override {
    if (ncclComm_t c = comm2.exchange(nullptr)) (void)rccl().CommDestroy(c);
    if (ncclComm_t c = comm.exchange(nullptr)) (void)rccl().CommDestroy(c);
    if (stream2) (void)hipStreamDestroy(stream2);
  }
  void abort() {   // (from the watchdog thread: unblocks the streams and any blocked call)
    if (ncclComm_t c = comm2.exchange(nullptr)) (void)rccl().CommAbort(c);
    if (ncclComm_t c = comm.exchange(nullptr)) (void)rccl().CommAbort(c);
  }
  hipStream_t bulk_stream() override { return comm2.load() ? stream2 : nullptr; }
  int group_bulk(const std::vector<XOp>& ops) override {
    ncclComm_t c2 = comm2.load();
    if (!c2) return group(ops);
    return run_group(ops, c2, stream2);
  }
  int check(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return GCZ_OK;
    err = std::string(what) + ": " + rccl().GetErrorString(r);
    return GCZ_ERR_DEVICE;
  }
  int self_copy(void* dst, const void* src, size_t bytes, hipStream_t st = nullptr) {
    if (bytes && hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st ? st : stream) != hipSuccess) {
      err = "rccl transport self copy failed";
      return GCZ_ERR_DEVICE;
    }
    return GCZ_OK;
  }
  int run(const std::vector<P2POp>& ops, const void* send, void* recv) {
    const auto* sb = static_cast<const char*>(send);
    auto* rb = static_cast<char*>(recv);
    ncclComm_t c = comm.load();
    if (!c) {
      err = "communicator aborted";
      return GCZ_ERR_DEVICE;
    }
    const P2POp& self = ops[size_t(me)];
    if (int rc = self_copy(rb + self.recv_off, sb + self.send_off, self.send_bytes)) return rc;
    RcclApi& a = rccl();
    if (int rc = check(a.GroupStart(), "ncclGroupStart")) return rc;
    for (const P2POp& o : ops) {
      if (o.peer == me) continue;
      if (o.send_bytes) {
        const ncclResult_t r = a.Send(sb + o.send_off, o.send_bytes, ncclUint8, o.peer, c, stream);
        if (r != ncclSuccess) { (void)a.GroupEnd(); return check(r, "ncclSend"); }
      }
      if (o.recv_bytes) {
        const ncclResult_t r = a.Recv(rb + o.recv_off, o.recv_bytes, ncclUint8, o.peer, c, stream);
        if (r != ncclSuccess) { (void)a.GroupEnd(); return check(r, "ncclRecv"); }
      }
    }
    return check(a.GroupEnd(), "ncclGroupEnd");
  }
  int alltoallv(const std::vector<u64>& M, bool rev, size_t elem, const std::vector<const void*>& send,
                const std::vector<void*>& recv) override {
    return run(p2p_plan(M, world, me, rev, elem, nullptr, nullptr), send[0], recv[0]);
  }
  // every op's self copy first, then all their sends / receives in one group (NCCL matches a
  // pair's several sends and receives in issue order)
  int group(const std::vector<XOp>& ops) override { return run_group(ops, comm.load(), stream); }
  int run_group(const std::vector<XOp>& ops, ncclComm_t c, hipStream_t st) {
    if (!c) {
      err = "communicator aborted";
      return GCZ_ERR_DEVICE;
    }
    std::vector<std::vector<P2POp>> plans;
    for (const XOp& o : ops) {
      plans.push_back(p2p_plan(o.M, world, me, o.rev, o.elem, o.sd.data(), o.rd.data()));
      const P2POp& self = plans.back()[size_t(me)];
      if (int rc = self_copy(static_cast<char*>(o.recv[0]) + self.recv_off,
                             static_cast<const char*>(o.send[0]) + self.send_off, self.send_bytes, st))
        return rc;
    }
    RcclApi& a = rccl();
    if (int rc = check(a.GroupStart(), "ncclGroupStart")) return rc;
    for (size_t k = 0; k < ops.size(); ++k) {
      const auto* sb = static_cast<const char*>(ops[k].send[0]);
      auto* rb = static_cast<char*>(ops[k].recv[0]);
      for (const P2POp& o : plans[k]) {
        if (o.peer == me) continue;
        if (o.send_bytes) {
          const ncclResult_t r = a.Send(sb + o.send_off, o.send_bytes, ncclUint8, o.peer, c, st);
          if (r != ncclSuccess) { (void)a.GroupEnd(); return check(r, "ncclSend"); }
        }
        if (o.recv_bytes) {
          const ncclResult_t r = a.Recv(rb + o.recv_off, o.recv_bytes, ncclUint8, o.peer, c, st);
          if (r != ncclSuccess) { (void)a.GroupEnd(); return check(r, "ncclRecv"); }
        }
      }
    }
    return check(a.GroupEnd(), "ncclGroupEnd");
  }
  int alltoallv_at(const std::vector<u64>& M, bool rev, size_t elem, const std::vector<u64>& sd,
                   const std::vector<u64>& rd, const std::vector<const void*>& send,
                   const std::vector<void*>& recv) override {
    return run(p2p_plan(M, world, me, rev, elem, sd.data(), rd.data()), send[0], recv[0]);
  }
  int allgather(size_t bytes, const std::vector<const void*>& send, const std::vector<void*>& recv) override {
    ncclComm_t c = comm.load();
    if (!c) { err = "communicator aborted"; return GCZ_ERR_DEVICE; }
    return check(rccl().AllGather(send[0], recv[0], bytes, ncclUint8, c, stream), "ncclAllGather");
  }
  int bcast0(size_t bytes, const std::vector<const void*>& send, const std::vector<void*>& recv) override {
    if (!bytes) return GCZ_OK;
    ncclComm_t c = comm.load();
    if (!c) { err = "communicator aborted"; return GCZ_ERR_DEVICE; }
    void* buf = me == 0 ? const_cast<void*>(send[0]) : recv[0];   // in place on the root
    return check(rccl().Broadcast(buf, buf, bytes, ncclUint8, 0, c, stream), "ncclBroadcast");
  }
  int gather0(const std::vector<u64>& cnt, size_t elem, const std::vector<const void*>& send,
              void* recv0) override {
    return run(p2p_plan(gather_matrix(cnt, world), world, me, false, elem, nullptr, nullptr), send[0],
               me == 0 ? recv0 : nullptr);
  }
};

// One rank per process, host-staged through a POSIX shared-memory file: the multi-process
// path (each process its own context, decisions from the gathered vectors, matching
// collective sequences) on ONE GPU, where RCCL refuses two ranks per device.  Testing
// only: every exchange is a D2H copy, a barrier, H2D copies, a barrier.
struct ShmTransport : Transport {
  struct Ctl {
    std::atomic<u32> arrived;
    std::atomic<u32> sense;
    std::atomic<u32> failed;
  };
  int me = 0;
  hipStream_t stream = nullptr;
  long timeout_s = 120;       // barrier limit (GCZ_DIST_TIMEOUT_S)
  size_t cap = 0;             // bytes per rank region
  size_t map_bytes = 0;
  char* base = nullptr;
  u32 local_sense = 0;
  ~ShmTransport() override {
    if (base) munmap(base, map_bytes);
  }
  Ctl* ctl() { return reinterpret_cast<Ctl*>(base); }
  char* region(int r) { return base + 4096 + size_t(r) * cap; }
  int barrier() {
    local_sense ^= 1u;
    Ctl* c = ctl();
    if (c->failed.load()) { err = "shm transport: a peer failed"; return GCZ_ERR_DEVICE; }
    if (c->arrived.fetch_add(1) + 1 == u32(world)) {
      c->arrived.store(0);
      c->sense.store(local_sense);
    } else {
      const auto t0 = std::chrono::steady_clock::now();
      while (c->sense.load() != local_sense) {
        if (c->failed.load()) { err = "shm transport: a peer failed"; return GCZ_ERR_DEVICE; }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(timeout_s)) {
          err = "shm transport: no peer arrived within " + std::to_string(timeout_s) + " s";
          c->failed.store(1);
          return GCZ_ERR_DEVICE;
        }
        std::this_thread::yield();
      }
    }
    return GCZ_OK;
  }
  int to_host(char* dst, const void* src, size_t bytes) {
    if (!bytes) return GCZ_OK;
    if (bytes > cap || hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, stream) != hipSuccess) {
      err = bytes > cap ? "shm transport: region too small" : "shm transport: D2H copy failed";
      ctl()->failed.store(1);
      return GCZ_ERR_DEVICE;
    }
    return GCZ_OK;
  }
  // every failure inside a collective raises `failed`, so the peers leave their barrier
  // at once instead of at the timeout (a group is single-use after a failure)
  int to_dev(void* dst, const char* src, size_t bytes) {
    if (bytes && hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream) != hipSuccess) {
      err = "shm transport: H2D copy failed";
      ctl()->failed.store(1);
      return GCZ_ERR_DEVICE;
    }
    return GCZ_OK;
  }
  int drain() {
    if (hipStreamSynchronize(stream) != hipSuccess) {
      err = "shm transport: stream";
      ctl()->failed.store(1);
      return GCZ_ERR_DEVICE;
    }
    return GCZ_OK;
  }
  int alltoallv_at(const std::vector<u64>& M, bool rev, size_t elem, const std::vector<u64>& sd,
                   const std::vector<u64>& rd, const std::vector<const void*>& send,
                   const std::vector<void*>& recv) override {
    const size_t R = size_t(world);
    if (int rc = drain()) return rc;
    for (int d = 0; d < world; ++d) {   // my segments, at their send displacements
      const size_t o = sd[me * R + d] * elem, n = mcount(M, world, rev, me, d) * elem;
      if (o + n > cap) { err = "shm transport: region too small"; ctl()->failed.store(1); return GCZ_ERR_DEVICE; }
      if (int rc = to_host(region(me) + o, static_cast<const char*>(send[0]) + o, n)) return rc;
    }
    if (int rc = drain()) return rc;
    if (int rc = barrier()) return rc;
    for (int s = 0; s < world; ++s)
      if (int rc = to_dev(static_cast<char*>(recv[0]) + rd[me * R + s] * elem,
                          region(s) + sd[s * R + me] * elem, mcount(M, world, rev, s, me) * elem))
        return rc;
    if (int rc = drain()) return rc;
    return barrier();
  }
  int alltoallv(const std::vector<u64>& M, bool rev, size_t elem, const std::vector<const void*>& send,
                const std::vector<void*>& recv) override {
    const size_t R = size_t(world);
    std::vector<u64> sd(R * R), rd(R * R);
    for (int s = 0; s < world; ++s)
      for (int d = 0; d < world; ++d) {
        sd[s * R + d] = send_displ(M, world, rev, s, d);
        rd[d * R + s] = recv_displ(M, world, rev, d, s);
      }
    return alltoallv_at(M, rev, elem, sd, rd, send, recv);
  }
  int allgather(size_t bytes, const std::vector<const void*>& send, const std::vector<void*>& recv) override {
    if (int rc = drain()) return rc;
    if (int rc = to_host(region(me), send[0], bytes)) return rc;
    if (int rc = drain()) return rc;
    if (int rc = barrier()) return rc;
    for (int s = 0; s < world; ++s)
      if (int rc = to_dev(static_cast<char*>(recv[0]) + size_t(s) * bytes, region(s), bytes)) return rc;
    if (int rc = drain()) return rc;
    return barrier();
  }
  int bcast0(size_t bytes, const std::vector<const void*>& send, const std::vector<void*>& recv) override {
    if (int rc = drain()) return rc;
    if (me == 0 && (rc_ = to_host(region(0), send[0], bytes))) return rc_;
    if (int rc = drain()) return rc;
    if (int rc = barrier()) return rc;
    if (me != 0) {
      if (int rc = to_dev(recv[0], region(0), bytes)) return rc;
      if (int rc = drain()) return rc;
    }
    return barrier();
  }
  int rc_ = 0;
  int gather0(const std::vector<u64>& cnt, size_t elem, const std::vector<const void*>& send,
              void* recv0) override {
    if (int rc = drain()) return rc;
    if (int rc = to_host(region(me), send[0], cnt[me] * elem)) return rc;
    if (int rc = drain()) return rc;
    if (int rc = barrier()) return rc;
    if (me == 0) {
      u64 o = 0;
      for (int s = 0; s < world; ++s) {
        if (int rc = to_dev(static_cast<char*>(recv0) + o * elem, region(s), cnt[s] * elem)) return rc;
        o += cnt[s];
      }
      if (int rc = drain()) return rc;
    }
    return barrier();
  }
};

// ---- partition -----------------------------------------------------------------

struct DistPlan {
  u64 S = 0;
  int R = 1, G = 0, D = 0;
  int Gh = 0;   // hash-consed (non-direct) levels from Gh on are gathered to rank 0 (G >= Gh)
  u64 B = 0;
  std::vector<u64> nk;   // global input count of node level k (nk[0] = S); pairs of level k = nk[k+1]

  void make(u64 S_, int R_) {
    S = S_;
    R = R_;
    nk.assign(1, S);
    while (nk.back() > 1 || nk.size() == 1) nk.push_back((nk.back() + 1) / 2);
    D = int(nk.size()) - 1;
    const u64 T = (S + R - 1) / R;
    // Levels 0 .. G-1 pair within a rank (>= 2^9 elements per rank after G levels); the words
    // left are gathered to rank 0, which finishes alone.  A direct level (every element
    // unique: ids are positions) costs no exchange, so direct levels stay distributed down to
    // G; but every distributed hash-consed level pays an exchange round (two host syncs, four
    // or five collectives) whatever its size, so a hash-consed level from Gh on -- ~2^23 words
    // left, t = 23 - ceil(log2 R) -- is gathered instead (GCZ_DIST_TAIL_LOG2 overrides t).
    // Uniform data: levels >= 1 are direct, the gather holds ~R * 2^9 words (round 3 gathered
    // 2^23: 5.2 MB over every link into rank 0 at R = 8, and rank 0 ran their direct levels).
    auto depth = [&](int t) {
      int g = T < (2ull << t) ? 0 : int(bit_width(T)) - 1 - t;
      g = std::min(g, 20);
      g = std::min(g, D - 1);
      return std::max(g, 0);
    };
    const char* env = std::getenv("GCZ_DIST_TAIL_LOG2");
    const int th = env ? std::atoi(env) : std::max(9, 23 - int(bit_width(u64(R) - 1)));
    Gh = depth(th);
    G = std::max(Gh, depth(9));
    const u64 g = 1ull << G;
    B = (T + g - 1) / g * g;
    // Rank 0 also finishes the gathered top alone, and its leaf level ranks the whole
    // dictionary (at 1 Gbase it first-holds 3.6-4.1 M of the 4.2 M leaves: their position
    // bitmap, ranks and leaves), work that does not shrink with its share; so it takes a
    // smaller share of B: 850 / 800 / 750 / 700 permille at R = 2 / 3 / 4 / >= 5, the rest
    // spread over the others (measured on 1 Gbase over virtual ranks, scripts/gpu_share.sh:
    // slowest rank 1.85 -> 1.81 ms at R = 2, 1.19 -> 1.07 at R = 4, 0.81 -> 0.77 at R = 8
    // against the earlier 1000 - 25 R; GCZ_DIST_RANK0_PERMILLE overrides, 1000 = even shares).  Only
    // where the ranks hold >= 2^20 strands, so every share stays a multiple of 2^G far
    // above 256.
    const char* e0 = std::getenv("GCZ_DIST_RANK0_PERMILLE");
    const u64 pm = e0 ? u64(std::max(500, std::min(1000, std::atoi(e0))))
                      : u64(R <= 2 ? 850 : R == 3 ? 800 : R == 4 ? 750 : 700);
    B0 = B1 = B;
    if (R > 1 && G > 0 && T >= (1ull << 20) && pm < 1000) {
      B0 = std::max<u64>(g, B * pm / 1000 / g * g);
      B1 = ((S - std::min(S, B0)) + u64(R - 1) - 1) / u64(R - 1);
      B1 = (B1 + g - 1) / g * g;
    }
  }
  u64 B0 = 0, B1 = 0;   // rank 0's strands, every other rank's (the last: the remainder)
  u64 first(int r) const { return r == 0 ? 0 : B0 + u64(r - 1) * B1; }
  // element range of rank r at the input of node level k (k = 0: strands), k <= G
  u64 start(int r, int k) const { return std::min(first(r) >> k, nk[k]); }
  u64 end(int r, int k) const { return std::min(first(r + 1) >> k, nk[k]); }
  u64 count(int r, int k) const { return end(r, k) - start(r, k); }
};

}  // namespace

namespace {
// Per local rank, the level being reconciled (see gcz_dist_device.h).
struct RankLevel {
  RecSrc src{};
  u64 grid_elems = 0;       // bucket grid: leaves -> capacity, nodes -> p
  const u64* ucount = nullptr;
  u32* w = nullptr;         // words to remap
  unsigned char* nf = nullptr;
  unsigned char* multi = nullptr;
  void* out = nullptr;      // rank's slice of the output layer
  bool leaves = false;
  const unsigned char* bases = nullptr;   // leaf level: for the bad-symbol report
  bool defer_remap = false;               // the next level's k_node_keys translates the words
  bool counted = false;                   // k_node_keys wrote the bucketing's tile counts
  const unsigned char* gmark = nullptr;   // leaf level: kNfGlobal strands already hold global ids
  bool identity = false;                  // rank 0's leaf level: local ids are the global ids
  bool keys_zeroed = false;               // k_node_keys zeroed gnf / gmul and the rank scan's descriptors
};
}  // namespace

struct gcz_group {
  int world = 1;
  std::vector<gcz_ctx*> ctx;   // local ranks
  std::vector<int> rank;       // their global ranks
  bool owns_ctx = false;
  Transport* tr = nullptr;
  std::string last_error;

  // ---- exchanges: numbered, logged with their bytes, bounded -------------------------
  // Every collective of a build is #seq in a sequence every rank runs identically.  The log
  // (gcz_group_xlog) gives each its bytes to / from the other ranks; GCZ_DIST_STALL =
  // "rank:seq:seconds" makes that rank sleep before #seq (tests of the bounds below).
  struct XRec {
    const char* name;
    int seq;
    std::vector<u64> sent, recvd;   // per local rank
    double t_us;                    // host enqueue time after the build began
  };
  std::vector<XRec> xlog;
  std::chrono::steady_clock::time_point t_build{};
  // RCCL has no timeout of its own: the watchdog thread is armed from a collective's enqueue
  // until the host sync that waits for it.  Past GCZ_DIST_TIMEOUT_S it names the first
  // collective that did not complete (events recorded behind each), prints it, aborts the
  // communicator (the stream and any blocked call return) and, should the build still not
  // return, ends the process.
  struct Watch {
    struct Pending {
      int seq;
      std::string what;
      hipEvent_t done;   // null while the enqueue call itself runs
    };
    RcclTransport* tr;
    int device, rank;
    long limit_s = dist_timeout_s();
    long grace_s = 30;   // after the abort: the build's return, else the process ends
    std::mutex mu;
    std::condition_variable cv;
    bool armed = false, stop = false;
    std::atomic<bool> fired{false};
    std::chrono::steady_clock::time_point deadline{};
    std::vector<Pending> pending;
    std::vector<hipEvent_t> pool;
    size_t used = 0;
    std::string msg;
    std::thread th;
    Watch(RcclTransport* t, int dev, int r) : tr(t), device(dev), rank(r) { th = std::thread([this] { loop(); }); }
    ~Watch() {
      {
        std::lock_guard<std::mutex> g(mu);
        stop = true;
      }
      cv.notify_all();
      th.join();
      for (hipEvent_t e : pool) (void)hipEventDestroy(e);
    }
    void begin(int seq, std::string what) {   // before the enqueue call
      std::lock_guard<std::mutex> g(mu);
      if (!armed) {
        armed = true;
        deadline = std::chrono::steady_clock::now() + std::chrono::seconds(limit_s);
        cv.notify_all();
      }
      pending.push_back({seq, std::move(what), nullptr});
    }
    void end(hipStream_t stream) {   // after it: an event behind the collective
      std::lock_guard<std::mutex> g(mu);
      if (used == pool.size()) {
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return;
        pool.push_back(e);
      }
      hipEvent_t e = pool[used++];
      if (hipEventRecord(e, stream) == hipSuccess && !pending.empty()) pending.back().done = e;
    }
    void disarm() {
      std::lock_guard<std::mutex> g(mu);
      armed = false;
      pending.clear();
      used = 0;
      cv.notify_all();
    }
    void loop() {
      if (device >= 0) (void)hipSetDevice(device);
      std::unique_lock<std::mutex> lk(mu);
      while (!stop) {
        if (!armed) {
          cv.wait(lk);
          continue;
        }
        if (cv.wait_until(lk, deadline) != std::cv_status::timeout || !armed || stop) continue;
        std::string what = "the host sync after the last collective";
        for (const Pending& p : pending)
          if (!p.done || hipEventQuery(p.done) == hipErrorNotReady) {
            what = p.what + (p.done ? "" : " (inside the enqueue call)");
            break;
          }
        msg = "rank " + std::to_string(rank) + ": " + what + " has not completed within " +
              std::to_string(limit_s) + " s (GCZ_DIST_TIMEOUT_S): a peer stalled or failed; RCCL communicator aborted";
        std::fprintf(stderr, "gcz watchdog: %s\n", msg.c_str());
        std::fflush(stderr);
        fired = true;
        armed = false;
        lk.unlock();
        tr->abort();
        lk.lock();
        // the aborted collective lets the build return (gcz_group::fail -> disarm clears
        // `pending`); if it does not, end the process
        const auto grace = std::chrono::steady_clock::now() + std::chrono::seconds(grace_s);
        while (!stop && !armed && pending.size() && std::chrono::steady_clock::now() < grace)
          cv.wait_until(lk, grace);
        if (!stop && pending.size()) {
          std::fprintf(stderr, "gcz watchdog: rank %d: the build did not return after the abort; exiting\n", rank);
          std::fflush(stderr);
          std::_Exit(70);
        }
      }
    }
  };
  std::unique_ptr<Watch> watch;
  int stall_rank = -1, stall_seq = -1, stall_s = 0;
  gcz_group() {
    if (const char* e = std::getenv("GCZ_DIST_STALL"))
      if (std::sscanf(e, "%d:%d:%d", &stall_rank, &stall_seq, &stall_s) != 3) stall_rank = -1;
  }
  int xbegin(const char* name, std::vector<u64> sent, std::vector<u64> recvd) {
    const int seq = int(xlog.size());
    const double t = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_build).count();
    for (int r : rank)
      if (r == stall_rank && seq == stall_seq) std::this_thread::sleep_for(std::chrono::seconds(stall_s));
    if (watch)
      watch->begin(seq, "collective #" + std::to_string(seq) + " " + name + " (this rank sends " +
                            std::to_string(sent[0]) + " B, receives " + std::to_string(recvd[0]) + " B)");
    xlog.push_back({name, seq, std::move(sent), std::move(recvd), t});
    return GCZ_OK;
  }
  int xend(int rc, hipStream_t st = nullptr) {
    if (watch) watch->end(st ? st : ctx[0]->stream);
    if (rc && tr) {
      const XRec& x = xlog.back();
      tr->err = "collective #" + std::to_string(x.seq) + " " + x.name + " (this rank sends " + std::to_string(x.sent[0]) +
                " B, receives " + std::to_string(x.recvd[0]) + " B): " + tr->err;
    }
    return rc;
  }
  // the host waits for its streams (the exchanges' counts and status words)
  int host_sync() {
    for (gcz_ctx* cx : ctx) {
      const hipError_t e = hipStreamSynchronize(cx->stream);
      if (watch && watch->fired) return fail(GCZ_ERR_DEVICE, watch->msg);
      if (e != hipSuccess) return dev_fail((std::string("hipStreamSynchronize: ") + hipGetErrorString(e)).c_str());
    }
    if (watch) watch->disarm();
    return GCZ_OK;
  }
  // Every rank's flag, allgathered on the RCCL communicator under the watchdog (group creation):
  // *all = 1 when each rank passed a nonzero `mine`.
  int agree(const char* what, int mine, int* all) {
    *all = 0;
    auto* rt = static_cast<RcclTransport*>(tr);
    hipStream_t st = ctx[0]->stream;
    std::vector<int> h(size_t(world) + 1, 0);
    h[0] = mine;
    void* d = nullptr;
    if (hipMalloc(&d, h.size() * 4) != hipSuccess) {
      last_error = std::string(what) + ": hipMalloc failed";
      return GCZ_ERR_DEVICE;
    }
    int rc = hipMemcpyAsync(d, h.data(), 4, hipMemcpyHostToDevice, st) == hipSuccess ? GCZ_OK : GCZ_ERR_DEVICE;
    if (!rc) {
      watch->begin(-1, what);
      ncclComm_t c = rt->comm.load();
      if (!c || rccl().AllGather(d, static_cast<int*>(d) + 1, 4, ncclUint8, c, st) != ncclSuccess) rc = GCZ_ERR_DEVICE;
      watch->end(st);
      if (!rc && hipMemcpyAsync(h.data() + 1, static_cast<int*>(d) + 1, size_t(world) * 4, hipMemcpyDeviceToHost, st) !=
                     hipSuccess)
        rc = GCZ_ERR_DEVICE;
      if (hipStreamSynchronize(st) != hipSuccess) rc = GCZ_ERR_DEVICE;
      if (watch->fired) {
        last_error = watch->msg;
        rc = GCZ_ERR_DEVICE;
      }
      watch->disarm();
    }
    (void)hipFree(d);
    if (rc) {
      if (last_error.empty()) last_error = std::string(what) + ": allgather failed";
      return rc;
    }
    int a = 1;
    for (int r = 0; r < world; ++r) a &= h[size_t(r) + 1] != 0 ? 1 : 0;
    *all = a;
    return GCZ_OK;
  }
  std::vector<u64> per_local(const std::function<u64(int)>& f) const {
    std::vector<u64> v;
    for (int r : rank) v.push_back(f(r));
    return v;
  }
  int x_alltoallv(const char* name, const std::vector<u64>& M, bool rev, size_t elem, const std::vector<const void*>& s,
                  const std::vector<void*>& r) {
    const int R = world;
    xbegin(name, per_local([&](int me) { u64 t = 0; for (int q = 0; q < R; ++q) if (q != me) t += mcount(M, R, rev, me, q); return t * elem; }),
           per_local([&](int me) { u64 t = 0; for (int q = 0; q < R; ++q) if (q != me) t += mcount(M, R, rev, q, me); return t * elem; }));
    return xend(tr->alltoallv(M, rev, elem, s, r));
  }
  int x_alltoallv_at(const char* name, const std::vector<u64>& M, bool rev, size_t elem, const std::vector<u64>& sd,
                     const std::vector<u64>& rd, const std::vector<const void*>& s, const std::vector<void*>& r) {
    const int R = world;
    xbegin(name, per_local([&](int me) { u64 t = 0; for (int q = 0; q < R; ++q) if (q != me) t += mcount(M, R, rev, me, q); return t * elem; }),
           per_local([&](int me) { u64 t = 0; for (int q = 0; q < R; ++q) if (q != me) t += mcount(M, R, rev, q, me); return t * elem; }));
    return xend(tr->alltoallv_at(M, rev, elem, sd, rd, s, r));
  }
  // One group of exchanges (Transport::group), logged as one collective with the ops' bytes.
  int x_group(const char* name, const std::vector<Transport::XOp>& ops) {
    const int R = world;
    auto tot = [&](int me, bool sent) {
      u64 t = 0;
      for (const Transport::XOp& o : ops)
        for (int q = 0; q < R; ++q)
          if (q != me) t += (sent ? mcount(o.M, R, o.rev, me, q) : mcount(o.M, R, o.rev, q, me)) * o.elem;
      return t;
    };
    xbegin(name, per_local([&](int me) { return tot(me, true); }), per_local([&](int me) { return tot(me, false); }));
    return xend(tr->group(ops));
  }
  // A bulk group (Transport::group_bulk) on the transport's second stream: it starts once the
  // build's stream reaches the last bulk_mark() (or the call itself); bulk_done() makes the
  // build's stream wait for it.
  hipEvent_t ev_bulk_in = nullptr, ev_bulk_out = nullptr;
  bool bulk_marked = false;
  int bulk_mark() {
    if (!tr->bulk_stream()) return GCZ_OK;
    if (!ev_bulk_in && (hipEventCreateWithFlags(&ev_bulk_in, hipEventDisableTiming) != hipSuccess ||
                        hipEventCreateWithFlags(&ev_bulk_out, hipEventDisableTiming) != hipSuccess))
      return dev_fail("bulk events");
    if (hipEventRecord(ev_bulk_in, ctx[0]->stream) != hipSuccess) return dev_fail("bulk stream order");
    bulk_marked = true;
    return GCZ_OK;
  }
  // (name: in line on the build's stream; name2: on the second stream -- the log says which ran)
  bool bulk_pending = false;   // a bulk group is queued that bulk_done() has not ordered yet
  int x_group_bulk(const char* name, const char* name2, const std::vector<Transport::XOp>& ops) {
    hipStream_t bs = tr->bulk_stream();
    if (bs) {
      if (!bulk_marked)
        if (int rc = bulk_mark()) return rc;
      bulk_marked = false;
      if (hipStreamWaitEvent(bs, ev_bulk_in, 0) != hipSuccess) return dev_fail("bulk stream order");
      name = name2;
    }
    const int R = world;
    auto tot = [&](int me, bool sent) {
      u64 t = 0;
      for (const Transport::XOp& o : ops)
        for (int q = 0; q < R; ++q)
          if (q != me) t += (sent ? mcount(o.M, R, o.rev, me, q) : mcount(o.M, R, o.rev, q, me)) * o.elem;
      return t;
    };
    xbegin(name, per_local([&](int me) { return tot(me, true); }), per_local([&](int me) { return tot(me, false); }));
    const int rc = xend(tr->group_bulk(ops), bs);
    if (bs && hipEventRecord(ev_bulk_out, bs) != hipSuccess) return dev_fail("bulk stream order");
    bulk_pending = bs != nullptr;
    return rc;
  }
  int bulk_done() {
    hipStream_t bs = tr->bulk_stream();
    if (bs && hipStreamWaitEvent(ctx[0]->stream, ev_bulk_out, 0) != hipSuccess) return dev_fail("bulk stream order");
    bulk_pending = false;
    return GCZ_OK;
  }
  int x_allgather(const char* name, size_t bytes, const std::vector<const void*>& s, const std::vector<void*>& r) {
    xbegin(name, per_local([&](int) { return u64(bytes) * u64(world - 1); }),
           per_local([&](int) { return u64(bytes) * u64(world - 1); }));
    return xend(tr->allgather(bytes, s, r));
  }
  int x_bcast0(const char* name, size_t bytes, const std::vector<const void*>& s, const std::vector<void*>& r) {
    xbegin(name, per_local([&](int me) { return me == 0 ? u64(bytes) * u64(world - 1) : u64(0); }),
           per_local([&](int me) { return me == 0 ? u64(0) : u64(bytes); }));
    return xend(tr->bcast0(bytes, s, r));
  }
  int x_gather0(const char* name, const std::vector<u64>& cnt, size_t elem, const std::vector<const void*>& s,
                void* recv0) {
    xbegin(name, per_local([&](int me) { return me == 0 ? u64(0) : cnt[size_t(me)] * elem; }),
           per_local([&](int me) {
             u64 t = 0;
             if (me == 0) for (int q = 1; q < world; ++q) t += cnt[size_t(q)];
             return t * elem;
           }));
    return xend(tr->gather0(cnt, elem, s, recv0));
  }
  // last build
  gcz_info info{};
  DistPlan plan;
  std::vector<std::vector<u64>> slice_off, slice_cnt;   // [layer + 1][global rank]
  std::vector<std::vector<u64>> node_base;              // [local][layer]: node offset within nodes_out
  bool allow_packed = true;
  // node levels: 0 auto (local dedupe only on repetitive data), 1 always, 2 never (GCZ_DIST_LOCAL)
  int dist_local = std::getenv("GCZ_DIST_LOCAL") ? std::atoi(std::getenv("GCZ_DIST_LOCAL")) : 0;
  // leaf dictionary: rank 0's first-occurrence keys of its first seed_chunks leaf chunks (0: off;
  // GCZ_DIST_SEED)
  int seed_chunks = std::getenv("GCZ_DIST_SEED") ? std::atoi(std::getenv("GCZ_DIST_SEED")) : 1;
  // leaf chunk plan of the ranks (first chunk S_r >> this; GCZ_DIST_LEAF_FIRST_LOG2): one
  // chunk of S_r / 8 makes rank 0's dictionary (3.85 M of the 4.2 M distinct uniform 12-mers)
  // in one insert / flagscan / resolve -- the other ranks wait for it -- and the seeded ranks'
  // later chunks mostly hit settled slots, so small chunks only add launches
  int leaf_first_log2 = std::getenv("GCZ_DIST_LEAF_FIRST_LOG2")
                            ? std::max(1, std::min(20, std::atoi(std::getenv("GCZ_DIST_LEAF_FIRST_LOG2"))))
                            : 3;
  bool any_predup = false;   // some rank's leaf probe found repetitive data (set by the leaf exchange)
  bool leaf_deferred = false;   // the leaf words keep local ids until layer 0's k_node_keys
  std::vector<u32> leaf_offs;   // ... and each local rank's leaf id offset
  std::vector<const unsigned char*> leaf_gmark;   // ... its seeded-strand marks
  std::vector<bool> leaf_identity;                // ... and whether its ids are already global

  int fail(int code, const std::string& what) {
    last_error = what;
    info.status = code;
    // the build returns: nothing of it is pending any more -- also after the watchdog fired, whose
    // thread would otherwise take the build for hung and end the process after its grace period
    // (a failing rank's peers are bounded by their own watchdogs)
    if (watch) watch->disarm();
    // a bulk group still queued on the second stream is ordered before whatever the build's
    // stream runs next, so every later sync of that stream (the next build's buffer growth, the
    // teardown) also covers it
    if (bulk_pending) {
      bulk_pending = false;
      if (ev_bulk_out) (void)hipStreamWaitEvent(ctx[0]->stream, ev_bulk_out, 0);
    }
    for (gcz_ctx* c : ctx) c->fail(code, "group build", what.c_str());
    return code;
  }
  int dev_fail(const char* what) {
    return fail(GCZ_ERR_DEVICE, std::string(what) + (tr && !tr->err.empty() ? ": " + tr->err : ""));
  }
  // a callee's device failure, its message kept: "what <- inner" (inner: the callee's own
  // message, else the transport's)
  int chain_fail(const char* what) {
    const std::string inner = !last_error.empty() ? last_error : tr ? tr->err : std::string();
    return fail(GCZ_ERR_DEVICE, std::string(what) + " <- " + inner);
  }
  int build(const void* const* d_bases, const u64* const* d_leaves, u64 S, int L);
  int assemble(gcz_ctx* dst);
  int alloc(int i, u64 leaf_cap);
  // The dense leaf level of every rank + the presence / r-first-list exchange
  // (gcz_dense.h); *used = false when some strand is not pure ACGT.
  int dense_leaves(const std::vector<const unsigned char*>& bases, const u64* const* d_leaves, int L,
                   std::vector<u64>& c, std::vector<u64>& off, u64& total, bool* used);
  int dense_mode = std::getenv("GCZ_DENSE") ? std::atoi(std::getenv("GCZ_DENSE")) : 1;   // 0: hash-table leaves
  // owners hash-cons levels without the local dedupe in LDS buckets (GCZ_OWNER_BUCKETS=0: the table)
  bool owner_buckets = !std::getenv("GCZ_OWNER_BUCKETS") || std::atoi(std::getenv("GCZ_OWNER_BUCKETS")) != 0;
  bool owner_two_pass = !std::getenv("GCZ_OWNER_TWO") || std::atoi(std::getenv("GCZ_OWNER_TWO")) != 0;
  // A node level's words keep their local ids after exchange() when defer_node_remap is set:
  // the next level's direct subtrees translate them on their load (DirectRemap), else
  // remap_level runs k_dist_remap.
  bool defer_node_remap = false;
  std::vector<u32> remap_off;   // each local rank's id offset of the last exchanged level
  int remap_level(std::vector<RankLevel>& lv, const std::vector<u64>& nwords) {
    for (int i = 0; i < int(ctx.size()); ++i) {
      gcz_ctx* cx = ctx[i];
      ProfScope ps_(cx, KID_REMAP);
      hipLaunchKernelGGL(k_dist_remap, dim3(unsigned(std::max<u64>(1, (nwords[i] + kBlock - 1) / kBlock))),
                         dim3(kBlock), 0, cx->stream, lv[i].w, nwords[i], lv[i].nf, lv[i].multi,
                         cx->dist->gid.as<u32>(), cx->dist->gmul.as<unsigned char>(), remap_off[i], lv[i].gmark);
      if (hipGetLastError() != hipSuccess) return dev_fail("remap");
    }
    return GCZ_OK;
  }
  int finish_top(int Gx, bool direct, u64 prev_total, const std::vector<u32*>& cur_in, std::vector<u64>& dcur,
                 bool fl, bool* failed);
  // The fused leaf + layer-0 schedule (gcz_dist_fast.h); *taken = false: not applicable to this
  // genome, or the attempt was discarded on every rank -- the general schedule follows.
  int build_fast(const std::vector<const unsigned char*>& bases, const u64* const* d_leaves, int L,
                 const std::vector<u64>& leaf_cap, bool* taken);
  int fast_mode = std::getenv("GCZ_DIST_FAST") ? std::atoi(std::getenv("GCZ_DIST_FAST")) : 1;   // 0: off
  // k_fl_scatter's look-back polls before a tile gives up (GCZ_FL_SPIN_CAP, testing; 0: every
  // tile after the first gives up at once -- the attempt is discarded on every rank)
  u32 fl_spin_cap = std::getenv("GCZ_FL_SPIN_CAP") ? u32(std::strtoul(std::getenv("GCZ_FL_SPIN_CAP"), nullptr, 10))
                                                   : kFlSpinCap;
  hipEvent_t ev_mid = nullptr;   // the fused schedule's mid-build read (status, counts)
  FlPairs fl_pairs{};            // ... and every rank's layer-0 pairs
  RecSrc fl_rs[kMaxRanks] = {};  // ... each local rank's layer-0 record source
  // segment boundaries of the fused schedule's compute stream, a zero-length profiled scope on
  // every local rank (bench.py splits each rank's kernel time at them: scripts/budget.py's model)
  // (GCZ_FL_CHECK=1: every segment synchronised and its first device error printed -- debugging)
  bool fl_check = std::getenv("GCZ_FL_CHECK") != nullptr;
  void fl_mark(const char* name) {
    for (gcz_ctx* cx : ctx) {
      ProfScope ps_(cx, KID_MARK);
      if (fl_check) {
        const hipError_t e = hipStreamSynchronize(cx->stream), e2 = hipGetLastError();
        if (e != hipSuccess || e2 != hipSuccess)
          std::fprintf(stderr, "gcz fused schedule: segment %s: %s / %s\n", name, hipGetErrorString(e), hipGetErrorString(e2));
      }
    }
  }
  Header* cx_hdr(int i) { return ctx[i]->hdr.as<Header>(); }
  int event_sync(hipEvent_t e);
  int build_done();
  int exchange(std::vector<RankLevel>& lv, const std::vector<u64>& nwords, u32 key_bits, u32 child_bits,
               std::vector<u64>& c, std::vector<u64>& off, u64& total, u64* err_global, int* err_sym,
               int* ovf_bits, bool nolocal = false, bool lookahead = false, u64* next_hashed_out = nullptr);
};

#define G_HIP(x)                                                                   \
  do {                                                                             \
    const hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) return dev_fail((std::string(#x) + ": " + hipGetErrorString(e_)).c_str()); \
  } while (0)
// (a device failure keeps the inner message: "outer <- inner")
#define G_RC(x)                                                                    \
  do {                                                                             \
    int rc_ = (x);                                                                 \
    if (rc_) return rc_ == GCZ_ERR_DEVICE ? chain_fail(#x) : rc_;                 \
  } while (0)

namespace {
constexpr int kRetry = -1000;   // internal: some rank overflowed a table, rebuild
}

int gcz_group::alloc(int i, u64 leaf_cap) {
  gcz_ctx* c = ctx[i];
  const int r = rank[i];
  const DistPlan& P = plan;
  const u64 S_r = P.count(r, 0);
  const u64 nG = r == 0 ? P.nk[P.Gh] : 0;   // (the gather happens at a level in [Gh, G])
  const u64 wmax = std::max(S_r, nG);
  if (!c->dist) c->dist = new gcz_dist_state();
  gcz_dist_state& d = *c->dist;
  // node storage: local slices of the distributed layers; rank 0 holds every layer from Gh on
  // whole (a gathered layer, or its slice at the region's start)
  node_base[i].assign(P.D + 1, 0);
  u64 nodes = 0;
  for (int k = 0; k < P.D; ++k) {
    node_base[i][k] = nodes;
    if (r == 0 && k >= P.Gh) nodes += P.nk[k + 1];
    else if (k < P.G) nodes += P.count(r, k + 1);
  }
  node_base[i][P.D] = nodes;
  const auto chunks = leaf_chunks(S_r, leaf_first_log2);
  u64 tiles = 0;
  auto ntiles = [](u64 n) { return (n + scan_tile(n) - 1) / scan_tile(n); };
  for (size_t q = 0; q + 1 < chunks.size(); ++q) tiles += ntiles(chunks[q + 1] - chunks[q]);
  for (int k = 0; k < P.D; ++k) {
    tiles += ntiles(k < P.G ? P.count(r, k + 1) : 0);
    if (r == 0 && k >= P.Gh) tiles += ntiles(P.nk[k + 1]);
  }
  int rc;
  if ((rc = c->ensure(c->wa, wmax * 4 + 16))) return rc;
  if ((rc = c->ensure(c->wb, wmax * 4 + 16))) return rc;
  if ((rc = c->ensure(c->grp, ((wmax + 63) / 64 + kGroupsPerTile) * sizeof(Group)))) return rc;
  if ((rc = c->ensure(c->desc, tiles * 8 + 64))) return rc;
  if ((rc = c->ensure(c->leaves_out, S_r * 8 + 16))) return rc;
  if ((rc = c->ensure(c->nodes_out, nodes * 8 + 16))) return rc;
  if ((rc = c->ensure(c->hdr, sizeof(Header)))) return rc;
  if ((rc = c->ensure(c->stats, kStatBytes))) return rc;
  if ((rc = c->ensure_marks(wmax))) return rc;
  const u64 pmax = std::max<u64>(P.G > 0 ? P.count(r, 1) : 0, nG > 1 ? (nG + 1) / 2 : 1);
  c->cap_boost = 0;   // (the single-device small-build boost is not used here)
  if ((rc = c->ensure(c->tab, std::max(leaf_cap, c->node_cap(pmax)) * 16))) return rc;
  if (!c->h_hdr && hipHostMalloc((void**)&c->h_hdr, sizeof(Header), hipHostMallocDefault) != hipSuccess)
    return GCZ_ERR_DEVICE;
  const u64 u = S_r + 16;
  if ((rc = c->ensure(d.scratch, u * 8))) return rc;
  if ((rc = c->ensure(d.gnf, u))) return rc;
  if ((rc = c->ensure(d.gmul, u))) return rc;
  if ((rc = c->ensure(d.gid, u * 4))) return rc;
  if ((rc = c->ensure(d.blockcnt, (u64(world) * ((u + kTile - 1) / kTile + 1)) * 4 + 64))) return rc;
  if ((rc = c->ensure(d.skey, u * 8))) return rc;
  if ((rc = c->ensure(d.sidx, u * 4))) return rc;
  if ((rc = c->ensure(d.sflag, u))) return rc;
  if ((rc = c->ensure(d.scval, u * 8))) return rc;
  if ((rc = c->ensure(d.sdval, u * 8))) return rc;
  if ((rc = c->ensure(d.clist, u * 4))) return rc;
  if ((rc = c->ensure(d.dhdr, kDistHdrBytes))) return rc;
  if ((rc = c->ensure(d.gath, size_t(world) * kSyncWords * 8))) return rc;
  if ((rc = c->ensure(d.gath2, size_t(world) * (2 + 2 * kMaxRanks) * 8))) return rc;
  if ((rc = c->ensure(d.gathf, size_t(world) * kFinalWords * 8))) return rc;
  if ((rc = c->ensure(d.ddesc, ((u + kTile - 1) / kTile) * 8 + 64))) return rc;
  if ((rc = c->ensure(d.tail_in, nG * 4 + 16))) return rc;
  if (!d.h_gath) {
    if (hipHostMalloc((void**)&d.h_gath, size_t(kMaxRanks) * kSyncWords * 8, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc((void**)&d.h_gath2, size_t(kMaxRanks) * (2 + 2 * kMaxRanks) * 8, hipHostMallocDefault) !=
            hipSuccess ||
        hipHostMalloc((void**)&d.h_gathf, size_t(kMaxRanks) * kFinalWords * 8, hipHostMallocDefault) != hipSuccess)
      return GCZ_ERR_DEVICE;
  }
  return GCZ_OK;
}


int gcz_group::dense_leaves(const std::vector<const unsigned char*>& bases, const u64* const* d_leaves, int L,
                            std::vector<u64>& c, std::vector<u64>& off, u64& total, bool* used) {
  *used = false;
  const int R = world, NL = int(ctx.size());
  const DistPlan& P = plan;
  const u64 ncodes = u64(1) << dense_code_bits(u32(L));
  const u64 nw = (ncodes + 63) / 64;   // presence bitmap words
  const u64 nwb = nw + 4;               // + the rank's status words (vec) behind its bitmap
  std::vector<LeafLevel> las(NL);
  // A. every rank's local first positions by code and presence bitmap.  The status words
  // (pure ACGT? / 0 / repetitive?) ride behind the bitmap, so exchange 1 is one
  // allgather; a rank that fails here still joins it with a failure word (vec[0] = 2), so its
  // peers leave together instead of waiting in a collective it never enters (RCCL has no
  // timeout).
  int local_rc = 0;
  for (int i = 0; i < NL; ++i) {
    gcz_ctx* cx = ctx[i];
    LeafLevel& la = las[i];
    la.bases = bases[i];
    la.leaves = d_leaves ? d_leaves[i] : nullptr;
    la.S = P.count(rank[i], 0);
    la.L = L;
    la.words = cx->wa.as<u32>();
    if (cx->ensure(cx->dl_seg, size_t(64 + 3 * R) * 8 + 64) || cx->ensure(cx->dl_pb, nwb * 8) ||
        cx->ensure(cx->dl_pbs, size_t(R) * nwb * 8 + 16))
      return dev_fail("dense leaf buffers");   // (no word to send: nothing else can be done)
    u64* vec = cx->dl_pb.as<u64>() + nw;
    bool u = false;
    Header* h = cx->hdr.as<Header>();
    cx->probe_ranks = unsigned(R);
    const int rc = cx->dense_phase_a(la, h, &h->count[0], false, true, &u, vec);   // (writes vec too)
    cx->probe_ranks = 1;
    if (!rc && !u) return GCZ_OK;   // L or sizes outside the dense level (the same on every rank)
    if (rc) {
      local_rc = rc;
      static const u64 failed_vec[3] = {2, 0, 0};
      G_HIP(hipMemcpyAsync(vec, failed_vec, sizeof(failed_vec), hipMemcpyHostToDevice, cx->stream));
      continue;
    }
  }
  if (local_rc && NL == R) return local_rc == GCZ_ERR_DEVICE ? dev_fail("dense leaves") : local_rc;
  // exchange 1: the presence bitmaps with the status words
  {
    std::vector<const void*> s;
    std::vector<void*> rv;
    for (gcz_ctx* cx : ctx) {
      s.push_back(cx->dl_pb.ptr);
      rv.push_back(cx->dl_pbs.ptr);
    }
    hipEvent_t e0{};
    ctx[0]->prof_begin(KID_EXCHANGE, e0);
    G_RC(x_allgather("leaf presence bitmaps + status", nwb * 8, s, rv));
    ctx[0]->prof_end(KID_EXCHANGE, e0);
  }
  // (no host sync here: the status words travel on in the exchange vectors below; a rank
  // with a non-ACGT strand runs B1 on in-bounds data -- its pack marked those strands -- and
  // every rank learns of it after exchange 2)
  // B1: r-first codes (held by no lower rank), their position bitmap and local ranks, and G =
  // those ranks in code order with the bucket prefixes in the exchange vector (gcz_dense.h)
  const u32 NB = ctx[0]->dl_plan.NB, RB = 1u << ctx[0]->dl_plan.IB;
  const u64 xw = (u64(NB) + 2 + 1) & ~u64(1);   // exchange vector words (u32), even
  for (int i = 0; i < NL; ++i) {
    gcz_ctx* cx = ctx[i];
    const int r = rank[i];
    const DensePlan& DP = cx->dl_plan;
    Header* h = cx->hdr.as<Header>();
    if (cx->ensure(cx->dl_pos, (u64(NB) + xw) * 4 + 64)) return dev_fail("dense leaf buffers");
    if (local_rc) {   // this rank's phase A failed: it joins exchange 2 with a failure word only
      static const u32 failed_xv[2] = {0, 4};   // (static: the async copy may read it after this scope)
      G_HIP(hipMemcpyAsync(cx->dl_pos.as<u32>() + NB, failed_xv, sizeof(failed_xv), hipMemcpyHostToDevice, cx->stream));
      continue;
    }
    const u64 nfb = (DP.S + 63) / 64, t = scan_tiles(nfb + 1);
    if (cx->ensure(cx->dl_lh, ncodes * 4 + 16) || cx->ensure(cx->dl_list, std::min<u64>(DP.S, ncodes) * 4 + 16) ||
        cx->ensure(cx->dl_pos, (u64(NB) + xw) * 4 + 64) || cx->ensure(cx->dl_lower, u64(R) * xw * 4 + 16))
      return dev_fail("dense leaf buffers");
    u32* bcnt = cx->dl_pos.as<u32>();
    u32* xv = bcnt + NB;
    // the popcount scan's descriptors and ticket: the ones dense_phase_a zeroed for the
    // single-device first-occurrence scan, which list mode does not run
    const u64 t_cnt = scan_tiles(u64(NB) * DP.nch + 1);
    u64* desc = cx->dl_desc.as<u64>() + t_cnt;
    u32* ticket = reinterpret_cast<u32*>(desc + t) + 1;
    {
      ProfScope ps_(cx, KID_DL_FIRST);
      G_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_dl_rfirst), hipFuncAttributeMaxDynamicSharedMemorySize,
                                int((DP.nch + 1) * 4)));
      hipLaunchKernelGGL(k_dl_rfirst, dim3(NB), dim3(kDThreads), (DP.nch + 1) * 4, cx->stream, cx->dl_fpg.as<u32>(), DP,
                         cx->dl_pbs.as<unsigned long long>(), nwb, r, cx->dl_fl.as<u32>(), cx->dl_fo.as<u32>(),
                         cx->dl_lh.as<u32>(), bcnt);
      hipLaunchKernelGGL(k_dl_fb, dim3(DP.nch), dim3(kDThreads), 0, cx->stream, cx->dl_fl.as<u32>(), cx->dl_fo.as<u32>(),
                         DP, cx->dl_fb.as<unsigned long long>());
      G_HIP(hipGetLastError());
    }
    {
      ProfScope ps_(cx, KID_DL_FBSCAN);
      hipLaunchKernelGGL(k_scan_excl<ScanPopc>, dim3(unsigned(t)), dim3(kScanThreads), 0, cx->stream,
                         ScanPopc{cx->dl_fb.as<unsigned long long>()}, nfb, cx->dl_wpre.as<u32>(), desc, ticket,
                         &h->count[0]);
      hipLaunchKernelGGL(k_dl_gq, dim3(NB), dim3(kDThreads), 0, cx->stream, cx->dl_lh.as<u32>(), bcnt, DP,
                         cx->dl_fb.as<unsigned long long>(), cx->dl_wpre.as<u32>(),
                         static_cast<const u64*>(&h->count[0]), cx->dl_list.as<u32>(), xv, cx->dl_pw.as<u32>(),
                         cx->leaves_out.as<u64>(), static_cast<const u64*>(cx->dl_pb.as<u64>() + nw));
      G_HIP(hipGetLastError());
    }
  }
  // exchange 2: the exchange vectors (r-first counts -> id offsets; bucket prefixes)
  {
    std::vector<const void*> s;
    std::vector<void*> rv;
    for (gcz_ctx* cx : ctx) {
      s.push_back(cx->dl_pos.as<u32>() + NB);
      rv.push_back(cx->dl_lower.ptr);
    }
    hipEvent_t e0{};
    ctx[0]->prof_begin(KID_EXCHANGE, e0);
    G_RC(x_allgather("leaf r-first counts + bucket prefixes", xw * 4, s, rv));
    ctx[0]->prof_end(KID_EXCHANGE, e0);
  }
  std::vector<u32> hx(size_t(R) * xw);
  G_HIP(hipMemcpyAsync(hx.data(), ctx[0]->dl_lower.ptr, hx.size() * 4, hipMemcpyDeviceToHost, ctx[0]->stream));
  G_RC(host_sync());
  {   // status words (gcz_dense.h k_dl_gq): bit 0 a non-ACGT strand, bit 1 repetitive data, bit 2 failed
    u32 any = 0;
    for (int r = 0; r < R; ++r) any |= hx[size_t(r) * xw + 1];
    if (any & 4) return local_rc && local_rc != GCZ_ERR_DEVICE ? local_rc : dev_fail("dense leaves (a rank failed)");
    if (any & 1) return GCZ_OK;   // some rank holds a non-ACGT strand: the hash-table leaf level
    any_predup = (any & 2) != 0;
  }
  c.assign(R, 0);
  off.assign(R + 1, 0);
  for (int r = 0; r < R; ++r) {
    c[r] = hx[size_t(r) * xw];
    off[r + 1] = off[r] + c[r];
  }
  total = off[R];
  if (total > u64(kIdx)) return fail(GCZ_ERR_CAPACITY, "more than 2^29-1 unique leaves");
  // exchange 3: every rank gets every G array, relayed in two steps so no link carries rank
  // 0's long one R - 1 times: piece q of array r goes to rank q, then each rank sends the
  // pieces it holds to all ranks; k_dl_ids_mr reads each element where its piece landed
  auto pc = [&](int r, int q) { return c[r] * u64(q) / u64(R); };   // start of piece q of array r
  std::vector<u64> M1(size_t(R) * R), T(R, 0), M2(size_t(R) * R), sd2(size_t(R) * R, 0), rd2(size_t(R) * R);
  for (int r = 0; r < R; ++r)
    for (int q = 0; q < R; ++q) {
      M1[size_t(r) * R + q] = pc(r, q + 1) - pc(r, q);
      T[q] += M1[size_t(r) * R + q];
    }
  for (int q = 0; q < R; ++q)
    for (int d = 0; d < R; ++d) {
      M2[size_t(q) * R + d] = T[q];
      u64 o = 0;
      for (int q2 = 0; q2 < q; ++q2) o += T[q2];
      rd2[size_t(d) * R + q] = o;
    }
  DlRelay relay{};
  {
    u64 o = 0;
    for (int q = 0; q < R; ++q)   // (relay order: piece index outer, list inner)
      for (int r = 0; r < R; ++r) {
        const size_t sg = size_t(r) * R + q;
        relay.seg_src[sg] = o;
        relay.seg_dst[sg] = off[r] + pc(r, q);
        relay.seg_len[sg] = M1[sg];
        o += M1[sg];
      }
    for (int r = 0; r <= R; ++r) relay.off[r] = off[r];
  }
  {
    std::vector<const void*> s;
    std::vector<void*> rv;
    for (int i = 0; i < NL; ++i) {
      gcz_ctx* cx = ctx[i];
      if (cx->ensure(cx->dl_stage, T[rank[i]] * 4 + 16) || cx->ensure(cx->dl_recv, total * 4 + 16))
        return dev_fail("dense leaf relay");
      s.push_back(cx->dl_list.ptr);
      rv.push_back(cx->dl_stage.ptr);
    }
    hipEvent_t e0{};
    ctx[0]->prof_begin(KID_EXCHANGE, e0);
    G_RC(x_alltoallv("leaf G arrays, relay 1", M1, false, 4, s, rv));
    std::vector<const void*> s2;
    std::vector<void*> rv2;
    for (gcz_ctx* cx : ctx) {
      s2.push_back(cx->dl_stage.ptr);
      rv2.push_back(cx->dl_recv.ptr);
    }
    G_RC(x_alltoallv_at("leaf G arrays, relay 2", M2, false, 4, sd2, rd2, s2, rv2));
    ctx[0]->prof_end(KID_EXCHANGE, e0);
  }
  // B2: the global id of every code held here and the final word per record, the words in
  // position order, and this rank's slice of the leaves
  for (int i = 0; i < NL; ++i) {
    gcz_ctx* cx = ctx[i];
    const int r = rank[i];
    const DensePlan& DP = cx->dl_plan;
    Header* h = cx->hdr.as<Header>();
    {
      ProfScope ps_(cx, KID_DL_IDS);
      if (cx->ensure(cx->dl_gid, sizeof(DlRelay) + 16)) return dev_fail("dense leaf relay table");
      // staged in pinned memory the context owns (the copy is asynchronous; the previous build's
      // copy has completed: every build ends with a host sync)
      gcz_dist_state& ds = *cx->dist;
      if (!ds.h_relay && hipHostMalloc((void**)&ds.h_relay, sizeof(DlRelay), hipHostMallocDefault) != hipSuccess)
        return dev_fail("dense leaf relay staging");
      *ds.h_relay = relay;
      G_HIP(hipMemcpyAsync(cx->dl_gid.ptr, ds.h_relay, sizeof(DlRelay), hipMemcpyHostToDevice, cx->stream));
      G_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_dl_ids_mr), hipFuncAttributeMaxDynamicSharedMemorySize,
                                int(RB * 4)));
      hipLaunchKernelGGL(k_dl_ids_mr, dim3(NB), dim3(kDThreads), RB * 4, cx->stream, cx->dl_rec.as<u32>(),
                         cx->dl_off.as<u32>(), DP, cx->dl_pbs.as<unsigned long long>(), nwb, cx->dl_lower.as<u32>(), xw,
                         static_cast<const u32*>(cx->dl_recv.as<u32>()), cx->dl_gid.as<DlRelay>(), R, r,
                         cx->dl_idrec.as<u32>());
      const u64 cr = c[r];
      if (cr && !dl_rleaves_sparse(cr, DP.S))   // (sparse: k_dl_gq wrote them)
        hipLaunchKernelGGL(k_dl_rleaves, dim3(unsigned((DP.S + 255) / 256)), dim3(256), 0, cx->stream,
                           cx->dl_fb.as<unsigned long long>(), cx->dl_wpre.as<u32>(), cx->dl_pw.as<u32>(), DP,
                           cx->leaves_out.as<u64>());
      G_HIP(hipGetLastError());
    }
    if (int rc = cx->dense_phase_b(las[i], h, nullptr, nullptr, true))
      return rc == GCZ_ERR_DEVICE ? dev_fail("dense leaves") : rc;
  }
  *used = true;
  return GCZ_OK;
}

// key_bits: bits of the owner-table key (leaves 4L, nodes 2 (child_bits + 2)); packed slots when
// key_bits + R + 2 <= 64, else wide.
// nolocal: the senders skipped the local dedupe of this level (k_node_keys), the owners
// find the first occurrence from the receive order (stable bucketing).
int gcz_group::exchange(std::vector<RankLevel>& lv, const std::vector<u64>& nwords, u32 key_bits, u32 child_bits,
                        std::vector<u64>& c, std::vector<u64>& off, u64& total, u64* err_global, int* err_sym,
                        int* ovf_bits, bool nolocal, bool lookahead, u64* next_hashed_out) {
  const int R = world, NL = int(ctx.size());
  u64 next_hashed = 0;
  if (next_hashed_out) *next_hashed_out = ~0ull;
  // 1. bucket the records by owner, pack the sync vector
  for (int i = 0; i < NL; ++i) {
    gcz_ctx* cx = ctx[i];
    gcz_dist_state& d = *cx->dist;
    RankLevel& L = lv[i];
    L.src.R = u32(R);
    DistHdr* dh = d.dhdr.as<DistHdr>();
    G_HIP(hipMemsetAsync(dh, 0, offsetof(DistHdr, cell), cx->stream));
    const u32 nb = u32(std::max<u64>(1, (L.grid_elems + kTile - 1) / kTile));
    hipEvent_t eb{};
    cx->prof_begin(KID_DIST, eb);
    if (!L.counted)
      hipLaunchKernelGGL(k_bucket_count, dim3(nb), dim3(kBlock), 0, cx->stream, L.src, d.blockcnt.as<u32>(), nb);
    if (u64(R) * nb <= kBscanSmall) {   // one block: the scan, the totals and the sync vector
      hipLaunchKernelGGL(k_bscan_small, dim3(1), dim3(1024), 0, cx->stream, d.blockcnt.as<u32>(), u32(R), nb, dh->sync,
                         cx->hdr.as<Header>(), L.ucount, L.bases);
      hipLaunchKernelGGL(k_bucket_scatter, dim3(nb), dim3(kBlock), 0, cx->stream, L.src, d.blockcnt.as<u32>(), nb,
                         d.skey.as<u64>(), d.sidx.as<u32>());
    } else {
      const u32 cpr = (nb + kScanChunk - 1) / kScanChunk;
      if (u64(R) * cpr > 1024) return fail(GCZ_ERR_CAPACITY, "bucket scan: too many chunks");
      if (cx->ensure(d.bchunk, u64(R) * cpr * 4 + 64)) return dev_fail("bucket scan");
      hipLaunchKernelGGL(k_bscan_sum, dim3(R * cpr), dim3(kBlock), 0, cx->stream, d.blockcnt.as<u32>(), nb, cpr,
                         d.bchunk.as<u32>());
      hipLaunchKernelGGL(k_bscan_top, dim3(1), dim3(1024), 0, cx->stream, d.bchunk.as<u32>(), u32(R), cpr, dh->sync);
      hipLaunchKernelGGL(k_bscan_down, dim3(R * cpr), dim3(kBlock), 0, cx->stream, d.blockcnt.as<u32>(), nb, cpr,
                         d.bchunk.as<u32>());
      hipLaunchKernelGGL(k_bucket_scatter, dim3(nb), dim3(kBlock), 0, cx->stream, L.src, d.blockcnt.as<u32>(), nb,
                         d.skey.as<u64>(), d.sidx.as<u32>());
      hipLaunchKernelGGL(k_dist_pack, dim3(1), dim3(1), 0, cx->stream, cx->hdr.as<Header>(), L.ucount, L.bases, dh,
                         u32(R));
    }
    G_HIP(hipGetLastError());
    cx->prof_end(KID_DIST, eb);
  }
  {
    std::vector<const void*> s;
    std::vector<void*> r;
    for (gcz_ctx* cx : ctx) {
      s.push_back(cx->dist->dhdr.as<DistHdr>()->sync);
      r.push_back(cx->dist->gath.ptr);
    }
    hipEvent_t e0{};
    ctx[0]->prof_begin(KID_EXCHANGE, e0);
    G_RC(x_allgather(lv[0].leaves ? "leaf owner counts" : "owner counts", kSyncWords * 8, s, r));
    ctx[0]->prof_end(KID_EXCHANGE, e0);
  }
  gcz_dist_state& d0 = *ctx[0]->dist;
  G_HIP(hipMemcpyAsync(d0.h_gath, d0.gath.ptr, size_t(R) * kSyncWords * 8, hipMemcpyDeviceToHost, ctx[0]->stream));
  G_RC(host_sync());
  const u64* gv = d0.h_gath;
  std::vector<u64> M(size_t(R) * R), u(R);
  u64 records = 0;
  *ovf_bits = 0;
  *err_global = ~0ull;
  *err_sym = 0;
  for (int s = 0; s < R; ++s) {
    const u64* v = gv + size_t(s) * kSyncWords;
    for (int q = 0; q < R; ++q) { M[size_t(s) * R + q] = v[q]; records += v[q]; }
    *ovf_bits |= int(v[R]);
    u[s] = v[R + 1];
    if (v[R + 4]) any_predup = true;
    if (v[R + 2] != ~0ull) {
      const u64 g = v[R + 2] + plan.start(s, 0) * u64(info.L);   // local byte offset -> genome offset
      if (g < *err_global) { *err_global = g; *err_sym = int(v[R + 3]); }
    }
  }
  if (*ovf_bits) return kRetry;
  if (*err_global != ~0ull) return GCZ_ERR_SYMBOL;

  auto sent = [&](int r) { u64 t = 0; for (int q = 0; q < R; ++q) t += M[size_t(r) * R + q]; return t; };
  auto recvd = [&](int r) { u64 t = 0; for (int q = 0; q < R; ++q) t += M[size_t(q) * R + r]; return t; };
  auto blocks = [](u64 n) { return dim3(unsigned(std::max<u64>(1, (n + kBlock - 1) / kBlock))); };
  auto displ_of = [&](int r) {   // source segments of rank r's receive buffer
    Displ D{};
    u64 o = 0;
    for (int q = 0; q < R; ++q) { D.d[q] = o; o += M[size_t(q) * R + r]; }
    for (int q = R; q <= kMaxRanks; ++q) D.d[q] = o;
    return D;
  };
  std::vector<OwnTab> otab(NL);
  std::vector<LevelTab> opos(NL);
  std::vector<char> olisted(NL, 0);   // the owner dedupe listed its not-first records (k_own_getid_list)

  auto send_displ_of = [&](int r) {   // destination segments of rank r's send buffer
    Displ D{};
    u64 o = 0;
    for (int q = 0; q < R; ++q) { D.d[q] = o; o += M[size_t(r) * R + q]; }
    for (int q = R; q <= kMaxRanks; ++q) D.d[q] = o;
    return D;
  };
  auto tiles_of = [](u64 n) { return (n + kTile - 1) / kTile; };
  auto tiles = [&](u64 n) { return dim3(unsigned(std::max<u64>(1, tiles_of(n)))); };

  // 2. owners decide first rank, repetition and sharing (A, B)
  if (records) {
    std::vector<const void*> s;
    std::vector<void*> rv;
    for (int i = 0; i < NL; ++i) {
      gcz_ctx* cx = ctx[i];
      gcz_dist_state& d = *cx->dist;
      const u64 nr = recvd(rank[i]);
      int rc;
      if ((rc = cx->ensure(d.rkey, nr * 8 + 16)) || (rc = cx->ensure(d.oslot, nr * 4 + 16)) ||
          (rc = cx->ensure(d.rflag, nr + 32)) || (rc = cx->ensure(d.rcval, nr * 8 + 16)) ||
          (rc = cx->ensure(d.olist, nr * 4 + 16)) ||
          (rc = cx->ensure(d.rdval, nr * 8 + 16)))
        return dev_fail("exchange buffers");
      const u64 cap = std::max<u64>(256, next_pow2(2 * nr));
      // nolocal: the records in receive order are the level's occurrences in position order,
      // so the owner hash-conses them like a single-device level (position-packed table, the
      // receive index as position, not-first / multi marks): one CAS per new key, no reply pass
      opos[i] = nolocal ? plan_table(d.owntab.ptr, cap, key_bits, std::max<u64>(nr, 2), child_bits,
                                     cx->allow_packed && !cx->force_wide, 0)
                        : LevelTab{};
      const bool packed = opos[i].packed || (key_bits + u32(R) + 2 <= 64 && !cx->force_wide);
      if ((rc = cx->ensure(d.owntab, cap * (packed ? 8 : 16)))) return dev_fail("owner table");
      opos[i].pt.tab = d.owntab.as<u64>();   // (re)allocated above
      if (packed && (rc = cx->ensure(d.oids, cap * 4))) return dev_fail("owner ids");
      if (opos[i].packed) {
        if ((rc = cx->ensure(d.omin, 2 * nr + 64))) return dev_fail("owner marks");
      } else if (nolocal && (rc = cx->ensure(d.omin, cap * 4))) {
        return dev_fail("owner first index");
      }
      otab[i] = OwnTab{};
      otab[i].tab = d.owntab.as<Slot>();
      otab[i].ptab = d.owntab.as<u64>();
      otab[i].ids = d.oids.as<u32>();
      otab[i].mask = u32(cap - 1);
      otab[i].packed = packed;
      otab[i].R = u32(R);
      otab[i].B = child_bits;
      otab[i].sh = u32(R) + 2;
      otab[i].nolocal = nolocal;
      otab[i].omin = nolocal ? d.omin.as<u32>() : nullptr;
      s.push_back(d.skey.ptr);
      rv.push_back(d.rkey.ptr);
    }
    {
      hipEvent_t e0{};
      ctx[0]->prof_begin(KID_EXCHANGE, e0);
      G_RC(x_alltoallv(lv[0].leaves ? "leaf keys to owners" : "keys to owners", M, false, 8, s, rv));
      ctx[0]->prof_end(KID_EXCHANGE, e0);
    }
    s.clear();
    rv.clear();
    for (int i = 0; i < NL; ++i) {
      gcz_ctx* cx = ctx[i];
      gcz_dist_state& d = *cx->dist;
      const u64 nr = recvd(rank[i]);
      ProfScope ps_(cx, KID_OWNER);
      // owner bucketed dedupe (no table): nolocal levels whose records pack into 8 bytes
      OwnBkt ob{};
      bool use_ob = false;
      if (opos[i].packed && owner_buckets && nr >= 2) {
        ob.T = opos[i].pt;
        ob.B = child_bits;
        ob.K = key_bits;
        ob.bb = 0;
        while (ob.bb < 12 && (nr >> ob.bb) > 4096) ++ob.bb;
        ob.nch = u32((nr + kDC - 1) / kDC);
        ob.nr = nr;
        use_ob = ob.K >= ob.bb && ob.K - ob.bb + kDLog <= 64 && ob.nch <= 8192;
      }
      // ... preferably as the single-device two-pass partition (whole-run writes)
      Bkt2Plan b2{};
      bool use_ob2 = false;
      if (use_ob && owner_two_pass) {
        u32 bb = 0;
        while (bb < u32(kBktMaxLog) && (nr >> bb) > 2560) ++bb;
        b2.T = opos[i].pt;
        b2.K = key_bits;
        b2.b1 = std::min<u32>(bb, kPartMaxB1);
        b2.b2 = bb - b2.b1;
        b2.G = (nr + kPartChunk - 1) / kPartChunk;
        const u64 mean_run = std::max<u64>(1, std::min<u64>(nr, kPartChunk) >> b2.b1);
        b2.SC = u32(std::max<u64>(1, std::min<u64>(128, u64(kFineCap / 2) / mean_run)));
        b2.SC = 1u << log2_exact(b2.SC);
        b2.P = kPartLog + log2_exact(b2.SC);
        b2.nslice = u32((b2.G + b2.SC - 1) / b2.SC);
        b2.olist = d.olist.as<u32>();
        b2.ocnt = &d.dhdr.as<DistHdr>()->lcnt[1];
        use_ob2 = key_bits >= bb && b2.b2 <= u32(kFineMaxB2) && key_bits - b2.b1 + kPartLog <= 64 &&
                  key_bits - bb + b2.P <= 64 && mean_run * b2.SC <= u64(kFineCap) / 2 && b2.nslice <= 512;
      }
      if (!use_ob)
        G_HIP(hipMemsetAsync(d.owntab.ptr, 0xff, size_t(otab[i].mask + 1) * (otab[i].packed ? 8 : 16), cx->stream));
      const Displ D = displ_of(rank[i]);
      if (opos[i].packed) {
        unsigned char* onf = d.omin.as<unsigned char>();
        unsigned char* omul = onf + nr + 32;
        if (!use_ob2) G_HIP(hipMemsetAsync(onf, 0, 2 * nr + 64, cx->stream));   // (ob2: k_ob_part zeroes the reply)
        if (use_ob2) {
          const u64 nfine = (u64(1) << b2.b1) * b2.nslice;
          if (cx->ensure(d.ob_seg, b2.G * kPartChunk * 8) || cx->ensure(d.ob_rt, b2.G * ((u64(1) << b2.b1) + 1) * 4 + 16) ||
              cx->ensure(d.ob_rec2, nfine * kFineCap * 8) || cx->ensure(d.ob_fo, nfine * ((u64(1) << b2.b2) + 1) * 4 + 16))
            return dev_fail("owner partition");
          G_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_ob_part),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, int(kPartChunk * 8)));
          G_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_bkt_fine),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, int(kFineCap * 8)));
          u32* ovf = &cx->hdr.as<Header>()->overflow;
          hipLaunchKernelGGL(k_ob_part, dim3(unsigned(b2.G)), dim3(kBktThreads), size_t(kPartChunk) * 8, cx->stream,
                             d.rkey.as<u64>(), nr, b2, child_bits, d.ob_seg.as<u64>(), d.ob_rt.as<u32>(),
                             d.rflag.as<unsigned char>());
          hipLaunchKernelGGL(k_bkt_fine, dim3(unsigned(nfine)), dim3(kBktThreads), size_t(kFineCap) * 8, cx->stream,
                             d.ob_seg.as<u64>(), d.ob_rt.as<u32>(), b2, d.ob_rec2.as<u64>(), d.ob_fo.as<u32>(),
                             static_cast<Header*>(nullptr), static_cast<const u64*>(nullptr), nr, ovf);
          olisted[i] = 1;
          hipLaunchKernelGGL(k_bkt_dedupe2<true>, dim3(unsigned(u64(1) << (b2.b1 + b2.b2))), dim3(kBktThreads), 0,
                             cx->stream, d.ob_rec2.as<u64>(), d.ob_fo.as<u32>(), b2, d.oslot.as<u32>(),
                             Marks{d.rflag.as<unsigned char>(), nullptr}, static_cast<Header*>(nullptr),
                             static_cast<const u64*>(nullptr), nr, ovf);
        } else if (use_ob) {
          const u64 ncnt = (u64(1) << ob.bb) * ob.nch, t = scan_tiles(ncnt + 1);
          if (cx->ensure(d.ob_cnt, ncnt * 4 + 16) || cx->ensure(d.ob_off, (ncnt + 1) * 4 + 16) ||
              cx->ensure(d.ob_desc, t * 8 + 64) || cx->ensure(d.ob_rec, nr * 8 + 16))
            return dev_fail("owner buckets");
          G_HIP(hipMemsetAsync(d.ob_desc.ptr, 0, t * 8 + 64, cx->stream));
          G_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_ob_dedupe),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, int((ob.nch + 1) * 4)));
          hipLaunchKernelGGL(k_ob_count, dim3(ob.nch), dim3(1024), 0, cx->stream, d.rkey.as<u64>(), ob,
                             d.ob_cnt.as<u32>());
          hipLaunchKernelGGL(k_scan_excl<ScanU32>, dim3(unsigned(t)), dim3(kScanThreads), 0, cx->stream,
                             ScanU32{d.ob_cnt.as<u32>(), ncnt}, ncnt + 1, d.ob_off.as<u32>(), d.ob_desc.as<u64>(),
                             reinterpret_cast<u32*>(d.ob_desc.as<u64>() + t), static_cast<u64*>(nullptr));
          hipLaunchKernelGGL(k_ob_scatter, dim3(ob.nch), dim3(1024), 0, cx->stream, d.rkey.as<u64>(), ob,
                             d.ob_off.as<u32>(), d.ob_rec.as<u64>());
          hipLaunchKernelGGL(k_ob_dedupe, dim3(1u << ob.bb), dim3(1024), (ob.nch + 1) * 4, cx->stream,
                             d.ob_rec.as<u64>(), d.ob_off.as<u32>(), ob, Marks{onf, omul}, d.oslot.as<u32>(),
                             &cx->hdr.as<Header>()->overflow);
        } else {
          hipLaunchKernelGGL(k_own_insert_pos, blocks(nr), dim3(kBlock), 0, cx->stream, d.rkey.as<u64>(), nr,
                             child_bits, opos[i].pt, Marks{onf, omul}, d.oslot.as<u32>(),
                             &cx->hdr.as<Header>()->overflow);
        }
        if (!use_ob2)
          hipLaunchKernelGGL(k_own_reply_marks, blocks(nr), dim3(kBlock), 0, cx->stream, onf, omul, nr,
                             d.rflag.as<unsigned char>());
      } else {
        if (nolocal) G_HIP(hipMemsetAsync(d.omin.ptr, 0xff, size_t(otab[i].mask + 1) * 4, cx->stream));
        hipLaunchKernelGGL(k_own_insert, blocks(nr), dim3(kBlock), 0, cx->stream, d.rkey.as<u64>(), nr, D, u32(R),
                           int(lv[i].leaves), otab[i], d.oslot.as<u32>(), &d.dhdr.as<DistHdr>()->final_vec[3]);
        hipLaunchKernelGGL(k_own_reply, blocks(nr), dim3(kBlock), 0, cx->stream, d.oslot.as<u32>(), nr, D, u32(R),
                           otab[i], d.rflag.as<unsigned char>());
        if (nolocal)
          hipLaunchKernelGGL(k_own_first, blocks(nr), dim3(kBlock), 0, cx->stream, d.oslot.as<u32>(), nr, otab[i],
                             d.rflag.as<unsigned char>());
      }
      G_HIP(hipGetLastError());
      s.push_back(d.rflag.ptr);
      rv.push_back(d.sflag.ptr);
    }
    {
      hipEvent_t e0{};
      ctx[0]->prof_begin(KID_EXCHANGE, e0);
      G_RC(x_alltoallv("owner replies", M, true, 1, s, rv));
      ctx[0]->prof_end(KID_EXCHANGE, e0);
    }
  }
  // 3. globally-first ranks in local order (straight into the rank's output slice);
  //    C / D record counts per owner
  for (int i = 0; i < NL; ++i) {
    gcz_ctx* cx = ctx[i];
    gcz_dist_state& d = *cx->dist;
    const u64 ur = u[rank[i]];
    DistHdr* dh = d.dhdr.as<DistHdr>();
    ProfScope ps_(cx, KID_IDS);
    if (!lv[i].keys_zeroed) {   // (k_node_keys zeroed them, and the rank scan's descriptors)
      G_HIP(hipMemsetAsync(d.gnf.ptr, 0, ur + 1, cx->stream));
      G_HIP(hipMemsetAsync(d.gmul.ptr, 0, ur + 1, cx->stream));
    }
    if (records) {
      const u64 ns = sent(rank[i]);
      if (cx->ensure(d.nfl, kNfListCap * 4 + 16)) return dev_fail("not-first list");
      hipLaunchKernelGGL(k_dist_flags, tiles(ns), dim3(kBlock), 0, cx->stream, d.sidx.as<u32>(), ns,
                         d.sflag.as<unsigned char>(), d.gnf.as<unsigned char>(), d.gmul.as<unsigned char>(),
                         send_displ_of(rank[i]), u32(R), &dh->sync2[1], d.clist.as<u32>(), &dh->lcnt[0],
                         d.nfl.as<u32>(), &dh->nnf);
      if (lookahead && nwords[i] > 0)
        hipLaunchKernelGGL(k_lookahead, blocks((nwords[i] + 1) / 2), dim3(kBlock), 0, cx->stream,
                           d.gmul.as<unsigned char>(), nwords[i], &dh->sync2[1 + 2 * R]);
      G_HIP(hipGetLastError());
    }
    const u64 tiles = std::max<u64>(1, tiles_of(ur));
    if (!lv[i].keys_zeroed) G_HIP(hipMemsetAsync(d.ddesc.ptr, 0, tiles * 8, cx->stream));
    // (records crossed ranks: k_dist_flags listed the positions not globally first; sparse
    // lists rank without the look-back chain)
    const u32* nfl = records ? d.nfl.as<u32>() : nullptr;
    if (lv[i].leaves)
      hipLaunchKernelGGL((k_dist_rank<u64>), dim3(unsigned(tiles)), dim3(kBlock), 0, cx->stream,
                         d.gnf.as<unsigned char>(), lv[i].ucount, d.gid.as<u32>(), d.ddesc.as<u64>(), &dh->ticket,
                         &dh->sync2[0], d.scratch.as<u64>(), static_cast<u64*>(lv[i].out), nfl,
                         static_cast<const u32*>(&dh->nnf));
    else
      hipLaunchKernelGGL((k_dist_rank<uint2>), dim3(unsigned(tiles)), dim3(kBlock), 0, cx->stream,
                         d.gnf.as<unsigned char>(), lv[i].ucount, d.gid.as<u32>(), d.ddesc.as<u64>(), &dh->ticket,
                         &dh->sync2[0], d.scratch.as<uint2>(), static_cast<uint2*>(lv[i].out), nfl,
                         static_cast<const u32*>(&dh->nnf));
    G_HIP(hipGetLastError());
  }
  c.assign(R, 0);
  std::vector<u64> MC(size_t(R) * R, 0), MD(size_t(R) * R, 0);
  u64 nc = 0, nd = 0;
  if (records) {
    const size_t W = 2 + 2 * size_t(R);
    std::vector<const void*> s;
    std::vector<void*> rv;
    for (gcz_ctx* cx : ctx) {
      s.push_back(cx->dist->dhdr.as<DistHdr>()->sync2);
      rv.push_back(cx->dist->gath2.ptr);
    }
    {
      hipEvent_t e0{};
      ctx[0]->prof_begin(KID_EXCHANGE, e0);
      G_RC(x_allgather("first counts + C/D sizes", W * 8, s, rv));
      ctx[0]->prof_end(KID_EXCHANGE, e0);
    }
    G_HIP(hipMemcpyAsync(d0.h_gath2, d0.gath2.ptr, size_t(R) * W * 8, hipMemcpyDeviceToHost, ctx[0]->stream));
    G_RC(host_sync());
    for (int s2 = 0; s2 < R; ++s2) {
      const u64* v = d0.h_gath2 + size_t(s2) * W;
      c[s2] = v[0];
      if (lookahead) next_hashed += v[1 + 2 * R];
      for (int q = 0; q < R; ++q) {
        MC[size_t(s2) * R + q] = v[1 + q];
        MD[size_t(s2) * R + q] = v[1 + R + q];
        nc += v[1 + q];
        nd += v[1 + R + q];
      }
    }
    if (lookahead && next_hashed_out) *next_hashed_out = next_hashed;
  } else {
    c = u;   // nothing crossed ranks: every local first is globally first
  }
  off.assign(R + 1, 0);
  for (int s2 = 0; s2 < R; ++s2) off[s2 + 1] = off[s2] + c[s2];
  total = off[R];
  if (total > u64(kIdx)) return fail(GCZ_ERR_CAPACITY, "more than 2^29-1 uniques in one layer");
  // 4. ids of keys held by several ranks or occurrences: C (first holder -> owner), D (owner ->
  //    the others), as (segment index, id) pairs placed at the A layout's segment starts
  std::vector<u64> SA(size_t(R) * R), RA(size_t(R) * R);
  for (int s2 = 0; s2 < R; ++s2)
    for (int q = 0; q < R; ++q) {
      SA[size_t(s2) * R + q] = send_displ(M, R, false, s2, q);
      RA[size_t(q) * R + s2] = recv_displ(M, R, false, q, s2);
    }
  auto counts_from = [&](const std::vector<u64>& X, int r, bool as_dest) {   // per peer, as a Displ
    Displ C{};
    for (int q = 0; q < R; ++q) C.d[q] = as_dest ? X[size_t(q) * R + r] : X[size_t(r) * R + q];
    return C;
  };
  if (nc) {
    std::vector<const void*> s;
    std::vector<void*> rv;
    for (int i = 0; i < NL; ++i) {
      gcz_ctx* cx = ctx[i];
      gcz_dist_state& d = *cx->dist;
      ProfScope ps_(cx, KID_IDS);
      u64 nci = 0;   // this rank's C records (k_dist_flags' list)
      for (int q = 0; q < R; ++q) nci += MC[size_t(rank[i]) * R + q];
      if (nci)
        hipLaunchKernelGGL(k_dist_cvals, blocks(nci), dim3(kBlock), 0, cx->stream, d.clist.as<u32>(), nci,
                           d.sidx.as<u32>(), send_displ_of(rank[i]), u32(R), d.gid.as<u32>(), u32(off[rank[i]]),
                           d.dhdr.as<DistHdr>()->ccur, d.scval.as<u64>());
      G_HIP(hipGetLastError());
      s.push_back(d.scval.ptr);
      rv.push_back(d.rcval.ptr);
    }
    {
      hipEvent_t e0{};
      ctx[0]->prof_begin(KID_EXCHANGE, e0);
      G_RC(x_alltoallv_at("C ids to owners", MC, false, 8, SA, RA, s, rv));
      ctx[0]->prof_end(KID_EXCHANGE, e0);
    }
    for (int i = 0; i < NL; ++i) {
      gcz_ctx* cx = ctx[i];
      gcz_dist_state& d = *cx->dist;
      ProfScope ps_(cx, KID_OWNER);
      u64 nco = 0;   // C records for this owner
      for (int q = 0; q < R; ++q) nco += MC[size_t(q) * R + rank[i]];
      if (nco)
        hipLaunchKernelGGL(k_own_setid, blocks(nco), dim3(kBlock), 0, cx->stream, d.rcval.as<u64>(), nco,
                           displ_of(rank[i]), counts_from(MC, rank[i], true), u32(R), d.oslot.as<u32>(), otab[i]);
      G_HIP(hipGetLastError());
    }
  }
  if (nd) {
    std::vector<const void*> s;
    std::vector<void*> rv;
    for (int i = 0; i < NL; ++i) {
      gcz_ctx* cx = ctx[i];
      gcz_dist_state& d = *cx->dist;
      const u64 nr = recvd(rank[i]);
      ProfScope ps_(cx, KID_OWNER);
      u64 ndo = 0;   // D records from this owner
      for (int q = 0; q < R; ++q) ndo += MD[size_t(q) * R + rank[i]];
      if (olisted[i]) {
        if (ndo)
          hipLaunchKernelGGL(k_own_getid_list, blocks(ndo), dim3(kBlock), 0, cx->stream, d.olist.as<u32>(), ndo,
                             d.oslot.as<u32>(), displ_of(rank[i]), u32(R), otab[i], d.dhdr.as<DistHdr>()->dcur,
                             d.rdval.as<u64>());
      } else {
        hipLaunchKernelGGL(k_own_getid, tiles(nr), dim3(kBlock), 0, cx->stream, d.oslot.as<u32>(), nr,
                           displ_of(rank[i]), u32(R), d.rflag.as<unsigned char>(), otab[i],
                           d.dhdr.as<DistHdr>()->dcur, d.rdval.as<u64>());
      }
      G_HIP(hipGetLastError());
      s.push_back(d.rdval.ptr);
      rv.push_back(d.sdval.ptr);
    }
    {
      hipEvent_t e0{};
      ctx[0]->prof_begin(KID_EXCHANGE, e0);
      G_RC(x_alltoallv_at("D ids to holders", MD, true, 8, RA, SA, s, rv));
      ctx[0]->prof_end(KID_EXCHANGE, e0);
    }
    for (int i = 0; i < NL; ++i) {
      gcz_ctx* cx = ctx[i];
      gcz_dist_state& d = *cx->dist;
      ProfScope ps_(cx, KID_IDS);
      u64 ndi = 0;   // D records for this rank
      for (int q = 0; q < R; ++q) ndi += MD[size_t(rank[i]) * R + q];
      if (ndi)
        hipLaunchKernelGGL(k_dist_dvals, blocks(ndi), dim3(kBlock), 0, cx->stream, d.sidx.as<u32>(), ndi,
                           send_displ_of(rank[i]), counts_from(MD, rank[i], false), u32(R), d.sdval.as<u64>(),
                           d.gid.as<u32>());
      G_HIP(hipGetLastError());
    }
  }
  // 5. local words -> global ids
  leaf_deferred = lv[0].leaves && lv[0].defer_remap && (dist_local == 2 || (dist_local == 0 && !any_predup)) &&
                  total != plan.nk[0];
  if (lv[0].leaves) {
    leaf_gmark.assign(NL, nullptr);
    leaf_identity.assign(NL, false);
    for (int i = 0; i < NL; ++i) {
      leaf_gmark[i] = lv[i].gmark;
      leaf_identity[i] = lv[i].identity;
    }
  }
  remap_off.assign(NL, 0);
  for (int i = 0; i < NL; ++i) remap_off[i] = u32(off[rank[i]]);
  for (int i = 0; i < NL; ++i) {
    if (leaf_deferred || lv[i].identity) continue;   // rank 0's leaf ids are already global
    if (!lv[i].leaves && defer_node_remap) continue;   // (the caller remaps: remap_level / direct levels)
    gcz_ctx* cx = ctx[i];
    gcz_dist_state& d = *cx->dist;
    const u64 nw = nwords[i];
    ProfScope ps_(cx, KID_REMAP);
    hipLaunchKernelGGL(k_dist_remap, blocks(nw), dim3(kBlock), 0, cx->stream, lv[i].w, nw, lv[i].nf, lv[i].multi,
                       d.gid.as<u32>(), d.gmul.as<unsigned char>(), u32(off[rank[i]]), lv[i].gmark);
    G_HIP(hipGetLastError());
  }
  return GCZ_OK;
}

// ---- the fused leaf + layer-0 schedule (gcz_dist_fast.h) -----------------------------------

namespace {
// The owner's two-pass dedupe of nr received layer-0 records with K-bit keys (exchange()'s
// k_ob_part / k_bkt_fine / k_bkt_dedupe2<true> path); false: the records do not fit it.
// Records per owner region of the fused schedule's send buffer (k_fl_scatter): the mean p / R
// plus 16 standard deviations of the binomial count (hashed owners) and a margin; a region that
// overflows all the same sends the attempt to the general schedule (status bit 4).
u64 fl_cap(u64 p, int R) {
  const double m = double(p) / double(R);
  // GCZ_FL_CAP_PERMILLE (tests): regions of that fraction of the mean, so that they overflow
  if (const char* e = std::getenv("GCZ_FL_CAP_PERMILLE"))
    if (const int pm = std::atoi(e); pm > 0) return std::max<u64>(1, u64(m * pm / 1000.0));
  return u64(m + 16.0 * std::sqrt(m) + 1024.0);
}

bool owner_two_pass_plan(u64 nr, u32 K, Bkt2Plan& b2) {
  u32 obb = 0;   // (exchange()'s single-pass precondition holds too)
  while (obb < 12 && (nr >> obb) > 4096) ++obb;
  const u64 nch = (nr + kDC - 1) / kDC;
  if (nr < 2 || K < obb || K - obb + kDLog > 64 || nch > 8192) return false;
  u32 bb = 0;
  while (bb < u32(kBktMaxLog) && (nr >> bb) > 2560) ++bb;
  b2 = Bkt2Plan{};
  b2.K = K;
  b2.b1 = std::min<u32>(bb, kPartMaxB1);
  b2.b2 = bb - b2.b1;
  b2.G = (nr + kPartChunk - 1) / kPartChunk;
  const u64 mean_run = std::max<u64>(1, std::min<u64>(nr, kPartChunk) >> b2.b1);
  b2.SC = u32(std::max<u64>(1, std::min<u64>(128, u64(kFineCap / 2) / mean_run)));
  b2.SC = 1u << log2_exact(b2.SC);
  b2.P = kPartLog + log2_exact(b2.SC);
  b2.nslice = u32((b2.G + b2.SC - 1) / b2.SC);
  return K >= bb && b2.b2 <= u32(kFineMaxB2) && K - b2.b1 + kPartLog <= 64 && K - bb + b2.P <= 64 &&
         mean_run * b2.SC <= u64(kFineCap) / 2 && b2.nslice <= 512;
}

Transport::XOp xop_a2a(const std::vector<u64>& M, int R, bool rev, size_t elem, std::vector<const void*> send,
                       std::vector<void*> recv) {
  Transport::XOp o;
  o.M = M;
  o.rev = rev;
  o.elem = elem;
  o.sd.assign(size_t(R) * R, 0);
  o.rd.assign(size_t(R) * R, 0);
  for (int s = 0; s < R; ++s)
    for (int d = 0; d < R; ++d) {
      o.sd[size_t(s) * R + d] = send_displ(M, R, rev, s, d);
      o.rd[size_t(d) * R + s] = recv_displ(M, R, rev, d, s);
    }
  o.send = std::move(send);
  o.recv = std::move(recv);
  return o;
}
// every rank's `n` elements to every rank, concatenated in rank order
Transport::XOp xop_allgather(int R, u64 n, size_t elem, std::vector<const void*> send, std::vector<void*> recv) {
  Transport::XOp o;
  o.M.assign(size_t(R) * R, n);
  o.elem = elem;
  o.sd.assign(size_t(R) * R, 0);
  o.rd.assign(size_t(R) * R, 0);
  for (int d = 0; d < R; ++d)
    for (int s = 0; s < R; ++s) o.rd[size_t(d) * R + s] = u64(s) * n;
  o.send = std::move(send);
  o.recv = std::move(recv);
  return o;
}
// segment d (of `seg` elements) of every rank's buffer to rank d, landing at segment s
Transport::XOp xop_fixed(int R, u64 seg, size_t elem, std::vector<const void*> send, std::vector<void*> recv) {
  Transport::XOp o;
  o.M.assign(size_t(R) * R, seg);
  o.elem = elem;
  o.sd.assign(size_t(R) * R, 0);
  o.rd.assign(size_t(R) * R, 0);
  for (int s = 0; s < R; ++s)
    for (int d = 0; d < R; ++d) {
      o.sd[size_t(s) * R + d] = u64(d) * seg;
      o.rd[size_t(d) * R + s] = u64(s) * seg;
    }
  o.send = std::move(send);
  o.recv = std::move(recv);
  return o;
}
}  // namespace

// The host waits for one event (the build goes on queued behind it); every collective enqueued
// before it has completed then, so the watchdog is disarmed.
int gcz_group::event_sync(hipEvent_t e) {
  const hipError_t rc = hipEventSynchronize(e);
  if (watch && watch->fired) return fail(GCZ_ERR_DEVICE, watch->msg);
  if (rc != hipSuccess) return dev_fail("hipEventSynchronize");
  if (watch) watch->disarm();
  return GCZ_OK;
}

int gcz_group::build_fast(const std::vector<const unsigned char*>& bases, const u64* const* d_leaves, int L,
                          const std::vector<u64>& leaf_cap, bool* taken) {
  *taken = false;
  const int R = world, NL = int(ctx.size());
  const DistPlan& P = plan;
  const int G = P.G, D = P.D;
  // applicable: several ranks of one node (k_fl_scatter's owner fields) with distributed levels to spare (G >= 2; the general schedule
  // gathers a small hash-consed layer 0 to rank 0 instead -- here its exchange rides in the leaf
  // level's collective groups, so it stays distributed), every rank with pairs of its own, the
  // dense leaf level's codes
  if (!fast_mode || R < 2 || R > kFlMaxRanks || L > 12 || G < 2 || dense_mode == 0) return GCZ_OK;
  for (int s = 0; s < R; ++s)
    if (P.count(s, 1) < 2) return GCZ_OK;
  const u64 ncodes = u64(1) << dense_code_bits(u32(L)), nw = (ncodes + 63) / 64;
  // Layer-0 records: R a power of two -> 6 bytes (PreKey: canonical-code ranks, the owner in
  // the mixed key's top bits); else the raw canonical pair in hashed-code labels, 8 bytes
  const u32 lgR = (R & (R - 1)) == 0 ? log2_exact(u64(R)) : 0u;
  const bool split = lgR > 0;
  const u32 Bc = 2 * u32(L) - 1;   // (a canonical code's top bit is 0: PreKey)
  const u32 child_bits = 2 * u32(L);  // (8-byte records: hashed code labels; the null pair is not exchanged)
  const u32 key_bits = split ? 2 * Bc + 3 - lgR : 2 * (child_bits + 2);
  if (split && key_bits > 48) return GCZ_OK;
  FlPairs& pairs = fl_pairs;
  pairs = FlPairs{};
  for (int s = 0; s < R; ++s) pairs.p[s] = P.count(s, 1);
  std::vector<LeafLevel> las(NL);
  std::vector<u64> dcur(NL, 0);
  // fixed capacities of the leaf relay's pieces (a list holds at most min(strands, canonical
  // 2-bit codes) entries: dna::canonical orbits, Burnside over {id, transpose, mirror, inversion})
  u64 ncanon = (u64(1) << (2 * L)) + (u64(1) << (2 * ((L + 1) / 2)));
  if (L % 2 == 0) ncanon += u64(1) << L;
  ncanon /= 4;
  u64 smax = 0;
  for (int s = 0; s < R; ++s) smax = std::max(smax, P.count(s, 0));
  const u64 cap1 = std::min(smax, ncanon) / u64(R) + 2, cap2 = std::min(P.S, ncanon) / u64(R) + u64(R) + 2;
  const u32 NB0 = u32(std::min<u64>(kDNBMax, ncodes));
  const u64 xw = (u64(NB0) + 2 + 1) & ~u64(1);
  const u32 syncw = u32(R) + 6;   // R1a's vector: owner counts, overflow, uniques, symbol, .., predup, non-ACGT
  // ---- C1 (+ C2, C3 queued before the mid-build read): the dense pack; layer 0's keys from the
  // pre-words counted per owner; R1a; the keys scattered by owner; the dense sort and presence
  for (int i = 0; i < NL; ++i) {
    gcz_ctx* cx = ctx[i];
    const int r = rank[i];
    if (int rc = alloc(i, leaf_cap[i])) return rc == GCZ_ERR_DEVICE ? dev_fail("allocation") : rc;
    gcz_dist_state& d = *cx->dist;
    if (!cx->ev_start) {
      G_HIP(hipEventCreate(&cx->ev_start));
      G_HIP(hipEventCreate(&cx->ev_stop));
    }
    G_HIP(hipEventRecord(cx->ev_start, cx->stream));
    // the build's zeroed state in one launch: the header and look-back descriptors, the schedule's
    // header, K2's look-back words and the C / D slots (their sizes are the plan's)
    const u64 p = P.count(r, 1);
    const u32 nb = u32(std::max<u64>(1, (p + kTile - 1) / kTile));
    const size_t cd = (size_t(R) * kFlSeg * 8 + 15) & ~size_t(15), fd = (u64(nb) * R * 8 + 64 + 15) & ~u64(15);
    if (cx->ensure(d.fl_desc, fd) || cx->ensure(d.scval, cd) || cx->ensure(d.rdval, cd))
      return dev_fail("fused schedule buffers");
    InitPlan ip{};
    ip.hdr = cx->hdr.as<Header>();
    ip.desc = cx->desc.as<uint4>();
    ip.ndesc16 = cx->desc.bytes / 16;
    ip.zero[0] = d.dhdr.as<uint4>();
    ip.nzero16[0] = kDistHdrBytes / 16;
    ip.zero[1] = d.fl_desc.as<uint4>();
    ip.nzero16[1] = fd / 16;
    ip.zero[2] = d.scval.as<uint4>();
    ip.nzero16[2] = cd / 16;
    ip.zero[3] = d.rdval.as<uint4>();
    ip.nzero16[3] = cd / 16;
    const u64 big = std::max<u64>({ip.ndesc16, ip.nzero16[1], ip.nzero16[2]});
    hipLaunchKernelGGL(k_build_init, dim3(unsigned(std::min<u64>(1024, std::max<u64>(1, (big + kBlock - 1) / kBlock)))),
                       dim3(kBlock), 0, cx->stream, ip);
    G_HIP(hipGetLastError());
    Header* h = cx->hdr.as<Header>();
    LeafLevel& la = las[i];
    la.bases = bases[i];
    la.leaves = d_leaves ? d_leaves[i] : nullptr;
    la.S = P.count(r, 0);
    la.L = L;
    la.words = cx->wa.as<u32>();
    if (cx->ensure(cx->dl_seg, size_t(64 + 3 * R) * 8 + 64) || cx->ensure(cx->dl_pb, (nw + 4) * 8) ||
        cx->ensure(cx->dl_pbs, size_t(R) * nw * 8 + 16))
      return dev_fail("dense leaf buffers");
    bool used = false;
    cx->probe_ranks = unsigned(R);
    const int rc = cx->dense_phase_a(la, h, &h->count[0], false, true, &used, cx->dl_pb.as<u64>() + nw, true);
    cx->probe_ranks = 1;
    if (rc) return rc == GCZ_ERR_DEVICE ? dev_fail("dense leaves") : rc;
    if (!used) return GCZ_OK;   // (sizes outside the dense level: the same on every rank)
    const u64 n = la.S;
    RecSrc& rs = fl_rs[i];
    rs = RecSrc{};
    rs.pre = cx->dl_pw.as<u32>();
    rs.n = n;
    rs.p = p;
    rs.R = u32(R);
    const u64 cap = fl_cap(p, R);
    if (split) {
      const DensePlan& DP = cx->dl_plan;
      const LevelTab mt = plan_table(nullptr, 256, 2 * Bc + 3, 2, Bc, true, 0);   // (its mix only)
      rs.pk.on = 1;
      rs.pk.Kinv = DP.Kinv;
      rs.pk.cmask = DP.hmask;
      rs.pk.Bc = Bc;
      rs.pk.K = 2 * Bc + 3;
      rs.pk.lgR = lgR;
      rs.pk.sh = mt.pt.sh;
      rs.pk.kmask = mt.pt.kmask;
      rs.pk.c1 = mt.pt.c1;
      rs.pk.c2 = mt.pt.c2;
      if (cx->ensure(d.skey_hi, u64(R) * cap * 2 + 16)) return dev_fail("fused schedule buffers");
    }
    // the send buffer: R regions of cap records; the look-back descriptors and their ticket
    if (cx->ensure(d.skey, u64(R) * cap * 8 + 16) || cx->ensure(d.sidx, u64(R) * cap * 4 + 16))
      return dev_fail("fused schedule buffers");
  }
  fl_mark("C1");
  for (int i = 0; i < NL; ++i) {   // C2: the keys scattered by owner (K2's input), the owner totals
    gcz_ctx* cx = ctx[i];
    gcz_dist_state& d = *cx->dist;
    const u64 p = P.count(rank[i], 1);
    const u32 nb = u32(std::max<u64>(1, (p + kTile - 1) / kTile));
    FlScatter a{};
    a.skey = d.skey.as<u64>();
    a.sidx = d.sidx.as<u32>();
    a.skey_hi = split ? d.skey_hi.as<unsigned short>() : nullptr;
    a.cap = fl_cap(p, R);
    a.desc = d.fl_desc.as<u64>();
    a.nb = nb;
    a.tot = d.dhdr.as<DistHdr>()->sync;
    a.h = cx->hdr.as<Header>();
    a.gnf = d.gnf.as<unsigned char>();
    a.gmul = d.gmul.as<unsigned char>();
    a.ddesc = d.ddesc.as<u64>();
    a.count_out = &cx->hdr.as<Header>()->count[kLayerSlot];
    a.spin_cap = fl_spin_cap;
    ProfScope ps_(cx, KID_DIST);
    hipLaunchKernelGGL(k_fl_scatter, dim3(std::min<u32>(nb, kFsGrid)), dim3(kFsThreads), 0, cx->stream, fl_rs[i], a);
    G_HIP(hipGetLastError());
  }
  fl_mark("C2");
  G_RC(bulk_mark());   // (K2 waits for the keys only, not for R1a or C3)
  // ---- R1a: status words + owner totals; the host reads them while C3 runs
  {
    std::vector<const void*> s;
    std::vector<void*> rv;
    for (gcz_ctx* cx : ctx) {
      s.push_back(cx->dist->dhdr.as<DistHdr>()->sync);
      rv.push_back(cx->dist->gath.ptr);
    }
    hipEvent_t e0{};
    ctx[0]->prof_begin(KID_EXCHANGE, e0);
    G_RC(x_allgather("R1a status + layer-0 owner counts", size_t(syncw) * 8, s, rv));
    ctx[0]->prof_end(KID_EXCHANGE, e0);
    gcz_dist_state& d0 = *ctx[0]->dist;
    if (!ev_mid) G_HIP(hipEventCreateWithFlags(&ev_mid, hipEventDisableTiming));
    G_HIP(hipMemcpyAsync(d0.h_gath, d0.gath.ptr, size_t(R) * syncw * 8, hipMemcpyDeviceToHost, ctx[0]->stream));
    G_HIP(hipEventRecord(ev_mid, ctx[0]->stream));
  }
  for (int i = 0; i < NL; ++i) {   // C3: the dense sort, first positions and the presence bitmap
    ctx[i]->dl_plan.gate = cx_hdr(i);   // (skipped on the device when the pack found repetitive data)
    int rc = ctx[i]->dense_phase_a2(las[i]);
    // (rank 0 first-holds every code it holds: its r-first lists come from this pass, before
    // the bitmaps' exchange, where it has slack; the other ranks' from k_dl_rfirst after it)
    if (!rc && rank[i] == 0)
      rc = ctx[i]->ensure(ctx[i]->dl_lh, ncodes * 4 + 16) || ctx[i]->ensure(ctx[i]->dl_pos, (u64(NB0) + xw) * 4 + 64)
               ? GCZ_ERR_DEVICE
               : 0;
    if (!rc)
      rc = ctx[i]->dense_phase_a3(cx_hdr(i), nullptr, true, ctx[i]->dl_pb.as<u64>() + nw,
                                  rank[i] == 0 ? ctx[i]->dl_lh.as<u32>() : nullptr,
                                  rank[i] == 0 ? ctx[i]->dl_pos.as<u32>() : nullptr);
    ctx[i]->dl_plan.gate = nullptr;
    if (rc) return rc == GCZ_ERR_DEVICE ? dev_fail("dense leaves") : rc;
  }
  fl_mark("C3");
  // ---- the mid-build read: the path, the keys' all-to-all sizes
  G_RC(event_sync(ev_mid));
  std::vector<u64> M(size_t(R) * R);
  {
    const u64* gv = ctx[0]->dist->h_gath;
    u64 st = 0;
    for (int s = 0; s < R; ++s) {
      const u64* v = gv + size_t(s) * syncw;
      st |= v[R] | v[R + 4] | v[R + 5];   // an overflow, repetitive data, a strand that is not pure ACGT
      for (int q = 0; q < R; ++q) M[size_t(s) * R + q] = v[q];
    }
    if (st) return GCZ_OK;   // every rank decides alike from the same words: the general schedule
  }
  auto recvd = [&](int r) { u64 t = 0; for (int q = 0; q < R; ++q) t += M[size_t(q) * R + r]; return t; };
  // every rank decides for every owner from the gathered counts: an owner whose records do not
  // take the two-pass dedupe or whose key table would not pack sends EVERY rank to the general
  // schedule together (a rank that failed alone would leave its peers waiting in K2)
  std::vector<Bkt2Plan> b2(R);
  for (int s = 0; s < R; ++s) {
    const u64 nr = recvd(s);
    if (!owner_two_pass_plan(nr, key_bits, b2[s])) return GCZ_OK;
    if (!plan_table(nullptr, std::max<u64>(256, next_pow2(2 * nr)), key_bits, std::max<u64>(nr, 2), child_bits, true, 0)
             .packed)
      return GCZ_OK;
  }
  auto displ_recv = [&](int r) {   // source segments of owner r's receive buffer
    Displ Dd{};
    u64 o = 0;
    for (int q = 0; q < R; ++q) { Dd.d[q] = o; o += M[size_t(q) * R + r]; }
    for (int q = R; q <= kMaxRanks; ++q) Dd.d[q] = o;
    return Dd;
  };
  // the replies packed 2 bits per record: ceil(count / 4) bytes per segment
  std::vector<u64> M4(size_t(R) * R);
  for (size_t q = 0; q < M4.size(); ++q) M4[q] = (M[q] + 3) / 4;
  auto displ4 = [&](int r, bool as_owner) {   // packed segments: owner r's per source / sender r's per owner
    Displ Dd{};
    u64 o = 0;
    for (int q = 0; q < R; ++q) { Dd.d[q] = o; o += as_owner ? M4[size_t(q) * R + r] : M4[size_t(r) * R + q]; }
    for (int q = R; q <= kMaxRanks; ++q) Dd.d[q] = o;
    return Dd;
  };
  // rank r's send buffer: owner q's records at [q cap_r, q cap_r + M[r][q]) (k_fl_scatter)
  auto displ_send = [&](int r) {
    Displ Dd{};
    const u64 cap = fl_cap(P.count(r, 1), R);
    for (int q = 0; q <= kMaxRanks; ++q) Dd.d[q] = u64(std::min(q, R)) * cap;
    return Dd;
  };
  auto displ_send_end = [&](int r) {
    Displ Dd{};
    const u64 cap = fl_cap(P.count(r, 1), R);
    for (int q = 0; q <= kMaxRanks; ++q) Dd.d[q] = q < R ? u64(q) * cap + M[size_t(r) * R + q] : u64(R) * cap;
    return Dd;
  };
  // owner-side tables and buffers
  std::vector<OwnTab> otab(NL);
  for (int i = 0; i < NL; ++i) {
    gcz_ctx* cx = ctx[i];
    gcz_dist_state& d = *cx->dist;
    const int r = rank[i];
    const u64 nr = recvd(r);
    const u64 cap = std::max<u64>(256, next_pow2(2 * nr));
    const LevelTab lt = plan_table(d.owntab.ptr, cap, key_bits, std::max<u64>(nr, 2), child_bits, true, 0);
    if (!lt.packed) return fail(GCZ_ERR_CAPACITY, "fused schedule: owner keys do not pack");   // (decided above for every owner)
    Bkt2Plan& bp = b2[r];
    bp.T = lt.pt;
    const u64 nfine = (u64(1) << bp.b1) * bp.nslice;
    const size_t cd = size_t(R) * kFlSeg * 8;
    if (cx->ensure(d.rkey, nr * 8 + 16) || cx->ensure(d.oslot, nr * 4 + 16) || cx->ensure(d.rflag, nr + 32) ||
        cx->ensure(d.olist, nr * 4 + 16) || cx->ensure(d.owntab, cap * 8) || cx->ensure(d.oids, cap * 4) ||
        cx->ensure(d.ob_seg, bp.G * kPartChunk * 8) || cx->ensure(d.ob_rt, bp.G * ((u64(1) << bp.b1) + 1) * 4 + 16) ||
        cx->ensure(d.ob_rec2, nfine * kFineCap * 8) || cx->ensure(d.ob_fo, nfine * ((u64(1) << bp.b2) + 1) * 4 + 16) ||
        cx->ensure(d.scval, cd) || cx->ensure(d.rcval, cd) || cx->ensure(d.rdval, cd) || cx->ensure(d.sdval, cd) ||
        cx->ensure(d.fl_g3, size_t(R) * kMaxRanks * 8 + 16) || cx->ensure(d.fl_g4, size_t(R) * 2 * 8 + 16) ||
        cx->ensure(d.nfl, kNfListCap * 4 + 16) || cx->ensure(d.omin, nr / 4 + u64(R) + 64) ||   // (packed replies)
        (split && cx->ensure(d.rkey_hi, nr * 2 + 16)) ||
        cx->ensure(cx->dl_stage, (2 * u64(R) * cap1 + cap2) * 4 + 16) || cx->ensure(cx->dl_recv, u64(R) * cap2 * 4 + 16) ||
        cx->ensure(cx->dl_gid, sizeof(DlRelay) + 16) || cx->ensure(d.fl_cntb, u64(R) * NB0 * 4 + 16) ||
        cx->ensure(cx->dl_lower, u64(R) * xw * 4 + 16) || cx->ensure(cx->dl_lh, ncodes * 4 + 16) ||
        cx->ensure(cx->dl_list, std::min<u64>(P.count(r, 0), ncodes) * 4 + 16) ||
        cx->ensure(cx->dl_pos, (u64(NB0) + xw) * 4 + 64))
      return dev_fail("fused schedule buffers");
    bp.T.tab = d.owntab.as<u64>();
    bp.olist = d.olist.as<u32>();
    bp.ocnt = &d.dhdr.as<DistHdr>()->lcnt[1];
    OwnTab& ot = otab[i];
    ot = OwnTab{};
    ot.tab = d.owntab.as<Slot>();
    ot.ptab = d.owntab.as<u64>();
    ot.ids = d.oids.as<u32>();
    ot.mask = u32(cap - 1);
    ot.packed = 1;
    ot.R = u32(R);
    ot.B = child_bits;
    ot.sh = u32(R) + 2;
    ot.nolocal = 1;
    // (the C / D slot counts and records, scval and rdval, were zeroed by C1's k_build_init)
  }
  // ---- K2: layer-0 keys to their owners, a bulk group beside the build's stream
  {
    std::vector<const void*> sk, sh;
    std::vector<void*> rk, rh;
    for (gcz_ctx* cx : ctx) {
      sk.push_back(cx->dist->skey.ptr);
      rk.push_back(cx->dist->rkey.ptr);
      sh.push_back(cx->dist->skey_hi.ptr);
      rh.push_back(cx->dist->rkey_hi.ptr);
    }
    std::vector<Transport::XOp> ops;
    // (sources send from their owner regions, owners receive back to back in source order)
    auto gapped = [&](size_t elem, const std::vector<const void*>& snd, const std::vector<void*>& rcv) {
      Transport::XOp o = xop_a2a(M, R, false, elem, snd, rcv);
      for (int s2 = 0; s2 < R; ++s2)
        for (int q = 0; q < R; ++q) o.sd[size_t(s2) * R + q] = displ_send(s2).d[q];
      return o;
    };
    if (split) {   // 6-byte records: low 32 bits | high 16 bits
      ops.push_back(gapped(4, sk, rk));
      ops.push_back(gapped(2, sh, rh));
    } else {
      ops.push_back(gapped(8, sk, rk));
    }
    hipEvent_t e0{};
    ctx[0]->prof_begin(KID_EXCHANGE, e0);
    G_RC(x_group_bulk("K2 [bulk] layer-0 keys to owners", "K2 [bulk, second stream] layer-0 keys to owners", ops));
    ctx[0]->prof_end(KID_EXCHANGE, e0);
  }
  // ---- R1b: the presence bitmaps
  {
    std::vector<const void*> s;
    std::vector<void*> rv;
    for (gcz_ctx* cx : ctx) {
      s.push_back(cx->dl_pb.ptr);
      rv.push_back(cx->dl_pbs.ptr);
    }
    hipEvent_t e0{};
    ctx[0]->prof_begin(KID_EXCHANGE, e0);
    G_RC(x_allgather("R1b leaf presence bitmaps", nw * 8, s, rv));
    ctx[0]->prof_end(KID_EXCHANGE, e0);
  }
  // ---- C4: every rank's r-first counts and bucket prefixes from the bitmaps, the relay table;
  // this rank's r-first codes, their position bitmap and local ranks, G in code order, relay 1 out
  const u32 RB = 1u << ctx[0]->dl_plan.IB;
  for (int i = 0; i < NL; ++i) {
    gcz_ctx* cx = ctx[i];
    gcz_dist_state& d = *cx->dist;
    const int r = rank[i];
    const DensePlan& DP = cx->dl_plan;
    Header* h = cx->hdr.as<Header>();
    DistHdr* dh = d.dhdr.as<DistHdr>();
    const u32 NB = DP.NB;
    const u64 nfb = (DP.S + 63) / 64, t = scan_tiles(nfb + 1);
    u32* bcnt = cx->dl_pos.as<u32>();
    u32* xv = bcnt + NB;   // (k_dl_gq's own exchange vector: unused by this schedule)
    const u64 t_cnt = scan_tiles(u64(NB) * DP.nch + 1);
    u64* desc = cx->dl_desc.as<u64>() + t_cnt;
    u32* ticket = reinterpret_cast<u32*>(desc + t) + 1;
    {
      ProfScope ps_(cx, KID_DL_FIRST);
      FlRelayOut fo{};
      fo.xvs = cx->dl_lower.as<u32>();
      fo.xw = xw;
      fo.me = u32(r);
      fo.cap2 = cap2;
      fo.T = cx->dl_gid.as<DlRelay>();
      fo.leaf = dh->fl_leaf;
      hipLaunchKernelGGL(k_fl_counts, dim3(NB), dim3(256), 0, cx->stream, cx->dl_pbs.as<unsigned long long>(), nw, R, DP,
                         d.fl_cntb.as<u32>());
      hipLaunchKernelGGL(k_fl_prefix_relay, dim3(1), dim3(kDThreads), 0, cx->stream,
                         static_cast<const u32*>(d.fl_cntb.as<u32>()), R, DP, fo);
      if (r > 0) {   // (rank 0's lists: k_dl_first, C3)
        G_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_dl_rfirst), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  int((DP.nch + 1) * 4)));
        hipLaunchKernelGGL(k_dl_rfirst, dim3(NB), dim3(kDThreads), (DP.nch + 1) * 4, cx->stream, cx->dl_fpg.as<u32>(), DP,
                           cx->dl_pbs.as<unsigned long long>(), nw, r, cx->dl_fl.as<u32>(), cx->dl_fo.as<u32>(),
                           cx->dl_lh.as<u32>(), bcnt);
      }
      hipLaunchKernelGGL(k_dl_fb, dim3(DP.nch), dim3(kDThreads), 0, cx->stream, cx->dl_fl.as<u32>(), cx->dl_fo.as<u32>(),
                         DP, cx->dl_fb.as<unsigned long long>());
      G_HIP(hipGetLastError());
    }
    {
      ProfScope ps_(cx, KID_DL_FBSCAN);
      hipLaunchKernelGGL(k_scan_excl<ScanPopc>, dim3(unsigned(t)), dim3(kScanThreads), 0, cx->stream,
                         ScanPopc{cx->dl_fb.as<unsigned long long>()}, nfb, cx->dl_wpre.as<u32>(), desc, ticket,
                         &h->count[0]);
      hipLaunchKernelGGL(k_dl_gq, dim3(NB), dim3(kDThreads), 0, cx->stream, cx->dl_lh.as<u32>(), bcnt, DP,
                         cx->dl_fb.as<unsigned long long>(), cx->dl_wpre.as<u32>(),
                         static_cast<const u64*>(&h->count[0]), cx->dl_list.as<u32>(), xv, cx->dl_pw.as<u32>(),
                         r > 0 ? cx->leaves_out.as<u64>() : nullptr,   // (k_fl_words_l0: rank 0's)
                         static_cast<const u64*>(cx->dl_pb.as<u64>() + nw));
      hipLaunchKernelGGL(k_fl_relay_out, dim3(2048), dim3(256), 0, cx->stream, static_cast<const u32*>(cx->dl_list.as<u32>()),
                         static_cast<const u64*>(dh->fl_leaf), u32(R), cap1, cx->dl_stage.as<u32>());
      G_HIP(hipGetLastError());
    }
  }
  fl_mark("C4");
  // ---- R2: leaf G arrays, relay 1 (fixed-capacity slots)
  {
    std::vector<const void*> s;
    std::vector<void*> rv;
    for (gcz_ctx* cx : ctx) {
      s.push_back(cx->dl_stage.ptr);
      rv.push_back(cx->dl_stage.as<u32>() + u64(R) * cap1);
    }
    hipEvent_t e0{};
    ctx[0]->prof_begin(KID_EXCHANGE, e0);
    G_RC(x_group("R2 leaf G arrays, relay 1", {xop_fixed(R, cap1, 4, s, rv)}));
    ctx[0]->prof_end(KID_EXCHANGE, e0);
  }
  // ---- C5 (after K2): owners hash-cons their records (first = lowest receive index: the
  // sources send in position order and arrive in rank order), count their not-first records per
  // source, pack the replies; relay 2 staged
  G_RC(bulk_done());
  for (int i = 0; i < NL; ++i) {
    gcz_ctx* cx = ctx[i];
    gcz_dist_state& d = *cx->dist;
    const int r = rank[i];
    const u64 nr = recvd(r);
    const Bkt2Plan& bp = b2[r];
    const u64 nfine = (u64(1) << bp.b1) * bp.nslice;
    u32* ovf = &cx->hdr.as<Header>()->overflow;
    DistHdr* dh = d.dhdr.as<DistHdr>();
    {
      ProfScope ps_(cx, KID_OWNER);
      G_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_ob_part), hipFuncAttributeMaxDynamicSharedMemorySize,
                                int(kPartChunk * 8)));
      G_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_bkt_fine), hipFuncAttributeMaxDynamicSharedMemorySize,
                                int(kFineCap * 8)));
      hipLaunchKernelGGL(k_ob_part, dim3(unsigned(bp.G)), dim3(kBktThreads), size_t(kPartChunk) * 8, cx->stream,
                         d.rkey.as<u64>(), nr, bp, child_bits, d.ob_seg.as<u64>(), d.ob_rt.as<u32>(),
                         d.rflag.as<unsigned char>(),
                         split ? static_cast<const unsigned short*>(d.rkey_hi.as<unsigned short>()) : nullptr);
      hipLaunchKernelGGL(k_bkt_fine, dim3(unsigned(nfine)), dim3(kBktThreads), size_t(kFineCap) * 8, cx->stream,
                         d.ob_seg.as<u64>(), d.ob_rt.as<u32>(), bp, d.ob_rec2.as<u64>(), d.ob_fo.as<u32>(),
                         static_cast<Header*>(nullptr), static_cast<const u64*>(nullptr), nr, ovf);
      // (the schedule takes non-repetitive data only: the bitmap dedupe, six buckets per CU in flight;
      // a bucket over its capacity sets the overflow word and every rank falls back)
      if (cx->dedupe_bm)
        hipLaunchKernelGGL(k_bkt_dedupe_bm<true>, dim3(unsigned(u64(1) << (bp.b1 + bp.b2))), dim3(kBmThreads), 0,
                           cx->stream, d.ob_rec2.as<u64>(), d.ob_fo.as<u32>(), bp, d.oslot.as<u32>(),
                           Marks{d.rflag.as<unsigned char>(), nullptr}, static_cast<Header*>(nullptr),
                           static_cast<const u64*>(nullptr), nr, ovf);
      else
        hipLaunchKernelGGL(k_bkt_dedupe2<true>, dim3(unsigned(u64(1) << (bp.b1 + bp.b2))), dim3(kBktThreads), 0,
                           cx->stream, d.ob_rec2.as<u64>(), d.ob_fo.as<u32>(), bp, d.oslot.as<u32>(),
                           Marks{d.rflag.as<unsigned char>(), nullptr}, static_cast<Header*>(nullptr),
                           static_cast<const u64*>(nullptr), nr, ovf);
      const Displ P4 = displ4(r, true);
      FlC5 c{};
      c.olist = d.olist.as<u32>();
      c.ocnt = &dh->lcnt[1];
      c.D = displ_recv(r);
      c.P4 = P4;
      c.onf = dh->fl_onf;
      c.rflag = d.rflag.as<unsigned char>();
      c.packed = d.omin.as<unsigned char>();
      c.npack = u32(std::max<u64>(1, (P4.d[R] + 255) / 256));
      c.got = cx->dl_stage.as<u32>() + u64(R) * cap1;
      c.xvs = cx->dl_lower.as<u32>();
      c.xw = xw;
      c.cap1 = cap1;
      c.me = u32(r);
      c.relay2 = cx->dl_stage.as<u32>() + 2 * u64(R) * cap1;
      hipLaunchKernelGGL(k_fl_c5, dim3(c.npack + 64 + 256), dim3(256), 0, cx->stream, c, u32(R));
      G_HIP(hipGetLastError());
    }
  }
  fl_mark("C5");
  // ---- R3: owner replies | leaf G arrays, relay 2 | the owners' not-first counts
  {
    std::vector<const void*> sf, sg, sn;
    std::vector<void*> rf, rg, rn;
    for (gcz_ctx* cx : ctx) {
      gcz_dist_state& d = *cx->dist;
      sf.push_back(d.omin.ptr);   // (the packed replies)
      rf.push_back(d.sflag.ptr);
      sg.push_back(cx->dl_stage.as<u32>() + 2 * u64(R) * cap1);
      rg.push_back(cx->dl_recv.ptr);
      sn.push_back(d.dhdr.as<DistHdr>()->fl_onf);
      rn.push_back(d.fl_g3.ptr);
    }
    hipEvent_t e0{};
    ctx[0]->prof_begin(KID_EXCHANGE, e0);
    G_RC(x_group("R3 owner replies | leaf G arrays, relay 2 | not-first counts",
                 {xop_a2a(M4, R, true, 1, sf, rf), xop_allgather(R, cap2, 4, sg, rg),
                  xop_allgather(R, u64(R), 8, sn, rn)}));
    ctx[0]->prof_end(KID_EXCHANGE, e0);
  }
  // ---- C6: senders: the replies -> global flags, look-ahead, local ranks of the globally-first
  // pairs, C records of the shared keys
  for (int i = 0; i < NL; ++i) {
    gcz_ctx* cx = ctx[i];
    gcz_dist_state& d = *cx->dist;
    const int r = rank[i];
    Header* h = cx->hdr.as<Header>();
    DistHdr* dh = d.dhdr.as<DistHdr>();
    const Displ SD = displ_send(r);
    const u64 ns = SD.d[R], p = P.count(r, 1);   // (the owner regions, gaps included)
    ProfScope ps_(cx, KID_IDS);
    auto tiles = [](u64 x) { return dim3(unsigned(std::max<u64>(1, (x + kTile - 1) / kTile))); };
    hipLaunchKernelGGL(k_dist_flags, tiles(ns), dim3(kBlock), 0, cx->stream, d.sidx.as<u32>(), ns,
                       d.sflag.as<unsigned char>(), d.gnf.as<unsigned char>(), d.gmul.as<unsigned char>(), SD, u32(R),
                       &dh->sync2[1], d.clist.as<u32>(), &dh->lcnt[0], d.nfl.as<u32>(), &dh->nnf,
                       static_cast<const unsigned char*>(d.sflag.as<unsigned char>()), displ4(r, false),
                       displ_send_end(r));
    hipLaunchKernelGGL(k_lookahead, dim3(unsigned(std::max<u64>(1, ((p + 1) / 2 + kBlock - 1) / kBlock))), dim3(kBlock), 0,
                       cx->stream, static_cast<const unsigned char*>(d.gmul.as<unsigned char>()), p, &dh->fl_r4[0]);
    hipLaunchKernelGGL((k_dist_rank<uint2>), tiles(p), dim3(kBlock), 0, cx->stream, d.gnf.as<unsigned char>(),
                       static_cast<const u64*>(&h->count[kLayerSlot]), d.gid.as<u32>(), d.ddesc.as<u64>(), &dh->ticket,
                       &dh->sync2[0], static_cast<const uint2*>(nullptr), static_cast<uint2*>(nullptr),
                       static_cast<const u32*>(d.nfl.as<u32>()), static_cast<const u32*>(&dh->nnf));
    // (R4's vector {look-ahead pairs, failure}: k_lookahead and a C slot overflow write it)
    hipLaunchKernelGGL(k_fl_cvals, dim3(16), dim3(256), 0, cx->stream, static_cast<const u32*>(d.clist.as<u32>()),
                       static_cast<const u32*>(&dh->lcnt[0]), static_cast<const u32*>(d.sidx.as<u32>()), SD, u32(R),
                       static_cast<const u32*>(d.gid.as<u32>()), static_cast<const u64*>(d.fl_g3.as<u64>()), pairs,
                       u32(r), d.scval.as<u64>(), dh->fl_r4);
    G_HIP(hipGetLastError());
  }
  fl_mark("C6");
  // ---- R4: C (first holders' ids to owners) | look-ahead + failures
  {
    std::vector<const void*> sc, sv;
    std::vector<void*> rc, rv;
    for (gcz_ctx* cx : ctx) {
      gcz_dist_state& d = *cx->dist;
      sc.push_back(d.scval.ptr);
      rc.push_back(d.rcval.ptr);
      sv.push_back(d.dhdr.as<DistHdr>()->fl_r4);
      rv.push_back(d.fl_g4.ptr);
    }
    hipEvent_t e0{};
    ctx[0]->prof_begin(KID_EXCHANGE, e0);
    G_RC(x_group("R4 C ids to owners | look-ahead + status",
                 {xop_fixed(R, kFlSeg, 8, sc, rc), xop_allgather(R, 2, 8, sv, rv)}));
    ctx[0]->prof_end(KID_EXCHANGE, e0);
  }
  // ---- C7: the leaf level's global ids (the relay has landed); owners: C -> D records
  for (int i = 0; i < NL; ++i) {
    gcz_ctx* cx = ctx[i];
    gcz_dist_state& d = *cx->dist;
    const int r = rank[i];
    const DensePlan& DP = cx->dl_plan;
    DistHdr* dh = d.dhdr.as<DistHdr>();
    {
      ProfScope ps_(cx, KID_DL_IDS);
      FlCd c{};
      c.rc = d.rcval.as<u64>();
      c.D = displ_recv(r);
      c.oslot = d.oslot.as<u32>();
      c.T = otab[i];
      c.olist = d.olist.as<u32>();
      c.ocnt = &dh->lcnt[1];
      c.dbuf = d.rdval.as<u64>();
      c.bad = &dh->fl_bad;
      G_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_fl_ids_cd), hipFuncAttributeMaxDynamicSharedMemorySize,
                                int(RB * 4)));
      hipLaunchKernelGGL(k_fl_ids_cd, dim3(DP.NB + 1), dim3(kDThreads), RB * 4, cx->stream, cx->dl_rec.as<u32>(),
                         cx->dl_off.as<u32>(), DP, cx->dl_pbs.as<unsigned long long>(), nw, cx->dl_lower.as<u32>(), xw,
                         static_cast<const u32*>(cx->dl_recv.as<u32>()), cx->dl_gid.as<DlRelay>(), R, r,
                         cx->dl_idrec.as<u32>(), c);
      G_HIP(hipGetLastError());
    }
  }
  fl_mark("C7");
  // ---- R5: D (owners forward the ids to the other holders)
  {
    std::vector<const void*> sd;
    std::vector<void*> rd;
    for (gcz_ctx* cx : ctx) {
      sd.push_back(cx->dist->rdval.ptr);
      rd.push_back(cx->dist->sdval.ptr);
    }
    hipEvent_t e0{};
    ctx[0]->prof_begin(KID_EXCHANGE, e0);
    G_RC(x_group("R5 D ids to holders", {xop_fixed(R, kFlSeg, 8, sd, rd)}));
    ctx[0]->prof_end(KID_EXCHANGE, e0);
  }
  // ---- C8: layer 0 with the global leaf ids, then the direct subtrees of levels 1 .. G-1
  // (guarded: they run only when layer 1 is direct everywhere and no rank failed)
  std::vector<u32*> cur_in(NL), cur_out(NL);
  for (int i = 0; i < NL; ++i) {
    gcz_ctx* cx = ctx[i];
    gcz_dist_state& d = *cx->dist;
    const int r = rank[i];
    DistHdr* dh = d.dhdr.as<DistHdr>();
    {   // the leaf words (global ids) into layer 0 in LDS, chunk by chunk; the rank's leaves
      ProfScope ps_(cx, KID_L0);
      const DensePlan& DP = cx->dl_plan;
      const int words_bytes = int((kDC + 2 * kDNBMax + 1 + 16 + kDC / 32 + kDC / 64) * 4);
      G_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_fl_words_l0), hipFuncAttributeMaxDynamicSharedMemorySize,
                                words_bytes));
      FlL0 a{};
      a.gnf = d.gnf.as<unsigned char>();
      a.gid = d.gid.as<u32>();
      a.gonf = d.fl_g3.as<u64>();
      a.g4 = d.fl_g4.as<u64>();
      a.pp = pairs;
      a.R = u32(R);
      a.me = u32(r);
      a.leaf = dh->fl_leaf;
      a.nodes = cx->nodes_out.as<uint2>() + node_base[i][0];
      a.words0 = cx->wb.as<u32>();
      a.guard = &dh->fl_guard;
      hipLaunchKernelGGL(k_fl_dpatch, dim3(unsigned((u64(R) * kFlCap + 255) / 256)), dim3(256), 0, cx->stream,
                         static_cast<const u64*>(d.sdval.as<u64>()), displ_send(r), u32(R),
                         static_cast<const u32*>(d.sidx.as<u32>()), d.gid.as<u32>(), &dh->fl_bad);
      hipLaunchKernelGGL(k_fl_words_l0, dim3(DP.nch), dim3(kDThreads), words_bytes, cx->stream, cx->dl_rec.as<u32>(),
                         cx->dl_idrec.as<u32>(), cx->dl_offt.as<u32>(), DP, cx->dl_fb.as<unsigned long long>(),
                         static_cast<const u32*>(cx->dl_pw.as<u32>()), cx->leaves_out.as<u64>(), a);
      G_HIP(hipGetLastError());
    }
    cur_in[i] = cx->wb.as<u32>();
    cur_out[i] = cx->wa.as<u32>();
  }
  slice_off.assign(D + 1, std::vector<u64>(R, 0));
  slice_cnt.assign(D + 1, std::vector<u64>(R, 0));
  for (int k = 1; k < G;) {
    const int nlev = std::min(kDirectLog, G - k);
    for (int i = 0; i < NL; ++i) {
      const int r = rank[i];
      if (P.count(r, k) == 0) continue;
      DirectPlan dp{};
      for (int q = 0; q <= nlev; ++q) dp.n[q] = P.count(r, k + q);
      for (int q = 0; q < nlev; ++q) {
        dp.layer_off[k + q] = node_base[i][k + q];
        dp.id_off[k + q] = u32(P.start(r, k + q + 1));
      }
      if (ctx[i]->direct_levels(cur_in[i], k, nlev, dp, cur_out[i], ctx[i]->hdr.as<Header>(), DirectRemap{},
                                &ctx[i]->dist->dhdr.as<DistHdr>()->fl_guard, 0))
        return dev_fail("direct levels");
    }
    for (int q = 0; q < nlev; ++q) {
      for (int s = 0; s < R; ++s) {
        slice_off[k + q + 1][s] = P.start(s, k + q + 1);
        slice_cnt[k + q + 1][s] = P.count(s, k + q + 1);
      }
      info.layer_size[k + q] = P.nk[k + q + 1];
    }
    for (int i = 0; i < NL; ++i) std::swap(cur_in[i], cur_out[i]);
    k += nlev;
  }
  fl_mark("C8");
  // ---- R6 / R7: the top on rank 0, the final vectors; any failure discards the attempt
  bool failed = false;
  G_RC(finish_top(G, true, P.nk[G], cur_in, dcur, true, &failed));
  if (failed) return GCZ_OK;   // (the general schedule rebuilds from scratch)
  const u64* gf = ctx[0]->dist->h_gathf;
  u64 l0 = 0, lv = 0;
  for (int s = 0; s < R; ++s) {
    slice_off[0][s] = lv;
    slice_cnt[0][s] = gf[size_t(s) * kFinalWords + 2];
    lv += slice_cnt[0][s];
    slice_off[1][s] = l0;
    slice_cnt[1][s] = gf[size_t(s) * kFinalWords + 3];
    l0 += slice_cnt[1][s];
  }
  if (lv > u64(kIdx)) return fail(GCZ_ERR_CAPACITY, "more than 2^29-1 unique leaves");
  info.layer_size[0] = l0;
  info.n_leaves = lv;
  info.leaf_path = 1;
  info.repetitive = 0;
  *taken = true;
  return GCZ_OK;
}

// The top of the tree (every build schedule): the words of level Gx gathered to rank 0, which
// runs the remaining levels (direct subtrees, hash-consed levels, the fused tail), then the
// final vectors allgathered and the one host sync of the build's end.  *failed: some rank's
// final vector flags a table overflow (general schedule: rebuild with wide tables) or, with fl
// (the fused schedule: its failure words in the vector), a failed attempt of that schedule.
int gcz_group::finish_top(int Gx, bool direct, u64 prev_total, const std::vector<u32*>& cur_in, std::vector<u64>& dcur,
                          bool fl, bool* failed) {
  const int R = world, NL = int(ctx.size());
  const DistPlan& P = plan;
  const int D = P.D;
  *failed = false;
  // ---- gather the last distributed level to rank 0, finish the top there ----
  {
    std::vector<u64> cnt(R);
    for (int s = 0; s < R; ++s) cnt[s] = P.count(s, Gx);
    std::vector<const void*> sv;
    void* recv0 = nullptr;
    for (int i = 0; i < NL; ++i) {
      sv.push_back(cur_in[i]);
      if (rank[i] == 0) recv0 = ctx[i]->dist->tail_in.ptr;
    }
    if (!recv0) recv0 = ctx[0]->dist->tail_in.ptr;   // not used off rank 0
    G_RC(x_gather0("top words to rank 0", cnt, 4, sv, recv0));
  }
  for (int i = 0; i < NL; ++i) {
    gcz_ctx* cx = ctx[i];
    Header* h = cx->hdr.as<Header>();
    DistHdr* dh = cx->dist->dhdr.as<DistHdr>();
    const bool tail = rank[i] == 0;
    if (tail) {
      u32* in = cx->dist->tail_in.as<u32>();
      u32* bufs[2] = {cx->wa.as<u32>(), cx->wb.as<u32>()};
      int nb = 0;
      u64 n = P.nk[Gx];
      hipLaunchKernelGGL(k_set_u64, dim3(1), dim3(1), 0, cx->stream, &dh->cell[Gx], direct ? n : ~0ull);
      u64 bound = prev_total;
      bool tail_done = false;
      for (int k = Gx; k < D; ++k) {
        if (n <= u64(kTailMaxN) && cx->use_tail) {   // the rest in one launch
          const u64* pc = k == Gx ? &dh->cell[Gx] : &h->count[kLayerSlot + k - 1];
          if (cx->tail_levels(in, n, pc, k, D, node_base[i], h)) return dev_fail("tail levels");
          tail_done = true;
          break;
        }
        if (direct) {   // host-known (every later level too): direct subtrees, ids = positions
          DirectPlan dp{};
          int nlev = 0;
          u64 m = n;
          dp.n[0] = n;
          while (nlev < kDirectLog && k + nlev < D && (m > u64(kTailMaxN) || !cx->use_tail)) {
            dp.layer_off[k + nlev] = node_base[i][k + nlev];
            m = P.nk[k + nlev + 1];
            dp.n[++nlev] = m;
          }
          if (cx->direct_levels(in, k, nlev, dp, bufs[nb], h)) return dev_fail("tail direct levels");
          in = bufs[nb];
          nb ^= 1;
          n = m;
          bound = m;
          k += nlev - 1;
          continue;
        }
        NodeLevel na;
        na.k = k;
        na.in = in;
        na.n = n;
        na.p = P.nk[k + 1];
        na.words = bufs[nb];
        na.out = cx->nodes_out.as<uint2>() + node_base[i][k];
        na.count = &h->count[kLayerSlot + k];
        na.bound = bound;
        na.prev_marks = k > Gx;
        na.pcount = k == Gx ? &dh->cell[Gx] : &h->count[kLayerSlot + k - 1];
        na.desc = cx->desc.as<u64>() + dcur[i];
        dcur[i] += (na.p + scan_tile(na.p) - 1) / scan_tile(na.p);
        na.ticket = &h->ticket[kLayerSlot + k];
        if (cx->node_level(na, h)) return dev_fail("tail level");
        in = bufs[nb];
        nb ^= 1;
        n = na.p;
        bound = na.p;
      }
      if (!tail_done) hipLaunchKernelGGL(k_root, dim3(1), dim3(1), 0, cx->stream, in, h);
    }
    if (fl)
      hipLaunchKernelGGL(k_fl_final, dim3(1), dim3(64), 0, cx->stream, h, dh, Gx, D, int(tail),
                         static_cast<const u32*>(&dh->fl_bad), static_cast<const u64*>(cx->dist->fl_g4.as<u64>()),
                         static_cast<const u64*>(cx->dist->fl_g3.as<u64>()), fl_pairs, u32(R), u32(rank[i]));
    else
      hipLaunchKernelGGL(k_dist_final, dim3(1), dim3(1), 0, cx->stream, h, dh, Gx, D, int(tail));
    G_HIP(hipGetLastError());
    G_HIP(hipEventRecord(cx->ev_stop, cx->stream));
  }
  {
    std::vector<const void*> s;
    std::vector<void*> rv;
    for (gcz_ctx* cx : ctx) {
      s.push_back(cx->dist->dhdr.as<DistHdr>()->final_vec);
      rv.push_back(cx->dist->gathf.ptr);
    }
    G_RC(x_allgather("final vectors", kFinalWords * 8, s, rv));
  }
  gcz_dist_state& d0 = *ctx[0]->dist;
  G_HIP(hipMemcpyAsync(d0.h_gathf, d0.gathf.ptr, size_t(R) * kFinalWords * 8, hipMemcpyDeviceToHost,
                       ctx[0]->stream));
  G_RC(host_sync());
  int fo = 0;
  for (int s = 0; s < R; ++s) fo |= int(d0.h_gathf[size_t(s) * kFinalWords]);
  if (fo) {
    *failed = true;
    return GCZ_OK;
  }
  const u64* f0 = d0.h_gathf;   // rank 0's vector
  info.root = u32(f0[1]);
  for (int k = Gx; k < D; ++k) {
    info.layer_size[k] = f0[4 + k];
    slice_off[k + 1][0] = 0;
    slice_cnt[k + 1][0] = f0[4 + k];
  }
  return GCZ_OK;
}

int gcz_group::build(const void* const* d_bases, const u64* const* d_leaves, u64 S, int L) {
  info = gcz_info{};
  info.L = L;
  info.status = GCZ_OK;
  last_error.clear();
  xlog.clear();
  t_build = std::chrono::steady_clock::now();
  const int R = world, NL = int(ctx.size());
  if (L < 1 || L > 16) return fail(GCZ_ERR_ARG, "leaf length L must be in 1..16");
  if (S == 0) return fail(GCZ_ERR_EMPTY, "fewer than L bases: nothing to build");
  if (R > kMaxRanks) return fail(GCZ_ERR_ARG, "at most 31 ranks");
  info.n_strands = S;
  plan.make(S, R);
  const DistPlan& P = plan;
  // Positions are rank-local (29-bit words, like the single-device build), so the
  // genome may exceed 2^29 strands as long as every rank's range fits; ids are global
  // and bounded per layer (checked per exchanged layer; a direct layer has nk[k+1] ids).
  for (int s = 0; s < R; ++s)
    if (P.count(s, 0) > u64(kIdx)) return fail(GCZ_ERR_CAPACITY, "more than 2^29-1 strands on one rank");
  if (P.nk.size() > 1 && P.nk[1] > u64(kIdx)) return fail(GCZ_ERR_CAPACITY, "more than 2^29-1 nodes in layer 0");
  const int G = P.G, D = P.D;
  if (D > GCZ_MAX_LAYERS) return fail(GCZ_ERR_CAPACITY, "too many layers");
  node_base.assign(NL, {});

  std::vector<u64> leaf_cap(NL);
  for (int i = 0; i < NL; ++i) {
    const u64 S_r = P.count(rank[i], 0);
    const u64 full = std::max<u64>(256, next_pow2(2 * S_r));
    leaf_cap[i] = S_r > (1ull << 22) ? std::min(full, u64(1) << 24) : full;   // (no state across builds)
  }
  allow_packed = true;
  for (gcz_ctx* cx : ctx) allow_packed = allow_packed && !cx->force_wide;

  // bases: 4-B aligned copies where needed (the leaf kernel stages with 4-B loads)
  std::vector<const unsigned char*> bases(NL, nullptr);
  for (int i = 0; d_bases && i < NL; ++i) {
    gcz_ctx* cx = ctx[i];
    const u64 nb = P.count(rank[i], 0) * u64(L);
    bases[i] = static_cast<const unsigned char*>(d_bases[i]);
    if (nb && (reinterpret_cast<uintptr_t>(d_bases[i]) & 3)) {
      if (cx->ensure(cx->input, nb + 16)) return dev_fail("realign buffer");
      G_HIP(hipMemcpyAsync(cx->input.ptr, d_bases[i], nb, hipMemcpyDeviceToDevice, cx->stream));
      bases[i] = cx->input.as<unsigned char>();
    }
  }

  // the fused leaf + layer-0 schedule where it applies (the general schedule below otherwise,
  // and after an attempt of it that some rank had to discard)
  {
    bool taken = false;
    G_RC(build_fast(bases, d_leaves, L, leaf_cap, &taken));
    if (taken) return build_done();
  }
  std::vector<RankLevel> lv(NL);
  for (int attempt = 0;; ++attempt) {
    if (attempt > 8) return fail(GCZ_ERR_CAPACITY, "hash table overflow persists");
    for (int i = 0; i < NL; ++i) {
      gcz_ctx* cx = ctx[i];
      cx->allow_packed = allow_packed;
      if (int rc = alloc(i, leaf_cap[i])) return rc == GCZ_ERR_DEVICE ? dev_fail("allocation") : rc;
      if (!cx->ev_start) {
        G_HIP(hipEventCreate(&cx->ev_start));
        G_HIP(hipEventCreate(&cx->ev_stop));
      }
      G_HIP(hipEventRecord(cx->ev_start, cx->stream));
      InitPlan ip{};   // header (err_offset = ~0) and the look-back descriptors, one launch
      ip.hdr = cx->hdr.as<Header>();
      ip.desc = cx->desc.as<uint4>();
      ip.ndesc16 = cx->desc.bytes / 16;
      hipLaunchKernelGGL(k_build_init, dim3(unsigned(std::min<u64>(1024, std::max<u64>(1, (ip.ndesc16 + kBlock - 1) / kBlock)))),
                         dim3(kBlock), 0, cx->stream, ip);
      G_HIP(hipGetLastError());
    }
    // per-rank descriptor cursors
    std::vector<u64> dcur(NL, 0);
    any_predup = false;

    std::vector<u64> c, off;
    u64 total = 0, err_global = 0;
    int err_sym = 0, ovf = 0;
    // ---- leaves: the dense level (pure ACGT, L <= 12) when every rank holds strands ----
    bool dense = false;
    if (dense_mode != 0 && L <= 12) {
      bool all = true;
      for (int s2 = 0; s2 < R; ++s2) all = all && P.count(s2, 0) > 0;
      if (all) G_RC(dense_leaves(bases, d_leaves, L, c, off, total, &dense));
    }
    if (dense) {
      leaf_deferred = false;
      leaf_identity.assign(NL, true);
      leaf_gmark.assign(NL, nullptr);
    }
    // ---- leaves ----
    // Leaf dictionary (bases input, R > 1).  Nothing precedes rank 0, so the first-occurrence
    // keys of its first c0 chunks carry their GLOBAL ids already.  Rank 0 runs those chunks,
    // the keys go to every rank (bcast0), and ranks > 0 seed their fresh leaf table with them
    // before their leaf level: their strands of dictionary keys take the final word from the
    // probe (kNfGlobal) and those keys never enter their local unique lists, so the leaf
    // exchange and the leaf-word translation shrink to the keys rank 0's prefix has not seen.
    // Rank 0 still sends all its keys to the owners, so any rank may go without seeding.
    const std::vector<u64> chunks0 = leaf_chunks(P.count(0, 0), leaf_first_log2);
    const int c0 = seed_chunks;
    const bool seeding = !dense && R > 1 && d_bases && c0 > 0 && int(chunks0.size()) - 1 > c0;
    std::vector<int> C(NL);
    std::vector<LeafLevel> las(NL);
    for (int i = 0; i < NL; ++i) {
      gcz_ctx* cx = ctx[i];
      Header* h = cx->hdr.as<Header>();
      const u64 S_r = P.count(rank[i], 0);
      LeafLevel& la = las[i];
      la.bases = bases[i];
      la.leaves = d_leaves ? d_leaves[i] : nullptr;
      la.S = S_r;
      la.L = L;
      la.cap = leaf_cap[i];
      la.adaptive = leaf_cap[i] < 2 * S_r;
      la.words = cx->wa.as<u32>();
      la.out = cx->dist->scratch.as<u64>();
      la.chunk_start = leaf_chunks(S_r, leaf_first_log2);
      C[i] = int(la.chunk_start.size()) - 1;
      for (int q = 0; q < C[i]; ++q) {
        la.desc_off.push_back(dcur[i]);
        const u64 len = la.chunk_start[q + 1] - la.chunk_start[q];
        dcur[i] += (len + scan_tile(len) - 1) / scan_tile(len);
      }
      la.desc = cx->desc.as<u64>();
      la.count = h->count;
      la.ticket = h->ticket;
      if (dense) continue;
      if (seeding) {   // every local id space must hold the dictionary's ids
        la.seed_n = P.count(0, 0) >= chunks0[c0] ? chunks0[c0] : 0;
        if (rank[i] != 0) continue;
        la.c_end = c0;
      }
      if (cx->leaf_level(la, h)) return dev_fail("leaf level");
    }
    if (seeding) {
      // the dictionary size (rank 0's uniques after c0 chunks), then the keys
      std::vector<const void*> sv;
      std::vector<void*> rv;
      for (int i = 0; i < NL; ++i) {
        gcz_ctx* cx = ctx[i];
        DistHdr* dh = cx->dist->dhdr.as<DistHdr>();
        if (rank[i] == 0)
          G_HIP(hipMemcpyAsync(&dh->sync[0], &cx->hdr.as<Header>()->count[c0 - 1], 8, hipMemcpyDeviceToDevice,
                               cx->stream));
        else
          G_HIP(hipMemsetAsync(&dh->sync[0], 0, 8, cx->stream));
        sv.push_back(&dh->sync[0]);
        rv.push_back(cx->dist->gath.ptr);
      }
      {
        hipEvent_t e0{};
        ctx[0]->prof_begin(KID_EXCHANGE, e0);
        G_RC(x_allgather("leaf dictionary size", 8, sv, rv));
        ctx[0]->prof_end(KID_EXCHANGE, e0);
      }
      gcz_dist_state& d0 = *ctx[0]->dist;
      G_HIP(hipMemcpyAsync(d0.h_gath, d0.gath.ptr, 8, hipMemcpyDeviceToHost, ctx[0]->stream));
      G_RC(host_sync());
      const u64 U = std::min<u64>(d0.h_gath[0], chunks0[c0]);
      std::vector<const void*> ks(NL, nullptr);
      std::vector<void*> kr(NL, nullptr);
      int i0 = -1;
      for (int i = 0; i < NL; ++i) {
        gcz_ctx* cx = ctx[i];
        if (cx->ensure(cx->dist->dict, U * 8 + 16)) return dev_fail("leaf dictionary");
        kr[i] = cx->dist->dict.ptr;
        if (rank[i] == 0) i0 = i;
      }
      // LocalTransport indexes by global rank (all ranks local); RCCL / shm by local slot 0
      if (NL == R) {
        ks[0] = ctx[i0]->dist->scratch.ptr;
      } else {
        ks[0] = i0 >= 0 ? ctx[i0]->dist->scratch.ptr : nullptr;
      }
      {
        hipEvent_t e0{};
        ctx[0]->prof_begin(KID_EXCHANGE, e0);
        G_RC(x_bcast0("leaf dictionary", U * 8, ks, kr));
        ctx[0]->prof_end(KID_EXCHANGE, e0);
      }
      for (int i = 0; i < NL; ++i) {
        LeafLevel& la = las[i];
        if (rank[i] == 0) {
          la.c_begin = c0;
          la.c_end = -1;
        } else {
          la.seed = ctx[i]->dist->dict.as<u64>();
          la.seed_n = U;
        }
        if (ctx[i]->leaf_level(la, ctx[i]->hdr.as<Header>())) return dev_fail("leaf level");
      }
    }
    for (int i = 0; i < NL && !dense; ++i) {
      gcz_ctx* cx = ctx[i];
      Header* h = cx->hdr.as<Header>();
      const u64 S_r = P.count(rank[i], 0);
      RankLevel& rl = lv[i];
      rl = RankLevel{};
      rl.src.leaves = cx->dist->scratch.as<u64>();
      rl.src.ucount = &h->count[C[i] - 1];
      rl.grid_elems = S_r;
      rl.ucount = &h->count[C[i] - 1];
      rl.w = cx->wa.as<u32>();
      rl.out = cx->leaves_out.ptr;
      rl.leaves = true;
      rl.bases = bases[i];
      rl.gmark = seeding ? cx->nf_set[0] : nullptr;
      rl.identity = rank[i] == 0;
    }
    // Without the local dedupe the leaf words are translated by layer 0's k_node_keys (one
    // pass instead of two), unless layer 0 turns out direct or is not distributed (exchange
    // decides once the leaf totals are known: leaf_deferred).
    for (int i = 0; i < NL; ++i) lv[i].defer_remap = P.Gh > 0;   // (layer 0 is distributed then)
    if (!dense) {
      std::vector<u64> nw(NL);
      for (int i = 0; i < NL; ++i) nw[i] = P.count(rank[i], 0);
      const int rc = exchange(lv, nw, d_leaves ? 64u : 4 * u32(L), 0, c, off, total, &err_global, &err_sym, &ovf);
      if (rc == kRetry) {   // every rank sees the same bits and takes the same decision
        if (ovf & 2) {
          for (int i = 0; i < NL; ++i)
            leaf_cap[i] = std::min(std::max<u64>(256, next_pow2(2 * P.count(rank[i], 0))), leaf_cap[i] * 8);
          if (attempt >= 1) allow_packed = false;
        }
        if (ovf & 1) allow_packed = false;
        continue;
      }
      if (rc == GCZ_ERR_SYMBOL) {
        info.error_offset = err_global;
        info.error_symbol = err_sym;
        for (gcz_ctx* cx : ctx) { cx->info.error_offset = err_global; cx->info.error_symbol = err_sym; }
        return fail(GCZ_ERR_SYMBOL, "unknown nucleotide symbol");
      }
      if (rc) return rc;
    }
    slice_off.assign(D + 1, std::vector<u64>(R, 0));
    slice_cnt.assign(D + 1, std::vector<u64>(R, 0));
    for (int s = 0; s < R; ++s) { slice_off[0][s] = off[s]; slice_cnt[0][s] = c[s]; }
    leaf_offs.assign(NL, 0);
    for (int i = 0; i < NL; ++i) leaf_offs[i] = u32(off[rank[i]]);
    info.n_leaves = total;
    info.leaf_path = dense ? 1u : 0u;
    info.repetitive = any_predup ? 1u : 0u;
    // The repetitive-data decision is the OR over the ranks' probes (each sampled only a
    // prefix of its own slice): every rank's node levels take the same path from here.
    if (any_predup) {
      static const u32 one = 1;
      for (gcz_ctx* cx : ctx)
        G_HIP(hipMemcpyAsync(&cx->hdr.as<Header>()->predup, &one, 4, hipMemcpyHostToDevice, cx->stream));
    }

    // ---- distributed node levels ----
    // Without repetitive data the local dedupe of a node level finds almost nothing and
    // only doubles the hashing: the pairs go straight to their owners.
    const bool nolocal = dist_local == 2 || (dist_local == 0 && !any_predup);
    u64 prev_total = total;        // uniques of the previous level (child id bound)
    bool direct = total == P.nk[0];
    bool retry = false;
    std::vector<u32*> cur_in(NL), cur_out(NL);
    for (int i = 0; i < NL; ++i) { cur_in[i] = ctx[i]->wa.as<u32>(); cur_out[i] = ctx[i]->wb.as<u32>(); }
    int Gx = G;   // the level whose input is gathered to rank 0
    bool remap_pending = false;   // the last exchanged level's words still hold local ids
    for (int k = 0; k < G && !retry; ++k) {
      if (!direct && k >= P.Gh) {   // a small hash-consed level: rank 0 finishes from here
        Gx = k;
        break;
      }
      if (direct) {   // host-known: direct subtrees, up to kDirectLog levels per launch, no exchange
        const int nlev = std::min(kDirectLog, G - k);
        for (int i = 0; i < NL; ++i) {
          const int r = rank[i];
          if (P.count(r, k) == 0) continue;
          DirectPlan dp{};
          for (int q = 0; q <= nlev; ++q) dp.n[q] = P.count(r, k + q);
          for (int q = 0; q < nlev; ++q) {
            dp.layer_off[k + q] = node_base[i][k + q];
            dp.id_off[k + q] = u32(P.start(r, k + q + 1));
          }
          DirectRemap rm{};
          if (remap_pending) rm = DirectRemap{ctx[i]->dist->gid.as<u32>(), remap_off[i]};
          if (ctx[i]->direct_levels(cur_in[i], k, nlev, dp, cur_out[i], ctx[i]->hdr.as<Header>(), rm))
            return dev_fail("direct levels");
        }
        remap_pending = false;
        for (int q = 0; q < nlev; ++q) {
          for (int s = 0; s < R; ++s) {
            slice_off[k + q + 1][s] = P.start(s, k + q + 1);
            slice_cnt[k + q + 1][s] = P.count(s, k + q + 1);
          }
          info.layer_size[k + q] = P.nk[k + q + 1];
        }
        prev_total = P.nk[k + nlev];
        for (int i = 0; i < NL; ++i) std::swap(cur_in[i], cur_out[i]);
        k += nlev - 1;
        continue;
      }
      for (int i = 0; i < NL; ++i) {
        gcz_ctx* cx = ctx[i];
        Header* h = cx->hdr.as<Header>();
        DistHdr* dh = cx->dist->dhdr.as<DistHdr>();
        const int r = rank[i];
        const u64 n = P.count(r, k), p = P.count(r, k + 1);
        if (!(nolocal && !direct))   // (only node_level reads the cell: k_node_keys levels need none)
          hipLaunchKernelGGL(k_set_u64, dim3(1), dim3(1), 0, cx->stream, &dh->cell[k], direct ? n : ~0ull);
        NodeLevel na;
        na.k = k;
        na.in = cur_in[i];
        na.n = n;
        na.p = p;
        na.words = cur_out[i];
        na.out = direct ? cx->nodes_out.as<uint2>() + node_base[i][k] : cx->dist->scratch.as<uint2>();
        na.count = &h->count[kLayerSlot + k];
        na.bound = prev_total;
        na.prev_marks = k > 0;
        na.pcount = &dh->cell[k];
        na.id_off = u32(P.start(r, k + 1));
        na.direct_known = direct;
        na.desc = cx->desc.as<u64>() + dcur[i];
        dcur[i] += (p + scan_tile(p) - 1) / scan_tile(p);
        na.ticket = &h->ticket[kLayerSlot + k];
        if (!(nolocal && !direct) && cx->node_level(na, h)) return dev_fail("node level");
        RankLevel& rl = lv[i];
        rl = RankLevel{};
        rl.src.in = cur_in[i];
        rl.src.n = n;
        rl.src.p = p;
        rl.src.words = cur_out[i];
        const int cs = (k + 1) & 1, ps = k & 1;
        rl.src.nf = cx->nf_set[cs];
        rl.src.multi = cx->multi_set[cs];
        rl.src.prev_nf = k > 0 ? cx->nf_set[ps] : nullptr;
        rl.src.prev_multi = k > 0 ? cx->multi_set[ps] : nullptr;
        rl.src.canon = nolocal && !direct ? cx->dist->scratch.as<uint2>() : nullptr;
        rl.grid_elems = p;
        rl.ucount = &h->count[kLayerSlot + k];
        rl.w = cur_out[i];
        rl.nf = cx->nf_set[cs];
        rl.multi = cx->multi_set[cs];
        rl.out = cx->nodes_out.as<uint2>() + node_base[i][k];
        if (nolocal && !direct) {   // the pairs go straight to their owners; keys + tile counts in one pass
          rl.src.R = u32(R);
          rl.counted = true;
          const u32 nb = u32(std::max<u64>(1, (p + kTile - 1) / kTile));
          const bool tr = k == 0 && leaf_deferred && !leaf_identity[i];
          ProfScope ps_(cx, KID_NODE);
          hipLaunchKernelGGL(k_node_keys, dim3(nb), dim3(kBlock), 0, cx->stream, cur_in[i], n, p, cur_out[i],
                             cx->dist->scratch.as<uint2>(), cx->nf_set[cs], cx->multi_set[cs], na.count,
                             tr ? cx->dist->gid.as<u32>() : nullptr, tr ? leaf_offs[i] : 0u, rl.src,
                             cx->dist->blockcnt.as<u32>(), nb, tr ? leaf_gmark[i] : nullptr,
                             cx->dist->gnf.as<unsigned char>(), cx->dist->gmul.as<unsigned char>(),
                             cx->dist->ddesc.as<u64>());
          rl.keys_zeroed = true;
          G_HIP(hipGetLastError());
        }
      }
      if (direct) {
        for (int s = 0; s < R; ++s) { slice_off[k + 1][s] = P.start(s, k + 1); slice_cnt[k + 1][s] = P.count(s, k + 1); }
        info.layer_size[k] = P.nk[k + 1];
        prev_total = P.nk[k + 1];
      } else {
        std::vector<u64> nw(NL);
        for (int i = 0; i < NL; ++i) nw[i] = P.count(rank[i], k + 1);
        const u32 cb = std::max<u32>(1, bit_width(prev_total));
        u64 next_hashed = ~0ull;
        defer_node_remap = true;
        const int rc = exchange(lv, nw, 2 * (cb + 2), cb, c, off, total, &err_global, &err_sym, &ovf, nolocal,
                                nolocal && k + 1 < G, &next_hashed);
        defer_node_remap = false;
        if (rc == kRetry) {
          allow_packed = false;
          retry = true;
          break;
        }
        if (rc) return rc;
        for (int s = 0; s < R; ++s) { slice_off[k + 1][s] = off[s]; slice_cnt[k + 1][s] = c[s]; }
        info.layer_size[k] = total;
        // all unique, or (look-ahead) every pair of the next level holds a singleton
        direct = total == P.nk[k + 1] || next_hashed == 0;
        prev_total = total;
        // the level's words to global ids: on the next direct subtrees' load, else a pass
        if (direct && k + 1 < G) remap_pending = true;
        else if (int rc2 = remap_level(lv, nw)) return rc2;
      }
      for (int i = 0; i < NL; ++i) std::swap(cur_in[i], cur_out[i]);
    }
    if (retry) continue;

    // ---- gather the last distributed level to rank 0, finish the top there ----
    bool fo = false;
    G_RC(finish_top(Gx, direct, prev_total, cur_in, dcur, false, &fo));
    if (fo) {
      allow_packed = false;
      continue;
    }
    break;
  }
  return build_done();
}

// The summary of a finished build (any schedule) into the group's and every context's info.
int gcz_group::build_done() {
  info.n_layers = plan.D;
  double ms = 0;
  for (gcz_ctx* cx : ctx) {
    float t = 0.f;
    if (hipEventElapsedTime(&t, cx->ev_start, cx->ev_stop) == hipSuccess) ms = std::max(ms, double(t));
  }
  info.build_ms = ms;
  for (gcz_ctx* cx : ctx) {
    cx->info = info;
    cx->info.status = GCZ_OK;
    if (cx->profile) cx->prof_collect();
  }
  return GCZ_OK;
}

// The whole tree in dst's arrays in the single-device layout (gcz_ctx::build: layer k at
// layer_off[k], ceil(n_k / 2) slots; leaves first), so dst's device sort, .dag writer,
// decompression and host fetch run on it as on a one-GPU build (reference: sort_tree / bytes /
// serialize, src/shared_tree.cpp:443-513).  Every layer is the rank-ordered concatenation of
// the rank slices: all ranks local -> device copies; one rank per process -> one gather to
// rank 0 per layer over the transport (dst: rank 0's context, a different one from the
// group's; unused on the other ranks).
int gcz_group::assemble(gcz_ctx* dst) {
  const int R = world, NL = int(ctx.size());
  const bool here = NL == R;   // every rank local
  int i0 = -1;
  for (int i = 0; i < NL; ++i)
    if (rank[i] == 0) i0 = i;
  const bool root = i0 >= 0;
  // (every rank has the same build status: the build's failures are decided collectively)
  if (info.status != GCZ_OK || slice_cnt.empty()) return fail(GCZ_ERR_ARG, "assemble: no finished build");
  const int D = info.n_layers;
  const u64 S = info.n_strands;
  std::vector<u64> loff(D + 1, 0);
  {
    u64 n = S;
    for (int k = 0; k < D; ++k) {
      const u64 p = (n + 1) / 2;
      loff[k + 1] = loff[k] + p;
      n = p;
    }
  }
  hipStream_t st = ctx[0]->stream;
  // rank 0's destination (a context, its arrays) is settled before any gather, and with one rank
  // per process every rank learns the outcome from one status allgather first: a rank 0 that
  // cannot take the tree fails the call on every rank instead of leaving the others blocked in
  // a gather it never joins
  int root_rc = GCZ_OK;
  std::string root_why;
  if (root) {
    if (!dst) {
      root_rc = GCZ_ERR_ARG;
      root_why = "assemble: rank 0 needs a destination context";
    } else if (dst->ensure(dst->leaves_out, S * 8 + 16) || dst->ensure(dst->nodes_out, loff[D] * 8 + 16)) {
      root_rc = GCZ_ERR_DEVICE;
      root_why = "assemble: destination arrays";
    } else {
      dst->layer_off = loff;
      if (dst->stream != st && hipStreamSynchronize(dst->stream) != hipSuccess) {   // (its earlier work on the arrays)
        root_rc = GCZ_ERR_DEVICE;
        root_why = "assemble: destination stream";
      }
    }
  }
  if (!here) {
    gcz_dist_state& d0 = *ctx[0]->dist;
    u64* word = &d0.dhdr.as<DistHdr>()->final_vec[0];
    static_assert(kFinalWords >= 1, "status word");
    G_HIP(hipMemsetAsync(word, root_rc ? 0xff : 0, 8, st));
    G_RC(x_allgather("assemble status", 8, {word}, {d0.gath.ptr}));
    G_HIP(hipMemcpyAsync(d0.h_gath, d0.gath.ptr, size_t(R) * 8, hipMemcpyDeviceToHost, st));
    G_RC(host_sync());
    for (int r = 0; r < R; ++r)
      if (d0.h_gath[r]) return root_rc ? fail(root_rc, root_why) : fail(GCZ_ERR_DEVICE, "assemble: rank 0 cannot take the tree");
  } else if (root_rc) {
    return fail(root_rc, root_why);
  }
  for (int layer = -1; layer < D; ++layer) {
    auto src_of = [&](int i) -> const void* {
      return layer < 0 ? ctx[i]->leaves_out.ptr : static_cast<const void*>(ctx[i]->nodes_out.as<uint2>() + node_base[i][layer]);
    };
    char* out = !root ? nullptr
                      : layer < 0 ? reinterpret_cast<char*>(dst->leaves_out.as<u64>())
                                  : reinterpret_cast<char*>(dst->nodes_out.as<uint2>() + loff[layer]);
    if (here) {
      for (int i = 0; i < NL; ++i) {
        const u64 o = slice_off[layer + 1][rank[i]], n = slice_cnt[layer + 1][rank[i]];
        if (n) G_HIP(hipMemcpyAsync(out + o * 8, src_of(i), n * 8, hipMemcpyDeviceToDevice, st));
      }
    } else {
      std::vector<u64> cnt(R);
      for (int r = 0; r < R; ++r) cnt[r] = slice_cnt[layer + 1][r];
      G_RC(x_gather0(layer < 0 ? "leaves to rank 0" : "tree layer to rank 0", cnt, 8, {src_of(0)}, out));
    }
  }
  G_RC(host_sync());
  if (root) {
    dst->info = info;
    dst->info.status = GCZ_OK;
    dst->dense_used = info.leaf_path == 1;
    dst->last_error.clear();
  }
  return GCZ_OK;
}

extern "C" {

int gcz_group_assemble(gcz_group* g, gcz_ctx* dst) {
  if (!g) return GCZ_ERR_ARG;
  if (hipSetDevice(g->ctx[0]->device) != hipSuccess) return GCZ_ERR_DEVICE;
  return g->assemble(dst);
}

int gcz_dist_unique_id(void* out, uint64_t cap) {
  if (!out || cap < NCCL_UNIQUE_ID_BYTES) return GCZ_ERR_ARG;
  RcclApi& a = rccl();
  if (!a.ok) return GCZ_ERR_DEVICE;
  ncclUniqueId id;
  if (a.GetUniqueId(&id) != ncclSuccess) return GCZ_ERR_DEVICE;
  std::memcpy(out, &id, NCCL_UNIQUE_ID_BYTES);
  return GCZ_OK;
}

int gcz_group_create_local(int device, int world, gcz_group** out) {
  if (!out || world < 1 || world > kMaxRanks) return GCZ_ERR_ARG;
  *out = nullptr;
  auto* g = new gcz_group();
  g->world = world;
  g->owns_ctx = true;
  auto* t = new LocalTransport();
  t->world = world;
  g->tr = t;
  for (int r = 0; r < world; ++r) {
    gcz_ctx* c = nullptr;
    if (int rc = gcz_ctx_create(device, &c)) {
      gcz_group_destroy(g);
      return rc;
    }
    if (r > 0) c->stream = g->ctx[0]->stream;   // one stream: the copies order the ranks
    g->ctx.push_back(c);
    g->rank.push_back(r);
  }
  t->stream = g->ctx[0]->stream;
  if (const char* e = std::getenv("GCZ_LOCAL_BULK"); e && std::atoi(e) != 0 && world > 1)
    if (hipStreamCreateWithFlags(&t->stream2, hipStreamNonBlocking) != hipSuccess) {
      t->stream2 = nullptr;
      gcz_group_destroy(g);
      return GCZ_ERR_DEVICE;
    }
  *out = g;
  return GCZ_OK;
}

int gcz_group_create_rccl(gcz_ctx* ctx, int rank, int world, const void* unique_id, gcz_group** out) {
  if (!ctx || !out || !unique_id || world < 1 || world > kMaxRanks || rank < 0 || rank >= world) return GCZ_ERR_ARG;
  *out = nullptr;
  RcclApi& a = rccl();
  if (!a.ok) {
    ctx->last_error = "librccl.so.1 could not be loaded";
    return GCZ_ERR_DEVICE;
  }
  if (hipSetDevice(ctx->device) != hipSuccess) return GCZ_ERR_DEVICE;
  auto* t = new RcclTransport();
  t->world = world;
  t->me = rank;
  t->stream = ctx->stream;
  ncclUniqueId id;
  std::memcpy(&id, unique_id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t comm = nullptr;
  const ncclResult_t r = a.CommInitRank(&comm, world, id, rank);
  if (r != ncclSuccess) {
    ctx->last_error = std::string("ncclCommInitRank: ") + a.GetErrorString(r);
    delete t;
    return GCZ_ERR_DEVICE;
  }
  t->comm.store(comm);
  auto* g = new gcz_group();
  g->world = world;
  g->tr = t;
  g->ctx.push_back(ctx);
  g->rank.push_back(rank);
  g->watch.reset(new gcz_group::Watch(t, ctx->device, rank));
  // The bulk communicator and stream, agreed by every rank: ncclCommSplit is collective over
  // `comm`, so it runs only where every rank wants it (GCZ_FL_BULK=0 on any rank, or an RCCL
  // without the entry point: none splits), and comm2 is kept only where every rank got both the
  // communicator and the stream -- else every rank drops it and bulk groups run in line on `comm`
  // and the build's stream, the path the tests cover.  Both agreements are allgathers on `comm`
  // under the watchdog (a peer that never arrives aborts the communicator after
  // GCZ_DIST_TIMEOUT_S, and creation fails).  (Also at world 1, where no build uses it: the
  // one-GPU tests run the split, the agreement and the second stream on the real library.)
  {
    const char* eb = std::getenv("GCZ_FL_BULK");
    const int want = a.CommSplit && !(eb && std::atoi(eb) == 0) ? 1 : 0;
    int all_want = 0;
    int rc = g->agree("group creation: bulk communicator wanted", want, &all_want);
    ncclComm_t c2 = nullptr;
    int have = 0;
    if (!rc && all_want) {
      g->watch->begin(-1, "group creation: ncclCommSplit");
      if (a.CommSplit(comm, 0, rank, &c2, nullptr) == ncclSuccess && c2)
        have = hipStreamCreateWithFlags(&t->stream2, hipStreamNonBlocking) == hipSuccess ? 1 : 0;
      g->watch->disarm();
      int all_have = 0;
      rc = g->agree("group creation: bulk communicator ready", have, &all_have);
      if (!rc && all_have) {
        t->comm2.store(c2);
        c2 = nullptr;
      }
    }
    if (c2) (void)a.CommDestroy(c2);
    if (!t->comm2.load() && t->stream2) {
      (void)hipStreamDestroy(t->stream2);
      t->stream2 = nullptr;
    }
    if (rc || g->watch->fired) {
      ctx->last_error = "group creation: " + (g->last_error.empty() ? std::string("the bulk communicator agreement failed")
                                                                    : g->last_error);
      gcz_group_destroy(g);
      return GCZ_ERR_DEVICE;
    }
  }
  *out = g;
  return GCZ_OK;
}

int gcz_group_create_shm(gcz_ctx* ctx, int rank, int world, const char* name, uint64_t region_bytes,
                         gcz_group** out) {
  if (!ctx || !out || !name || world < 1 || world > kMaxRanks || rank < 0 || rank >= world || region_bytes == 0)
    return GCZ_ERR_ARG;
  *out = nullptr;
  const size_t cap = (region_bytes + 4095) / 4096 * 4096;
  const size_t bytes = 4096 + cap * size_t(world);
  // rank 0 creates and sizes a fresh object (a stale one of the same name is removed
  // first; a new object reads as zeros, so the control words start at 0); the others
  // wait for its size.  Names must be unique per job (bench.py derives them from the port).
  int fd = -1;
  if (rank == 0) {
    (void)shm_unlink(name);
    fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0 || ftruncate(fd, off_t(bytes)) != 0) {
      if (fd >= 0) close(fd);
      ctx->last_error = std::string("shm_open/ftruncate failed: ") + name;
      return GCZ_ERR_DEVICE;
    }
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      fd = shm_open(name, O_RDWR, 0600);
      struct stat st{};
      if (fd >= 0 && fstat(fd, &st) == 0 && size_t(st.st_size) == bytes) break;
      if (fd >= 0) close(fd);
      fd = -1;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) {
        ctx->last_error = std::string("shm transport: no region from rank 0: ") + name;
        return GCZ_ERR_DEVICE;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    ctx->last_error = "shm transport: mmap failed";
    return GCZ_ERR_DEVICE;
  }
  auto* t = new ShmTransport();
  t->world = world;
  t->me = rank;
  t->stream = ctx->stream;
  t->timeout_s = dist_timeout_s();
  t->cap = cap;
  t->map_bytes = bytes;
  t->base = static_cast<char*>(p);
  // every rank has mapped the region before anyone uses it (the control words start at 0)
  if (t->barrier() != GCZ_OK) {
    ctx->last_error = t->err;
    delete t;
    return GCZ_ERR_DEVICE;
  }
  if (rank == 0) shm_unlink(name);   // every rank holds its mapping: the name can go
  auto* g = new gcz_group();
  g->world = world;
  g->tr = t;
  g->ctx.push_back(ctx);
  g->rank.push_back(rank);
  *out = g;
  return GCZ_OK;
}

void gcz_group_destroy(gcz_group* g) {
  if (!g) return;
  if (g->watch && !g->watch->fired) g->watch->begin(-1, "teardown (collectives a failed build left queued)");
  for (gcz_ctx* c : g->ctx) (void)hipStreamSynchronize(c->stream);
  if (g->tr)   // (a bulk group a failed build left on the second stream, under the same watchdog)
    if (hipStream_t bs = g->tr->bulk_stream()) (void)hipStreamSynchronize(bs);
  g->watch.reset();
  for (hipEvent_t e : {g->ev_mid, g->ev_bulk_in, g->ev_bulk_out})   // (after the streams that wait on them)
    if (e) (void)hipEventDestroy(e);
  delete g->tr;
  if (g->owns_ctx) {
    // virtual ranks borrowed rank 0's stream (or, split builds, the parent context's)
    for (size_t i = 0; i < g->ctx.size(); ++i) g->ctx[i]->stream = g->ctx[i]->own_stream;
    for (gcz_ctx* c : g->ctx) gcz_ctx_destroy(c);
  }
  delete g;
}

int gcz_group_xlog(const gcz_group* g, int local, uint64_t* rec, const char** names, int cap) {
  if (!g || local < 0 || local >= int(g->ctx.size())) return -1;
  const int n = int(g->xlog.size());
  for (int i = 0; i < n && i < cap; ++i) {
    const gcz_group::XRec& x = g->xlog[size_t(i)];
    if (rec) {
      rec[4 * i] = u64(x.seq);
      rec[4 * i + 1] = x.sent[size_t(local)];
      rec[4 * i + 2] = x.recvd[size_t(local)];
      rec[4 * i + 3] = u64(x.t_us);
    }
    if (names) names[i] = x.name;
  }
  return n;
}

// The RCCL watchdog's lifecycle without a GPU or a communicator (tests/test_transport_plan.py):
// a collective is marked pending, the watchdog fires after limit_s, then -- when build_returns --
// the build's failure path runs (gcz_group::fail's disarm) and the process must still be alive
// grace_s + 1 s later.  Returns 0 when it fired and the process survived (it ends with exit code
// 70 when the build never returns, which is the other half of the contract).
int gcz_dist_watch_selftest(int limit_s, int grace_s, int build_returns) {
  RcclTransport t;
  gcz_group::Watch w(&t, -1, 0);
  w.limit_s = limit_s;
  w.grace_s = grace_s;
  w.begin(0, "collective #0 selftest");
  const auto t0 = std::chrono::steady_clock::now();
  while (!w.fired && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(limit_s + 10))
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  if (!w.fired) return 1;
  if (build_returns) w.disarm();
  std::this_thread::sleep_for(std::chrono::seconds(grace_s + 1));
  return 0;
}

int gcz_dist_p2p_plan(int world, int me, const uint64_t* M, int reverse, uint64_t elem, const uint64_t* sd,
                      const uint64_t* rd, uint64_t* out) {
  if (world < 1 || world > kMaxRanks || me < 0 || me >= world || !M || !out) return GCZ_ERR_ARG;
  const std::vector<u64> Mv(M, M + size_t(world) * size_t(world));   // (uint64_t -> u64)
  const auto ops = p2p_plan(Mv, world, me, reverse != 0, size_t(elem), reinterpret_cast<const u64*>(sd),
                            reinterpret_cast<const u64*>(rd));
  for (int q = 0; q < world; ++q) {
    const P2POp& o = ops[size_t(q)];
    out[5 * q] = o.send_off;
    out[5 * q + 1] = o.send_bytes;
    out[5 * q + 2] = o.recv_off;
    out[5 * q + 3] = o.recv_bytes;
    out[5 * q + 4] = u64(o.peer);
  }
  return GCZ_OK;
}

int gcz_dist_gather_plan(int world, int me, const uint64_t* cnt, uint64_t elem, uint64_t* out) {
  if (world < 1 || world > kMaxRanks || me < 0 || me >= world || !cnt || !out) return GCZ_ERR_ARG;
  const std::vector<u64> c(cnt, cnt + world);
  const std::vector<u64> Mu = gather_matrix(c, world);
  const std::vector<uint64_t> M(Mu.begin(), Mu.end());
  return gcz_dist_p2p_plan(world, me, M.data(), 0, elem, nullptr, nullptr, out);
}

int gcz_group_n_local(const gcz_group* g) { return g ? int(g->ctx.size()) : 0; }
int gcz_group_rank(const gcz_group* g, int i) { return g && i >= 0 && i < int(g->ctx.size()) ? g->rank[i] : -1; }
int gcz_group_world(const gcz_group* g) { return g ? g->world : 0; }
int gcz_group_canary_check(gcz_group* g, char* msg, uint64_t cap) {
  if (!g) return GCZ_ERR_ARG;
  if (hipSetDevice(g->ctx[0]->device) != hipSuccess) return GCZ_ERR_DEVICE;
  if (g->tr)
    if (hipStream_t bs = g->tr->bulk_stream()) (void)hipStreamSynchronize(bs);
  std::string out;
  int n = 0;
  for (size_t i = 0; i < g->ctx.size(); ++i) {
    std::string o;
    const int k = gcz_canary_scan(g->ctx[i], o);
    if (k < 0) return -1;
    if (k) out += "local rank " + std::to_string(i) + ": " + o;
    n += k;
  }
  if (msg && cap) std::snprintf(msg, size_t(cap), "%s", out.c_str());
  return n;
}
int gcz_group_has_bulk(gcz_group* g) { return g && g->tr && g->tr->bulk_stream() ? 1 : 0; }
gcz_ctx* gcz_group_ctx(gcz_group* g, int i) { return g && i >= 0 && i < int(g->ctx.size()) ? g->ctx[i] : nullptr; }
const char* gcz_group_last_error(const gcz_group* g) { return g ? g->last_error.c_str() : "null group"; }

int gcz_dist_plan(uint64_t S, int world, int rank, uint64_t* s0, uint64_t* s1, int* G) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world) return GCZ_ERR_ARG;
  if (S == 0) {
    if (s0) *s0 = 0;
    if (s1) *s1 = 0;
    if (G) *G = 0;
    return GCZ_OK;
  }
  DistPlan p;
  p.make(S, world);
  if (s0) *s0 = p.start(rank, 0);
  if (s1) *s1 = p.end(rank, 0);
  if (G) *G = p.G;
  return GCZ_OK;
}

int gcz_group_build_device_bases(gcz_group* g, const void* const* d_bases, uint64_t S, int L) {
  if (!g || !d_bases) return GCZ_ERR_ARG;
  if (hipSetDevice(g->ctx[0]->device) != hipSuccess) return GCZ_ERR_DEVICE;
  return g->build(d_bases, nullptr, S, L);
}

int gcz_group_build_device_leaves(gcz_group* g, const uint64_t* const* d_leaves, uint64_t S, int L) {
  if (!g || !d_leaves) return GCZ_ERR_ARG;
  if (hipSetDevice(g->ctx[0]->device) != hipSuccess) return GCZ_ERR_DEVICE;
  return g->build(nullptr, reinterpret_cast<const u64* const*>(d_leaves), S, L);
}

int gcz_group_info(const gcz_group* g, gcz_info* out) {
  if (!g || !out) return GCZ_ERR_ARG;
  *out = g->info;
  return GCZ_OK;
}

int gcz_group_slice(const gcz_group* g, int i, int layer, uint64_t* offset, uint64_t* count) {
  if (!g || i < 0 || i >= int(g->ctx.size()) || g->info.status != GCZ_OK) return GCZ_ERR_ARG;
  if (layer < -1 || layer >= g->info.n_layers) return GCZ_ERR_ARG;
  const int r = g->rank[i];
  if (offset) *offset = g->slice_off[layer + 1][r];
  if (count) *count = g->slice_cnt[layer + 1][r];
  return GCZ_OK;
}

int gcz_group_copy_slice(gcz_group* g, int i, int layer, void* host_out) {
  uint64_t off = 0, cnt = 0;
  if (int rc = gcz_group_slice(g, i, layer, &off, &cnt)) return rc;
  if (!cnt) return GCZ_OK;
  if (!host_out) return GCZ_ERR_ARG;
  gcz_ctx* c = g->ctx[i];
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  const void* src = layer < 0 ? c->leaves_out.ptr
                              : static_cast<const void*>(c->nodes_out.as<uint2>() + g->node_base[i][layer]);
  if (hipMemcpyAsync(host_out, src, cnt * 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess) return GCZ_ERR_DEVICE;
  return hipStreamSynchronize(c->stream) == hipSuccess ? GCZ_OK : GCZ_ERR_DEVICE;
}

int gcz_group_fetch(gcz_group* g, gcz_tree* t) {
  if (!g || !t || g->info.status != GCZ_OK || int(g->ctx.size()) != g->world) return GCZ_ERR_ARG;
  t->L = g->info.L;
  t->root = g->info.root;
  t->leaves.assign(g->info.n_leaves, 0);
  t->layers.assign(g->info.n_layers, {});
  for (int k = 0; k < g->info.n_layers; ++k) t->layers[k].assign(2 * g->info.layer_size[k], 0);
  for (int i = 0; i < g->world; ++i) {
    for (int layer = -1; layer < g->info.n_layers; ++layer) {
      uint64_t off = 0, cnt = 0;
      if (int rc = gcz_group_slice(g, i, layer, &off, &cnt)) return rc;
      if (!cnt) continue;
      void* dst = layer < 0 ? static_cast<void*>(t->leaves.data() + off)
                            : static_cast<void*>(t->layers[layer].data() + 2 * off);
      if (int rc = gcz_group_copy_slice(g, i, layer, dst)) return rc;
    }
  }
  return GCZ_OK;
}

}  // extern "C"

// ---- single-device builds beyond 2^29 - 1 strands ---------------------------------------
// The single-device build keeps positions in the 29-bit index field of its words.  The
// reference bounds only ids to 29 bits; its positions are size_t (src/shared_tree.cpp:630-672,
// 743-763: segments of 2^25 strands), so it builds longer genomes, e.g. > 6.44 Gbase at
// L = 12 or > 537 Mbase at L = 1.  Such a genome is built here by R virtual ranks on the
// context's own device and stream (the multi-rank build above: rank-local positions, global
// ids), and the rank slices are then concatenated into the context's arrays in the layout of
// a single-device build, so copy-out, the device sort, the .dag writer and decompression see
// one ordinary build.  The virtual ranks persist in the context for the next such build.
#define SPLIT_HIP(x)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) return c->fail(GCZ_ERR_DEVICE, #x, hipGetErrorString(e_));  \
  } while (0)
int gcz_split_build(gcz_ctx* c, const void* d_bases, const u64* d_leaves, u64 S, int L) {
  const u64 share = std::max<u64>(1024, std::min<u64>(c->split_share, u64(kIdx) / 2));
  const int R = int(std::max<u64>(2, (S + share - 1) / share));
  if (R > kMaxRanks)
    return c->fail(GCZ_ERR_CAPACITY, "build", "genome too long for one device (more than 31 * 2^28 strands)");
  gcz_group*& g = c->split;
  if (g && g->world != R) {
    gcz_group_destroy(g);
    g = nullptr;
  }
  if (!g) {
    if (int rc = gcz_group_create_local(c->device, R, &g)) return c->fail(rc, "build", "virtual ranks could not be created");
    for (gcz_ctx* v : g->ctx) v->profile = false;
  }
  if (hipSetDevice(c->device) != hipSuccess) return c->fail(GCZ_ERR_DEVICE, "build", "hipSetDevice");
  for (gcz_ctx* v : g->ctx) v->stream = c->stream;   // one stream orders ranks, copies and later calls
  static_cast<LocalTransport*>(g->tr)->stream = c->stream;
  if (!c->ev_start) {
    SPLIT_HIP(hipEventCreate(&c->ev_start));
    SPLIT_HIP(hipEventCreate(&c->ev_stop));
  }
  std::vector<const void*> bases(R, nullptr);
  std::vector<const u64*> leaves(R, nullptr);
  for (int r = 0; r < R; ++r) {
    uint64_t s0 = 0, s1 = 0;
    gcz_dist_plan(S, R, r, &s0, &s1, nullptr);
    if (d_bases) bases[r] = static_cast<const unsigned char*>(d_bases) + s0 * u64(L);
    if (d_leaves) leaves[r] = d_leaves + s0;
  }
  SPLIT_HIP(hipEventRecord(c->ev_start, c->stream));
  const int rc = g->build(d_bases ? bases.data() : nullptr, d_leaves ? leaves.data() : nullptr, S, L);
  if (rc) {
    const gcz_info keep = g->info;
    c->fail(rc, "build", g->last_error.c_str());
    c->info = keep;
    c->info.status = rc;
    return rc;
  }
  // assemble: the layout of gcz_ctx::build (one stream: the copies follow the build)
  const gcz_info& gi = g->info;
  if (int e = g->assemble(c)) {
    c->fail(e, "build", g->last_error.c_str());
    return e;
  }
  SPLIT_HIP(hipEventRecord(c->ev_stop, c->stream));
  SPLIT_HIP(hipEventSynchronize(c->ev_stop));
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, c->ev_start, c->ev_stop);
  c->info = gi;
  c->info.status = GCZ_OK;
  c->info.n_strands = S;
  c->info.build_ms = ms;
  c->info.build_ms_all = ms;
  c->dense_used = gi.leaf_path == 1;
  c->last_error.clear();
  return GCZ_OK;
}
