/*
 * gcz.h — C ABI of the MI355X-native shared_tree construction engine (libgcz).
 *
 * This is the drop-in boundary for the reference's hot path.  The reference
 * (Quinten-van-Woerkom/genome-compression) has no FFI of its own: its
 * replaceable engine is `tree_constructor` behind the `shared_tree`
 * constructors (include/shared_tree.h:158-162, src/shared_tree.cpp:207-215,
 * called from compress.cpp:183 and tests/test.cpp:240,274,298,339,395).  The
 * entry points below are what a binding of that engine needs: plain pointers
 * and sizes, no C++/torch types.  include/shared_tree.h (this repo) rebuilds the
 * reference's C++ surface on top of them; INTEGRATION.md shows the ctypes /
 * C++ bindings a maintainer adds.
 *
 * Word layout (reference in-memory `pointer`, include/shared_tree.h:73-76):
 *   bits 0-28 index, bit 29 mirror, bit 30 transpose, bit 31 invariant.
 * A node is two words (left, right); the null child is 0x9fffffff.
 * Leaves are nibble-packed `dna` values (include/dna.h:20-32,73-74).
 */
#ifndef GCZ_H
#define GCZ_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(GCZ_BUILDING)
#define GCZ_API __attribute__((visibility("default")))
#else
#define GCZ_API
#endif

/* Status codes.  The reference never returns errors: it prints and exits
 * (src/dna.cpp:44-47 unknown symbol -> exit(1); src/fasta_reader.cpp:15-18,109-112
 * I/O -> exit(1)).  The C++ wrapper maps these codes back to that behaviour. */
enum {
  GCZ_OK = 0,
  GCZ_ERR_SYMBOL = 1,   /* unknown nucleotide symbol; see gcz_info.error_offset */
  GCZ_ERR_IO = 2,       /* file could not be opened/read */
  GCZ_ERR_CAPACITY = 3, /* more than 2^29-1 unique items in one layer */
  GCZ_ERR_DEVICE = 4,   /* HIP runtime error */
  GCZ_ERR_ARG = 5,      /* invalid argument (L outside 1..16, null pointer, ...) */
  GCZ_ERR_EMPTY = 6     /* fewer than L bases: the reference has no tree to build */
};

#define GCZ_NULL_WORD 0x9fffffffu
#define GCZ_MAX_LAYERS 64

typedef struct gcz_ctx gcz_ctx;     /* one device + stream + workspace */
typedef struct gcz_tree gcz_tree;   /* host-resident shared tree */

/* Summary of the last build (shared_tree::depth/leaf_count/node_count, shared_tree.h:164-170). */
typedef struct {
  int status;                        /* GCZ_* of the last build */
  int L;                             /* leaf length dna::size() */
  int n_layers;                      /* node layers; depth() = n_layers + 1 */
  uint32_t root;                     /* root pointer word (keeps m/t bits) */
  uint64_t n_strands;                /* S = width() of the tree */
  uint64_t n_leaves;                 /* unique canonical leaves */
  uint64_t layer_size[GCZ_MAX_LAYERS];
  uint64_t error_offset;             /* GCZ_ERR_SYMBOL: byte offset into the bases */
  int error_symbol;                  /* the offending byte */
  double build_ms;                   /* device time of the build (hipEvents) */
  uint64_t hashed_pairs;             /* node pairs hash-consed (others skipped as provably unique) */
  uint64_t bucketed_pairs;           /* ... of which through the bucketed LDS dedupe (not the table) */
  uint32_t leaf_path;                /* 0: hash-table leaf level, 1: dense sort (pure ACGT, L <= 12) */
  uint32_t attempts;                 /* device builds this call ran: > 1 after a rebuild (a bucket
                                        overflow, leaf-table regrowth or the wide-table fallback) */
  double build_ms_all;               /* device time of every attempt (build_ms: the last one) */
  uint32_t repetitive;               /* the node levels took the repetitive-data path (LDS pre-dedupe;
                                        decided by a probe of the first leaf chunk) */
  uint32_t handed_back;              /* dedupe buckets the bitmap kernel handed to the table kernel
                                        (hot keys; all levels of the last attempt) */
} gcz_info;

/* ---- device context ---------------------------------------------------- */
GCZ_API int gcz_ctx_create(int device, gcz_ctx **out);
GCZ_API void gcz_ctx_destroy(gcz_ctx *ctx);
/* Launch on a caller stream (hipStream_t); NULL restores the context's own stream. */
GCZ_API int gcz_ctx_set_stream(gcz_ctx *ctx, void *hip_stream);
GCZ_API void *gcz_ctx_stream(gcz_ctx *ctx);
GCZ_API const char *gcz_ctx_last_error(gcz_ctx *ctx);

/* Device memory helpers on the context's device/stream, so FFI callers need no
 * other GPU runtime for staging inputs. */
GCZ_API void *gcz_dev_alloc(gcz_ctx *ctx, uint64_t bytes);
GCZ_API int gcz_dev_free(gcz_ctx *ctx, void *ptr);
GCZ_API int gcz_memcpy_h2d(gcz_ctx *ctx, void *dst, const void *src, uint64_t bytes);
/* Prepare the upload of a `bytes`-byte input (gcz_build_host_*): the input buffer
 * allocated and touched, the host -> device path warmed (a cold process's first copy
 * runs at about half the link rate).  Optional; the C++ surface runs it while the
 * input file is mapped. */
GCZ_API int gcz_upload_reserve(gcz_ctx *ctx, uint64_t bytes);
GCZ_API int gcz_memcpy_d2h(gcz_ctx *ctx, void *dst, const void *src, uint64_t bytes);
GCZ_API int gcz_ctx_sync(gcz_ctx *ctx);

/* ---- builds ------------------------------------------------------------ *
 * Replace tree_constructor::reduce (src/shared_tree.cpp:719-763).  The result
 * stays resident in HBM inside ctx until the next build; fetch it with
 * gcz_info_get / gcz_copy_leaves / gcz_copy_layer / gcz_tree_fetch.
 * All builds are asynchronous on the context stream except that they return
 * after validating results (one small D2H of the level counts). */

/* bases: device pointer to raw nucleotide bytes (no FASTA line structure);
 * the tail beyond a multiple of L is ignored (src/fasta_reader.cpp:60-61). */
GCZ_API int gcz_build_device_bases(gcz_ctx *ctx, const void *d_bases, uint64_t nbases, int L);
/* leaves: device pointer to S nibble-packed strands (shared_tree(std::vector<dna>&),
 * src/shared_tree.cpp:212-215). */
GCZ_API int gcz_build_device_leaves(gcz_ctx *ctx, const uint64_t *d_leaves, uint64_t S, int L);
/* Host conveniences: FASTA bytes (line structure per src/fasta_reader.cpp:40-68)
 * or host leaves; copied to the device, then built. */
GCZ_API int gcz_build_host_fasta(gcz_ctx *ctx, const void *fasta, uint64_t nbytes, int L);
GCZ_API int gcz_build_host_leaves(gcz_ctx *ctx, const uint64_t *leaves, uint64_t S, int L);
/* A FASTA file already in device memory: the line contract (headers, blank lines;
 * src/fasta_reader.cpp:40-68) runs on the device, then the build. */
GCZ_API int gcz_build_device_fasta(gcz_ctx *ctx, const void *d_file, uint64_t n, int L);
/* fasta_reader{path, buffer_strands} + tree_constructor::reduce(file) (src/fasta_reader.cpp:13-35,
 * src/shared_tree.cpp:719-736): the reader's buffers of B = min(n / L + 1, buffer_strands)
 * strands (0: the default 1 << 22) shape both the line contract (a line that crosses a buffer
 * boundary) and the tree, every buffer being reduced to its own subtree before the roots are
 * combined.  For a power-of-two B >= 2 (the default reader) the tree equals gcz_build_*_fasta's.
 * first_strand (a multiple of B) skips the buffers read_into already handed out. */
GCZ_API int gcz_build_host_fasta_buffered(gcz_ctx *ctx, const void *fasta, uint64_t nbytes, int L,
                                          uint64_t buffer_strands, uint64_t first_strand);
GCZ_API int gcz_build_device_fasta_buffered(gcz_ctx *ctx, const void *d_file, uint64_t n, int L,
                                            uint64_t buffer_strands, uint64_t first_strand);
/* The device line contract alone (as gcz_fasta_extract): bases of d_file into d_out
 * (cap bytes; null: count only). */
GCZ_API int gcz_fasta_extract_device(gcz_ctx *ctx, const void *d_file, uint64_t n, int L, uint64_t buffer_strands,
                                     void *d_out, uint64_t cap, uint64_t *nbases);

GCZ_API int gcz_info_get(gcz_ctx *ctx, gcz_info *out);
GCZ_API int gcz_copy_leaves(gcz_ctx *ctx, uint64_t *host_out);                /* n_leaves u64 */
GCZ_API int gcz_copy_layer(gcz_ctx *ctx, int layer, uint32_t *host_out);      /* 2*layer_size words */
/* The whole DAG in one call: leaves (n_leaves u64) and every layer (layers_out[k]: 2*layer_size
 * words), through a pinned staging ring with parallel host copies -- the fast path into fresh,
 * unpinned host memory.  Fills what the reference's tree_constructor appends to
 * shared_tree::leaves / nodes (include/shared_tree.h:221-223, src/shared_tree.cpp:298-308). */
GCZ_API int gcz_fetch_host(gcz_ctx *ctx, uint64_t *leaves_out, uint32_t *const *layers_out);
/* Pin the fetch's staging ring for a DAG of `total_bytes` ahead of time (64 MB at most, ~16 ms;
 * gcz_fetch_host otherwise does it on its first call). */
GCZ_API int gcz_fetch_reserve(gcz_ctx *ctx, uint64_t total_bytes);
/* Host storage for fetched trees (the allocator of the drop-in's shared_tree containers, the
 * reference's std::vector members at include/shared_tree.h:221-222): arrays of >= 4 MB are
 * 2 MB-aligned mappings advised as transparent huge pages (the fetch faults them in 2 MB steps
 * on several threads); gcz_host_free takes the same byte count.  NULL when the memory cannot be
 * had (nothing throws through the C ABI). */
GCZ_API void *gcz_host_alloc(uint64_t bytes);
GCZ_API void gcz_host_free(void *p, uint64_t bytes);
/* Pre-fault `bytes` of that storage (2 MB pages, `threads` host threads) as a pool the next
 * large gcz_host_alloc calls are carved from -- the drop-in does it while the HIP runtime
 * starts, so the fetch copies into present pages; gcz_host_pool_release unmaps what is left. */
GCZ_API int gcz_host_prefault(uint64_t bytes, int threads);
GCZ_API void gcz_host_pool_release(int async);   /* async: unmapped on a detached thread */

/* Device pointers of the last build (valid until the next build). */
GCZ_API const uint64_t *gcz_device_leaves(gcz_ctx *ctx);
GCZ_API const uint32_t *gcz_device_layer(gcz_ctx *ctx, int layer);

/* ---- per-kernel timing (hipEvents on the launch stream) ---------------- */
GCZ_API int gcz_profile_enable(gcz_ctx *ctx, int on);
/* Kernel `k` of the profile table: name, launches, total ms.  Returns 0, or -1 past the end. */
GCZ_API int gcz_profile_entry(gcz_ctx *ctx, int k, const char **name, uint64_t *launches, double *total_ms);
GCZ_API void gcz_profile_reset(gcz_ctx *ctx);
/* Timeline of the profiled scopes since the last reset: entry i is out[3i..3i+2] =
 * (kernel index as in gcz_profile_entry, start in ms after the build's start event,
 * duration in ms).  Copies min(count, cap) entries; returns the count. */
GCZ_API uint64_t gcz_profile_trace(gcz_ctx *ctx, float *out, uint64_t cap);

/* ---- host tree (shared_tree container operations) ---------------------- */
GCZ_API gcz_tree *gcz_tree_new(void);
GCZ_API void gcz_tree_free(gcz_tree *t);
GCZ_API int gcz_tree_fetch(gcz_ctx *ctx, gcz_tree *t);          /* D2H of the last build */
GCZ_API int gcz_tree_n_layers(const gcz_tree *t);
GCZ_API uint64_t gcz_tree_n_leaves(const gcz_tree *t);
GCZ_API uint64_t gcz_tree_layer_size(const gcz_tree *t, int layer);
GCZ_API uint32_t gcz_tree_root(const gcz_tree *t);
GCZ_API int gcz_tree_L(const gcz_tree *t);
GCZ_API const uint64_t *gcz_tree_leaves(const gcz_tree *t);
GCZ_API const uint32_t *gcz_tree_layer(const gcz_tree *t, int layer);
/* Frequency sort (src/shared_tree.cpp:316-483), bytes() (:488-496),
 * serialize() (:504-513), width() (shared_tree.h:165). */
GCZ_API void gcz_tree_sort(gcz_tree *t);
GCZ_API uint64_t gcz_tree_bytes(const gcz_tree *t);
GCZ_API uint64_t gcz_tree_serialize(const gcz_tree *t, uint8_t *buf, uint64_t cap);
GCZ_API uint64_t gcz_tree_width(const gcz_tree *t);
/* Fill a host tree from raw arrays (e.g. a tree built elsewhere): leaves, then
 * layers bottom-up (2 words per node), then the root word. */
GCZ_API void gcz_tree_set_leaves(gcz_tree *t, int L, const uint64_t *leaves, uint64_t n);
GCZ_API void gcz_tree_push_layer(gcz_tree *t, const uint32_t *words, uint64_t n_nodes);
GCZ_API void gcz_tree_set_root(gcz_tree *t, uint32_t root);
/* shared_tree::deserialize (src/shared_tree.cpp:520-538): the .dag format
 * drops the invariant bit, so every loaded pointer has bit 31 clear.
 * Returns GCZ_OK or GCZ_ERR_ARG on a truncated buffer. */
GCZ_API int gcz_tree_deserialize(gcz_tree *t, int L, const uint8_t *buf, uint64_t n);

/* ---- host utilities ---------------------------------------------------- */
/* FASTA line contract of src/fasta_reader.cpp:40-68 (headers, blank lines, the
 * fresh peek where a line crosses a reader buffer of buffer_strands strands;
 * 0 = the reference default 1 << 22, include/fasta_reader.h:23) for leaves of
 * L nucleotides; writes the concatenated bases to out (capacity >= n) and
 * returns their count. */
GCZ_API uint64_t gcz_fasta_extract(const uint8_t *file, uint64_t n, int L, uint64_t buffer_strands, uint8_t *out);
/* Synthetic genomes (genome-compression_amd/csrc/synth.h), multi-threaded. */
GCZ_API void gcz_synth_fill(char *out, int kind, uint64_t seed, uint64_t begin, uint64_t end);
GCZ_API uint64_t gcz_synth_default_seed(void);

/* ---- frequency sort, bytes(), .dag on the device ----------
 * Act on the last build of ctx, in place: the same result as gcz_tree_sort /
 * gcz_tree_bytes / gcz_tree_serialize on the fetched tree (reference
 * shared_tree::sort_tree, bytes, serialize: src/shared_tree.cpp:443-513). */
GCZ_API int gcz_sort_device(gcz_ctx *ctx);
/* The device buffers gcz_sort_device needs for the last build, allocated ahead (callable on
 * another thread while the tree is fetched; gcz_sort_device then finds them in place). */
GCZ_API int gcz_sort_reserve(gcz_ctx *ctx);
GCZ_API int gcz_bytes_device(gcz_ctx *ctx, uint64_t *out);
/* .dag bytes into host_buf (cap >= *written, else GCZ_ERR_ARG with *written set). */
GCZ_API int gcz_serialize_device(gcz_ctx *ctx, uint8_t *host_buf, uint64_t cap, uint64_t *written);
/* .dag bytes left in device memory owned by ctx (valid until the next call). */
GCZ_API const uint8_t *gcz_device_dag(gcz_ctx *ctx, uint64_t *written);

/* Decompression of the last build (shared_tree::operator[] / iterator for every
 * index, src/shared_tree.cpp:268-291,553-614): S*L upper-case IUPAC symbols. */
GCZ_API int gcz_decompress_device(gcz_ctx *ctx, void *d_out, uint64_t cap);
GCZ_API int gcz_decompress(gcz_ctx *ctx, uint8_t *host_out, uint64_t cap);

/* ---- multi-rank build ---------------------
 * R ranks own contiguous strand ranges; every hash-consed level is reconciled
 * through key owners (all-to-all), ids stay the global first-occurrence ranks,
 * so rank r holds a contiguous slice [offset, offset + count) of every layer
 * and the layers are the rank-ordered concatenation of the slices (identical
 * to gcz_build_*).  Rank order = position order.  Replaces the same
 * tree_constructor::reduce as gcz_build_device_bases, spread over GPUs. */
typedef struct gcz_group gcz_group;
/* 128-byte RCCL unique id (rank 0 creates it, every rank passes it to create). */
GCZ_API int gcz_dist_unique_id(void *out, uint64_t cap);
/* One rank of a `world`-rank job on ctx's device (one process per GPU, RCCL). */
GCZ_API int gcz_group_create_rccl(gcz_ctx *ctx, int rank, int world, const void *unique_id, gcz_group **out);
/* `world` virtual ranks sharing one device, exchanges as device copies (testing). */
GCZ_API int gcz_group_create_local(int device, int world, gcz_group **out);
/* One rank per process, exchanges host-staged through a fresh POSIX shared-memory object
 * `name` (region_bytes per rank, sparse; unlinked once every rank has mapped it): the
 * multi-process path on a single GPU, where RCCL refuses two ranks per device (testing). */
GCZ_API int gcz_group_create_shm(gcz_ctx *ctx, int rank, int world, const char *name, uint64_t region_bytes,
                                 gcz_group **out);
GCZ_API void gcz_group_destroy(gcz_group *g);
GCZ_API int gcz_group_world(const gcz_group *g);
GCZ_API int gcz_group_n_local(const gcz_group *g);          /* ranks driven by this process */
GCZ_API int gcz_group_rank(const gcz_group *g, int local);
GCZ_API gcz_ctx *gcz_group_ctx(gcz_group *g, int local);
GCZ_API const char *gcz_group_last_error(const gcz_group *g);
/* 1 when the group runs bulk groups (the fused schedule's layer-0 key all-to-all) on a second
 * stream: RCCL groups whose ranks all created the split communicator and its stream (agreed at
 * creation; GCZ_FL_BULK=0 on any rank turns it off everywhere), local groups with
 * GCZ_LOCAL_BULK=1 (testing). */
GCZ_API int gcz_group_has_bulk(gcz_group *g);
/* GCZ_CANARY=1 at context creation (testing): every device buffer the library sizes ends in a
 * 4 KB guard band of 0xA5 bytes; the checks synchronise and return the number of buffers whose
 * band was overwritten (an out-of-bounds store), describing the first ones in msg (may be
 * NULL), or -1 when the context was created without canaries. */
GCZ_API int gcz_ctx_canary_check(gcz_ctx *ctx, char *msg, uint64_t cap);
GCZ_API int gcz_group_canary_check(gcz_group *g, char *msg, uint64_t cap);
/* The guard-band check finds a planted store one byte past a 1000-byte buffer: 0 = it does. */
GCZ_API int gcz_ctx_canary_selftest(gcz_ctx *ctx);
/* The exchanges of the group's last build, in order (every rank runs the same sequence):
 * returns their number; for i < cap, rec[4 i ..] = {sequence number, bytes local rank `local`
 * sent to other ranks, bytes it received from them, host enqueue time in us after the build
 * began}, names[i] = the exchange's name (static string).  Either array may be NULL.
 * Bounds: GCZ_DIST_TIMEOUT_S (default 180) limits one exchange -- the RCCL watchdog names the
 * collective that did not complete and aborts the communicator, the shm barrier fails;
 * GCZ_DIST_STALL="rank:seq:seconds" makes a rank sleep before exchange #seq (testing). */
GCZ_API int gcz_group_xlog(const gcz_group *g, int local, uint64_t *rec, const char **names, int cap);
/* The point-to-point transfers rank `me` issues in an all-to-all of `world` ranks (the RCCL
 * transport's own arithmetic, for host tests): counts M[s * world + d] elements of `elem` bytes
 * (reverse != 0: the transposed exchange), segments packed in peer order or at the explicit
 * element displacements sd[s * world + d] (sender s) / rd[d * world + s] (receiver d); NULL sd/rd
 * = packed.  out[5 q ..] = {send offset, send bytes, receive offset, receive bytes, q} in bytes for
 * peer q (q == me: the local copy).  gcz_dist_gather_plan: the gather of cnt[r] elements of every
 * rank r to rank 0, concatenated in rank order. */
GCZ_API int gcz_dist_p2p_plan(int world, int me, const uint64_t *M, int reverse, uint64_t elem, const uint64_t *sd,
                              const uint64_t *rd, uint64_t *out);
GCZ_API int gcz_dist_gather_plan(int world, int me, const uint64_t *cnt, uint64_t elem, uint64_t *out);
/* The RCCL watchdog's lifecycle without a GPU (tests): a pending collective, the watchdog fires
 * after limit_s; build_returns != 0: the build's failure path runs and the process is still alive
 * grace_s + 1 s later (returns 0); build_returns == 0: the process ends with exit code 70. */
GCZ_API int gcz_dist_watch_selftest(int limit_s, int grace_s, int build_returns);
/* Strands [s0, s1) of `rank` for an S-strand genome; G = distributed node levels. */
GCZ_API int gcz_dist_plan(uint64_t S, int world, int rank, uint64_t *s0, uint64_t *s1, int *G);
/* d_bases[i]: device ASCII bases of local rank i's strands ((s1 - s0) * L bytes). */
GCZ_API int gcz_group_build_device_bases(gcz_group *g, const void *const *d_bases, uint64_t S, int L);
/* d_leaves[i]: device packed strands [s0, s1) of local rank i (shared_tree(std::vector<dna>&)). */
GCZ_API int gcz_group_build_device_leaves(gcz_group *g, const uint64_t *const *d_leaves, uint64_t S, int L);
GCZ_API int gcz_group_info(const gcz_group *g, gcz_info *out);   /* whole-tree summary */
/* Slice of local rank i in layer (-1 = leaves): ids [offset, offset + count). */
GCZ_API int gcz_group_slice(const gcz_group *g, int local, int layer, uint64_t *offset, uint64_t *count);
GCZ_API int gcz_group_copy_slice(gcz_group *g, int local, int layer, void *host_out);
/* Whole tree to the host (every rank local, i.e. gcz_group_create_local). */
GCZ_API int gcz_group_fetch(gcz_group *g, gcz_tree *t);
/* The last build's whole tree into `dst` (rank 0's process: a context on rank 0's device other
 * than the group's own; ignored elsewhere, every rank calls) in the single-device layout: each
 * layer's rank slices gathered device to device (RCCL / shm gather to rank 0, or copies when all
 * ranks are local).  Afterwards gcz_sort_device, gcz_device_dag / gcz_serialize_device,
 * gcz_decompress_device and gcz_fetch_host work on dst as after a one-GPU build -- the device
 * ratio path of a distributed tree (reference: sort_tree / bytes / serialize,
 * src/shared_tree.cpp:443-513). */
GCZ_API int gcz_group_assemble(gcz_group *g, gcz_ctx *dst);

#ifdef __cplusplus
}
#endif
#endif
