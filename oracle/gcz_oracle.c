/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-threaded restatement of the reference's shared_tree
 * construction path (Quinten-van-Woerkom/genome-compression).  It exists to
 * CHECK the MI355X product path; it is never linked into, loaded by or called
 * from the product (libgcz).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may use it.
 *
 * Parity pin: this restatement is checked against golden vectors produced by
 * the compiled reference itself (oracle/ref_harness.cpp, built into
 * oracle/_ref/ from /root/reference sources) and committed under
 * tests/golden/ (see tests/golden/make_goldens.sh).
 *
 * Every function cites the reference file:line whose behaviour it restates.
 * All paths below are relative to the reference repository root.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------ */
/* Leaf codec: include/dna.h:20-32 (nac codes), src/dna.cpp:25-49 (to_nac)   */
/* ------------------------------------------------------------------------ */
static int8_t NAC[256];
static int nac_ready = 0;

static void nac_init(void) {
  if (nac_ready) return;
  memset(NAC, -1, sizeof NAC);
  const char *sym = "ACGTRYKMBVDHSWN-";
  const int8_t code[16] = {1, 2, 4, 8, 3, 12, 7, 14, 5, 10, 11, 13, 0, 9, 6, 15};
  for (int i = 0; i < 16; ++i) {
    NAC[(unsigned char)sym[i]] = code[i];
    if (sym[i] >= 'A' && sym[i] <= 'Z') NAC[(unsigned char)(sym[i] - 'A' + 'a')] = code[i];
  }
  nac_ready = 1;
}

/* to_nac: case-insensitive IUPAC symbol -> 4-bit code, -1 when unknown. */
ORC_API int orc_nac(int ch) { nac_init(); return NAC[ch & 0xff]; }

/* dna::transposed (src/dna.cpp:104-111): bit-reverse every nibble. */
ORC_API uint64_t orc_leaf_transposed(uint64_t v) {
  v = ((v >> 1) & 0x5555555555555555ull) | ((v & 0x5555555555555555ull) << 1);
  v = ((v >> 2) & 0x3333333333333333ull) | ((v & 0x3333333333333333ull) << 2);
  return v;
}

/* dna::mirrored (src/dna.cpp:116-121): reverse the order of the low L nibbles,
 * result starts from zero (so bits above 4L are dropped). */
ORC_API uint64_t orc_leaf_mirrored(uint64_t v, int L) {
  uint64_t r = 0;
  for (int i = 0; i < L; ++i) r |= ((v >> (4 * (L - 1 - i))) & 0xfull) << (4 * i);
  return r;
}

/* dna::canonical (src/dna.cpp:135-143) + variadic_min (include/utility.h:158-170):
 * minimum of (value, m, t) over the four symmetry variants; inv = palindrome.
 * Returns the canonical value, writes m/t/inv. */
ORC_API uint64_t orc_leaf_canonical(uint64_t x, int L, int *m, int *t, int *inv) {
  uint64_t tr = orc_leaf_transposed(x);
  uint64_t mi = orc_leaf_mirrored(x, L);
  uint64_t in = orc_leaf_mirrored(tr, L);   /* inverted = transposed().mirrored() (dna.h:51) */
  *inv = (x == mi);
  uint64_t best = x; int bm = 0, bt = 0;
  /* candidate order as in dna.cpp:137-142: current, transpose, mirror, invert */
  const uint64_t cv[3] = {tr, mi, in};
  const int cm[3] = {0, 1, 1}, ct[3] = {1, 0, 1};
  for (int c = 0; c < 3; ++c) {
    int less = cv[c] < best || (cv[c] == best && (cm[c] < bm || (cm[c] == bm && ct[c] < bt)));
    if (less) { best = cv[c]; bm = cm[c]; bt = ct[c]; }
  }
  *m = bm; *t = bt;
  return best;
}

/* ------------------------------------------------------------------------ */
/* Pointer word algebra: include/shared_tree.h:36-77, src/shared_tree.cpp:76-107
 * word = index(29) | mirror<<29 | transpose<<30 | invariant<<31              */
/* ------------------------------------------------------------------------ */
#define NULL_INDEX 0x1fffffffu
#define NULL_WORD 0x9fffffffu
static inline uint32_t UL(uint32_t w) { return w & 0x7fffffffu; }                /* to_ulong :103-107 */
static inline uint32_t W(uint32_t i, int m, int t, int v) {                       /* ctor :85-86 */
  return i | ((uint32_t)(m && !v) << 29) | ((uint32_t)(t != 0) << 30) | ((uint32_t)(v != 0) << 31);
}
/* transform ctor (src/shared_tree.cpp:76-80) */
static inline uint32_t XF(uint32_t w, int M, int T) {
  int m = (w >> 29) & 1, t = (w >> 30) & 1, v = (w >> 31) & 1;
  int nm = (M != m) && !v;
  int nt = (T != t) && (UL(w) != NULL_INDEX);
  return (w & 0x1fffffffu) | ((uint32_t)nm << 29) | ((uint32_t)nt << 30) | ((uint32_t)v << 31);
}

ORC_API uint32_t orc_ptr_xf(uint32_t w, int M, int T) { return XF(w, M, T); }

/* node::canonical (include/shared_tree.h:115-126): min over (key, m, t) of
 * id=(l,r), mir=(M(r),M(l)), tra=(T(l),T(r)), inv=(I(r),I(l)); key compares
 * to_ulong of both children (shared_tree.h:53-55,110). */
ORC_API void orc_node_canonical(uint32_t l, uint32_t r, uint32_t *cl, uint32_t *cr, int *m, int *t) {
  uint32_t vl[4], vr[4];
  const int vm[4] = {0, 1, 0, 1}, vt[4] = {0, 0, 1, 1};   /* candidate order shared_tree.h:121-124 */
  vl[0] = XF(l, 0, 0);  vr[0] = XF(r, 0, 0);
  vl[1] = XF(r, 1, 0);  vr[1] = XF(l, 1, 0);
  vl[2] = XF(l, 0, 1);  vr[2] = XF(r, 0, 1);
  vl[3] = XF(r, 1, 1);  vr[3] = XF(l, 1, 1);
  int b = 0;
  for (int c = 1; c < 4; ++c) {
    uint64_t kc = ((uint64_t)UL(vl[c]) << 32) | UL(vr[c]);
    uint64_t kb = ((uint64_t)UL(vl[b]) << 32) | UL(vr[b]);
    int less = kc < kb || (kc == kb && (vm[c] < vm[b] || (vm[c] == vm[b] && vt[c] < vt[b])));
    if (less) b = c;
  }
  *cl = vl[b]; *cr = vr[b]; *m = vm[b]; *t = vt[b];
}

/* ------------------------------------------------------------------------ */
/* FASTA ingest: src/fasta_reader.cpp:40-68 (load_buffer)                    */
/* ------------------------------------------------------------------------ */
/* Restates the reader's line contract over a whole file held in memory:
 *  - at each line start, if the byte is '>' or '\n' ONE line is skipped
 *    (fasta_reader.cpp:49-51), then the following line is read as data
 *    without a second peek (so a 2nd header line becomes data);
 *  - data line bodies are concatenated (:52-57);
 *  - buffer boundaries.  load_buffer fills cap = B*L data bytes per buffer,
 *    B = min(file_size/L + 1, buffer_strands) when file_size/L + 1 >= buffer_strands,
 *    else file_size/L + 1 (:22-31).  A getline that fills the buffer exactly also
 *    extracts a newline that follows (libstdc++ getline), so a line ending on a
 *    boundary behaves as anywhere else.  A data line that CROSSES a boundary
 *    resumes, in the next load_buffer, with a fresh peek at the byte at the
 *    boundary (:48-51): if that byte is '>', the rest of the line is skipped and
 *    the following line is read as data.  (Pinned against the compiled reference
 *    at small buffer sizes by tests/test_reader_boundary.py.)
 * buffer_strands = 0 means the reference default 1<<22 (fasta_reader.h:23).
 * Truncation to a multiple of L happens in the caller (fasta_reader.cpp:60-61).
 * Returns the number of bases written to out (out must hold n bytes). */
ORC_API uint64_t orc_fasta_extract(const uint8_t *f, uint64_t n, int L, uint64_t buffer_strands, uint8_t *out) {
  if (!buffer_strands) buffer_strands = (uint64_t)1 << 22;
  const uint64_t fs = n / (uint64_t)L + 1;
  const uint64_t cap = (fs < buffer_strands ? fs : buffer_strands) * (uint64_t)L;
  uint64_t pos = 0, j = 0;
  int forced = 0;   /* the line after a skip is data without a peek */
  while (pos < n) {
    if (!forced && (f[pos] == '>' || f[pos] == '\n')) {
      const uint8_t *nl = memchr(f + pos, '\n', n - pos);
      pos = nl ? (uint64_t)(nl - f) + 1 : n;
      forced = 1;
      continue;
    }
    forced = 0;
    const uint8_t *nl = memchr(f + pos, '\n', n - pos);
    uint64_t end = nl ? (uint64_t)(nl - f) : n;
    /* boundaries strictly inside [j, j + len) */
    for (uint64_t k = j / cap + 1; k * cap < j + (end - pos); ++k) {
      if (f[pos + (k * cap - j)] == '>') {
        end = pos + (k * cap - j);
        forced = 1;
        break;
      }
    }
    memcpy(out + j, f + pos, end - pos);
    j += end - pos;
    pos = nl ? (uint64_t)(nl - f) + 1 : n;
  }
  return j;
}

/* dna::dna(string_view) (src/dna.cpp:79-84) + dna::set (:187-197) applied to
 * every L-byte window (fasta_reader.cpp:66-67).  Returns -1 on success or the
 * base index of the first unknown symbol (to_nac exits there, dna.cpp:44-47). */
ORC_API int64_t orc_pack(const uint8_t *bases, uint64_t S, int L, uint64_t *leaves) {
  nac_init();
  for (uint64_t i = 0; i < S; ++i) {
    uint64_t v = 0;
    for (int c = 0; c < L; ++c) {
      int code = NAC[bases[i * L + c]];
      if (code < 0) return (int64_t)(i * L + c);
      v |= (uint64_t)code << (4 * c);
    }
    leaves[i] = v;
  }
  return -1;
}

/* ------------------------------------------------------------------------ */
/* Hash-consing builder: src/shared_tree.cpp:621-763, include/shared_tree.h:245-316 */
/* ------------------------------------------------------------------------ */
typedef struct {
  uint64_t *keys;
  uint32_t *vals;
  uint8_t *used;
  uint64_t mask;
} orc_map;

static uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33; return x;
}

static void map_init(orc_map *mp, uint64_t n) {
  uint64_t cap = 16;
  while (cap < 2 * n + 16) cap <<= 1;
  mp->keys = malloc(cap * sizeof(uint64_t));
  mp->vals = malloc(cap * sizeof(uint32_t));
  mp->used = calloc(cap, 1);
  mp->mask = cap - 1;
}
static void map_free(orc_map *mp) { free(mp->keys); free(mp->vals); free(mp->used); }

/* emplace-without-overwrite (phmap emplace, external/parallel_hashmap/phmap.h:2784):
 * returns the stored value; *inserted set when the key was new. */
static uint32_t map_emplace(orc_map *mp, uint64_t key, uint32_t val, int *inserted) {
  uint64_t s = mix64(key) & mp->mask;
  for (;;) {
    if (!mp->used[s]) {
      mp->used[s] = 1; mp->keys[s] = key; mp->vals[s] = val; *inserted = 1; return val;
    }
    if (mp->keys[s] == key) { *inserted = 0; return mp->vals[s]; }
    s = (s + 1) & mp->mask;
  }
}

typedef struct {
  int L;
  uint64_t S;
  uint64_t n_leaves;
  uint64_t *leaves;          /* canonical leaf values, first-occurrence order */
  int n_layers;
  uint64_t *layer_n;         /* unique nodes per layer */
  uint32_t **layer_words;    /* 2 words (left,right) per node, raw incl. bit 31 */
  uint32_t root;
} orc_tree;

/* tree_constructor::emplace_leaf (src/shared_tree.cpp:630-637) */
static uint32_t emplace_leaf(orc_tree *tr, orc_map *mp, uint64_t leaf) {
  int m, t, v, ins;
  uint64_t c = orc_leaf_canonical(leaf, tr->L, &m, &t, &v);
  uint32_t id = map_emplace(mp, c, (uint32_t)tr->n_leaves, &ins);
  if (ins) tr->leaves[tr->n_leaves++] = c;
  return W(id, m, t, v);
}

/* tree_constructor::emplace_node (src/shared_tree.cpp:662-672); right = NULL_WORD
 * for the unary tail (utility.h:25, shared_tree.h:101). */
static uint32_t emplace_node(orc_tree *tr, int layer, orc_map *mp, uint32_t l, uint32_t r) {
  uint32_t cl, cr; int m, t, ins;
  l = XF(l, 0, 0); r = XF(r, 0, 0);                 /* node{left,right} copies (shared_tree.h:101) */
  orc_node_canonical(l, r, &cl, &cr, &m, &t);
  uint64_t key = ((uint64_t)UL(cl) << 32) | UL(cr);
  uint64_t cnt = tr->layer_n[layer];
  uint32_t id = map_emplace(mp, key, (uint32_t)cnt, &ins);
  if (ins) {
    tr->layer_words[layer][2 * cnt] = cl;
    tr->layer_words[layer][2 * cnt + 1] = cr;
    tr->layer_n[layer] = cnt + 1;
  }
  int v = UL(l) == UL(XF(r, 1, 0));                 /* left == right.mirrored() (:670) */
  return W(id, m, t, v);
}

/* Global level-by-level build.  Output-equivalent to the reference's segmented
 * reduce (shared_tree.h:305-316, shared_tree.cpp:677-763): segment sizes are
 * powers of two so pairing never crosses a segment boundary and the unary
 * tail rule (utility.h:17-29) only fires at the global tail. */
ORC_API orc_tree *orc_build(const uint64_t *leaves, uint64_t S, int L) {
  if (S == 0 || L < 1 || L > 16) return NULL;
  orc_tree *tr = calloc(1, sizeof *tr);
  tr->L = L; tr->S = S;
  tr->leaves = malloc(S * sizeof(uint64_t));
  int maxl = 2;
  for (uint64_t n = S; n > 1; n = (n + 1) / 2) ++maxl;
  tr->layer_n = calloc(maxl, sizeof(uint64_t));
  tr->layer_words = calloc(maxl, sizeof(uint32_t *));

  /* leaves + layer 0 (reduce_leaves, shared_tree.h:282-299) */
  uint64_t n = (S + 1) / 2;
  uint32_t *cur = malloc(n * sizeof(uint32_t));
  orc_map lm, nm;
  map_init(&lm, S);
  map_init(&nm, n);
  tr->layer_words[0] = malloc(2 * n * sizeof(uint32_t));
  for (uint64_t j = 0; j < n; ++j) {
    uint32_t lp = emplace_leaf(tr, &lm, leaves[2 * j]);
    uint32_t rp = (2 * j + 1 < S) ? emplace_leaf(tr, &lm, leaves[2 * j + 1]) : NULL_WORD;
    cur[j] = emplace_node(tr, 0, &nm, lp, rp);
  }
  map_free(&lm); map_free(&nm);
  tr->n_layers = 1;

  /* higher layers (reduce_nodes, shared_tree.cpp:697-712) */
  while (n > 1) {
    int layer = tr->n_layers++;
    uint64_t p = (n + 1) / 2;
    uint32_t *nxt = malloc(p * sizeof(uint32_t));
    tr->layer_words[layer] = malloc(2 * p * sizeof(uint32_t));
    map_init(&nm, p);
    for (uint64_t j = 0; j < p; ++j) {
      uint32_t r = (2 * j + 1 < n) ? cur[2 * j + 1] : NULL_WORD;
      nxt[j] = emplace_node(tr, layer, &nm, cur[2 * j], r);
    }
    map_free(&nm);
    free(cur); cur = nxt; n = p;
  }
  tr->root = cur[0];
  free(cur);
  return tr;
}

/* Segmented build: tree_constructor::reduce(fasta_reader&) over reader buffers of B strands
 * (src/shared_tree.cpp:719-736).  Each buffer goes through reduce_segment
 * (include/shared_tree.h:305-316): reduce_leaves (:282-299), then reduce_nodes
 * (src/shared_tree.cpp:697-712) while the layer holds more than one element or is shallower
 * than the tree; its root is kept.  reduce_roots (:677-692) then pairs the roots upwards.
 * Every layer's dictionary lives across the buffers, so ids are first-occurrence ranks in
 * buffer order.  For a power-of-two B >= 2 this is orc_build's tree. */
static void seg_reduce(orc_tree *tr, orc_map *maps, int layer, const uint32_t *in, uint64_t n, uint32_t *out) {
  if (layer >= tr->n_layers) tr->n_layers = layer + 1;      /* add_layer (:701-704) */
  for (uint64_t j = 0; 2 * j < n; ++j)                       /* foreach_pair, utility.h:17-29 */
    out[j] = emplace_node(tr, layer, &maps[layer], in[2 * j], 2 * j + 1 < n ? in[2 * j + 1] : NULL_WORD);
}

ORC_API orc_tree *orc_build_segmented(const uint64_t *leaves, uint64_t S, int L, uint64_t B) {
  if (S == 0 || L < 1 || L > 16 || B == 0) return NULL;
  enum { MAXL = 64 };
  /* node bound per layer: every buffer's layer k has ceil(len_k / 2) nodes; the roots above */
  const uint64_t nseg = (S + B - 1) / B, last = S - (nseg - 1) * B;
  uint64_t bound[MAXL] = {0};
  int depth = 0;                                   /* layers of one full buffer's subtree */
  for (uint64_t b = B; depth == 0 || b > 1; b = (b + 1) / 2) ++depth;
  {
    uint64_t b = B, e = last;
    for (int k = 0; k < depth; ++k) {
      bound[k] = (nseg - 1) * ((b + 1) / 2) + (e + 1) / 2;
      b = (b + 1) / 2;
      e = (e + 1) / 2;
    }
    int k = depth;
    for (uint64_t r = nseg; r > 1; r = (r + 1) / 2) {
      if (k >= MAXL) return NULL;
      bound[k++] = (r + 1) / 2;
    }
  }
  orc_tree *tr = calloc(1, sizeof *tr);
  tr->L = L; tr->S = S;
  tr->leaves = malloc(S * sizeof(uint64_t));
  tr->layer_n = calloc(MAXL, sizeof(uint64_t));
  tr->layer_words = calloc(MAXL, sizeof(uint32_t *));
  orc_map lm, maps[MAXL];
  map_init(&lm, S);
  for (int k = 0; k < MAXL && bound[k]; ++k) {
    tr->layer_words[k] = malloc(2 * bound[k] * sizeof(uint32_t));
    map_init(&maps[k], bound[k]);
  }
  uint32_t *roots = malloc(nseg * sizeof(uint32_t));
  uint32_t *a = malloc((B + 1) * sizeof(uint32_t)), *b = malloc((B + 1) * sizeof(uint32_t));
  for (uint64_t s = 0; s < nseg; ++s) {
    const uint64_t s0 = s * B, len = s + 1 < nseg ? B : last;
    for (uint64_t i = 0; i < len; ++i) a[i] = emplace_leaf(tr, &lm, leaves[s0 + i]);
    uint64_t n = len;
    seg_reduce(tr, maps, 0, a, n, b);                        /* reduce_leaves */
    n = (n + 1) / 2;
    for (int index = 1; n > 1 || index < tr->n_layers; ++index) {   /* reduce_segment loop */
      seg_reduce(tr, maps, index, b, n, a);
      uint32_t *t = a; a = b; b = t;
      n = (n + 1) / 2;
    }
    roots[s] = b[0];
  }
  uint64_t n = nseg;
  uint32_t *r2 = malloc(nseg * sizeof(uint32_t));
  for (int index = tr->n_layers; n > 1; ++index) {           /* reduce_roots */
    seg_reduce(tr, maps, index, roots, n, r2);
    uint32_t *t = roots; roots = r2; r2 = t;
    n = (n + 1) / 2;
  }
  tr->root = roots[0];
  free(roots); free(r2); free(a); free(b);
  map_free(&lm);
  for (int k = 0; k < MAXL && bound[k]; ++k) map_free(&maps[k]);
  return tr;
}

ORC_API void orc_free(orc_tree *tr) {
  if (!tr) return;
  for (int i = 0; i < tr->n_layers; ++i) free(tr->layer_words[i]);
  free(tr->layer_words); free(tr->layer_n); free(tr->leaves); free(tr);
}

ORC_API int orc_n_layers(const orc_tree *tr) { return tr->n_layers; }
ORC_API uint64_t orc_n_leaves(const orc_tree *tr) { return tr->n_leaves; }
ORC_API uint64_t orc_layer_size(const orc_tree *tr, int k) { return tr->layer_n[k]; }
ORC_API uint32_t orc_root(const orc_tree *tr) { return tr->root; }
ORC_API void orc_copy_leaves(const orc_tree *tr, uint64_t *out) {
  memcpy(out, tr->leaves, tr->n_leaves * sizeof(uint64_t));
}
ORC_API void orc_copy_layer(const orc_tree *tr, int k, uint32_t *out) {
  memcpy(out, tr->layer_words[k], 2 * tr->layer_n[k] * sizeof(uint32_t));
}

/* ------------------------------------------------------------------------ */
/* Frequency sort: src/shared_tree.cpp:316-483 (histogram, rewire_nodes,      */
/* sort_leaves, sort_nodes, sort_tree).  Net effect: the leaves and node      */
/* layers 0..D-2 are each permuted by descending reference count from their   */
/* parent layer (null children not counted), ties by old index (stable_sort), */
/* and the parents' child indices are rewired keeping the m/t/v bits.         */
/* ------------------------------------------------------------------------ */
static uint64_t *g_cnt;
static int cmp_desc(const void *a, const void *b) {
  uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
  if (g_cnt[x] != g_cnt[y]) return g_cnt[x] > g_cnt[y] ? -1 : 1;
  return x < y ? -1 : (x > y);
}

/* permute child layer `child_n` items referenced by layer `parent` */
static uint64_t *sort_perm(orc_tree *tr, int parent, uint64_t child_n) {
  uint64_t *cnt = calloc(child_n ? child_n : 1, sizeof(uint64_t));
  uint32_t *pw = tr->layer_words[parent];
  for (uint64_t i = 0; i < 2 * tr->layer_n[parent]; ++i) {
    uint32_t w = pw[i];
    if (UL(w) != NULL_INDEX) ++cnt[w & 0x1fffffffu];                   /* histogram :316-326 */
  }
  uint64_t *order = malloc((child_n ? child_n : 1) * sizeof(uint64_t));
  for (uint64_t i = 0; i < child_n; ++i) order[i] = i;
  g_cnt = cnt;
  qsort(order, child_n, sizeof(uint64_t), cmp_desc);                   /* stable via index tie-break */
  uint64_t *newpos = malloc((child_n ? child_n : 1) * sizeof(uint64_t));
  for (uint64_t i = 0; i < child_n; ++i) newpos[order[i]] = i;         /* invert_indices :360-365 */
  for (uint64_t i = 0; i < 2 * tr->layer_n[parent]; ++i) {             /* rewire_nodes :383-403 */
    uint32_t w = pw[i];
    if (UL(w) == NULL_INDEX) continue;
    pw[i] = (w & 0xe0000000u) | (uint32_t)newpos[w & 0x1fffffffu];
  }
  free(cnt); free(order);
  return newpos;
}

ORC_API void orc_sort_tree(orc_tree *tr) {
  /* leaves, referenced by layer 0 (sort_leaves :409-420) */
  uint64_t *np = sort_perm(tr, 0, tr->n_leaves);
  uint64_t *nl = malloc(tr->n_leaves * sizeof(uint64_t));
  for (uint64_t i = 0; i < tr->n_leaves; ++i) nl[np[i]] = tr->leaves[i];   /* reorder_layer :371-377 */
  free(tr->leaves); tr->leaves = nl; free(np);
  /* node layers 0..D-2, referenced by layer l+1 (sort_nodes :426-436; loops :455,469) */
  for (int l = 0; l + 1 < tr->n_layers; ++l) {
    uint64_t cn = tr->layer_n[l];
    np = sort_perm(tr, l + 1, cn);
    uint32_t *w = malloc(2 * (cn ? cn : 1) * sizeof(uint32_t));
    for (uint64_t i = 0; i < cn; ++i) {
      w[2 * np[i]] = tr->layer_words[l][2 * i];
      w[2 * np[i] + 1] = tr->layer_words[l][2 * i + 1];
    }
    free(tr->layer_words[l]); tr->layer_words[l] = w; free(np);
  }
}

/* ------------------------------------------------------------------------ */
/* bytes() and .dag serialisation: src/shared_tree.cpp:25-67,122-142,488-513; */
/* include/utility.h:178-184 (big-endian binary_write)                        */
/* ------------------------------------------------------------------------ */
static int ptr_segment(uint32_t idx) {                 /* layer_segment / compress_pointer :36-58 */
  if (idx == NULL_INDEX) return 3;
  if (idx < 16u) return 0;
  if (idx < 16u + 4096u) return 1;
  if (idx < 16u + 4096u + 1048576u) return 2;
  return 3;
}
static const uint32_t SEG_BITS[4] = {4, 12, 20, 28};
static const uint32_t SEG_START[4] = {0, 16, 16 + 4096, 16 + 4096 + 1048576};

static uint64_t ptr_bytes(uint32_t w) { return (4 + SEG_BITS[ptr_segment(w & 0x1fffffffu)]) / 8; }

ORC_API uint64_t orc_bytes(const orc_tree *tr) {         /* shared_tree::bytes :488-496 */
  uint64_t b = ptr_bytes(tr->root) + 8 + tr->n_leaves * (uint64_t)((tr->L + 1) / 2);
  for (int l = 0; l < tr->n_layers; ++l) {
    b += 8;
    for (uint64_t i = 0; i < 2 * tr->layer_n[l]; ++i) b += ptr_bytes(tr->layer_words[l][i]);
  }
  return b;
}

static uint8_t *put_be(uint8_t *o, uint64_t v, int nbytes) {
  for (int i = nbytes - 1; i >= 0; --i) *o++ = (uint8_t)(v >> (8 * i));
  return o;
}

static uint8_t *put_ptr(uint8_t *o, uint32_t w) {       /* pointer::serialize :133-142 */
  uint32_t idx = w & 0x1fffffffu;
  int seg = ptr_segment(idx);
  uint32_t off = (idx == NULL_INDEX) ? 0xfffffffu : idx - SEG_START[seg];
  int sh = (int)SEG_BITS[seg] - 4;
  *o++ = (uint8_t)((off >> sh) | (((w >> 29) & 1) << 4) | (((w >> 30) & 1) << 5) | (seg << 6));
  for (sh -= 8; sh >= 0; sh -= 8) *o++ = (uint8_t)(off >> sh);
  return o;
}

/* shared_tree::serialize (:504-513).  Writes into buf (capacity cap) and
 * returns the number of bytes, or 0 when cap is too small. */
ORC_API uint64_t orc_serialize(const orc_tree *tr, uint8_t *buf, uint64_t cap) {
  uint64_t need = orc_bytes(tr);
  if (cap < need) return 0;
  uint8_t *o = buf;
  o = put_ptr(o, tr->root);
  o = put_be(o, tr->n_leaves, 8);
  int lb = (tr->L + 1) / 2;
  for (uint64_t i = 0; i < tr->n_leaves; ++i) o = put_be(o, tr->leaves[i], lb);
  for (int l = 0; l < tr->n_layers; ++l) {
    o = put_be(o, tr->layer_n[l], 8);
    for (uint64_t i = 0; i < 2 * tr->layer_n[l]; ++i) o = put_ptr(o, tr->layer_words[l][i]);
  }
  return (uint64_t)(o - buf);
}

/* shared_tree::children / width (include/shared_tree.h:165, src/shared_tree.cpp:252-259),
 * computed bottom-up instead of by recursion. */
ORC_API uint64_t orc_width(const orc_tree *tr) {
  uint64_t *w = NULL;
  for (int l = 0; l < tr->n_layers; ++l) {
    uint64_t n = tr->layer_n[l];
    uint64_t *nw = malloc((n ? n : 1) * sizeof(uint64_t));
    for (uint64_t i = 0; i < n; ++i) {
      uint64_t s = 0;
      for (int c = 0; c < 2; ++c) {
        uint32_t x = tr->layer_words[l][2 * i + c];
        if (UL(x) == NULL_INDEX) continue;
        s += (l == 0) ? 1 : w[x & 0x1fffffffu];
      }
      nw[i] = s;
    }
    free(w); w = nw;
  }
  uint64_t r = w[tr->root & 0x1fffffffu];
  free(w);
  return r;
}
