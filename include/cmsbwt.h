/* cmsbwt.h — C ABI of the MI355X-native CMS-BWT engine (libcmsbwt.so).
 *
 * The reference (fmasillo/CMS-BWT) has no plugin/FFI surface: its boundary is
 * the `cmsbwt` process plus one C++ function,
 *     void computeBWT(Args, std::string& ref, std::string& coll)
 * (CMS-BWT.h:69, CMS-BWT-functions.cpp:1788-1797), which is non-reentrant,
 * owns all memory and reports errors with exit().  This header is what a
 * maintainer would bind instead (ctypes / cgo / JNI stubs in INTEGRATION.md):
 *   - cmsbwt_run()      replaces computeBWT() (+ main.cpp's list-file step);
 *   - the ctx API       exposes the hot path stage by stage for parity tests
 *                       and for callers that keep inputs resident in HBM.
 * Plain pointers and sizes only; all functions return 0 on success and a
 * CMSBWT_E* code otherwise (never exit()).  One context per thread.
 */
#ifndef CMSBWT_H
#define CMSBWT_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CMSBWT_OK 0
#define CMSBWT_EIO 1        /* file missing/unreadable (reference: exit(1))        */
#define CMSBWT_EARG 2       /* bad argument / call order                            */
#define CMSBWT_EINPUT 3     /* input on which the reference is undefined            */
#define CMSBWT_EDEVICE 4    /* HIP runtime error or HIP code object not loadable    */
#define CMSBWT_ELIMIT 5     /* size limit (reference int32/uint32 limits)           */
#define CMSBWT_EORDER 6     /* reserved, no longer returned: a sharded step that    */
                            /* meets comparator ambiguity is redone as a gather    */
                            /* step (every head to rank 0, one-GPU merge with the  */
                            /* std::map replay there; rank 0 then needs the memory */
                            /* of a one-GPU merge of all heads, ~135 B per head)   */
#define CMSBWT_EINTERNAL 7  /* unexpected host exception (thread creation, ...)     */

/* utils.h:8-14 struct Args, plus engine knobs. */
typedef struct cmsbwt_args {
  uint64_t prefix;      /* -p  (UINT64_MAX = whole file), FN:223, FN:1258-1263  */
  uint32_t buffer_gb;   /* -b  (small path memory knob only; no output effect)  */
  int32_t rle;          /* -r  1 = <out>.rl_bwt, 0 = <out>.bwt                  */
  const char* outname;  /* -o  basename (NULL = list file name)                 */
  int32_t device;       /* HIP device ordinal (rank 0's device with n_gpus > 1)  */
  int32_t verbose;      /* 1 = stage times on stderr                            */
  int32_t n_gpus;       /* ranks in this process (0/1 = one GPU); rank k runs on */
                        /* device (device + k) % device count, so ranks may     */
                        /* share a GPU (tests)                                  */
  int32_t backend;      /* n_gpus > 1: CMSBWT_BACKEND_PEER or _RCCL              */
} cmsbwt_args;

/* Transports of the in-process multi-GPU run (cmsbwt_run with n_gpus > 1).
 * PEER: all-to-alls, reductions and the run gather as pulls between the
 *   ranks' HBM buffers (hipMemcpyPeerAsync over xGMI; device-local copies
 *   when ranks share a GPU).
 * RCCL: the same exchanges as RCCL send/recv groups and all-reduces on a
 *   communicator made by ncclCommInitAll (needs one distinct GPU per rank;
 *   librccl is opened at run time). */
#define CMSBWT_BACKEND_PEER 0
#define CMSBWT_BACKEND_RCCL 1

/* Statistics mirrored from the reference .log (FN:1417-1422, 1452, 1515,
 * 1606-1608) plus engine timings. */
typedef struct cmsbwt_stats {
  uint64_t n;             /* augmented reference length _n                      */
  uint64_t sn;            /* _sn after the collection pass                      */
  uint64_t ndocs;         /* documents = D-1                                    */
  uint64_t chars;         /* collection sequence bytes N (separators excluded)  */
  uint64_t heads;         /* headNumber                                         */
  uint64_t positions;     /* phrasesSet.size()                                  */
  uint64_t keys;          /* uniqueHeadNumber (distinct (pos,len,isaNext))      */
  uint64_t rank;          /* final Rank                                         */
  uint64_t current_sum;   /* currentSum                                         */
  uint64_t counter_bad, counter_good, counter_nothing;
  uint64_t runs;          /* records in .rl_bwt (or runs of .bwt)               */
  uint64_t symbols;       /* sum of run lengths                                 */
  uint64_t order_violations; /* comparator ambiguities (match.h:27-33) found:   */
                             /* resolved by the host std::map replay          */
  double t_index_s, t_upload_s, t_ms_walk_s, t_merge_s, t_write_s;
  double ms_walk_kernel_ms;  /* device time of the MS-walk kernel               */
  double counter_kernel_ms;  /* device time of the counterSmallerThanHead kernel */
  uint64_t counter_work;     /* (item, offset) pairs visited by that kernel     */
  uint64_t order_invariant;  /* 1: every isaNext suffix starts with its head's   */
                             /* mismatch byte, comparator provably consistent   */
  /* the rest of the reference's .log keys */
  uint64_t ref_file_bytes;   /* `n = `              reference file size, FN:166 */
  uint64_t ref_read_size;    /* `Reference (size = ` read, before trimming, FN:205 */
  uint64_t coll_file_bytes;  /* `ftello(infile): `  collection file size, FN:222 */
  uint64_t sn_initial;       /* `sn: ` / `_sx.len: ` min(file size, -p), FN:223 */
  int64_t first_rank_to_head, last_rank_to_head;  /* FN:1476-1477 (-1: n/a)   */
  double t_augment_ms, t_sa_ms, t_isa_ms, t_lcp_ms, t_rmq_ms, t_bwt_ms;  /* FN:240-299 */
  double t_ranks_ms;         /* ranks .. next-head ranks, FN:1429-1498          */
  double t_libsais_int_ms;   /* head-string suffix sort, FN:1455-1461           */
  double t_counter_ms;       /* counterSmallerThanHead, FN:1517-1611            */
  uint64_t host_queries;     /* counter queries answered by the std::map replay */
  uint64_t device_peak_bytes; /* high-water mark of this context's HBM buffers  */
} cmsbwt_stats;

typedef struct cmsbwt_ctx cmsbwt_ctx;

/* Whole run, replaces computeBWT (FN:1788) for the CLI: index the reference,
 * read the collection with the reference's getline semantics, compute, write
 * <outname>.rl_bwt | .bwt (+ .counterSmallerThanHead_true when _n < 1e6,
 * FN:919-924) and <outname>.log.
 * ABI: cmsbwt_run reads and writes the version-1 layouts only (args up to
 * `verbose`, stats up to `host_queries`), so binaries built against the
 * version-1 header stay safe; cmsbwt_run_sized takes sizeof(cmsbwt_args) and
 * sizeof(cmsbwt_stats) of the caller's header (unknown trailing args fields
 * read as zero) and is what new callers use (n_gpus, backend,
 * device_peak_bytes).
 * NOTE: cmsbwt_run therefore IGNORES args->n_gpus and args->backend (it
 * cannot know whether the caller's struct holds them) and always runs on one
 * GPU; a caller that sets n_gpus > 1 must call cmsbwt_run_sized (the CLI and
 * the Python mirror do).  With CMSBWT_VERBOSE=1 cmsbwt_run says so on stderr. */
#define CMSBWT_ABI_VERSION 2
int cmsbwt_abi_version(void);
int cmsbwt_run(const cmsbwt_args* args, const char* ref_path, const char* coll_path,
               cmsbwt_stats* stats_out);
int cmsbwt_run_sized(const cmsbwt_args* args, uint64_t args_size, const char* ref_path, const char* coll_path,
                     cmsbwt_stats* stats_out, uint64_t stats_size);

int cmsbwt_ctx_create(int device, cmsbwt_ctx** out);
void cmsbwt_ctx_destroy(cmsbwt_ctx* ctx);
const char* cmsbwt_last_error(const cmsbwt_ctx* ctx);

/* initialize_reference (FN:151-310): read FASTA/raw, trim (FN:208-213),
 * augment (FN:231-237), then SA/ISA/LCP/PLCP/BWT and the walk tables built in
 * HBM (ref_index.hip; CMSBWT_HOST_INDEX=1 builds them on the host instead). */
int cmsbwt_load_reference_file(cmsbwt_ctx* ctx, const char* ref_path);
/* Same from bytes already read and trimmed (no augmentation applied yet). */
int cmsbwt_load_reference(cmsbwt_ctx* ctx, const uint8_t* ref, uint64_t len);

/* Collection reader (FN:1138-1275): getline semantics, '>'/blank lines split
 * documents, unterminated last line dropped, -p cut.  Uploads to HBM. */
int cmsbwt_load_collection_file(cmsbwt_ctx* ctx, const char* coll_path, uint64_t prefix);
/* Rank `rank` of `world`'s share of the collection file (multi-GPU ingest,
 * no -p): the documents closed inside bytes [bounds[rank], bounds[rank+1])
 * of cmsbwt_host_shard_bounds, read with the same getline semantics
 * (FN:1138-1147); the ranks' documents, in rank order, are the file's. */
int cmsbwt_load_collection_file_range(cmsbwt_ctx* ctx, const char* coll_path, uint32_t rank, uint32_t world);
/* Documents from host memory: doc k = text[doc_off[k] .. doc_off[k+1]). */
int cmsbwt_load_collection(cmsbwt_ctx* ctx, const uint8_t* text, const uint64_t* doc_off,
                           uint64_t ndocs);
/* Synthetic workload generated directly in HBM (synth.h):
 * copies [copy_begin, copy_begin+ncopies) of the reference seeded by `seed`. */
int cmsbwt_load_collection_synth(cmsbwt_ctx* ctx, uint64_t seed, uint64_t copy_begin,
                                 uint64_t ncopies, double p, int leading_empty_doc);

/* Hot path.  ms_walk = FN:1151-1212 (+ j-scan FN:1359-1385); merge = the
 * rest of FN:1387-1777 into device-resident runs. */
int cmsbwt_ms_walk(cmsbwt_ctx* ctx);
int cmsbwt_merge(cmsbwt_ctx* ctx, int rle);
/* ms_walk + merge, synchronised; the unit bench.py times. */
int cmsbwt_step(cmsbwt_ctx* ctx, int rle);

int cmsbwt_get_stats(const cmsbwt_ctx* ctx, cmsbwt_stats* out);
/* Packed 9-byte (uint64 LE length, uint8 char) records, FN:1708-1709. */
uint64_t cmsbwt_num_runs(const cmsbwt_ctx* ctx);
int cmsbwt_copy_runs(cmsbwt_ctx* ctx, uint8_t* out, uint64_t cap_bytes);
/* Write <outname>.rl_bwt (rle=1, runs of the last merge(rle=1)) or
 * <outname>.bwt (rle=0, expanded runs of the last merge(rle=0)). */
int cmsbwt_write_output(cmsbwt_ctx* ctx, const char* outname, int rle);

/* Stage arrays for parity tests, named like the oracle's dumps:
 * h_start h_pos h_len (u32) h_smaller h_lchar (u8) h_isa h_tonext (u32)
 * h_nexthead (u16) bucket (i64, pos-indexed) rank2head head2rank (i32, H+1)
 * bwtheads (u8, H) counters (u64, H+1).  Returns the byte size via *bytes
 * when out == NULL. */
int cmsbwt_copy_array(cmsbwt_ctx* ctx, const char* name, void* out, uint64_t* bytes);

/* Multi-GPU exchange (documents are sharded by contiguous ranges; the walk
 * and j-scan are document-local, the merge is global).  A shard's walk
 * results are copied out with cmsbwt_copy_array ("h_*", plus "diff" int32
 * n+1 and "hashead" uint8 n; dst may be host or device memory).  The merge
 * rank imports the concatenation of all shards in document order (heads)
 * with the summed diff and OR-ed hashead, then calls cmsbwt_merge.
 * arrays[] order: h_start h_pos h_len h_smaller h_lchar h_isa h_tonext
 * h_nexthead diff hashead.  flags bit 0: every shard reported
 * stats.order_invariant (lets the merge skip per-query ambiguity checks). */
int cmsbwt_walk_import(cmsbwt_ctx* ctx, uint64_t heads, uint64_t ndocs, uint64_t chars, uint32_t flags,
                       const void* const* arrays);

/* Multi-GPU merge, sharded by reference position (replaces
 * the single-process merge of FN:1387-1777 when documents are sharded over
 * `world` ranks).  Rank k owns positions [k*n/world, (k+1)*n/world) and the
 * head-string group labels [1 + k*H/world, 1 + (k+1)*H/world).  Every
 * pointer is DEVICE memory of this context's GPU; the caller moves data
 * between the calls (cmsbwt/dist.py: all-to-all / all-reduce over RCCL):
 *   ms_walk; dm_begin
 *   dm_route_heads -> counts; dm_pack_heads -> 5 int32/head; all-to-all
 *   dm_group(recv) -> buf[3n+1] (items, heads per SA rank; run difference
 *     array); all-reduce(sum) -> dm_labels -> back (label | unresolved << 32
 *     per received head); reverse all-to-all -> dm_dbl_init
 *   while (all-reduced active > 0): dm_dbl_route(h) -> counts;
 *     dm_dbl_pack -> 2 words/element; all-to-all; dm_dbl_sort -> result
 *     (label | unresolved << 32);
 *     reverse all-to-all -> dm_dbl_apply; h *= 2
 *   dm_pack_ranks -> 3 words/head (rank, next-head rank, BWT character);
 *     all-to-all (head counts) -> dm_load_ranks
 *   dm_route_halo -> counts; dm_pack_halo -> 6 words/item + nhr words;
 *     all-to-all -> dm_counter -> {bad, good, nothing, violations, errors, items}
 *   dm_units -> int64[2*(E+n-1)]; all-reduce(sum) -> dm_emit -> nlocal
 *     (rank 0: 0, its runs are placed directly);
 *   dm_copy_stream; gather to rank 0 -> dm_finish (rank 0) -> runs.
 * flags bit 0: every shard reported stats.order_invariant. */
int cmsbwt_dm_begin(cmsbwt_ctx* ctx, uint32_t world, uint32_t rank, uint64_t heads_total, uint64_t docs_total,
                    uint32_t flags, int rle);
int cmsbwt_dm_route_heads(cmsbwt_ctx* ctx, uint64_t* counts);
int cmsbwt_dm_pack_heads(cmsbwt_ctx* ctx, int32_t* out);
int cmsbwt_dm_group(cmsbwt_ctx* ctx, const int32_t* recv, uint64_t nrecv, uint32_t* sa_counts);
int cmsbwt_dm_labels(cmsbwt_ctx* ctx, const uint32_t* sa_counts, uint64_t* back);
int cmsbwt_dm_dbl_init(cmsbwt_ctx* ctx, const uint64_t* labels, uint64_t* active);
int cmsbwt_dm_dbl_route(cmsbwt_ctx* ctx, uint64_t h, uint64_t* counts);
int cmsbwt_dm_dbl_pack(cmsbwt_ctx* ctx, int32_t* out);
int cmsbwt_dm_dbl_sort(cmsbwt_ctx* ctx, const int32_t* recv, uint64_t nrecv, uint64_t* result);
int cmsbwt_dm_dbl_apply(cmsbwt_ctx* ctx, const uint64_t* back, uint64_t* active);
int cmsbwt_dm_pack_ranks(cmsbwt_ctx* ctx, int32_t* out);
int cmsbwt_dm_load_ranks(cmsbwt_ctx* ctx, const int32_t* recv);
int cmsbwt_dm_route_halo(cmsbwt_ctx* ctx, uint64_t* item_counts, uint64_t* word_counts);
int cmsbwt_dm_pack_halo(cmsbwt_ctx* ctx, int32_t* headers, int32_t* words);
int cmsbwt_dm_counter(cmsbwt_ctx* ctx, const int32_t* headers, uint64_t nitems, const int32_t* words,
                      uint64_t nwords, uint64_t* stats6);
int cmsbwt_dm_units(cmsbwt_ctx* ctx, int64_t* units);
int cmsbwt_dm_emit(cmsbwt_ctx* ctx, const int64_t* units, uint64_t* nlocal);
int cmsbwt_dm_copy_stream(cmsbwt_ctx* ctx, uint64_t* starts, uint8_t* chars);
/* rank 0: starts/chars/counts per source rank (device pointers); gstats =
 * {heads, keys, ndocs, chars, bad, good, nothing, violations} over all ranks */
int cmsbwt_dm_finish(cmsbwt_ctx* ctx, const uint64_t* const* starts, const uint8_t* const* chars,
                     const uint64_t* counts, const uint64_t* gstats);

/* Rank groups: the multi-GPU step over resident inputs (bench.py --gpus N
 * without torchrun; the same walk + position-sharded merge as cmsbwt_run with
 * n_gpus > 1, main.cpp:123 / FN:1788-1797).  cmsbwt_group_create makes
 * `world` rank contexts, rank k on device (device + k) % device count (ranks
 * may share a GPU; RCCL needs distinct GPUs); the caller loads each rank's
 * reference and document shard through cmsbwt_group_ctx + the ctx API (the
 * ranks' documents, in rank order, form the collection); cmsbwt_group_step
 * runs every rank's walk and the sharded merge (one host thread per rank,
 * synchronous) and leaves the runs and the global statistics in rank 0's
 * context.  per_rank (world entries, may be NULL) receives the stage times. */
typedef struct cmsbwt_group cmsbwt_group;
typedef struct cmsbwt_rank_times {
  double walk_ms, merge_ms, walk_kernel_ms;
  uint64_t heads, chars, device_peak_bytes;
  int32_t gathered; /* 1: the step ran as a gather step (one-GPU merge on rank 0) */
  int32_t device;
} cmsbwt_rank_times;
int cmsbwt_group_create(int world, int device, int backend, cmsbwt_group** out);
cmsbwt_ctx* cmsbwt_group_ctx(cmsbwt_group* g, int rank);
int cmsbwt_group_step(cmsbwt_group* g, int rle, cmsbwt_rank_times* per_rank);
const char* cmsbwt_group_last_error(const cmsbwt_group* g);
void cmsbwt_group_destroy(cmsbwt_group* g);

/* Self-test of the device scan / compaction primitives against host results
 * (what = "exscan" | "inscan" | "select"; offset = element offset of both
 * buffers, inplace = scan with out == in).  *mismatches = 0 when equal. */
int cmsbwt_selftest(cmsbwt_ctx* ctx, const char* what, uint64_t n, uint64_t offset, int inplace,
                    uint64_t* mismatches);

/* Host-only helpers (no GPU needed), exposed for tests of the host logic:
 * the collection reader (FN:1138-1275) and the reference suffix array
 * (libsais call site FN:247).  For the reader, pass NULL buffers to query
 * sizes; text excludes separators, doc_off has ndocs+1 entries. */
int cmsbwt_host_read_collection(const char* path, uint64_t prefix, uint8_t* text, uint64_t text_cap,
                                uint64_t* text_len, uint64_t* doc_off, uint64_t doc_cap, uint64_t* ndocs,
                                uint64_t* sn);
int cmsbwt_host_suffix_array(const uint8_t* s, uint64_t n, int32_t* sa_out);
/* Byte bounds (world + 1 entries) of the collection shards: bounds[k] is the
 * first byte after the last document-ending line (empty or '>') that starts
 * before k * size / world; bounds[0] = 0, bounds[world] = size. */
int cmsbwt_host_shard_bounds(const char* coll_path, uint32_t world, uint64_t* bounds);

#ifdef __cplusplus
}
#endif
#endif /* CMSBWT_H */
