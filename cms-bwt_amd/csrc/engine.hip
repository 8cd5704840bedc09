// engine.hip — the C ABI of include/cmsbwt.h over cmsbwt::Engine (engine.h).
#include <cstddef>
#include "engine.h"
#include "run_log.h"
#include "ctx_view.h"

// ---- ctx_view.h: the multi-GPU driver's view of a rank's engine
namespace cmsbwt {
CtxView ctx_view(const cmsbwt_ctx* c) {
  const Engine& e = *c->e;
  CtxView v;
  v.device = e.device;
  v.st = e.st;
  v.n = e.R.n;
  v.H = e.H;
  v.ndocs = e.ndocs;
  v.chars = e.chars;
  v.sn = e.sn;
  v.collTail = e.collTail;
  v.orderInvariant = e.orderInvariant;
  const void* h[8] = {e.hStart.p, e.hPos.p, e.hLen.p, e.hSmall.p, e.hChar.p, e.hIsa.p, e.hTonext.p, e.hNext.p};
  for (int k = 0; k < 8; k++) v.heads[k] = h[k];
  v.diff = e.diff.p;
  v.hasHead = e.hasHead.p;
  v.dmItems = e.dm.IS.K;
  v.dmItemPos = e.dm.IS.pos.p;
  v.dmGrp = e.dm.grp.p;
  v.dmU = e.dm.U;
  v.dmLabelBias = e.dm.labelBias;
  v.stats = e.stats;
  v.devicePeak = e.alloc.peak + e.sideAlloc.peak;
  return v;
}
void* ctx_alloc(cmsbwt_ctx* c, uint64_t bytes) {
  g_alloc = &c->e->alloc;
  (void)hipSetDevice(c->e->device);
  try {
    return c->e->alloc.get(std::max<uint64_t>(bytes, 1));
  } catch (const HipError& he) {
    throw CtxError{CMSBWT_EDEVICE, he.msg};
  }
}
void ctx_free(cmsbwt_ctx* c, void* p) {
  if (p) c->e->alloc.put(p);
}
uint64_t ctx_count_distinct(cmsbwt_ctx* c, const uint32_t* v, uint32_t k) {
  if (!k) return 0;
  Engine& e = *c->e;
  g_alloc = &e.alloc;
  try {
    DBuf<unsigned long long> r;
    r.alloc(1);
    r.zero(e.st);
    mk_count_distinct(v, k, r.p, e.st);
    return e.read1(r.p);
  } catch (const HipError& he) {
    throw CtxError{CMSBWT_EDEVICE, he.msg};
  }
}
}  // namespace cmsbwt

// =========================================================================
// C ABI
using cmsbwt::Engine;
using cmsbwt::HipError;


template <class F>
static int guard(cmsbwt_ctx* c, F&& f) {
  if (c && c->e) {
    cmsbwt::g_alloc = &c->e->alloc;
    (void)hipSetDevice(c->e->device);
  }
  try {
    f();
    return CMSBWT_OK;
  } catch (const cmsbwt::InputError& ie) {
    if (c) c->err = ie.msg;
    return ie.code;
  } catch (const cmsbwt::HipError& he) {
    if (c) c->err = he.msg;
    return CMSBWT_EDEVICE;
  } catch (const std::bad_alloc&) {
    if (c) c->err = "host out of memory";
    return CMSBWT_ELIMIT;
  } catch (const std::exception& ex) {  // std::system_error (threads), length_error, ...
    if (c) c->err = std::string("internal error: ") + ex.what();
    return CMSBWT_EINTERNAL;
  } catch (...) {  // nothing may unwind through the C ABI
    if (c) c->err = "internal error: unknown exception";
    return CMSBWT_EINTERNAL;
  }
}

extern "C" {

int cmsbwt_ctx_create(int device, cmsbwt_ctx** out) {
  if (!out) return CMSBWT_EARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0) return CMSBWT_EDEVICE;
  cmsbwt_ctx* c = new cmsbwt_ctx();
  int rc = guard(c, [&] { c->e = new Engine(device); });
  if (rc) { delete c; return rc; }
  *out = c;
  return CMSBWT_OK;
}

void cmsbwt_ctx_destroy(cmsbwt_ctx* ctx) {
  if (!ctx) return;
  delete ctx->e;
  delete ctx;
}

const char* cmsbwt_last_error(const cmsbwt_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int cmsbwt_load_reference_file(cmsbwt_ctx* ctx, const char* path) {
  if (!ctx || !path) return CMSBWT_EARG;
  return guard(ctx, [&] {
    std::string x, err;
    uint64_t fb = 0, rs = 0;
    if (!cmsbwt::read_reference(path, x, err, &fb, &rs)) throw cmsbwt::InputError{CMSBWT_EIO, err};
    ctx->e->hix.file_bytes = fb;
    ctx->e->hix.read_size = rs;
    ctx->e->load_reference_bytes(x);
  });
}

int cmsbwt_load_reference(cmsbwt_ctx* ctx, const uint8_t* ref, uint64_t len) {
  if (!ctx || (!ref && len)) return CMSBWT_EARG;
  return guard(ctx, [&] {
    ctx->e->hix.file_bytes = ctx->e->hix.read_size = len;
    ctx->e->load_reference_bytes(std::string((const char*)ref, len));
  });
}

int cmsbwt_load_collection_file(cmsbwt_ctx* ctx, const char* path, uint64_t prefix) {
  if (!ctx || !path) return CMSBWT_EARG;
  return guard(ctx, [&] {
    // Without -p the lines are resolved on the device over the raw bytes
    // (coll_read.hip); the -p cut (FN:1142-1146) keeps the host reader, as
    // does CMSBWT_HOST_READER=1.
    const char* hr = getenv("CMSBWT_HOST_READER");
    if (prefix == UINT64_MAX && !(hr && *hr && *hr != '0')) {
      ctx->e->load_collection_file_gpu(path);
    } else {
      cmsbwt::Collection c;
      std::string err;
      if (!cmsbwt::read_collection(path, prefix, c, err)) throw cmsbwt::InputError{CMSBWT_EIO, err};
      ctx->e->upload_collection(c);
    }
    struct stat sb;  // FN:221-224: ftello of the collection and the initial _sn
    const uint64_t fsz = stat(path, &sb) == 0 ? (uint64_t)sb.st_size : 0;
    ctx->e->stats.coll_file_bytes = fsz;
    ctx->e->stats.sn_initial = std::min<uint64_t>(fsz, prefix);
  });
}

int cmsbwt_load_collection_file_range(cmsbwt_ctx* ctx, const char* path, uint32_t rank, uint32_t world) {
  if (!ctx || !path || world == 0 || rank >= world) return CMSBWT_EARG;
  return guard(ctx, [&] {
    std::vector<uint64_t> b;
    uint64_t fsz = 0;
    std::string err;
    if (!cmsbwt::shard_bounds(path, world, b, fsz, err)) throw cmsbwt::InputError{CMSBWT_EIO, err};
    ctx->e->load_collection_file_gpu(path, b[rank], b[rank + 1] - b[rank]);
    ctx->e->stats.coll_file_bytes = fsz;
    ctx->e->stats.sn_initial = fsz;
  });
}

int cmsbwt_host_shard_bounds(const char* path, uint32_t world, uint64_t* bounds) {
  if (!path || !bounds || world == 0) return CMSBWT_EARG;
  std::vector<uint64_t> b;
  uint64_t fsz = 0;
  std::string err;
  if (!cmsbwt::shard_bounds(path, world, b, fsz, err)) return CMSBWT_EIO;
  for (uint32_t k = 0; k <= world; k++) bounds[k] = b[k];
  return CMSBWT_OK;
}

int cmsbwt_load_collection(cmsbwt_ctx* ctx, const uint8_t* text, const uint64_t* doc_off, uint64_t ndocs) {
  if (!ctx || !doc_off) return CMSBWT_EARG;
  return guard(ctx, [&] {
    cmsbwt::Collection c;
    c.off.assign(1, 0);
    for (uint64_t d = 0; d < ndocs; d++) {
      if (doc_off[d + 1] < doc_off[d]) throw cmsbwt::InputError{CMSBWT_EARG, "doc offsets not ascending"};
      c.text.insert(c.text.end(), text + doc_off[d], text + doc_off[d + 1]);
      c.text.push_back(2);
      c.off.push_back(c.text.size());
    }
    c.chars = c.text.size() - ndocs;
    c.sn = c.text.size();
    ctx->e->upload_collection(c);
  });
}

int cmsbwt_load_collection_synth(cmsbwt_ctx* ctx, uint64_t seed, uint64_t copy_begin, uint64_t ncopies, double p,
                                 int leading_empty_doc) {
  if (!ctx) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->load_synth(seed, copy_begin, ncopies, p, leading_empty_doc); });
}

int cmsbwt_ms_walk(cmsbwt_ctx* ctx) {
  if (!ctx) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->ms_walk(); });
}

int cmsbwt_merge(cmsbwt_ctx* ctx, int rle) {
  if (!ctx) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->merge(rle); });
}

int cmsbwt_step(cmsbwt_ctx* ctx, int rle) {
  if (!ctx) return CMSBWT_EARG;
  return guard(ctx, [&] {
    ctx->e->ms_walk();
    ctx->e->merge(rle);
  });
}

int cmsbwt_walk_import(cmsbwt_ctx* ctx, uint64_t heads, uint64_t ndocs, uint64_t chars, uint32_t flags,
                       const void* const* arrays) {
  if (!ctx || !arrays) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->walk_import(heads, ndocs, chars, flags, arrays); });
}

int cmsbwt_get_stats(const cmsbwt_ctx* ctx, cmsbwt_stats* out) {
  if (!ctx || !out) return CMSBWT_EARG;
  *out = ctx->e->stats;
  out->device_peak_bytes = ctx->e->alloc.peak + ctx->e->sideAlloc.peak;
  return CMSBWT_OK;
}

uint64_t cmsbwt_num_runs(const cmsbwt_ctx* ctx) { return ctx && ctx->e->merged ? ctx->e->nruns : 0; }

int cmsbwt_copy_runs(cmsbwt_ctx* ctx, uint8_t* out, uint64_t cap) {
  if (!ctx || !out) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->copy_runs(out, cap); });
}

int cmsbwt_write_output(cmsbwt_ctx* ctx, const char* outname, int rle) {
  if (!ctx || !outname) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->write_output(outname, rle); });
}

int cmsbwt_copy_array(cmsbwt_ctx* ctx, const char* name, void* out, uint64_t* bytes) {
  if (!ctx || !name) return CMSBWT_EARG;
  return guard(ctx, [&] {
    uint64_t b = ctx->e->copy_array(name, out);
    if (bytes) *bytes = b;
  });
}

// Device primitives checked against host results (tests/test_gpu_primitives.py):
// "exscan" / "inscan" (u32 plus, tile scan or rocPRIM per CMSBWT_ROCPRIM_SCAN,
// init 7 for the exclusive scan), "select" (flagged compaction).  Values are
// pseudo-random; `offset` shifts both buffers by that many elements (unaligned
// pointers), `inplace` runs a scan with out == in.
int cmsbwt_selftest(cmsbwt_ctx* ctx, const char* what, uint64_t n, uint64_t offset, int inplace, uint64_t* mismatches) {
  if (!ctx || !what || !mismatches || n >= (1ull << 31)) return CMSBWT_EARG;
  return guard(ctx, [&] {
    cmsbwt::Engine& e = *ctx->e;
    const std::string w = what;
    std::vector<uint32_t> in(n), fl(n), want;
    uint64_t z = 0x9E3779B97F4A7C15ull * (n + 1) + offset;
    for (uint64_t i = 0; i < n; i++) {
      z ^= z << 13; z ^= z >> 7; z ^= z << 17;
      in[i] = (uint32_t)(z >> 40) & 0xffff;  // sums stay below 2^32
      fl[i] = (uint32_t)(z >> 20) & 1;
    }
    cmsbwt::DBuf<uint32_t> a, b, f;
    a.alloc(n + offset + 1);
    b.alloc(n + offset + 1);
    f.alloc(n + 1);
    HIPCHK(hipMemcpyAsync(a.p + offset, in.data(), n * 4, hipMemcpyHostToDevice, e.st));
    HIPCHK(hipMemcpyAsync(f.p, fl.data(), n * 4, hipMemcpyHostToDevice, e.st));
    uint32_t* src = a.p + offset;
    uint32_t* dst = inplace ? src : b.p + offset;
    uint64_t cnt = n;
    if (w == "exscan") {
      e.exscan((const uint32_t*)src, dst, 7u, n);
      uint32_t acc = 7;
      for (uint64_t i = 0; i < n; i++) { want.push_back(acc); acc += in[i]; }
    } else if (w == "inscan") {
      e.inscan((const uint32_t*)src, dst, n, rocprim::plus<uint32_t>());
      uint32_t acc = 0;
      for (uint64_t i = 0; i < n; i++) { acc += in[i]; want.push_back(acc); }
    } else if (w == "select") {
      if (inplace) throw cmsbwt::InputError{CMSBWT_EARG, "select cannot run in place"};
      cnt = e.select_flagged(src, f.p, dst, (uint32_t)n);
      for (uint64_t i = 0; i < n; i++) if (fl[i]) want.push_back(in[i]);
    } else {
      throw cmsbwt::InputError{CMSBWT_EARG, "unknown selftest " + w};
    }
    std::vector<uint32_t> got(cnt);
    if (cnt) HIPCHK(hipMemcpyAsync(got.data(), dst, cnt * 4, hipMemcpyDeviceToHost, e.st));
    e.sync();
    uint64_t bad = cnt == want.size() ? 0 : 1 + (uint64_t)std::max(cnt, (uint64_t)want.size());
    for (uint64_t i = 0; i < std::min<uint64_t>(cnt, want.size()); i++) bad += got[i] != want[i];
    *mismatches = bad;
  });
}

int cmsbwt_host_read_collection(const char* path, uint64_t prefix, uint8_t* text, uint64_t text_cap,
                                uint64_t* text_len, uint64_t* doc_off, uint64_t doc_cap, uint64_t* ndocs,
                                uint64_t* sn) {
  if (!path) return CMSBWT_EARG;
  cmsbwt::Collection c;
  std::string err;
  if (!cmsbwt::read_collection(path, prefix, c, err)) return CMSBWT_EIO;
  const uint64_t nd = c.ndocs();
  if (text_len) *text_len = c.chars;
  if (ndocs) *ndocs = nd;
  if (sn) *sn = c.sn;
  if (text && text_cap < c.chars) return CMSBWT_EARG;
  if (doc_off && doc_cap < nd + 1) return CMSBWT_EARG;
  uint64_t o = 0;
  for (uint64_t d = 0; d < nd; d++) {
    uint64_t len = c.off[d + 1] - c.off[d] - 1;
    if (doc_off) doc_off[d] = o;
    if (text) memcpy(text + o, c.text.data() + c.off[d], len);
    o += len;
  }
  if (doc_off) doc_off[nd] = o;
  return CMSBWT_OK;
}

int cmsbwt_host_suffix_array(const uint8_t* s, uint64_t n, int32_t* sa_out) {
  if ((!s || !sa_out) && n) return CMSBWT_EARG;
  if (n >= (1ull << 31) - 2) return CMSBWT_ELIMIT;
  std::vector<int32_t> v(n);
  for (uint64_t i = 0; i < n; i++) v[i] = s[i];
  cmsbwt::suffix_array_sais(v.data(), sa_out, (int64_t)n, 256);
  return CMSBWT_OK;
}

// Whole run with the reference's log (FN keys in the reference's order,
// SURVEY.md App. C): initialize_reference FN:151-310, then the large- or
// small-reference collection pass (FN:1093-1628 / FN:312-936) and a writer.
static int run_impl(const cmsbwt_args* a, const char* ref_path, const char* coll_path, cmsbwt_stats* stats_out);

// ABI: cmsbwt_run keeps the version-1 layouts (no n_gpus/backend, stats up to
// host_queries), so a caller built against the old header never has fields
// read or written past its structs; cmsbwt_run_sized takes the caller's
// struct sizes (fields it does not know read as zero: one GPU, PEER).
int cmsbwt_abi_version(void) { return CMSBWT_ABI_VERSION; }

int cmsbwt_run_sized(const cmsbwt_args* a, uint64_t args_size, const char* ref_path, const char* coll_path,
                     cmsbwt_stats* stats_out, uint64_t stats_size) {
  if (!a || args_size < offsetof(cmsbwt_args, n_gpus)) return CMSBWT_EARG;
  cmsbwt_args full{};
  memcpy(&full, a, std::min<uint64_t>(args_size, sizeof full));
  cmsbwt_stats st{};
  const int rc = run_impl(&full, ref_path, coll_path, &st);
  if (stats_out) memcpy(stats_out, &st, std::min<uint64_t>(stats_size, sizeof st));
  return rc;
}

int cmsbwt_run(const cmsbwt_args* a, const char* ref_path, const char* coll_path, cmsbwt_stats* stats_out) {
  // (version-1 layout: n_gpus and backend are not read, include/cmsbwt.h)
  const char* v = getenv("CMSBWT_VERBOSE");
  if (v && *v && *v != '0')
    fprintf(stderr, "cmsbwt_run: version-1 arguments, one GPU (n_gpus/backend need cmsbwt_run_sized)\n");
  return cmsbwt_run_sized(a, offsetof(cmsbwt_args, n_gpus), ref_path, coll_path, stats_out,
                          offsetof(cmsbwt_stats, device_peak_bytes));
}

static int run_impl(const cmsbwt_args* a, const char* ref_path, const char* coll_path, cmsbwt_stats* stats_out) {
  if (!a || !ref_path || !coll_path || !a->outname) return CMSBWT_EARG;
  if (a->n_gpus > 1) return cmsbwt::run_multi(a, ref_path, coll_path, stats_out);  // multi.hip
  std::string out = a->outname;
  std::ofstream log(out + ".log");
  cmsbwt_ctx* ctx = nullptr;
  auto tc0 = std::chrono::steady_clock::now();
  int rc = cmsbwt_ctx_create(a->device, &ctx);
  const double tCtx = std::chrono::duration<double>(std::chrono::steady_clock::now() - tc0).count();
  if (rc) {
    log << "HIP device " << a->device << " unavailable\n";
    return rc;
  }
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto ms = [](std::chrono::steady_clock::time_point x, std::chrono::steady_clock::time_point y) {
    return (long long)std::chrono::duration_cast<std::chrono::milliseconds>(y - x).count();
  };
  auto fail = [&](int code) {
    log << ctx->err << "\n";
    cmsbwt_ctx_destroy(ctx);
    return code;
  };
  auto t0 = now();
  log << "About to read ref\n";
  {
    // FN:155-160: the reference is opened first (errno reported)
    FILE* f = fopen(ref_path, "r");
    if (!f) {
      log << "Error opening file of base sequence " << ref_path << ", errno=" << errno << '\n';
      cmsbwt_ctx_destroy(ctx);
      return CMSBWT_EIO;
    }
    fclose(f);
  }
  Engine& e = *ctx->e;
  {
    // the collection streams into HBM (reader threads, their own streams)
    // while the reference index is built on the engine stream; the device
    // reader then starts from the uploaded bytes.  Only for the device reader
    // path (no -p); errors are reported at the load, after the reference's.
    const char* hr = getenv("CMSBWT_HOST_READER");
    const char* ov = getenv("CMSBWT_OVERLAP_UPLOAD");
    if (a->prefix == UINT64_MAX && !(hr && *hr && *hr != '0') && !(ov && *ov == '0')) {
      try {
        e.upload_file_begin(coll_path);
      } catch (...) {
        // no overlap (e.g. out of pinned memory): the load reads the file itself
      }
    }
  }
  rc = cmsbwt_load_reference_file(ctx, ref_path);
  if (rc == CMSBWT_EDEVICE && e.pend.on) {
    // the index did not fit beside the collection's raw bytes: stop the
    // overlapped upload, free its buffer and build the index alone (the
    // collection is then read after it, as without the overlap)
    e.upload_file_end(false);
    cmsbwt::g_alloc = &e.alloc;
    e.alloc.trim();
    e.sideAlloc.trim();
    rc = cmsbwt_load_reference_file(ctx, ref_path);
  }
  if (rc) {
    if (e.hix.file_bytes) log << "n = " << e.hix.file_bytes << '\n';
    return fail(rc);
  }
  const cmsbwt_stats& s = e.stats;
  const uint64_t sn0 = [&] {  // FN:215-224: the collection is opened here, before augmenting
    struct stat sb;
    return stat(coll_path, &sb) == 0 ? (uint64_t)sb.st_size : ~0ull;
  }();
  if (cmsbwt::log_reference(log, s, sn0, a->prefix, coll_path, ms(t0, now()))) {
    cmsbwt_ctx_destroy(ctx);
    return CMSBWT_EIO;
  }
  auto t1 = now();
  rc = cmsbwt_load_collection_file(ctx, coll_path, a->prefix);
  if (rc) return fail(rc);
  const bool small = e.R.n < 1000000;  // FN:1792: small-reference path below 1e6
  cmsbwt::log_collection_start(log, s, e.R.n);
  rc = cmsbwt_ms_walk(ctx);
  if (rc) return fail(rc);
  log << "Finished parsing file of length: " << e.sn << "\n";
  rc = cmsbwt_merge(ctx, a->rle ? 1 : 0);
  if (rc) return fail(rc);
  cmsbwt::log_collection_end(log, s, small, e.sn, a->buffer_gb);
  rc = cmsbwt_write_output(ctx, out.c_str(), a->rle ? 1 : 0);
  if (rc) return fail(rc);
  log << "MS-walk kernel: " << s.ms_walk_kernel_ms << " ms; collection pass: " << ms(t1, now()) << " ms\n";
  log.flush();
  if (stats_out) *stats_out = e.stats;
  auto td0 = now();
  if (a->verbose) fprintf(stderr, "context %.3fs ", tCtx);
  if (a->verbose)
    fprintf(stderr, "index %.3fs (sa %.3fs, tables %.3fs) upload %.3fs walk %.3fs (kernel %.2fms) merge %.3fs write %.3fs runs %llu ",
            s.t_index_s, e.hix.t_sa, e.hix.t_lcp, s.t_upload_s, s.t_ms_walk_s, s.ms_walk_kernel_ms, s.t_merge_s, s.t_write_s,
            (unsigned long long)s.runs);
  cmsbwt_ctx_destroy(ctx);
  if (a->verbose) fprintf(stderr, "teardown %.3fs\n", std::chrono::duration<double>(now() - td0).count());
  return CMSBWT_OK;
}

// ---- position-sharded merge (include/cmsbwt.h "Multi-GPU merge")
int cmsbwt_dm_begin(cmsbwt_ctx* ctx, uint32_t world, uint32_t rank, uint64_t heads_total, uint64_t docs_total,
                    uint32_t flags, int rle) {
  if (!ctx) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->dm_begin(world, rank, heads_total, docs_total, flags, rle); });
}
int cmsbwt_dm_route_heads(cmsbwt_ctx* ctx, uint64_t* counts) {
  if (!ctx || !counts) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->dm_route_heads(counts); });
}
int cmsbwt_dm_pack_heads(cmsbwt_ctx* ctx, int32_t* out) {
  if (!ctx) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->dm_pack_heads(out); });
}
int cmsbwt_dm_group(cmsbwt_ctx* ctx, const int32_t* recv, uint64_t nrecv, uint32_t* sa_counts) {
  if (!ctx || !sa_counts) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->dm_group(recv, nrecv, sa_counts); });
}
int cmsbwt_dm_labels(cmsbwt_ctx* ctx, const uint32_t* sa_counts, uint64_t* back) {
  if (!ctx || !sa_counts) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->dm_labels(sa_counts, (unsigned long long*)back); });
}
int cmsbwt_dm_dbl_init(cmsbwt_ctx* ctx, const uint64_t* labels, uint64_t* active) {
  if (!ctx || !active) return CMSBWT_EARG;
  return guard(ctx, [&] { *active = ctx->e->dm_dbl_init((const unsigned long long*)labels); });
}
int cmsbwt_dm_dbl_route(cmsbwt_ctx* ctx, uint64_t h, uint64_t* counts) {
  if (!ctx || !counts) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->dm_dbl_route(h, counts); });
}
int cmsbwt_dm_dbl_pack(cmsbwt_ctx* ctx, int32_t* out) {
  if (!ctx) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->dm_dbl_pack(out); });
}
int cmsbwt_dm_dbl_sort(cmsbwt_ctx* ctx, const int32_t* recv, uint64_t nrecv, uint64_t* result) {
  if (!ctx) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->dm_dbl_sort(recv, nrecv, (unsigned long long*)result); });
}
int cmsbwt_dm_dbl_apply(cmsbwt_ctx* ctx, const uint64_t* back, uint64_t* active) {
  if (!ctx || !active) return CMSBWT_EARG;
  return guard(ctx, [&] { *active = ctx->e->dm_dbl_apply((const unsigned long long*)back); });
}
int cmsbwt_dm_pack_ranks(cmsbwt_ctx* ctx, int32_t* out) {
  if (!ctx) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->dm_pack_ranks(out); });
}
int cmsbwt_dm_load_ranks(cmsbwt_ctx* ctx, const int32_t* recv) {
  if (!ctx) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->dm_load_ranks(recv); });
}
int cmsbwt_dm_route_halo(cmsbwt_ctx* ctx, uint64_t* item_counts, uint64_t* word_counts) {
  if (!ctx || !item_counts || !word_counts) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->dm_route_halo(item_counts, word_counts); });
}
int cmsbwt_dm_pack_halo(cmsbwt_ctx* ctx, int32_t* headers, int32_t* words) {
  if (!ctx) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->dm_pack_halo(headers, words); });
}
int cmsbwt_dm_counter(cmsbwt_ctx* ctx, const int32_t* headers, uint64_t nitems, const int32_t* words, uint64_t nwords,
                      uint64_t* stats6) {
  if (!ctx || !stats6) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->dm_counter(headers, nitems, words, nwords, stats6); });
}
int cmsbwt_dm_units(cmsbwt_ctx* ctx, int64_t* units) {
  if (!ctx || !units) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->dm_units(units); });
}
int cmsbwt_dm_emit(cmsbwt_ctx* ctx, const int64_t* units, uint64_t* nlocal) {
  if (!ctx || !units || !nlocal) return CMSBWT_EARG;
  return guard(ctx, [&] { *nlocal = ctx->e->dm_emit(units); });
}
int cmsbwt_dm_copy_stream(cmsbwt_ctx* ctx, uint64_t* starts, uint8_t* chars) {
  if (!ctx) return CMSBWT_EARG;
  return guard(ctx, [&] { ctx->e->dm_copy_stream((unsigned long long*)starts, chars); });
}
int cmsbwt_dm_finish(cmsbwt_ctx* ctx, const uint64_t* const* starts, const uint8_t* const* chars,
                     const uint64_t* counts, const uint64_t* gstats) {
  if (!ctx || !starts || !chars || !counts || !gstats) return CMSBWT_EARG;
  return guard(ctx, [&] {
    ctx->e->dm_finish((const unsigned long long* const*)starts, chars, counts, gstats);
  });
}

}  // extern "C"

// The position-sharded merge's Engine members, in this translation unit (see
// the Makefile): engine.h's rocPRIM instantiations are emitted once.
#include "dist_merge.hip"
