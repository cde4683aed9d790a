/*
 * mccs_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference mCCS allreduce path, used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the CHECKER.
 * The product path (mccs_amd/, libmccs_hip.so) never links, loads or calls
 * anything in this directory.
 *
 * Restated from (paths relative to the reference root):
 *   element ops ........ src/collectives/src/reduce_kernel.h:16-30 (FuncSum/FuncProd),
 *                        :32-46 (generic Max/Min), :237-259 (FuncSum<half> = __hadd2,
 *                        fp16 RNE), :338-404 (Max/Min<half>: fmaxf/fminf), :357-384 (bf16)
 *   reduce / reduce-copy  src/collectives/src/common_kernel.h:485-685 (ReduceOrCopyMulti:
 *                        vals = src[0]; vals = fn(vals, src[i]); stored to every dst)
 *   ring schedule ...... src/collectives/src/all_reduce.h:10-87 (runRing: chunk size,
 *                        loop size, realChunkSize rounding, chunk→ring-index ownership,
 *                        per-hop operand order fn(own input, received))
 *   operand order ...... src/collectives/src/prims_simple.h:174-177 (srcs[0] = user input,
 *                        srcs[1] = received FIFO slot)
 *   allgather .......... src/collectives/src/all_gather.h:7-79
 *   task schema ........ src/mccs/src/proxy/plan.rs:602-635 (get_task_schema)
 *   ring index ......... src/mccs/src/proxy/engine.rs:269-320 (user_ranks, index)
 *
 * Parity pinning: the integer path is pinned by the
 * reference's allreduce_proto known-answer test (src/mccs_examples/
 * allreduce_proto/src/main.rs:111: 2042*n + n(n-1)/2); the ABI layout by
 * compiling the reference devcomm.h (oracle/_ref/ref_layout); fp16/fp32
 * summation ORDER is restated from all_reduce.h and is not pinned by any
 * reference fp test ("parity unpinned" beyond exact-sum fixtures).
 *
 * dtype codes follow mccsDevDataType_t (collectives.h:177-192), op codes
 * mccsDevRedOp_t (collectives.h:194-198).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#if defined(__F16C__) && defined(__AVX2__)
#include <immintrin.h>
#endif

enum { T_I8 = 0, T_U8, T_I32, T_U32, T_I64, T_U64, T_F16, T_F32, T_F64, T_BF16, T_NUM };
enum { OP_SUM = 0, OP_PROD, OP_MAX, OP_MIN, OP_NUM };

static const size_t kElemSize[T_NUM] = {1, 1, 4, 4, 8, 8, 2, 4, 8, 2};

size_t oracle_elem_size(int dtype) { return (dtype >= 0 && dtype < T_NUM) ? kElemSize[dtype] : 0; }

/* ---------------- IEEE binary16 / bfloat16 <-> binary32 ------------------ */
static float u32_as_f32(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t f32_as_u32(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

float oracle_half_to_float(uint16_t h) {
  uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  uint32_t exp = (h >> 10) & 0x1f, man = h & 0x3ffu;
  if (exp == 0) {
    if (man == 0) return u32_as_f32(sign);
    /* subnormal: man * 2^-24, exact in binary32 */
    float v = (float)man * 5.9604644775390625e-08f;
    return sign ? -v : v;
  }
  if (exp == 31) return u32_as_f32(sign | 0x7f800000u | (man << 13) | (man ? 0x00400000u : 0));
  return u32_as_f32(sign | ((exp + 112) << 23) | (man << 13));
}

/* binary32 -> binary16, round to nearest even (the rounding of __float2half_rn /
 * __hadd's result).  Double rounding through binary32 is innocuous for + and
 * x because 24 >= 2*11+2. */
uint16_t oracle_float_to_half(float f) {
  uint32_t u = f32_as_u32(f);
  uint32_t sign = (u >> 16) & 0x8000u;
  uint32_t a = u & 0x7fffffffu;
  if (a >= 0x7f800000u) /* inf / nan */
    return (uint16_t)(sign | 0x7c00u | (a > 0x7f800000u ? 0x200u : 0));
  if (a >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u); /* rounds to >= 65520 -> inf */
  if (a < 0x38800000u) {                                   /* result subnormal or zero */
    /* value = a as float; half subnormal unit = 2^-24 */
    float v = u32_as_f32(a) * 16777216.0f; /* exact scaling by 2^24 */
    /* round v to nearest even integer */
    float r = rintf(v); /* default FE_TONEAREST */
    return (uint16_t)(sign | (uint32_t)r);
  }
  uint32_t exp = (a >> 23) - 112, man = a & 0x7fffffu;
  uint32_t h = (exp << 10) | (man >> 13);
  uint32_t rem = man & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h += 1; /* carry may bump exponent: ok */
  return (uint16_t)(sign | h);
}

float oracle_bf16_to_float(uint16_t b) { return u32_as_f32((uint32_t)b << 16); }

uint16_t oracle_float_to_bf16(float f) {
  uint32_t u = f32_as_u32(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u); /* quiet nan */
  uint32_t r = u + 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(r >> 16);
}

/* ---------------- element ops: acc[i] = fn(a[i], b[i]) ------------------- */
/* fn(x, y) for each (dtype, op); x is the FIRST operand as in FuncSum(x, y). */
#define DEF_INT_OPS(NAME, T, UT)                                                              \
  static void NAME(int op, T *out, const T *x, const T *y, size_t n) {                         \
    size_t i;                                                                                  \
    switch (op) {                                                                              \
      case OP_SUM: for (i = 0; i < n; ++i) out[i] = (T)((UT)x[i] + (UT)y[i]); break;           \
      case OP_PROD: for (i = 0; i < n; ++i) out[i] = (T)((UT)x[i] * (UT)y[i]); break;          \
      case OP_MAX: for (i = 0; i < n; ++i) out[i] = (x[i] < y[i]) ? y[i] : x[i]; break;        \
      case OP_MIN: for (i = 0; i < n; ++i) out[i] = (x[i] < y[i]) ? x[i] : y[i]; break;        \
    }                                                                                          \
  }
DEF_INT_OPS(ops_i8, int8_t, uint8_t)
DEF_INT_OPS(ops_u8, uint8_t, uint8_t)
DEF_INT_OPS(ops_i32, int32_t, uint32_t)
DEF_INT_OPS(ops_u32, uint32_t, uint32_t)
DEF_INT_OPS(ops_i64, int64_t, uint64_t)
DEF_INT_OPS(ops_u64, uint64_t, uint64_t)

#define DEF_FP_OPS(NAME, T)                                                                    \
  static void NAME(int op, T *out, const T *x, const T *y, size_t n) {                         \
    size_t i;                                                                                  \
    switch (op) {                                                                              \
      case OP_SUM: for (i = 0; i < n; ++i) out[i] = x[i] + y[i]; break;                        \
      case OP_PROD: for (i = 0; i < n; ++i) out[i] = x[i] * y[i]; break;                       \
      case OP_MAX: for (i = 0; i < n; ++i) out[i] = (x[i] < y[i]) ? y[i] : x[i]; break;        \
      case OP_MIN: for (i = 0; i < n; ++i) out[i] = (x[i] < y[i]) ? x[i] : y[i]; break;        \
    }                                                                                          \
  }
DEF_FP_OPS(ops_f32, float)
DEF_FP_OPS(ops_f64, double)

/* half and bfloat16: computed in binary32, rounded once (== __hadd2/__hmul2,
 * and == fmaxf/fminf then round for Max/Min, reduce_kernel.h:338-404). */
static float fp_apply(int op, float a, float b) {
  switch (op) {
    case OP_SUM: return a + b;
    case OP_PROD: return a * b;
    case OP_MAX: return fmaxf(a, b);
    default: return fminf(a, b);
  }
}
static void ops_f16(int op, uint16_t *out, const uint16_t *x, const uint16_t *y, size_t n) {
  for (size_t i = 0; i < n; ++i)
    out[i] = oracle_float_to_half(fp_apply(op, oracle_half_to_float(x[i]), oracle_half_to_float(y[i])));
}
static void ops_bf16(int op, uint16_t *out, const uint16_t *x, const uint16_t *y, size_t n) {
  for (size_t i = 0; i < n; ++i)
    out[i] = oracle_float_to_bf16(fp_apply(op, oracle_bf16_to_float(x[i]), oracle_bf16_to_float(y[i])));
}

/* out = fn(x, y) elementwise over n elements (out may alias x or y). */
int oracle_apply(int dtype, int op, void *out, const void *x, const void *y, size_t n) {
  if (op < 0 || op >= OP_NUM) return -1;
  switch (dtype) {
    case T_I8: ops_i8(op, out, x, y, n); break;
    case T_U8: ops_u8(op, out, x, y, n); break;
    case T_I32: ops_i32(op, out, x, y, n); break;
    case T_U32: ops_u32(op, out, x, y, n); break;
    case T_I64: ops_i64(op, out, x, y, n); break;
    case T_U64: ops_u64(op, out, x, y, n); break;
    case T_F16: ops_f16(op, out, x, y, n); break;
    case T_F32: ops_f32(op, out, x, y, n); break;
    case T_F64: ops_f64(op, out, x, y, n); break;
    case T_BF16: ops_bf16(op, out, x, y, n); break;
    default: return -1;
  }
  return 0;
}

/* ReduceOrCopyMulti (common_kernel.h:485-685): vals = src[0];
 * vals = fn(vals, src[i]) for i = 1..nsrcs-1; vals stored to every dst. */
int oracle_reduce_copy(int dtype, int op, const void *const *srcs, int nsrcs, void *const *dsts,
                       int ndsts, size_t count) {
  if (nsrcs < 1 || ndsts < 1 || dtype < 0 || dtype >= T_NUM) return -1;
  size_t es = kElemSize[dtype];
  char *acc = (char *)malloc(count * es + 1);
  if (!acc) return -2;
  memcpy(acc, srcs[0], count * es);
  for (int i = 1; i < nsrcs; ++i)
    if (oracle_apply(dtype, op, acc, acc, srcs[i], count)) { free(acc); return -1; }
  for (int d = 0; d < ndsts; ++d) memcpy(dsts[d], acc, count * es);
  free(acc);
  return 0;
}

/* ---------------- host schema (plan.rs:602-635) -------------------------- */
void oracle_task_schema(size_t total_bytes, int nchannels_cfg, int *nch_out, int *nthreads_out) {
  size_t nch = (size_t)nchannels_cfg, nthr = 512; /* MCCS_SIMPLE_MAX_N_THREADS */
  while (total_bytes < nch * nthr * 64 /* MCCS_SIMPLE_THREAD_THRESHOLD */) {
    if (nch >= 2) nch -= 1;
    else if (nthr % 128 == 0) nthr /= 2;
    else break;
  }
  nthr += 32;
  if (nthr / 32 < 3) nthr = 32 * 3;
  *nch_out = (int)nch;
  *nthreads_out = (int)nthr;
}

/* ---------------- ring schedule (all_reduce.h:10-87) --------------------- */
static long long div_up_ll(long long x, long long y) { return (x + y - 1) / y; }
static long long round_up_ll(long long x, long long y) { return (x + y - 1) - (x + y - 1) % y; }

/* Calls visit(ctx, bid, chunk, offset, nelem) for every (channel, chunk) of
 * the AllReduce loop exactly as runRing walks it.  `chunk` is a ring index. */
typedef void (*chunk_visit_fn)(void *ctx, int bid, int chunk, long long offset, long long nelem);

int oracle_ring_walk(size_t count, int nranks, int nchannels, int nthreads_ref, int buff_size,
                     int elem_size, chunk_visit_fn visit, void *ctx) {
  if (nranks < 1 || nchannels < 1 || elem_size < 1 || nthreads_ref <= 32) return -1;
  const long long chunkSize = (long long)(int)(buff_size / 8 / elem_size * 4); /* CHUNKSTEPS = 4 */
  const long long loopSize = (long long)nchannels * nranks * chunkSize;
  const long long size = (long long)count;
  const long long gran = (long long)(nthreads_ref - 32) * 8 / elem_size;
  for (long long gridOffset = 0; gridOffset < size; gridOffset += loopSize) {
    long long rcs = chunkSize;
    long long rest = div_up_ll(size - gridOffset, (long long)nchannels * nranks);
    if (rest < rcs) rcs = rest;
    rcs = round_up_ll(rcs, gran);
    rcs = (long long)(int)rcs;
    for (int bid = 0; bid < nchannels; ++bid)
      for (int chunk = 0; chunk < nranks; ++chunk) {
        long long offset = gridOffset + (long long)bid * nranks * rcs + (long long)chunk * rcs;
        long long nelem = rcs < size - offset ? rcs : size - offset;
        visit(ctx, bid, chunk, offset, nelem);
      }
  }
  return 0;
}

struct ring_ctx {
  int dtype, op, nranks;
  size_t es;
  const void *const *inputs;
  void *const *outputs;
  const int *ring_orders; /* [bid][pos] user rank at ring position pos, NULL = identity */
  int *owner;             /* optional: owner user rank per element */
  char *tmp;
  int err;
};

/* user rank holding ring index k on channel bid (engine.rs:274-286):
 * index(r) = (pos(r) - pos(0)) mod n  =>  rank at index k = ring[(pos(0) + k) mod n] */
static int rank_at_index(const struct ring_ctx *c, int bid, int k) {
  int n = c->nranks;
  k %= n;
  if (!c->ring_orders) return k;
  const int *ring = c->ring_orders + (size_t)bid * n;
  int pos0 = 0;
  while (pos0 < n && ring[pos0] != 0) ++pos0;
  return ring[(pos0 + k) % n];
}

static void ring_visit(void *vctx, int bid, int chunk, long long offset, long long nelem) {
  struct ring_ctx *c = (struct ring_ctx *)vctx;
  if (nelem <= 0 || c->err) return;
  const int n = c->nranks;
  const size_t es = c->es, bytes = (size_t)nelem * es, off = (size_t)offset * es;
  /* acc = x[idx chunk+1]; then acc = fn(x[idx chunk+j], acc), j = 2..n */
  memcpy(c->tmp, (const char *)c->inputs[rank_at_index(c, bid, chunk + 1)] + off, bytes);
  for (int j = 2; j <= n; ++j) {
    const char *x = (const char *)c->inputs[rank_at_index(c, bid, chunk + j)] + off;
    if (oracle_apply(c->dtype, c->op, c->tmp, x, c->tmp, (size_t)nelem)) { c->err = 1; return; }
  }
  if (c->outputs)
    for (int r = 0; r < n; ++r) memcpy((char *)c->outputs[r] + off, c->tmp, bytes);
  if (c->owner) {
    int own = rank_at_index(c, bid, chunk);
    for (long long e = 0; e < nelem; ++e) c->owner[offset + e] = own;
  }
}

/* Restates the result of mccsKernel_AllReduce_RING_SIMPLE_<op>_<T> on every
 * rank.  inputs[r]/outputs[r] are rank r's send/recv buffers (outputs may
 * alias inputs: the walk reads every input chunk before any output write of
 * that chunk, and chunks are disjoint).  ring_orders: nchannels x nranks ring
 * lists (comm_patterns_override), NULL = 0->1->...->n-1 on every channel.
 * nranks == 1 is defined as a copy (the reference builds no connectors). */
int oracle_ring_allreduce(int dtype, int op, int nranks, const void *const *inputs,
                          void *const *outputs, size_t count, int nchannels, int nthreads_ref,
                          int buff_size, const int *ring_orders, int *owner_out) {
  if (dtype < 0 || dtype >= T_NUM || op < 0 || op >= OP_NUM || nranks < 1) return -1;
  struct ring_ctx c;
  memset(&c, 0, sizeof c);
  c.dtype = dtype; c.op = op; c.nranks = nranks; c.es = kElemSize[dtype];
  c.inputs = inputs; c.outputs = outputs; c.ring_orders = ring_orders; c.owner = owner_out;
  if (nranks == 1) {
    if (outputs && outputs[0] != inputs[0]) memmove(outputs[0], inputs[0], count * c.es);
    if (owner_out) for (size_t e = 0; e < count; ++e) owner_out[e] = 0;
    return 0;
  }
  /* snapshot inputs if any output aliases an input: the walk writes outputs of
   * chunk k on every rank before reading chunk k+1, which is fine, but keep
   * the restatement independent of that argument. */
  const void **in_copy = (const void **)calloc((size_t)nranks, sizeof(void *));
  if (!in_copy) return -2;
  for (int r = 0; r < nranks; ++r) {
    void *p = malloc(count * c.es + 1);
    if (!p) return -2;
    memcpy(p, inputs[r], count * c.es);
    in_copy[r] = p;
  }
  c.inputs = in_copy;
  /* largest chunk: buff_size/8*4 bytes rounded up to the thread granule */
  {
    size_t gran_b = (size_t)(nthreads_ref > 32 ? nthreads_ref - 32 : 1) * 8;
    size_t chunk_b = (size_t)buff_size / 2;
    c.tmp = (char *)malloc((chunk_b + gran_b - 1) / gran_b * gran_b + 64);
  }
  int rc = c.tmp ? oracle_ring_walk(count, nranks, nchannels, nthreads_ref, buff_size, (int)c.es,
                                    ring_visit, &c)
                 : -2;
  free(c.tmp);
  for (int r = 0; r < nranks; ++r) free((void *)in_copy[r]);
  free(in_copy);
  return rc ? rc : (c.err ? -3 : 0);
}

/* ---------------- the same ring result, chunk-parallel ------------------- */
/* For the BASELINE sizes (8 x 1 GiB fp16 = 4 Gi element-ops): the chunks of
 * the walk are disjoint, and each chunk's value depends only on the inputs at
 * its own offsets, so chunks may be evaluated in any order on any thread.
 * Writes the common result of every rank into `output`, which must not
 * overlap any input (no snapshot is taken).  Elements of the walk in
 * [lo, hi) only when hi > lo (hi = 0: all). */
struct walk_rec { int bid, chunk; long long offset, nelem; };
struct walk_list { struct walk_rec *v; size_t n, cap; long long lo, hi; int err; };

static void collect_visit(void *vctx, int bid, int chunk, long long offset, long long nelem) {
  struct walk_list *w = (struct walk_list *)vctx;
  if (nelem <= 0 || w->err) return;
  if (w->hi > w->lo) { /* clip to [lo, hi) */
    long long a = offset > w->lo ? offset : w->lo, b = offset + nelem < w->hi ? offset + nelem : w->hi;
    if (b <= a) return;
    offset = a; nelem = b - a;
  }
  if (w->n == w->cap) {
    size_t cap = w->cap ? 2 * w->cap : 1024;
    struct walk_rec *v = (struct walk_rec *)realloc(w->v, cap * sizeof *v);
    if (!v) { w->err = 1; return; }
    w->v = v; w->cap = cap;
  }
  w->v[w->n++] = (struct walk_rec){bid, chunk, offset, nelem};
}

struct mt_ring_job {
  struct ring_ctx c; /* per-thread copy; c.outputs[0] is the single output */
  const struct walk_list *w;
  size_t first, step;
};

static void *mt_ring_worker(void *arg) {
  struct mt_ring_job *j = (struct mt_ring_job *)arg;
  struct ring_ctx *c = &j->c;
  const int n = c->nranks;
  for (size_t i = j->first; i < j->w->n && !c->err; i += j->step) {
    const struct walk_rec *r = &j->w->v[i];
    const size_t off = (size_t)r->offset * c->es, bytes = (size_t)r->nelem * c->es;
    char *acc = (char *)c->outputs[0] + off;
    /* the order of ring_visit: acc = x[idx chunk+1]; acc = fn(x[idx chunk+j], acc) */
    memcpy(acc, (const char *)c->inputs[rank_at_index(c, r->bid, r->chunk + 1)] + off, bytes);
    for (int k = 2; k <= n; ++k) {
      const char *x = (const char *)c->inputs[rank_at_index(c, r->bid, r->chunk + k)] + off;
      if (oracle_apply(c->dtype, c->op, acc, x, acc, (size_t)r->nelem)) c->err = 1;
    }
  }
  return NULL;
}

int oracle_ring_allreduce_mt(int dtype, int op, int nranks, const void *const *inputs, void *output,
                             size_t count, int nchannels, int nthreads_ref, int buff_size,
                             const int *ring_orders, long long lo, long long hi, int nthreads) {
  if (dtype < 0 || dtype >= T_NUM || op < 0 || op >= OP_NUM || nranks < 2) return -1;
  struct walk_list w;
  memset(&w, 0, sizeof w);
  w.lo = lo; w.hi = hi;
  int rc = oracle_ring_walk(count, nranks, nchannels, nthreads_ref, buff_size, (int)kElemSize[dtype],
                            collect_visit, &w);
  if (rc || w.err) { free(w.v); return rc ? rc : -2; }
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  struct mt_ring_job *jobs = (struct mt_ring_job *)calloc((size_t)nthreads, sizeof *jobs);
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof *th);
  void *outs[1] = {output};
  if (!jobs || !th) { free(jobs); free(th); free(w.v); return -2; }
  for (int t = 0; t < nthreads; ++t) {
    struct ring_ctx *c = &jobs[t].c;
    c->dtype = dtype; c->op = op; c->nranks = nranks; c->es = kElemSize[dtype];
    c->inputs = inputs; c->outputs = outs; c->ring_orders = ring_orders;
    jobs[t].w = &w; jobs[t].first = (size_t)t; jobs[t].step = (size_t)nthreads;
    if (t && pthread_create(&th[t], NULL, mt_ring_worker, &jobs[t]) != 0) {
      mt_ring_worker(&jobs[t]);
      th[t] = 0;
    }
  }
  mt_ring_worker(&jobs[0]);
  int err = jobs[0].c.err;
  for (int t = 1; t < nthreads; ++t) {
    if (th[t]) pthread_join(th[t], NULL);
    err |= jobs[t].c.err;
  }
  free(jobs); free(th); free(w.v);
  return err ? -3 : 0;
}

/* AllGather (all_gather.h:7-79, byte-count semantics of the int8 kernel):
 * rank r's output holds every rank's input block at offset rank*count. */
int oracle_ring_allgather(int nranks, const void *const *inputs, void *const *outputs, size_t nbytes) {
  for (int r = 0; r < nranks; ++r)
    for (int s = 0; s < nranks; ++s)
      memcpy((char *)outputs[r] + (size_t)s * nbytes, inputs[s], nbytes);
  return 0;
}

/* ---------------- CPU baseline: threaded elementwise reduce -------------- */
struct mt_job {
  int dtype, op, nsrcs;
  const void *const *srcs;
  void *dst;
  size_t lo, hi;
};

static void reduce_range(const struct mt_job *j) {
  size_t es = kElemSize[j->dtype], n = j->hi - j->lo;
  char *dst = (char *)j->dst + j->lo * es;
  const char *s0 = (const char *)j->srcs[0] + j->lo * es;
#if defined(__F16C__) && defined(__AVX2__)
  if (j->dtype == T_F16 && j->op == OP_SUM && j->nsrcs == 2) {
    const char *s1 = (const char *)j->srcs[1] + j->lo * es;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
      __m256 a = _mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(s0 + 2 * i)));
      __m256 b = _mm256_cvtph_ps(_mm_loadu_si128((const __m128i *)(s1 + 2 * i)));
      _mm_storeu_si128((__m128i *)(dst + 2 * i),
                       _mm256_cvtps_ph(_mm256_add_ps(a, b), _MM_FROUND_TO_NEAREST_INT));
    }
    if (i < n) ops_f16(OP_SUM, (uint16_t *)(dst + 2 * i), (const uint16_t *)(s0 + 2 * i),
                       (const uint16_t *)(s1 + 2 * i), n - i);
    return;
  }
#endif
  if (j->dtype == T_F32 && j->op == OP_SUM && j->nsrcs == 2) {
    const float *a = (const float *)s0, *b = (const float *)j->srcs[1] + j->lo;
    float *c = (float *)dst;
    for (size_t i = 0; i < n; ++i) c[i] = a[i] + b[i];
    return;
  }
  if (j->dtype == T_F32 && j->op == OP_SUM && j->nsrcs > 2) {
    /* n-source sum in L1-sized blocks: every source read once, dst written once */
    float *c = (float *)dst;
    for (size_t b = 0; b < n; b += 2048) {
      const size_t m = n - b < 2048 ? n - b : 2048;
      const float *a0 = (const float *)s0 + b;
      for (size_t i = 0; i < m; ++i) c[b + i] = a0[i];
      for (int k = 1; k < j->nsrcs; ++k) {
        const float *ak = (const float *)j->srcs[k] + j->lo + b;
        for (size_t i = 0; i < m; ++i) c[b + i] = ak[i] + c[b + i];
      }
    }
    return;
  }
  if (dst != s0) memcpy(dst, s0, n * es);
  for (int i = 1; i < j->nsrcs; ++i)
    oracle_apply(j->dtype, j->op, dst, dst, (const char *)j->srcs[i] + j->lo * es, n);
}

static void *mt_worker(void *arg) { reduce_range((const struct mt_job *)arg); return NULL; }

/* dst = reduce(srcs) split over nthreads pthreads (contiguous ranges). */
int oracle_reduce_mt(int dtype, int op, const void *const *srcs, int nsrcs, void *dst, size_t count,
                     int nthreads) {
  if (dtype < 0 || dtype >= T_NUM || op < 0 || op >= OP_NUM || nsrcs < 1) return -1;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 1024) nthreads = 1024;
  struct mt_job *jobs = (struct mt_job *)calloc((size_t)nthreads, sizeof *jobs);
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof *th);
  if (!jobs || !th) { free(jobs); free(th); return -2; }
  size_t per = (count + (size_t)nthreads - 1) / (size_t)nthreads;
  per = (per + 63) & ~(size_t)63;
  int started = 0;
  for (int t = 0; t < nthreads; ++t) {
    size_t lo = (size_t)t * per, hi = lo + per;
    if (lo >= count) break;
    if (hi > count) hi = count;
    jobs[t] = (struct mt_job){dtype, op, nsrcs, srcs, dst, lo, hi};
    if (t == 0) continue;
    if (pthread_create(&th[t], NULL, mt_worker, &jobs[t]) != 0) { reduce_range(&jobs[t]); th[t] = 0; }
    started = t;
  }
  if (count) reduce_range(&jobs[0]);
  for (int t = 1; t <= started; ++t)
    if (th[t]) pthread_join(th[t], NULL);
  free(jobs);
  free(th);
  return 0;
}
