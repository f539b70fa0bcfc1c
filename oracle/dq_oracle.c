/*
 * dq_oracle.c -- TEST INFRASTRUCTURE ONLY: C restatement of the reference's aggregation
 * semantics for the fused scan and HLL++, used (a) as the large-size parity checker in
 * tests/ and (b) as bench.py's `cpu_baseline` (kind "port").  Never linked into or called by
 * the product library.
 *
 * Restated (not copied) from, per reference file:
 *   count(*) / Size                         Size.scala:35-47, Analyzer.scala:428-432
 *   Completeness = sum(isNotNull)           Completeness.scala:38-40
 *   Compliance = sum(cast(pred as int))     Compliance.scala:47-50 (pred: column OP literal)
 *   Sum / Mean (Spark Sum: int64 wrap for integral, sequential fp64 for double)
 *                                           Sum.scala:38-41, Mean.scala:38-42
 *   StandardDeviation = Spark CentralMomentAgg(2) per-row update, then
 *                       StandardDeviationState.sum across partitions
 *                                           StandardDeviation.scala:37-44, StatefulStdDevPop.scala:24-34
 *   Minimum / Maximum (Spark NaN-safe order) Minimum.scala:38-41, Maximum.scala:38-41
 *   HLL++ register update                   StatefulHyperloglogPlus.scala:89-115
 * Partitions are processed like Spark's local[N]: one sequential pass per partition, partial
 * states merged in partition order with the State.sum formulas.
 *
 * Parity of this file is pinned against oracle/pyoracle.py (itself pinned by the reference's
 * known answers) in tests/test_c_oracle.py.
 */
#include <math.h>
#include <pthread.h>

#define DQO_MAX_THREADS 1024 /* threads of the timed baseline (the GPU box host has 256 CPUs) */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------ data generation */
static uint64_t splitmix64(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static double unit01(uint64_t* s) { return (double)(splitmix64(s) >> 11) * (1.0 / 9007199254740992.0); }

/* C2 column `col` (0..3 int64 uniform [-2^30, 2^32); 4,5 fp64 uniform [0, 1e6); 6,7 fp64
 * N(1e3, 1e2)), Bernoulli(0.05) NULLs; rows [begin, end) of a deterministic stream. */
void dqo_gen_c2(int64_t begin, int64_t end, uint64_t seed, int col, void* values,
                uint8_t* validity) {
  for (int64_t r = begin; r < end; ++r) {
    uint64_t s = seed * 0x100000001B3ull + (uint64_t)col * 0x9E3779B97F4A7C15ull + (uint64_t)r * 0xD1B54A32D192ED03ull;
    if (col < 4) {
      const uint64_t range = (1ull << 32) + (1ull << 30);
      ((int64_t*)values)[r] = -(int64_t)(1ll << 30) + (int64_t)(splitmix64(&s) % range);
    } else if (col < 6) {
      ((double*)values)[r] = unit01(&s) * 1e6;
    } else {
      double u1 = unit01(&s), u2 = unit01(&s);
      if (u1 < 1e-300) u1 = 1e-300;
      ((double*)values)[r] = 1e3 + 1e2 * sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
    }
    const int valid = unit01(&s) >= 0.05;
    if (valid) validity[r >> 3] |= (uint8_t)(1u << (r & 7));
    else validity[r >> 3] &= (uint8_t)~(1u << (r & 7));
  }
}

/* ------------------------------------------------------------------ column scan */
enum { DQO_INT64 = 5, DQO_FLOAT64 = 7 };
enum { OP_EQ = 0, OP_NE, OP_LT, OP_LE, OP_GT, OP_GE };

typedef struct dqo_colstate {
  int64_t rows;       /* count(*)                                  */
  int64_t n_sel;      /* non-null values                           */
  int64_t pm, pn;     /* predicate TRUE / NOT NULL                 */
  int64_t isum;       /* Spark LongType sum (wrapping)             */
  double fsum;        /* Spark DoubleType sum (sequential)         */
  double n, avg, m2;  /* CentralMomentAgg buffer                   */
  double vmin, vmax;  /* as double (int64 compared as int64 first) */
  int64_t imin, imax;
} dqo_colstate;

static int nan_safe_lt(double a, double b) { /* NaN is the largest value */
  const int an = a != a, bn = b != b;
  if (an || bn) return !an && bn;
  return a < b;
}

static int cmp_apply(int op, int ord) {
  switch (op) {
    case OP_EQ: return ord == 0;
    case OP_NE: return ord != 0;
    case OP_LT: return ord < 0;
    case OP_LE: return ord <= 0;
    case OP_GT: return ord > 0;
    default: return ord >= 0;
  }
}

static void colstate_init(dqo_colstate* s) {
  memset(s, 0, sizeof(*s));
  s->imin = INT64_MAX;
  s->imax = INT64_MIN;
  s->vmin = NAN;
  s->vmax = NAN;
}

/* pred_as_f64: compare in double (Spark coercion), else int64 against lit_i */
static void scan_column(int type, const void* values, const uint8_t* validity, int64_t begin,
                        int64_t end, int pred_op, int pred_as_f64, int64_t lit_i, double lit_f,
                        dqo_colstate* s) {
  int have = 0;
  for (int64_t r = begin; r < end; ++r) {
    s->rows += 1;
    const int valid = validity ? (validity[r >> 3] >> (r & 7)) & 1 : 1;
    if (!valid) continue;
    double x;
    int ord;
    if (type == DQO_INT64) {
      const int64_t v = ((const int64_t*)values)[r];
      s->isum = (int64_t)((uint64_t)s->isum + (uint64_t)v);
      if (v < s->imin) s->imin = v;
      if (v > s->imax) s->imax = v;
      x = (double)v;
      if (pred_as_f64) {
        ord = (x > lit_f) - (x < lit_f);
      } else {
        ord = (v > lit_i) - (v < lit_i);
      }
    } else {
      x = ((const double*)values)[r];
      s->fsum += x;
      if (!have || nan_safe_lt(x, s->vmin)) s->vmin = x;
      if (!have || nan_safe_lt(s->vmax, x)) s->vmax = x;
      const int xn = x != x, ln = lit_f != lit_f;
      ord = (xn || ln) ? (xn - ln) : ((x > lit_f) - (x < lit_f));
    }
    have = 1;
    s->n_sel += 1;
    if (pred_op >= 0) {
      s->pn += 1;
      s->pm += cmp_apply(pred_op, ord);
    }
    /* CentralMomentAgg update (Spark 2.2.2): one fp64 divide per row */
    const double n1 = s->n + 1.0;
    const double delta = x - s->avg;
    const double delta_n = delta / n1;
    s->avg += delta_n;
    s->m2 += delta * (delta - delta_n);
    s->n = n1;
  }
  if (type == DQO_INT64 && s->n_sel > 0) {
    s->vmin = (double)s->imin;
    s->vmax = (double)s->imax;
  }
}

/* State.sum of two partition states (StandardDeviation.scala:37-44, Sum/Mean/Min/Max.sum) */
static void colstate_merge(dqo_colstate* a, const dqo_colstate* b, int type) {
  a->rows += b->rows;
  a->pm += b->pm;
  a->pn += b->pn;
  a->isum = (int64_t)((uint64_t)a->isum + (uint64_t)b->isum);
  a->fsum += b->fsum;
  if (b->n_sel > 0) {
    if (a->n_sel == 0) {
      a->vmin = b->vmin;
      a->vmax = b->vmax;
    } else if (type == DQO_INT64) {
      a->vmin = fmin(a->vmin, b->vmin);
      a->vmax = fmax(a->vmax, b->vmax);
    } else { /* Java Math.min/max: NaN propagates */
      a->vmin = (a->vmin != a->vmin || b->vmin != b->vmin) ? NAN : fmin(a->vmin, b->vmin);
      a->vmax = (a->vmax != a->vmax || b->vmax != b->vmax) ? NAN : fmax(a->vmax, b->vmax);
    }
    const double new_n = a->n + b->n;
    const double delta = b->avg - a->avg;
    const double delta_n = new_n == 0.0 ? 0.0 : delta / new_n;
    a->avg = a->avg + delta_n * b->n;
    a->m2 = a->m2 + b->m2 + delta * delta_n * a->n * b->n;
    a->n = new_n;
  }
  a->n_sel += b->n_sel;
}

typedef struct {
  int ncols;
  const int* types;
  const void* const* values;
  const uint8_t* const* validity;
  const int* pred_op;
  const int* pred_as_f64;
  const int64_t* lit_i;
  const double* lit_f;
  int64_t begin, end;
  dqo_colstate* out; /* ncols */
} part_job;

static void* run_part(void* arg) {
  part_job* j = (part_job*)arg;
  for (int c = 0; c < j->ncols; ++c) {
    colstate_init(&j->out[c]);
    scan_column(j->types[c], j->values[c], j->validity[c], j->begin, j->end, j->pred_op[c],
                j->pred_as_f64[c], j->lit_i[c], j->lit_f[c], &j->out[c]);
  }
  return NULL;
}

/* Scan `rows` rows of `ncols` columns in `parts` contiguous partitions on `threads` threads;
 * writes the merged state of every column to out[ncols]. */
int dqo_scan(int64_t rows, int ncols, const int* types, const void* const* values,
             const uint8_t* const* validity, const int* pred_op, const int* pred_as_f64,
             const int64_t* lit_i, const double* lit_f, int parts, dqo_colstate* out) {
  if (parts < 1) parts = 1;
  part_job* jobs = (part_job*)calloc((size_t)parts, sizeof(part_job));
  dqo_colstate* states = (dqo_colstate*)calloc((size_t)parts * ncols, sizeof(dqo_colstate));
  pthread_t* th = (pthread_t*)calloc((size_t)parts, sizeof(pthread_t));
  if (!jobs || !states || !th) return -1;
  for (int p = 0; p < parts; ++p) {
    jobs[p] = (part_job){ncols, types, values, validity, pred_op, pred_as_f64, lit_i, lit_f,
                         rows * p / parts, rows * (p + 1) / parts, states + (size_t)p * ncols};
    pthread_create(&th[p], NULL, run_part, &jobs[p]);
  }
  for (int p = 0; p < parts; ++p) pthread_join(th[p], NULL);
  for (int c = 0; c < ncols; ++c) {
    out[c] = states[c];
    for (int p = 1; p < parts; ++p) colstate_merge(&out[c], &states[(size_t)p * ncols + c], types[c]);
  }
  free(jobs);
  free(states);
  free(th);
  return 0;
}

typedef struct {
  int64_t b, e;
  void** values;
  uint8_t** validity;
} gen_job;

static void* gen_thread(void* arg) {
  gen_job* j = (gen_job*)arg;
  for (int c = 0; c < 8; ++c) dqo_gen_c2(j->b, j->e, 42, c, j->values[c], j->validity[c]);
  return NULL;
}

/* bench.py cpu_baseline: generate a C2 sample (untimed), time dqo_scan over it. */
typedef struct {
  int64_t b, e;
  void** values;
  uint8_t** validity;
  uint8_t regs[8][512];
} hll_job;

void dqo_hll_registers(int type, int64_t n, const void* values, const int32_t* offsets,
                       const uint8_t* validity, uint8_t* regs512);

static void* hll_thread(void* arg) {
  hll_job* j = (hll_job*)arg;
  for (int c = 0; c < 8; ++c)
    dqo_hll_registers(c < 4 ? 5 : 7, j->e - j->b, (const uint8_t*)j->values[c] + j->b * 8, NULL,
                      j->validity[c] + (j->b >> 3), j->regs[c]);
  return NULL;
}

/* C2 with ApproxCountDistinct too: the scan, then the HLL registers of the 8 columns (row
 * partitions per thread, merged by register max = DeequHyperLogLogPlusPlusUtils.merge). */
double dqo_time_c2_hll_for(int64_t rows, int threads, dqo_colstate* out8, uint8_t* regs8x512, double min_secs,
                           int* passes);

double dqo_time_c2_hll(int64_t rows, int threads, dqo_colstate* out8, uint8_t* regs8x512) {
  int passes = 0;
  return dqo_time_c2_hll_for(rows, threads, out8, regs8x512, 0.0, &passes);
}

double dqo_time_c2(int64_t rows, int threads, dqo_colstate* out8) {
  return dqo_time_c2_hll(rows, threads, out8, NULL);
}

/* Timed passes over one generated sample until at least min_secs have been spent (1 pass when
 * min_secs <= 0); returns the total seconds of the *passes passes (each pass = the whole scan and
 * HLL; the results are those of the last pass -- every pass computes the same states). */
double dqo_time_c2_hll_for(int64_t rows, int threads, dqo_colstate* out8, uint8_t* regs8x512, double min_secs,
                           int* passes) {
  int types[8], pred_op[8], as_f64[8];
  int64_t lit_i[8];
  double lit_f[8];
  void* values[8];
  uint8_t* validity[8];
  for (int c = 0; c < 8; ++c) {
    types[c] = c < 4 ? DQO_INT64 : DQO_FLOAT64;
    values[c] = malloc((size_t)rows * 8);
    validity[c] = (uint8_t*)calloc((size_t)(rows + 7) / 8 + 8, 1);
    if (!values[c] || !validity[c]) return -1.0;
    pred_op[c] = c < 4 ? OP_GE : OP_GT;
    as_f64[c] = c >= 4;
    lit_i[c] = 0;
    lit_f[c] = c < 4 ? 0.0 : (c < 6 ? 5e5 : 1e3);
  }
  /* untimed generation, in byte-aligned slices so threads never share a bitmap byte */
  {
    const int ng = threads < 1 ? 1 : (threads > DQO_MAX_THREADS ? DQO_MAX_THREADS : threads);
    pthread_t th[DQO_MAX_THREADS];
    gen_job jobs[DQO_MAX_THREADS];
    for (int t = 0; t < ng; ++t) {
      const int64_t b = (rows * t / ng) & ~7ll;
      const int64_t e = t == ng - 1 ? rows : ((rows * (t + 1) / ng) & ~7ll);
      jobs[t] = (gen_job){b, e, values, validity};
      pthread_create(&th[t], NULL, gen_thread, &jobs[t]);
    }
    for (int t = 0; t < ng; ++t) pthread_join(th[t], NULL);
  }
  struct timespec t0, t1;
  double total = 0.0;
  int done = 0;
  do {
  clock_gettime(CLOCK_MONOTONIC, &t0);
  dqo_scan(rows, 8, types, (const void* const*)values, (const uint8_t* const*)validity, pred_op,
           as_f64, lit_i, lit_f, threads, out8);
  if (regs8x512) {
    const int ng = threads < 1 ? 1 : (threads > DQO_MAX_THREADS ? DQO_MAX_THREADS : threads);
    pthread_t th[DQO_MAX_THREADS];
    hll_job* jobs = (hll_job*)calloc((size_t)ng, sizeof(hll_job));
    if (!jobs) return -1.0;
    for (int t = 0; t < ng; ++t) {
      jobs[t].b = (rows * t / ng) & ~7ll;
      jobs[t].e = t == ng - 1 ? rows : ((rows * (t + 1) / ng) & ~7ll);
      jobs[t].values = values;
      jobs[t].validity = validity;
      pthread_create(&th[t], NULL, hll_thread, &jobs[t]);
    }
    for (int t = 0; t < ng; ++t) pthread_join(th[t], NULL);
    memset(regs8x512, 0, 8 * 512);
    for (int t = 0; t < ng; ++t)
      for (int c = 0; c < 8; ++c)
        for (int r = 0; r < 512; ++r)
          if (jobs[t].regs[c][r] > regs8x512[c * 512 + r]) regs8x512[c * 512 + r] = jobs[t].regs[c][r];
    free(jobs);
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  total += (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
  ++done;
  } while (total < min_secs && done < 1000);
  for (int c = 0; c < 8; ++c) {
    free(values[c]);
    free(validity[c]);
  }
  *passes = done;
  return total;
}

/* ------------------------------------------------------------------ XXH64 + HLL registers */
static const uint64_t P1 = 0x9E3779B185EBCA87ull, P2 = 0xC2B2AE3D27D4EB4Full,
                      P3 = 0x165667B19E3779F9ull, P4 = 0x85EBCA77C2B2AE63ull,
                      P5 = 0x27D4EB2F165667C5ull;
static uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint64_t rnd(uint64_t a, uint64_t l) { a += l * P2; a = rotl(a, 31); return a * P1; }
static uint64_t fmix(uint64_t h) {
  h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
  return h;
}

uint64_t dqo_xxh64(const uint8_t* p, size_t len, uint64_t seed) {
  const uint8_t* end = p + len;
  uint64_t h, k;
  uint32_t w;
  if (len >= 32) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    while (p + 32 <= end) {
      memcpy(&k, p, 8); v1 = rnd(v1, k);
      memcpy(&k, p + 8, 8); v2 = rnd(v2, k);
      memcpy(&k, p + 16, 8); v3 = rnd(v3, k);
      memcpy(&k, p + 24, 8); v4 = rnd(v4, k);
      p += 32;
    }
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    h ^= rnd(0, v1); h = h * P1 + P4;
    h ^= rnd(0, v2); h = h * P1 + P4;
    h ^= rnd(0, v3); h = h * P1 + P4;
    h ^= rnd(0, v4); h = h * P1 + P4;
  } else {
    h = seed + P5;
  }
  h += (uint64_t)len;
  while (p + 8 <= end) {
    memcpy(&k, p, 8);
    h ^= rnd(0, k);
    h = rotl(h, 27) * P1 + P4;
    p += 8;
  }
  if (p + 4 <= end) {
    memcpy(&w, p, 4);
    h ^= (uint64_t)w * P1;
    h = rotl(h, 23) * P2 + P3;
    p += 4;
  }
  while (p < end) {
    h ^= (uint64_t)(*p) * P5;
    h = rotl(h, 11) * P1;
    ++p;
  }
  return fmix(h);
}

static void hll_update(uint8_t* regs, uint64_t x) {
  const uint32_t idx = (uint32_t)(x >> 55);
  const uint64_t w = (x << 9) | (1ull << 8);
  const uint8_t pw = (uint8_t)(__builtin_clzll(w) + 1);
  if (pw > regs[idx]) regs[idx] = pw;
}

/* type: 5 int64 (hashLong), 4 int32 (hashInt), 7 fp64 (doubleToLongBits), 8 utf8 */
void dqo_hll_registers(int type, int64_t n, const void* values, const int32_t* offsets,
                       const uint8_t* validity, uint8_t* regs512) {
  memset(regs512, 0, 512);
  for (int64_t r = 0; r < n; ++r) {
    if (validity && !((validity[r >> 3] >> (r & 7)) & 1)) continue;
    uint8_t buf[8];
    if (type == 5) {
      memcpy(buf, (const int64_t*)values + r, 8);
      hll_update(regs512, dqo_xxh64(buf, 8, 42));
    } else if (type == 4) {
      memcpy(buf, (const int32_t*)values + r, 4);
      hll_update(regs512, dqo_xxh64(buf, 4, 42));
    } else if (type == 7) {
      double d = ((const double*)values)[r];
      uint64_t bits;
      memcpy(&bits, &d, 8);
      if (d != d) bits = 0x7ff8000000000000ull;
      memcpy(buf, &bits, 8);
      hll_update(regs512, dqo_xxh64(buf, 8, 42));
    } else if (type == 8) {
      const uint8_t* chars = (const uint8_t*)values;
      hll_update(regs512, dqo_xxh64(chars + offsets[r], (size_t)(offsets[r + 1] - offsets[r]), 42));
    }
  }
}

/* dqo_hll_registers over row slices on `threads` threads, merged by register max
 * (DeequHyperLogLogPlusPlusUtils.merge, StatefulHyperloglogPlus.scala:188-208): the whole-job
 * check of bench.py --c3-verify (1e9 values).  Slices start at multiples of 8 rows. */
typedef struct {
  int type;
  int64_t b, e;
  const void* values;
  const uint8_t* validity;
  uint8_t regs[512];
} hll_mt_job;

static void* hll_mt_thread(void* arg) {
  hll_mt_job* j = (hll_mt_job*)arg;
  const size_t w = j->type == 4 ? 4 : 8;
  dqo_hll_registers(j->type, j->e - j->b, (const uint8_t*)j->values + j->b * w, NULL,
                    j->validity ? j->validity + (j->b >> 3) : NULL, j->regs);
  return NULL;
}

void dqo_hll_registers_mt(int type, int64_t n, const void* values, const uint8_t* validity, uint8_t* regs512,
                          int threads) {
  const int nt = threads < 1 ? 1 : (threads > DQO_MAX_THREADS ? DQO_MAX_THREADS : threads);
  pthread_t th[DQO_MAX_THREADS];
  hll_mt_job* jobs = (hll_mt_job*)calloc((size_t)nt, sizeof(hll_mt_job));
  const int64_t per = ((n + nt - 1) / nt + 7) & ~(int64_t)7;
  for (int t = 0; t < nt; ++t) {
    jobs[t].type = type;
    jobs[t].b = per * t < n ? per * t : n;
    jobs[t].e = per * (t + 1) < n ? per * (t + 1) : n;
    jobs[t].values = values;
    jobs[t].validity = validity;
    pthread_create(&th[t], NULL, hll_mt_thread, &jobs[t]);
  }
  memset(regs512, 0, 512);
  for (int t = 0; t < nt; ++t) {
    pthread_join(th[t], NULL);
    for (int i = 0; i < 512; ++i)
      if (jobs[t].regs[i] > regs512[i]) regs512[i] = jobs[t].regs[i];
  }
  free(jobs);
}
