/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  This is the parity checker, never the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Plain-C restatement of the reference's CPU MSM path for Edwards-BLS12
 * (ark-ed-on-bls12-377, -x^2 + y^2 = 1 + 3021 x^2 y^2 over the 253-bit BLS12-377 scalar field):
 *
 *   field Fq            ark-ff 0.4 Montgomery backend as used by bytes.rs / lib.rs (64-bit limbs)
 *   point add           src/submission/wgsl/curve.wgsl:36-63  (add_points, 9M, unified)
 *   point double        src/submission/wgsl/curve.wgsl:93-114 (double_point_in_place)
 *   split               src/submission/msm-macro/src/lib.rs:73-177 (unsigned, MSB-first windows)
 *   bucket_cpu          src/submission/msm-wasm/src/lib.rs:24-44
 *   bucket_sum_cpu      src/submission/msm-wasm/src/lib.rs:46-56
 *   reduce_last         src/submission/msm-wasm/src/lib.rs:88-104
 *   msm_end_to_end      src/submission/msm-wasm/src/lib.rs:106-121 (windows in parallel, as rayon)
 *   point_add_affine    src/submission/msm-wasm/src/lib.rs:240-253
 *   read_fq / write_fq  src/submission/msm-wasm/src/bytes.rs:11-44 (big-endian u32 words)
 *   getPointFromX       src/reference/utils/FieldMath.ts:31-55
 *
 * Pinned by: the reference's known-answer tests (wasmFunctions.test.ts:4-49,
 * FieldMath.test.ts:5-97, webgpu/utils.test.ts:4-41) and the survey-recorded Aleo-wasm MSM
 * outputs at 2^12 / 2^16 / 2^20, all in tests/golden/.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t l[4]; } fq; /* Montgomery, R = 2^256 */
typedef struct { fq x, y, t, z; } ept;  /* extended projective */

static const uint64_t MOD[4] = {0x0a11800000000001ULL, 0x59aa76fed0000001ULL, 0x60b44d1e5c37b001ULL,
                                0x12ab655e9a2ca556ULL};
static const uint64_t INV = 0x0a117fffffffffffULL; /* -p^-1 mod 2^64 */
static const uint64_t R1[4] = {0x7d1c7ffffffffff3ULL, 0x7257f50f6ffffff2ULL, 0x16d81575512c0feeULL,
                               0x0d4bda322bbb9a9dULL};
static const uint64_t R2[4] = {0x25d577bab861857bULL, 0xcc2c27b58860591fULL, 0xa7cc008fe5dc8593ULL,
                               0x011fdae7eff1c939ULL};
/* subgroup order r (AleoConstants.ts:5) */
static const uint64_t ORDER[4] = {0xb95aee9ac33fd9ffULL, 0x5293a3afc43c8afeULL, 0x982d1347970dec00ULL,
                                  0x04aad957a68b2955ULL};

static int cmp4(const uint64_t* a, const uint64_t* b) {
  for (int i = 3; i >= 0; i--) {
    if (a[i] > b[i]) return 1;
    if (a[i] < b[i]) return -1;
  }
  return 0;
}
static void sub4(uint64_t* a, const uint64_t* b) {
  uint64_t br = 0;
  for (int i = 0; i < 4; i++) {
    u128 t = (u128)a[i] - b[i] - br;
    a[i] = (uint64_t)t;
    br = (uint64_t)(t >> 64) & 1;
  }
}

static fq f_mul(fq a, fq b) {
  uint64_t t[6] = {0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c = (u128)a.l[j] * b.l[i] + t[j] + (uint64_t)c;
      t[j] = (uint64_t)c;
      c >>= 64;
    }
    u128 s = (u128)t[4] + (uint64_t)c;
    t[4] = (uint64_t)s;
    t[5] = (uint64_t)(s >> 64);
    uint64_t m = t[0] * INV;
    c = ((u128)m * MOD[0] + t[0]) >> 64;
    for (int j = 1; j < 4; j++) {
      c = (u128)m * MOD[j] + t[j] + (uint64_t)c;
      t[j - 1] = (uint64_t)c;
      c >>= 64;
    }
    s = (u128)t[4] + (uint64_t)c;
    t[3] = (uint64_t)s;
    t[4] = t[5] + (uint64_t)(s >> 64);
  }
  fq r;
  memcpy(r.l, t, 32);
  if (t[4] || cmp4(r.l, MOD) >= 0) sub4(r.l, MOD);
  return r;
}
static fq f_add(fq a, fq b) {
  fq r;
  uint64_t c = 0;
  for (int i = 0; i < 4; i++) {
    u128 s = (u128)a.l[i] + b.l[i] + c;
    r.l[i] = (uint64_t)s;
    c = (uint64_t)(s >> 64);
  }
  if (cmp4(r.l, MOD) >= 0) sub4(r.l, MOD);
  return r;
}
static fq f_sub(fq a, fq b) {
  fq r = a;
  if (cmp4(a.l, b.l) < 0) {
    uint64_t c = 0;
    for (int i = 0; i < 4; i++) {
      u128 s = (u128)r.l[i] + MOD[i] + c;
      r.l[i] = (uint64_t)s;
      c = (uint64_t)(s >> 64);
    }
  }
  sub4(r.l, b.l);
  return r;
}
static fq f_zero(void) { fq r = {{0, 0, 0, 0}}; return r; }
static fq f_one(void) { fq r; memcpy(r.l, R1, 32); return r; }
static int f_is_zero(fq a) { return !(a.l[0] | a.l[1] | a.l[2] | a.l[3]); }
static int f_eq(fq a, fq b) { return !memcmp(a.l, b.l, 32); }
static fq f_from_std(const uint64_t s[4]) {
  fq a, r2;
  memcpy(a.l, s, 32);
  memcpy(r2.l, R2, 32);
  return f_mul(a, r2);
}
static void f_to_std(fq a, uint64_t s[4]) {
  fq one = {{1, 0, 0, 0}};
  fq r = f_mul(a, one);
  memcpy(s, r.l, 32);
}
static fq f_small(uint64_t v) {
  uint64_t s[4] = {v, 0, 0, 0};
  return f_from_std(s);
}
static fq f_pow(fq a, const uint64_t e[4]) {
  fq r = f_one();
  for (int i = 3; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      r = f_mul(r, r);
      if ((e[i] >> b) & 1) r = f_mul(r, a);
    }
  return r;
}
static fq f_inv(fq a) {
  uint64_t e[4];
  memcpy(e, MOD, 32);
  e[0] -= 2;
  return f_pow(a, e);
}

/* big-endian u32[8] <-> standard 64-bit limbs (bytes.rs:11-20, 33-44) */
static void be_to_std(const uint32_t* w, uint64_t s[4]) {
  for (int i = 0; i < 4; i++) s[i] = ((uint64_t)w[6 - 2 * i] << 32) | w[7 - 2 * i];
}
static void std_to_be(const uint64_t s[4], uint32_t* w) {
  for (int i = 0; i < 4; i++) {
    w[7 - 2 * i] = (uint32_t)s[i];
    w[6 - 2 * i] = (uint32_t)(s[i] >> 32);
  }
}

/* ---- curve (a = -1, d = 3021) ---- */
static fq D_M; /* d in Montgomery form, initialised lazily */
static void init_consts(void) {
  static int done = 0;
  if (!done) {
    D_M = f_small(3021);
    done = 1;
  }
}
static ept p_zero(void) {
  ept r = {f_zero(), f_one(), f_zero(), f_one()};
  return r;
}
static int p_is_zero(const ept* p) { return f_is_zero(p->x) && f_eq(p->y, p->z); }

/* curve.wgsl:36-63 add_points */
static ept p_add(const ept* p1, const ept* p2) {
  fq a = f_mul(p1->x, p2->x);
  fq b = f_mul(p1->y, p2->y);
  fq c = f_mul(f_mul(p1->t, p2->t), D_M);
  fq d = f_mul(p1->z, p2->z);
  fq e = f_mul(f_add(p1->x, p1->y), f_add(p2->x, p2->y));
  fq h = f_add(b, a);
  e = f_sub(e, h);
  fq f = f_sub(d, c);
  fq g = f_add(d, c);
  ept r = {f_mul(e, f), f_mul(g, h), f_mul(e, h), f_mul(f, g)};
  return r;
}
/* curve.wgsl:93-114 double_point_in_place */
static ept p_dbl(const ept* p) {
  fq a = f_mul(p->x, p->x);
  fq b = f_mul(p->y, p->y);
  fq c = f_mul(p->z, p->z);
  c = f_add(c, c);
  fq d = f_sub(f_zero(), a); /* mul_by_a, a = -1 */
  fq h = f_sub(d, b);
  fq e = f_add(p->x, p->y);
  e = f_mul(e, e);
  e = f_add(e, h);
  fq g = f_add(d, b);
  fq f = f_sub(g, c);
  ept r = {f_mul(e, f), f_mul(g, h), f_mul(e, h), f_mul(f, g)};
  return r;
}
static void p_to_affine(const ept* p, uint64_t x[4], uint64_t y[4]) {
  fq zi = f_inv(p->z);
  f_to_std(f_mul(p->x, zi), x);
  f_to_std(f_mul(p->y, zi), y);
}
static ept p_from_affine(const uint64_t x[4], const uint64_t y[4]) {
  ept r;
  r.x = f_from_std(x);
  r.y = f_from_std(y);
  r.t = f_mul(r.x, r.y);
  r.z = f_one();
  return r;
}
/* double-and-add on a 256-bit little-endian scalar (FieldMath.ts:82-98 multiplyUnsafe role) */
static ept p_mul(const ept* p, const uint64_t k[4]) {
  ept r = p_zero();
  for (int i = 3; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      r = p_dbl(&r);
      if ((k[i] >> b) & 1) r = p_add(&r, p);
    }
  return r;
}
static void write_affine_be(const ept* p, uint32_t* out16) {
  uint64_t x[4], y[4];
  p_to_affine(p, x, y);
  std_to_be(x, out16);
  std_to_be(y, out16 + 8);
}

/* ================================ exported API ================================ */

/* field ops on standard-form 64-bit limbs: op 0 mul, 1 add, 2 sub, 3 inv, 4 double */
int oracle_field_op(int op, const uint64_t* a, const uint64_t* b, uint64_t* out) {
  init_consts();
  if (cmp4(a, MOD) >= 0 || (op <= 2 && cmp4(b, MOD) >= 0)) return -3;
  fq x = f_from_std(a), y = op <= 2 ? f_from_std(b) : f_zero(), r;
  switch (op) {
    case 0: r = f_mul(x, y); break;
    case 1: r = f_add(x, y); break;
    case 2: r = f_sub(x, y); break;
    case 3: r = f_inv(x); break;
    case 4: r = f_add(x, x); break;
    default: return -1;
  }
  f_to_std(r, out);
  return 0;
}

/* affine points as BE u32[16] (x|y) */
int oracle_point_add(const uint32_t* a16, const uint32_t* b16, uint32_t* out16) {
  init_consts();
  uint64_t ax[4], ay[4], bx[4], by[4];
  be_to_std(a16, ax); be_to_std(a16 + 8, ay); be_to_std(b16, bx); be_to_std(b16 + 8, by);
  ept p = p_from_affine(ax, ay), q = p_from_affine(bx, by);
  ept r = p_add(&p, &q);
  write_affine_be(&r, out16);
  return 0;
}
int oracle_point_double(const uint32_t* a16, uint32_t* out16) {
  init_consts();
  uint64_t ax[4], ay[4];
  be_to_std(a16, ax); be_to_std(a16 + 8, ay);
  ept p = p_from_affine(ax, ay);
  ept r = p_dbl(&p);
  write_affine_be(&r, out16);
  return 0;
}
/* scalar: BE u32[8] */
int oracle_scalar_mul(const uint32_t* a16, const uint32_t* k8, uint32_t* out16) {
  init_consts();
  uint64_t ax[4], ay[4], k[4];
  be_to_std(a16, ax); be_to_std(a16 + 8, ay); be_to_std(k8, k);
  ept p = p_from_affine(ax, ay);
  ept r = p_mul(&p, k);
  write_affine_be(&r, out16);
  return 0;
}
int oracle_on_curve(const uint32_t* a16) {
  init_consts();
  uint64_t ax[4], ay[4];
  be_to_std(a16, ax); be_to_std(a16 + 8, ay);
  fq x = f_from_std(ax), y = f_from_std(ay);
  fq x2 = f_mul(x, x), y2 = f_mul(y, y);
  fq lhs = f_sub(y2, x2);
  fq rhs = f_add(f_one(), f_mul(D_M, f_mul(x2, y2)));
  return f_eq(lhs, rhs);
}

/* msm-macro split: out[j*n + i], j = 0 most significant window */
uint32_t oracle_split_windows(uint32_t c) { return (256 + c - 1) / c; }
int oracle_split(uint32_t c, const uint32_t* scalars_be, size_t n, uint32_t* out) {
  uint32_t nw = oracle_split_windows(c);
  for (size_t s = 0; s < n; s++) {
    uint64_t k[4];
    be_to_std(scalars_be + 8 * s, k);
    for (uint32_t i = 0; i < nw; i++) { /* i = 0 least significant (msm-macro lib.rs:96-100) */
      uint32_t v = 0;
      for (uint32_t b = 0; b < c; b++) {
        uint32_t pos = i * c + b;
        if (pos >= 256) break;
        v |= (uint32_t)((k[pos / 64] >> (pos % 64)) & 1) << b;
      }
      out[(size_t)(nw - 1 - i) * n + s] = v;
    }
  }
  return 0;
}

typedef struct {
  const uint32_t* digits; /* this window's digits of the job's points */
  const ept* points;
  size_t n;
  uint32_t c;
  ept result;
} win_job;

/* bucket_cpu (lib.rs:24-44) + bucket_sum_cpu (lib.rs:46-56) for one window over a slice of the
 * points (the window's sum is the sum of its slices' sums: the bucket sum is linear) */
static void window_job(win_job* j) {
  size_t nb = (size_t)1 << j->c;
  ept* bucket = (ept*)malloc(nb * sizeof(ept));
  for (size_t b = 0; b < nb; b++) bucket[b] = p_zero();
  for (size_t i = 0; i < j->n; i++) {
    uint32_t id = j->digits[i];
    if (id == 0) continue;
    if (p_is_zero(&bucket[id]))
      bucket[id] = j->points[i];
    else
      bucket[id] = p_add(&bucket[id], &j->points[i]);
  }
  ept sum = p_zero(), carry = p_zero();
  for (size_t i = nb - 1; i >= 1; i--) {
    if (!p_is_zero(&bucket[i])) carry = p_add(&carry, &bucket[i]);
    sum = p_add(&sum, &carry);
  }
  free(bucket);
  j->result = sum;
}

typedef struct {
  win_job* jobs;
  uint32_t njobs;
  uint32_t next;
  pthread_mutex_t mu;
} job_queue;

static void* job_worker(void* arg) {
  job_queue* q = (job_queue*)arg;
  for (;;) {
    pthread_mutex_lock(&q->mu);
    uint32_t k = q->next++;
    pthread_mutex_unlock(&q->mu);
    if (k >= q->njobs) return NULL;
    window_job(&q->jobs[k]);
  }
}

/* msm_end_to_end (lib.rs:106-121): returns 0, or -3 if a coordinate >= p (bytes.rs:19 panics).
 * The reference's rayon parallelism is over windows; here the jobs are (window, point slice)
 * pairs on `threads` workers, so every host core stays busy whatever the window count. */
int oracle_msm(uint32_t c, const uint32_t* scalars_be, const uint32_t* points_be, size_t n, int threads,
               uint32_t* out16) {
  init_consts();
  if (c < 1 || c > 24) return -2;
  uint32_t nw = oracle_split_windows(c);
  ept* pts = (ept*)malloc((n ? n : 1) * sizeof(ept));
  for (size_t i = 0; i < n; i++) { /* read_points (bytes.rs:59-71) */
    uint64_t s[4];
    fq* f[4] = {&pts[i].x, &pts[i].y, &pts[i].t, &pts[i].z};
    for (int q = 0; q < 4; q++) {
      be_to_std(points_be + 32 * i + 8 * q, s);
      if (cmp4(s, MOD) >= 0) {
        free(pts);
        return -3;
      }
      *f[q] = f_from_std(s);
    }
  }
  uint32_t* split = (uint32_t*)malloc(((size_t)nw * n + 1) * sizeof(uint32_t));
  oracle_split(c, scalars_be, n, split);
  if (threads < 1) threads = 1;
  /* slices per window: at least two jobs per worker, at least 4096 points per slice */
  uint32_t ns = (uint32_t)((2 * (size_t)threads + nw - 1) / nw);
  if (ns > n / 4096) ns = (uint32_t)(n / 4096);
  if (ns < 1) ns = 1;
  job_queue q;
  q.njobs = nw * ns;
  q.next = 0;
  q.jobs = (win_job*)calloc(q.njobs, sizeof(win_job));
  pthread_mutex_init(&q.mu, NULL);
  for (uint32_t w = 0; w < nw; w++)
    for (uint32_t sl = 0; sl < ns; sl++) {
      size_t lo = n * sl / ns, hi = n * (sl + 1) / ns;
      win_job* j = &q.jobs[w * ns + sl];
      j->digits = split + (size_t)w * n + lo;
      j->points = pts + lo;
      j->n = hi - lo;
      j->c = c;
    }
  uint32_t nth = (uint32_t)threads < q.njobs ? (uint32_t)threads : q.njobs;
  pthread_t* th = (pthread_t*)malloc(nth * sizeof(pthread_t));
  for (uint32_t t = 0; t < nth; t++) pthread_create(&th[t], NULL, job_worker, &q);
  for (uint32_t t = 0; t < nth; t++) pthread_join(th[t], NULL);
  pthread_mutex_destroy(&q.mu);
  win_job* jobs = (win_job*)calloc(nw, sizeof(win_job));
  for (uint32_t w = 0; w < nw; w++) {
    jobs[w].result = p_zero();
    for (uint32_t sl = 0; sl < ns; sl++) jobs[w].result = p_add(&jobs[w].result, &q.jobs[w * ns + sl].result);
  }
  free(q.jobs);
  /* reduce_last (lib.rs:88-104): windows MSB-first, sum = 2^c sum + W */
  ept sum = p_zero();
  for (uint32_t w = 0; w < nw; w++) {
    for (uint32_t k = 0; k < c; k++) sum = p_dbl(&sum);
    sum = p_add(&sum, &jobs[w].result);
  }
  write_affine_be(&sum, out16);
  free(th);
  free(jobs);
  free(split);
  free(pts);
  return 0;
}

/* point_add_affine (lib.rs:240-253) */
int oracle_point_add_affine(const uint32_t* a16, const uint32_t* b16, uint32_t* out16) {
  return oracle_point_add(a16, b16, out16);
}

/* getPointFromX (FieldMath.ts:31-55): y^2 = (a x^2 - 1) / (d x^2 - 1); pick the root with [r]P = O.
 * Returns 0 and writes BE y, or -1 if x^2 gives a non-square. */
static int f_sqrt(fq a, fq* out) {
  /* Tonelli-Shanks, p - 1 = 2^47 * q */
  if (f_is_zero(a)) {
    *out = a;
    return 0;
  }
  uint64_t pm1[4];
  memcpy(pm1, MOD, 32);
  pm1[0] -= 1;
  uint64_t q[4];
  memcpy(q, pm1, 32);
  int s = 0;
  while (!(q[0] & 1)) {
    for (int i = 0; i < 4; i++) q[i] = (q[i] >> 1) | (i < 3 ? q[i + 1] << 63 : 0);
    s++;
  }
  uint64_t e[4]; /* (p-1)/2 */
  for (int i = 0; i < 4; i++) e[i] = (pm1[i] >> 1) | (i < 3 ? pm1[i + 1] << 63 : 0);
  if (!f_eq(f_pow(a, e), f_one())) return -1;
  fq z = f_small(2);
  while (f_eq(f_pow(z, e), f_one())) z = f_add(z, f_one());
  uint64_t q1[4]; /* (q+1)/2 */
  memcpy(q1, q, 32);
  q1[0] += 1; /* q odd: no carry past limb 0 since q[0] != 0xff..ff here */
  for (int i = 0; i < 4; i++) q1[i] = (q1[i] >> 1) | (i < 3 ? q1[i + 1] << 63 : 0);
  int m = s;
  fq c = f_pow(z, q), t = f_pow(a, q), r = f_pow(a, q1);
  while (!f_eq(t, f_one())) {
    int i = 0;
    fq t2 = t;
    while (!f_eq(t2, f_one())) {
      t2 = f_mul(t2, t2);
      i++;
    }
    fq b = c;
    for (int k = 0; k < m - i - 1; k++) b = f_mul(b, b);
    m = i;
    c = f_mul(b, b);
    t = f_mul(t, c);
    r = f_mul(r, b);
  }
  *out = r;
  return 0;
}
int oracle_point_from_x(const uint32_t* x8, uint32_t* y8) {
  init_consts();
  uint64_t xs[4];
  be_to_std(x8, xs);
  fq x = f_from_std(xs);
  fq x2 = f_mul(x, x);
  fq num = f_sub(f_sub(f_zero(), x2), f_one()); /* a x^2 - 1 */
  fq den = f_sub(f_mul(D_M, x2), f_one());      /* d x^2 - 1 */
  fq y2 = f_mul(num, f_inv(den));
  fq y;
  if (f_sqrt(y2, &y)) return -1;
  ept p;
  p.x = x;
  p.y = y;
  p.t = f_mul(x, y);
  p.z = f_one();
  ept rp = p_mul(&p, ORDER);
  if (!p_is_zero(&rp)) y = f_sub(f_zero(), y);
  uint64_t ys[4];
  f_to_std(y, ys);
  std_to_be(ys, y8);
  return 0;
}

/* Test-input generator: points_be[i] = (k0 + i*step) * G as wire points (x|y|t|z, z = 1). */
int oracle_gen_points(const uint32_t* g16, const uint32_t* k0_8, uint64_t step, size_t n, uint32_t* points_be) {
  init_consts();
  uint64_t gx[4], gy[4], k0[4];
  be_to_std(g16, gx);
  be_to_std(g16 + 8, gy);
  be_to_std(k0_8, k0);
  ept g = p_from_affine(gx, gy);
  ept cur = p_mul(&g, k0);
  uint64_t st[4] = {step, 0, 0, 0};
  ept stp = p_mul(&g, st);
  /* batch-normalise in blocks with Montgomery's trick */
  const size_t BLK = 1024;
  ept* blk = (ept*)malloc(BLK * sizeof(ept));
  fq* pref = (fq*)malloc(BLK * sizeof(fq));
  for (size_t base = 0; base < n; base += BLK) {
    size_t m = n - base < BLK ? n - base : BLK;
    for (size_t i = 0; i < m; i++) {
      blk[i] = cur;
      cur = p_add(&cur, &stp);
    }
    fq acc = f_one();
    for (size_t i = 0; i < m; i++) {
      pref[i] = acc;
      acc = f_mul(acc, blk[i].z);
    }
    fq inv = f_inv(acc);
    for (size_t ii = m; ii-- > 0;) {
      fq zi = f_mul(inv, pref[ii]);
      inv = f_mul(inv, blk[ii].z);
      uint64_t x[4], y[4], t[4], one[4] = {1, 0, 0, 0};
      fq xa = f_mul(blk[ii].x, zi), ya = f_mul(blk[ii].y, zi);
      f_to_std(xa, x);
      f_to_std(ya, y);
      f_to_std(f_mul(xa, ya), t);
      uint32_t* o = points_be + 32 * (base + ii);
      std_to_be(x, o);
      std_to_be(y, o + 8);
      std_to_be(t, o + 16);
      std_to_be(one, o + 24);
    }
  }
  free(blk);
  free(pref);
  return 0;
}
