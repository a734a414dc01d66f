/* CPU baseline — TEST/BASELINE INFRASTRUCTURE ONLY (never shipped or measured
 * as the product).
 *
 * C restatement of the reference's DJN private-key encryption
 * (python/common/crypto/paillier/paillier.py:189-209,273-287, utils.py:38-76)
 * on the same GMP routines gmpy2 calls (mpz_powm / mpz_mul / mpz_fdiv_r),
 * loaded from the system libgmp.so.10 with dlopen (no GMP headers in the
 * image, so the few prototypes used are declared here; mpz_t layout is GMP's
 * stable public ABI). Used as bench.py's cpu_baseline when it builds/loads,
 * and (gmpb_encrypt_batch) as the fast checker of the GPU parity tests at the
 * production table windows, after tests/test_cpu_baseline.py has pinned it to
 * the reference's golden ciphertexts.
 */
#include <dlfcn.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct {
  int alloc;
  int size;
  void* d;
} mpz_s;
typedef mpz_s mpz_t[1];

static void (*z_init)(mpz_s*);
static void (*z_clear)(mpz_s*);
static void (*z_import)(mpz_s*, size_t, int, size_t, int, size_t, const void*);
static void* (*z_export)(void*, size_t*, int, size_t, int, size_t, const mpz_s*);
static void (*z_powm)(mpz_s*, const mpz_s*, const mpz_s*, const mpz_s*);
static void (*z_mul)(mpz_s*, const mpz_s*, const mpz_s*);
static void (*z_add)(mpz_s*, const mpz_s*, const mpz_s*);
static void (*z_sub)(mpz_s*, const mpz_s*, const mpz_s*);
static void (*z_add_ui)(mpz_s*, const mpz_s*, unsigned long);
static void (*z_fdiv_r)(mpz_s*, const mpz_s*, const mpz_s*);
static void (*z_set_si)(mpz_s*, long);

static int loaded = 0;

int gmpb_load(void) {
  if (loaded) return 0;
  void* h = dlopen("libgmp.so.10", RTLD_NOW);
  if (!h) return -1;
#define SYM(v, n) if (!(*(void**)&v = dlsym(h, n))) return -2;
  SYM(z_init, "__gmpz_init")
  SYM(z_clear, "__gmpz_clear")
  SYM(z_import, "__gmpz_import")
  SYM(z_export, "__gmpz_export")
  SYM(z_powm, "__gmpz_powm")
  SYM(z_mul, "__gmpz_mul")
  SYM(z_add, "__gmpz_add")
  SYM(z_sub, "__gmpz_sub")
  SYM(z_add_ui, "__gmpz_add_ui")
  SYM(z_fdiv_r, "__gmpz_fdiv_r")
  SYM(z_set_si, "__gmpz_set_si")
#undef SYM
  loaded = 1;
  return 0;
}

typedef struct {
  mpz_t n, n2, p2, q2, q2inv, hp, hq;
  int nw;
} key_t_;

static void imp(mpz_s* z, const uint32_t* w, int nw) { z_import(z, (size_t)nw, -1, 4, 0, 0, w); }

static void key_init(key_t_* k, const uint32_t* n, const uint32_t* n2, const uint32_t* p2, const uint32_t* q2,
                     const uint32_t* q2inv, const uint32_t* hp, const uint32_t* hq, int nw) {
  mpz_s* all[] = {k->n, k->n2, k->p2, k->q2, k->q2inv, k->hp, k->hq};
  for (int i = 0; i < 7; ++i) z_init(all[i]);
  imp(k->n, n, nw);
  imp(k->n2, n2, 2 * nw);
  imp(k->p2, p2, nw);
  imp(k->q2, q2, nw);
  imp(k->q2inv, q2inv, nw);
  imp(k->hp, hp, nw);
  imp(k->hq, hq, nw);
  k->nw = nw;
}

static void key_clear(key_t_* k) {
  mpz_s* all[] = {k->n, k->n2, k->p2, k->q2, k->q2inv, k->hp, k->hq};
  for (int i = 0; i < 7; ++i) z_clear(all[i]);
}

/* c = (n m + 1) * CRT(hp^a mod p^2, hq^a mod q^2) mod n^2 for signed m (|m| < 2^62) */
static void encrypt_one(const key_t_* k, long long m_signed, const uint32_t* a_words, int aw, mpz_s* out, mpz_s* t1,
                        mpz_s* t2, mpz_s* a, mpz_s* m) {
  z_import(a, (size_t)aw, -1, 4, 0, 0, a_words);
  z_set_si(m, m_signed);
  if (m_signed < 0) z_add(m, m, k->n);          /* encode: m mod n (encoder.py:53) */
  z_mul(t1, k->n, m);                            /* n m + 1 (paillier.py:283) */
  z_add_ui(t1, t1, 1);
  z_fdiv_r(out, t1, k->n2);
  z_powm(t1, k->hp, a, k->p2);                   /* paillier.py:207-208 */
  z_powm(t2, k->hq, a, k->q2);
  z_sub(m, t1, t2);                              /* crt (utils.py:38-43) over p^2, q^2 */
  z_mul(m, m, k->q2inv);
  z_fdiv_r(m, m, k->p2);
  z_mul(m, m, k->q2);
  z_add(m, m, t2);
  z_fdiv_r(t1, m, k->n2);
  z_mul(t2, out, t1);                            /* paillier.py:231 */
  z_fdiv_r(out, t2, k->n2);
}

/* One encryption (for testing the baseline against the oracle). */
int gmpb_encrypt_one(const uint32_t* n, const uint32_t* n2, const uint32_t* p2, const uint32_t* q2,
                     const uint32_t* q2inv, const uint32_t* hp, const uint32_t* hq, int nw, long long m,
                     const uint32_t* a_words, int aw, uint32_t* out_words) {
  if (gmpb_load()) return -1;
  key_t_ k;
  key_init(&k, n, n2, p2, q2, q2inv, hp, hq, nw);
  mpz_t out, t1, t2, a, mm;
  z_init(out); z_init(t1); z_init(t2); z_init(a); z_init(mm);
  encrypt_one(&k, m, a_words, aw, out, t1, t2, a, mm);
  memset(out_words, 0, (size_t)2 * nw * 4);
  size_t cnt = 0;
  z_export(out_words, &cnt, -1, 4, 0, 0, out);
  z_clear(out); z_clear(t1); z_clear(t2); z_clear(a); z_clear(mm);
  key_clear(&k);
  return 0;
}

/* Batch checker for the GPU parity tests: c_i = (1 + n m_i) * CRT(hp^a_i mod p^2,
 * hq^a_i mod q^2) mod n^2 (paillier.py:189-209,283; utils.py:38-43) for full
 * nw-word residues m_i (already encoded, 0 <= m_i < n) and aw-word a_i, on
 * `threads` threads. Elements i = t, t + threads, ... go to thread t. */
typedef struct {
  const key_t_* k;
  const uint32_t* m;
  const uint32_t* a;
  uint32_t* out;
  int64_t count;
  int aw, t, threads;
} batch_t;

static void* batch_worker(void* arg) {
  batch_t* b = (batch_t*)arg;
  const key_t_* k = b->k;
  const int nw = k->nw;
  mpz_t out, t1, t2, a, m;
  z_init(out); z_init(t1); z_init(t2); z_init(a); z_init(m);
  for (int64_t i = b->t; i < b->count; i += b->threads) {
    imp(m, b->m + (size_t)i * nw, nw);
    z_import(a, (size_t)b->aw, -1, 4, 0, 0, b->a + (size_t)i * b->aw);
    z_mul(t1, k->n, m);
    z_add_ui(t1, t1, 1);
    z_fdiv_r(out, t1, k->n2);
    z_powm(t1, k->hp, a, k->p2);
    z_powm(t2, k->hq, a, k->q2);
    z_sub(m, t1, t2);
    z_mul(m, m, k->q2inv);
    z_fdiv_r(m, m, k->p2);
    z_mul(m, m, k->q2);
    z_add(m, m, t2);
    z_fdiv_r(t1, m, k->n2);
    z_mul(t2, out, t1);
    z_fdiv_r(out, t2, k->n2);
    uint32_t* o = b->out + (size_t)i * 2 * nw;
    memset(o, 0, (size_t)2 * nw * 4);
    size_t cnt = 0;
    z_export(o, &cnt, -1, 4, 0, 0, out);
  }
  z_clear(out); z_clear(t1); z_clear(t2); z_clear(a); z_clear(m);
  return NULL;
}

int gmpb_encrypt_batch(const uint32_t* n, const uint32_t* n2, const uint32_t* p2, const uint32_t* q2,
                       const uint32_t* q2inv, const uint32_t* hp, const uint32_t* hq, int nw, const uint32_t* m_words,
                       const uint32_t* a_words, int aw, int64_t count, int threads, uint32_t* out_words) {
  if (gmpb_load()) return -1;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  key_t_ k;
  key_init(&k, n, n2, p2, q2, q2inv, hp, hq, nw);
  pthread_t th[256];
  batch_t jobs[256];
  for (int i = 0; i < threads; ++i) {
    jobs[i] = (batch_t){&k, m_words, a_words, out_words, count, aw, i, threads};
    pthread_create(&th[i], NULL, batch_worker, &jobs[i]);
  }
  for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
  key_clear(&k);
  return 0;
}

typedef struct {
  const key_t_* k;
  double seconds;
  uint64_t seed;
  uint64_t count;
} job_t;

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static uint64_t xs(uint64_t* s) {
  uint64_t x = *s;
  x ^= x << 13;
  x ^= x >> 7;
  x ^= x << 17;
  return *s = x;
}

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  mpz_t out, t1, t2, a, mm;
  z_init(out); z_init(t1); z_init(t2); z_init(a); z_init(mm);
  uint32_t aw[32];
  uint64_t s = j->seed | 1;
  double t0 = now();
  uint64_t c = 0;
  while (now() - t0 < j->seconds) {
    for (int i = 0; i < 32; ++i) aw[i] = (uint32_t)xs(&s);
    aw[31] &= 0x7fffffffu;  /* a < 2^1023 <= djn_exp_bound */
    /* precision-7 encode of a N(0,1)-ish value: round(x * 2^24) */
    double x = ((double)(xs(&s) >> 11) / 9007199254740992.0 - 0.5) * 8.0;
    long long m = (long long)llrint(x * 16777216.0);
    encrypt_one(j->k, m, aw, 32, out, t1, t2, a, mm);
    ++c;
  }
  j->count = c;
  z_clear(out); z_clear(t1); z_clear(t2); z_clear(a); z_clear(mm);
  return NULL;
}

/* Encryptions/s over `threads` threads for ~`seconds` (2048-bit keys, 32-word a). */
int gmpb_bench(const uint32_t* n, const uint32_t* n2, const uint32_t* p2, const uint32_t* q2, const uint32_t* q2inv,
               const uint32_t* hp, const uint32_t* hq, int nw, double seconds, int threads, uint64_t* total,
               double* wall) {
  if (gmpb_load()) return -1;
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  key_t_ k;
  key_init(&k, n, n2, p2, q2, q2inv, hp, hq, nw);
  pthread_t th[256];
  job_t jobs[256];
  double t0 = now();
  for (int i = 0; i < threads; ++i) {
    jobs[i].k = &k;
    jobs[i].seconds = seconds;
    jobs[i].seed = 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1);
    jobs[i].count = 0;
    pthread_create(&th[i], NULL, worker, &jobs[i]);
  }
  uint64_t tot = 0;
  for (int i = 0; i < threads; ++i) {
    pthread_join(th[i], NULL);
    tot += jobs[i].count;
  }
  *wall = now() - t0;
  *total = tot;
  key_clear(&k);
  return 0;
}
