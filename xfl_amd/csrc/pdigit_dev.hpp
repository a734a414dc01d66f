// Arithmetic mod P^2 in Montgomery digits (limb-level model:
// tools/pdigit_model.py MontDigits).
//
// P is a prime of K limbs of W = 28 bits and R = 2^(W K) (2048-bit keys: K =
// 37, R = 2^1036 > 4096 P). A residue x mod P^2 is held as two K-limb
// integers (a, c) with
//
//     x R^2 = R a + P c   (mod P^2)
//
// - the usual Montgomery form mod P^2 (R^2 = 2^(28*74) is the factor of the
// 74-limb Montgomery products of bn_dev.hpp) written in mixed radix (R, P).
// The product of (a, c) and (e, f) is
//
//     a' = REDC(a e)                   = (a e + m P) / R
//     c' = REDC(a f + c e) + (R-1-m) + E,      E = (1 - R) mod P,
//
// where m (K digits) is the first reduction's quotient: a e = R a' - m P
// exactly, so R^2 a e = R^3 a' - R^2 P m and
// (R a + P c)(R e + P f) = R^2 (R a' + P (R^-1 (a f + c e) - m))  (mod P^2).
// Both reductions run as ONE operand-scanning loop over the limbs of (e, f)
// with lazy 64-bit accumulators T1, T2 (the shift by W folded into the mad
// destinations, as Mont::step1); digit m_i of the first is known at step i,
// and (MASK - m_i + E_i) enters the top of T2 at that step, landing at weight
// 2^(W i) of c'. Per step: K mads e_i a + K mads m_i P, and 3K mads e_i c +
// f_i a + m'_i P: 5 K^2 = 6,845 mads per product, against 2 (2K)^2 = 10,952
// for the Montgomery product on the 74-limb modulus P^2.
//
// Ranges (checked by the model over product chains): table digits e, f < P;
// a' < P (1 + 2P/R) and c' < R + 4P, so the state stays bounded; the top
// limb of c may exceed 2^28 and is kept unmasked. Every accumulator stays
// below 2^63 (3K products of < 2^57 plus carries).
#pragma once
#include "bn_dev.hpp"

namespace xhe {

template <int K_>
struct PMD {
  static constexpr int K = K_, W = 28, BL = 6;
  static constexpr int NQ = (2 * K + 3) / 4;  // quads of an interleaved row (e_i, f_i pairs)
  static constexpr uint32_t MASK = (1u << W) - 1u;
  static_assert((K - 1) % BL == 0, "positions 1..K-1 in blocks of 6");
  static_assert((double)(3 * K + 2) * (double)(1ull << 57) < 18446744073709551616.0, "accumulator bound");

  uint32_t p[K];   // P, wave-uniform (SGPRs for the kernel's lifetime)
  uint32_t n0inv;  // -P^-1 mod 2^W

  XHE_DEV void init(const uint32_t* __restrict__ P, uint32_t ninv) {
#pragma unroll
    for (int j = 0; j < K; ++j) p[j] = __builtin_amdgcn_readfirstlane(P[j]);
    n0inv = ninv;
  }

  // T1[j-1+k] = T1[j+k] + e a[j+k] + m P[j+k], k = 0..5 (tied accumulators:
  // T1[j-1+k] is written after T1[j-1+k]'s old value was consumed)
  XHE_DEV void blk1(uint64_t (&T)[K], const uint32_t (&a)[K], uint32_t e, uint32_t m, int j) const {
    asm("v_mad_u64_u32 %0, vcc, %7, %9, %1\n\t"
        "v_mad_u64_u32 %1, vcc, %7, %10, %2\n\t"
        "v_mad_u64_u32 %2, vcc, %7, %11, %3\n\t"
        "v_mad_u64_u32 %3, vcc, %7, %12, %4\n\t"
        "v_mad_u64_u32 %4, vcc, %7, %13, %5\n\t"
        "v_mad_u64_u32 %5, vcc, %7, %14, %6\n\t"
        "v_mad_u64_u32 %0, vcc, %8, %15, %0\n\t"
        "v_mad_u64_u32 %1, vcc, %8, %16, %1\n\t"
        "v_mad_u64_u32 %2, vcc, %8, %17, %2\n\t"
        "v_mad_u64_u32 %3, vcc, %8, %18, %3\n\t"
        "v_mad_u64_u32 %4, vcc, %8, %19, %4\n\t"
        "v_mad_u64_u32 %5, vcc, %8, %20, %5"
        : "+v"(T[j - 1]), "+v"(T[j]), "+v"(T[j + 1]), "+v"(T[j + 2]), "+v"(T[j + 3]), "+v"(T[j + 4])
        : "v"(T[j + 5]), "v"(e), "v"(m), "v"(a[j]), "v"(a[j + 1]), "v"(a[j + 2]), "v"(a[j + 3]), "v"(a[j + 4]),
          "v"(a[j + 5]), "s"(p[j]), "s"(p[j + 1]), "s"(p[j + 2]), "s"(p[j + 3]), "s"(p[j + 4]), "s"(p[j + 5])
        : "vcc");
  }
  // T2[j-1+k] = T2[j+k] + e c[j+k] + f a[j+k] + m P[j+k], k = 0..5
  XHE_DEV void blk2(uint64_t (&T)[K], const uint32_t (&c)[K], const uint32_t (&a)[K], uint32_t e, uint32_t f,
                    uint32_t m, int j) const {
    asm("v_mad_u64_u32 %0, vcc, %7, %10, %1\n\t"
        "v_mad_u64_u32 %1, vcc, %7, %11, %2\n\t"
        "v_mad_u64_u32 %2, vcc, %7, %12, %3\n\t"
        "v_mad_u64_u32 %3, vcc, %7, %13, %4\n\t"
        "v_mad_u64_u32 %4, vcc, %7, %14, %5\n\t"
        "v_mad_u64_u32 %5, vcc, %7, %15, %6\n\t"
        "v_mad_u64_u32 %0, vcc, %8, %16, %0\n\t"
        "v_mad_u64_u32 %1, vcc, %8, %17, %1\n\t"
        "v_mad_u64_u32 %2, vcc, %8, %18, %2\n\t"
        "v_mad_u64_u32 %3, vcc, %8, %19, %3\n\t"
        "v_mad_u64_u32 %4, vcc, %8, %20, %4\n\t"
        "v_mad_u64_u32 %5, vcc, %8, %21, %5\n\t"
        "v_mad_u64_u32 %0, vcc, %9, %22, %0\n\t"
        "v_mad_u64_u32 %1, vcc, %9, %23, %1\n\t"
        "v_mad_u64_u32 %2, vcc, %9, %24, %2\n\t"
        "v_mad_u64_u32 %3, vcc, %9, %25, %3\n\t"
        "v_mad_u64_u32 %4, vcc, %9, %26, %4\n\t"
        "v_mad_u64_u32 %5, vcc, %9, %27, %5"
        : "+v"(T[j - 1]), "+v"(T[j]), "+v"(T[j + 1]), "+v"(T[j + 2]), "+v"(T[j + 3]), "+v"(T[j + 4])
        : "v"(T[j + 5]), "v"(e), "v"(f), "v"(m), "v"(c[j]), "v"(c[j + 1]), "v"(c[j + 2]), "v"(c[j + 3]),
          "v"(c[j + 4]), "v"(c[j + 5]), "v"(a[j]), "v"(a[j + 1]), "v"(a[j + 2]), "v"(a[j + 3]), "v"(a[j + 4]),
          "v"(a[j + 5]), "s"(p[j]), "s"(p[j + 1]), "s"(p[j + 2]), "s"(p[j + 3]), "s"(p[j + 4]), "s"(p[j + 5])
        : "vcc");
  }

  // squaring form of blk2: T2[j-1+k] = T2[j+k] + e2 c[j+k] + m P[j+k] (e2 = 2 a_i)
  XHE_DEV void blk2s(uint64_t (&T)[K], const uint32_t (&c)[K], uint32_t e2, uint32_t m, int j) const {
    asm("v_mad_u64_u32 %0, vcc, %7, %9, %1\n\t"
        "v_mad_u64_u32 %1, vcc, %7, %10, %2\n\t"
        "v_mad_u64_u32 %2, vcc, %7, %11, %3\n\t"
        "v_mad_u64_u32 %3, vcc, %7, %12, %4\n\t"
        "v_mad_u64_u32 %4, vcc, %7, %13, %5\n\t"
        "v_mad_u64_u32 %5, vcc, %7, %14, %6\n\t"
        "v_mad_u64_u32 %0, vcc, %8, %15, %0\n\t"
        "v_mad_u64_u32 %1, vcc, %8, %16, %1\n\t"
        "v_mad_u64_u32 %2, vcc, %8, %17, %2\n\t"
        "v_mad_u64_u32 %3, vcc, %8, %18, %3\n\t"
        "v_mad_u64_u32 %4, vcc, %8, %19, %4\n\t"
        "v_mad_u64_u32 %5, vcc, %8, %20, %5"
        : "+v"(T[j - 1]), "+v"(T[j]), "+v"(T[j + 1]), "+v"(T[j + 2]), "+v"(T[j + 3]), "+v"(T[j + 4])
        : "v"(T[j + 5]), "v"(e2), "v"(m), "v"(c[j]), "v"(c[j + 1]), "v"(c[j + 2]), "v"(c[j + 3]), "v"(c[j + 4]),
          "v"(c[j + 5]), "s"(p[j]), "s"(p[j + 1]), "s"(p[j + 2]), "s"(p[j + 3]), "s"(p[j + 4]), "s"(p[j + 5])
        : "vcc");
  }

  // One step of the two interleaved reductions on row limbs (e, f). Entry:
  // x1 = T1[0] + e a[0], x2 = T2[0] + e c[0] + f a[0] and their digits m1, m2;
  // the next step's (en, fn) values are formed under this step's mads (each
  // link of that dependent chain after its own block pair, as Mont::step1).
  // topc = MASK + E_i.
  // SQ: the squaring step - (e, f) = (a_i, c_i) of the state itself, and
  // T2 takes (2 a_i) c instead of a_i c + c_i a (the same sum, 2 a c: K mads
  // fewer per step; 2 a_i < 2^29 keeps every accumulator below 2^63).
  template <bool SQ = false>
  XHE_DEV void step(uint64_t (&T1)[K], uint64_t (&T2)[K], const uint32_t (&a)[K], const uint32_t (&c)[K],
                    uint32_t e, uint32_t f, uint32_t en, uint32_t fn, uint32_t& m1, uint32_t& m2, uint64_t& x1,
                    uint64_t& x2, uint32_t topc) const {
    uint64_t x1n = 0, x2n = 0;
    uint32_t t1 = 0, t2 = 0, m1n = 0, m2n = 0;
    x1 = mad64s(m1, p[0], x1);  // now = 0 (mod 2^W)
    x2 = mad64s(m2, p[0], x2);
#pragma unroll
    for (int b = 0; b < (K - 1) / BL; ++b) {
      const int j = 1 + BL * b;
      blk1(T1, a, e, m1, j);
      if constexpr (SQ) blk2s(T2, c, e << 1, m2, j);
      else blk2(T2, c, a, e, f, m2, j);
      if (b == 0) {
        T1[0] += x1 >> W;
        T2[0] += x2 >> W;
        asm volatile("" : "+v"(T1[0]), "+v"(T2[0]));
      } else if (b == 1) {
        x1n = mad64(en, a[0], T1[0]);
        if constexpr (SQ) x2n = mad64(en << 1, c[0], T2[0]);
        else x2n = mad64(fn, a[0], mad64(en, c[0], T2[0]));
        asm volatile("" : "+v"(x1n), "+v"(x2n));
      } else if (b == 2) {
        t1 = (uint32_t)x1n * n0inv;
        t2 = (uint32_t)x2n * n0inv;
        asm volatile("" : "+v"(t1), "+v"(t2));
      } else if (b == 3) {
        m1n = t1 & MASK;
        m2n = t2 & MASK;
        asm volatile("" : "+v"(m1n), "+v"(m2n));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    T1[K - 1] = 0;
    T2[K - 1] = (uint64_t)(topc - m1);  // (MASK - m1) + E_i at weight 2^(W i) of c'
    x1 = x1n;
    x2 = x2n;
    m1 = m1n;
    m2 = m2n;
  }

  // (a, c) <- (a, c) (x) (e, f): the row's limbs interleaved in the lane's
  // slot of a quad-major LDS image (quad q = e_2q, f_2q, e_2q+1, f_2q+1 at
  // slot[q * 256]); topc: K words MASK + E_i (LDS, shared by the block).
  XHE_DEV void mul(uint32_t (&a)[K], uint32_t (&c)[K], const uint32_t* slot, const uint32_t* topc) const {
    run<false>(a, c, slot, topc);
  }
  // (a, c) <- (a, c)^2: the state parked in the slot (same layout) as the
  // streamed operand; 4 K^2 mads (squaring steps)
  XHE_DEV void sqr(uint32_t (&a)[K], uint32_t (&c)[K], const uint32_t* slot, const uint32_t* topc) const {
    run<true>(a, c, slot, topc);
  }
  template <bool SQ>
  XHE_DEV void run(uint32_t (&a)[K], uint32_t (&c)[K], const uint32_t* slot, const uint32_t* topc) const {
    uint64_t T1[K], T2[K];
#pragma unroll
    for (int j = 0; j < K; ++j) T1[j] = T2[j] = 0;
    // one (e_i, f_i) pair in flight ahead of the step that consumes it (a
    // ds_read_b64 at the start of the step before): 4 row registers live
    // instead of two whole quads
    uint2 p0 = *reinterpret_cast<const uint2*>(slot);
    uint64_t x1 = mad64(p0.x, a[0], 0ull);
    uint64_t x2 = SQ ? mad64(p0.x << 1, c[0], 0ull) : mad64(p0.y, a[0], mad64(p0.x, c[0], 0ull));
    uint32_t m1 = ((uint32_t)x1 * n0inv) & MASK, m2 = ((uint32_t)x2 * n0inv) & MASK;
    for (int q = 0; q < K / 2; ++q) {
      const uint32_t* sq = slot + q * 256;
      const uint2 tc = *reinterpret_cast<const uint2*>(topc + 2 * q);
      const uint2 p1 = *reinterpret_cast<const uint2*>(sq + 2);
      __builtin_amdgcn_sched_barrier(0);
      step<SQ>(T1, T2, a, c, p0.x, p0.y, p1.x, p1.y, m1, m2, x1, x2, tc.x);
      __builtin_amdgcn_sched_barrier(0);
      p0 = *reinterpret_cast<const uint2*>(sq + 256);
      __builtin_amdgcn_sched_barrier(0);
      step<SQ>(T1, T2, a, c, p1.x, p1.y, p0.x, p0.y, m1, m2, x1, x2, tc.y);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (K & 1) step<SQ>(T1, T2, a, c, p0.x, p0.y, 0u, 0u, m1, m2, x1, x2, topc[K - 1]);
    normalize(T1, a);
    normalize(T2, c);
  }

  // carry-normalise into W-bit limbs; the top limb keeps the final carry
  XHE_DEV static void normalize(const uint64_t (&T)[K], uint32_t (&b)[K]) {
    uint64_t cy = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint64_t x = T[j] + cy;
      b[j] = j + 1 < K ? ((uint32_t)x & MASK) : (uint32_t)x;
      cy = x >> W;
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // X = R a + P c as 2K limbs (< 2^13 P^2: the 74-limb Montgomery
  // representation x R^2 of the residue, unreduced), for the products mod P^2
  // that follow (Mont<2K, 28, 1> accepts one operand up to R^2/P^2 times its
  // modulus). Operand scanning, fully unrolled: K^2 mads.
  XHE_DEV void to_mont2(const uint32_t (&a)[K], const uint32_t (&c)[K], uint32_t (&x)[2 * K]) const {
    uint64_t T[2 * K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      T[j] = 0;
      T[K + j] = a[j];
    }
#pragma unroll
    for (int i = 0; i < K; ++i) {
#pragma unroll
      for (int j = 0; j < K; ++j) T[i + j] = mad64s(c[j], p[i], T[i + j]);
    }
    uint64_t cy = 0;
#pragma unroll
    for (int j = 0; j < 2 * K; ++j) {
      const uint64_t v = T[j] + cy;
      x[j] = j + 1 < 2 * K ? ((uint32_t)v & MASK) : (uint32_t)v;
      cy = v >> W;
    }
  }
};

// ---------------------------------------------------------------- conversion
// REDC by P of a 2K-limb value given as lazy 64-bit column sums T (value <
// R P): t = T R^-1 mod P (< 2P, K limbs, normalised) and the quotient digits
// m (T + m P = R t). Plain code: used once per table row, not in the hot loop.
template <int K>
XHE_DEV void pmd_redc_wide(const PMD<K>& M, uint64_t (&T)[2 * K], uint32_t (&t)[K], uint32_t (&m)[K]) {
  constexpr uint32_t MASK = PMD<K>::MASK;
  uint64_t cy = 0;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    uint64_t x = T[i] + cy;
    const uint32_t mi = ((uint32_t)x * M.n0inv) & MASK;
    m[i] = mi;
    x = mad64s(mi, M.p[0], x);
    cy = x >> 28;
#pragma unroll
    for (int j = 1; j < K; ++j) T[i + j] = mad64s(mi, M.p[j], T[i + j]);
    __builtin_amdgcn_sched_barrier(0);  // one row at a time (rows interleaved by the scheduler spill)
  }
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint64_t x = T[K + j] + cy;
    t[j] = j + 1 < K ? ((uint32_t)x & MASK) : (uint32_t)x;
    cy = x >> 28;
  }
}

// r - s (K limbs each, both < 2^(28K)); returns the borrow out (1 if r < s)
template <int K>
XHE_DEV uint32_t pmd_sub(uint32_t (&r)[K], const uint32_t (&s)[K]) {
  int64_t br = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int64_t v = (int64_t)r[j] - (int64_t)s[j] + br;
    r[j] = (uint32_t)v & ((1u << 28) - 1u);
    br = v >> 28;  // 0 or -1
  }
  return br ? 1u : 0u;
}

// r <- r - P if r >= P (r < 2^(28K)); returns whether it subtracted. Two
// passes (the borrow of r - P, then a masked subtraction) instead of a copy
// and a select: no second K-limb temporary.
template <int K>
XHE_DEV bool pmd_csub(const PMD<K>& M, uint32_t (&r)[K]) {
  int64_t br = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) br = ((int64_t)r[j] - (int64_t)M.p[j] + br) >> 28;
  const bool ge = br == 0;
  br = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int64_t v = (int64_t)r[j] - (int64_t)(ge ? M.p[j] : 0u) + br;
    r[j] = (uint32_t)v & ((1u << 28) - 1u);
    br = v >> 28;
  }
  return ge;
}

// m mod P for 0 <= m < 2^(28K) (< 2^13 P at K = 37), in place: one
// quotient limb q from 32-bit tops (m >> (28K - 32) over (P >> (28K - 32))
// + 1; P >= 2^(28K - 13), so the estimate is at most 3 below floor(m / P)),
// then m - q P and three conditional subtractions of P.
template <int K>
XHE_DEV void pmd_mod_small(const PMD<K>& M, uint32_t (&m)[K]) {
  constexpr uint32_t MASK = PMD<K>::MASK;
  const uint32_t mt = (m[K - 1] << 4) | (m[K - 2] >> 24);      // bits [28K - 32, 28K)
  const uint32_t pt = (M.p[K - 1] << 4) | (M.p[K - 2] >> 24);  // >= 2^19
  const uint32_t q = mt / (pt + 1u);
  uint64_t cy = 0;
  int64_t br = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint64_t qp = (uint64_t)q * M.p[j] + cy;
    cy = qp >> 28;
    const int64_t v = (int64_t)m[j] - (int64_t)(qp & MASK) + br;
    m[j] = (uint32_t)v & MASK;
    br = v >> 28;
  }
#pragma unroll
  for (int t = 0; t < 3; ++t) pmd_csub<K>(M, m);
}

// Table-row conversion: a reduced residue X = x R^2 mod P^2 (< P^2, 2K limbs:
// the 74-limb Montgomery form the table kernels produce) into its Montgomery
// digits (e, f), both in [0, P). REDC gives X = R t - m P with t < 2P, m <
// R; then e = t mod P and f = ([t >= P] R - m) mod P.
template <int K>
XHE_DEV void pmd_from_mont2(const PMD<K>& M, const uint32_t (&X)[2 * K], const uint32_t* RmodP, uint32_t (&e)[K],
                            uint32_t (&f)[K]) {
  uint32_t m[K];
  {
    uint64_t T[2 * K];
#pragma unroll
    for (int j = 0; j < 2 * K; ++j) T[j] = X[j];
    pmd_redc_wide<K>(M, T, e, m);
  }
  __builtin_amdgcn_sched_barrier(0);
  const bool ge = pmd_csub<K>(M, e);  // t >= P
  __builtin_amdgcn_sched_barrier(0);
  pmd_mod_small<K>(M, m);
  __builtin_amdgcn_sched_barrier(0);
  // f = (ge ? R mod P : 0) - (m mod P), plus P on a borrow
  int64_t br = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int64_t v = (int64_t)(ge ? RmodP[j] : 0u) - (int64_t)m[j] + br;
    f[j] = (uint32_t)v & ((1u << 28) - 1u);
    br = v >> 28;
  }
  if (br) {
    int64_t cy = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const int64_t v = (int64_t)f[j] + (int64_t)M.p[j] + cy;
      f[j] = (uint32_t)v & ((1u << 28) - 1u);
      cy = v >> 28;
    }
  }
}

// The interleaved row image: a lane's packed row (RW = 2K' words: digit e in
// words [0, RW/2), f in [RW/2, RW), little-endian, staged quad-major in its
// slot by LDS-DMA) rewritten in the same slot as NQ quads of 28-bit limb pairs
// (e_2q, f_2q, e_2q+1, f_2q+1). The packed words go through registers first
// (the image grows from RW/4 to NQ quads in place).
template <int K, int RW>
XHE_DEV void unpack_pairs_lds(uint32_t* slot) {
  constexpr int HW = RW / 2;
  uint32_t w[RW];
#pragma unroll
  for (int q = 0; q < RW / 4; ++q) {
    const uint4 v = *reinterpret_cast<const uint4*>(slot + q * 256);
    w[4 * q] = v.x;
    w[4 * q + 1] = v.y;
    w[4 * q + 2] = v.z;
    w[4 * q + 3] = v.w;
  }
  auto limb = [&](int base, int i) -> uint32_t {
    const int bit = 28 * i, k = bit >> 5, sh = bit & 31;
    const uint32_t lo = k < HW ? w[base + k] : 0u, hi = k + 1 < HW ? w[base + k + 1] : 0u;
    return i < K ? (__builtin_amdgcn_alignbit(hi, lo, sh) & ((1u << 28) - 1u)) : 0u;
  };
#pragma unroll
  for (int q = 0; q < (2 * K + 3) / 4; ++q)
    *reinterpret_cast<uint4*>(slot + q * 256) =
        make_uint4(limb(0, 2 * q), limb(HW, 2 * q), limb(0, 2 * q + 1), limb(HW, 2 * q + 1));
}

}  // namespace xhe
