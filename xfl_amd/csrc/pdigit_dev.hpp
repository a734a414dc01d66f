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

  // One block of 6 positions of both accumulators in ONE asm statement (tied
  // accumulators: T[j-1+k] is written after its old value was consumed, so
  // the registers stay put and no rotation copies appear; the compiler puts
  // a hazard nop after every asm statement, so one statement per block):
  //   T1[j-1+k] = T1[j+k] + e a[j+k] + m1 P[j+k]
  //   T2[j-1+k] = T2[j+k] + e c[j+k] + f a[j+k] + m2 P[j+k]   (SQ: f (= 2 a_i) c[j+k] + m2 P[j+k])
  template <bool SQ>
  XHE_DEV void blk12(uint64_t (&T1)[K], uint64_t (&T2)[K], const uint32_t (&a)[K], const uint32_t (&c)[K],
                     uint32_t e, uint32_t f, uint32_t m1, uint32_t m2, int j) const {
    if constexpr (SQ) {
      asm(
        "v_mad_u64_u32 %0, vcc, %14, %18, %1\n\t"
        "v_mad_u64_u32 %1, vcc, %14, %19, %2\n\t"
        "v_mad_u64_u32 %2, vcc, %14, %20, %3\n\t"
        "v_mad_u64_u32 %3, vcc, %14, %21, %4\n\t"
        "v_mad_u64_u32 %4, vcc, %14, %22, %5\n\t"
        "v_mad_u64_u32 %5, vcc, %14, %23, %12\n\t"
        "v_mad_u64_u32 %6, vcc, %15, %24, %7\n\t"
        "v_mad_u64_u32 %7, vcc, %15, %25, %8\n\t"
        "v_mad_u64_u32 %8, vcc, %15, %26, %9\n\t"
        "v_mad_u64_u32 %9, vcc, %15, %27, %10\n\t"
        "v_mad_u64_u32 %10, vcc, %15, %28, %11\n\t"
        "v_mad_u64_u32 %11, vcc, %15, %29, %13\n\t"
        "v_mad_u64_u32 %0, vcc, %16, %30, %0\n\t"
        "v_mad_u64_u32 %1, vcc, %16, %31, %1\n\t"
        "v_mad_u64_u32 %2, vcc, %16, %32, %2\n\t"
        "v_mad_u64_u32 %3, vcc, %16, %33, %3\n\t"
        "v_mad_u64_u32 %4, vcc, %16, %34, %4\n\t"
        "v_mad_u64_u32 %5, vcc, %16, %35, %5\n\t"
        "v_mad_u64_u32 %6, vcc, %17, %30, %6\n\t"
        "v_mad_u64_u32 %7, vcc, %17, %31, %7\n\t"
        "v_mad_u64_u32 %8, vcc, %17, %32, %8\n\t"
        "v_mad_u64_u32 %9, vcc, %17, %33, %9\n\t"
        "v_mad_u64_u32 %10, vcc, %17, %34, %10\n\t"
        "v_mad_u64_u32 %11, vcc, %17, %35, %11"
          : "+v"(T1[j - 1]), "+v"(T1[j]), "+v"(T1[j + 1]), "+v"(T1[j + 2]), "+v"(T1[j + 3]), "+v"(T1[j + 4]),
            "+v"(T2[j - 1]), "+v"(T2[j]), "+v"(T2[j + 1]), "+v"(T2[j + 2]), "+v"(T2[j + 3]), "+v"(T2[j + 4])
          : "v"(T1[j + 5]), "v"(T2[j + 5]), "v"(e), "v"(f), "v"(m1), "v"(m2), "v"(a[j]), "v"(a[j + 1]),
            "v"(a[j + 2]), "v"(a[j + 3]), "v"(a[j + 4]), "v"(a[j + 5]), "v"(c[j]), "v"(c[j + 1]), "v"(c[j + 2]),
            "v"(c[j + 3]), "v"(c[j + 4]), "v"(c[j + 5]), "s"(p[j]), "s"(p[j + 1]), "s"(p[j + 2]), "s"(p[j + 3]),
            "s"(p[j + 4]), "s"(p[j + 5])
          : "vcc");
    } else {
      asm(
        "v_mad_u64_u32 %0, vcc, %14, %18, %1\n\t"
        "v_mad_u64_u32 %1, vcc, %14, %19, %2\n\t"
        "v_mad_u64_u32 %2, vcc, %14, %20, %3\n\t"
        "v_mad_u64_u32 %3, vcc, %14, %21, %4\n\t"
        "v_mad_u64_u32 %4, vcc, %14, %22, %5\n\t"
        "v_mad_u64_u32 %5, vcc, %14, %23, %12\n\t"
        "v_mad_u64_u32 %6, vcc, %14, %24, %7\n\t"
        "v_mad_u64_u32 %7, vcc, %14, %25, %8\n\t"
        "v_mad_u64_u32 %8, vcc, %14, %26, %9\n\t"
        "v_mad_u64_u32 %9, vcc, %14, %27, %10\n\t"
        "v_mad_u64_u32 %10, vcc, %14, %28, %11\n\t"
        "v_mad_u64_u32 %11, vcc, %14, %29, %13\n\t"
        "v_mad_u64_u32 %0, vcc, %16, %30, %0\n\t"
        "v_mad_u64_u32 %1, vcc, %16, %31, %1\n\t"
        "v_mad_u64_u32 %2, vcc, %16, %32, %2\n\t"
        "v_mad_u64_u32 %3, vcc, %16, %33, %3\n\t"
        "v_mad_u64_u32 %4, vcc, %16, %34, %4\n\t"
        "v_mad_u64_u32 %5, vcc, %16, %35, %5\n\t"
        "v_mad_u64_u32 %6, vcc, %15, %18, %6\n\t"
        "v_mad_u64_u32 %7, vcc, %15, %19, %7\n\t"
        "v_mad_u64_u32 %8, vcc, %15, %20, %8\n\t"
        "v_mad_u64_u32 %9, vcc, %15, %21, %9\n\t"
        "v_mad_u64_u32 %10, vcc, %15, %22, %10\n\t"
        "v_mad_u64_u32 %11, vcc, %15, %23, %11\n\t"
        "v_mad_u64_u32 %6, vcc, %17, %30, %6\n\t"
        "v_mad_u64_u32 %7, vcc, %17, %31, %7\n\t"
        "v_mad_u64_u32 %8, vcc, %17, %32, %8\n\t"
        "v_mad_u64_u32 %9, vcc, %17, %33, %9\n\t"
        "v_mad_u64_u32 %10, vcc, %17, %34, %10\n\t"
        "v_mad_u64_u32 %11, vcc, %17, %35, %11"
          : "+v"(T1[j - 1]), "+v"(T1[j]), "+v"(T1[j + 1]), "+v"(T1[j + 2]), "+v"(T1[j + 3]), "+v"(T1[j + 4]),
            "+v"(T2[j - 1]), "+v"(T2[j]), "+v"(T2[j + 1]), "+v"(T2[j + 2]), "+v"(T2[j + 3]), "+v"(T2[j + 4])
          : "v"(T1[j + 5]), "v"(T2[j + 5]), "v"(e), "v"(f), "v"(m1), "v"(m2), "v"(a[j]), "v"(a[j + 1]),
            "v"(a[j + 2]), "v"(a[j + 3]), "v"(a[j + 4]), "v"(a[j + 5]), "v"(c[j]), "v"(c[j + 1]), "v"(c[j + 2]),
            "v"(c[j + 3]), "v"(c[j + 4]), "v"(c[j + 5]), "s"(p[j]), "s"(p[j + 1]), "s"(p[j + 2]), "s"(p[j + 3]),
            "s"(p[j + 4]), "s"(p[j + 5])
          : "vcc");
    }
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
    asm("v_mad_u64_u32 %0, vcc, %2, %4, %0\n\t"  // x1 += m1 P_0: now = 0 (mod 2^W); x2 likewise
        "v_mad_u64_u32 %1, vcc, %3, %4, %1"
        : "+v"(x1), "+v"(x2)
        : "v"(m1), "v"(m2), "s"(p[0])
        : "vcc");
#pragma unroll
    for (int b = 0; b < (K - 1) / BL; ++b) {
      const int j = 1 + BL * b;
      blk12<SQ>(T1, T2, a, c, e, SQ ? (e << 1) : f, m1, m2, j);
      if (b == 0) {
        T1[0] += x1 >> W;
        T2[0] += x2 >> W;
        asm volatile("" : "+v"(T1[0]), "+v"(T2[0]));
      } else if (b == 1) {
        if constexpr (SQ) {
          asm("v_mad_u64_u32 %0, vcc, %2, %3, %5\n\t"
              "v_mad_u64_u32 %1, vcc, %4, %7, %6"
              : "=&v"(x1n), "=v"(x2n)
              : "v"(en), "v"(a[0]), "v"(en << 1), "v"(T1[0]), "v"(T2[0]), "v"(c[0])
              : "vcc");
        } else {
          asm("v_mad_u64_u32 %0, vcc, %2, %4, %6\n\t"
              "v_mad_u64_u32 %1, vcc, %2, %5, %7\n\t"
              "v_mad_u64_u32 %1, vcc, %3, %4, %1"
              : "=&v"(x1n), "=&v"(x2n)
              : "v"(en), "v"(fn), "v"(a[0]), "v"(c[0]), "v"(T1[0]), "v"(T2[0])
              : "vcc");
        }
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

namespace xhe {

// ---------------------------------------------------------------------------
// Montgomery digits mod n^2 over TPI lanes (PMDX; 2048-bit keys: K = 80
// limbs of W = 27 bits, R = 2^2160, TPI = 4 lanes of L = 20 limbs). The same
// representation and product as PMD with the modulus n in place of P
// (x R^2 = R a + n c mod n^2), spread over a lane group like Mont<K, 27, TPI>:
// lane g holds limbs [gL, (g+1)L) of a, c and of the two lazy accumulators.
// 27-bit limbs because the columns collect 3 products of up to 2^56 per step
// over K = 80 steps (tools/pdigit_model.py NDigits: columns below 2^62).
// The operand (e_i, f_i) of step i is read by all lanes of the group from
// one LDS pair (a broadcast read; `OpLds`) or from a uniform global row
// (`OpRow`, the conversion constants); the quotient digits m1, m2 are formed
// on lane 0 and broadcast by DPP, and each step hands the low limb of every
// lane down to the lane before (from_next) while the lane keeps its carry -
// the multi-lane Montgomery step of bn_dev.hpp with two accumulators.
struct OpLds {  // pair i of a group's operand at p[i * stride]
  const uint2* p;
  int stride;
  XHE_DEV uint2 load(int i) const { return p[i * stride]; }
};
struct OpRow {  // a uniform row of K pairs (key constants)
  const uint2* __restrict__ p;
  XHE_DEV uint2 load(int i) const { return p[i]; }
};

template <int K_, int TPI_>
struct PMDX {
  static constexpr int K = K_, TPI = TPI_, L = K_ / TPI_, W = 27;
  static constexpr uint32_t MASK = (1u << W) - 1u;
  using G = Grp<TPI_>;
  using MN = Mont<K_, 27, TPI_>;  // the same limbs mod n: Montgomery products, reduce_once, I/O
  static_assert(K_ % TPI_ == 0 && L >= 8, "lane groups of at least 8 limbs");
  static_assert((double)K_ * (double)(5ull << 54) < 18446744073709551616.0, "accumulator bound");

  MN M;  // n limbs of this lane (M.nl), n0inv

  XHE_DEV void init(const uint32_t* N, uint32_t ninv) { M.init(N, ninv); }
  XHE_DEV static bool last() { return G::g() == TPI - 1; }

  // Blocks of 4 limbs of both accumulators in one asm statement (tied in/out
  // accumulators: T[j-1+k] is written after its old value was consumed, so
  // the registers stay put and no rotation copies appear; one statement per
  // block keeps the hazard nops the compiler puts after each asm low):
  //   T1[j-1+k] = T1[j+k] + e a[j+k] + m1 n[j+k]
  //   T2[j-1+k] = T2[j+k] + e c[j+k] + f a[j+k] + m2 n[j+k]   (SQ: 2e c[j+k] + m2 n[j+k])
  template <bool SQ>
  XHE_DEV void blk4(uint64_t (&T1)[L], uint64_t (&T2)[L], const uint32_t (&a)[L], const uint32_t (&c)[L],
                    uint32_t e, uint32_t f, uint32_t m1, uint32_t m2, int j) const {
    if constexpr (SQ) {
      // f carries 2e
      asm("v_mad_u64_u32 %0, vcc, %10, %14, %1\n\t"
          "v_mad_u64_u32 %1, vcc, %10, %15, %2\n\t"
          "v_mad_u64_u32 %2, vcc, %10, %16, %3\n\t"
          "v_mad_u64_u32 %3, vcc, %10, %17, %8\n\t"
          "v_mad_u64_u32 %4, vcc, %11, %18, %5\n\t"
          "v_mad_u64_u32 %5, vcc, %11, %19, %6\n\t"
          "v_mad_u64_u32 %6, vcc, %11, %20, %7\n\t"
          "v_mad_u64_u32 %7, vcc, %11, %21, %9\n\t"
          "v_mad_u64_u32 %0, vcc, %12, %22, %0\n\t"
          "v_mad_u64_u32 %1, vcc, %12, %23, %1\n\t"
          "v_mad_u64_u32 %2, vcc, %12, %24, %2\n\t"
          "v_mad_u64_u32 %3, vcc, %12, %25, %3\n\t"
          "v_mad_u64_u32 %4, vcc, %13, %22, %4\n\t"
          "v_mad_u64_u32 %5, vcc, %13, %23, %5\n\t"
          "v_mad_u64_u32 %6, vcc, %13, %24, %6\n\t"
          "v_mad_u64_u32 %7, vcc, %13, %25, %7"
          : "+v"(T1[j - 1]), "+v"(T1[j]), "+v"(T1[j + 1]), "+v"(T1[j + 2]), "+v"(T2[j - 1]), "+v"(T2[j]),
            "+v"(T2[j + 1]), "+v"(T2[j + 2])
          : "v"(T1[j + 3]), "v"(T2[j + 3]), "v"(e), "v"(f), "v"(m1), "v"(m2), "v"(a[j]), "v"(a[j + 1]),
            "v"(a[j + 2]), "v"(a[j + 3]), "v"(c[j]), "v"(c[j + 1]), "v"(c[j + 2]), "v"(c[j + 3]), "v"(M.nl[j]),
            "v"(M.nl[j + 1]), "v"(M.nl[j + 2]), "v"(M.nl[j + 3])
          : "vcc");
    } else {
      // T1: e a + m1 n; T2: e c + f a + m2 n (a[j..] are shared by both)
      asm("v_mad_u64_u32 %0, vcc, %10, %14, %1\n\t"
          "v_mad_u64_u32 %1, vcc, %10, %15, %2\n\t"
          "v_mad_u64_u32 %2, vcc, %10, %16, %3\n\t"
          "v_mad_u64_u32 %3, vcc, %10, %17, %8\n\t"
          "v_mad_u64_u32 %4, vcc, %10, %18, %5\n\t"
          "v_mad_u64_u32 %5, vcc, %10, %19, %6\n\t"
          "v_mad_u64_u32 %6, vcc, %10, %20, %7\n\t"
          "v_mad_u64_u32 %7, vcc, %10, %21, %9\n\t"
          "v_mad_u64_u32 %4, vcc, %11, %14, %4\n\t"
          "v_mad_u64_u32 %5, vcc, %11, %15, %5\n\t"
          "v_mad_u64_u32 %6, vcc, %11, %16, %6\n\t"
          "v_mad_u64_u32 %7, vcc, %11, %17, %7\n\t"
          "v_mad_u64_u32 %0, vcc, %12, %22, %0\n\t"
          "v_mad_u64_u32 %1, vcc, %12, %23, %1\n\t"
          "v_mad_u64_u32 %2, vcc, %12, %24, %2\n\t"
          "v_mad_u64_u32 %3, vcc, %12, %25, %3\n\t"
          "v_mad_u64_u32 %4, vcc, %13, %22, %4\n\t"
          "v_mad_u64_u32 %5, vcc, %13, %23, %5\n\t"
          "v_mad_u64_u32 %6, vcc, %13, %24, %6\n\t"
          "v_mad_u64_u32 %7, vcc, %13, %25, %7"
          : "+v"(T1[j - 1]), "+v"(T1[j]), "+v"(T1[j + 1]), "+v"(T1[j + 2]), "+v"(T2[j - 1]), "+v"(T2[j]),
            "+v"(T2[j + 1]), "+v"(T2[j + 2])
          : "v"(T1[j + 3]), "v"(T2[j + 3]), "v"(e), "v"(f), "v"(m1), "v"(m2), "v"(a[j]), "v"(a[j + 1]),
            "v"(a[j + 2]), "v"(a[j + 3]), "v"(c[j]), "v"(c[j + 1]), "v"(c[j + 2]), "v"(c[j + 3]), "v"(M.nl[j]),
            "v"(M.nl[j + 1]), "v"(M.nl[j + 2]), "v"(M.nl[j + 3])
          : "vcc");
    }
  }

  // one position of both accumulators in one asm statement (the tail past
  // the 4-limb blocks; separate mad statements each cost a hazard nop)
  template <bool SQ>
  XHE_DEV void blk1(uint64_t (&T1)[L], uint64_t (&T2)[L], const uint32_t (&a)[L], const uint32_t (&c)[L],
                    uint32_t e, uint32_t f, uint32_t m1, uint32_t m2, int j) const {
    if constexpr (SQ) {  // f carries 2e
      asm("v_mad_u64_u32 %0, vcc, %4, %6, %2\n\t"
          "v_mad_u64_u32 %1, vcc, %5, %7, %3\n\t"
          "v_mad_u64_u32 %0, vcc, %8, %10, %0\n\t"
          "v_mad_u64_u32 %1, vcc, %9, %10, %1"
          : "+v"(T1[j - 1]), "+v"(T2[j - 1])
          : "v"(T1[j]), "v"(T2[j]), "v"(e), "v"(f), "v"(a[j]), "v"(c[j]), "v"(m1), "v"(m2), "v"(M.nl[j])
          : "vcc");
    } else {
      asm("v_mad_u64_u32 %0, vcc, %4, %6, %2\n\t"
          "v_mad_u64_u32 %1, vcc, %4, %7, %3\n\t"
          "v_mad_u64_u32 %0, vcc, %8, %10, %0\n\t"
          "v_mad_u64_u32 %1, vcc, %5, %6, %1\n\t"
          "v_mad_u64_u32 %1, vcc, %9, %10, %1"
          : "+v"(T1[j - 1]), "+v"(T2[j - 1])
          : "v"(T1[j]), "v"(T2[j]), "v"(e), "v"(f), "v"(a[j]), "v"(c[j]), "v"(m1), "v"(m2), "v"(M.nl[j])
          : "vcc");
    }
  }

  // one step of the two interleaved reductions (see PMD::step); entry: x1 =
  // T1[0] + e a[0], x2 = T2[0] + e c[0] + f a[0] (or 2e c[0]) and the
  // broadcast digits m1, m2; the next step's x and m are formed under this
  // step's mads, one link after each block. topc: MASK + E_i (used by the
  // group's last lane).
  template <bool SQ>
  XHE_DEV void step(uint64_t (&T1)[L], uint64_t (&T2)[L], const uint32_t (&a)[L], const uint32_t (&c)[L],
                    uint32_t e, uint32_t f, uint32_t en, uint32_t fn, uint32_t& m1, uint32_t& m2, uint64_t& x1,
                    uint64_t& x2, uint32_t topc) const {
    static_assert(L >= 8, "positions 1..L-1: 4-limb blocks and a tail");
    uint64_t v1, v2;  // v1 = x1 + m1 n_0 (lane 0: = 0 mod 2^W), v2 likewise, one statement
    asm("v_mad_u64_u32 %0, vcc, %2, %4, %5\n\t"
        "v_mad_u64_u32 %1, vcc, %3, %4, %6"
        : "=&v"(v1), "=v"(v2)
        : "v"(m1), "v"(m2), "v"(M.nl[0]), "v"(x1), "v"(x2)
        : "vcc");
    // the limbs handed down to lane g-1 (DPP sources well before the DPP)
    const uint32_t h1 = (uint32_t)v1 & MASK, h2 = (uint32_t)v2 & MASK;
    const uint32_t f2 = SQ ? (e << 1) : f;
    uint64_t x1n = 0, x2n = 0;
    uint32_t t1 = 0, t2 = 0, d1 = 0, d2 = 0;
    int stage = 0;
    auto advance = [&]() XHE_INL {
      if (stage == 0) {
        T1[0] += v1 >> W;
        T2[0] += v2 >> W;
        asm volatile("" : "+v"(T1[0]), "+v"(T2[0]));
      } else if (stage == 1) {
        if constexpr (SQ) {
          asm("v_mad_u64_u32 %0, vcc, %2, %3, %5\n\t"
              "v_mad_u64_u32 %1, vcc, %4, %7, %6"
              : "=&v"(x1n), "=v"(x2n)
              : "v"(en), "v"(a[0]), "v"(en << 1), "v"(T1[0]), "v"(T2[0]), "v"(c[0])
              : "vcc");
        } else {
          asm("v_mad_u64_u32 %0, vcc, %2, %4, %6\n\t"
              "v_mad_u64_u32 %1, vcc, %2, %5, %7\n\t"
              "v_mad_u64_u32 %1, vcc, %3, %4, %1"
              : "=&v"(x1n), "=&v"(x2n)
              : "v"(en), "v"(fn), "v"(a[0]), "v"(c[0]), "v"(T1[0]), "v"(T2[0])
              : "vcc");
        }
        asm volatile("" : "+v"(x1n), "+v"(x2n));
      } else if (stage == 2) {
        t1 = (uint32_t)x1n * M.n0inv;
        t2 = (uint32_t)x2n * M.n0inv;
        d1 = G::from_next(h1);
        d2 = G::from_next_any(h2);  // (the last lane takes topc - m1 instead)
        asm volatile("" : "+v"(t1), "+v"(t2), "+v"(d1), "+v"(d2));
      } else if (stage == 3) {
        t1 = G::bcast0(t1 & MASK);
        t2 = G::bcast0(t2 & MASK);
        asm volatile("" : "+v"(t1), "+v"(t2));
      }
      ++stage;
      __builtin_amdgcn_sched_barrier(0);
    };
    int j = 1;
#pragma unroll
    for (; j + 4 <= L; j += 4) {
      blk4<SQ>(T1, T2, a, c, e, f2, m1, m2, j);
      advance();
    }
#pragma unroll
    for (; j < L; ++j) blk1<SQ>(T1, T2, a, c, e, f2, m1, m2, j);  // the tail
    while (stage < 4) advance();
    T1[L - 1] = d1;
    T2[L - 1] = last() ? (uint64_t)(topc - m1) : (uint64_t)d2;
    x1 = x1n;
    x2 = x2n;
    m1 = t1;
    m2 = t2;
  }

  // (a, c) <- (a, c) (x) operand; SQ: the operand is (a, c) itself (parked
  // in the group's LDS pairs by the caller), 4 K^2 instead of 5 K^2 mads
  template <bool SQ, class OP>
  XHE_DEV void run(uint32_t (&a)[L], uint32_t (&c)[L], const OP& op, const uint32_t* topc) const {
    uint64_t T1[L], T2[L];
#pragma unroll
    for (int j = 0; j < L; ++j) T1[j] = T2[j] = 0;
    uint2 p0 = op.load(0);
    uint64_t x1 = mad64(p0.x, a[0], 0ull);
    uint64_t x2 = SQ ? mad64(p0.x << 1, c[0], 0ull) : mad64(p0.y, a[0], mad64(p0.x, c[0], 0ull));
    uint32_t m1 = G::bcast0(((uint32_t)x1 * M.n0inv) & MASK), m2 = G::bcast0(((uint32_t)x2 * M.n0inv) & MASK);
    for (int i = 0; i < K; i += 2) {
      const uint2 tc = *reinterpret_cast<const uint2*>(topc + i);
      const uint2 p1 = op.load(i + 1);
      __builtin_amdgcn_sched_barrier(0);
      step<SQ>(T1, T2, a, c, p0.x, p0.y, p1.x, p1.y, m1, m2, x1, x2, tc.x);
      __builtin_amdgcn_sched_barrier(0);
      p0 = op.load(i + 2 < K ? i + 2 : i);
      __builtin_amdgcn_sched_barrier(0);
      step<SQ>(T1, T2, a, c, p1.x, p1.y, p0.x, p0.y, m1, m2, x1, x2, tc.y);
      __builtin_amdgcn_sched_barrier(0);
    }
    normalize_top(T1, a);
    normalize_top(T2, c);
  }

  // carry-normalise lazy columns into W-bit limbs across the group; what
  // leaves the group's top limb stays in it (unmasked): c' may exceed R
  XHE_DEV static void normalize_top(const uint64_t (&T)[L], uint32_t (&b)[L]) {
    uint64_t cy = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const uint64_t x = T[j] + cy;
      b[j] = (uint32_t)x & MASK;
      cy = x >> W;
      __builtin_amdgcn_sched_barrier(0);
    }
    // one round of lane-to-lane carries (cy < 2^38), then every lane's carry
    // out is 0 or 1 and passes a lane only when all its limbs are MASK: a
    // carry-lookahead on the wave's lane masks as Mont::normalize, except that
    // the group's top lane keeps its carry out in its top limb
    const bool top = last();
    uint64_t cin = G::from_prev64(cy);
    uint64_t out = top ? cy : 0ull;
    uint32_t all = 1u;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const uint64_t x = (uint64_t)b[j] + cin;
      b[j] = (uint32_t)x & MASK;
      cin = x >> W;
      all &= (b[j] == MASK) ? 1u : 0u;
    }
    // generate: cin (0 or 1) leaves the lane; propagate: all limbs MASK
    constexpr uint64_t tops = TPI == 16 ? 0x8000800080008000ull : TPI == 8 ? 0x8080808080808080ull
                              : TPI == 4 ? 0x8888888888888888ull : 0xAAAAAAAAAAAAAAAAull;
    const uint64_t gm = __builtin_amdgcn_ballot_w64(cin != 0);
    const uint64_t pm = __builtin_amdgcn_ballot_w64(all != 0);
    const uint64_t gi = gm & ~tops, ti = (gm | pm) & ~tops;
    const uint64_t cm = (gi + ti) ^ gi ^ ti;  // carries into each lane (none across groups)
    uint32_t ci = (uint32_t)(cm >> (threadIdx.x & 63)) & 1u;
    // the top lane's own carry out: generated there, or propagated through it
    if (top) out += cin + ((all && ci) ? 1u : 0u);
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const uint32_t x = b[j] + ci;
      b[j] = x & MASK;
      ci = x >> W;
    }
    if (top) b[L - 1] += (uint32_t)out << W;
  }

  // group-uniform DPP broadcast of lane k's value (k a constant after unrolling)
  template <int k>
  XHE_DEV static uint32_t from_lane(uint32_t v) {
    if constexpr (TPI == 4) return G::template dpp<k | (k << 2) | (k << 4) | (k << 6)>(v);
    else if constexpr (TPI == 2) return G::template dpp<k | (k << 2) | ((2 + k) << 4) | ((2 + k) << 6)>(v);
    else if constexpr (TPI == 8) {  // half rows: lane k of each half
      const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x150 + k, 0xF, 0xF, true);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x158 + k, 0xF, 0xF, true);
      return G::upper8() ? hi : lo;
    } else return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x150 + k, 0xF, 0xF, true);  // row_newbcast
  }
  // (k a constant after unrolling: the dispatch folds away)
  XHE_DEV static uint32_t from_lane_i(uint32_t v, int k) {
    static_assert(TPI == 4 || TPI == 2 || TPI == 8 || TPI == 16, "");
    if constexpr (TPI == 2) return k == 0 ? from_lane<0>(v) : from_lane<1>(v);
    else if constexpr (TPI == 4)
      return k == 0 ? from_lane<0>(v) : k == 1 ? from_lane<1>(v) : k == 2 ? from_lane<2>(v) : from_lane<3>(v);
    else if constexpr (TPI == 8) {
      switch (k) {
        case 0: return from_lane<0>(v);
        case 1: return from_lane<1>(v);
        case 2: return from_lane<2>(v);
        case 3: return from_lane<3>(v);
        case 4: return from_lane<4>(v);
        case 5: return from_lane<5>(v);
        case 6: return from_lane<6>(v);
        default: return from_lane<7>(v);
      }
    } else {
      switch (k) {
        case 0: return from_lane<0>(v);
        case 1: return from_lane<1>(v);
        case 2: return from_lane<2>(v);
        case 3: return from_lane<3>(v);
        case 4: return from_lane<4>(v);
        case 5: return from_lane<5>(v);
        case 6: return from_lane<6>(v);
        case 7: return from_lane<7>(v);
        case 8: return from_lane<8>(v);
        case 9: return from_lane<9>(v);
        case 10: return from_lane<10>(v);
        case 11: return from_lane<11>(v);
        case 12: return from_lane<12>(v);
        case 13: return from_lane<13>(v);
        case 14: return from_lane<14>(v);
        default: return from_lane<15>(v);
      }
    }
  }

  // REDC with the quotient digits kept: T (lazy K-limb columns per lane) +
  // m n = R t. HI: a 2K-limb input whose limb K + gL + j is xh[j] of lane g,
  // entering at the group's last lane at step gL + j (else a K-limb input).
  // On return T holds t (lazy columns) and lane g holds digits gL..gL+L-1 of
  // m in mq.
  // b (masked limbs, < 2^(WK)) <- b - n if b >= n; returns whether it
  // subtracted (group-uniform). Mont::reduce_once with the flag kept.
  XHE_DEV bool csub(uint32_t (&b)[L]) const {
    uint32_t d[L];
    uint32_t br = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const int64_t x = (int64_t)b[j] - (int64_t)M.nl[j] - (int64_t)br;
      br = x < 0 ? 1u : 0u;
      d[j] = (uint32_t)(x + ((int64_t)br << W));
    }
    uint32_t total = br;
#pragma unroll
    for (int r = 1; r < TPI; ++r) {
      uint32_t bin = G::from_prev(br);
#pragma unroll
      for (int j = 0; j < L; ++j) {
        const int64_t x = (int64_t)d[j] - (int64_t)bin;
        bin = x < 0 ? 1u : 0u;
        d[j] = (uint32_t)(x + ((int64_t)bin << W));
      }
      br = bin;
      total |= bin;
    }
    br = G::bcast_last(total);
    if (!br) {
#pragma unroll
      for (int j = 0; j < L; ++j) b[j] = d[j];
    }
    return br == 0;
  }

  template <bool HI>
  XHE_DEV void redc_q(uint64_t (&T)[L], const uint32_t (&xh)[L], uint32_t (&mq)[L]) const {
    const int g = G::g();
    const bool top = last();
#pragma unroll
    for (int ib = 0; ib < TPI; ++ib) {
#pragma unroll
      for (int jj = 0; jj < L; ++jj) {
        const uint32_t m = G::bcast0(((uint32_t)T[0] * M.n0inv) & MASK);
        mq[jj] = g == ib ? m : mq[jj];
        const uint64_t v = mad64(m, M.nl[0], T[0]);
        mad_shift(T, M.nl, m);
        T[0] += v >> W;
        const uint32_t d = G::from_next((uint32_t)v & MASK);
        const uint32_t h = HI ? from_lane_i(xh[jj], ib) : 0u;
        T[L - 1] = top ? (uint64_t)h : (uint64_t)d;
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
};


// ---------------------------------------------------------------------------
// Building blocks of the PMDX kernels. Per element group: the operand pairs of
// its products in LDS (pair i at ops[i * ostride], ostride = groups per block),
// a table of digit states in global memory (pair i of entry t at
// tab[(t K + i) gs], gs = group slots of the grid, tab pre-offset by the
// group's slot).

// limbs [FIRST, FIRST + L) of a little-endian word array (W-bit limbs; zero
// beyond nwords): immediate shifts, every word loaded once
template <int W, int L, int FIRST>
XHE_DEV void limbs_at(uint32_t (&b)[L], const uint32_t* __restrict__ w, int nwords) {
#pragma unroll
  for (int j = 0; j < L; ++j) {
    const int bit = W * (FIRST + j), k = bit >> 5, sh = bit & 31;
    const uint32_t lo = word_or0(w, k, nwords);
    const uint32_t hi = sh + W > 32 ? word_or0(w, k + 1, nwords) : 0u;
    b[j] = (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) & ((1u << W) - 1u);
  }
}
// lane g's limbs [BASE + gL, BASE + (g+1) L) (lane index dispatched to
// compile-time copies, as Mont::load_words)
template <class D, int BASE, int GG = 0>
XHE_DEV void pmdx_load(uint32_t (&b)[D::L], const uint32_t* __restrict__ w, int nwords, int g) {
  if constexpr (GG == D::TPI - 1) {
    limbs_at<D::W, D::L, BASE + GG * D::L>(b, w, nwords);
  } else {
    if (g == GG) limbs_at<D::W, D::L, BASE + GG * D::L>(b, w, nwords);
    else pmdx_load<D, BASE, GG + 1>(b, w, nwords, g);
  }
}

// the per-lane table addresses are formed at each use (laundered base):
// hoisted out of the exponentiation loop they would hold 2 VGPRs per pair
// and the product's accumulators would spill (as opaque() in bn_dev.hpp)
template <class T>
XHE_DEV T* pmdx_launder(T* p) {
  int zero = 0;
  asm volatile("" : "+s"(zero));
  return p + zero;
}

template <class D>
XHE_DEV void pmdx_park(const uint32_t (&a)[D::L], const uint32_t (&c)[D::L], uint2* ops, int ostride) {
  const int g = D::G::g();
#pragma unroll
  for (int j = 0; j < D::L; ++j) ops[(g * D::L + j) * ostride] = make_uint2(a[j], c[j]);
}
template <class D>
XHE_DEV void pmdx_put(const uint32_t (&a)[D::L], const uint32_t (&c)[D::L], uint2* tab, int t, int gs) {
  const int g = D::G::g();
  uint2* p = pmdx_launder(tab) + ((size_t)t * D::K + g * D::L) * gs;
#pragma unroll
  for (int j = 0; j < D::L; ++j) p[(size_t)j * gs] = make_uint2(a[j], c[j]);
}
template <class D>
XHE_DEV void pmdx_get(uint32_t (&a)[D::L], uint32_t (&c)[D::L], const uint2* tab, int t, int gs) {
  const int g = D::G::g();
  const uint2* p = pmdx_launder(tab) + ((size_t)t * D::K + g * D::L) * gs;
#pragma unroll
  for (int j = 0; j < D::L; ++j) {
    const uint2 v = p[(size_t)j * gs];
    a[j] = v.x;
    c[j] = v.y;
  }
}
template <class D>
XHE_DEV void pmdx_tab_to_ops(const uint2* tab, int t, int gs, uint2* ops, int ostride) {
  const int g = D::G::g();
  const uint2* p = pmdx_launder(tab) + ((size_t)t * D::K + g * D::L) * gs;
  uint2 v[D::L];
#pragma unroll
  for (int j = 0; j < D::L; ++j) v[j] = p[(size_t)j * gs];
#pragma unroll
  for (int j = 0; j < D::L; ++j) ops[(g * D::L + j) * ostride] = v[j];
}
// digit states in HBM between kernels: pair i of element e at st[i count + e]
template <class D>
XHE_DEV void ndig_st_store(const uint32_t (&a)[D::L], const uint32_t (&c)[D::L], uint2* st, int64_t count, int64_t e) {
  const int g = D::G::g();
  uint2* p = pmdx_launder(st) + e;
#pragma unroll
  for (int j = 0; j < D::L; ++j) p[(size_t)(g * D::L + j) * count] = make_uint2(a[j], c[j]);
}
template <class D>
XHE_DEV void ndig_st_load(uint32_t (&a)[D::L], uint32_t (&c)[D::L], const uint2* st, int64_t count, int64_t e) {
  const int g = D::G::g();
  const uint2* p = pmdx_launder(st) + e;
#pragma unroll
  for (int j = 0; j < D::L; ++j) {
    const uint2 v = p[(size_t)(g * D::L + j) * count];
    a[j] = v.x;
    c[j] = v.y;
  }
}

// a packed digit row (e in words [0, hw), f in [hw, 2 hw), little-endian) into
// the group's operand pairs (each lane unpacks its own limbs)
template <class D>
XHE_DEV void pmdx_stage_row(const uint32_t* __restrict__ row, int hw, uint2* ops, int ostride) {
  const int g = D::G::g();
  uint32_t le[D::L], lf[D::L];
  pmdx_load<D, 0>(le, row, hw, g);
  pmdx_load<D, 0>(lf, row + hw, hw, g);
#pragma unroll
  for (int j = 0; j < D::L; ++j) ops[(g * D::L + j) * ostride] = make_uint2(le[j], lf[j]);
}

template <class D>
XHE_DEV void pmdx_row_to_tab(const uint2* __restrict__ row, uint2* tab, int t, int gs) {
  const int g = D::G::g();
  uint2* p = pmdx_launder(tab) + ((size_t)t * D::K + g * D::L) * gs;
#pragma unroll
  for (int j = 0; j < D::L; ++j) p[(size_t)j * gs] = row[g * D::L + j];
}

// plain x (2K limbs lo | hi, W-bit, < n^2) -> its digits (a, c):
//   X = x + ceil(R/n) n^2 (kn2, 2K limbs), REDC(X): X + m n = R t with t in
//   [n, 2n]; (t - n, R - m) are the digits of x R^-2 (R (t - n) + n (R - m) =
//   X - R n + n R ... = R t - n m = X = x mod n^2); one product by the digits
//   of R^2 mod n^2 (dw) gives x's. (tools/pdigit_model.py NDigits.to_digits)
template <class D>
XHE_DEV void pmdx_to_digits(const D& X, const uint32_t (&lo)[D::L], const uint32_t (&hi)[D::L],
                            const uint32_t* __restrict__ kn2, const uint32_t* __restrict__ rmn,
                            const uint2* __restrict__ dw, const uint32_t* topc, uint32_t (&a)[D::L],
                            uint32_t (&c)[D::L]) {
  constexpr int L = D::L, K = D::K;
  const int g = D::G::g();
  uint64_t T[L];
  uint32_t xh[L], mq[L];
#pragma unroll
  for (int j = 0; j < L; ++j) {
    T[j] = (uint64_t)lo[j] + kn2[g * L + j];
    xh[j] = hi[j] + kn2[K + g * L + j];
    mq[j] = 0;
  }
  X.template redc_q<true>(T, xh, mq);
  D::normalize_top(T, a);  // t
#pragma unroll
  for (int j = 0; j < L; ++j) T[j] = (uint64_t)a[j] + rmn[g * L + j];
  D::normalize_top(T, a);  // t - n + R
  if (D::last()) a[L - 1] &= D::MASK;
#pragma unroll
  for (int j = 0; j < L; ++j) T[j] = (uint64_t)(D::MASK - mq[j]) + ((g == 0 && j == 0) ? 1u : 0u);
  D::normalize_top(T, c);  // R - m
  X.template run<false>(a, c, OpRow{dw}, topc);
}

// digits (a, c) -> plain y = y0 + n y1 (y0, y1 in [0, n)):
//   y0 = REDC(a) - delta n (quotient m_a), u = REDC(c),
//   y1 = (REDC((u - m_a) + R n) + delta) mod n   (NDigits.from_digits)
template <class D>
XHE_DEV void pmdx_from_digits(const D& X, const uint32_t (&a)[D::L], const uint32_t (&c)[D::L],
                              uint32_t (&y0)[D::L], uint32_t (&y1)[D::L]) {
  constexpr int L = D::L;
  const int g = D::G::g();
  uint64_t T[L];
  uint32_t mqa[L], xh[L];
#pragma unroll
  for (int j = 0; j < L; ++j) {
    T[j] = a[j];
    mqa[j] = 0;
    xh[j] = 0;
  }
  X.template redc_q<false>(T, xh, mqa);
  D::normalize_top(T, y0);
  const bool delta = X.csub(y0);
#pragma unroll
  for (int j = 0; j < L; ++j) T[j] = c[j];
  X.template redc_q<false>(T, xh, y1);  // quotient not needed (y1 as scratch)
  D::normalize_top(T, y1);              // u < n + 2
  // s = u + (R - m_a); b = [s >= R] (u >= m_a); w = (s mod R) + R (n - 1 + b)
#pragma unroll
  for (int j = 0; j < L; ++j) T[j] = (uint64_t)y1[j] + (D::MASK - mqa[j]) + ((g == 0 && j == 0) ? 1u : 0u);
  D::normalize_top(T, y1);
  const uint32_t b = D::G::bcast_last(D::last() ? (y1[L - 1] >> D::W) : 0u);
  if (D::last()) y1[L - 1] &= D::MASK;
#pragma unroll
  for (int j = 0; j < L; ++j) {
    xh[j] = X.M.nl[j];
    T[j] = y1[j];
  }
  if (g == 0) xh[0] = xh[0] - 1u + b;
  X.template redc_q<true>(T, xh, mqa);
  D::normalize_top(T, y1);  // < 2n + 1
  if (delta && g == 0) {
#pragma unroll
    for (int j = 0; j < L; ++j) T[j] = y1[j] + (j == 0 ? 1u : 0u);
  } else {
#pragma unroll
    for (int j = 0; j < L; ++j) T[j] = y1[j];
  }
  D::normalize_top(T, y1);
  X.M.reduce_once(y1);
  X.M.reduce_once(y1);
}

// (a, c) <- (a, c)^E for an exponent shared by the wave (5-bit sliding
// window, odd powers in tab entries 0..15; pmd_pow_uniform's schedule)
template <class D>
XHE_DEV void pmdx_pow_uniform(const D& X, uint32_t (&a)[D::L], uint32_t (&c)[D::L], const uint32_t* ex, int ebits,
                              uint2* tab, int gs, uint2* ops, int ostride, const uint32_t* topc) {
  auto bit = [&](int i) { return (ex[i >> 5] >> (i & 31)) & 1u; };
  const OpLds op{ops, ostride};
  auto square = [&]() XHE_INL {
    pmdx_park<D>(a, c, ops, ostride);
    wave_sync_mem_();
    X.template run<true>(a, c, op, topc);
    wave_sync_mem_();
  };
  pmdx_put<D>(a, c, tab, 0, gs);
  square();  // x^2
  pmdx_park<D>(a, c, ops, ostride);
  wave_sync_mem_();
  pmdx_get<D>(a, c, tab, 0, gs);
#pragma unroll 1
  for (int t = 1; t < 16; ++t) {
    X.template run<false>(a, c, op, topc);  // x^(2t+1) = x^(2t-1) x^2
    pmdx_put<D>(a, c, tab, t, gs);
  }
  wave_sync_mem_();
  int i = ebits - 1;
  while (i >= 0 && !bit(i)) --i;
  int pend_sq = 0, pend_mul = -1;
  {
    int j = i - 4 < 0 ? 0 : i - 4;
    while (!bit(j)) ++j;
    uint32_t val = 0;
    for (int k = i; k >= j; --k) val = (val << 1) | bit(k);
    pmdx_get<D>(a, c, tab, (int)(val >> 1), gs);
    i = j - 1;
  }
#pragma unroll 1
  while (true) {
    if (pend_sq > 0) {
      square();
      --pend_sq;
    } else if (pend_mul >= 0) {
      pmdx_tab_to_ops<D>(tab, pend_mul, gs, ops, ostride);
      wave_sync_mem_();
      X.template run<false>(a, c, op, topc);
      wave_sync_mem_();
      pend_mul = -1;
    } else if (i < 0) {
      break;
    } else if (!bit(i)) {
      pend_sq = 1;
      --i;
    } else {
      int j = i - 4 < 0 ? 0 : i - 4;
      while (!bit(j)) ++j;
      uint32_t val = 0;
      for (int k = i; k >= j; --k) val = (val << 1) | bit(k);
      pend_sq = i - j + 1;
      pend_mul = (int)(val >> 1);
      i = j - 1;
    }
  }
}

// (a, c) <- (a, c)^k, k per element: 4-bit fixed windows (a uniform
// schedule), entries x^0 (the digits of 1, d1) .. x^15 in tab
template <class D, class DIGIT>
XHE_DEV void pmdx_pow_window4(const D& X, uint32_t (&a)[D::L], uint32_t (&c)[D::L], int nwin, const DIGIT& digit,
                              const uint2* __restrict__ d1, uint2* tab, int gs, uint2* ops, int ostride,
                              const uint32_t* topc) {
  const OpLds op{ops, ostride};
  pmdx_row_to_tab<D>(d1, tab, 0, gs);
  pmdx_put<D>(a, c, tab, 1, gs);
  pmdx_park<D>(a, c, ops, ostride);
  wave_sync_mem_();
#pragma unroll 1
  for (int t = 2; t < 16; ++t) {
    X.template run<false>(a, c, op, topc);  // x^t = x^(t-1) x
    pmdx_put<D>(a, c, tab, t, gs);
  }
  wave_sync_mem_();
  pmdx_get<D>(a, c, tab, (int)digit(nwin - 1), gs);
#pragma unroll 1
  for (int w = nwin - 2; w >= 0; --w) {
#pragma unroll 1
    for (int s = 0; s < 4; ++s) {
      pmdx_park<D>(a, c, ops, ostride);
      wave_sync_mem_();
      X.template run<true>(a, c, op, topc);
      wave_sync_mem_();
    }
    pmdx_tab_to_ops<D>(tab, (int)digit(w), gs, ops, ostride);
    wave_sync_mem_();
    X.template run<false>(a, c, op, topc);
    wave_sync_mem_();
  }
}

}  // namespace xhe
