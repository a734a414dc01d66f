// Arithmetic mod P^2 in base-P digits (DESIGN.md §4 "Next: arithmetic mod
// p^2 in base-p digits"; limb-level model and cost: tools/pdigit_model.py).
//
// x mod P^2 is held as two digits x = x0 + P x1, 0 <= x0, x1 < P, each K
// limbs of W = 28 bits (one limb per VGPR, one lane per residue):
//
//   (x0 + P x1)(y0 + P y1) = d0 + P ((d1 + x0 y1 + x1 y0) mod P)  (mod P^2)
//   with x0 y0 = d0 + P d1,
//
// three K x K products plus two Barrett reductions by P (HAC 14.42 in radix
// b = 2^28, the quotient from the product columns >= K-1 only, at most three
// corrections) instead of a Montgomery product on the 2K-limb modulus P^2.
// Products are column sums (product scanning) in NACC independent 64-bit
// partial sums; every column sum stays below 2^64 (at most 2K products of
// < 2^56 plus a carry: < 2^62.3 at K = 37).
//
// Development state: exercised by tests/native/pdigit_selftest.hip against
// host big integers and timed there against Mont<2K, 28, 1>::mul; not yet on
// a product path of the library.
#pragma once
#include "bn_dev.hpp"

namespace xhe {

template <int K_>
struct PDig {
  static constexpr int K = K_, W = 28, NACC = 4;
  static constexpr uint32_t MASK = (1u << W) - 1u;
  static_assert((double)(2 * K + 4) * (double)(1ull << (2 * W)) < 1.8e19, "column sums must stay below 2^64");

  const uint32_t* __restrict__ P;   // K limbs (wave-uniform)
  const uint32_t* __restrict__ MU;  // K + 1 limbs: floor(b^2K / P)

  // sum_{i in [lo, hi]} a[i] * b[c - i] + carry, NACC independent chains
  template <class FA, class FB>
  XHE_DEV static uint64_t column(int c, int lo, int hi, FA a, FB b, uint64_t carry) {
    uint64_t s[NACC] = {};
    s[0] = carry;
#pragma unroll
    for (int i = lo; i <= hi; ++i) s[(i - lo) % NACC] = a(i, b(c - i), s[(i - lo) % NACC]);
#pragma unroll
    for (int k = 1; k < NACC; ++k) s[0] += s[k];
    return s[0];
  }

  // T = a * b, 2K normalised limbs (a, b < P)
  XHE_DEV void mul_full(const uint32_t (&a)[K], const uint32_t (&b)[K], uint32_t (&T)[2 * K]) const {
    uint64_t carry = 0;
#pragma unroll
    for (int c = 0; c < 2 * K - 1; ++c) {
      const int lo = c - (K - 1) > 0 ? c - (K - 1) : 0, hi = c < K - 1 ? c : K - 1;
      const uint64_t s = column(c, lo, hi, [&](int i, uint32_t bv, uint64_t acc) { return mad64(a[i], bv, acc); },
                                [&](int j) { return b[j]; }, carry);
      T[c] = (uint32_t)s & MASK;
      carry = s >> W;
    }
    T[2 * K - 1] = (uint32_t)carry;
  }

  // T = a^2, 2K normalised limbs
  XHE_DEV void sqr_full(const uint32_t (&a)[K], uint32_t (&T)[2 * K]) const {
    uint64_t carry = 0;
#pragma unroll
    for (int c = 0; c < 2 * K - 1; ++c) {
      const int lo = c - (K - 1) > 0 ? c - (K - 1) : 0;
      uint64_t s[NACC] = {};
#pragma unroll
      for (int i = lo; 2 * i < c; ++i) s[(i - lo) % NACC] = mad64(a[i], a[c - i], s[(i - lo) % NACC]);
#pragma unroll
      for (int k = 1; k < NACC; ++k) s[0] += s[k];
      uint64_t x = (s[0] << 1) + carry;
      if ((c & 1) == 0) x = mad64(a[c / 2], a[c / 2], x);
      T[c] = (uint32_t)x & MASK;
      carry = x >> W;
    }
    T[2 * K - 1] = (uint32_t)carry;
  }

  // U = s * (a*b + c*d) + e, 2K normalised limbs (s = 1 or 2; e < P)
  XHE_DEV void cross(const uint32_t (&a)[K], const uint32_t (&b)[K], const uint32_t (&c_)[K], const uint32_t (&d)[K],
                     int twice, const uint32_t (&e)[K], uint32_t (&U)[2 * K]) const {
    uint64_t carry = 0;
#pragma unroll
    for (int c = 0; c < 2 * K - 1; ++c) {
      const int lo = c - (K - 1) > 0 ? c - (K - 1) : 0, hi = c < K - 1 ? c : K - 1;
      uint64_t s[NACC] = {};
#pragma unroll
      for (int i = lo; i <= hi; ++i) {
        s[(i - lo) % NACC] = mad64(a[i], b[c - i], s[(i - lo) % NACC]);
        if (!twice) s[(i - lo + 2) % NACC] = mad64(c_[i], d[c - i], s[(i - lo + 2) % NACC]);
      }
#pragma unroll
      for (int k = 1; k < NACC; ++k) s[0] += s[k];
      uint64_t x = (twice ? (s[0] << 1) : s[0]) + carry + (c < K ? (uint64_t)e[c] : 0ull);
      U[c] = (uint32_t)x & MASK;
      carry = x >> W;
    }
    U[2 * K - 1] = (uint32_t)carry;
  }

  // r = T mod P (K limbs), and with WANT_Q q = floor(T / P) (K limbs), for
  // T < min(b^2K, P * b^K) given as 2K normalised limbs.
  template <bool WANT_Q>
  XHE_DEV void barrett(const uint32_t (&T)[2 * K], uint32_t (&r)[K], uint32_t (&q)[K]) const {
    // q3 = floor(q1 * MU / b^(K+1)), q1 = T[K-1 .. 2K): the product's columns
    // >= K-1 only (the skipped ones would add at most one to q3)
    uint32_t q3[K + 1];
    uint64_t carry = 0;
#pragma unroll
    for (int c = K - 1; c <= 2 * K; ++c) {
      const int lo = c - K > 0 ? c - K : 0, hi = c < K ? c : K;
      uint64_t s[NACC] = {};
      s[0] = carry;
#pragma unroll
      for (int i = lo; i <= hi; ++i) s[(i - lo) % NACC] = mad64s(T[K - 1 + i], MU[c - i], s[(i - lo) % NACC]);
#pragma unroll
      for (int k = 1; k < NACC; ++k) s[0] += s[k];
      if (c >= K + 1) q3[c - (K + 1)] = (uint32_t)s[0] & MASK;
      carry = s[0] >> W;
    }
    q3[K] = (uint32_t)carry;
    // r = (T - q3 P) mod b^(K+1): the low K+1 columns of q3 * P
    uint32_t rr[K + 1];
    carry = 0;
    int64_t borrow = 0;
#pragma unroll
    for (int c = 0; c <= K; ++c) {
      const int hi = c < K - 1 ? c : K - 1;
      uint64_t s[NACC] = {};
      s[0] = carry;
#pragma unroll
      for (int j = 0; j <= hi; ++j) s[j % NACC] = mad64s(q3[c - j], P[j], s[j % NACC]);
#pragma unroll
      for (int k = 1; k < NACC; ++k) s[0] += s[k];
      carry = s[0] >> W;
      const int64_t v = (int64_t)T[c] - (int64_t)((uint32_t)s[0] & MASK) + borrow;
      rr[c] = (uint32_t)v & MASK;
      borrow = v >> W;  // arithmetic shift: 0 or -1
    }
    // at most three subtractions of P (branch-free: keep r - P when it did not borrow)
    uint32_t fix = 0;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      uint32_t d[K + 1];
      int64_t b = 0;
#pragma unroll
      for (int i = 0; i <= K; ++i) {
        const int64_t v = (int64_t)rr[i] - (int64_t)(i < K ? P[i] : 0u) + b;
        d[i] = (uint32_t)v & MASK;
        b = v >> W;
      }
      const bool ge = b == 0;
      fix += ge ? 1u : 0u;
#pragma unroll
      for (int i = 0; i <= K; ++i) rr[i] = ge ? d[i] : rr[i];
    }
#pragma unroll
    for (int i = 0; i < K; ++i) r[i] = rr[i];
    if constexpr (WANT_Q) {
      uint32_t c2 = fix;
#pragma unroll
      for (int i = 0; i < K; ++i) {
        const uint32_t v = q3[i] + c2;
        q[i] = v & MASK;
        c2 = v >> W;
      }
    }
  }

  // (x0, x1) <- (x0, x1) * (y0, y1) mod P^2
  XHE_DEV void mul(uint32_t (&x0)[K], uint32_t (&x1)[K], const uint32_t (&y0)[K], const uint32_t (&y1)[K]) const {
    uint32_t U[2 * K], T[2 * K], d1[K], z[K];
    const uint32_t zero[K] = {};
    cross(x0, y1, x1, y0, 0, zero, U);  // x0 y1 + x1 y0 (d1 added below)
    mul_full(x0, y0, T);
    barrett<true>(T, x0, d1);            // x0 <- d0
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 2 * K; ++i) {    // U += d1
      const uint32_t v = U[i] + (i < K ? d1[i] : 0u) + c;
      U[i] = v & MASK;
      c = v >> W;
    }
    barrett<false>(U, x1, z);
  }

  // (x0, x1) <- (x0, x1)^2 mod P^2
  XHE_DEV void sqr(uint32_t (&x0)[K], uint32_t (&x1)[K]) const {
    uint32_t U[2 * K], T[2 * K], d1[K], z[K];
    sqr_full(x0, T);
    uint32_t d0[K];
    barrett<true>(T, d0, d1);
    cross(x0, x1, x0, x1, 1, d1, U);     // 2 x0 x1 + d1
#pragma unroll
    for (int i = 0; i < K; ++i) x0[i] = d0[i];
    barrett<false>(U, x1, z);
  }
};

}  // namespace xhe
