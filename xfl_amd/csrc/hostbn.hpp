// Host-side multi-precision integers for key setup (runs once per key).
//
// Derives the per-key constants of PaillierContext.init
// (reference python/common/crypto/paillier/context.py:28-71) and the
// Montgomery constants the device kernels need. Not on the per-element path.
#pragma once
#include <atomic>
#include <stdint.h>

#include <algorithm>
#include <stdexcept>
#include <vector>

namespace xhe {

struct BigU {
  std::vector<uint32_t> w;  // little-endian 32-bit words, no leading zeros

  BigU() = default;
  explicit BigU(uint64_t v) {
    if (v) w.push_back((uint32_t)v);
    if (v >> 32) w.push_back((uint32_t)(v >> 32));
  }
  static BigU from_words(const uint32_t* p, size_t n) {
    BigU r;
    r.w.assign(p, p + n);
    r.trim();
    return r;
  }
  void trim() {
    while (!w.empty() && w.back() == 0) w.pop_back();
  }
  bool is_zero() const { return w.empty(); }
  size_t bits() const {
    if (w.empty()) return 0;
    return 32 * (w.size() - 1) + (32 - __builtin_clz(w.back()));
  }
  uint32_t word(size_t i) const { return i < w.size() ? w[i] : 0u; }
  int bit(size_t i) const { return (int)((word(i >> 5) >> (i & 31)) & 1u); }
  void to_words(uint32_t* out, size_t n) const {
    if (w.size() > n) throw std::runtime_error("BigU::to_words: value too large");
    for (size_t i = 0; i < n; ++i) out[i] = word(i);
  }
  // W-bit limbs, S of them (value must fit)
  std::vector<uint32_t> to_limbs(int W, int S) const {
    if ((int)bits() > W * S) throw std::runtime_error("BigU::to_limbs: value too large");
    std::vector<uint32_t> r(S);
    uint64_t mask = (1ull << W) - 1;
    for (int j = 0; j < S; ++j) {
      size_t bitpos = (size_t)W * j;
      size_t k = bitpos >> 5, sh = bitpos & 31;
      uint64_t v = (uint64_t)word(k) | ((uint64_t)word(k + 1) << 32);
      r[j] = (uint32_t)((v >> sh) & mask);
    }
    return r;
  }
};

inline int cmp(const BigU& a, const BigU& b) {
  if (a.w.size() != b.w.size()) return a.w.size() < b.w.size() ? -1 : 1;
  for (size_t i = a.w.size(); i-- > 0;)
    if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
  return 0;
}

inline BigU add(const BigU& a, const BigU& b) {
  BigU r;
  size_t n = std::max(a.w.size(), b.w.size());
  r.w.resize(n + 1);
  uint64_t c = 0;
  for (size_t i = 0; i < n; ++i) {
    c += (uint64_t)a.word(i) + b.word(i);
    r.w[i] = (uint32_t)c;
    c >>= 32;
  }
  r.w[n] = (uint32_t)c;
  r.trim();
  return r;
}

// a - b, requires a >= b
inline BigU sub(const BigU& a, const BigU& b) {
  if (cmp(a, b) < 0) throw std::runtime_error("BigU::sub: negative result");
  BigU r;
  r.w.resize(a.w.size());
  int64_t br = 0;
  for (size_t i = 0; i < a.w.size(); ++i) {
    int64_t d = (int64_t)a.w[i] - (int64_t)b.word(i) - br;
    br = d < 0;
    r.w[i] = (uint32_t)(d + (br << 32));
  }
  r.trim();
  return r;
}

inline BigU mul(const BigU& a, const BigU& b) {
  BigU r;
  if (a.is_zero() || b.is_zero()) return r;
  r.w.assign(a.w.size() + b.w.size(), 0);
  for (size_t i = 0; i < a.w.size(); ++i) {
    uint64_t c = 0;
    for (size_t j = 0; j < b.w.size(); ++j) {
      c += (uint64_t)a.w[i] * b.w[j] + r.w[i + j];
      r.w[i + j] = (uint32_t)c;
      c >>= 32;
    }
    r.w[i + b.w.size()] = (uint32_t)c;
  }
  r.trim();
  return r;
}

inline BigU shl(const BigU& a, size_t s) {
  BigU r;
  if (a.is_zero()) return r;
  size_t ws = s >> 5, bs = s & 31;
  r.w.assign(a.w.size() + ws + 1, 0);
  for (size_t i = 0; i < a.w.size(); ++i) {
    uint64_t v = (uint64_t)a.w[i] << bs;
    r.w[i + ws] |= (uint32_t)v;
    r.w[i + ws + 1] |= (uint32_t)(v >> 32);
  }
  r.trim();
  return r;
}

inline BigU pow2(size_t s) { return shl(BigU(1), s); }

// q = a / m, r = a % m (binary long division over the quotient bits only)
inline void divmod(const BigU& a, const BigU& m, BigU* q, BigU* r) {
  if (m.is_zero()) throw std::runtime_error("BigU::divmod: division by zero");
  size_t ab = a.bits(), mb = m.bits();
  BigU quo, rem;
  if (ab < mb) {
    if (q) *q = quo;
    if (r) *r = a;
    return;
  }
  size_t s = ab - mb;
  // rem = a >> s
  rem.w.assign(((ab - s) + 31) / 32 + 1, 0);
  for (size_t i = 0; i < ab - s; ++i)
    if (a.bit(i + s)) rem.w[i >> 5] |= 1u << (i & 31);
  rem.trim();
  quo.w.assign(s / 32 + 1, 0);
  for (size_t k = s + 1; k-- > 0;) {
    if (k != s) {
      rem = shl(rem, 1);
      if (a.bit(k)) {
        if (rem.w.empty()) rem.w.push_back(0);
        rem.w[0] |= 1u;
      }
    }
    if (cmp(rem, m) >= 0) {
      rem = sub(rem, m);
      quo.w[k >> 5] |= 1u << (k & 31);
    }
  }
  quo.trim();
  if (q) *q = quo;
  if (r) *r = rem;
}

inline BigU mod(const BigU& a, const BigU& m) {
  BigU r;
  divmod(a, m, nullptr, &r);
  return r;
}

inline BigU mulmod(const BigU& a, const BigU& b, const BigU& m) { return mod(mul(a, b), m); }

// (a - b) mod m for a, b < m
inline BigU submod(const BigU& a, const BigU& b, const BigU& m) {
  if (cmp(a, b) >= 0) return sub(a, b);
  return sub(add(a, m), b);
}

// a^-1 mod m (extended Euclid); throws if not invertible (utils.py:71-76)
inline BigU modinv(const BigU& a, const BigU& m) {
  BigU r0 = m, r1 = mod(a, m), t0(0), t1(1);
  while (!r1.is_zero()) {
    BigU qq, rr;
    divmod(r0, r1, &qq, &rr);
    BigU t2 = submod(t0, mulmod(qq, t1, m), m);
    r0 = r1;
    r1 = rr;
    t0 = t1;
    t1 = t2;
  }
  if (!(r0.w.size() == 1 && r0.w[0] == 1)) throw std::runtime_error("modinv: no inverse exists");
  return t0;
}

// x^-1 mod m for odd m and 0 <= x < m (binary extended Euclid on 64-bit
// words, O(bits^2 / 64) word operations: ~1 ms at 4096 bits); returns false
// when gcd(x, m) != 1. Used for the one inverse per batch at the root of the
// device product tree (batch inversion, utils.py:71-76 semantics).
inline bool modinv_words_binary(const uint32_t* x32, const uint32_t* m32, int nw32, uint32_t* out32) {
  const int W = (nw32 + 1) / 2 + 1;  // one spare word for (a + m) before halving
  std::vector<uint64_t> u(W, 0), v(W, 0), x1(W, 0), x2(W, 0), m(W, 0);
  for (int i = 0; i < nw32; ++i) {
    u[i / 2] |= (uint64_t)x32[i] << (32 * (i & 1));
    m[i / 2] |= (uint64_t)m32[i] << (32 * (i & 1));
  }
  v = m;
  x1[0] = 1;
  auto is_one = [&](const std::vector<uint64_t>& a) {
    if (a[0] != 1) return false;
    for (int i = 1; i < W; ++i)
      if (a[i]) return false;
    return true;
  };
  auto is_zero = [&](const std::vector<uint64_t>& a) {
    for (int i = 0; i < W; ++i)
      if (a[i]) return false;
    return true;
  };
  auto half = [&](std::vector<uint64_t>& a) {
    for (int i = 0; i < W; ++i) a[i] = (a[i] >> 1) | (i + 1 < W ? a[i + 1] << 63 : 0);
  };
  auto add_to = [&](std::vector<uint64_t>& a, const std::vector<uint64_t>& b) {
    unsigned __int128 c = 0;
    for (int i = 0; i < W; ++i) {
      c += (unsigned __int128)a[i] + b[i];
      a[i] = (uint64_t)c;
      c >>= 64;
    }
  };
  auto sub_to = [&](std::vector<uint64_t>& a, const std::vector<uint64_t>& b) {  // a >= b
    uint64_t br = 0;
    for (int i = 0; i < W; ++i) {
      unsigned __int128 d = (unsigned __int128)a[i] - b[i] - br;
      a[i] = (uint64_t)d;
      br = (uint64_t)(d >> 64) & 1;
    }
  };
  auto geq = [&](const std::vector<uint64_t>& a, const std::vector<uint64_t>& b) {
    for (int i = W - 1; i >= 0; --i)
      if (a[i] != b[i]) return a[i] > b[i];
    return true;
  };
  auto halve_mod = [&](std::vector<uint64_t>& a) {  // a / 2 mod m
    if (a[0] & 1) add_to(a, m);
    half(a);
  };
  auto submod_to = [&](std::vector<uint64_t>& a, const std::vector<uint64_t>& b) {  // a = (a - b) mod m
    if (!geq(a, b)) add_to(a, m);
    sub_to(a, b);
  };
  if (is_zero(u)) return false;
  while (!is_one(u) && !is_one(v)) {
    while ((u[0] & 1) == 0) {
      half(u);
      halve_mod(x1);
    }
    while ((v[0] & 1) == 0) {
      half(v);
      halve_mod(x2);
    }
    if (geq(u, v)) {
      sub_to(u, v);
      submod_to(x1, x2);
    } else {
      sub_to(v, u);
      submod_to(x2, x1);
    }
    if (is_zero(u) || is_zero(v)) return false;
  }
  const std::vector<uint64_t>& r = is_one(u) ? x1 : x2;
  for (int i = 0; i < nw32; ++i) out32[i] = (uint32_t)(r[i / 2] >> (32 * (i & 1)));
  return true;
}

// x^-1 mod m for odd m, x < m: the binary extended GCD with the iterations
// batched KB = 62 at a time (the approach of T. Pornin, "Optimized Binary GCD for
// Modular Inversion", 2020). A batch runs on 126-bit approximations of a and b
// (their low KB bits, exact, and their top KB + 2 bits at a common position):
// the parity tests are exact, the comparisons approximate; the batch's 2x2
// update matrix (entries <= 2^KB) is then applied once to the full-width a, b
// and to the Bezout cofactors u, v mod m (each divided by 2^KB with one
// Montgomery step), and a row that came out negative is negated. About 2 len(m) / KB
// batches of a few linear passes, instead of ~2 len(m) full-width shift /
// subtract passes. Returns false when gcd(x, m) != 1; falls back to the plain
// binary algorithm if the batch budget runs out (never observed).
// how often modinv_words ran out of its batch budget and took the binary
// algorithm (a test hook: the batched path is expected to always converge).
// Atomic: inversions run on several host threads at once (one per device or
// stream); the count is per process (never reset).
inline std::atomic<int>& modinv_fallbacks() {
  static std::atomic<int> n{0};
  return n;
}

inline bool modinv_words(const uint32_t* x32, const uint32_t* m32, int nw32, uint32_t* out32) {
  if (nw32 <= 0 || !(m32[0] & 1)) return modinv_words_binary(x32, m32, nw32, out32);
  const int W = (nw32 + 1) / 2 + 1;
  using u64 = uint64_t;
  using i128 = __int128;
  std::vector<u64> a(W, 0), b(W, 0), u(W, 0), v(W, 0), m(W, 0), t(W + 1, 0);
  for (int i = 0; i < nw32; ++i) {
    a[i / 2] |= (u64)x32[i] << (32 * (i & 1));
    m[i / 2] |= (u64)m32[i] << (32 * (i & 1));
  }
  b = m;
  u[0] = 1;
  auto bitlen = [&](const std::vector<u64>& x) {
    for (int i = W - 1; i >= 0; --i)
      if (x[i]) return 64 * i + 64 - __builtin_clzll(x[i]);
    return 0;
  };
  auto is_zero = [&](const std::vector<u64>& x) {
    for (int i = 0; i < W; ++i)
      if (x[i]) return false;
    return true;
  };
  auto geq = [&](const std::vector<u64>& x, const std::vector<u64>& y) {
    for (int i = W - 1; i >= 0; --i)
      if (x[i] != y[i]) return x[i] > y[i];
    return true;
  };
  if (!geq(m, a) || (geq(a, m) && geq(m, a))) return modinv_words_binary(x32, m32, nw32, out32);  // x >= m
  auto bits_at = [&](const std::vector<u64>& x, int pos) -> u64 {  // 64 bits of x from bit pos
    int w = pos >> 6, sh = pos & 63;
    u64 lo = w < W ? x[w] : 0, hi = w + 1 < W ? x[w + 1] : 0;
    return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
  };
  // KB = 62 steps per batch (round 4; was 31): 126-bit approximations (the
  // low 62 bits exact, the top 64 at a common position) in unsigned
  // __int128, update factors |f| + |g| <= 2^62 in int64, so the linear passes
  // below (f x + g y, |.| < 2^126 per word) stay inside __int128: half the
  // batches of the same passes (4096-bit root inverse 172 -> ~90 us here).
  constexpr int KB = 62;
  using u128 = unsigned __int128;
  const u64 MK = (1ull << KB) - 1;
  // r = (f x + g y) / 2^KB, exact; returns true when negative (r then holds
  // the magnitude)
  auto lin_shift = [&](int64_t f, const std::vector<u64>& x, int64_t g, const std::vector<u64>& y,
                       std::vector<u64>& r) {
    i128 c = 0;
    for (int i = 0; i < W; ++i) {
      c += (i128)f * (i128)x[i] + (i128)g * (i128)y[i];
      t[i] = (u64)c;
      c >>= 64;
    }
    t[W] = (u64)(int64_t)c;
    bool neg = (int64_t)t[W] < 0;
    if (neg) {  // two's complement negate over W+1 words
      unsigned carry = 1;
      for (int i = 0; i <= W; ++i) {
        u64 nv = ~t[i] + carry;
        carry = (carry && nv == 0) ? 1 : 0;
        t[i] = nv;
      }
    }
    for (int i = 0; i < W; ++i) r[i] = (t[i] >> KB) | (t[i + 1] << (64 - KB));
    return neg;
  };
  // -m^-1 mod 2^64 (Newton)
  u64 minv = 1;
  for (int i = 0; i < 6; ++i) minv *= 2 - m[0] * minv;
  const u64 mneg_inv = (u64)0 - minv;
  // r = (f x + g y) 2^-KB mod m, x, y in [0, m)
  auto lin_mod = [&](int64_t f, const std::vector<u64>& x, int64_t g, const std::vector<u64>& y,
                     std::vector<u64>& r) {
    i128 c = 0;
    for (int i = 0; i < W; ++i) {
      c += (i128)f * (i128)x[i] + (i128)g * (i128)y[i];
      t[i] = (u64)c;
      c >>= 64;
    }
    t[W] = (u64)(int64_t)c;
    const u64 q = (t[0] * mneg_inv) & MK;  // t + q m = 0 (mod 2^KB)
    unsigned __int128 cc = 0;
    i128 sc = 0;
    for (int i = 0; i < W; ++i) {
      cc += (unsigned __int128)t[i] + (unsigned __int128)q * m[i];
      t[i] = (u64)cc;
      cc >>= 64;
    }
    sc = (i128)(int64_t)t[W] + (i128)(u64)cc;
    t[W] = (u64)sc;
    // shift right KB (arithmetic), value in (-3m, 3m)
    for (int i = 0; i < W; ++i) r[i] = (t[i] >> KB) | (t[i + 1] << (64 - KB));
    int64_t top = (int64_t)t[W] >> KB;  // sign word of the shifted value (0 or -1)
    // bring into [0, m)
    for (int it = 0; it < 4 && top < 0; ++it) {  // add m
      unsigned __int128 k2 = 0;
      for (int i = 0; i < W; ++i) {
        k2 += (unsigned __int128)r[i] + m[i];
        r[i] = (u64)k2;
        k2 >>= 64;
      }
      top += (int64_t)k2;
    }
    while (geq(r, m)) {
      u64 br = 0;
      for (int i = 0; i < W; ++i) {
        unsigned __int128 d = (unsigned __int128)r[i] - m[i] - br;
        r[i] = (u64)d;
        br = (u64)(d >> 64) & 1;
      }
    }
  };
  std::vector<u64> na(W), nb(W), nu(W), nv(W);
  const int max_batches = (2 * 64 * W) / KB + 16;
  for (int batch = 0; batch < max_batches; ++batch) {
    if (is_zero(a)) {
      // b = gcd(x, m)
      if (b[0] != 1) return false;
      for (int i = 1; i < W; ++i)
        if (b[i]) return false;
      for (int i = 0; i < nw32; ++i) out32[i] = (uint32_t)(v[i / 2] >> (32 * (i & 1)));
      return true;
    }
    // the top 64 bits at a common position above the exact low KB bits; when
    // both fit in 128 bits the u128 holds them whole (the exact binary steps)
    const int n = std::max(bitlen(a), bitlen(b));
    u128 xa, xb;
    if (n <= 128) {  // exact
      xa = (u128)a[0] | ((u128)(W > 1 ? a[1] : 0) << 64);
      xb = (u128)b[0] | ((u128)(W > 1 ? b[1] : 0) << 64);
    } else {
      xa = ((u128)bits_at(a, n - 64) << KB) | (a[0] & MK);
      xb = ((u128)bits_at(b, n - 64) << KB) | (b[0] & MK);
    }
    int64_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
    for (int j = 0; j < KB; ++j) {
      if ((uint64_t)xa & 1) {
        if (xa < xb) {
          std::swap(xa, xb);
          std::swap(f0, f1);
          std::swap(g0, g1);
        }
        xa -= xb;
        f0 -= f1;
        g0 -= g1;
      }
      xa >>= 1;
      f1 *= 2;  // |f1|, |g1| <= 2^62: no overflow (a shift of a negative value would be UB)
      g1 *= 2;
    }
    if (lin_shift(f0, a, g0, b, na)) {
      f0 = -f0;
      g0 = -g0;
    }
    if (lin_shift(f1, a, g1, b, nb)) {
      f1 = -f1;
      g1 = -g1;
    }
    lin_mod(f0, u, g0, v, nu);
    lin_mod(f1, u, g1, v, nv);
    a.swap(na);
    b.swap(nb);
    u.swap(nu);
    v.swap(nv);
  }
  modinv_fallbacks().fetch_add(1, std::memory_order_relaxed);  // never observed; tests/test_host_modinv.py asserts it stays 0
  return modinv_words_binary(x32, m32, nw32, out32);
}

// a^e mod m, plain square-and-multiply (key setup only)
inline BigU powmod(const BigU& a, const BigU& e, const BigU& m) {
  BigU r = mod(BigU(1), m), b = mod(a, m);
  for (size_t i = e.bits(); i-- > 0;) {
    r = mulmod(r, r, m);
    if (e.bit(i)) r = mulmod(r, b, m);
  }
  return r;
}

// -m^-1 mod 2^W for odd m (Newton iteration on the low word)
inline uint32_t mont_ninv(uint32_t m0, int W) {
  uint32_t x = 1;
  for (int i = 0; i < 5; ++i) x *= 2u - m0 * x;  // x = m0^-1 mod 2^32
  uint32_t r = (uint32_t)(0u - x);
  return W == 32 ? r : (r & ((1u << W) - 1));
}

}  // namespace xhe
