// xhe: C-ABI over the gfx950 Paillier kernels (see include/xhe.h).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <memory>
#include <mutex>
#include <atomic>
#include <stdexcept>
#include <unordered_map>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/xhe.h"
#include "abi_common.hpp"
#include "hostbn.hpp"
#include "xhe_kernels.hpp"
#include "dec_wave.hpp"
#include "barrett_dev.hpp"
#include "rns_dev.hpp"

using namespace xhe;

namespace {

int fail(int code, const std::string& msg) { return xhe_fail(code, msg); }

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t _e = (x);                                                                   \
    if (_e != hipSuccess) throw HipError(std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

// ------------------------------------------------------------------ shapes
// Limb shapes per key size: MP2 for residues mod p^2/q^2, MP for mod p/q.
struct Shape2048 {
  static constexpr int K = 2048, RW = K / 32, RW2 = K / 16;  // packed table row words mod p^2 / n^2
  using MP2 = Mont<74, 28, 1>;
  using MP2L = Mont<76, 28, 4>;   // low-latency (small-batch) decrypt shape
  using MP2X = Mont<80, 28, 16>;  // lowest latency: one 16-lane DPP row per residue (tiny batches)
  using MP = Mont<37, 28, 1>;
  using MN2 = Mont<152, 27, 4>;
  using MN2X = Mont<160, 27, 16>;  // n^2 ops on small batches: one 16-lane DPP row per residue
};
struct Shape3072 {
  static constexpr int K = 3072, RW = K / 32, RW2 = K / 16;  // packed table row words mod p^2 / n^2
  using MP2 = Mont<110, 28, 2>;
  using MP2L = Mont<112, 28, 4>;
  using MP2X = Mont<112, 28, 16>;
  using MP = Mont<56, 28, 2>;
  using MN2 = Mont<228, 27, 4>;
  using MN2X = Mont<240, 27, 16>;
  using PDX = PMDX<60, 2>;   // Montgomery digits mod p^2, q^2: k_djn_pmdx's products (2 lanes of 30 limbs)
  using PDXO = PMDX<60, 4>;  // its conversions (k_pmdx_enc_out, k_tab_to_pmdx; 2 lanes would spill there)
  using PDXP = PMDX<60, 4>;  // the decrypt exponentiation (2 lanes spill 70 VGPRs in pmdx_pow_uniform)
};
// 4096-bit keys (the LR/LinReg/Pearson/WoE operators' OneOf(2048, 4096, 8192)):
// 28-bit limbs would overflow the lazy 64-bit accumulator at S = 147
// ((2S+2) 2^56 >= 2^64), so every modulus uses 27-bit limbs. p^2 residues
// take 4 lanes (38 limbs each), n^2 residues one 16-lane DPP row (19 each)
// in both the batch and the small-batch shapes; the mod-p limbs share W with
// p^2 so k_dec_fin reads k_dec_pow's rows unchanged.
struct Shape4096 {
  static constexpr int K = 4096, RW = K / 32, RW2 = K / 16;  // packed table row words mod p^2 / n^2
  using MP2 = Mont<152, 27, 4>;
  using MP2L = Mont<152, 27, 4>;
  using MP2X = Mont<160, 27, 16>;
  using MP = Mont<76, 27, 4>;
  using MN2 = Mont<304, 27, 16>;
  using MN2X = Mont<304, 27, 16>;
  using PDX = PMDX<80, 4>;
  using PDXO = PMDX<80, 4>;
  using PDXP = PMDX<80, 4>;
};

// 8192-bit keys: p^2 (8192 bits) in one 16-lane row of 27-bit limbs, p in 4
// lanes; n^2 (16384 bits) needs 26-bit limbs for the lazy accumulator
// ((2S+2) 2^52 < 2^64 at S = 640), 40 per lane of a 16-lane row.
struct Shape8192 {
  static constexpr int K = 8192, RW = K / 32, RW2 = K / 16;  // packed table row words mod p^2 / n^2
  using MP2 = Mont<304, 27, 16>;
  using MP2L = Mont<304, 27, 16>;
  using MP2X = Mont<304, 27, 16>;
  using MP = Mont<152, 27, 4>;
  using MN2 = Mont<640, 26, 16>;
  using MN2X = Mont<640, 26, 16>;
  // Montgomery digits mod p^2, q^2 (4096-bit primes: 160 limbs of 27 bits,
  // R = 2^4320): the products (encrypt and decrypt exponentiations) on half
  // rows, 8 lanes of 20 limbs (no spills: 170 / 230 VGPRs); the conversions
  // on whole 16-lane rows (8 lanes spill 44 VGPRs in k_pmdx_enc_out)
  using PDX = PMDX<160, 8>;
  using PDXO = PMDX<160, 16>;
  using PDXP = PMDX<160, 8>;
};

// XHE_ONLY_BITS=K (XHE_ONLY_2048 = 2048): a development build with one key
// size's shapes only (a fraction of the compile time, for kernel A/B runs
// through $XHE_LIB); the shipped library has every key size.
#if defined(XHE_ONLY_2048) && !defined(XHE_ONLY_BITS)
#define XHE_ONLY_BITS 2048
#endif
#ifdef XHE_ONLY_BITS
constexpr bool key_bits_supported(int K) { return K == XHE_ONLY_BITS; }
template <class F>
decltype(auto) with_shape(int, F&& f) {
  if constexpr (XHE_ONLY_BITS == 2048) return f(Shape2048{});
  else if constexpr (XHE_ONLY_BITS == 3072) return f(Shape3072{});
  else if constexpr (XHE_ONLY_BITS == 4096) return f(Shape4096{});
  else return f(Shape8192{});
}
#else
constexpr bool key_bits_supported(int K) { return K == 2048 || K == 3072 || K == 4096 || K == 8192; }

// Calls f(ShapeK{}) for the key size K (checked at xhe_key_create).
template <class F>
decltype(auto) with_shape(int K, F&& f) {
  if (K == 2048) return f(Shape2048{});
  if (K == 3072) return f(Shape3072{});
  if (K == 4096) return f(Shape4096{});
  return f(Shape8192{});
}
#endif

#if XHE_NDIG
// $XHE_NDIG_PUB=0: public DJN keys keep Montgomery n^2 tables (k_djn_pub; A/B)
bool ndig_pub_on() {
  static const bool on = [] {
    const char* e = getenv("XHE_NDIG_PUB");
    return !(e && e[0] == '0');
  }();
  return on;
}
#endif

struct ModSpec {
  int S, W;
  int S4() const { return (S + 3) & ~3; }
};

// ------------------------------------------------------------------ blob
struct Blob {
  std::vector<uint32_t> h;
  size_t put(const std::vector<uint32_t>& v, size_t min_words = 0) {
    size_t off = h.size();
    size_t len = std::max(v.size(), min_words);
    len = (len + 3) & ~(size_t)3;
    h.resize(off + len, 0u);
    std::copy(v.begin(), v.end(), h.begin() + off);
    return off;
  }
  size_t put_limbs(const BigU& x, const ModSpec& s) { return put(x.to_limbs(s.W, s.S), s.S4()); }
  size_t put_words(const BigU& x, int nw) {
    std::vector<uint32_t> v(nw);
    x.to_words(v.data(), nw);
    return put(v);
  }
};

// ---- RNS small-batch decrypt constants (rns_dev.hpp k_dec_rns; checked
// against tools/rns_model.py, which builds the same bases)
namespace rnsh {
inline bool prime32(uint32_t n) {  // deterministic Miller-Rabin for n < 2^32
  if (n < 2) return false;
  for (uint32_t p : {2u, 3u, 5u, 7u})
    if (n % p == 0) return n == p;
  uint32_t d = n - 1;
  int r = 0;
  while (!(d & 1)) d >>= 1, ++r;
  for (uint64_t a : {2ull, 3ull, 5ull, 7ull}) {
    uint64_t x = 1, b = a, e = d;
    while (e) {
      if (e & 1) x = x * b % n;
      b = b * b % n;
      e >>= 1;
    }
    if (x == 1 || x == n - 1) continue;
    bool ok = false;
    for (int i = 1; i < r && !ok; ++i) {
      x = x * x % n;
      ok = x == n - 1;
    }
    if (!ok) return false;
  }
  return true;
}
inline uint32_t inv_mod(uint32_t a, uint32_t m) {  // a^-1 mod m (gcd = 1)
  int64_t t0 = 0, t1 = 1, r0 = m, r1 = a % m;
  while (r1) {
    const int64_t q = r0 / r1;
    std::swap(r0, r1);
    r1 -= q * r0;
    std::swap(t0, t1);
    t1 -= q * t0;
  }
  return (uint32_t)((t0 % (int64_t)m + m) % m);
}
inline uint32_t inv_2_32(uint32_t a) {  // odd a
  uint32_t x = a;
  for (int i = 0; i < 5; ++i) x *= 2u - a * x;
  return x;
}
inline uint32_t shoup_const(uint32_t w, uint32_t m) {  // floor(w 2^32 / m), w < m
  return (uint32_t)(((uint64_t)w << 32) / m);
}
inline uint32_t mod_small(const BigU& x, uint32_t m) {  // m = 0: mod 2^32
  if (m == 0) return x.word(0);
  uint64_t r = 0;
  for (size_t k = x.w.size(); k-- > 0;) r = ((r << 32) | x.w[k]) % m;
  return (uint32_t)r;
}
struct Bases {
  std::vector<uint32_t> b, b2;  // B and B' (the 2 RK largest primes below 2^28, interleaved)
  BigU M, M2;
  std::vector<BigU> Mi, M2j;
  std::vector<uint32_t> shared;  // the S_* block
};
inline const Bases& bases() {
  static const Bases B = [] {
    using namespace rns;
    Bases r;
    std::vector<uint32_t> pr;
    for (uint32_t c = (1u << 28) - 1; (int)pr.size() < 2 * RK; c -= 2)
      if (prime32(c)) pr.push_back(c);
    for (int i = 0; i < 2 * RK; ++i) (i % 2 ? r.b2 : r.b).push_back(pr[i]);
    r.M = BigU(1);
    r.M2 = BigU(1);
    for (int i = 0; i < RK; ++i) {
      r.M = mul(r.M, BigU(r.b[i]));
      r.M2 = mul(r.M2, BigU(r.b2[i]));
    }
    for (int i = 0; i < RK; ++i) {
      BigU q;
      divmod(r.M, BigU(r.b[i]), &q, nullptr);
      r.Mi.push_back(q);
      divmod(r.M2, BigU(r.b2[i]), &q, nullptr);
      r.M2j.push_back(q);
    }
    std::vector<uint32_t>& s = r.shared;
    s.assign(S_WORDS, 0u);
    for (int slot = 0; slot < NSLOT; ++slot) {  // slot = 80 base + channel; B' channel RCH is r
      const bool gB = slot < 80;
      const int ch = gB ? slot : slot - 80;
      const bool isr = !gB && ch == RCH;
      if (!(ch < RK || isr)) continue;
      const uint32_t m = isr ? 0u : (gB ? r.b[ch] : r.b2[ch]);
      if (m) {
        s[S_M + slot] = m;
        s[S_MU + slot] = (uint32_t)((1ull << 59) / m);
        s[S_T32 + slot] = (uint32_t)((1ull << 32) % m);
      }
      for (int i = 0; i < RK; ++i)  // B: |M'_j|_(m_i); B': |M_i|_(m'_j); 2^32: |M_i|_(2^32)
        s[S_ROWS + i * NSLOT + slot] = gB ? mod_small(r.M2j[i], m) : mod_small(r.Mi[i], m);
      if (gB) {
        s[S_B + slot] = mod_small(r.M2, m);                       // |M'|_(m_i)
        s[S_C + slot] = inv_mod(mod_small(r.Mi[ch], m), m);        // |M_i^-1|_(m_i)
      } else if (!isr) {
        const uint64_t minv = inv_mod(mod_small(r.M, m), m);
        s[S_B + slot] = (uint32_t)minv;                                               // |M^-1|_(m'_j)
        s[S_C + slot] = (uint32_t)(minv * inv_mod(mod_small(r.M2j[ch], m), m) % m);  // |M^-1 M'_j^-1|_(m'_j)
        s[S_D + slot] = r.M2j[ch].word(0);                                            // |M'_j|_(2^32)
      } else {
        s[S_B + slot] = inv_2_32(r.M.word(0));  // M^-1 mod 2^32
      }
      if (m) {
        s[S_BS + slot] = shoup_const(s[S_B + slot], m);
        s[S_CS + slot] = shoup_const(s[S_C + slot], m);
      }
    }
    for (int i = 0; i < RK; ++i) {
      const std::vector<uint32_t> l = r.Mi[i].to_limbs(28, RKP);
      for (int c = 0; c < RKP; ++c) s[S_MPOS + i * RKP + c] = l[c];
    }
    const std::vector<uint32_t> lm = r.M.to_limbs(28, RKP);
    for (int c = 0; c < RKP; ++c) s[S_MFULL + c] = lm[c];
    s[S_M2RINV] = inv_2_32(r.M2.word(0));
    return r;
  }();
  return B;
}
// the per-prime block for N = P^2: |-N^-1 M_i^-1| (B), |N M^-1| and |N M^-1
// M'_j^-1| (B'), N mod 2^32; M^3 mod N in every channel; and the exponent P - 1
// as the kernel's sliding-window schedule (5-bit windows, the rule of
// pow_uniform_exp: each window ends in a set bit)
inline std::vector<uint32_t> prime_block(const BigU& P) {
  using namespace rns;
  const Bases& b = bases();
  const BigU N = mul(P, P);
  std::vector<uint32_t> v(P_WORDS, 0u);
  const BigU MN = mod(b.M, N);
  const BigU M3 = mulmod(mulmod(MN, MN, N), MN, N);
  for (int slot = 0; slot < NSLOT; ++slot) {
    const bool gB = slot < 80;
    const int ch = gB ? slot : slot - 80;
    const bool isr = !gB && ch == RCH;
    if (!(ch < RK || isr)) continue;
    const uint32_t m = isr ? 0u : (gB ? b.b[ch] : b.b2[ch]);
    if (gB) {
      const uint64_t ni = inv_mod(mod_small(N, m), m), mi = inv_mod(mod_small(b.Mi[ch], m), m);
      v[P_A + slot] = (uint32_t)((m - ni * mi % m) % m);
    } else if (!isr) {
      const uint64_t nm = (uint64_t)mod_small(N, m) * inv_mod(mod_small(b.M, m), m) % m;
      v[P_A + slot] = (uint32_t)nm;
      v[P_A2 + slot] = (uint32_t)(nm * inv_mod(mod_small(b.M2j[ch], m), m) % m);
      v[P_A2S + slot] = shoup_const(v[P_A2 + slot], m);
    } else {
      v[P_A + slot] = N.word(0);
    }
    if (m) v[P_AS + slot] = shoup_const(v[P_A + slot], m);
    v[P_M3 + slot] = mod_small(M3, m);
  }
  // schedule over e = P - 1 (bits high to low)
  const BigU e = sub(P, BigU(1));
  const int nb = (int)e.bits();
  auto bit = [&](int i) { return (e.word((size_t)i / 32) >> (i % 32)) & 1u; };  // i: from the bottom
  auto window = [&](int hi, int* lo_out) {  // the window from bit hi down (at most 5 bits, ends in a set bit)
    int lo = std::max(hi - 4, 0);
    while (!bit(lo)) ++lo;
    uint32_t val = 0;
    for (int i = hi; i >= lo; --i) val = val << 1 | bit(i);
    *lo_out = lo;
    return val;
  };
  int ns = 0, lo;
  const uint32_t first = window(nb - 1, &lo);
  v[P_SCHED + ns++] = (first - 1) / 2;
  int i = lo - 1;
  uint32_t sq = 0;
  while (i >= 0) {
    if (!bit(i)) {
      ++sq;
      --i;
      continue;
    }
    const uint32_t w = window(i, &lo);
    sq += (uint32_t)(i - lo + 1);
    if (ns >= P_SCHED_MAX) throw std::runtime_error("rns schedule overflow");
    v[P_SCHED + ns++] = sq << 8 | ((w - 1) / 2 + 1);
    sq = 0;
    i = lo - 1;
  }
  if (sq) {
    if (ns >= P_SCHED_MAX) throw std::runtime_error("rns schedule overflow");
    v[P_SCHED + ns++] = sq << 8;
  }
  v[P_NS] = (uint32_t)ns;
  return v;
}
}  // namespace rnsh

struct ModOff {
  size_t N, R1, R2, R3, Rpow = 0;
  uint32_t n0inv;
  int npow = 0;
};

// npow > 0 also stores R^j mod M for j < npow (consecutive rows of S4 limbs):
// the fix-up factors of chains over plain residues (k_chunk_prod, raw inputs)
ModOff put_mod(Blob& bl, const BigU& M, const ModSpec& s, int npow = 0) {
  ModOff o;
  BigU R = pow2((size_t)s.W * s.S);
  BigU R1 = mod(R, M);
  BigU R2 = mulmod(R1, R1, M);
  BigU R3 = mulmod(R2, R1, M);
  o.N = bl.put_limbs(M, s);
  o.R1 = bl.put_limbs(R1, s);
  o.R2 = bl.put_limbs(R2, s);
  o.R3 = bl.put_limbs(R3, s);
  o.n0inv = mont_ninv(M.word(0), s.W);
  if (npow > 0) {
    BigU x = mod(BigU(1), M);
    for (int j = 0; j < npow; ++j) {
      const size_t off = bl.put_limbs(x, s);
      if (j == 0) o.Rpow = off;
      x = mulmod(x, R1, M);
    }
    o.npow = npow;
  }
  return o;
}

}  // namespace

struct xhe_key {
  int device = 0;
  int K = 0, nw = 0, n2w = 0;
  bool priv = false, djn = false;
  int rand_bits = 0, rand_words = 0;
  ModSpec mp2{}, mp{}, mn2{}, mp2L{}, mp2X{}, mn2X{};
  uint32_t* d_blob = nullptr;
  uint32_t* d_tab = nullptr;
  KeyDev kd{};
  std::vector<uint32_t> n_host;   // n words (for host-side checks)
  std::vector<uint32_t> n2_host;  // n^2 words (host inverse at the batch-inversion root)
  int n_bits = 0;
  int dneg = 0;  // smallest d with 1 << d >= min_value_for_negative (= n - n // 3): alignment gaps from
                 // here on take _raw_mul's negative branch (paillier.py:79-86, 173-187)
};

namespace {

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int dev) {
    HIPCHK(hipGetDevice(&prev));
    if (prev != dev) HIPCHK(hipSetDevice(dev));
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

template <class MP2, int RW>
void build_tables_m(xhe_key* k, const ModDev& md, const uint32_t* d_hM, uint32_t* d_tab, uint32_t* d_chain,
                    uint32_t* d_ws, hipStream_t s);

// Window layout of a fixed-base table over rand_bits exponent bits: uniform
// ceil(rand_bits/win) windows, or (split) floor(rand_bits/win) windows of
// which the first rand_bits mod win are win+1 bits wide (KeyDev::nhi).
void win_layout(int rand_bits, int win, bool split, int* nwin, int* nhi) {
  *nwin = (rand_bits + win - 1) / win;
  *nhi = 0;
  if (split && rand_bits % win != 0 && rand_bits % win <= rand_bits / win) {
    *nwin = rand_bits / win;
    *nhi = rand_bits % win;
  }
}

int64_t chain_rows_h(int win) { return ((int64_t)1 << (win / 2)) + ((int64_t)1 << (win - win / 2)); }

// Tables of one modulus, or of p^2 and q^2 concurrently on two streams.
template <class MP2, int RW>
void build_tables_sync(xhe_key* k, const ModDev* md, const uint32_t* const* d_hM, uint32_t* const* d_tab, int count) {
  hipStream_t st[2] = {nullptr, nullptr};
  uint32_t* ws[2] = {nullptr, nullptr};
  uint32_t* chain[2] = {nullptr, nullptr};
  const int win = k->kd.win, nwin = k->kd.nwin, nhi = k->kd.nhi;
  const size_t chain_words =
      (size_t)std::max<int64_t>(nhi ? (nhi + 1) * chain_rows_h(win + 1) : 0, (nwin - nhi) * chain_rows_h(win)) *
      MP2::S4;
  for (int i = 0; i < count; ++i) {
    HIPCHK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    HIPCHK(hipMalloc(&ws[i], MP2::S4 * sizeof(uint32_t) * 4));
    HIPCHK(hipMalloc(&chain[i], chain_words * sizeof(uint32_t)));
    build_tables_m<MP2, RW>(k, md[i], d_hM[i], d_tab[i], chain[i], ws[i], st[i]);
  }
  for (int i = 0; i < count; ++i) {
    HIPCHK(hipStreamSynchronize(st[i]));
    HIPCHK(hipFree(ws[i]));
    HIPCHK(hipFree(chain[i]));
    HIPCHK(hipStreamDestroy(st[i]));
  }
}

// One uniform table segment (nwin windows of win bits starting at base
// d_base), enqueued on `s` (no synchronisation; d_ws and d_chain must stay
// alive until s has drained): window bases (low entry 1 of every window) =
// base^(2^(win w)) by one squaring chain over nbases >= nwin windows, every
// window's low and high chains by doubling levels (k_tab_level: log2 depth
// instead of 2^(win/2)), then every packed row as one product of a high and a
// low entry.
template <class MP2, int RW>
void build_tables_seg(const ModDev& md, const uint32_t* d_base, int win, int nwin, int nbases, uint32_t* d_tab,
                      int64_t rs, uint32_t* d_chain, uint32_t* d_ws, hipStream_t s) {
  const int half = win / 2;
  hipLaunchKernelGGL(k_tab_bases<MP2>, dim3(1), dim3(64), 0, s, md, d_base, win, nbases, d_chain, d_ws);
  HIPCHK(hipGetLastError());
  auto blocks = [&](int64_t groups) { return dim3((unsigned)std::max<int64_t>(1, (groups * MP2::TPI + 255) / 256)); };
  hipLaunchKernelGGL(k_tab_one<MP2>, blocks(nwin), dim3(256), 0, s, md, win, nwin, d_chain);
  HIPCHK(hipGetLastError());
  const int lim_lo = (1 << half) + 1, lim_hi = 1 << (win - half);
  for (int t = 0; (1 << t) < lim_lo - 1; ++t) {
    hipLaunchKernelGGL(k_tab_level<MP2>, blocks((int64_t)nwin << t), dim3(256), 0, s, md, md.N, win, nwin, t, 0,
                       lim_lo, d_chain);
    HIPCHK(hipGetLastError());
  }
  for (int t = 0; (1 << t) < lim_hi - 1; ++t) {
    hipLaunchKernelGGL(k_tab_level<MP2>, blocks((int64_t)nwin << t), dim3(256), 0, s, md, md.N, win, nwin, t, half,
                       lim_hi, d_chain);
    HIPCHK(hipGetLastError());
  }
  int64_t rows = (int64_t)nwin << win;
  hipLaunchKernelGGL((k_tab_combine<MP2, RW>), blocks(rows), dim3(256), 0, s, md, md.N, win, nwin, d_chain, d_tab,
                     rs);
  HIPCHK(hipGetLastError());
}

// A key's tables (layout win_layout / win_digit): uniform, or the nhi wide
// windows first, whose base chain runs one window further to
// h^(2^(nhi (win+1))), the base of the narrow windows that follow.
template <class MP2, int RW>
void build_tables_m(xhe_key* k, const ModDev& md, const uint32_t* d_hM, uint32_t* d_tab, uint32_t* d_chain,
                    uint32_t* d_ws, hipStream_t s) {
  const int win = k->kd.win, nwin = k->kd.nwin, nhi = k->kd.nhi;
  const int64_t rs = RW == k->K / 32 ? k->kd.tab_rs : RW;  // p^2/q^2 rows (maybe interleaved) or n^2 rows
  if (nhi == 0) {
    build_tables_seg<MP2, RW>(md, d_hM, win, nwin, nwin, d_tab, rs, d_chain, d_ws, s);
    return;
  }
  uint32_t* base2 = d_ws + 2 * MP2::S4;  // d_ws rows: 0 = squaring scratch, 2 = the narrow windows' base
  build_tables_seg<MP2, RW>(md, d_hM, win + 1, nhi, nhi + 1, d_tab, rs, d_chain, d_ws, s);
  HIPCHK(hipMemcpyAsync(base2, d_chain + ((size_t)nhi * chain_rows_h(win + 1) + 1) * MP2::S4,
                        MP2::S4 * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  build_tables_seg<MP2, RW>(md, base2, win, nwin - nhi, nwin - nhi, d_tab + ((size_t)nhi << (win + 1)) * rs, rs,
                            d_chain, d_ws, s);
}

ModDev moddev(uint32_t* base, const ModOff& o) {
  return ModDev{base + o.N, base + o.R1, base + o.R2, base + o.R3, o.n0inv, o.npow ? base + o.Rpow : nullptr};
}

void key_create_impl(xhe_key* k, const BigU& n, const BigU* p, const BigU* q, const BigU* h, int win) {
  Blob bl;
  const int K = k->K;
  BigU n2 = mul(n, n);
  size_t o_n = bl.put_words(n, k->nw);
  size_t o_n2 = bl.put_words(n2, k->n2w);
  BigU maxpos, minneg;
  divmod(n, BigU(3), &maxpos, nullptr);
  minneg = sub(n, maxpos);
  size_t o_maxpos = bl.put_words(maxpos, k->nw);
  size_t o_minneg = bl.put_words(minneg, k->nw);
  size_t o_nlim = bl.put_limbs(n, k->mp2);
  ModOff o_n2m = put_mod(bl, n2, k->mn2, kRpowRows);
  ModOff o_n2X = put_mod(bl, n2, k->mn2X, kRpowRows);
  size_t o_n2wN = 0, o_n2wnp = 0, o_n2wC = 0, o_n2wR2 = 0, o_n2mu = 0;
  if (K == 2048) {  // k_add_barrett: mu = floor(beta^(2S) / n^2), beta = 2^27, S = 152
    static_assert(bar::S == 152, "Barrett constants are for 2048-bit keys");
    BigU mu;
    divmod(pow2((size_t)27 * 2 * bar::S), n2, &mu, nullptr);
    o_n2mu = bl.put_limbs(mu, ModSpec{bar::S + 1, 27});
  }
  if (K == 2048) {  // k_mexp_horner_wave
    const ModSpec sw{154, 27};
    const BigU Rw = pow2((size_t)27 * 154), RX = pow2((size_t)k->mn2X.W * k->mn2X.S);
    o_n2wN = bl.put_limbs(n2, sw);
    o_n2wnp = bl.put_limbs(sub(Rw, modinv(n2, Rw)), sw);
    const BigU Rwn = mod(Rw, n2);
    o_n2wC = bl.put_limbs(mulmod(mulmod(Rwn, Rwn, n2), modinv(mod(RX, n2), n2), n2), sw);
    o_n2wR2 = bl.put_limbs(mulmod(Rwn, Rwn, n2), sw);
  }
  size_t o_nR2n2, o_hMn2 = 0;
  {
    BigU Rn2 = mod(pow2((size_t)k->mn2.W * k->mn2.S), n2);
    o_nR2n2 = bl.put_limbs(mulmod(n, mulmod(Rn2, Rn2, n2), n2), k->mn2);
    if (h && !p) o_hMn2 = bl.put_limbs(mulmod(mod(*h, n2), Rn2, n2), k->mn2);  // public DJN table base
  }
#if XHE_NDIG
  // Montgomery digits mod n^2 (PMDX<80, 4>, pdigit_dev.hpp): n in 80 limbs of
  // 27 bits, R = 2^2160; ceil(R/n) n^2 (the input conversion's offset), R - n,
  // the digits (e, f) of R^2 mod n^2 and of 1 (R e + n f = X R^2 mod n^2),
  // MASK + E_i with E = (1 - R) mod n
  struct {
    ModOff nd;
    size_t kn2 = 0, rmn = 0, dw = 0, d1 = 0, topc = 0, dwt = 0;
  } on;
  if (K == 2048) {
    const ModSpec sn{80, 27};
    on.nd = put_mod(bl, n, sn);
    const BigU R = pow2((size_t)27 * 80);
    BigU q;
    divmod(sub(add(R, n), BigU(1)), n, &q, nullptr);  // ceil(R / n)
    on.kn2 = bl.put_limbs(mul(q, n2), ModSpec{160, 27});
    on.rmn = bl.put_limbs(sub(R, n), sn);
    const BigU Rn = mod(R, n), Rinv = modinv(Rn, n);
    auto digits = [&](const BigU& X) {
      const BigU e = mulmod(mod(X, n), Rinv, n);
      BigU Q;
      divmod(add(X, mul(R, sub(n, e))), n, &Q, nullptr);  // (X - R e) / n + R
      const BigU f = submod(mod(Q, n), Rn, n);
      const std::vector<uint32_t> el = e.to_limbs(27, 80), fl = f.to_limbs(27, 80);
      std::vector<uint32_t> v(160);
      for (int i = 0; i < 80; ++i) {
        v[2 * i] = el[i];
        v[2 * i + 1] = fl[i];
      }
      return bl.put(v);
    };
    const BigU R2 = mulmod(mod(R, n2), mod(R, n2), n2);  // R^2 mod n^2
    on.d1 = digits(R2);                                   // 1 R^2
    on.dw = digits(mulmod(R2, R2, n2));                   // R^2 R^2
    // R^2 R_MN2^-1 (R_MN2 = 2^(27*152), the public DJN tables' Montgomery
    // factor): converts their rows to canonical digits (k_tab_to_pmdx, n)
    const BigU RM = mod(pow2((size_t)k->mn2.W * k->mn2.S), n2);
    on.dwt = digits(mulmod(mulmod(R2, R2, n2), modinv(RM, n2), n2));  // X = w R^2, w = R^2 R_MN2^-1
    std::vector<uint32_t> tc = submod(BigU(1), Rn, n).to_limbs(27, 80);
    for (auto& x : tc) x += (1u << 27) - 1u;
    on.topc = bl.put(tc);
  }
#endif
  // randomness bound (paillier.py:195 djn_exp_bound = 2^(bitlen(n)//2); :215 r < n)
  k->rand_bits = k->djn ? (int)(n.bits() / 2) : (int)n.bits();
  k->rand_words = (k->rand_bits + 31) / 32;

  struct {
    ModOff p2, q2, p, q, p2L, q2L, p2X, q2X;
    size_t nR2C_p2X = 0, nR2C_q2X = 0, R1C_p2X = 0, R1C_q2X = 0;
    size_t nR_p2 = 0, nR_q2 = 0;
    size_t nR2_p2L = 0, nR2_q2L = 0;
    size_t nR2_p2 = 0, nR2_q2 = 0, q2invR = 0, q2_lim = 0, p2x4 = 0, hM_p2 = 0, hM_q2 = 0;
    size_t pm1 = 0, qm1 = 0, pinv = 0, qinv = 0, hpR = 0, hqR = 0, qinvpR = 0, q_lim = 0, p2x = 0, p_lim = 0;
    size_t ep = 0, eq = 0;
    size_t topc_p = 0, topc_q = 0;
    size_t nprime_p2 = 0, nprime_q2 = 0;
    size_t rns = 0, rns_p = 0, rns_q = 0;
    ModOff xd[2];
    size_t xkn2[2] = {0, 0}, xrmn[2] = {0, 0}, xtopc[2] = {0, 0}, xfold[2] = {0, 0}, xdwt[2] = {0, 0};
    size_t xdw[2] = {0, 0}, xhpR[2] = {0, 0};
  } o;
  int pm1_bits = 0, qm1_bits = 0, ep_bits = 0, eq_bits = 0;
  if (k->priv) {
    const BigU &P = *p, &Q = *q;
    BigU p2 = mul(P, P), q2 = mul(Q, Q);
    const ModSpec& s2 = k->mp2;
    const ModSpec& s1 = k->mp;
    o.p2 = put_mod(bl, p2, s2);
    o.p2L = put_mod(bl, p2, k->mp2L);
    o.q2L = put_mod(bl, q2, k->mp2L);
    o.p2X = put_mod(bl, p2, k->mp2X);
    o.q2X = put_mod(bl, q2, k->mp2X);
    o.q2 = put_mod(bl, q2, s2);
    if (K == 2048) {  // -P^-2 mod R for k_dec_wave's parallel REDC
      const BigU R = pow2((size_t)s2.W * s2.S);
      o.nprime_p2 = bl.put_limbs(sub(R, modinv(p2, R)), s2);
      o.nprime_q2 = bl.put_limbs(sub(R, modinv(q2, R)), s2);
      // the RNS decrypt's bases (shared by every key) and per-prime constants
      o.rns = bl.put(rnsh::bases().shared);
      o.rns_p = bl.put(rnsh::prime_block(P));
      o.rns_q = bl.put(rnsh::prime_block(Q));
    }
    BigU R2p = pow2((size_t)s2.W * s2.S);
    BigU Rp2 = mod(R2p, p2), Rq2 = mod(R2p, q2);
    // n R^2 mod P^2
    o.nR2_p2 = bl.put_limbs(mulmod(mod(n, p2), mulmod(Rp2, Rp2, p2), p2), s2);
    o.nR2_q2 = bl.put_limbs(mulmod(mod(n, q2), mulmod(Rq2, Rq2, q2), q2), s2);
    {  // n R_L^2 mod P^2 for the 4-lane shape (k_nodjn_crt<MP2L, 1>)
      const ModSpec& sL = k->mp2L;
      BigU RL = pow2((size_t)sL.W * sL.S);
      BigU RLp = mod(RL, p2), RLq = mod(RL, q2);
      o.nR2_p2L = bl.put_limbs(mulmod(mod(n, p2), mulmod(RLp, RLp, p2), p2), sL);
      o.nR2_q2L = bl.put_limbs(mulmod(mod(n, q2), mulmod(RLq, RLq, q2), q2), sL);
    }
    o.nR_p2 = bl.put_limbs(mulmod(mod(n, p2), Rp2, p2), s2);  // n R mod P^2
    o.nR_q2 = bl.put_limbs(mulmod(mod(n, q2), Rq2, q2), s2);
    // CRT constants (context.py:46)
    BigU q2inv = modinv(q2, p2);
    o.q2invR = bl.put_limbs(mulmod(q2inv, Rp2, p2), s2);
    o.q2_lim = bl.put_limbs(q2, s2);
    o.p2x4 = bl.put_limbs(shl(p2, 2), s2);
    if (k->djn) {
      o.hM_p2 = bl.put_limbs(mulmod(mod(*h, p2), Rp2, p2), s2);  // h_pow_n mod p^2 (context.py:63)
      o.hM_q2 = bl.put_limbs(mulmod(mod(*h, q2), Rq2, q2), s2);
      // 16-lane small-batch shape on the same tables (k_djn_pow_x)
      int nwin, nhi;
      win_layout(k->rand_bits, win & 0xff, (win & XHE_WIN_SPLIT) != 0, &nwin, &nhi);
      const ModSpec& sx = k->mp2X;
      BigU Rx = pow2((size_t)sx.W * sx.S);
      BigU Cexp = pow2((size_t)(sx.S - s2.S) * s2.W * nwin);  // (R'/R)^nwin
      auto put_x = [&](const BigU& P2, size_t* nr2c, size_t* r1c) {
        BigU C = mod(Cexp, P2), RxP = mod(Rx, P2);
        BigU CR = mulmod(C, RxP, P2);
        *r1c = bl.put_limbs(CR, sx);
        *nr2c = bl.put_limbs(mulmod(mod(n, P2), mulmod(CR, RxP, P2), P2), sx);
      };
      put_x(p2, &o.nR2C_p2X, &o.R1C_p2X);
      put_x(q2, &o.nR2C_q2X, &o.R1C_q2X);
    }
    // mod p / q (decrypt)
    o.p = put_mod(bl, P, s1);
    o.q = put_mod(bl, Q, s1);
    BigU pm1 = sub(P, BigU(1)), qm1 = sub(Q, BigU(1));
    pm1_bits = (int)pm1.bits();
    qm1_bits = (int)qm1.bits();
    o.pm1 = bl.put_words(pm1, k->nw / 2 + 1);
    o.qm1 = bl.put_words(qm1, k->nw / 2 + 1);
    BigU T = pow2((size_t)s1.W * s1.S);
    o.pinv = bl.put_limbs(modinv(P, T), s1);
    o.qinv = bl.put_limbs(modinv(Q, T), s1);
    // hp = L_p((n+1)^(p-1) mod p^2)^-1 mod p (context.py:47,193-194). By the
    // binomial theorem (n+1)^(p-1) = 1 + (p-1) n (mod n^2, hence mod p^2).
    auto hfun = [&](const BigU& X, const BigU& X2) {
      BigU x = mod(add(BigU(1), mul(sub(X, BigU(1)), n)), X2);
      BigU L;
      divmod(sub(x, BigU(1)), X, &L, nullptr);
      return modinv(L, X);
    };
    BigU hp = hfun(P, p2), hq = hfun(Q, q2);
    BigU Rp = mod(T, P), Rq = mod(T, Q);
    o.hpR = bl.put_limbs(mulmod(hp, Rp, P), s1);
    o.hqR = bl.put_limbs(mulmod(hq, Rq, Q), s1);
    o.qinvpR = bl.put_limbs(mulmod(modinv(Q, P), Rp, P), s1);  // context.py:43
    o.q_lim = bl.put_limbs(Q, s1);
#if XHE_PMD && XHE_LDS_ROWS
    if (K == 2048) {
      // Montgomery-digit kernels (k_djn_pmd, k_dec_pmd): MASK + E_i, E = (1 - R) mod P,
      // R = 2^(28*37) (= the mod-p shape's R, so R mod P is kd.p.R1)
      auto topc = [&](const BigU& X) {
        std::vector<uint32_t> v = submod(BigU(1), mod(T, X), X).to_limbs(28, 37);
        for (auto& x : v) x += (1u << 28) - 1u;
        return bl.put(v);
      };
      o.topc_p = topc(P);
      o.topc_q = topc(Q);
    }
#endif
#if XHE_PMDX
    if (K == 3072 || K == 4096 || K == 8192) {
      // Montgomery digits mod P^2 over 4 lanes (k_djn_pmdx, k_dec_pmdx_*): per
      // prime the modulus P in K limbs of 27 bits (R = 2^(27 K)), ceil(R/P)
      // P^2, R - P, MASK + E_i, the fold constant Q R^3 mod P, the digits of
      // R^2 R_MP2^-1 mod P^2 (R_MP2: the MP2 shape's R, the tables' factor)
      // and of R^2 mod P^2 (plain conversion), and hp R mod P (decrypt)
      const int KD = K == 3072 ? 60 : K == 4096 ? 80 : 160;
      const ModSpec sd{KD, 27};
      const BigU Rd = pow2((size_t)27 * KD), RM = pow2((size_t)s2.W * s2.S);
      for (int i = 0; i < 2; ++i) {
        const BigU& X = i ? Q : P;
        const BigU& Y = i ? P : Q;
        const BigU X2 = i ? q2 : p2;
        o.xd[i] = put_mod(bl, X, sd);
        BigU cq;
        divmod(sub(add(Rd, X), BigU(1)), X, &cq, nullptr);
        o.xkn2[i] = bl.put_limbs(mul(cq, X2), ModSpec{2 * KD, 27});
        o.xrmn[i] = bl.put_limbs(sub(Rd, X), sd);
        const BigU RdX = mod(Rd, X);
        std::vector<uint32_t> tc = submod(BigU(1), RdX, X).to_limbs(27, KD);
        for (auto& x : tc) x += (1u << 27) - 1u;
        o.xtopc[i] = bl.put(tc);
        o.xfold[i] = bl.put_limbs(mulmod(mod(Y, X), mulmod(mulmod(RdX, RdX, X), RdX, X), X), sd);
        // digits (e, f) of w: R e + X f = w R^2 (mod X^2), as K interleaved pairs;
        // Xw = w R^2 mod X^2
        auto put_digits = [&](const BigU& Xw) {
          const BigU e = mulmod(mod(Xw, X), modinv(RdX, X), X);
          BigU Qd;
          divmod(add(Xw, mul(Rd, sub(X, e))), X, &Qd, nullptr);
          const BigU f = submod(mod(Qd, X), RdX, X);
          const std::vector<uint32_t> el = e.to_limbs(27, KD), fl = f.to_limbs(27, KD);
          std::vector<uint32_t> v(2 * KD);
          for (int j = 0; j < KD; ++j) {
            v[2 * j] = el[j];
            v[2 * j + 1] = fl[j];
          }
          return bl.put(v);
        };
        const BigU Rd2 = mulmod(mod(Rd, X2), mod(Rd, X2), X2);
        const BigU Rd4 = mulmod(Rd2, Rd2, X2);
        o.xdwt[i] = put_digits(mulmod(Rd4, modinv(mod(RM, X2), X2), X2));  // w = R^2 R_MP2^-1
        o.xdw[i] = put_digits(Rd4);                                        // w = R^2
        o.xhpR[i] = bl.put_limbs(mulmod(i ? hq : hp, RdX, X), sd);
      }
    }
#endif
    o.p2x = bl.put_limbs(shl(P, 1), s1);
    o.p_lim = bl.put_limbs(P, s1);
    // non-DJN private obfuscation exponents ep = n mod phi(p^2) (context.py:51-52)
    BigU ep = mod(n, mul(P, sub(P, BigU(1)))), eq = mod(n, mul(Q, sub(Q, BigU(1))));
    ep_bits = (int)ep.bits();
    eq_bits = (int)eq.bits();
    o.ep = bl.put_words(ep, k->nw);
    o.eq = bl.put_words(eq, k->nw);
  }
  // upload
  HIPCHK(hipMalloc(&k->d_blob, bl.h.size() * sizeof(uint32_t)));
  HIPCHK(hipMemcpy(k->d_blob, bl.h.data(), bl.h.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  uint32_t* B = k->d_blob;
  KeyDev& kd = k->kd;
  kd.K = K;
  kd.nw = k->nw;
  kd.n2w = k->n2w;
  kd.priv = k->priv;
  kd.djn = k->djn;
  kd.n_words = B + o_n;
  kd.n2_words = B + o_n2;
  kd.maxpos = B + o_maxpos;
  kd.minneg = B + o_minneg;
  kd.n_lim = B + o_nlim;
  kd.n2 = moddev(B, o_n2m);
  kd.n2X = moddev(B, o_n2X);
  if (K == 2048) {
    kd.n2w_N = B + o_n2wN;
    kd.n2w_np = B + o_n2wnp;
    kd.n2w_C = B + o_n2wC;
    kd.n2w_R2 = B + o_n2wR2;
    kd.n2_mu = B + o_n2mu;
  }
  kd.nR2_n2 = B + o_nR2n2;
  kd.n_bits = (int)n.bits();
#if XHE_NDIG
  if (K == 2048) {
    kd.ndig = 1;
    kd.nd = moddev(B, on.nd);
    kd.nd_kn2 = B + on.kn2;
    kd.nd_rmn = B + on.rmn;
    kd.nd_topc = B + on.topc;
    kd.nd_dw = reinterpret_cast<const uint2*>(B + on.dw);
    kd.nd_d1 = reinterpret_cast<const uint2*>(B + on.d1);
    kd.nd_dwt = reinterpret_cast<const uint2*>(B + on.dwt);
  }
#endif
  if (k->priv) {
    kd.p2 = moddev(B, o.p2);
    kd.p2L = moddev(B, o.p2L);
    kd.q2L = moddev(B, o.q2L);
    kd.p2X = moddev(B, o.p2X);
    kd.q2X = moddev(B, o.q2X);
    kd.q2 = moddev(B, o.q2);
    kd.nR2_p2 = B + o.nR2_p2;
    kd.nR_p2 = B + o.nR_p2;
    kd.nR_q2 = B + o.nR_q2;
    kd.nR2C_p2X = B + o.nR2C_p2X;
    kd.nR2C_q2X = B + o.nR2C_q2X;
    kd.R1C_p2X = B + o.R1C_p2X;
    kd.R1C_q2X = B + o.R1C_q2X;
    kd.nR2_q2 = B + o.nR2_q2;
    kd.nR2_p2L = B + o.nR2_p2L;
    kd.nR2_q2L = B + o.nR2_q2L;
    kd.q2invR_p2 = B + o.q2invR;
    kd.q2_lim = B + o.q2_lim;
    kd.p2x4_lim = B + o.p2x4;
    kd.p = moddev(B, o.p);
    kd.q = moddev(B, o.q);
    kd.pm1_words = B + o.pm1;
    kd.qm1_words = B + o.qm1;
    kd.pm1_bits = pm1_bits;
    kd.qm1_bits = qm1_bits;
    kd.pinv_lim = B + o.pinv;
    kd.qinv_lim = B + o.qinv;
    kd.hpR = B + o.hpR;
    kd.hqR = B + o.hqR;
    kd.qinvpR = B + o.qinvpR;
    kd.q_lim = B + o.q_lim;
    kd.p2x_lim = B + o.p2x;
    kd.p_lim = B + o.p_lim;
    kd.ep_words = B + o.ep;
    kd.eq_words = B + o.eq;
    kd.ep_bits = ep_bits;
    kd.eq_bits = eq_bits;
    if (K == 2048) {
      kd.p2_nprime = B + o.nprime_p2;
      kd.q2_nprime = B + o.nprime_q2;
      kd.rns = B + o.rns;
      kd.rns_p = B + o.rns_p;
      kd.rns_q = B + o.rns_q;
    }
#if XHE_PMD && XHE_LDS_ROWS
    if (K == 2048) {
      kd.topc_p = B + o.topc_p;
      kd.topc_q = B + o.topc_q;
    }
#endif
#if XHE_PMDX
    if (K == 3072 || K == 4096 || K == 8192) {
      kd.pmdx_dec = 1;
      kd.x_dw_p = reinterpret_cast<const uint2*>(B + o.xdw[0]);
      kd.x_dw_q = reinterpret_cast<const uint2*>(B + o.xdw[1]);
      kd.x_hpR_p = B + o.xhpR[0];
      kd.x_hpR_q = B + o.xhpR[1];
      kd.dp = moddev(B, o.xd[0]);
      kd.dq = moddev(B, o.xd[1]);
      kd.x_kn2_p = B + o.xkn2[0];
      kd.x_kn2_q = B + o.xkn2[1];
      kd.x_rmn_p = B + o.xrmn[0];
      kd.x_rmn_q = B + o.xrmn[1];
      kd.x_topc_p = B + o.xtopc[0];
      kd.x_topc_q = B + o.xtopc[1];
      kd.x_fold_p = B + o.xfold[0];
      kd.x_fold_q = B + o.xfold[1];
      kd.x_dwt_p = reinterpret_cast<const uint2*>(B + o.xdwt[0]);
      kd.x_dwt_q = reinterpret_cast<const uint2*>(B + o.xdwt[1]);
    }
#endif
    if (k->djn) {
      kd.win = win & 0xff;
      win_layout(k->rand_bits, kd.win, (win & XHE_WIN_SPLIT) != 0, &kd.nwin, &kd.nhi);
      size_t rows = (size_t)(kd.nwin + kd.nhi) << kd.win;
      size_t tab_words = rows * (size_t)(K / 32);  // packed rows: Shape::RW = K/32 words (p^2 < 2^K)
      HIPCHK(hipMalloc(&k->d_tab, 2 * tab_words * sizeof(uint32_t)));
      kd.tab_rs = K / 32;
      kd.tab_p2 = k->d_tab;
      kd.tab_q2 = k->d_tab + tab_words;
      const ModDev mds[2] = {kd.p2, kd.q2};
      const uint32_t* hms[2] = {B + o.hM_p2, B + o.hM_q2};
      uint32_t* tabs[2] = {const_cast<uint32_t*>(kd.tab_p2), const_cast<uint32_t*>(kd.tab_q2)};
      with_shape(K, [&](auto sh) {
        using Sh = decltype(sh);
        build_tables_sync<typename Sh::MP2, Sh::RW>(k, mds, hms, tabs, 2);
      });
#if XHE_PMD && XHE_LDS_ROWS
      if (K == 2048) {
        // rows as Montgomery digits (e, f) for k_djn_pmd
        kd.pmd = 1;
        const int64_t trows = (int64_t)(kd.nwin + kd.nhi) << kd.win;
        const ModDev mp[2] = {kd.p, kd.q};
        for (int i = 0; i < 2; ++i) {
          hipLaunchKernelGGL((k_tab_to_pmd<37, 64>), dim3((unsigned)((trows + 255) / 256)), dim3(256), 0, nullptr,
                             mp[i].N, mp[i].n0inv, mp[i].R1, tabs[i], trows, (int64_t)kd.tab_rs);
          HIPCHK(hipGetLastError());
        }
        HIPCHK(hipDeviceSynchronize());
      }
#endif
#if XHE_PMDX
      if (K == 3072 || K == 4096 || K == 8192) {
        // rows as Montgomery digits (e, f) for k_djn_pmdx
        kd.pmdx = 1;
        const int64_t trows = (int64_t)(kd.nwin + kd.nhi) << kd.win;
        with_shape(K, [&](auto sh) {
          using Sh = decltype(sh);
          if constexpr (Sh::K == 3072 || Sh::K == 4096 || Sh::K == 8192) {
            using D = typename Sh::PDXO;
            for (int i = 0; i < 2; ++i) {
              hipLaunchKernelGGL((k_tab_to_pmdx<D, Sh::RW>), dim3((unsigned)((trows * D::TPI + 127) / 128)),
                                 dim3(128), 0, nullptr, kd, i, tabs[i], trows, (int64_t)kd.tab_rs);
              HIPCHK(hipGetLastError());
            }
          }
        });
        HIPCHK(hipDeviceSynchronize());
      }
#endif
    }
  }
  if (!k->priv && k->djn) {
    kd.win = win & 0xff;
    win_layout(k->rand_bits, kd.win, false, &kd.nwin, &kd.nhi);  // public tables stay uniform
    size_t rows = (size_t)kd.nwin << kd.win;
    size_t tab_words = rows * (size_t)(K / 16);  // packed rows: Shape::RW2 = n2w words
    HIPCHK(hipMalloc(&k->d_tab, tab_words * sizeof(uint32_t)));
    kd.tab_n2 = k->d_tab;
    const uint32_t* hm = B + o_hMn2;
    uint32_t* tab = k->d_tab;
    with_shape(K, [&](auto sh) {
      using Sh = decltype(sh);
      build_tables_sync<typename Sh::MN2, Sh::RW2>(k, &kd.n2, &hm, &tab, 1);
    });
#if XHE_NDIG
    if (K == 2048 && ndig_pub_on()) {
      // rows as canonical Montgomery digits of n (e, f < n: 64 + 64 words,
      // still 512 B) for k_djn_pub_nd
      kd.pub_nd = 1;
      using D = PMDX<80, 4>;
      hipLaunchKernelGGL((k_tab_to_pmdx<D, 128>), dim3((unsigned)((rows * D::TPI + 127) / 128)), dim3(128), 0, nullptr,
                         kd, 2, tab, (int64_t)rows, (int64_t)128);
      HIPCHK(hipGetLastError());
      HIPCHK(hipDeviceSynchronize());
    }
#endif
  }
}

int blocks_for(int64_t count, int tpi, int cap) {
  int64_t threads = count * tpi;
  int64_t b = (threads + 255) / 256;
  if (b < 1) b = 1;
  return (int)std::min<int64_t>(b, cap);
}

// Workspaces of the kernel entry points. Normally stream-ordered pool
// allocations; inside a host pipeline's chunk (t_ws set) they come from that
// chunk slot's cache and are kept for the whole call: with the pool, a
// workspace freed on one slot's stream and wanted by the next slot's call
// made hipMallocAsync hold the host until the first stream drained, which
// serialised the pipeline. Reuse within a slot is safe: its calls run in
// stream order, and a slot is reused only after its stream has drained.
struct WsCache {
  struct Blk {
    void* p;
    size_t bytes;
    bool used;
  };
  std::vector<Blk> blk;
  hipStream_t s = nullptr;
  WsCache() = default;
  WsCache(const WsCache&) = delete;
  WsCache& operator=(const WsCache&) = delete;
  ~WsCache() {
    for (auto& b : blk) (void)hipFreeAsync(b.p, s);
  }
};
thread_local WsCache* t_ws = nullptr;

// Outside a host pipeline, a workspace freed on stream s is kept on s's free
// list for the next call on s (stream order makes that reuse safe) instead of
// going back to the pool: a pipelined Paillier.encrypt alternates its pieces
// between two streams, and a request on one stream for memory the other had
// just freed made hipMallocAsync hold the host until that stream drained
// (the launches serialised behind each other). At most kStreamWsKeep bytes
// are kept per stream; a block is reused for requests of at least half its
// size.
constexpr size_t kStreamWsKeep = (size_t)2 << 30;
struct StreamWs {
  struct Blk {
    void* p;
    size_t bytes;
  };
  std::mutex mu;
  std::unordered_map<hipStream_t, std::vector<Blk>> free;  // oldest first
  std::unordered_map<void*, size_t> size;                  // blocks handed out
};
StreamWs& stream_ws() {
  static StreamWs* w = new StreamWs();  // process lifetime (no teardown order with the runtime)
  return *w;
}

void ws_alloc(void** p, size_t bytes, hipStream_t s) {
  if (t_ws) {
    for (auto& b : t_ws->blk)
      if (!b.used && b.bytes >= bytes) {
        b.used = true;
        *p = b.p;
        return;
      }
    HIPCHK(hipMallocAsync(p, bytes, s));
    t_ws->blk.push_back({*p, bytes, true});
    return;
  }
  StreamWs& w = stream_ws();
  {
    std::lock_guard<std::mutex> g(w.mu);
    auto it = w.free.find(s);
    if (it != w.free.end()) {
      std::vector<StreamWs::Blk>& v = it->second;
      size_t best = v.size();
      for (size_t i = 0; i < v.size(); ++i)
        if (v[i].bytes >= bytes && v[i].bytes / 2 <= bytes && (best == v.size() || v[i].bytes < v[best].bytes))
          best = i;
      if (best < v.size()) {
        *p = v[best].p;
        w.size[*p] = v[best].bytes;
        v.erase(v.begin() + (ptrdiff_t)best);
        return;
      }
    }
  }
  HIPCHK(hipMallocAsync(p, bytes, s));
  std::lock_guard<std::mutex> g(w.mu);
  w.size[*p] = bytes;
}

void ws_free(void* p, hipStream_t s) {
  if (t_ws)
    for (auto& b : t_ws->blk)
      if (b.p == p) {
        b.used = false;
        return;
      }
  StreamWs& w = stream_ws();
  std::vector<void*> drop;
  {
    std::lock_guard<std::mutex> g(w.mu);
    auto it = w.size.find(p);
    if (it == w.size.end()) {
      drop.push_back(p);  // not one of ours (allocated inside a host pipeline's cache, never here)
    } else {
      std::vector<StreamWs::Blk>& v = w.free[s];
      v.push_back({p, it->second});
      w.size.erase(it);
      size_t total = 0;
      for (const auto& b : v) total += b.bytes;
      while (total > kStreamWsKeep && !v.empty()) {
        total -= v.front().bytes;
        drop.push_back(v.front().p);
        v.erase(v.begin());
      }
    }
  }
  for (void* q : drop) HIPCHK(hipFreeAsync(q, s));
}

constexpr int64_t kChunk = 1 << 20;  // elements per launch chunk (bounds workspace)

// ---- optional per-kernel timing (hipEvents on the launch stream)
struct ProfRec {
  std::string name;
  hipEvent_t a, b;
};
std::mutex g_prof_mu;
bool g_prof_on = false;
std::vector<ProfRec> g_prof;

struct ProfScope {
  hipEvent_t a = nullptr, b = nullptr;
  hipStream_t s;
  const char* name;
  bool on;
  ProfScope(const char* n, hipStream_t st) : s(st), name(n) {
    {
      std::lock_guard<std::mutex> lk(g_prof_mu);
      on = g_prof_on;
    }
    if (on) {
      HIPCHK(hipEventCreate(&a));
      HIPCHK(hipEventCreate(&b));
      HIPCHK(hipEventRecord(a, s));
    }
  }
  ~ProfScope() {
    if (!on) return;
    if (hipEventRecord(b, s) != hipSuccess) return;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof.push_back({name, a, b});
  }
};

// DJN private encryption in the 16-lane shape up to kEncRowMax elements
// (tools/dec_shapes.py --enc: 64 elements 0.50 ms vs 1.95 ms one lane per
// residue, 16 k 1.86 vs 2.16 ms, 64 k 6.2 vs 3.8 ms); $XHE_ENC_TPI (16 or 0)
// pins it.
constexpr int64_t kEncRowMax = 20480;
bool enc_row(int64_t count) {
  static const int pin = [] {
    const char* e = std::getenv("XHE_ENC_TPI");
    return e ? std::atoi(e) : -1;
  }();
  return pin >= 0 ? pin == 16 : count <= kEncRowMax;
}

// CRT of the two prime rows in ws into ciphertext words (k_crt_enc; the
// one-lane shape writes through LDS so its stores are whole lines)
template <class Sh, class MP2 = typename Sh::MP2>
void crt_enc_launch(const xhe_key* k, int64_t n, uint32_t* ws, uint32_t* ct, hipStream_t s) {
  const int blocks = (int)((n * MP2::TPI + 255) / 256);
  if constexpr (MP2::TPI == 1)
    hipLaunchKernelGGL((k_crt_enc_w<MP2, 2 * Sh::K / 32>), dim3(blocks), dim3(256), 0, s, k->kd, k->kd.p2.N, n, ws,
                       ct);
  else
    hipLaunchKernelGGL(k_crt_enc<MP2>, dim3(blocks), dim3(256), 0, s, k->kd, k->kd.p2.N, n, ws, ct);
  HIPCHK(hipGetLastError());
}

// lanes per element of k_djn_pmd: 16 up to 2 k elements, 4 up to 16 k, else
// 1 (the chip holds ~128 k one-lane residues: 2 waves x 1024 SIMDs x 64);
// $XHE_PMD_SPLIT pins it (1, 4 or 16)
int pmd_split(int64_t n) {
  static const int pin = [] {
    const char* e = getenv("XHE_PMD_SPLIT");
    return e ? atoi(e) : 0;
  }();
  if (pin == 1 || pin == 4 || pin == 16) return pin;
  return n <= 2048 ? 16 : n <= 16384 ? 4 : 1;
}

template <class Sh>
void encrypt_impl(const xhe_key* k, const uint32_t* m, const uint32_t* r, int64_t count, uint32_t* ct, hipStream_t s) {
  using MP2 = typename Sh::MP2;
  int64_t chunk = std::min<int64_t>(count, kChunk);
  uint32_t* ws = nullptr;
  ws_alloc((void**)&ws, (size_t)2 * 2 * MP2::S4 * chunk * sizeof(uint32_t), s);
  uint2* xst = nullptr;  // k_djn_pmdx workspaces (allocated on first use)
  uint32_t *xrows = nullptr, *xwords = nullptr;
  for (int64_t off = 0; off < count; off += chunk) {
    int64_t n = std::min(chunk, count - off);
    int blocks = (int)((n * MP2::TPI + 255) / 256);
#if XHE_PMD && XHE_LDS_ROWS
    if constexpr (Sh::K == 2048) {
      if (k->kd.pmd) {
        ProfScope ps("k_djn_pmd", s);
        // small batches split each element's windows over G lanes (latency:
        // ~nwin/G + log2 G dependent products instead of nwin)
        const int G = pmd_split(n);
        const dim3 grid((unsigned)((n * G + 127) / 128), 2);
        auto launch = [&](auto kern) {
          hipLaunchKernelGGL(kern, grid, dim3(128), 0, s, k->kd, k->kd.p.N, k->kd.q.N, k->kd.p2.N, k->kd.q2.N,
                             m + (size_t)off * k->nw, r + (size_t)off * k->rand_words, k->rand_words, n, ws);
        };
        if (G == 16) launch(k_djn_pmd<MP2, 37, Sh::RW, 16>);
        else if (G == 4) launch(k_djn_pmd<MP2, 37, Sh::RW, 4>);
        else launch(k_djn_pmd<MP2, 37, Sh::RW, 1>);
        HIPCHK(hipGetLastError());
        crt_enc_launch<Sh>(k, n, ws, ct + (size_t)off * k->n2w, s);
        continue;
      }
    }
#endif
#if XHE_PMDX
    if constexpr (Sh::K == 3072 || Sh::K == 4096 || Sh::K == 8192) {
      if (k->kd.pmdx) {
        using D = typename Sh::PDX;
        if (!xst) {
          ws_alloc((void**)&xst, (size_t)2 * D::K * chunk * sizeof(uint2), s);
          ws_alloc((void**)&xrows, (size_t)2 * 2 * Sh::PDXO::MN::S4 * chunk * sizeof(uint32_t), s);
          ws_alloc((void**)&xwords, (size_t)2 * chunk * Sh::RW * sizeof(uint32_t), s);
        }
        const dim3 g4((unsigned)((n * D::TPI + 127) / 128), 2);
        {
          ProfScope ps("k_djn_pmdx", s);
          hipLaunchKernelGGL((k_djn_pmdx<D, Sh::RW>), g4, dim3(128), 0, s, k->kd, r + (size_t)off * k->rand_words,
                             k->rand_words, n, xst);
          HIPCHK(hipGetLastError());
        }
        using DO = typename Sh::PDXO;  // the same state layout ([pair][count]) whatever the lanes per element
        hipLaunchKernelGGL((k_pmdx_enc_out<DO, Sh::RW>), dim3((unsigned)((n * DO::TPI + 127) / 128), 2), dim3(128), 0,
                           s, k->kd, m + (size_t)off * k->nw, n, xst, xrows, xwords);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(k_words_to_rows<MP2>, dim3((unsigned)((n * MP2::TPI + 255) / 256), 2), dim3(256), 0, s,
                           xwords, Sh::RW, n, ws);
        HIPCHK(hipGetLastError());
        crt_enc_launch<Sh>(k, n, ws, ct + (size_t)off * k->n2w, s);
        continue;
      }
    }
#endif
    if (enc_row(n)) {
      // small batch: one 16-lane DPP row per residue (latency-bound regime)
      using MX = typename Sh::MP2X;
      hipLaunchKernelGGL((k_djn_pow_x<MX, MP2::S4, Sh::RW>), dim3((unsigned)((n * MX::TPI + 255) / 256), 2), dim3(256), 0, s,
                         k->kd, m + (size_t)off * k->nw, r + (size_t)off * k->rand_words, k->rand_words, n, ws);
      HIPCHK(hipGetLastError());
    } else {
      // labelled by the kernel rocprof shows (k_djn_pow_lds / k_djn_pow)
      ProfScope ps(XHE_LDS_ROWS && MP2::TPI == 1 ? "k_djn_pow_lds" : "k_djn_pow", s);
#if XHE_LDS_ROWS
      if constexpr (MP2::TPI == 1) {
        const dim3 grid((unsigned)((n + 127) / 128), 2);
        hipLaunchKernelGGL((k_djn_pow_lds<MP2, Sh::RW>), grid, dim3(128), 0, s, k->kd,
                           k->kd.p2.N, k->kd.q2.N, m + (size_t)off * k->nw, r + (size_t)off * k->rand_words,
                           k->rand_words, n, ws);
      } else
#endif
      hipLaunchKernelGGL((k_djn_pow<MP2, Sh::RW>), dim3(blocks, 2), dim3(256), 0, s, k->kd, k->kd.p2.N, k->kd.q2.N,
                         m + (size_t)off * k->nw,
                         r + (size_t)off * k->rand_words, k->rand_words, n, ws);
      HIPCHK(hipGetLastError());
    }
    crt_enc_launch<Sh>(k, n, ws, ct + (size_t)off * k->n2w, s);
  }
  ws_free(ws, s);
  if (xst) {
    ws_free(xst, s);
    ws_free(xrows, s);
    ws_free(xwords, s);
  }
}

// grid for per-group-workspace (grid-stride) kernels
template <class M_>
int pow_grid(int64_t count, int cap_blocks) {
  return (int)std::min<int64_t>((count * M_::TPI + 255) / 256, cap_blocks);
}

template <class Sh>
void encrypt_pub_djn_impl(const xhe_key* k, const uint32_t* m, const uint32_t* r, int64_t count, uint32_t* ct,
                          hipStream_t s) {
#if XHE_NDIG
  if constexpr (Sh::K == 2048) {
    if (k->kd.pub_nd) {
      // fixed-base products in Montgomery digits of n (k_djn_pub_nd), then
      // (1 + n m) folded in base n on the way out (k_ndig_out)
      using D = PMDX<80, 4>;  // ND2048
      const int64_t chunk = std::min<int64_t>(count, kChunk);
      uint2* st = nullptr;
      uint32_t* rows = nullptr;
      ws_alloc((void**)&st, (size_t)D::K * chunk * sizeof(uint2), s);
      ws_alloc((void**)&rows, (size_t)2 * D::MN::S4 * chunk * sizeof(uint32_t), s);
      for (int64_t off = 0; off < count; off += chunk) {
        const int64_t n = std::min(chunk, count - off);
        const int eb = (int)((n * D::TPI + 127) / 128);
        {
          ProfScope ps("k_djn_pub", s);
          hipLaunchKernelGGL((k_djn_pub_nd<D, Sh::RW2>), dim3(eb), dim3(128), 0, s, k->kd,
                             r + (size_t)off * k->rand_words, k->rand_words, n, st);
          HIPCHK(hipGetLastError());
        }
        hipLaunchKernelGGL((k_ndig_out<D, true>), dim3(eb), dim3(128), 0, s, k->kd, st, m + (size_t)off * k->nw, n,
                           ct + (size_t)off * k->n2w, rows);
        HIPCHK(hipGetLastError());
      }
      ws_free(st, s);
      ws_free(rows, s);
      return;
    }
  }
#endif
  using MN2 = typename Sh::MN2;
  int64_t chunk = std::min<int64_t>(count, kChunk);
  uint32_t* ws = nullptr;
  ws_alloc((void**)&ws, (size_t)MN2::S4 * chunk * sizeof(uint32_t), s);
  for (int64_t off = 0; off < count; off += chunk) {
    int64_t n = std::min(chunk, count - off);
    int blocks = (int)((n * MN2::TPI + 255) / 256);
    ProfScope ps("k_djn_pub", s);
    hipLaunchKernelGGL((k_djn_pub<MN2, Sh::RW2>), dim3(blocks), dim3(256), 0, s, k->kd, k->kd.n2.N, m + (size_t)off * k->nw,
                       r + (size_t)off * k->rand_words, k->rand_words, n, ws, ct + (size_t)off * k->n2w);
    HIPCHK(hipGetLastError());
  }
  ws_free(ws, s);
}

#if XHE_NDIG
using ND2048 = PMDX<80, 4>;
// $XHE_NDIG=0: the Montgomery mod-n^2 kernels instead (A/B measurement)
bool ndig_on() {
  static const bool on = [] {
    const char* e = getenv("XHE_NDIG");
    return !(e && e[0] == '0');
  }();
  return on;
}
// in -> exponentiation -> out over chunks of up to kChunk elements; the
// exponentiation runs grid-stride over at most 1024 blocks (32 element groups
// each, one digit table per group slot)
template <class IN, class POW, class OUT>
void ndig_run(int64_t count, hipStream_t s, IN&& in, POW&& pw, OUT&& out) {
  using D = ND2048;
  const int64_t chunk = std::min<int64_t>(count, kChunk);
  const int pblocks = (int)std::min<int64_t>((chunk + NdigWs<D>::GPB - 1) / NdigWs<D>::GPB, 1024);
  uint2 *st = nullptr, *tab = nullptr;
  uint32_t* rows = nullptr;
  ws_alloc((void**)&st, (size_t)D::K * chunk * sizeof(uint2), s);
  ws_alloc((void**)&tab, NdigWs<D>::tab_bytes_per_slot() * (size_t)pblocks * NdigWs<D>::GPB, s);
  ws_alloc((void**)&rows, (size_t)2 * D::MN::S4 * chunk * sizeof(uint32_t), s);
  for (int64_t off = 0; off < count; off += chunk) {
    const int64_t n = std::min(chunk, count - off);
    const int eblocks = (int)((n * D::TPI + 127) / 128);
    in(eblocks, off, n, st);
    HIPCHK(hipGetLastError());
    pw(std::min<int>(pblocks, (int)((n + NdigWs<D>::GPB - 1) / NdigWs<D>::GPB)), off, n, st, tab);
    HIPCHK(hipGetLastError());
    out(eblocks, off, n, st, rows);
    HIPCHK(hipGetLastError());
  }
  ws_free(st, s);
  ws_free(tab, s);
  ws_free(rows, s);
}
#endif

#if XHE_PMD && XHE_LDS_ROWS
// $XHE_NODJN_PMD=0: the Montgomery k_nodjn_crt instead (A/B measurement)
bool nodjn_pmd_on() {
  static const bool on = [] {
    const char* e = getenv("XHE_NODJN_PMD");
    return !(e && e[0] == '0');
  }();
  return on;
}

// Private non-DJN encryption of 2048-bit keys in Montgomery digits: r mod
// P^2 -> digits (k_dec_pmd_in), r^(e_P) by the decrypt's digit
// exponentiation (k_dec_pmd_pow, the exponent e_P = n mod phi(P^2) shared by
// every lane), (1 + n m) folded in on the way out (k_nodjn_pmd_out), CRT.
template <class Sh>
void encrypt_nodjn_pmd(const xhe_key* k, const uint32_t* m, const uint32_t* r, int64_t count, uint32_t* ct,
                       hipStream_t s) {
  using MP2 = typename Sh::MP2;
  constexpr int NQ = PMD<37>::NQ;
  const int64_t chunk = std::min<int64_t>(count, kChunk);
  const int pow_blocks = (int)std::min<int64_t>((chunk + 127) / 128, 1024);
  const int64_t lanes = (int64_t)pow_blocks * 128;
  uint4 *ws = nullptr, *st = nullptr;
  uint32_t* rows = nullptr;
  ws_alloc((void**)&ws, (size_t)2 * 16 * NQ * lanes * sizeof(uint4), s);
  ws_alloc((void**)&st, (size_t)2 * NQ * chunk * sizeof(uint4), s);
  ws_alloc((void**)&rows, (size_t)2 * 2 * MP2::S4 * chunk * sizeof(uint32_t), s);
  for (int64_t off = 0; off < count; off += chunk) {
    const int64_t n = std::min(chunk, count - off);
    const dim3 g1((unsigned)((n + 127) / 128), 2);
    hipLaunchKernelGGL((k_dec_pmd_in<MP2, 37>), g1, dim3(128), 0, s, k->kd, k->kd.p.N, k->kd.q.N, k->kd.p2.N,
                       k->kd.q2.N, r + (size_t)off * k->rand_words, k->rand_words, n, st);
    HIPCHK(hipGetLastError());
    {
      ProfScope ps("k_nodjn_crt", s);
      hipLaunchKernelGGL((k_dec_pmd_pow<37>), dim3((unsigned)std::min<int64_t>((n + 127) / 128, pow_blocks), 2),
                         dim3(128), 0, s, k->kd, k->kd.p.N, k->kd.q.N, 1, n, st, ws);
      HIPCHK(hipGetLastError());
    }
    hipLaunchKernelGGL((k_nodjn_pmd_out<MP2, 37>), g1, dim3(128), 0, s, k->kd, k->kd.p.N, k->kd.q.N, k->kd.p2.N,
                       k->kd.q2.N, m + (size_t)off * k->nw, n, st, rows);
    HIPCHK(hipGetLastError());
    crt_enc_launch<Sh>(k, n, rows, ct + (size_t)off * k->n2w, s);
  }
  ws_free(ws, s);
  ws_free(st, s);
  ws_free(rows, s);
}
#endif

template <class Sh>
void encrypt_nodjn_impl(const xhe_key* k, const uint32_t* m, const uint32_t* r, int64_t count, uint32_t* ct,
                        hipStream_t s) {
#if XHE_PMD && XHE_LDS_ROWS
  if constexpr (Sh::K == 2048) {
    if (k->priv && nodjn_pmd_on()) {
      encrypt_nodjn_pmd<Sh>(k, m, r, count, ct, s);
      return;
    }
  }
#endif
  if (k->priv) {
    using MP2 = typename Sh::MP2;
    // 2-lane batch shapes (3072 bits, 55 limbs per lane) spill in this
    // variable-base exponentiation (9.7 k enc/s): run it in the 4-lane shape.
    constexpr bool wide = MP2::TPI == 2;
    using MPE = std::conditional_t<wide, typename Sh::MP2L, MP2>;
    int64_t chunk = std::min<int64_t>(count, kChunk);
    int pb = pow_grid<MPE>(chunk, 512);
    int64_t groups = (int64_t)pb * 256 / MPE::TPI;
    uint32_t *ws = nullptr, *rows = nullptr;
    ws_alloc((void**)&ws, (size_t)2 * 18 * MPE::S4 * groups * sizeof(uint32_t), s);
    ws_alloc((void**)&rows, (size_t)2 * 2 * MP2::S4 * chunk * sizeof(uint32_t), s);
    for (int64_t off = 0; off < count; off += chunk) {
      int64_t n = std::min(chunk, count - off);
      {
        ProfScope ps("k_nodjn_crt", s);
        const ModDev& mp = wide ? k->kd.p2L : k->kd.p2;
        const ModDev& mq = wide ? k->kd.q2L : k->kd.q2;
        hipLaunchKernelGGL((k_nodjn_crt<MPE, wide ? 1 : 0, MP2::S4>), dim3(pb, 2), dim3(256), 0, s, k->kd, mp.N, mq.N,
                           m + (size_t)off * k->nw, r + (size_t)off * k->rand_words, k->rand_words, n, rows, ws);
        HIPCHK(hipGetLastError());
      }
      crt_enc_launch<Sh>(k, n, rows, ct + (size_t)off * k->n2w, s);
    }
    ws_free(ws, s);
    ws_free(rows, s);
  } else {
#if XHE_NDIG
    if constexpr (Sh::K == 2048) {
      if (k->kd.ndig && ndig_on()) {
        ndig_run(
            count, s,
            [&](int b, int64_t off, int64_t n, uint2* st) {
              hipLaunchKernelGGL((k_ndig_in<ND2048, false>), dim3(b), dim3(128), 0, s, k->kd,
                                 r + (size_t)off * k->rand_words, k->rand_words, n, st);
            },
            [&](int b, int64_t, int64_t n, uint2* st, uint2* tab) {
              ProfScope ps("k_nodjn_pub", s);
              hipLaunchKernelGGL(k_ndig_pow_n<ND2048>, dim3(b), dim3(128), 0, s, k->kd, n, st, tab);
            },
            [&](int b, int64_t off, int64_t n, uint2* st, uint32_t* rows) {
              hipLaunchKernelGGL((k_ndig_out<ND2048, true>), dim3(b), dim3(128), 0, s, k->kd, st,
                                 m + (size_t)off * k->nw, n, ct + (size_t)off * k->n2w, rows);
            });
        return;
      }
    }
#endif
    using MN2 = typename Sh::MN2;
    int64_t chunk = std::min<int64_t>(count, kChunk);
    int pb = pow_grid<MN2>(chunk, 512);
    int64_t groups = (int64_t)pb * 256 / MN2::TPI;
    uint32_t* ws = nullptr;
    ws_alloc((void**)&ws, (size_t)18 * MN2::S4 * groups * sizeof(uint32_t), s);
    for (int64_t off = 0; off < count; off += chunk) {
      int64_t n = std::min(chunk, count - off);
      ProfScope ps("k_nodjn_pub", s);
      hipLaunchKernelGGL(k_nodjn_pub<MN2>, dim3(pb), dim3(256), 0, s, k->kd, k->kd.n2.N, m + (size_t)off * k->nw,
                         r + (size_t)off * k->rand_words, k->rand_words, n, ct + (size_t)off * k->n2w, ws);
      HIPCHK(hipGetLastError());
    }
    ws_free(ws, s);
  }
}

// n^2 constants of the MN2 shape (see n2dev in xhe_kernels.hpp).
template <class MN2>
const ModDev& n2h(const xhe_key* k) {
  if constexpr (MN2::TPI == 16) return k->kd.n2X;
  else return k->kd.n2;
}

// Shape of the n^2 ciphertext ops by batch size: one 16-lane DPP row per
// residue up to kN2RowMax elements (latency-bound: a few ciphertexts leave the
// chip idle and each element's chain of dependent products sets the time),
// 4 lanes beyond. $XHE_N2_TPI (4 or 16) pins one shape (A/B measurement).
constexpr int64_t kN2RowMax = 4096;
bool n2_row(int64_t count) {
  static const int pin = [] {
    const char* e = std::getenv("XHE_N2_TPI");
    int t = e ? std::atoi(e) : 0;
    return (t == 4 || t == 16) ? t : 0;
  }();
  return pin ? pin == 16 : count <= kN2RowMax;
}

// Adds of a few elements run one 16-wave block per element (k_mulmod_wave,
// 2048-bit keys) up to kWaveAddMax elements, with or without alignment
// squarings (kWaveAddMinD: the plain product of the LR step's noise add, 15
// elements, took 56 us in the 16-lane k_mulmod_n2). $XHE_ADD_WAVE=0 keeps
// the lane shapes (A/B).
constexpr int64_t kWaveAddMax = 256;
constexpr int kWaveAddMinD = 0;
bool add_wave_on() {
  static const bool on = [] {
    const char* e = getenv("XHE_ADD_WAVE");
    return !(e && e[0] == '0');
  }();
  return on;
}


// Equal-exponent adds of 2048-bit ciphertexts in the 4-lane regime run the
// one-product Barrett kernel (k_add_barrett); $XHE_ADD_BAR=0 keeps the
// Montgomery pair (k_mulmod_n2) for the A/B.
bool add_bar_on() {
  static const bool on = [] {
    const char* e = getenv("XHE_ADD_BAR");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <class Sh, class MN2 = typename Sh::MN2>
void mulmod_impl(const xhe_key* k, const uint32_t* a, const int32_t* ea, const uint32_t* b, const int32_t* eb,
                 int64_t count, int dmax, uint32_t* out, int32_t* eout, hipStream_t s) {
  if constexpr (Sh::K == 2048) {
    if (count <= kWaveAddMax && dmax >= kWaveAddMinD && add_wave_on()) {
      hipLaunchKernelGGL((k_mulmod_wave<154, 16>), dim3((unsigned)count), dim3(1024), 0, s, k->kd, a, ea, b, eb, count,
                         out, eout);
      HIPCHK(hipGetLastError());
      return;
    }
  }
  if constexpr (Sh::K == 2048 && MN2::TPI == 4) {
    if (dmax == 0 && add_bar_on()) {
      ProfScope ps("k_add_barrett", s);
      const int64_t blocks = (count + bar::EPB - 1) / bar::EPB;
      hipLaunchKernelGGL(k_add_barrett, dim3((unsigned)blocks), dim3(bar::TPB), 0, s, k->kd, a, ea, b, eb, count, out,
                         eout);
      HIPCHK(hipGetLastError());
      return;
    }
  }
  int64_t chunk = std::min<int64_t>(count, kChunk);
  uint32_t* ws = nullptr;
  ws_alloc((void**)&ws, (size_t)2 * MN2::S4 * chunk * sizeof(uint32_t), s);
  for (int64_t off = 0; off < count; off += chunk) {
    int64_t n = std::min(chunk, count - off);
    int blocks = (int)((n * MN2::TPI + 255) / 256);
    hipLaunchKernelGGL(k_mulmod_n2<MN2>, dim3(blocks), dim3(256), 0, s, k->kd, n2h<MN2>(k).N, a + (size_t)off * k->n2w,
                       ea ? ea + off : nullptr, b + (size_t)off * k->n2w, eb ? eb + off : nullptr, n, dmax,
                       out + (size_t)off * k->n2w, eout ? eout + off : nullptr, ws);
    HIPCHK(hipGetLastError());
  }
  ws_free(ws, s);
}

template <class Sh, class MN2 = typename Sh::MN2>
void powmod_impl(const xhe_key* k, const uint32_t* c, const uint32_t* kw_, int kw, int kbits, int64_t count,
                 uint32_t* out, hipStream_t s) {
#if XHE_NDIG
  if constexpr (Sh::K == 2048 && MN2::TPI == 4) {
    if (k->kd.ndig && ndig_on()) {
      ndig_run(
          count, s,
          [&](int b, int64_t off, int64_t n, uint2* st) {
            hipLaunchKernelGGL((k_ndig_in<ND2048, true>), dim3(b), dim3(128), 0, s, k->kd, c + (size_t)off * k->n2w,
                               k->n2w, n, st);
          },
          [&](int b, int64_t off, int64_t n, uint2* st, uint2* tab) {
            ProfScope ps("k_powmod_n2", s);
            hipLaunchKernelGGL(k_ndig_pow_k<ND2048>, dim3(b), dim3(128), 0, s, k->kd, kw_ + (size_t)off * kw, kw,
                               kbits, n, st, tab);
          },
          [&](int b, int64_t off, int64_t n, uint2* st, uint32_t* rows) {
            hipLaunchKernelGGL((k_ndig_out<ND2048, false>), dim3(b), dim3(128), 0, s, k->kd, st, nullptr, n,
                               out + (size_t)off * k->n2w, rows);
          });
      return;
    }
  }
#endif
  int64_t chunk = std::min<int64_t>(count, kChunk);
  int pb = pow_grid<MN2>(chunk, 512);
  int64_t groups = (int64_t)pb * 256 / MN2::TPI;
  uint32_t* ws = nullptr;
  ws_alloc((void**)&ws, (size_t)17 * MN2::S4 * groups * sizeof(uint32_t), s);
  for (int64_t off = 0; off < count; off += chunk) {
    int64_t n = std::min(chunk, count - off);
    ProfScope ps("k_powmod_n2", s);
    hipLaunchKernelGGL(k_powmod_n2<MN2>, dim3(pb), dim3(256), 0, s, k->kd, n2h<MN2>(k).N, c + (size_t)off * k->n2w,
                       kw_ + (size_t)off * kw, kw, kbits, n, out + (size_t)off * k->n2w, ws);
    HIPCHK(hipGetLastError());
  }
  ws_free(ws, s);
}

// Batch inversion mod n^2 via a product tree (Montgomery's trick in parallel).
template <class Sh, class MN2 = typename Sh::MN2>
int invert_impl(const xhe_key* k, const uint32_t* c, int64_t count, uint32_t* out, hipStream_t s) {
  const int S4 = MN2::S4;
  std::vector<int64_t> sizes{count};
  while (sizes.back() > 1) sizes.push_back((sizes.back() + 1) / 2);
  std::vector<size_t> offs;
  size_t tot = 0;
  for (auto n : sizes) {
    offs.push_back(tot);
    tot += (size_t)S4 * n;
  }
  if constexpr (Sh::K == 2048 && MN2::TPI == 16) {  // (a 1024-thread block: the 16-lane 2048-bit shape's registers)
  if (count <= 256) {
    // small batch: a product tree of whole-block products (dec_wave.hpp
    // k_wtree_*), one launch per level
    constexpr int KW = 154;
    std::vector<int64_t> woff;
    int64_t wtot = 0;
    for (auto n : sizes) {
      woff.push_back(wtot);
      wtot += n;
    }
    const int nlev = (int)sizes.size();
    uint32_t *lv = nullptr, *inv = nullptr, *wds = nullptr;
    HIPCHK(hipMallocAsync((void**)&lv, (size_t)wtot * KW * 4, s));
    HIPCHK(hipMallocAsync((void**)&inv, (size_t)wtot * KW * 4, s));
    HIPCHK(hipMallocAsync((void**)&wds, (size_t)2 * k->n2w * 4, s));
    auto node = [&](uint32_t* b, int l) { return b + (size_t)woff[l] * KW; };
    hipLaunchKernelGGL((k_wtree_in<KW, 16>), dim3((unsigned)count), dim3(1024), 0, s, k->kd, c, lv);
    HIPCHK(hipGetLastError());
    for (int l = 1; l < nlev; ++l) {
      hipLaunchKernelGGL((k_wtree_up<KW, 16>), dim3((unsigned)sizes[l]), dim3(1024), 0, s, k->kd, node(lv, l - 1),
                         sizes[l - 1], node(lv, l));
      HIPCHK(hipGetLastError());
    }
    hipLaunchKernelGGL((k_wtree_out<KW, 16>), dim3(1), dim3(1024), 0, s, k->kd, node(lv, nlev - 1), wds);
    HIPCHK(hipGetLastError());
    std::vector<uint32_t> root(k->n2w), yinv(k->n2w);
    HIPCHK(hipMemcpyAsync(root.data(), wds, (size_t)k->n2w * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (!modinv_words(root.data(), k->n2_host.data(), k->n2w, yinv.data())) {
      (void)hipFreeAsync(lv, s);
      (void)hipFreeAsync(inv, s);
      (void)hipFreeAsync(wds, s);
      return fail(XHE_ENOINV, "invert(a, b) no inverse exists");
    }
    HIPCHK(hipMemcpyAsync(wds + k->n2w, yinv.data(), (size_t)k->n2w * 4, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL((k_wtree_in<KW, 16>), dim3(1), dim3(1024), 0, s, k->kd, wds + k->n2w, node(inv, nlev - 1));
    HIPCHK(hipGetLastError());
    for (int l = nlev - 2; l >= 0; --l) {
      hipLaunchKernelGGL((k_wtree_down<KW, 16>), dim3((unsigned)sizes[l]), dim3(1024), 0, s, k->kd, node(inv, l + 1),
                         node(lv, l), sizes[l], node(inv, l));
      HIPCHK(hipGetLastError());
    }
    hipLaunchKernelGGL((k_wtree_out<KW, 16>), dim3((unsigned)count), dim3(1024), 0, s, k->kd, inv, out);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));  // yinv is host memory of this frame
    (void)hipFreeAsync(lv, s);
    (void)hipFreeAsync(inv, s);
    (void)hipFreeAsync(wds, s);
    return XHE_OK;
  }
  }
  uint32_t *lv = nullptr, *inv = nullptr, *scr = nullptr;
  int32_t* st = nullptr;
  HIPCHK(hipMallocAsync((void**)&lv, tot * 4, s));
  HIPCHK(hipMallocAsync((void**)&inv, tot * 4, s));
  HIPCHK(hipMallocAsync((void**)&scr, (size_t)(4 * (k->n2w + 1) + 2 * k->n2w + 8) * 4, s));
  HIPCHK(hipMallocAsync((void**)&st, 4, s));
  auto blocks = [&](int64_t n) { return dim3((unsigned)((n * MN2::TPI + 255) / 256)); };
  hipLaunchKernelGGL(k_to_mont_rows<MN2>, blocks(count), dim3(256), 0, s, k->kd, n2h<MN2>(k).N, c, count, lv);
  HIPCHK(hipGetLastError());
  for (size_t l = 1; l < sizes.size(); ++l) {
    hipLaunchKernelGGL(k_tree_up<MN2>, blocks(sizes[l]), dim3(256), 0, s, k->kd, n2h<MN2>(k).N, lv + offs[l - 1],
                       sizes[l - 1], lv + offs[l], sizes[l]);
    HIPCHK(hipGetLastError());
  }
  size_t top = offs.back();
  uint32_t* y_words = scr + 4 * (k->n2w + 1);
  uint32_t* r_words = y_words + k->n2w;
  hipLaunchKernelGGL(k_row_pack<MN2>, dim3(1), dim3(64), 0, s, k->kd, n2h<MN2>(k).N, lv + top, r_words);
  HIPCHK(hipGetLastError());
  // The one scalar inverse of the batch (the tree root, (prod c_i) R) is a
  // sequential extended Euclid: ~1 ms on a host core vs a single GPU lane's
  // tens of milliseconds. Everything per element stays on the device.
  std::vector<uint32_t> root(k->n2w), yinv(k->n2w);
  HIPCHK(hipMemcpyAsync(root.data(), r_words, (size_t)k->n2w * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (!modinv_words(root.data(), k->n2_host.data(), k->n2w, yinv.data())) {
    (void)hipFree(lv);
    (void)hipFree(inv);
    (void)hipFree(scr);
    (void)hipFree(st);
    return fail(XHE_ENOINV, "invert(a, b) no inverse exists");
  }
  HIPCHK(hipMemcpyAsync(y_words, yinv.data(), (size_t)k->n2w * 4, hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_inv_to_row<MN2>, dim3(1), dim3(64), 0, s, k->kd, n2h<MN2>(k).N, y_words, inv + top);
  HIPCHK(hipGetLastError());
  for (size_t l = sizes.size() - 1; l >= 1; --l) {
    hipLaunchKernelGGL(k_tree_down<MN2>, blocks(sizes[l - 1]), dim3(256), 0, s, k->kd, n2h<MN2>(k).N, inv + offs[l],
                       sizes[l], lv + offs[l - 1], sizes[l - 1], inv + offs[l - 1]);
    HIPCHK(hipGetLastError());
  }
  hipLaunchKernelGGL(k_from_mont_rows<MN2>, blocks(count), dim3(256), 0, s, k->kd, n2h<MN2>(k).N, inv, count, out);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s));
  (void)hipFree(lv);
  (void)hipFree(inv);
  (void)hipFree(scr);
  (void)hipFree(st);
  return XHE_OK;
}

// Small host -> device uploads made while enqueuing (the segment plans):
// copied into a pinned slot whose previous copy has completed (one event per
// slot), so the enqueue never waits for the stream. A pageable source would
// need the stream synchronised before the frame that owns it returns - which
// made every groupby sum wait for the previous call's kernels.
class HostStage {
  struct Slot {
    void* p = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    int dev = -1;
  };
  std::mutex mu_;
  std::vector<Slot> slots_;

 public:
  void upload(void* dst, const void* src, size_t n, hipStream_t s, int dev) {
    std::lock_guard<std::mutex> g(mu_);
    Slot* use = nullptr;
    for (Slot& sl : slots_)
      if (sl.dev == dev && sl.cap >= n && hipEventQuery(sl.ev) == hipSuccess) {
        use = &sl;
        break;
      }
    if (!use) {
      Slot sl;
      sl.dev = dev;
      sl.cap = std::max<size_t>(n, 64 << 10);
      HIPCHK(hipHostMalloc(&sl.p, sl.cap, hipHostMallocDefault));
      HIPCHK(hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming));
      slots_.push_back(sl);
      use = &slots_.back();
    }
    memcpy(use->p, src, n);
    HIPCHK(hipMemcpyAsync(dst, use->p, n, hipMemcpyHostToDevice, s));
    HIPCHK(hipEventRecord(use->ev, s));
  }
};
HostStage& host_stage() {
  static HostStage* st = new HostStage();  // process lifetime (no teardown order with the runtime)
  return *st;
}

// Reduce segment-ordered rows [S4][count] to one Montgomery row per segment
// (seg: nseg+1 offsets) by levels of k_chunk_prod (C rows per chunk). The
// input rows are Montgomery rows, or plain residues with raw = true (the
// first level then returns each chunk to Montgomery form). Takes ownership
// of `rows`; returns a new [S4][nseg] buffer (hipFree by the caller); an
// empty segment yields the Montgomery one.
template <class Sh, class MN2 = typename Sh::MN2>
uint32_t* reduce_segments(const xhe_key* k, uint32_t* rows, int64_t count, std::vector<int64_t> seg, hipStream_t s,
                          bool raw = false, const uint32_t* words = nullptr) {
  // words: raw input as ciphertext words ([count][n2w]) instead of rows
  // (the first level unpacks them itself; rows is then unused)
  const int S4 = MN2::S4;
  const int64_t nseg = (int64_t)seg.size() - 1;
  // Lane groups the chip holds at 2 waves per SIMD: while a level has at least
  // that many chunks of kRawChunk rows it is throughput-bound and takes long
  // chunks; above that the levels are latency-bound (a chunk is a chain of
  // dependent products), and chunks of 4 give the shortest chain in all
  // (log4 levels x 4 products, against log32 levels x 32).
  constexpr int64_t kFill = 131072 / MN2::TPI;
  auto blocks = [&](int64_t n) { return dim3((unsigned)std::max<int64_t>(1, (n * MN2::TPI + 255) / 256)); };
  // segments of one length (the mat-vec): the chunks are computed in the
  // kernel, no plan upload and no host sync
  bool uniform = nseg > 0;
  for (int64_t i = 1; i < nseg && uniform; ++i) uniform = seg[i + 1] - seg[i] == seg[1] - seg[0];
  uniform = uniform && seg[1] - seg[0] > 0;
  // plan every level on the host first: (first, stride, count) of every chunk
  // of every level go up in one copy, and the levels run back to back
  struct Level {
    size_t plan_off;
    int64_t n_in, n_out, seg_len, ncs;
    bool raw;
  };
  std::vector<int64_t> all;
  std::vector<Level> plan;
  int64_t n_cur = count;
  bool first = true;
  while (true) {
    bool ones = true;  // every segment is one row: nothing left to multiply
    for (int64_t i = 0; i < nseg; ++i)
      if (seg[i + 1] - seg[i] != 1) {
        ones = false;
        break;
      }
    if (ones && !(first && raw)) break;  // (plain rows still need Montgomery form)
    // the longest chunks that still leave kFill lane groups (4 .. kRawChunk):
    // a 100 k-row, 256-bin histogram took chunks of 32 on its first level (a
    // 33-product chain with a quarter of the chip busy) and now takes 4
    const int64_t C = std::max<int64_t>(4, std::min<int64_t>(kRawChunk, n_cur / kFill));
    std::vector<int64_t> nseg_b{0};
    const size_t off = all.size();
    int64_t seg_len = 0, ncs = 0;
    if (uniform) {
      seg_len = seg[1] - seg[0];
      ncs = (seg_len + C - 1) / C;
      for (int64_t i = 0; i < nseg; ++i) nseg_b.push_back(nseg_b.back() + ncs);
    } else {
      for (int64_t i = 0; i < nseg; ++i) {
        const int64_t len = seg[i + 1] - seg[i];
        const int64_t nch = std::max<int64_t>(1, (len + C - 1) / C);  // an empty segment: one (empty) chunk
        for (int64_t t = 0; t < nch; ++t) {
          all.push_back(seg[i] + t);
          all.push_back(nch);
          all.push_back(t < len ? (len - t + nch - 1) / nch : 0);
        }
        nseg_b.push_back(nseg_b.back() + nch);
      }
    }
    const int64_t n_out = nseg_b.back();
    plan.push_back({off, n_cur, n_out, seg_len, ncs, first && raw});
    n_cur = n_out;
    seg.swap(nseg_b);
    first = false;
  }
  if (plan.empty()) return rows;  // already one Montgomery row per segment
  int64_t* dplan = nullptr;
  if (!all.empty()) {
    HIPCHK(hipMallocAsync((void**)&dplan, all.size() * 8, s));
    host_stage().upload(dplan, all.data(), all.size() * 8, s, k->device);  // no host sync
  }
  uint32_t* cur = rows;
  for (const Level& L : plan) {
    uint32_t* nxt = nullptr;
    HIPCHK(hipMallocAsync((void**)&nxt, (size_t)S4 * std::max<int64_t>(L.n_out, 1) * 4, s));
    if (L.raw && words)
      hipLaunchKernelGGL((k_chunk_prod_words<MN2, Sh::RW2>), blocks(L.n_out), dim3(256), 0, s, k->kd,
                         n2h<MN2>(k).N, words, uniform ? nullptr : dplan + L.plan_off, L.seg_len, L.ncs, L.n_out, nxt);
    else
      hipLaunchKernelGGL(k_chunk_prod<MN2>, blocks(L.n_out), dim3(256), 0, s, k->kd, n2h<MN2>(k).N, cur, L.n_in,
                         uniform ? nullptr : dplan + L.plan_off, L.seg_len, L.ncs, L.n_out, nxt, L.raw ? 1 : 0);
    HIPCHK(hipGetLastError());
    if (cur) HIPCHK(hipFreeAsync(cur, s));
    cur = nxt;
  }
  if (dplan) HIPCHK(hipFreeAsync(dplan, s));
  return cur;
}

// Segmented modular product: out[s] = prod_{i in seg s} c_i^(2^d_i) mod n^2.
// seg_begin: nseg+1 offsets into the (already segment-ordered) inputs.
template <class Sh, class MN2 = typename Sh::MN2>
void segprod_impl(const xhe_key* k, const uint32_t* c, const int32_t* d, int dmax, int64_t count,
                  const int64_t* seg_begin_host, int64_t nseg, uint32_t* out, hipStream_t s) {
  const int S4 = MN2::S4;
  auto blocks = [&](int64_t n) { return dim3((unsigned)std::max<int64_t>(1, (n * MN2::TPI + 255) / 256)); };
  uint32_t *rows = nullptr, *sq = nullptr;
  // no alignment anywhere: the first level reads the ciphertext words itself
  // ($XHE_SUM_WORDS=0: the k_align_mont transpose first, A/B)
  static const bool words_on = [] {
    const char* e = getenv("XHE_SUM_WORDS");
    return !(e && e[0] == '0');
  }();
  const bool direct = count > 0 && (dmax == 0 || !d) && words_on;
  if (!direct) {
    HIPCHK(hipMallocAsync((void**)&rows, (size_t)S4 * std::max<int64_t>(count, 1) * 4, s));
    HIPCHK(hipMallocAsync((void**)&sq, (size_t)S4 * std::max<int64_t>(count, 1) * 4, s));
  }
  if (count > 0 && !direct) {
    hipLaunchKernelGGL(k_align_mont<MN2>, blocks(count), dim3(256), 0, s, k->kd, n2h<MN2>(k).N, c, d, count, dmax,
                       rows, sq);
    HIPCHK(hipGetLastError());
  }
  uint32_t* cur = reduce_segments<Sh, MN2>(
      k, rows, count, std::vector<int64_t>(seg_begin_host, seg_begin_host + nseg + 1), s, true, direct ? c : nullptr);
  hipLaunchKernelGGL(k_from_mont_rows<MN2>, blocks(nseg), dim3(256), 0, s, k->kd, n2h<MN2>(k).N, cur, nseg, out);
  HIPCHK(hipGetLastError());
  (void)hipFreeAsync(cur, s);  // stream-ordered: no host sync (the output is ready in stream order)
  if (sq) (void)hipFreeAsync(sq, s);
}

// Window bits for a multi-exponentiation: minimise table products
// nbases*(2^c - 2) plus gathered products ncols*nterms*ceil(kbits/c), with the
// tables capped at ~2 GiB.
int mexp_window(int64_t nbases, int64_t ncols, int64_t nterms, int kbits, int s4) {
  int best = 1;
  double best_cost = 1e300;
  for (int c = 1; c <= 8; ++c) {
    if (c > 1 && (double)(nbases << c) * s4 * 4 > 2147483648.0) break;
    double cost = (double)nbases * ((1 << c) - 2) + (double)ncols * nterms * ((kbits + c - 1) / c) +
                  (double)ncols * kbits;
    if (cost < best_cost) {
      best_cost = cost;
      best = c;
    }
  }
  return best;
}

// Multi-exponentiation out[j] = prod_t bases[idx[j][t]]^k[j][t] mod n^2.
template <class Sh, class MN2 = typename Sh::MN2>
void multiexp_impl(const xhe_key* k, const uint32_t* bases, int64_t nbases, const int32_t* idx, const uint32_t* kx,
                   int kw, int kbits, int64_t ncols, int64_t nterms, int c, uint32_t* out, hipStream_t s) {
  const int S4 = MN2::S4;
  auto blocks = [&](int64_t n) { return dim3((unsigned)std::max<int64_t>(1, (n * MN2::TPI + 255) / 256)); };
  const int nwin = std::max(1, (kbits + c - 1) / c);
  uint32_t *tab = nullptr, *rows = nullptr, *sq = nullptr;
  HIPCHK(hipMallocAsync((void**)&tab, ((size_t)nbases << c) * S4 * 4, s));
  {
    ProfScope ps("k_mexp_tab", s);
    // by levels of entries (c + 1 dependent products per base); one launch
    // per level
    for (int lvl = 1; lvl <= c; ++lvl) {
      const int64_t per = lvl <= 1 ? 1 : lvl < c ? ((int64_t)1 << (lvl - 1)) : ((int64_t)1 << (lvl - 1)) - 1;
      hipLaunchKernelGGL(k_mexp_tab_lvl<MN2>, blocks(nbases * per), dim3(256), 0, s, k->kd, n2h<MN2>(k).N, bases,
                         nbases, c, lvl, tab);
      HIPCHK(hipGetLastError());
    }
  }
  // enough lane groups to fill the chip, at least 2 terms per group
  const int64_t segs = ncols * nwin;
  const int64_t target_groups = 131072 / MN2::TPI;
  const int64_t chunk = std::max<int64_t>(2, std::min<int64_t>(64, (segs * nterms + target_groups - 1) / target_groups));
  const int64_t nchunks = (nterms + chunk - 1) / chunk;
  const int64_t n_out = segs * nchunks;
  HIPCHK(hipMallocAsync((void**)&rows, (size_t)S4 * n_out * 4, s));
  {
    ProfScope ps("k_mexp_gather", s);
    hipLaunchKernelGGL(k_mexp_gather<MN2>, blocks(n_out), dim3(256), 0, s, k->kd, n2h<MN2>(k).N, tab, c, idx, kx, kw,
                       nterms, nwin, nchunks, chunk, n_out, rows);
    HIPCHK(hipGetLastError());
  }
  std::vector<int64_t> seg(segs + 1);
  for (int64_t i = 0; i <= segs; ++i) seg[i] = i * nchunks;
  uint32_t* P = reduce_segments<Sh, MN2>(k, rows, n_out, std::move(seg), s);
  HIPCHK(hipMallocAsync((void**)&sq, (size_t)S4 * ncols * 4, s));
  {
    ProfScope ps("k_mexp_horner", s);
    bool wave = false;
    if constexpr (Sh::K == 2048 && MN2::TPI == 16) {
      // small batches: one 16-wave block per column (latency; k_mexp_horner_wave)
      static const bool on = [] {
        const char* e = getenv("XHE_MEXP_WAVE");
        return !(e && e[0] == '0');
      }();
      if (on && ncols <= 4096) {
        hipLaunchKernelGGL((k_mexp_horner_wave<154, 16>), dim3((unsigned)ncols), dim3(1024), 0, s, k->kd, P, nwin, c,
                           ncols, out);
        wave = true;
      }
    }
    if (!wave)
      hipLaunchKernelGGL(k_mexp_horner<MN2>, blocks(ncols), dim3(256), 0, s, k->kd, n2h<MN2>(k).N, P, nwin, c, ncols,
                         sq, out);
    HIPCHK(hipGetLastError());
  }
  (void)hipFreeAsync(tab, s);  // stream-ordered frees: no host sync
  (void)hipFreeAsync(P, s);
  (void)hipFreeAsync(sq, s);
}

template <class Sh>
void raw_encrypt_impl(const xhe_key* k, const uint32_t* m, int64_t count, uint32_t* ct, hipStream_t s) {
  using MP2 = typename Sh::MP2;
  int64_t chunk = std::min<int64_t>(count, kChunk);
  uint32_t* ws = nullptr;
  ws_alloc((void**)&ws, (size_t)2 * MP2::S4 * chunk * sizeof(uint32_t), s);
  for (int64_t off = 0; off < count; off += chunk) {
    int64_t n = std::min(chunk, count - off);
    int blocks = (int)((n * MP2::TPI + 255) / 256);
    hipLaunchKernelGGL(k_raw_enc<MP2>, dim3(blocks), dim3(256), 0, s, k->kd, m + (size_t)off * k->nw, n, ws,
                       ct + (size_t)off * k->n2w);
    HIPCHK(hipGetLastError());
  }
  ws_free(ws, s);
}

// Decrypt exponentiation shapes by batch size (latency- vs throughput-bound):
// one 16-lane DPP row per residue up to kDecRowMax elements, 4 lanes up to
// kDecQuadMax, one lane beyond (crossovers measured with tools/dec_shapes.py:
// 16 lanes 6.0 ms flat to 1 k elements, 8.9 ms at 4 k, 15.8 ms at 8 k vs
// 11.3/11.8/11.9 ms for 4 lanes; 4 lanes 20-21 ms at 16 k vs 36 ms for 1
// lane, 40 ms at 32 k vs 37 ms). $XHE_DEC_TPI (1, 4 or 16) pins one shape.
constexpr int64_t kDecRowMax = 5120;
// One 256-thread block per residue (k_dec_rns, 2048-bit keys) up to
// kDecWaveMax elements (tools/dec_shapes.py, profiles/r6: 1,024 elements
// 5.68 ms vs 6.11 ms in 16 lanes, 1,536 8.34 vs 6.13 ms); $XHE_DEC_TPI=64
// pins it.
constexpr int64_t kDecWaveMax = 1024;
constexpr int64_t kDecQuadMax = 28672;

int dec_tpi_override() {
  static const int v = [] {
    const char* e = std::getenv("XHE_DEC_TPI");
    int t = e ? std::atoi(e) : 0;
    return (t == 1 || t == 4 || t == 16 || t == 64) ? t : 0;
  }();
  return v;
}

template <class MP2S, int SHAPE, class MP2>
void dec_pow_launch(const xhe_key* k, const uint32_t* ct, int64_t n, int64_t chunk, uint32_t* xrows,
                    hipStream_t s) {
  int pow_blocks = (int)std::min<int64_t>((chunk * MP2S::TPI + 255) / 256, 512);
  int64_t groups = (int64_t)pow_blocks * 256 / MP2S::TPI;
  uint32_t* ws = nullptr;
  ws_alloc((void**)&ws, (size_t)2 * 17 * MP2S::S4 * groups * sizeof(uint32_t), s);
  const ModDev& mp = SHAPE == 2 ? k->kd.p2X : SHAPE == 1 ? k->kd.p2L : k->kd.p2;
  const ModDev& mq = SHAPE == 2 ? k->kd.q2X : SHAPE == 1 ? k->kd.q2L : k->kd.q2;
  {
    ProfScope ps("k_dec_pow", s);
    hipLaunchKernelGGL((k_dec_pow<MP2S, SHAPE>), dim3(pow_blocks, 2), dim3(256), 0, s, k->kd, mp.N, mq.N, ct, n,
                       (int)MP2::S4, xrows, ws);
    HIPCHK(hipGetLastError());
  }
  ws_free(ws, s);
}

#if XHE_PMD && XHE_LDS_ROWS
// one lane per residue, exponentiation in Montgomery digits (2048-bit keys)
template <class MP2>
void dec_pmd_launch(const xhe_key* k, const uint32_t* ct, int64_t n, int64_t chunk, uint32_t* xrows, hipStream_t s) {
  constexpr int NQ = PMD<37>::NQ;
  const int pow_blocks = (int)std::min<int64_t>((chunk + 127) / 128, 1024);
  const int64_t lanes = (int64_t)pow_blocks * 128;
  uint4 *ws = nullptr, *st = nullptr;
  ws_alloc((void**)&ws, (size_t)2 * 16 * NQ * lanes * sizeof(uint4), s);
  ws_alloc((void**)&st, (size_t)2 * NQ * chunk * sizeof(uint4), s);
  const dim3 g1((unsigned)((n + 127) / 128), 2);
  hipLaunchKernelGGL((k_dec_pmd_in<MP2, 37>), g1, dim3(128), 0, s, k->kd, k->kd.p.N, k->kd.q.N, k->kd.p2.N,
                     k->kd.q2.N, ct, k->n2w, n, st);
  HIPCHK(hipGetLastError());
  {
    ProfScope ps("k_dec_pow", s);
    hipLaunchKernelGGL((k_dec_pmd_pow<37>), dim3(pow_blocks, 2), dim3(128), 0, s, k->kd, k->kd.p.N, k->kd.q.N, 0, n,
                       st, ws);
    HIPCHK(hipGetLastError());
  }
  hipLaunchKernelGGL((k_dec_pmd_out<MP2, 37>), g1, dim3(128), 0, s, k->kd, k->kd.p.N, k->kd.q.N, k->kd.p2.N,
                     k->kd.q2.N, n, st, (int)MP2::S4, xrows);
  HIPCHK(hipGetLastError());
  ws_free(ws, s);
  ws_free(st, s);
}
#endif

#if XHE_PMDX
// $XHE_DEC_PMDX=0: the Montgomery decrypt shapes instead (A/B measurement)
bool dec_pmdx_on() {
  static const bool on = [] {
    const char* e = getenv("XHE_DEC_PMDX");
    return !(e && e[0] == '0');
  }();
  return on;
}

// 3072/4096-bit decrypt in Montgomery digits up to m_P (k_dec_pmdx_*, see
// xhe_kernels.hpp): writes mrows [prime][2 S4][count] as k_dec_fin does
template <class Sh>
void dec_pmdx_launch(const xhe_key* k, const uint32_t* ct, int64_t n, int64_t chunk, uint32_t* mrows,
                     hipStream_t s) {
  using DO = typename Sh::PDXO;  // conversions (register room)
  using DP = typename Sh::PDXP;  // the exponentiation
  using MP2L = typename Sh::MP2L;
  using MP = typename Sh::MP;
  constexpr int RW = Sh::RW, NWH = Sh::K / 64;
  constexpr int SCR = MP2L::S4 > DO::MN::S4 ? MP2L::S4 : DO::MN::S4;
  constexpr int GPB = 128 / DP::TPI;
  const int pow_blocks = (int)std::min<int64_t>((chunk + GPB - 1) / GPB, 1024);
  const int64_t gs = (int64_t)pow_blocks * GPB;
  uint32_t *words = nullptr, *scr = nullptr;
  uint2 *st = nullptr, *tab = nullptr;
  ws_alloc((void**)&words, (size_t)2 * chunk * RW * sizeof(uint32_t), s);
  ws_alloc((void**)&scr, (size_t)2 * SCR * chunk * sizeof(uint32_t), s);
  ws_alloc((void**)&st, (size_t)2 * DP::K * chunk * sizeof(uint2), s);
  ws_alloc((void**)&tab, (size_t)2 * 16 * DP::K * gs * sizeof(uint2), s);
  hipLaunchKernelGGL((k_p2_reduce_words<MP2L, RW>), dim3((unsigned)((n * MP2L::TPI + 255) / 256), 2), dim3(256), 0, s,
                     k->kd, ct, n, scr, words);
  HIPCHK(hipGetLastError());
  const dim3 go((unsigned)((n * DO::TPI + 127) / 128), 2);
  hipLaunchKernelGGL((k_dec_pmdx_in<DO, RW>), go, dim3(128), 0, s, k->kd, words, n, st);
  HIPCHK(hipGetLastError());
  {
    ProfScope ps("k_dec_pow", s);
    const int pb = (int)std::min<int64_t>((n + GPB - 1) / GPB, pow_blocks);
    hipLaunchKernelGGL(k_dec_pmdx_pow<DP>, dim3(pb, 2), dim3(128), 0, s, k->kd, n, st, tab);
    HIPCHK(hipGetLastError());
  }
  hipLaunchKernelGGL((k_dec_pmdx_out<DO, NWH>), go, dim3(128), 0, s, k->kd, n, st, scr, words);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_words_to_rows<MP>, dim3((unsigned)((n * MP::TPI + 255) / 256), 2), dim3(256), 0, s, words,
                     NWH, n, mrows);
  HIPCHK(hipGetLastError());
  ws_free(words, s);
  ws_free(scr, s);
  ws_free(st, s);
  ws_free(tab, s);
}
#endif

// $XHE_DEC_RNS=0: the small-batch 2048-bit decrypt on k_dec_wave (the
// WaveMont product) instead of k_dec_rns (A/B measurement)
bool dec_rns_on() {
  static const bool on = [] {
    const char* e = getenv("XHE_DEC_RNS");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <class Sh>
void decrypt_impl(const xhe_key* k, const uint32_t* ct, int64_t count, uint32_t* m, hipStream_t s) {
  using MP2 = typename Sh::MP2;
  using MP = typename Sh::MP;
  const int pin = dec_tpi_override();
  // Multi-lane key sizes take the 4-lane shape for every larger batch: at 3072
  // bits the 2-lane batch shape (55 limbs per lane) decrypted 25.5 k/s where
  // 4096 bits in 4 lanes reach 133 k/s (profiles/r1/keysizes/).
  constexpr bool wave_ok = Sh::K == 2048;
  const int tpi = pin ? (pin == 64 && !wave_ok ? 16 : pin)
                      : (wave_ok && count <= kDecWaveMax)          ? 64
                      : count <= kDecRowMax                        ? 16
                      : (count <= kDecQuadMax || MP2::TPI > 1) ? 4
                                                                   : 1;
  int64_t chunk = std::min<int64_t>(count, kChunk);
  uint32_t *xrows = nullptr, *mrows = nullptr;
  ws_alloc((void**)&xrows, (size_t)2 * MP2::S4 * chunk * sizeof(uint32_t), s);
  ws_alloc((void**)&mrows, (size_t)2 * 2 * MP::S4 * chunk * sizeof(uint32_t), s);
  for (int64_t off = 0; off < count; off += chunk) {
    int64_t n = std::min(chunk, count - off);
    const uint32_t* cto = ct + (size_t)off * k->n2w;
#if XHE_PMDX
    if constexpr (Sh::K == 3072 || Sh::K == 4096 || Sh::K == 8192) {
      if (k->kd.pmdx_dec && dec_pmdx_on() && (pin ? pin == 1 : tpi == 4)) {
        // batches: digits (the 16-lane shape keeps the small ones)
        dec_pmdx_launch<Sh>(k, cto, n, chunk, mrows, s);
        const int cblocks = (int)((n * MP::TPI + 255) / 256);
        hipLaunchKernelGGL(k_crt_dec<MP>, dim3(cblocks), dim3(256), 0, s, k->kd, k->kd.p.N, n, mrows,
                           m + (size_t)off * k->nw);
        HIPCHK(hipGetLastError());
        continue;
      }
    }
#endif
    if (tpi == 64) {
      if constexpr (wave_ok) {
        static_assert(MP2::S == 74 && MP2::W == 28, "k_dec_wave / k_dec_rns share the MP2 limbs");
        if (k->kd.rns && dec_rns_on()) {
          ProfScope ps("k_dec_rns", s);
          hipLaunchKernelGGL(k_dec_rns, dim3((unsigned)n, 2), dim3(rns::NT), 0, s, k->kd, cto, n, (int)MP2::S4, xrows);
          HIPCHK(hipGetLastError());
        } else {
          ProfScope ps("k_dec_wave", s);
          hipLaunchKernelGGL((k_dec_wave<74, XHE_DEC_NWV>), dim3((unsigned)n, 2), dim3(64 * XHE_DEC_NWV), 0, s, k->kd,
                             cto, n, (int)MP2::S4, xrows);
          HIPCHK(hipGetLastError());
        }
      }
    } else if (tpi == 16) dec_pow_launch<typename Sh::MP2X, 2, MP2>(k, cto, n, chunk, xrows, s);
    else if (tpi == 4) dec_pow_launch<typename Sh::MP2L, 1, MP2>(k, cto, n, chunk, xrows, s);
#if XHE_PMD && XHE_LDS_ROWS
    else if constexpr (Sh::K == 2048) dec_pmd_launch<MP2>(k, cto, n, chunk, xrows, s);
#endif
    else dec_pow_launch<MP2, 0, MP2>(k, cto, n, chunk, xrows, s);
    int blocks = (int)((n * MP::TPI + 255) / 256);
    hipLaunchKernelGGL((k_dec_fin<MP2, MP>), dim3(blocks, 2), dim3(256), 0, s, k->kd, k->kd.p.N, k->kd.q.N, n,
                       xrows, mrows);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(k_crt_dec<MP>, dim3(blocks), dim3(256), 0, s, k->kd, k->kd.p.N, n, mrows,
                       m + (size_t)off * k->nw);
    HIPCHK(hipGetLastError());
  }
  ws_free(xrows, s);
  ws_free(mrows, s);
}

template <class F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const HipError& e) {
    return fail(XHE_EHIP, e.what());
  } catch (const std::exception& e) {
    return fail(XHE_EINVAL, e.what());
  }
}

}  // namespace

int xhe_segprod(const xhe_key* key, const uint32_t* c_dev, const int32_t* d_dev, int dmax, int64_t count,
                const int64_t* seg_begin, int64_t nseg, uint32_t* out_dev, void* stream) {
  return guarded([&]() -> int {
    if (!key || !seg_begin || nseg <= 0 || (count > 0 && !c_dev) || !out_dev || dmax < 0)
      return fail(XHE_EINVAL, "xhe_segprod: bad argument");
    if (seg_begin[0] != 0 || seg_begin[nseg] != count) return fail(XHE_EINVAL, "xhe_segprod: bad segment offsets");
    for (int64_t i = 0; i < nseg; ++i)
      if (seg_begin[i + 1] < seg_begin[i]) return fail(XHE_EINVAL, "xhe_segprod: offsets must be non-decreasing");
    DevGuard dg(key->device);
    const bool row = n2_row(count);
    hipStream_t hs = (hipStream_t)stream;
    with_shape(key->K, [&](auto sh) {
      using Sh = decltype(sh);
      if (row) segprod_impl<Sh, typename Sh::MN2X>(key, c_dev, d_dev, dmax, count, seg_begin, nseg, out_dev, hs);
      else segprod_impl<Sh>(key, c_dev, d_dev, dmax, count, seg_begin, nseg, out_dev, hs);
    });
    return XHE_OK;
  });
}

namespace {
struct DevBuf {
  void* p = nullptr;
  DevBuf(size_t bytes, hipStream_t s) { HIPCHK(hipMallocAsync(&p, std::max<size_t>(bytes, 4), s)); }
  ~DevBuf() { (void)hipFree(p); }
  template <class T>
  T* as() const { return (T*)p; }
};
struct Stream {
  hipStream_t s = nullptr;
  Stream() { HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking)); }
  ~Stream() {
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
  }
};

// After a ciphertext add whose alignment gap reaches key->dneg: the
// reference's _decrease_exponent_to raises the operand of larger exponent to
// the scalar 1 << d through _raw_mul, whose negative branch (1 << d >=
// min_value_for_negative) gives c^(2^d - n) where the add kernel computed
// c^(2^d) (paillier.py:79-86, 173-187). out *= x^-n with x = that operand on
// those elements and 1 elsewhere: x^n by the per-element power, one batch
// inversion, one product. Only reached when dmax >= dneg (gaps of ~bitlen(n)
// exponent steps: precision=None values around 1e+-300).
template <class Sh, class MN2>
int mulmod_gap_fix(const xhe_key* k, const uint32_t* a, const int32_t* ea, const uint32_t* b, const int32_t* eb,
                   int64_t count, uint32_t* out, hipStream_t s) {
  const size_t cb = (size_t)k->n2w * 4;
  DevBuf x(count * cb, s), kx((size_t)count * k->nw * 4, s), z(count * cb, s), zi(count * cb, s), t(count * cb, s);
  hipLaunchKernelGGL(k_gap_pick, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, k->kd, a, ea, b, eb, count,
                     k->dneg, x.as<uint32_t>(), kx.as<uint32_t>());
  HIPCHK(hipGetLastError());
  powmod_impl<Sh, MN2>(k, x.as<uint32_t>(), kx.as<uint32_t>(), k->nw, k->n_bits, count, z.as<uint32_t>(), s);
  const int rc = invert_impl<Sh, MN2>(k, z.as<uint32_t>(), count, zi.as<uint32_t>(), s);
  if (rc != XHE_OK) return rc;
  mulmod_impl<Sh, MN2>(k, out, nullptr, zi.as<uint32_t>(), nullptr, count, 0, t.as<uint32_t>(), nullptr, s);
  HIPCHK(hipMemcpyAsync(out, t.p, count * cb, hipMemcpyDeviceToDevice, s));
  HIPCHK(hipStreamSynchronize(s));  // the DevBufs are freed on return
  return XHE_OK;
}

// The stream-ordered allocator (hipMallocAsync, the entry points'
// workspaces) returns freed memory to the device at each synchronisation by
// default (release threshold 0), so every synchronised call would map its
// workspaces afresh. Keep up to kPoolKeep bytes cached in the device's
// default pool instead (set once per device, at key creation) - small next to
// the tables, so HBM stays available to the caller (torch's allocator does not
// draw from this pool).
#ifndef XHE_POOL_KEEP_MB
#define XHE_POOL_KEEP_MB 2048
#endif
constexpr uint64_t kPoolKeep = (uint64_t)XHE_POOL_KEEP_MB << 20;
void keep_pool_memory(int device) {
  static std::mutex mu;
  static bool done[64] = {};
  std::lock_guard<std::mutex> g(mu);
  if (device < 0 || device >= 64 || done[device] || kPoolKeep == 0) return;
  hipMemPool_t pool;
  if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
    uint64_t keep = kPoolKeep;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
  }
  done[device] = true;
}

// Pinned staging ring for the host-buffer entry points. A copy between the
// device and pageable memory goes through the runtime's small bounce buffers
// (~10 GB/s) and holds the calling thread; from or into pinned memory it is
// one DMA at the link rate and asynchronous. One ring per device is kept for
// the process lifetime and grown on demand; a call that finds it in use by
// another thread gets a ring of its own. Slot b holds one chunk's parts
// (inputs and outputs) at fixed offsets.
class PinnedSlots {
 public:
  PinnedSlots(int device, int depth, const std::vector<size_t>& part_bytes) {
    size_t off = 0;
    for (size_t b : part_bytes) {
      off_.push_back(off);
      off += (b + 255) & ~(size_t)255;
    }
    slot_ = off;
    const size_t need = std::max<size_t>(slot_ * depth, 256);
    Ring& r = ring(device);
    lock_ = std::unique_lock<std::mutex>(r.mu, std::try_to_lock);
    if (lock_.owns_lock()) {
      if (r.bytes < need) {
        if (r.p) HIPCHK(hipHostFree(r.p));
        r.p = nullptr;
        r.bytes = 0;
        HIPCHK(hipHostMalloc((void**)&r.p, need, hipHostMallocDefault));
        r.bytes = need;
      }
      base_ = r.p;
    } else {
      HIPCHK(hipHostMalloc((void**)&own_, need, hipHostMallocDefault));
      base_ = own_;
    }
  }
  ~PinnedSlots() {
    if (own_) (void)hipHostFree(own_);
  }
  PinnedSlots(const PinnedSlots&) = delete;
  PinnedSlots& operator=(const PinnedSlots&) = delete;
  uint8_t* at(int b, int k) const { return base_ + (size_t)b * slot_ + off_[k]; }

 private:
  struct Ring {
    std::mutex mu;
    uint8_t* p = nullptr;
    size_t bytes = 0;
  };
  static Ring& ring(int device) {
    static Ring rings[64];
    return rings[device & 63];
  }
  std::vector<size_t> off_;
  size_t slot_ = 0;
  std::unique_lock<std::mutex> lock_;
  uint8_t* base_ = nullptr;
  uint8_t* own_ = nullptr;
};

// A per-element host buffer of an element-chunked host call: elem_bytes per
// element; host == nullptr marks an absent optional argument.
struct HostPart {
  const void* host;
  size_t elem_bytes;
};

// Elements per chunk of the host-buffer pipelines for the encryption kernels
// ($XHE_HOST_CHUNK overrides, for A/B runs).
int64_t host_chunk(int64_t dflt) {
  static const int64_t v = [] {
    const char* e = getenv("XHE_HOST_CHUNK");
    return e ? std::max<int64_t>(1024, atoll(e)) : (int64_t)0;
  }();
  return v ? v : dflt;
}

// RAII hipEvent without timing (ordering only)
struct Event {
  hipEvent_t e = nullptr;
  Event() { HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming)); }
  ~Event() { (void)hipEventDestroy(e); }
};

// Element-chunked host-buffer call. Chunk c uses slot b = c % depth and
// stream b: host threads copy its inputs into pinned slot b (xhe_host_copy),
// the upload, run(b, off, n, din, dout, stream)'s kernels and the download
// into the slot follow in stream order, and once the download has landed host
// threads copy the results into the caller's buffers. Chunk c + depth - 1 is
// staged and enqueued before chunk c is drained, so the host copies and both
// DMA directions overlap the kernels. The kernels of chunk c wait for those of
// chunk c - 1 (an event): kernels of different chunks do not share the CUs (a
// big kernel next to a small one on another stream stretches the small one
// from microseconds to milliseconds and stalls the chain behind it), while
// each copy stays in its own stream behind its own kernels, where the runtime
// gives it to a DMA engine (a cross-stream wait in front of a copy made the
// runtime run it as a blit kernel on the CUs instead). Batches whose chunk
// moves < 1 MiB copy straight from and to the caller's memory.
template <class Run>
int host_pipeline(const xhe_key* key, int64_t count, int64_t chunk, const std::vector<HostPart>& in,
                  const std::vector<HostPart>& out, Run&& run) {
  if (count <= 0) return XHE_OK;
  static const bool trace = getenv("XHE_HOST_TRACE") != nullptr;  // per-chunk timings to stderr
  // Kernels of consecutive chunks run one after another ($XHE_HOST_OVERLAP
  // lets them overlap instead: then the three streams' chunks advance in
  // lockstep - each one's small kernels wait for CU slots behind the others'
  // big ones - and the copy-out comes in bursts; 17.6-18.8 vs 19.5-20.4 M/s).
  static const bool serial = getenv("XHE_HOST_OVERLAP") == nullptr;
  chunk = std::max<int64_t>(1, std::min(chunk, count));
  const int64_t nch = (count + chunk - 1) / chunk;
  const int D = (int)std::min<int64_t>(nch, 3);
  const int ni = (int)in.size(), no = (int)out.size();
  std::vector<size_t> parts;
  size_t per_chunk = 0;
  for (auto& h : in) parts.push_back(h.elem_bytes * chunk), per_chunk += h.elem_bytes * chunk;
  for (auto& h : out) parts.push_back(h.elem_bytes * chunk), per_chunk += h.elem_bytes * chunk;
  const bool staged = per_chunk >= ((size_t)1 << 20);
  // only as many streams/events as slots: a one-chunk call (small batches:
  // the LR operators' per-batch calls) pays for one stream, as a plain call
  std::vector<std::unique_ptr<Stream>> st_;
  std::vector<std::unique_ptr<Event>> ev_;
  for (int b = 0; b < D; ++b) {
    st_.emplace_back(new Stream());
    ev_.emplace_back(new Event());
  }
  auto st = [&](int b) -> Stream& { return *st_[b]; };
  auto ev_k = [&](int b) -> Event& { return *ev_[b]; };
  WsCache wsc[3];  // destroyed before the streams (frees are stream-ordered)
  for (int b = 0; b < D; ++b) wsc[b].s = st(b).s;
  std::vector<std::unique_ptr<DevBuf>> dev;  // [slot][part]
  for (int b = 0; b < D; ++b)
    for (size_t k = 0; k < parts.size(); ++k) dev.emplace_back(new DevBuf(parts[k], st(b).s));
  std::unique_ptr<PinnedSlots> pin;
  if (staged) pin.reset(new PinnedSlots(key->device, D, parts));
  // Declared after `pin`, so destroyed before it: on every exit (a non-OK rc,
  // a HIPCHK throw) the slot streams drain before the pinned ring goes back to
  // the device's pool, where another caller may take it while this call's
  // copies are still landing in it.
  struct Drain {
    std::vector<std::unique_ptr<Stream>>& s;
    ~Drain() {
      for (auto& x : s) (void)hipStreamSynchronize(x->s);
    }
  } drain{st_};
  // test hook: run() of this chunk fails (error-path tests). Armed only when
  // XHE_TEST_HOOKS=1 is set as well, so a stray variable cannot fail a call.
  static const int64_t fail_chunk = [] {
    const char* on = getenv("XHE_TEST_HOOKS");
    const char* e = getenv("XHE_TEST_FAIL_CHUNK");
    return (on && on[0] == '1' && e) ? (int64_t)atoll(e) : (int64_t)-1;
  }();
  auto dptr = [&](int b, int k) { return dev[(size_t)b * parts.size() + k]->p; };
  auto enqueue = [&](int64_t c) -> int {
    const int b = (int)(c % D);
    static std::atomic<bool> fired{false};  // the hook fails one call per process
    if (c == fail_chunk && !fired.exchange(true))
      return fail(XHE_EINVAL, "host pipeline: injected failure (XHE_TEST_FAIL_CHUNK)");
    const int64_t off = c * chunk, n = std::min(chunk, count - off);
    hipStream_t s = st(b).s;
    const auto tin = std::chrono::steady_clock::now();
    std::vector<void*> din(ni), dout(no);
    for (int k = 0; k < ni; ++k) {
      din[k] = in[k].host ? dptr(b, k) : nullptr;
      if (!in[k].host) continue;
      const uint8_t* src = static_cast<const uint8_t*>(in[k].host) + (size_t)off * in[k].elem_bytes;
      const size_t nb = (size_t)n * in[k].elem_bytes;
      if (staged) {
        xhe_host_copy(pin->at(b, k), src, (int64_t)nb);
        src = pin->at(b, k);
      }
      HIPCHK(hipMemcpyAsync(din[k], src, nb, hipMemcpyHostToDevice, s));
    }
    if (trace)
      fprintf(stderr, "[host_pipeline] chunk %lld: staged inputs %.3f ms\n", (long long)c,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tin).count());
    if (serial && c > 0) HIPCHK(hipStreamWaitEvent(s, ev_k((int)((c - 1) % D)).e, 0));
    for (int k = 0; k < no; ++k) dout[k] = out[k].host ? dptr(b, ni + k) : nullptr;
    const auto tr = std::chrono::steady_clock::now();
    for (auto& w : wsc[b].blk) w.used = false;
    t_ws = &wsc[b];
    int rc;
    try {
      rc = run(b, off, n, din.data(), dout.data(), s);
    } catch (...) {
      t_ws = nullptr;
      throw;
    }
    t_ws = nullptr;
    if (rc != XHE_OK) return rc;
    HIPCHK(hipEventRecord(ev_k(b).e, s));
    const auto td = std::chrono::steady_clock::now();
    for (int k = 0; k < no; ++k)
      if (out[k].host) {
        void* dst = staged ? (void*)pin->at(b, ni + k)
                           : (void*)(static_cast<uint8_t*>(const_cast<void*>(out[k].host)) + (size_t)off * out[k].elem_bytes);
        HIPCHK(hipMemcpyAsync(dst, dout[k], (size_t)n * out[k].elem_bytes, hipMemcpyDeviceToHost, s));
      }
    if (trace)
      fprintf(stderr, "[host_pipeline] chunk %lld: run %.3f ms, d2h enqueue %.3f ms\n", (long long)c,
              std::chrono::duration<double, std::milli>(td - tr).count(),
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - td).count());
    return XHE_OK;
  };
  int rc = XHE_OK;
  for (int64_t c = 0; c + 1 < D; ++c)
    if ((rc = enqueue(c)) != XHE_OK) return rc;
  for (int64_t c = 0; c < nch; ++c) {
    // slot (c - 1) % D was drained last iteration (its stream has finished)
    if (c + D - 1 < nch && (rc = enqueue(c + D - 1)) != XHE_OK) return rc;
    const int b = (int)(c % D);
    const int64_t off = c * chunk, n = std::min(chunk, count - off);
    const auto t0 = std::chrono::steady_clock::now();
    HIPCHK(hipStreamSynchronize(st(b).s));
    const auto t1 = std::chrono::steady_clock::now();
    if (staged)
      for (int k = 0; k < no; ++k)
        if (out[k].host)
          xhe_host_copy(static_cast<uint8_t*>(const_cast<void*>(out[k].host)) + (size_t)off * out[k].elem_bytes,
                        pin->at(b, ni + k), (int64_t)((size_t)n * out[k].elem_bytes));
    if (trace) {
      const auto t2 = std::chrono::steady_clock::now();
      fprintf(stderr, "[host_pipeline] chunk %lld: wait %.3f ms, copy-out %.3f ms\n", (long long)c,
              std::chrono::duration<double, std::milli>(t1 - t0).count(),
              std::chrono::duration<double, std::milli>(t2 - t1).count());
    }
  }
  return XHE_OK;
}
}  // namespace

namespace {
// Draws for elements [base, base + count) of the stream (seed32, nonce).
void rand_impl(const xhe_key* key, const uint8_t* seed32, uint64_t nonce, int64_t base, int64_t count,
               uint32_t* rand_dev, int32_t* status_dev, hipStream_t s) {
  ChaChaKey ck;
  memcpy(ck.k, seed32, 32);
  ck.nonce0 = (uint32_t)nonce;
  ck.nonce1 = (uint32_t)(nonce >> 32);
  if (key->djn) {
    // no rejection: one thread per ChaCha20 block, the element's lanes adjacent
    int tpe = 1;
    while (tpe < (key->rand_words + 15) / 16) tpe <<= 1;
    int blocks = (int)((count * tpe + 255) / 256);
    hipLaunchKernelGGL(k_rand_djn, dim3(blocks), dim3(256), 0, s, ck, base, count, key->rand_words, key->rand_bits,
                       tpe, rand_dev, status_dev);
  } else {
    int blocks = (int)((count + 255) / 256);
    hipLaunchKernelGGL(k_rand_below, dim3(blocks), dim3(256), 0, s, ck, base, count, key->rand_words,
                       key->rand_bits, key->kd.n_words, rand_dev, status_dev);
  }
  HIPCHK(hipGetLastError());
}
}  // namespace

// row gather (SCATTER = false: dst[i] = src[idx[i]]) or scatter (dst[idx[i]] =
// src[i]), one word per thread, grid-stride (xhe_gather_rows / xhe_scatter_rows)
template <bool SCATTER>
__global__ void k_move_rows(const uint32_t* __restrict__ src, const int64_t* __restrict__ idx, int64_t count,
                            int words, uint32_t* __restrict__ dst) {
  const int64_t tot = count * words;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < tot; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / words, w = t - i * words;
    if (SCATTER) dst[idx[i] * words + w] = src[t];
    else dst[t] = src[idx[i] * words + w];
  }
}

// bit length of each row's value (little-endian words, row-major): what the
// wire layout of Paillier.serialize needs per element (its LONG1/LONG4 byte
// count, paillier.py:244-258), so the host can size the payload before the
// ciphertext words come down
__global__ void k_row_bits(const uint32_t* __restrict__ w, int64_t count, int n2w, int16_t* __restrict__ bits) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint32_t* r = w + (size_t)i * n2w;
  int k = n2w - 1;
  while (k >= 0 && r[k] == 0u) --k;
  bits[i] = (int16_t)(k < 0 ? 0 : 32 * k + 32 - __clz((int)r[k]));
}

extern "C" {

#if XHE_RNS_PROBE
// (probe builds only) k_dec_rns's cycle probe of its last launch: 16 values
int xhe_rns_probe_read(unsigned long long* out) {
  return guarded([&]() -> int {
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rns_probe), 16 * sizeof(unsigned long long), 0,
                               hipMemcpyDeviceToHost));
    return XHE_OK;
  });
}
#endif

int xhe_rns_constants(const uint32_t* p_words, int pw, uint32_t* shared_out, uint32_t* prime_out) {
  return guarded([&]() -> int {
    if (!p_words || pw <= 0 || !shared_out || !prime_out) return fail(XHE_EINVAL, "xhe_rns_constants: bad argument");
    const BigU P = BigU::from_words(p_words, (size_t)pw);
    if (P.bits() > 1024 || P.bits() < 2) return fail(XHE_EINVAL, "xhe_rns_constants: P must have 2..1024 bits");
    const std::vector<uint32_t>& sh = rnsh::bases().shared;
    std::copy(sh.begin(), sh.end(), shared_out);
    const std::vector<uint32_t> pb = rnsh::prime_block(P);
    std::copy(pb.begin(), pb.end(), prime_out);
    return XHE_OK;
  });
}

int xhe_row_bits(const uint32_t* words_dev, int64_t count, int n2w, int16_t* bits_dev, void* stream) {
  return guarded([&]() -> int {
    if (count < 0 || n2w <= 0 || n2w > 1023) return fail(XHE_EINVAL, "xhe_row_bits: bad size");
    if (count == 0) return XHE_OK;
    if (!words_dev || !bits_dev) return fail(XHE_EINVAL, "xhe_row_bits: null argument");
    hipLaunchKernelGGL(k_row_bits, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       words_dev, count, n2w, bits_dev);
    HIPCHK(hipGetLastError());
    return XHE_OK;
  });
}

int xhe_key_create(int device, int key_bits, const uint32_t* n_words, const uint32_t* p_words,
                   const uint32_t* q_words, const uint32_t* h_pow_n_words, int win_bits, xhe_key** out) {
  return guarded([&]() -> int {
    if (!out || !n_words) return fail(XHE_EINVAL, "xhe_key_create: null argument");
    *out = nullptr;
    if (!key_bits_supported(key_bits))
      return fail(XHE_ENOTSUP, "xhe_key_create: key_bits must be 2048, 3072, 4096 or 8192");
    if ((p_words == nullptr) != (q_words == nullptr)) return fail(XHE_EINVAL, "xhe_key_create: need both p and q");
    if (win_bits == 0) {
      const char* ev = getenv("XHE_WIN_BITS");  // "23" or "23s" (split layout), as _native.parse_win
      win_bits = ev ? atoi(ev) : 16;
      if (ev && win_bits > 0 && ev[strlen(ev) - 1] == 's') win_bits |= XHE_WIN_SPLIT;
    }
    const int wbase = win_bits & ~XHE_WIN_SPLIT;
    if (wbase < 2 || wbase > ((win_bits & XHE_WIN_SPLIT) ? 23 : 24))
      return fail(XHE_EINVAL, "xhe_key_create: win_bits must be in [2, 24] (split: [2, 23])");
    std::unique_ptr<xhe_key> k(new xhe_key());
    k->device = device;
    k->K = key_bits;
    k->nw = key_bits / 32;
    k->n2w = 2 * k->nw;
    k->priv = p_words != nullptr;
    k->djn = h_pow_n_words != nullptr;
    with_shape(key_bits, [&](auto sh) {
      using Sh = decltype(sh);
      k->mp2 = {Sh::MP2::S, Sh::MP2::W};
      k->mp2L = {Sh::MP2L::S, Sh::MP2L::W};
      k->mp2X = {Sh::MP2X::S, Sh::MP2X::W};
      k->mp = {Sh::MP::S, Sh::MP::W};
      k->mn2 = {Sh::MN2::S, Sh::MN2::W};
      k->mn2X = {Sh::MN2X::S, Sh::MN2X::W};
    });
    BigU n = BigU::from_words(n_words, k->nw);
    if ((int)n.bits() > key_bits || n.bits() + 2 < (size_t)key_bits)
      return fail(XHE_EINVAL, "xhe_key_create: n does not match key_bits");
    k->n_host.assign(n_words, n_words + k->nw);
    k->n2_host.assign(k->n2w, 0u);
    mul(n, n).to_words(k->n2_host.data(), k->n2w);
    k->n_bits = (int)n.bits();
    {
      BigU third, rem;
      divmod(n, BigU(3), &third, &rem);
      k->dneg = (int)sub(sub(n, third), BigU(1)).bits();  // 2^d >= t  <=>  d >= bitlen(t - 1)
    }
    BigU p, q, h;
    if (k->priv) {
      p = BigU::from_words(p_words, k->nw / 2);
      q = BigU::from_words(q_words, k->nw / 2);
      if (cmp(mul(p, q), n) != 0) return fail(XHE_EINVAL, "xhe_key_create: n != p*q");
      if (p.bits() * 2 > (size_t)key_bits + 0 || q.bits() * 2 > (size_t)key_bits)
        return fail(XHE_ENOTSUP, "xhe_key_create: p and q must each have key_bits/2 bits");
      if ((p.w[0] & 1) == 0 || (q.w[0] & 1) == 0) return fail(XHE_EINVAL, "xhe_key_create: p, q must be odd");
    }
    if (k->djn) h = BigU::from_words(h_pow_n_words, k->n2w);
    DevGuard dg(device);
    keep_pool_memory(device);
    key_create_impl(k.get(), n, k->priv ? &p : nullptr, k->priv ? &q : nullptr, k->djn ? &h : nullptr, win_bits);
    *out = k.release();
    return XHE_OK;
  });
}

void xhe_key_destroy(xhe_key* key) {
  if (!key) return;
  int prev = -1;
  if (hipGetDevice(&prev) == hipSuccess && prev != key->device) (void)hipSetDevice(key->device);
  if (key->d_blob) (void)hipFree(key->d_blob);
  if (key->d_tab) (void)hipFree(key->d_tab);
  if (prev >= 0 && prev != key->device) (void)hipSetDevice(prev);
  delete key;
}

int xhe_key_info(const xhe_key* key, int* key_bits, int* nw, int* n2w, int* rand_words, int* rand_bits, int* flags) {
  if (!key) return fail(XHE_EINVAL, "xhe_key_info: null key");
  if (key_bits) *key_bits = key->K;
  if (nw) *nw = key->nw;
  if (n2w) *n2w = key->n2w;
  if (rand_words) *rand_words = key->rand_words;
  if (rand_bits) *rand_bits = key->rand_bits;
  if (flags) *flags = (key->priv ? 1 : 0) | (key->djn ? 2 : 0);
  return XHE_OK;
}

int xhe_encode_f64(const xhe_key* key, const double* x_dev, int64_t count, int precision, int has_max,
                   int max_exponent, uint32_t* m_dev, int32_t* exp_dev, int32_t* status_dev, void* stream) {
  return guarded([&]() -> int {
    if (!key || (count > 0 && (!x_dev || !m_dev || !exp_dev || !status_dev)))
      return fail(XHE_EINVAL, "xhe_encode_f64: null argument");
    if (count <= 0) return XHE_OK;
    DevGuard dg(key->device);
    int mode = precision < 0 ? 0 : 1;
    // -ceil(log2(10) * precision) (encoder.py:39), computed exactly as Python does in float64
    int e0 = precision < 0 ? 0 : -(int)std::ceil(std::log2(10.0) * (double)precision);
    int blocks = (int)((count * (key->nw / 4) + 255) / 256);  // one thread per 16-byte quad of m
    hipLaunchKernelGGL(k_encode_f64, dim3(blocks), dim3(256), 0, (hipStream_t)stream, x_dev, count, mode, e0,
                       has_max, max_exponent, key->kd.n_words, key->nw, m_dev, exp_dev, status_dev);
    HIPCHK(hipGetLastError());
    return XHE_OK;
  });
}

int xhe_rand(const xhe_key* key, const uint8_t* seed32, uint64_t nonce, int64_t count, uint32_t* rand_dev,
             int32_t* status_dev, void* stream) {
  return guarded([&]() -> int {
    if (!key || !seed32 || (count > 0 && !rand_dev)) return fail(XHE_EINVAL, "xhe_rand: null argument");
    if (count <= 0) return XHE_OK;
    DevGuard dg(key->device);
    rand_impl(key, seed32, nonce, 0, count, rand_dev, status_dev, (hipStream_t)stream);
    return XHE_OK;
  });
}

int xhe_encrypt(const xhe_key* key, const uint32_t* m_dev, const uint32_t* rand_dev, int64_t count, uint32_t* ct_dev,
                void* stream) {
  return guarded([&]() -> int {
    if (!key || (count > 0 && (!m_dev || !ct_dev))) return fail(XHE_EINVAL, "xhe_encrypt: null argument");
    if (count <= 0) return XHE_OK;
    DevGuard dg(key->device);
    hipStream_t s = (hipStream_t)stream;
    if (!rand_dev) {
      with_shape(key->K, [&](auto sh) { raw_encrypt_impl<decltype(sh)>(key, m_dev, count, ct_dev, s); });
      return XHE_OK;
    }
    if (key->djn && key->priv) {
      with_shape(key->K, [&](auto sh) { encrypt_impl<decltype(sh)>(key, m_dev, rand_dev, count, ct_dev, s); });
    } else if (key->djn) {
      with_shape(key->K, [&](auto sh) { encrypt_pub_djn_impl<decltype(sh)>(key, m_dev, rand_dev, count, ct_dev, s); });
    } else {
      with_shape(key->K, [&](auto sh) { encrypt_nodjn_impl<decltype(sh)>(key, m_dev, rand_dev, count, ct_dev, s); });
    }
    return XHE_OK;
  });
}

int xhe_decrypt(const xhe_key* key, const uint32_t* ct_dev, int64_t count, uint32_t* m_dev, void* stream) {
  return guarded([&]() -> int {
    if (!key || (count > 0 && (!ct_dev || !m_dev))) return fail(XHE_EINVAL, "xhe_decrypt: null argument");
    if (!key->priv) return fail(XHE_EINVAL, "Try to decrypt a paillier ciphertext by a public key.");
    if (count <= 0) return XHE_OK;
    DevGuard dg(key->device);
    with_shape(key->K, [&](auto sh) { decrypt_impl<decltype(sh)>(key, ct_dev, count, m_dev, (hipStream_t)stream); });
    return XHE_OK;
  });
}

int xhe_decode(const xhe_key* key, const uint32_t* m_dev, const int32_t* exp_dev, int64_t count, double* f64_dev,
               float* f32_dev, int32_t* status_dev, void* stream) {
  return guarded([&]() -> int {
    if (!key || (count > 0 && (!m_dev || !exp_dev || !f64_dev || !f32_dev || !status_dev)))
      return fail(XHE_EINVAL, "xhe_decode: null argument");
    if (count <= 0) return XHE_OK;
    DevGuard dg(key->device);
    int blocks = (int)((count + 255) / 256);
    hipLaunchKernelGGL(k_decode, dim3(blocks), dim3(256), 0, (hipStream_t)stream, m_dev, exp_dev, count, key->kd,
                       f64_dev, f32_dev, status_dev);
    HIPCHK(hipGetLastError());
    return XHE_OK;
  });
}

int xhe_encrypt_host(const xhe_key* key, const uint32_t* m, const uint32_t* rand, int64_t count, uint32_t* ct) {
  return guarded([&]() -> int {
    if (!key || (count > 0 && (!m || !ct))) return fail(XHE_EINVAL, "xhe_encrypt_host: null argument");
    if (count <= 0) return XHE_OK;
    DevGuard dg(key->device);
    return host_pipeline(key, count, 1 << 17, {{m, (size_t)key->nw * 4}, {rand, (size_t)key->rand_words * 4}},
                         {{ct, (size_t)key->n2w * 4}},
                         [&](int, int64_t, int64_t n, void* const* din, void* const* dout, hipStream_t s) -> int {
                           return xhe_encrypt(key, (const uint32_t*)din[0], (const uint32_t*)din[1], n,
                                              (uint32_t*)dout[0], s);
                         });
  });
}

int xhe_decrypt_host(const xhe_key* key, const uint32_t* ct, int64_t count, uint32_t* m) {
  return guarded([&]() -> int {
    if (!key || (count > 0 && (!ct || !m))) return fail(XHE_EINVAL, "xhe_decrypt_host: null argument");
    if (!key->priv) return fail(XHE_EINVAL, "Try to decrypt a paillier ciphertext by a public key.");
    if (count <= 0) return XHE_OK;
    DevGuard dg(key->device);
    return host_pipeline(key, count, 1 << 17, {{ct, (size_t)key->n2w * 4}}, {{m, (size_t)key->nw * 4}},
                         [&](int, int64_t, int64_t n, void* const* din, void* const* dout, hipStream_t s) -> int {
                           return xhe_decrypt(key, (const uint32_t*)din[0], n, (uint32_t*)dout[0], s);
                         });
  });
}

int xhe_mulmod(const xhe_key* key, const uint32_t* a_dev, const int32_t* ea_dev, const uint32_t* b_dev,
               const int32_t* eb_dev, int64_t count, int dmax, uint32_t* out_dev, int32_t* eout_dev, void* stream) {
  return guarded([&]() -> int {
    if (!key || (count > 0 && (!a_dev || !b_dev || !out_dev)) || dmax < 0)
      return fail(XHE_EINVAL, "xhe_mulmod: bad argument");
    if (count <= 0) return XHE_OK;
    DevGuard dg(key->device);
    const bool row = n2_row(count);
    hipStream_t hs = (hipStream_t)stream;
    return with_shape(key->K, [&](auto sh) -> int {
      using Sh = decltype(sh);
      if (row) mulmod_impl<Sh, typename Sh::MN2X>(key, a_dev, ea_dev, b_dev, eb_dev, count, dmax, out_dev, eout_dev, hs);
      else mulmod_impl<Sh>(key, a_dev, ea_dev, b_dev, eb_dev, count, dmax, out_dev, eout_dev, hs);
      // a NULL exponent array means all exponents 0 (include/xhe.h), so one
      // array alone can still carry a gap >= dneg
      if ((ea_dev || eb_dev) && dmax >= key->dneg)
        return row ? mulmod_gap_fix<Sh, typename Sh::MN2X>(key, a_dev, ea_dev, b_dev, eb_dev, count, out_dev, hs)
                   : mulmod_gap_fix<Sh, typename Sh::MN2>(key, a_dev, ea_dev, b_dev, eb_dev, count, out_dev, hs);
      return XHE_OK;
    });
  });
}

int xhe_powmod(const xhe_key* key, const uint32_t* c_dev, const uint32_t* k_dev, int kw, int kbits, int64_t count,
               uint32_t* out_dev, void* stream) {
  return guarded([&]() -> int {
    if (!key || (count > 0 && (!c_dev || !k_dev || !out_dev)) || kw <= 0 || kbits < 0 || kbits > 32 * kw)
      return fail(XHE_EINVAL, "xhe_powmod: bad argument");
    if (count <= 0) return XHE_OK;
    DevGuard dg(key->device);
    const bool row = n2_row(count);
    hipStream_t hs = (hipStream_t)stream;
    with_shape(key->K, [&](auto sh) {
      using Sh = decltype(sh);
      if (row) powmod_impl<Sh, typename Sh::MN2X>(key, c_dev, k_dev, kw, kbits, count, out_dev, hs);
      else powmod_impl<Sh>(key, c_dev, k_dev, kw, kbits, count, out_dev, hs);
    });
    return XHE_OK;
  });
}

int xhe_invert(const xhe_key* key, const uint32_t* c_dev, int64_t count, uint32_t* out_dev, void* stream) {
  return guarded([&]() -> int {
    if (!key || (count > 0 && (!c_dev || !out_dev))) return fail(XHE_EINVAL, "xhe_invert: null argument");
    if (count <= 0) return XHE_OK;
    DevGuard dg(key->device);
    const bool row = n2_row(count);
    hipStream_t hs = (hipStream_t)stream;
    return with_shape(key->K, [&](auto sh) -> int {
      using Sh = decltype(sh);
      return row ? invert_impl<Sh, typename Sh::MN2X>(key, c_dev, count, out_dev, hs)
                 : invert_impl<Sh>(key, c_dev, count, out_dev, hs);
    });
  });
}


int xhe_encrypt_f64_host(const xhe_key* key, const double* x, int64_t count, int precision, int has_max,
                         int max_exponent, int obfuscate, const uint8_t* seed32, uint64_t nonce, uint32_t* ct,
                         int32_t* exps, int32_t* status) {
  return guarded([&]() -> int {
    if (!key || (count > 0 && (!x || !ct || !exps || !status)) || (obfuscate && !seed32))
      return fail(XHE_EINVAL, "xhe_encrypt_f64_host: null argument");
    if (count <= 0) return XHE_OK;
    DevGuard dg(key->device);
    // chunks of 256 k elements through host_pipeline (with the kernels of
    // consecutive chunks serialised, a chunk's last partial round of waves is
    // idle time: 128 k chunks ran 21.8 M/s device-resident, 256 k 25.8 M/s,
    // tools/chunk_rate.py); the randomness is drawn at global element
    // positions, so the ciphertexts do not depend on the chunking
    const int64_t chunk = host_chunk(1 << 18), cmax = std::min<int64_t>(chunk, count);
    std::unique_ptr<DevBuf> dm[3], dr[3];
    return host_pipeline(
        key, count, chunk, {{x, 8}}, {{ct, (size_t)key->n2w * 4}, {exps, 4}, {status, 4}},
        [&](int b, int64_t off, int64_t n, void* const* din, void* const* dout, hipStream_t s) -> int {
          if (!dm[b]) {
            dm[b].reset(new DevBuf((size_t)cmax * key->nw * 4, s));
            dr[b].reset(new DevBuf(obfuscate ? (size_t)cmax * key->rand_words * 4 : 4, s));
          }
          int rc = xhe_encode_f64(key, (const double*)din[0], n, precision, has_max, max_exponent,
                                  dm[b]->as<uint32_t>(), (int32_t*)dout[1], (int32_t*)dout[2], s);
          if (rc != XHE_OK) return rc;
          if (obfuscate) rand_impl(key, seed32, nonce, off, n, dr[b]->as<uint32_t>(), nullptr, s);
          return xhe_encrypt(key, dm[b]->as<uint32_t>(), obfuscate ? dr[b]->as<uint32_t>() : nullptr, n,
                             (uint32_t*)dout[0], s);
        });
  });
}

int xhe_encrypt_words_host(const xhe_key* key, const uint32_t* m, int64_t count, int obfuscate,
                           const uint8_t* seed32, uint64_t nonce, uint32_t* ct) {
  return guarded([&]() -> int {
    if (!key || (count > 0 && (!m || !ct)) || (obfuscate && !seed32))
      return fail(XHE_EINVAL, "xhe_encrypt_words_host: null argument");
    if (count <= 0) return XHE_OK;
    DevGuard dg(key->device);
    const int64_t chunk = host_chunk(1 << 18), cmax = std::min<int64_t>(chunk, count);
    std::unique_ptr<DevBuf> dr[3];
    return host_pipeline(
        key, count, chunk, {{m, (size_t)key->nw * 4}}, {{ct, (size_t)key->n2w * 4}},
        [&](int b, int64_t off, int64_t n, void* const* din, void* const* dout, hipStream_t s) -> int {
          if (obfuscate) {
            if (!dr[b]) dr[b].reset(new DevBuf((size_t)cmax * key->rand_words * 4, s));
            rand_impl(key, seed32, nonce, off, n, dr[b]->as<uint32_t>(), nullptr, s);
          }
          return xhe_encrypt(key, (const uint32_t*)din[0], obfuscate ? dr[b]->as<uint32_t>() : nullptr, n,
                             (uint32_t*)dout[0], s);
        });
  });
}

int xhe_decrypt_decode_host(const xhe_key* key, const uint32_t* ct, const int32_t* exps, int64_t count, double* f64,
                            float* f32, int32_t* status, uint32_t* m_out) {
  return guarded([&]() -> int {
    if (!key || (count > 0 && (!ct || !exps || !f64 || !f32 || !status)))
      return fail(XHE_EINVAL, "xhe_decrypt_decode_host: null argument");
    if (!key->priv) return fail(XHE_EINVAL, "Try to decrypt a paillier ciphertext by a public key.");
    if (count <= 0) return XHE_OK;
    DevGuard dg(key->device);
    const int64_t chunk = host_chunk(1 << 17), cmax = std::min<int64_t>(chunk, count);
    std::unique_ptr<DevBuf> dm[3];
    return host_pipeline(
        key, count, chunk, {{ct, (size_t)key->n2w * 4}, {exps, 4}},
        {{f64, 8}, {f32, 4}, {status, 4}, {m_out, (size_t)key->nw * 4}},
        [&](int b, int64_t, int64_t n, void* const* din, void* const* dout, hipStream_t s) -> int {
          uint32_t* m = (uint32_t*)dout[3];
          if (!m) {
            if (!dm[b]) dm[b].reset(new DevBuf((size_t)cmax * key->nw * 4, s));
            m = dm[b]->as<uint32_t>();
          }
          int rc = xhe_decrypt(key, (const uint32_t*)din[0], n, m, s);
          if (rc != XHE_OK) return rc;
          return xhe_decode(key, m, (const int32_t*)din[1], n, (double*)dout[0], (float*)dout[1],
                            (int32_t*)dout[2], s);
        });
  });
}

int xhe_mulmod_host(const xhe_key* key, const uint32_t* a, const int32_t* ea, const uint32_t* b, const int32_t* eb,
                    int64_t count, int dmax, uint32_t* out, int32_t* eout) {
  return guarded([&]() -> int {
    if (!key || (count > 0 && (!a || !b || !out))) return fail(XHE_EINVAL, "xhe_mulmod_host: null argument");
    if (count <= 0) return XHE_OK;
    DevGuard dg(key->device);
    const size_t cb = (size_t)key->n2w * 4;
    return host_pipeline(
        key, count, 1 << 16, {{a, cb}, {ea, 4}, {b, cb}, {eb, 4}}, {{out, cb}, {eout, 4}},
        [&](int, int64_t, int64_t n, void* const* din, void* const* dout, hipStream_t s) -> int {
          return xhe_mulmod(key, (const uint32_t*)din[0], (const int32_t*)din[1], (const uint32_t*)din[2],
                            (const int32_t*)din[3], n, dmax, (uint32_t*)dout[0], (int32_t*)dout[1], s);
        });
  });
}

int xhe_powmod_host(const xhe_key* key, const uint32_t* c, const uint32_t* k, int kw, int kbits, int64_t count,
                    int invert_first, uint32_t* out) {
  return guarded([&]() -> int {
    if (!key || (count > 0 && (!c || !k || !out))) return fail(XHE_EINVAL, "xhe_powmod_host: null argument");
    if (count <= 0) return XHE_OK;
    DevGuard dg(key->device);
    const size_t cb = (size_t)key->n2w * 4;
    const int64_t chunk = 1 << 16, cmax = std::min<int64_t>(chunk, count);
    std::unique_ptr<DevBuf> dinv[3];
    return host_pipeline(
        key, count, chunk, {{c, cb}, {k, (size_t)kw * 4}}, {{out, cb}},
        [&](int b, int64_t, int64_t n, void* const* din, void* const* dout, hipStream_t s) -> int {
          const uint32_t* base = (const uint32_t*)din[0];
          if (invert_first) {
            if (!dinv[b]) dinv[b].reset(new DevBuf((size_t)cmax * cb, s));
            int rc = xhe_invert(key, base, n, dinv[b]->as<uint32_t>(), s);
            if (rc != XHE_OK) return rc;
            base = dinv[b]->as<uint32_t>();
          }
          return xhe_powmod(key, base, (const uint32_t*)din[1], kw, kbits, n, (uint32_t*)dout[0], s);
        });
  });
}

int xhe_segprod_host(const xhe_key* key, const uint32_t* c, const int32_t* d, int dmax, int64_t count,
                     const int64_t* seg_begin, int64_t nseg, uint32_t* out) {
  return guarded([&]() -> int {
    if (!key || !seg_begin || nseg <= 0 || (count > 0 && !c) || !out) return fail(XHE_EINVAL, "xhe_segprod_host: bad argument");
    DevGuard dg(key->device);
    Stream st;
    size_t cw = (size_t)std::max<int64_t>(count, 1) * key->n2w * 4;
    DevBuf dc(cw, st.s), dd((size_t)std::max<int64_t>(count, 1) * 4, st.s), dout((size_t)nseg * key->n2w * 4, st.s);
    if (count > 0) HIPCHK(hipMemcpyAsync(dc.p, c, (size_t)count * key->n2w * 4, hipMemcpyHostToDevice, st.s));
    if (d && count > 0) HIPCHK(hipMemcpyAsync(dd.p, d, count * 4, hipMemcpyHostToDevice, st.s));
    int rc = xhe_segprod(key, dc.as<uint32_t>(), d ? dd.as<int32_t>() : nullptr, dmax, count, seg_begin, nseg,
                         dout.as<uint32_t>(), st.s);
    if (rc != XHE_OK) return rc;
    HIPCHK(hipMemcpyAsync(out, dout.p, (size_t)nseg * key->n2w * 4, hipMemcpyDeviceToHost, st.s));
    HIPCHK(hipStreamSynchronize(st.s));
    return XHE_OK;
  });
}

int xhe_multiexp(const xhe_key* key, const uint32_t* bases_dev, int64_t nbases, const int32_t* idx_dev,
                 const uint32_t* k_dev, int kw, int kbits, int64_t ncols, int64_t nterms, int win_bits,
                 uint32_t* out_dev, void* stream) {
  return guarded([&]() -> int {
    if (!key || nbases <= 0 || ncols <= 0 || nterms <= 0 || !bases_dev || !idx_dev || !k_dev || !out_dev || kw <= 0 ||
        kbits < 0 || kbits > 32 * kw || win_bits < 0 || win_bits > 8)
      return fail(XHE_EINVAL, "xhe_multiexp: bad argument");
    if (ncols * nterms > (int64_t)1 << 31 || nbases > (int64_t)1 << 30)
      return fail(XHE_EINVAL, "xhe_multiexp: problem too large for one call");
    DevGuard dg(key->device);
    const bool row = n2_row(std::max(nbases, ncols));
    const int s4 = with_shape(key->K, [&](auto sh) -> int {
      using Sh = decltype(sh);
      return row ? Sh::MN2X::S4 : Sh::MN2::S4;
    });
    const int c = win_bits ? win_bits : mexp_window(nbases, ncols, nterms, std::max(kbits, 1), s4);
    const int kb = std::max(kbits, 1);
    hipStream_t hs = (hipStream_t)stream;
    with_shape(key->K, [&](auto sh) {
      using Sh = decltype(sh);
      if (row)
        multiexp_impl<Sh, typename Sh::MN2X>(key, bases_dev, nbases, idx_dev, k_dev, kw, kb, ncols, nterms, c, out_dev,
                                             hs);
      else
        multiexp_impl<Sh>(key, bases_dev, nbases, idx_dev, k_dev, kw, kb, ncols, nterms, c, out_dev, hs);
    });
    return XHE_OK;
  });
}

int xhe_multiexp_host(const xhe_key* key, const uint32_t* bases, int64_t nbases, const int32_t* idx, const uint32_t* k,
                      int kw, int kbits, int64_t ncols, int64_t nterms, int win_bits, uint32_t* out) {
  return guarded([&]() -> int {
    if (!key || nbases <= 0 || ncols <= 0 || nterms <= 0 || !bases || !idx || !k || !out || kw <= 0)
      return fail(XHE_EINVAL, "xhe_multiexp_host: bad argument");
    for (int64_t i = 0; i < ncols * nterms; ++i)
      if (idx[i] < 0 || idx[i] >= nbases) return fail(XHE_EINVAL, "xhe_multiexp_host: base index out of range");
    DevGuard dg(key->device);
    Stream st;
    DevBuf db((size_t)nbases * key->n2w * 4, st.s), di((size_t)ncols * nterms * 4, st.s),
        dk((size_t)ncols * nterms * kw * 4, st.s), dout((size_t)ncols * key->n2w * 4, st.s);
    HIPCHK(hipMemcpyAsync(db.p, bases, (size_t)nbases * key->n2w * 4, hipMemcpyHostToDevice, st.s));
    HIPCHK(hipMemcpyAsync(di.p, idx, (size_t)ncols * nterms * 4, hipMemcpyHostToDevice, st.s));
    HIPCHK(hipMemcpyAsync(dk.p, k, (size_t)ncols * nterms * kw * 4, hipMemcpyHostToDevice, st.s));
    int rc = xhe_multiexp(key, db.as<uint32_t>(), nbases, di.as<int32_t>(), dk.as<uint32_t>(), kw, kbits, ncols, nterms,
                          win_bits, dout.as<uint32_t>(), st.s);
    if (rc != XHE_OK) return rc;
    HIPCHK(hipMemcpyAsync(out, dout.p, (size_t)ncols * key->n2w * 4, hipMemcpyDeviceToHost, st.s));
    HIPCHK(hipStreamSynchronize(st.s));
    return XHE_OK;
  });
}

int xhe_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int xhe_gather_rows(const uint32_t* src_dev, const int64_t* idx_dev, int64_t count, int words, uint32_t* dst_dev,
                    void* stream) {
  return guarded([&]() -> int {
    if (count < 0 || words <= 0) return fail(XHE_EINVAL, "xhe_gather_rows: bad size");
    if (count == 0) return XHE_OK;
    if (!src_dev || !idx_dev || !dst_dev) return fail(XHE_EINVAL, "xhe_gather_rows: null argument");
    const int64_t tot = count * words;
    const unsigned blocks = (unsigned)std::min<int64_t>((tot + 255) / 256, 65536);
    hipLaunchKernelGGL(k_move_rows<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, src_dev, idx_dev, count,
                       words, dst_dev);
    HIPCHK(hipGetLastError());
    return XHE_OK;
  });
}

int xhe_scatter_rows(const uint32_t* src_dev, const int64_t* idx_dev, int64_t count, int words, uint32_t* dst_dev,
                     void* stream) {
  return guarded([&]() -> int {
    if (count < 0 || words <= 0) return fail(XHE_EINVAL, "xhe_scatter_rows: bad size");
    if (count == 0) return XHE_OK;
    if (!src_dev || !idx_dev || !dst_dev) return fail(XHE_EINVAL, "xhe_scatter_rows: null argument");
    const int64_t tot = count * words;
    const unsigned blocks = (unsigned)std::min<int64_t>((tot + 255) / 256, 65536);
    hipLaunchKernelGGL(k_move_rows<true>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, src_dev, idx_dev, count,
                       words, dst_dev);
    HIPCHK(hipGetLastError());
    return XHE_OK;
  });
}

int xhe_synchronize(void* stream) {
  hipError_t e = hipStreamSynchronize((hipStream_t)stream);
  if (e != hipSuccess) return fail(XHE_EHIP, hipGetErrorString(e));
  return XHE_OK;
}

int xhe_profile(int enable) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_prof_on = enable != 0;
  for (auto& r : g_prof) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  g_prof.clear();
  return XHE_OK;
}

int xhe_profile_read(const char* kernel, double* total_ms, int64_t* launches) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  double t = 0;
  int64_t n = 0;
  for (auto& r : g_prof) {
    if (kernel && r.name != kernel) continue;
    if (hipEventSynchronize(r.b) != hipSuccess) return fail(XHE_EHIP, "xhe_profile_read: event sync failed");
    float ms = 0;
    if (hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) return fail(XHE_EHIP, "xhe_profile_read: elapsed failed");
    t += ms;
    ++n;
  }
  if (total_ms) *total_ms = t;
  if (launches) *launches = n;
  return XHE_OK;
}


}  // extern "C"
