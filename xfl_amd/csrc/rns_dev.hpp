// Small-batch decrypt exponentiation in a residue number system (2048-bit
// keys): X_P = c^(P-1) mod P^2 for one residue per 384-thread block, every
// Montgomery product as two base extensions instead of WaveMont's six LDS
// column phases (dec_wave.hpp; its 1.7 us products set the LR demo's 2.1 ms
// decrypt, paillier.py:341-368 / label_trainer.py:252-259).
//
// A value x < LAM N (N = P^2, LAM = RK + 1) is held as its residues modulo two
// bases of RK = 74 primes below 2^28, B and B' (M, M' ~ 2^2072), and mod 2^32
// (the redundant channel r). One product x y M^-1 mod N (Bajard/Kawamura RNS
// Montgomery with a Shenoy-Kumaresan exact extension):
//   all       t = x y per channel
//   B         xi_i = t_i |-N^-1 M_i^-1|_(m_i)                -> LDS
//   -- barrier --
//   B'        qh'_j = sum_i xi_i |M_i|_(m'_j)  (fast extension: qh = q + alpha M)
//             r'_j = t'_j |M^-1| + qh'_j |N M^-1|,
//             xi'_j = t'_j |M^-1 M'_j^-1| + qh'_j |N M^-1 M'_j^-1|        -> LDS
//   r         r_r = (t_r + (sum_i xi_i |M_i|_(2^32)) N) M^-1 mod 2^32     -> LDS
//             the B' waves also sum xi'_j |M'_j|_(2^32) (DPP)           -> LDS
//   -- barrier --
//   B         beta = (sum_j xi'_j |M'_j|_(2^32) - r_r) M'^-1 mod 2^32  (exact, < RK)
//             r_i = sum_j xi'_j |M'_j|_(m_i) - beta |M'|_(m_i)
// Threads: waves 0-2 hold B, waves 3-5 B' and r. A channel ch = 3 l + (wave
// mod 3) (l = lane mod 32 < 25; ch = 74 of the B' waves is r) lives in two
// lanes of one wave, l and l + 32: each sums half of every extension (40 of
// the 80 zero-padded terms, eight 64-bit accumulators, sums < 2^62), the
// halves meet through v_permlane32_swap, and both lanes carry on with the
// channel (only the low one stores). The t terms of B' are taken before the
// first barrier, and every multiplication by a constant is a Shoup product
// (one correction) so the chains after each barrier stay short.
// tools/rns_model.py checks the algorithm, the bounds (r < LAM N when M >=
// LAM^2 N; alpha, beta < RK; column sums < 2^63) and the Barrett reductions
// below for every modulus against Python integers; tests/test_rns_constants.py
// emulates this kernel's arithmetic on the constant blocks.
#pragma once
#include "xhe_kernels.hpp"

namespace xhe {
namespace rns {

constexpr int RK = 74;      // moduli per base
constexpr int RKP = 76;     // limbs of M_i, M at the exit (28 bits)
constexpr int RT = 80;      // extension terms, zero-padded (two halves of 40)
constexpr int HT = RT / 2;
constexpr int NT = 384;     // threads per residue
constexpr int NSLOT = 160;  // constant slots: B channels 0..79, B' channels 80..159 (r: 154)
constexpr int RCH = 74;     // the B' waves' channel number of r
constexpr uint32_t LMASK = (1u << 28) - 1u;

// constant blocks (words): shared by every key (the bases), then per prime;
// per-slot arrays of NSLOT
constexpr int S_M = 0, S_MU = 160, S_T32 = 320, S_B = 480, S_BS = 640, S_C = 800, S_CS = 960, S_D = 1120;
constexpr int S_ROWS = 1280;                // [RT][NSLOT]: B: |M'_j|_(m_i); B': |M_i|_(m'_j); r: |M_i|_(2^32)
constexpr int S_MPOS = S_ROWS + RT * NSLOT; // [RK][RKP] 28-bit limbs of M_i = M / m_i
constexpr int S_MFULL = S_MPOS + RK * RKP;  // [RKP] limbs of M
constexpr int S_M2RINV = S_MFULL + RKP;     // M'^-1 mod 2^32
constexpr int S_WORDS = S_M2RINV + 4;
// per prime: P_A (B: |-N^-1 M_i^-1|; B': |N M^-1|; r: N mod 2^32) and its
// Shoup companion, P_A2 (B': |N M^-1 M'_j^-1|) and companion, M^3 mod N per
// channel, then the exponent P - 1 as a window schedule: P_NS entries, [0] =
// the start value's table index, then (squarings << 8) | (t + 1) (t + 1 = 0:
// no product)
constexpr int P_A = 0, P_AS = 160, P_A2 = 320, P_A2S = 480, P_M3 = 640, P_NS = 800, P_SCHED = 804;
constexpr int P_SCHED_MAX = 1280;
constexpr int P_WORDS = P_SCHED + P_SCHED_MAX + 4;
static_assert(S_WORDS == XHE_RNS_SHARED_WORDS && P_WORDS == XHE_RNS_PRIME_WORDS, "include/xhe.h sizes");

// x < 2^59 -> x mod m (m in (2^27, 2^28), mu = floor(2^59 / m) in (2^31, 2^32)):
// the quotient estimate is short by at most 3
XHE_DEV uint32_t red(uint64_t x, uint32_t m, uint32_t mu) {
  const uint32_t q = __umulhi((uint32_t)(x >> 27), mu);
  uint32_t r = (uint32_t)x - q * m;
  r = min(r, r - m);
  r = min(r, r - m);
  return min(r, r - m);
}
// x < 2^63: the high word folded by 2^32 mod m first
XHE_DEV uint32_t red64(uint64_t x, uint32_t m, uint32_t mu, uint32_t t32) {
  return red((uint64_t)(uint32_t)(x >> 32) * t32 + (uint32_t)x, m, mu);
}
// a w mod m for a constant w < m and ws = floor(w 2^32 / m) (Shoup): a w - q m
// lies in [0, 2m) for any a < 2^32
XHE_DEV uint32_t shoup(uint32_t a, uint32_t w, uint32_t ws, uint32_t m) {
  const uint32_t r = a * w - __umulhi(a, ws) * m;
  return min(r, r - m);
}

struct Chan {
  uint32_t m, mu, t32;
  bool r32;  // the mod-2^32 channel
  XHE_DEV uint32_t mul(uint32_t a, uint32_t b) const {
    const uint64_t p = (uint64_t)a * b;
    return r32 ? (uint32_t)p : red(p, m, mu);
  }
  XHE_DEV uint32_t add(uint32_t a, uint32_t b) const {
    const uint32_t s = a + b;
    return r32 ? s : min(s, s - m);
  }
};

struct Lds {
  uint32_t xi[RT];   // B -> B': xi_i (zero beyond RK)
  uint32_t xi2[RT];  // B' -> B: xi'_j
  uint32_t part[4];  // per B' wave: sum xi'_j |M'_j|_(2^32)
  uint32_t rr;       // r mod 2^32
  uint32_t alpha;
  int64_t col[RKP];  // exit: the positional columns
  uint32_t tab[16 * NT];  // [power][thread]: x^(2k+1) of every thread's channel
};

// acc[0..7] += 8 terms: two operand quads against row[4q .. 4q + 7]
XHE_DEV void mad8(uint64_t (&a)[8], const uint4& x0, const uint4& x1, const uint32_t* r) {
  asm("v_mad_u64_u32 %0, vcc, %8, %16, %0\n\t"
      "v_mad_u64_u32 %1, vcc, %9, %17, %1\n\t"
      "v_mad_u64_u32 %2, vcc, %10, %18, %2\n\t"
      "v_mad_u64_u32 %3, vcc, %11, %19, %3\n\t"
      "v_mad_u64_u32 %4, vcc, %12, %20, %4\n\t"
      "v_mad_u64_u32 %5, vcc, %13, %21, %5\n\t"
      "v_mad_u64_u32 %6, vcc, %14, %22, %6\n\t"
      "v_mad_u64_u32 %7, vcc, %15, %23, %7"
      : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
      : "v"(x0.x), "v"(x0.y), "v"(x0.z), "v"(x0.w), "v"(x1.x), "v"(x1.y), "v"(x1.z), "v"(x1.w), "v"(r[0]), "v"(r[1]),
        "v"(r[2]), "v"(r[3]), "v"(r[4]), "v"(r[5]), "v"(r[6]), "v"(r[7])
      : "vcc");
}
// a + b as one v_lshl_add_u64 (asm: the compiler re-associated a C sum tree
// into a chain of seven dependent adds)
XHE_DEV uint64_t add64(uint64_t a, uint64_t b) {
  uint64_t r;
  asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// this lane's half of sum_i v[i] row[i]: its 40 terms (v = the half's base)
// into eight independent accumulators, the operand quads read in two batches
// of five (register room for two blocks per CU), the sums added as a tree
XHE_DEV uint64_t ext_half(const uint32_t* v, const uint32_t (&row)[HT]) {
  const uint4* vq = reinterpret_cast<const uint4*>(v);
  uint64_t a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint4 x[6];
#pragma unroll
  for (int q = 0; q < 5; ++q) x[q] = vq[q];
  mad8(a, x[0], x[1], row);
  mad8(a, x[2], x[3], row + 8);
  x[5] = vq[5];
  mad8(a, x[4], x[5], row + 16);
#pragma unroll
  for (int q = 6; q < 10; ++q) x[q - 6] = vq[q];
  mad8(a, x[0], x[1], row + 24);
  mad8(a, x[2], x[3], row + 32);
  return add64(add64(add64(a[0], a[1]), add64(a[2], a[3])), add64(add64(a[4], a[5]), add64(a[6], a[7])));
}

// v of this lane + v of lane (l xor 32): v_permlane32_swap exchanges the low
// half-wave of one register with the high half-wave of the other, so with v in
// both, the two results hold (own, partner) in some order in every lane;
// every lane of the wave active
XHE_DEV uint64_t add_partner(uint64_t v) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  const auto l2 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto h2 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return ((uint64_t)h2[0] << 32 | l2[0]) + ((uint64_t)h2[1] << 32 | l2[1]);
}

// sum of v over the 64 lanes of the wave (row inclusive scans, then the
// rows' last lanes); every lane active
XHE_DEV uint32_t wave_sum(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 15) + (uint32_t)__builtin_amdgcn_readlane((int)v, 31) +
         (uint32_t)__builtin_amdgcn_readlane((int)v, 47) + (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

}  // namespace rns

#ifndef XHE_RNS_PROBE
#define XHE_RNS_PROBE 0
#endif
#ifndef XHE_RNS_WPE
#define XHE_RNS_WPE 4
#endif
#if XHE_RNS_PROBE
// cycle probe of block (0, 0) (a -D XHE_RNS_PROBE=1 build, tools/rns_probe.py):
// per role (B wave 0, B' wave 3) the shader clocks spent from a product's
// start to its first barrier's exit, between the barriers, and from the
// second barrier to the product's end, summed over the products; the
// product count; the kernel's clocks and the 100 MHz real-time span
__device__ unsigned long long g_rns_probe[16];
#endif

// k_dec_rns: the same rows as k_dec_wave (X_P = (c^(P-1) mod P^2) - 1,
// [prime][xs4][count], limbs of 28 bits beyond K zero) with the same 5-bit
// sliding-window schedule over P - 1 (16 odd powers, one register each per
// channel), precomputed per key. grid (count, 2): blockIdx.y is the prime.
// At most 128 VGPRs (4 waves per SIMD): two blocks per CU, whose six-wave
// shape puts two waves on SIMDs 0 and 1 (178 VGPRs allowed one block, and
// batches of 256+ residues took twice as long).
__global__ void __launch_bounds__(rns::NT, XHE_RNS_WPE) k_dec_rns(KeyDev key, const uint32_t* __restrict__ c_words,
                                                     int64_t count, int xs4, uint32_t* __restrict__ xrows) {
  using namespace rns;
  constexpr int K = 74;  // limbs of 28 bits of P^2 (the MP2 rows)
  __shared__ __attribute__((aligned(16))) Lds s;
  const int t = (int)threadIdx.x;
  const int prime = blockIdx.y;
  const int64_t e = blockIdx.x;
  const int w = t >> 6, lane = t & 63, h = lane >> 5;
  const bool gB = w < 3;  // waves 0-2: base B; waves 3-5: base B' and the 2^32 channel
  const int wv = gB ? w : w - 3;
  const int ch = 3 * (lane & 31) + wv;  // < 75 when lane mod 32 < 25
  const bool isr = !gB && ch == RCH;
  const bool act = ch < RK;             // a channel of B or B' (r excluded)
  const int slot = (gB ? 0 : 80) + (ch < 80 ? ch : 79);
  const uint32_t* S = key.rns;
  const uint32_t* Pb = prime ? key.rns_q : key.rns_p;
  Chan c;
  c.m = S[S_M + slot];
  c.mu = S[S_MU + slot];
  c.t32 = S[S_T32 + slot];
  c.r32 = isr;
  const uint32_t cb = S[S_B + slot], cbs = S[S_BS + slot], cc = S[S_C + slot], ccs = S[S_CS + slot];
  const uint32_t cd = S[S_D + slot], m2rinv = S[S_M2RINV];
  const uint32_t ca = Pb[P_A + slot], cas = Pb[P_AS + slot], ca2 = Pb[P_A2 + slot], ca2s = Pb[P_A2S + slot];
  const uint32_t m3 = Pb[P_M3 + slot];
  uint32_t row[HT];
#pragma unroll
  for (int i = 0; i < HT; ++i) row[i] = S[S_ROWS + (h * HT + i) * NSLOT + slot];
  if (t < RT) {
    s.xi[t] = 0u;
    s.xi2[t] = 0u;
  }
  __syncthreads();

#if XHE_RNS_PROBE
  const uint64_t pr_t0 = __builtin_amdgcn_s_memtime(), pr_r0 = __builtin_amdgcn_s_memrealtime();
  uint64_t pr_d1 = 0, pr_d2 = 0, pr_d3 = 0, pr_n = 0, pr_a = 0;
#define RNS_PROBE(stmt) stmt
#else
#define RNS_PROBE(stmt)
#endif
  // x y M^-1 mod N in every channel (two barriers; roles are wave-uniform)
  auto mul = [&](uint32_t x, uint32_t y) -> uint32_t {
    RNS_PROBE(pr_a = __builtin_amdgcn_s_memtime());
    const uint32_t tt = c.mul(x, y);
    uint32_t tm = 0u, ta = 0u;
    if (gB) {
      if (act && h == 0) s.xi[ch] = shoup(tt, ca, cas, c.m);  // ca = |-N^-1 M_i^-1|
    } else if (!isr) {
      tm = shoup(tt, cb, cbs, c.m);  // cb = |M^-1|
      ta = shoup(tt, cc, ccs, c.m);  // cc = |M^-1 M'_j^-1|
    }
    __syncthreads();
    RNS_PROBE(const uint64_t pr_b = __builtin_amdgcn_s_memtime(); pr_d1 += pr_b - pr_a);
    uint32_t res = 0u;
    if (!gB) {
      const uint64_t acc = add_partner(ext_half(s.xi + h * HT, row));
      uint32_t u = 0u;
      if (isr) {  // ca = N mod 2^32, cb = M^-1 mod 2^32
        res = (tt + (uint32_t)acc * ca) * cb;
        if (h == 0) s.rr = res;
      } else {    // ca = |N M^-1|, ca2 = |N M^-1 M'_j^-1|, cd = |M'_j|_(2^32)
        const uint32_t qh = red64(acc, c.m, c.mu, c.t32);
        res = c.add(tm, shoup(qh, ca, cas, c.m));
        const uint32_t x2 = c.add(ta, shoup(qh, ca2, ca2s, c.m));
        if (act && h == 0) {
          s.xi2[ch] = x2;
          u = x2 * cd;
        }
      }
      const uint32_t sum = wave_sum(u);
      if (lane == 0) s.part[wv] = sum;
    }
    __syncthreads();
    RNS_PROBE(const uint64_t pr_c = __builtin_amdgcn_s_memtime(); pr_d2 += pr_c - pr_b);
    if (gB) {  // cb = |M'|_(m_i)
      const uint64_t acc = add_partner(ext_half(s.xi2 + h * HT, row));
      const uint32_t beta = (s.part[0] + s.part[1] + s.part[2] - s.rr) * m2rinv;
      const uint32_t d = red64(acc, c.m, c.mu, c.t32) - shoup(beta, cb, cbs, c.m);
      res = min(d, d + c.m);
    }
    RNS_PROBE(pr_d3 += __builtin_amdgcn_s_memtime() - pr_c; ++pr_n);
    return res;
  };

  // c mod m from the ciphertext words (Horner from the top word), then
  // c M^-1 (one REDC: c < 2^4096 < M N) and c M (times M^3 mod N)
  uint32_t x;
  {
    const uint32_t* cw = c_words + (size_t)e * key.n2w;
    uint32_t acc = 0u;
    for (int k = key.n2w - 1; k >= 0; --k) acc = red((uint64_t)acc * c.t32 + cw[k], c.m, c.mu);
    x = isr ? cw[0] : acc;
  }
  x = mul(x, 1u);
  x = mul(x, m3);
  // odd powers x, x^3 .. x^31, each thread's in its own LDS column (a table
  // product reads its operand back once; registers hold the extension rows)
  uint32_t* tab = s.tab + t;
  tab[0] = x;
  const uint32_t x2 = mul(x, x);
#pragma unroll 1
  for (int k = 1; k < 16; ++k) {
    x = mul(x, x2);
    tab[k * NT] = x;
  }
  auto pick = [&](uint32_t v) { return tab[v * NT]; };
  // the 5-bit sliding-window schedule over P - 1, precomputed per key
  // (scalar loads, one per window)
  const uint32_t* sc = Pb + P_SCHED;
  const int ns = (int)Pb[P_NS];
  x = pick(sc[0]);
#pragma unroll 1
  for (int k = 1; k < ns; ++k) {
    const uint32_t wd = sc[k];
#pragma unroll 1
    for (uint32_t q = wd >> 8; q; --q) x = mul(x, x);
    if (wd & 0xFFu) x = mul(x, pick((wd & 0xFFu) - 1u));
  }
  x = mul(x, 1u);  // out of Montgomery form: X < LAM N, X = c^(P-1) mod N

  // exit: X = sum_i xi_i M_i - alpha M (xi_i = X_i |M_i^-1|, alpha from the
  // 2^32 channel), as 28-bit columns, then reduced mod N by thread 0
  if (gB && act && h == 0) s.xi[ch] = c.mul(x, cc);  // cc = |M_i^-1|
  __syncthreads();
  if (w == 5) {  // r's wave (whole, for the swap): cb = M^-1 mod 2^32
    const uint32_t sx = (uint32_t)add_partner(ext_half(s.xi + h * HT, row));
    if (isr && h == 0) s.alpha = (sx - x) * cb;
  }
  int64_t colv = 0;
  if (t < RKP) {
    const uint32_t* mp = S + S_MPOS + t;
    uint64_t a0 = 0, a1 = 0;
#pragma unroll 2
    for (int q = 0; q < RK; q += 2) {
      a0 += (uint64_t)s.xi[q] * mp[q * RKP];
      a1 += (uint64_t)s.xi[q + 1] * mp[(q + 1) * RKP];
    }
    colv = (int64_t)(a0 + a1);
  }
  __syncthreads();
  if (t < RKP) s.col[t] = colv - (int64_t)((uint64_t)s.alpha * S[S_MFULL + t]);
  __syncthreads();
  if (t == 0) {
    const ModDev& md = prime ? key.q2 : key.p2;
    uint32_t v[RKP];
    int64_t cy = 0;
#pragma unroll
    for (int j = 0; j < RKP; ++j) {
      const int64_t a = s.col[j] + cy;
      v[j] = (uint32_t)(a & (int64_t)LMASK);
      cy = a >> 28;  // arithmetic: the columns may be negative before the carries
    }
    // X < 75 N: subtract q N with q = floor(X / N) from the top limbs, then fix up
    double xd = 0.0, nd = 0.0;
#pragma unroll
    for (int j = RKP - 1; j >= K - 4; --j) {
      xd = xd * 268435456.0 + (double)v[j];
      nd = nd * 268435456.0 + (double)(j < K ? md.N[j] : 0u);
    }
    const uint32_t q = (uint32_t)(xd / nd);
    int64_t br = 0;
#pragma unroll
    for (int j = 0; j < RKP; ++j) {
      const int64_t a = (int64_t)v[j] - (int64_t)q * (j < K ? md.N[j] : 0u) + br;
      v[j] = (uint32_t)(a & (int64_t)LMASK);
      br = a >> 28;
    }
    for (int fix = 0; fix < 4; ++fix) {  // q is off by at most one: add N while negative, subtract while >= N
      bool ge = br == 0;
      if (ge)
        for (int j = RKP - 1; j >= 0; --j) {
          const uint32_t nj = j < K ? md.N[j] : 0u;
          if (v[j] != nj) {
            ge = v[j] > nj;
            break;
          }
        }
      if (br == 0 && !ge) break;
      const int64_t sg = br < 0 ? 1 : -1;
      int64_t cr = 0;
      for (int j = 0; j < RKP; ++j) {
        const int64_t a = (int64_t)v[j] + sg * (int64_t)(j < K ? md.N[j] : 0u) + cr;
        v[j] = (uint32_t)(a & (int64_t)LMASK);
        cr = a >> 28;
      }
      br += cr;
    }
    // X - 1 (X = 1 mod P, so X >= 1)
    uint32_t* out = xrows + (size_t)prime * xs4 * count + e;
    int64_t b1 = 1;
    for (int j = 0; j < K; ++j) {
      const int64_t a = (int64_t)v[j] - b1;
      b1 = a < 0 ? 1 : 0;
      out[(size_t)j * count] = (uint32_t)(a + (b1 << 28));
    }
    for (int j = K; j < xs4; ++j) out[(size_t)j * count] = 0u;
  }
#if XHE_RNS_PROBE
  if (blockIdx.x == 0 && blockIdx.y == 0 && (t == 0 || t == 192)) {
    unsigned long long* o = g_rns_probe + (t ? 4 : 0);
    o[0] = pr_d1;
    o[1] = pr_d2;
    o[2] = pr_d3;
    o[3] = pr_n;
    if (t == 0) {
      g_rns_probe[8] = __builtin_amdgcn_s_memtime() - pr_t0;
      g_rns_probe[9] = __builtin_amdgcn_s_memrealtime() - pr_r0;
    }
  }
#endif
#undef RNS_PROBE
}

}  // namespace xhe
