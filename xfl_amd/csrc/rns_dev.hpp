// Small-batch decrypt exponentiation in a residue number system (2048-bit
// keys): X_P = c^(P-1) mod P^2 for one residue per 256-thread block, every
// Montgomery product as two base extensions instead of WaveMont's six LDS
// column phases (dec_wave.hpp; its 1.7 us products set the LR demo's 2.1 ms
// decrypt, paillier.py:341-368 / label_trainer.py:252-259).
//
// A value x < LAM N (N = P^2, LAM = RK + 1) is held as its residues modulo two
// bases of RK = 74 primes below 2^28 - B (threads 0..73) and B' (threads
// 128..201), M, M' ~ 2^2072 - and mod 2^32 (thread 202, the redundant
// channel). One product x y M^-1 mod N (Bajard/Kawamura RNS Montgomery with a
// Shenoy-Kumaresan exact extension):
//   all       t = x y per channel
//   B         xi_i = t_i |-N^-1 M_i^-1|_(m_i)                -> LDS
//   -- barrier --
//   B'        qh'_j = sum_i xi_i |M_i|_(m'_j)  (fast extension: qh = q + alpha M)
//             r'_j = (t'_j + qh'_j N) |M^-1|_(m'_j),  xi'_j = r'_j |M'_j^-1|  -> LDS
//   r         r_r = (t_r + (sum_i xi_i |M_i|_(2^32)) N) M^-1 mod 2^32     -> LDS
//             the B' waves also sum xi'_j |M'_j|_(2^32) (DPP)           -> LDS
//   -- barrier --
//   B         beta = (sum_j xi'_j |M'_j|_(2^32) - r_r) M'^-1 mod 2^32  (exact, < RK)
//             r_i = sum_j xi'_j |M'_j|_(m_i) - beta |M'|_(m_i)
// Each extension is RK = 74 independent 28 x 28-bit mads per thread into four
// 64-bit accumulators (sums < 2^62.3), the operands one broadcast
// ds_read_b128 per 4 terms, the thread's own row of the extension matrix in
// registers. tools/rns_model.py checks the algorithm, the bounds (r < LAM N
// when M >= LAM^2 N; alpha, beta < RK; column sums < 2^63) and the Barrett
// reductions below for every modulus against Python integers.
#pragma once
#include "xhe_kernels.hpp"

namespace xhe {
namespace rns {

constexpr int RK = 74;      // moduli per base
constexpr int RKP = 76;     // padded to whole quads (the extra terms are zero)
constexpr int NT = 256;     // threads per residue
constexpr int RLANE = 202;  // the mod-2^32 channel
constexpr uint32_t LMASK = (1u << 28) - 1u;

// constant blocks (words): shared by every key (the bases), then per prime
constexpr int S_M = 0, S_MU = 256, S_T32 = 512, S_B = 768, S_C = 1024, S_D = 1280, S_ROWS = 1536;
constexpr int S_MPOS = S_ROWS + RKP * NT;  // [RK][RKP] 28-bit limbs of M_i = M / m_i
constexpr int S_MFULL = S_MPOS + RK * RKP;  // [RKP] limbs of M
constexpr int S_M2RINV = S_MFULL + RKP;     // M'^-1 mod 2^32
constexpr int S_WORDS = S_M2RINV + 4;
// per prime: P_A (B: |-N^-1 M_i^-1|; B': |N M^-1|; 2^32: N), P_A2 (B': |N M^-1 M'_j^-1|),
// M^3 mod N per channel, then the exponent P - 1 as a window schedule: P_NS
// entries, [0] = the start value's table index, then (squarings << 8) | (t + 1)
// (t + 1 = 0: no product)
constexpr int P_A = 0, P_A2 = 256, P_M3 = 512, P_NS = 768, P_SCHED = 772, P_SCHED_MAX = 1280;
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
  uint32_t xi[RKP];   // B -> B': xi_i
  uint32_t xi2[RKP];  // B' -> B: xi'_j
  uint32_t part[2];   // per B' wave: sum xi'_j |M'_j|_(2^32)
  uint32_t rr;        // r mod 2^32
  uint32_t alpha;
  int64_t col[RKP];   // exit: the positional columns
};

// sum_i v[i] row[i] over RKP terms: every operand quad read first (in-order
// LDS returns, so each block waits only for its own quad), then four
// independent accumulators, one asm statement per quad (written as plain C
// the compiler folded the four chains into one 76-mad dependency chain)
XHE_DEV uint64_t ext_sum(const uint32_t* v, const uint32_t (&row)[RKP]) {
  uint4 x[RKP / 4];
#pragma unroll
  for (int q = 0; q < RKP / 4; ++q) x[q] = reinterpret_cast<const uint4*>(v)[q];
  uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
#pragma unroll
  for (int q = 0; q < RKP / 4; ++q)
    asm("v_mad_u64_u32 %0, vcc, %4, %8, %0\n\t"
        "v_mad_u64_u32 %1, vcc, %5, %9, %1\n\t"
        "v_mad_u64_u32 %2, vcc, %6, %10, %2\n\t"
        "v_mad_u64_u32 %3, vcc, %7, %11, %3"
        : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3)
        : "v"(x[q].x), "v"(x[q].y), "v"(x[q].z), "v"(x[q].w), "v"(row[4 * q]), "v"(row[4 * q + 1]),
          "v"(row[4 * q + 2]), "v"(row[4 * q + 3])
        : "vcc");
  return (a0 + a1) + (a2 + a3);
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

// k_dec_rns: the same rows as k_dec_wave (X_P = (c^(P-1) mod P^2) - 1,
// [prime][xs4][count], limbs of 28 bits beyond K zero) with the same 5-bit
// sliding-window schedule over P - 1 (16 odd powers, now one register each per
// channel). grid (count, 2): blockIdx.y is the prime.
__global__ void __launch_bounds__(rns::NT) k_dec_rns(KeyDev key, const uint32_t* __restrict__ c_words,
                                                     int64_t count, int xs4, uint32_t* __restrict__ xrows) {
  using namespace rns;
  constexpr int K = 74;  // limbs of 28 bits of P^2 (the MP2 rows)
  __shared__ __attribute__((aligned(16))) Lds s;
  const int t = (int)threadIdx.x;
  const int prime = blockIdx.y;
  const int64_t e = blockIdx.x;
  const bool gB = t < 128;                     // waves 0, 1: base B; waves 2, 3: base B' and the 2^32 channel
  const int ch = gB ? t : t - 128;
  const bool isr = t == RLANE;
  const bool act = ch < RK || isr;
  const uint32_t* S = key.rns;
  const uint32_t* Pb = prime ? key.rns_q : key.rns_p;
  Chan c;
  c.m = S[S_M + t];
  c.mu = S[S_MU + t];
  c.t32 = S[S_T32 + t];
  c.r32 = isr;
  const uint32_t cb = S[S_B + t], cc = S[S_C + t], cd = S[S_D + t], m2rinv = S[S_M2RINV];
  const uint32_t ca = Pb[P_A + t], ca2 = Pb[P_A2 + t], m3 = Pb[P_M3 + t];
  uint32_t row[RKP];
#pragma unroll
  for (int i = 0; i < RKP; ++i) row[i] = S[S_ROWS + i * NT + t];
  if (t < RKP) {
    s.xi[t] = 0u;
    s.xi2[t] = 0u;
  }
  __syncthreads();

  // x y M^-1 mod N in every channel (two barriers; the roles are wave-uniform).
  // B' lanes: r' = t |M^-1| + qh |N M^-1| and xi' = t |M^-1 M'_j^-1| + qh
  // |N M^-1 M'_j^-1|, the t terms taken before the barrier, so after the
  // extension only two independent products remain on the critical path.
  auto mul = [&](uint32_t x, uint32_t y) -> uint32_t {
    const uint32_t tt = c.mul(x, y);
    uint32_t tm = 0u, ta = 0u;
    if (gB) {
      if (act) s.xi[ch] = c.mul(tt, ca);  // ca = |-N^-1 M_i^-1|
    } else if (!isr) {
      tm = c.mul(tt, cb);  // cb = |M^-1|
      ta = c.mul(tt, cc);  // cc = |M^-1 M'_j^-1|
    }
    __syncthreads();
    uint32_t res = 0u;
    if (!gB) {
      const uint64_t acc = ext_sum(s.xi, row);
      uint32_t u = 0u;
      if (isr) {  // ca = N mod 2^32, cb = M^-1 mod 2^32
        res = (tt + (uint32_t)acc * ca) * cb;
        s.rr = res;
      } else {    // ca = |N M^-1|, ca2 = |N M^-1 M'_j^-1|, cd = |M'_j|_(2^32)
        const uint32_t qh = red64(acc, c.m, c.mu, c.t32);
        res = c.add(tm, c.mul(qh, ca));
        const uint32_t x2 = c.add(ta, c.mul(qh, ca2));
        if (act) {
          s.xi2[ch] = x2;
          u = x2 * cd;
        }
      }
      const uint32_t sum = wave_sum(u);
      if ((t & 63) == 0) s.part[(t >> 6) - 2] = sum;
    }
    __syncthreads();
    if (gB) {  // cb = |M'|_(m_i)
      const uint64_t acc = ext_sum(s.xi2, row);
      const uint32_t beta = (s.part[0] + s.part[1] - s.rr) * m2rinv;
      const uint32_t d = red64(acc, c.m, c.mu, c.t32) - c.mul(beta, cb);
      res = min(d, d + c.m);
    }
    return res;
  };

  // c mod m_i from the ciphertext words (Horner from the top word), then
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
  // odd powers x, x^3 .. x^31 (registers: the loop is unrolled)
  uint32_t tab[16];
  tab[0] = x;
  const uint32_t x2 = mul(x, x);
#pragma unroll
  for (int k = 1; k < 16; ++k) tab[k] = mul(tab[k - 1], x2);
  auto pick = [&](uint32_t v) {  // tab[v] for a wave-uniform v (no dynamic register indexing)
    uint32_t r = tab[0];
#pragma unroll
    for (int k = 1; k < 16; ++k) r = v == (uint32_t)k ? tab[k] : r;
    return r;
  };
  // the 5-bit sliding-window schedule over P - 1, precomputed per key
  // (scalar loads, one per window)
  const uint32_t* sc = Pb + P_SCHED;
  const int ns = (int)Pb[P_NS];
  x = pick(sc[0]);
#pragma unroll 1
  for (int k = 1; k < ns; ++k) {
    const uint32_t w = sc[k];
#pragma unroll 1
    for (uint32_t q = w >> 8; q; --q) x = mul(x, x);
    if (w & 0xFFu) x = mul(x, pick((w & 0xFFu) - 1u));
  }
  x = mul(x, 1u);  // out of Montgomery form: X < LAM N, X = c^(P-1) mod N

  // exit: X = sum_i xi_i M_i - alpha M (xi_i = X_i |M_i^-1|, alpha from the
  // 2^32 channel), as 28-bit columns, then reduced mod N by thread 0
  if (gB && act) s.xi[ch] = c.mul(x, cc);  // cc = |M_i^-1|
  __syncthreads();
  if (isr) s.alpha = ((uint32_t)ext_sum(s.xi, row) - x) * cb;  // cb = M^-1 mod 2^32
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
}

}  // namespace xhe
