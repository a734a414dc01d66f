// One-wave decrypt exponentiation for small batches (2048-bit keys).
//
// k_dec_pow spreads a residue's Montgomery product over at most one 16-lane
// DPP row: its K-step operand-scanning loop is a chain of dependent
// quotient digits (mad -> mul -> row broadcast -> hand-down), ~130 cycles a
// step, and a 15-element decrypt (the LR demo's batch, SURVEY.md cfg 1) waits
// ~1,210 such products. Here a whole 64-lane wave works on one residue
// mod P^2 and the product has no serial digit chain:
//
//   T = a b          column sums, lane l owns columns l and l + K
//   m = (T mod R) N' mod R          (N' = -N^-1 mod R, low columns only)
//   x = (T + m N) / R               exact: U = T + m N = 0 (mod R)
//
// (Montgomery's REDC as three column products, R = 2^(28 K); the same limbs
// and R as the one-lane MP2 shape Mont<74, 28, 1>, so the rows it writes are
// k_dec_pow's.) Column c of a b is sum_t a_t b_(c-t): with the multiplicand
// stored zero-padded in LDS as Z = (0^K, b, 0^K), lane l accumulates
// a_t Z[K + l - t] (column l) and a_t Z[2K + l - t] (column l + K) for t =
// 0..K-1 - wave-uniform a_t (an LDS broadcast), immediate LDS offsets, no
// selects, K terms per pair. Pairs l >= 64 (K = 74: ten of them) are cut
// into chunks of CH terms spread over the threads and added in with LDS
// atomics.
//
// Column sums are lazy 64-bit (74 products below 2^56 + carries < 2^64) and
// normalised by passes that move each column's upper bits one and two limbs
// up (no carry chain): limbs end at most MASK + 2, which keeps the next
// product's columns in range. Dropping what crosses limb K - 1 keeps a value
// mod R (m and T mod R need no more); the exact U / R needs only whether the
// low part's remainder is 0 or R after two passes - one ballot. Ranges: inputs
// < 2N (R > 2^24 N), so T / R < N / 2^22, m < R (1 + 2^-26) and U / R < 2N.
#pragma once
#include "bn_dev.hpp"

namespace xhe {

#ifndef XHE_WAVE_PROF
#define XHE_WAVE_PROF 0  // dev builds: cycles per phase of block (0, 0), printed at the end
#endif
#if XHE_WAVE_PROF
__device__ unsigned long long g_wave_prof[8];
__device__ unsigned long long g_wave_t;
#define XHE_WAVE_T(ph)                                                         \
  do {                                                                         \
    if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0) {              \
      const unsigned long long now_ = clock64();                               \
      if ((ph) >= 0) g_wave_prof[(ph)] += now_ - g_wave_t;                     \
      g_wave_t = now_;                                                         \
    }                                                                          \
  } while (0)
#else
#define XHE_WAVE_T(ph) \
  do {                 \
  } while (0)
#endif

// NWV waves per residue (NT threads). A product's columns are summed by
// thread (q, s): columns 4q..4q+3 over terms t in [s TS, (s+1) TS), NQF
// column quads of the full product (NQL of the low-only quotient product) by
// NS term slices, added into the LDS columns with 64-bit LDS atomics. Thread
// (q, s) reads its TS/4 quads of a and TS/4 + 1 aligned quads of the
// zero-padded multiplicand (term quads u and u + 1 share one): 9 LDS reads
// for 64 mads, all in flight at once. The slices run past K (a is zero there)
// and the quads past the triangle of nonzero terms (z is zero there): 2.2x
// the mads of the exact column sums, cheap next to the LDS round trips that
// set a product's latency.
template <int K, int NWV, int W_ = 28>
struct WaveMont {
  static constexpr int W = W_;  // 28 mod P^2 (k_dec_wave); 27 mod n^2 (k_mexp_horner_wave: 2K W-bit
                                // products per column stay below 2^64 at K = 154)
  static constexpr int K_ = K;
  static constexpr uint32_t MASK = (1u << W) - 1u;
  static constexpr int NT = 64 * NWV;  // threads per residue
  // terms per slice: 8 when the threads hold every (quad, 8-term slice), else 16
  static constexpr int TS = ((2 * K - 1 + 3) / 4) * ((K + 7) / 8) <= NT ? 8 : 16;
  static constexpr int NS = (K + TS - 1) / TS;
  static constexpr int NQF = (2 * K - 1 + 3) / 4, NQL = (K + 3) / 4;
  static_assert(NQF * NS <= NT, "one (quad, slice) per thread");
  static_assert(K < NT, "one limb per thread in the passes");
  static constexpr int KP = (NS * TS + 3) & ~3;  // operand rows, zero from K to the last slice's end
  static constexpr int G = 3;                    // zero guards below column 0
  // multiplicand rows Z: b at [ZO, ZO + K), zeros around it (reads reach
  // ZO - NS TS - 4 .. ZO + 4 NQF)
  static constexpr int ZO = (NS * TS + 4 + 3) & ~3;
  static constexpr int ZS = (ZO + 4 * NQF + 4 + 3) & ~3;

  struct Lds {  // operand rows first: 16-byte aligned for the broadcast quad reads
    uint32_t x[KP], r3[KP], one[KP], tl[KP], mq[KP];
    uint32_t tab[16][KP];  // odd powers x^(2t+1)
    uint32_t zb[ZS];   // (0^ZO, b, 0...): the multiplicand of the next product
    uint32_t zn[ZS];   // N, Z-padded (m N)
    uint32_t znp[ZS];  // N' = -N^-1 mod R, Z-padded (m = T N')
    uint64_t col[2][G + 2 * K];  // column sums (T, then U = T + m N); two buffers, one zeroed ahead
    uint64_t mcol[G + 4 * NQL];  // columns of m
    uint32_t exw[64];            // the exponent P - 1 (<= 2048 bits)
  };

  static XHE_DEV int tid() { return (int)threadIdx.x; }
  static XHE_DEV void sync() { __syncthreads(); }

  // acc[i] += a_r z[4 + i - r] for r, i < 4: one term quad of a column quad,
  // 16 mads in one statement (a hazard nop follows every asm statement; the
  // same accumulator recurs every 4 mads)
  static XHE_DEV void mad16(uint64_t (&acc)[4], const uint32_t (&a)[4], const uint32_t (&z)[8]) {
    asm("v_mad_u64_u32 %0, vcc, %4, %12, %0\n\t"
        "v_mad_u64_u32 %1, vcc, %4, %13, %1\n\t"
        "v_mad_u64_u32 %2, vcc, %4, %14, %2\n\t"
        "v_mad_u64_u32 %3, vcc, %4, %15, %3\n\t"
        "v_mad_u64_u32 %0, vcc, %5, %11, %0\n\t"
        "v_mad_u64_u32 %1, vcc, %5, %12, %1\n\t"
        "v_mad_u64_u32 %2, vcc, %5, %13, %2\n\t"
        "v_mad_u64_u32 %3, vcc, %5, %14, %3\n\t"
        "v_mad_u64_u32 %0, vcc, %6, %10, %0\n\t"
        "v_mad_u64_u32 %1, vcc, %6, %11, %1\n\t"
        "v_mad_u64_u32 %2, vcc, %6, %12, %2\n\t"
        "v_mad_u64_u32 %3, vcc, %6, %13, %3\n\t"
        "v_mad_u64_u32 %0, vcc, %7, %9, %0\n\t"
        "v_mad_u64_u32 %1, vcc, %7, %10, %1\n\t"
        "v_mad_u64_u32 %2, vcc, %7, %11, %2\n\t"
        "v_mad_u64_u32 %3, vcc, %7, %12, %3"
        : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])
        : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(z[0]), "v"(z[1]), "v"(z[2]), "v"(z[3]), "v"(z[4]),
          "v"(z[5]), "v"(z[6]), "v"(z[7])
        : "vcc");
  }

  // limb j of the three-way split of columns (exact: sum lim_j 2^(W j) = sum col_j 2^(W j))
  static XHE_DEV uint32_t split3(const uint64_t* cg, int j) {
    const uint64_t c0 = cg[j], c1 = cg[j - 1], c2 = cg[j - 2];
    return ((uint32_t)c0 & MASK) + ((uint32_t)(c1 >> W) & MASK) + (uint32_t)(c2 >> (2 * W));
  }
  // limb j after a second pass (<= MASK + 2); cg = col + G, j >= 0
  static XHE_DEV uint32_t norm(const uint64_t* cg, int j) {
    return (split3(cg, j) & MASK) + (split3(cg, j - 1) >> W);
  }
  // col += a x b over quad columns (see TS above): thread (q, s) reads its
  // slice of a as TS/4 quads and the multiplicand as TS/4 + 1 aligned quads
  // (consecutive term quads share one), 4 TS mads into four accumulators
  // (one per column), then one LDS atomic per column. LO: columns < K + 2
  // only (the quotient product; its columns from K on are never read).
  // ZERO: the idle threads zero the other column buffer (last read by the
  // previous product's tail, next written by the next product).
  template <bool LO>
  static XHE_DEV void prodq(const uint32_t* a, const uint32_t* z, uint64_t* col, uint64_t* zero = nullptr) {
    constexpr int NQ = LO ? NQL : NQF;
    const int q = tid() % NQ, sl = tid() / NQ;
    if (sl < NS) {
      const int t0 = sl * TS;
      uint4 av[TS / 4], zq[TS / 4 + 1];
#pragma unroll
      for (int u = 0; u < TS / 4; ++u) av[u] = *reinterpret_cast<const uint4*>(a + t0 + 4 * u);
      // quad u of terms needs Z[B_u - 4 .. B_u + 3], B_u = ZO + 4q - t0 - 4u:
      // zq[u + 1] = Z[B_u - 4 ..], zq[u] = Z[B_u ..]
      const uint32_t* zb0 = z + (ZO + 4 * q - t0);
#pragma unroll
      for (int u = 0; u <= TS / 4; ++u) zq[u] = *reinterpret_cast<const uint4*>(zb0 - 4 * u);
      // two accumulator sets (term quads alternate), so one quad's mads do
      // not wait on the previous quad's
      uint64_t acc[2][4] = {{0ull, 0ull, 0ull, 0ull}, {0ull, 0ull, 0ull, 0ull}};
#pragma unroll
      for (int u = 0; u < TS / 4; ++u) {
        const uint32_t zz[8] = {zq[u + 1].x, zq[u + 1].y, zq[u + 1].z, zq[u + 1].w,
                                zq[u].x,     zq[u].y,     zq[u].z,     zq[u].w};  // Z[B_u - 4 + k]
        const uint32_t at[4] = {av[u].x, av[u].y, av[u].z, av[u].w};
        mad16(acc[u & 1], at, zz);  // column 4q + i, term t0 + 4u + r: Z[B_u + i - r]
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
        atomicAdd((unsigned long long*)&col[G + 4 * q + i], (unsigned long long)(acc[0][i] + acc[1][i]));
    } else if (zero) {
      for (int i = tid() - NQ * NS; i < 2 * K; i += NT - NQ * NS) zero[G + i] = 0ull;
    }
    sync();
  }

  // dst = U / R from the columns of U = T + m N (= 0 mod R). The low part reduced
  // twice, L = sum v_j 2^(W j) (v_j <= MASK + 2), is 0 or R; if R then
  // v_(K-1) >= MASK - 1 (the limbs below sum to < 2^(W (K-1)) (1 + 3/MASK)),
  // else every v_j is 0: the carry out of the low part is v_(K-1) != 0, which
  // every thread reads for itself (no ballot).
  // (the threads from K on zero mcol: last read by this product's U phase,
  // next written by the next product's quotient)
  static XHE_DEV void tail(Lds& s, int cur, uint32_t* dst, bool zbw) {
    const uint64_t* cg = s.col[cur] + G;
    const uint32_t k = norm(cg, K - 1) != 0u ? 1u : 0u;
    const uint32_t e0 = (split3(cg, K - 1) >> W) + k;  // into limb 0 of U / R
    for (int i = tid(); i < K; i += NT) {
      const uint32_t hi = split3(cg, K + i) + (i == 0 ? e0 : 0u);
      const uint32_t hp = i == 0 ? 0u : split3(cg, K + i - 1) + (i == 1 ? e0 : 0u);
      const uint32_t v = (hi & MASK) + (hp >> W);
      dst[i] = v;
      if (zbw) s.zb[ZO + i] = v;
    }
    for (int i = tid() - K; i >= 0 && i < 4 * NQL; i += NT - K) s.mcol[G + i] = 0ull;
    sync();
  }

  // out = columns [0, K) mod R as limbs <= MASK + 2
  static XHE_DEV void norm_low(const uint64_t* col, uint32_t* out) {
    for (int j = tid(); j < K; j += NT) out[j] = norm(col + G, j);
    sync();
  }
  // the same for T (the first pass of a product); the threads beyond K zero
  // the other column buffer (last read by the previous product's tail, next
  // written by the next product) and mcol (last read by the previous
  // product, next written by this one's quotient product)
  static XHE_DEV void norm_low_t(Lds& s, int cur) {
    const int j = tid();
    if (j < K) {
      s.tl[j] = norm(s.col[cur] + G, j);
    } else {
      for (int i = j - K; i < 2 * K; i += NT - K) s.col[cur ^ 1][G + i] = 0ull;
      for (int i = j - K; i < 4 * NQL; i += NT - K) s.mcol[G + i] = 0ull;
    }
    sync();
  }

  // dst = REDC(T), T in s.col[cur] (< R N): T R^-1 mod N (< 2N): T's low
  // limbs, the quotient product m = (T mod R) N' mod R, m's limbs, the U
  // product, the tail (five LDS phases after T's own)
  static XHE_DEV void reduce(Lds& s, int cur, uint32_t* dst, bool zbw) {
    norm_low_t(s, cur);
    prodq<true>(s.tl, s.znp, s.mcol);  // m = (T mod R) N' mod R
    XHE_WAVE_T(1);
    norm_low(s.mcol, s.mq);
    prodq<false>(s.mq, s.zn, s.col[cur]);  // U = T + m N
    XHE_WAVE_T(2);
    tail(s, cur, dst, zbw);
    XHE_WAVE_T(3);
  }

  // dst = a b R^-1 mod N (< 2N), b in s.zb; zbw: the result also becomes the
  // next multiplicand. cur flips (the product's columns go to the zeroed buffer).
  static XHE_DEV void mul(Lds& s, int& cur, const uint32_t* a, uint32_t* dst, bool zbw) {
    cur ^= 1;
    XHE_WAVE_T(-1);
    prodq<false>(a, s.zb, s.col[cur]);
    XHE_WAVE_T(0);
    reduce(s, cur, dst, zbw);
  }

  static XHE_DEV void copy_in(uint32_t* dst, const uint32_t* src, int n) {
    for (int j = tid(); j < n; j += NT) dst[j] = src[j];
  }
};

#ifndef XHE_DEC_NWV
#define XHE_DEC_NWV 4  // waves per residue of k_dec_wave
#endif

// k_dec_wave: X_P = (c^(P-1) mod P^2) - 1 for one residue per block of NWV
// waves (grid (count, 2): blockIdx.y is the prime), rows as k_dec_pow<MP2, 0>
// writes them ([prime][xs4][count], limbs beyond K zero). Same window
// schedule as pow_uniform_exp (5-bit sliding window over P - 1, 16 odd powers
// in LDS), one product site.
template <int K, int NWV>
__global__ void __launch_bounds__(64 * NWV) k_dec_wave(KeyDev key, const uint32_t* __restrict__ c_words,
                                                       int64_t count, int xs4, uint32_t* __restrict__ xrows) {
  using WM = WaveMont<K, NWV>;
  constexpr uint32_t MASK = WM::MASK;
#if XHE_WAVE_PROF
  if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0) {
    for (int q = 0; q < 7; ++q) g_wave_prof[q] = 0;
    g_wave_prof[7] = clock64();
  }
#endif
  constexpr int NT = WM::NT;
  __shared__ __attribute__((aligned(16))) typename WM::Lds s;
  const int l = WM::tid();
  const int prime = blockIdx.y;
  const int64_t e = blockIdx.x;
  const ModDev& md = prime ? key.q2 : key.p2;
  const uint32_t* np = prime ? key.q2_nprime : key.p2_nprime;
  const uint32_t* ex = prime ? key.qm1_words : key.pm1_words;
  const int ebits = prime ? key.qm1_bits : key.pm1_bits;
  {
    uint32_t* w = reinterpret_cast<uint32_t*>(&s);
    for (int j = l; j < (int)(sizeof(s) / 4); j += NT) w[j] = 0u;
  }
  WM::sync();
  for (int j = l; j < K; j += NT) {
    s.zn[WM::ZO + j] = md.N[j];
    s.znp[WM::ZO + j] = np[j];
    s.r3[j] = md.R3[j];
  }
  if (l == 0) s.one[0] = 1u;
  for (int j = l; j < (ebits + 31) / 32 && j < 64; j += NT) s.exw[j] = ex[j];
  int cur = 0;
  {  // c (n2w words, < 2^(28 * 2K)) as 2K limbs in the columns
    const uint32_t* cw = c_words + (size_t)e * key.n2w;
    const int n2w = key.n2w;
    for (int j = l; j < 2 * K; j += NT) {
      const int bit = 28 * j, k = bit >> 5, sh = bit & 31;
      const uint32_t lo = word_or0(cw, k, n2w), hw = word_or0(cw, k + 1, n2w);
      s.col[cur][WM::G + j] = (uint32_t)((((uint64_t)hw << 32) | lo) >> sh) & MASK;
    }
  }
  WM::sync();
  WM::reduce(s, cur, s.x, true);  // c R^-1 mod P^2

  // exponent bits k in (32 (wi - 1), 32 wi + 31] from two words (wi = i >> 5)
  auto bits64 = [&](int i, int& base) {
    const int wi = i >> 5;
    base = (wi - 1) * 32;
    return ((uint64_t)s.exw[wi] << 32) | (wi > 0 ? s.exw[wi - 1] : 0u);
  };
  int i = ebits - 1;
  while (i >= 0 && !((ex[i >> 5] >> (i & 31)) & 1u)) --i;
  int step = 0, pend_sq = 0, pend_mul = -1;
  bool fin = false;
#pragma unroll 1
  while (true) {
    const uint32_t* a;
    uint32_t* dst = s.x;
    bool zbw = true;
    if (step == 0) {  // c R^-1 R^3 R^-1 = c R
      a = s.r3;
      step = 1;
    } else if (step == 1) {  // tab[0] = x; x = zb = x^2
      WM::copy_in(s.tab[0], s.x, K);
      WM::sync();
      a = s.x;
      step = 2;
    } else if (step < 17) {  // tab[t] = tab[t-1] x^2 (x^2 stays in zb)
      a = s.tab[step - 2];
      dst = s.tab[step - 1];
      zbw = false;
      ++step;
    } else if (pend_sq > 0) {
      a = s.x;
      --pend_sq;
    } else if (pend_mul >= 0) {
      a = s.tab[pend_mul];
      pend_mul = -1;
    } else if (i >= 0) {
      int base;
      const uint64_t v = bits64(i, base);
      auto bit = [&](int k) { return (uint32_t)(v >> (k - base)) & 1u; };
      if (step == 17 || bit(i)) {  // a window [i..j] ending in a set bit
        int j = i - 4 < 0 ? 0 : i - 4;
        while (!bit(j)) ++j;
        uint32_t val = 0;
        for (int k = i; k >= j; --k) val = (val << 1) | bit(k);
        if (step == 17) {  // the first window's odd power is the start value
          WM::copy_in(s.x, s.tab[val >> 1], K);
          WM::copy_in(s.zb + WM::ZO, s.tab[val >> 1], K);
          WM::sync();
          step = 18;
        } else {
          pend_sq = i - j + 1;
          pend_mul = (int)(val >> 1);
        }
        i = j - 1;
      } else {
        pend_sq = 1;
        --i;
      }
      continue;
    } else if (!fin) {  // x R^-1: out of Montgomery form
      a = s.one;
      fin = true;
    } else {
      break;
    }
    WM::mul(s, cur, a, dst, zbw);
  }

  // x < 2N in limbs <= MASK + 2: normalise, subtract N once if x >= N, then
  // X = x - 1 mod 2^(28 K) (x = 1 mod P), written by thread 0
  if (l == 0) {
    uint32_t v[K];
    uint32_t cy = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t t = s.x[j] + cy;
      v[j] = t & MASK;
      cy = t >> 28;
    }
    int64_t br = 0;
    uint32_t d[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const int64_t t = (int64_t)v[j] - (int64_t)md.N[j] - br;
      br = t < 0 ? 1 : 0;
      d[j] = (uint32_t)(t + (br << 28));
    }
    const bool ge = br == 0;
    br = 1;  // minus one
    uint32_t* out = xrows + (size_t)prime * xs4 * count + e;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const int64_t t = (int64_t)(ge ? d[j] : v[j]) - br;
      br = t < 0 ? 1 : 0;
      out[(size_t)j * count] = (uint32_t)(t + (br << 28));
    }
    for (int j = K; j < xs4; ++j) out[(size_t)j * count] = 0u;
#if XHE_WAVE_PROF
    if (blockIdx.x == 0 && blockIdx.y == 0)
      printf("wave prof (cycles, all products): prod1 %llu prod2 %llu prod3 %llu tail %llu total %llu\n",
             g_wave_prof[0], g_wave_prof[1] - 0, g_wave_prof[2], g_wave_prof[3], clock64() - g_wave_prof[7]);
#endif
  }
}

}  // namespace xhe

namespace xhe {

// ---------------------------------------------------------------------------
// Horner of the encrypted mat-vec (k_mexp_horner) with one block of NWV waves
// per column, for the small batches of the LR step (2048-bit keys; the
// 16-lane shape's P rows). out[j] = prod_w P[j][w]^(2^(c w)) is a chain of
// ~kbits squarings and nwin - 1 products - latency, ~10 us per product in the
// 16-lane shape - so here each product is WaveMont's column product (4 LDS
// phases, no serial digit chain) mod n^2 in 154 limbs of 27 bits (R_w =
// 2^4158). The P rows are Montgomery rows of the 16-lane shape (P R_X, R_X =
// 2^(27*160), limbs of the same 27 bits, canonical so limbs from 154 on are
// zero): MontW(P R_X, C) with C = R_w^2 R_X^-1 mod n^2 puts P into wave form,
// and a window product is MontW(MontW(acc, P R_X), C) = acc P (wave form).
// Out: MontW(1, acc) = the plain product (< 2N), normalised, reduced once and
// packed to n2w words by one thread.
template <int K, int NWV>
__global__ void __launch_bounds__(64 * NWV) k_mexp_horner_wave(KeyDev key, const uint32_t* __restrict__ P, int nwin,
                                                               int c, int64_t ncols, uint32_t* __restrict__ out) {
  using WM = WaveMont<K, NWV, 27>;
  constexpr uint32_t MASK = WM::MASK;
  constexpr int NT = WM::NT;
  __shared__ __attribute__((aligned(16))) typename WM::Lds s;
  const int l = WM::tid();
  const int64_t j = blockIdx.x;
  {
    uint32_t* w = reinterpret_cast<uint32_t*>(&s);
    for (int i = l; i < (int)(sizeof(s) / 4); i += NT) w[i] = 0u;
  }
  WM::sync();
  for (int i = l; i < K; i += NT) {
    s.zn[WM::ZO + i] = key.n2w_N[i];
    s.znp[WM::ZO + i] = key.n2w_np[i];
    s.r3[i] = key.n2w_C[i];  // C = R_w^2 R_X^-1 (the a-operand of the second window product)
    s.zb[WM::ZO + i] = key.n2w_C[i];
  }
  if (l == 0) s.one[0] = 1u;
  const int64_t pst = ncols * nwin;  // P: [limb][ncols * nwin], column j's window w at j * nwin + w
  auto load_p = [&](int w) {
    const uint32_t* pj = P + j * nwin + w;
    for (int i = l; i < K; i += NT) s.tl[i] = pj[(size_t)i * pst];
  };
  load_p(nwin - 1);
  WM::sync();
  int cur = 0;
  WM::mul(s, cur, s.tl, s.x, true);  // P_top R_X C / R_w = P_top R_w
  for (int w = nwin - 2; w >= 0; --w) {
#pragma unroll 1
    for (int r = 0; r < c; ++r) WM::mul(s, cur, s.x, s.x, true);  // acc^2 (a = zb = acc)
    load_p(w);
    WM::sync();
    WM::mul(s, cur, s.tl, s.x, true);  // acc P R_X / R_w
    WM::mul(s, cur, s.r3, s.x, true);  // * C / R_w: acc P (wave form)
  }
  WM::mul(s, cur, s.one, s.x, false);  // plain, < 2N, limbs <= MASK + 2
  if (l == 0) {
    // normalise, subtract N once if x >= N, pack to n2w words
    uint32_t cy = 0;
    for (int i = 0; i < K; ++i) {
      const uint32_t t = s.x[i] + cy;
      s.x[i] = t & MASK;
      cy = t >> WM::W;
    }
    int64_t br = 0;
    for (int i = 0; i < K; ++i) br = ((int64_t)s.x[i] - (int64_t)s.zn[WM::ZO + i] + br) >> WM::W;
    if (br == 0) {  // x >= N
      br = 0;
      for (int i = 0; i < K; ++i) {
        const int64_t t = (int64_t)s.x[i] - (int64_t)s.zn[WM::ZO + i] + br;
        s.x[i] = (uint32_t)t & MASK;
        br = t >> WM::W;
      }
    }
    uint32_t* o = out + (size_t)j * key.n2w;
    uint64_t acc = 0;
    int have = 0, wi = 0;
    for (int i = 0; i < K && wi < key.n2w; ++i) {
      acc |= (uint64_t)s.x[i] << have;
      have += WM::W;
      while (have >= 32 && wi < key.n2w) {
        o[wi++] = (uint32_t)acc;
        acc >>= 32;
        have -= 32;
      }
    }
    while (wi < key.n2w) {
      o[wi++] = (uint32_t)acc;
      acc >>= 32;
    }
  }
}


// Ciphertext add with exponent alignment for small batches (2048-bit keys; the
// LR step's "+ noise", paillier.py:106-123, 79-86): out = x^(2^d) y mod n^2
// with x the operand of larger exponent, d its gap - a chain of d squarings
// (~10 us each in the 16-lane shape) - here one block of NWV waves per
// element: x R_w = MontW(x, R_w^2 mod n^2), d squarings, MontW(x^(2^d) R_w,
// y) = x^(2^d) y (plain), normalised and packed by one thread. eout = the
// smaller exponent (as k_mulmod_n2).
template <int K, int NWV>
__global__ void __launch_bounds__(64 * NWV) k_mulmod_wave(KeyDev key, const uint32_t* __restrict__ a,
                                                          const int32_t* __restrict__ ea, const uint32_t* __restrict__ b,
                                                          const int32_t* __restrict__ eb, int64_t count,
                                                          uint32_t* __restrict__ out, int32_t* __restrict__ eout) {
  using WM = WaveMont<K, NWV, 27>;
  constexpr uint32_t MASK = WM::MASK;
  constexpr int NT = WM::NT;
  __shared__ __attribute__((aligned(16))) typename WM::Lds s;
  const int l = WM::tid();
  const int64_t e = blockIdx.x;
  {
    uint32_t* w = reinterpret_cast<uint32_t*>(&s);
    for (int i = l; i < (int)(sizeof(s) / 4); i += NT) w[i] = 0u;
  }
  WM::sync();
  const int e1 = ea ? ea[e] : 0, e2 = eb ? eb[e] : 0;
  const bool xb = e2 > e1;
  const int d = (xb ? e2 - e1 : e1 - e2);
  const uint32_t* xw = (xb ? b : a) + (size_t)e * key.n2w;
  const uint32_t* yw = (xb ? a : b) + (size_t)e * key.n2w;
  // W-bit limbs of x into tl (a-operand), y into r3, R_w^2 into the multiplicand
  auto limbs = [&](const uint32_t* wv, uint32_t* dst) {
    for (int i = l; i < K; i += NT) {
      const int bit = WM::W * i, k = bit >> 5, sh = bit & 31;
      const uint32_t lo = word_or0(wv, k, key.n2w), hi = word_or0(wv, k + 1, key.n2w);
      dst[i] = (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) & MASK;
    }
  };
  limbs(xw, s.tl);
  limbs(yw, s.r3);
  for (int i = l; i < K; i += NT) {
    s.zn[WM::ZO + i] = key.n2w_N[i];
    s.znp[WM::ZO + i] = key.n2w_np[i];
    s.zb[WM::ZO + i] = key.n2w_R2[i];
  }
  WM::sync();
  int cur = 0;
  WM::mul(s, cur, s.tl, s.x, true);  // x R_w
#pragma unroll 1
  for (int r = 0; r < d; ++r) WM::mul(s, cur, s.x, s.x, true);  // squarings (a = zb = x)
  WM::mul(s, cur, s.r3, s.x, false);  // y x^(2^d) R_w / R_w: plain, < 2N
  if (l == 0) {
    uint32_t cy = 0;
    for (int i = 0; i < K; ++i) {
      const uint32_t t = s.x[i] + cy;
      s.x[i] = t & MASK;
      cy = t >> WM::W;
    }
    int64_t br = 0;
    for (int i = 0; i < K; ++i) br = ((int64_t)s.x[i] - (int64_t)s.zn[WM::ZO + i] + br) >> WM::W;
    if (br == 0) {
      br = 0;
      for (int i = 0; i < K; ++i) {
        const int64_t t = (int64_t)s.x[i] - (int64_t)s.zn[WM::ZO + i] + br;
        s.x[i] = (uint32_t)t & MASK;
        br = t >> WM::W;
      }
    }
    uint32_t* o = out + (size_t)e * key.n2w;
    uint64_t acc = 0;
    int have = 0, wi = 0;
    for (int i = 0; i < K && wi < key.n2w; ++i) {
      acc |= (uint64_t)s.x[i] << have;
      have += WM::W;
      while (have >= 32 && wi < key.n2w) {
        o[wi++] = (uint32_t)acc;
        acc >>= 32;
        have -= 32;
      }
    }
    while (wi < key.n2w) {
      o[wi++] = (uint32_t)acc;
      acc >>= 32;
    }
    if (eout) eout[e] = e1 < e2 ? e1 : e2;
  }
}


// ---------------------------------------------------------------------------
// Batch inversion mod n^2 for small batches (2048-bit keys, up to 256
// elements: the LR step's bases with negative coefficients) as a product
// tree of whole-block WaveMont products, one block per node and one launch
// per level: the tree's latency is its depth in products (~5 us each), not
// the 16-lane shape's ~25 us per product (the round-4 single-block sweeps).
// Nodes are kept in wave-limb form (K limbs of 27 bits) times R_w; the root
// leaves in plain words for the host's inverse and comes back the same way.
template <class WM>
XHE_DEV void wave_init_n2(typename WM::Lds& s, const KeyDev& key) {
  uint32_t* w = reinterpret_cast<uint32_t*>(&s);
  for (int i = WM::tid(); i < (int)(sizeof(s) / 4); i += WM::NT) w[i] = 0u;
  WM::sync();
  for (int i = WM::tid(); i < WM::K_; i += WM::NT) {
    s.zn[WM::ZO + i] = key.n2w_N[i];
    s.znp[WM::ZO + i] = key.n2w_np[i];
  }
}
// limbs of a packed residue (nwords words)
template <class WM>
XHE_DEV void wave_limbs_in(const uint32_t* __restrict__ wv, int nwords, uint32_t* dst) {
  for (int i = WM::tid(); i < WM::K_; i += WM::NT) {
    const int bit = WM::W * i, k = bit >> 5, sh = bit & 31;
    const uint32_t lo = word_or0(wv, k, nwords), hi = word_or0(wv, k + 1, nwords);
    dst[i] = (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) & WM::MASK;
  }
}
// x (< 2N, limbs <= MASK + 2) -> x mod N packed into nwords words, by thread 0
template <class WM>
XHE_DEV void wave_words_out(uint32_t* x, const uint32_t* zn, int nwords, uint32_t* __restrict__ o) {
  constexpr int K = WM::K_;
  if (WM::tid() != 0) return;
  uint32_t cy = 0;
  for (int i = 0; i < K; ++i) {
    const uint32_t t = x[i] + cy;
    x[i] = t & WM::MASK;
    cy = t >> WM::W;
  }
  int64_t br = 0;
  for (int i = 0; i < K; ++i) br = ((int64_t)x[i] - (int64_t)zn[WM::ZO + i] + br) >> WM::W;
  if (br == 0) {  // x >= N
    for (int i = 0; i < K; ++i) {
      const int64_t t = (int64_t)x[i] - (int64_t)zn[WM::ZO + i] + br;
      x[i] = (uint32_t)t & WM::MASK;
      br = t >> WM::W;
    }
  }
  uint64_t acc = 0;
  int have = 0, wi = 0;
  for (int i = 0; i < K && wi < nwords; ++i) {
    acc |= (uint64_t)x[i] << have;
    have += WM::W;
    while (have >= 32 && wi < nwords) {
      o[wi++] = (uint32_t)acc;
      acc >>= 32;
      have -= 32;
    }
  }
  while (wi < nwords) {
    o[wi++] = (uint32_t)acc;
    acc >>= 32;
  }
}

// mode 0: node[e] = words[e] R_w (MontW(x, R_w^2)); mode 1: root words
// (plain inverse from the host) -> inv node, the same conversion
template <int K, int NWV>
__global__ void __launch_bounds__(64 * NWV) k_wtree_in(KeyDev key, const uint32_t* __restrict__ words,
                                                       uint32_t* __restrict__ node) {
  using WM = WaveMont<K, NWV, 27>;
  __shared__ __attribute__((aligned(16))) typename WM::Lds s;
  const int64_t e = blockIdx.x;
  wave_init_n2<WM>(s, key);
  wave_limbs_in<WM>(words + (size_t)e * key.n2w, key.n2w, s.tl);
  for (int i = WM::tid(); i < K; i += WM::NT) s.zb[WM::ZO + i] = key.n2w_R2[i];
  WM::sync();
  int cur = 0;
  WM::mul(s, cur, s.tl, s.x, false);
  for (int i = WM::tid(); i < K; i += WM::NT) node[(size_t)e * K + i] = s.x[i];
}

// up-sweep level: parent i = child 2i x child 2i+1 (a lone last child is
// copied up)
template <int K, int NWV>
__global__ void __launch_bounds__(64 * NWV) k_wtree_up(KeyDev key, const uint32_t* __restrict__ child, int64_t nchild,
                                                       uint32_t* __restrict__ parent) {
  using WM = WaveMont<K, NWV, 27>;
  __shared__ __attribute__((aligned(16))) typename WM::Lds s;
  const int64_t i = blockIdx.x;
  const uint32_t* a = child + (size_t)(2 * i) * K;
  if (2 * i + 1 >= nchild) {
    for (int j = WM::tid(); j < K; j += WM::NT) parent[(size_t)i * K + j] = a[j];
    return;
  }
  wave_init_n2<WM>(s, key);
  for (int j = WM::tid(); j < K; j += WM::NT) {
    s.tl[j] = a[j];
    s.zb[WM::ZO + j] = a[K + j];
  }
  WM::sync();
  int cur = 0;
  WM::mul(s, cur, s.tl, s.x, false);
  for (int j = WM::tid(); j < K; j += WM::NT) parent[(size_t)i * K + j] = s.x[j];
}

// down-sweep level: inv child i = inv parent (i/2) x node sibling (i^1), or
// the parent's inverse for a lone child
template <int K, int NWV>
__global__ void __launch_bounds__(64 * NWV) k_wtree_down(KeyDev key, const uint32_t* __restrict__ inv_parent,
                                                         const uint32_t* __restrict__ node, int64_t nchild,
                                                         uint32_t* __restrict__ inv_child) {
  using WM = WaveMont<K, NWV, 27>;
  __shared__ __attribute__((aligned(16))) typename WM::Lds s;
  const int64_t i = blockIdx.x, sib = i ^ 1;
  const uint32_t* ip = inv_parent + (size_t)(i >> 1) * K;
  if (sib >= nchild) {
    for (int j = WM::tid(); j < K; j += WM::NT) inv_child[(size_t)i * K + j] = ip[j];
    return;
  }
  wave_init_n2<WM>(s, key);
  for (int j = WM::tid(); j < K; j += WM::NT) {
    s.tl[j] = ip[j];
    s.zb[WM::ZO + j] = node[(size_t)sib * K + j];
  }
  WM::sync();
  int cur = 0;
  WM::mul(s, cur, s.tl, s.x, false);
  for (int j = WM::tid(); j < K; j += WM::NT) inv_child[(size_t)i * K + j] = s.x[j];
}

// node[e] R_w -> plain words (MontW(x R_w, 1), reduced below N)
template <int K, int NWV>
__global__ void __launch_bounds__(64 * NWV) k_wtree_out(KeyDev key, const uint32_t* __restrict__ node,
                                                        uint32_t* __restrict__ words) {
  using WM = WaveMont<K, NWV, 27>;
  __shared__ __attribute__((aligned(16))) typename WM::Lds s;
  const int64_t e = blockIdx.x;
  wave_init_n2<WM>(s, key);
  for (int j = WM::tid(); j < K; j += WM::NT) s.tl[j] = node[(size_t)e * K + j];
  if (WM::tid() == 0) s.zb[WM::ZO] = 1u;
  WM::sync();
  int cur = 0;
  WM::mul(s, cur, s.tl, s.x, false);
  wave_words_out<WM>(s.x, s.zn, key.n2w, words + (size_t)e * key.n2w);
}

}  // namespace xhe
