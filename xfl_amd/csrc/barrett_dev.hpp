// One-product ciphertext add mod n^2 for 2048-bit keys: c = x y mod N, N = n^2
// (paillier.py:106-123,153-154: _add_encrypted with equal exponents), by
// product scanning and Barrett reduction (HAC 14.42) instead of two
// Montgomery products (x R by R^2, then x R * y * R^-1).
//
// 27-bit limbs, S = 152 (N < beta^S, N >= beta^(S-1), beta = 2^27):
//   A  T  = x y                 304 columns (S^2 = 23.1 k mads)
//   B  q3 = floor(floor(T / beta^(S-1)) mu / beta^(S+1)), mu = floor(beta^2S / N),
//          from the columns 148 .. 307 of q1 mu only (~12 k mads)
//   C  r2 = q3 N mod beta^160   columns < 160 (~12 k mads)
//   D  r  = (T - r2) mod beta^160 = T - q3 N (< 4N), then r -= N while r >= N
// ~47 k mads against 2 x 2 S^2 = 92.4 k for the Montgomery pair, and no
// workspace round trip through HBM. tools/barrett_model.py checks this limb
// schedule (rounds, truncation, carries, bounds) against Python integers.
//
// Layout: G = 8 lanes per element, 32 elements per 256-thread block. A round
// covers 4G columns, lane g the 4 columns C0 + 4g .. C0 + 4g + 3; all lanes of
// a wave walk the same terms i (wave-uniform loop bounds), the "x" operand
// x_i .. x_{i+3} is one ds_read_b128 shared by the group, the "y" operand is a
// window y_{c-i-3} .. y_{c-i+3} in registers that slides by one b128 per 4
// terms (16 mads per two LDS reads). Each round's 64-bit column sums are
// carried into 27-bit limbs in-lane, lane to lane (a carry-lookahead over the
// wave's lane masks, as Mont::normalize) and round to round. 8 lanes rather
// than 4: the same LDS per element in flight, twice the waves to hide the
// latencies (3 per SIMD), half the registers per lane.
#pragma once
#include "bn_dev.hpp"

namespace xhe {
namespace bar {

constexpr int W = 27;
constexpr uint32_t MASK = (1u << W) - 1u;
constexpr int S = 152;          // limbs of n^2 at 2048-bit keys
#ifndef XHE_BAR_G
#define XHE_BAR_G 8
#endif
constexpr int G = XHE_BAR_G;    // lanes per element (8; 4 for A/B: 16-column rounds)
static_assert(G == 8 || G == 4, "8 or 4 lanes per element");
constexpr int RCOLS = 4 * G;    // columns per round
constexpr int YOFF = 4 * G + 7; // y-role rows: limb j at [YOFF + j]; >= 4G + 6 zeros in front, = 3 mod 4
constexpr int YLEN = (YOFF + (S + 1) + 4 * G + 3 + 3) & ~3;  // ... and >= 4G + 2 zeros behind (LY <= S + 1)
constexpr int XLEN = 160;       // x-role rows: limb i at [i], zeros to XLEN (LX <= S + 1, + 7 for the last pair)
constexpr int XB = 0, YB = XLEN;
constexpr int STRIDE = 400;     // words per element (= 16 mod 64: the elements of a b128 lane group spread over the banks)
constexpr int TPB = 32 * G;     // threads per block (32 elements: the LDS of three blocks per CU)
constexpr int EPB = TPB / G;    // elements per block
constexpr int LDS_WORDS = EPB * STRIDE + 2 * YLEN;  // + the shared mu and N rows
static_assert(XB + XLEN <= YB && YB + YLEN <= STRIDE, "element rows overlap");
static_assert(STRIDE % 64 == 16, "bank spread of the element rows");
static_assert(LDS_WORDS * 4 * 3 <= 160 * 1024, "three blocks per CU");
static_assert(YOFF % 4 == 3 && XLEN % 4 == 0 && YB % 4 == 0 && STRIDE % 4 == 0, "b128 alignment of the windows");

using M4 = Mont<S, W, 4>;  // limb I/O: the group's two halves are two 4-lane groups

XHE_DEV int lane_g() { return (int)(threadIdx.x & (G - 1)); }
// lane g-1's value (garbage at g = 0: callers replace it)
XHE_DEV uint32_t prev_lane(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
}
// lane G-1's value of the group
XHE_DEV uint32_t last_lane(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((threadIdx.x & 63) | (G - 1)) << 2), (int)v);
}
XHE_DEV uint64_t prev_lane64(uint64_t v) {
  return (uint64_t)prev_lane((uint32_t)v) | ((uint64_t)prev_lane((uint32_t)(v >> 32)) << 32);
}
XHE_DEV uint64_t last_lane64(uint64_t v) {
  return (uint64_t)last_lane((uint32_t)v) | ((uint64_t)last_lane((uint32_t)(v >> 32)) << 32);
}
constexpr uint64_t TOPS = G == 8 ? 0x8080808080808080ull : 0x8888888888888888ull;  // the last lane of every group

// acc[k] += x_ii w[k - ii + 3] for ii, k < 4 (w[t] = y_{c-i0-3+t} of a block
// of 4 terms i0 .. i0+3): 16 mads in one statement (a separate asm per mad
// costs an s_nop after each: it writes vcc)
XHE_DEV void mad_block(uint64_t (&acc)[4], const uint4& x, const uint4& w03, uint32_t w4, uint32_t w5, uint32_t w6) {
  asm("v_mad_u64_u32 %0, vcc, %4, %11, %0\n\t"
      "v_mad_u64_u32 %1, vcc, %4, %12, %1\n\t"
      "v_mad_u64_u32 %2, vcc, %4, %13, %2\n\t"
      "v_mad_u64_u32 %3, vcc, %4, %14, %3\n\t"
      "v_mad_u64_u32 %0, vcc, %5, %10, %0\n\t"
      "v_mad_u64_u32 %1, vcc, %5, %11, %1\n\t"
      "v_mad_u64_u32 %2, vcc, %5, %12, %2\n\t"
      "v_mad_u64_u32 %3, vcc, %5, %13, %3\n\t"
      "v_mad_u64_u32 %0, vcc, %6, %9, %0\n\t"
      "v_mad_u64_u32 %1, vcc, %6, %10, %1\n\t"
      "v_mad_u64_u32 %2, vcc, %6, %11, %2\n\t"
      "v_mad_u64_u32 %3, vcc, %6, %12, %3\n\t"
      "v_mad_u64_u32 %0, vcc, %7, %8, %0\n\t"
      "v_mad_u64_u32 %1, vcc, %7, %9, %1\n\t"
      "v_mad_u64_u32 %2, vcc, %7, %10, %2\n\t"
      "v_mad_u64_u32 %3, vcc, %7, %11, %3"
      : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])
      : "v"(x.x), "v"(x.y), "v"(x.z), "v"(x.w), "v"(w03.x), "v"(w03.y), "v"(w03.z), "v"(w03.w), "v"(w4), "v"(w5),
        "v"(w6)
      : "vcc");
}

// The operands of one pair of 4-term blocks (terms i0 .. i0+7)
struct Pair {
  uint4 ya, xa, yb, xb;  // y_{c-i0-3 .. c-i0}, x_{i0 .. i0+3}, y_{c-i0-7 .. c-i0-4}, x_{i0+4 .. i0+7}
};
XHE_DEV Pair load_pair(const uint32_t* yp, const uint32_t* xp, int p) {
  Pair q;
  q.ya = *reinterpret_cast<const uint4*>(yp - 8 * p);
  q.xa = *reinterpret_cast<const uint4*>(xp + 8 * p);
  q.yb = *reinterpret_cast<const uint4*>(yp - 8 * p - 4);
  q.xb = *reinterpret_cast<const uint4*>(xp + 8 * p + 4);
  return q;
}
// the pair's 32 mads; w4..w6 = y_{c-i0+1 .. c-i0+3}
XHE_DEV void mad_pair(uint64_t (&acc)[4], const Pair& q, uint32_t w4, uint32_t w5, uint32_t w6) {
  mad_block(acc, q.xa, q.ya, w4, w5, w6);
  mad_block(acc, q.xb, q.yb, q.ya.x, q.ya.y, q.ya.z);
}

// lane g's column sums acc[k] = sum_i x_i y_{C0 + 4g + k - i} over the terms
// of columns [C0, C0 + 4G): x at xr[i] (LX limbs, zeros to XLEN), y at
// yr[YOFF + j] (LY limbs, zero-padded). Terms go in pairs of 4-term blocks
// (the range rounded up to a multiple of 8 with zero x), so the window's two
// halves alternate roles, and two pairs per iteration carry the window in
// each other's registers (no moves). Loading a pair ahead measured no faster
// (the kernel is VALU-issue-bound, 93 % busy). Not unrolled further:
// unrolled, the compiler hoisted every LDS read of a round and spilled.
XHE_DEV void cols(const uint32_t* xr, const uint32_t* yr, int C0, int g, int LX, int LY, uint64_t (&acc)[4]) {
  int ilo = C0 - (LY - 1);
  ilo = ilo < 0 ? 0 : ilo;
  int ihi = C0 + RCOLS - 1;
  ihi = ihi > LX - 1 ? LX - 1 : ihi;
  const int ib0 = ilo & ~3;
  const int npair = (ihi + 1 - ib0 + 7) >> 3;
  const int c = C0 + 4 * g;
#pragma unroll
  for (int k = 0; k < 4; ++k) acc[k] = 0;
  // w4..w6 = y_{c-i0+1} .. y_{c-i0+3} (the part of the window carried over)
  const uint4 pv = *reinterpret_cast<const uint4*>(yr + YOFF + 1 + c - ib0);
  uint32_t w4 = pv.x, w5 = pv.y, w6 = pv.z;
  const uint32_t* yp = yr + YOFF - 3 + c - ib0;  // y_{c-i0-3} at yp[-(i0 - ib0)]
  const uint32_t* xp = xr + ib0;
#pragma unroll 1
  for (int p = 0; p < npair; p += 2) {
    // two pairs per iteration, the window carried in the other pair's
    // registers (no moves); the second pair is skipped (wave-uniform) when
    // the count is odd
    const Pair A = load_pair(yp, xp, p);
    mad_pair(acc, A, w4, w5, w6);
    if (p + 1 < npair) {
      const Pair B = load_pair(yp, xp, p + 1);
      mad_pair(acc, B, A.yb.x, A.yb.y, A.yb.z);
      w4 = B.yb.x;
      w5 = B.yb.y;
      w6 = B.yb.z;
    } else {
      w4 = A.yb.x;
      w5 = A.yb.y;
      w6 = A.yb.z;
    }
  }
}

// lane g's 4 column sums -> limbs l[k]; rc = carry into the round (the same
// value in every lane of the group); returns the carry out of the round (in
// every lane of the group)
XHE_DEV uint64_t norm(const uint64_t (&acc)[4], uint32_t (&l)[4], uint64_t rc, int g) {
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint64_t x = acc[k] + c;
    l[k] = (uint32_t)x & MASK;
    c = x >> W;
  }
  uint64_t t = prev_lane64(c);  // the previous lane's carry (lane 0: the round's)
  if (g == 0) t = rc;
  uint32_t all = 1u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint64_t x = (uint64_t)l[k] + t;
    l[k] = (uint32_t)x & MASK;
    t = x >> W;  // 0 or 1 once the first limbs have absorbed t < 2^40
    all &= l[k] == MASK ? 1u : 0u;
  }
  // carries of 0/1 rippling across lanes: generate = t, propagate = all MASK
  const uint64_t gm = __builtin_amdgcn_ballot_w64(t != 0) & ~TOPS;
  const uint64_t pm = (gm | __builtin_amdgcn_ballot_w64(all != 0)) & ~TOPS;
  const uint64_t cm = (gm + pm) ^ gm ^ pm;
  uint32_t ci = (uint32_t)(cm >> (threadIdx.x & 63)) & 1u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t x = l[k] + ci;
    l[k] = x & MASK;
    ci = x >> W;
  }
  return last_lane64(c + t + ci);  // the last lane's: its own carry and its ripple
}

// out = (a - b - bin) over 4 limbs per lane and the group's lanes, borrows
// rippling from lane to lane; bin enters lane 0 (the same value in every
// lane); returns the borrow out of the last lane (in every lane of the group)
XHE_DEV uint32_t sub_round(const uint32_t (&a)[4], const uint32_t (&b)[4], uint32_t (&out)[4], uint32_t bin, int g) {
  uint32_t br = g == 0 ? bin : 0u;
  uint32_t zero = 1u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int32_t x = (int32_t)a[k] - (int32_t)b[k] - (int32_t)br;
    br = x < 0 ? 1u : 0u;
    out[k] = (uint32_t)(x + (int32_t)(br << W));
    zero &= out[k] == 0u ? 1u : 0u;
  }
  // borrows: generate = br, propagate = all limbs zero (0 - 1 borrows again)
  const uint64_t gm = __builtin_amdgcn_ballot_w64(br != 0) & ~TOPS;
  const uint64_t pm = (gm | __builtin_amdgcn_ballot_w64(zero != 0)) & ~TOPS;
  const uint64_t cm = (gm + pm) ^ gm ^ pm;
  uint32_t bi = (uint32_t)(cm >> (threadIdx.x & 63)) & 1u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int32_t x = (int32_t)out[k] - (int32_t)bi;
    bi = x < 0 ? 1u : 0u;
    out[k] = (uint32_t)(x + (int32_t)(bi << W));
  }
  return last_lane(br + bi);
}

}  // namespace bar

// c = a * b mod n^2 for 2048-bit keys, equal exponents (eout = min(ea, eb)).
// mu: floor(2^(27*304) / n^2) as 153 limbs of 27 bits (KeyDev::n2_mu).
__global__ void __launch_bounds__(bar::TPB, bar::G == 8 ? 3 : 2) k_add_barrett(KeyDev key, const uint32_t* __restrict__ a,
                                                          const int32_t* __restrict__ ea,
                                                          const uint32_t* __restrict__ bw,
                                                          const int32_t* __restrict__ eb, int64_t count,
                                                          uint32_t* __restrict__ out, int32_t* __restrict__ eout) {
  using namespace bar;
  __shared__ __attribute__((aligned(16))) uint32_t lds[LDS_WORDS];
  uint32_t* mu = lds + EPB * STRIDE;
  uint32_t* nb = mu + YLEN;
  for (int t = threadIdx.x; t < YLEN; t += blockDim.x) {
    const int j = t - YOFF;
    mu[t] = (j >= 0 && j < S + 1) ? key.n2_mu[j] : 0u;
    nb[t] = (j >= 0 && j < S) ? key.n2.N[j] : 0u;
  }
  __syncthreads();
  const int le = threadIdx.x / G;  // element within the block
  const int64_t e0 = (int64_t)blockIdx.x * EPB + le;
  const bool live = e0 < count;
  const int64_t e = live ? e0 : count - 1;  // idle groups recompute the last element (no stores)
  const int g = lane_g();
  const int half = g >> 2;  // I/O: lanes 0-3 handle x (then the result), lanes 4-7 y
  uint32_t* xr = lds + le * STRIDE + XB;
  uint32_t* yr = lds + le * STRIDE + YB;
  M4 M;  // limb I/O only (load_words / store_words)
  {
    uint32_t b[M4::L];
    M.load_words(b, (half ? bw : a) + (size_t)e * key.n2w, key.n2w);
    uint32_t* dst = half ? yr + YOFF : xr;
#pragma unroll
    for (int j = 0; j < M4::L; ++j) dst[(g & 3) * M4::L + j] = b[j];
    if constexpr (G == 4) {  // one 4-lane group loads both operands
      M.load_words(b, bw + (size_t)e * key.n2w, key.n2w);
#pragma unroll
      for (int j = 0; j < M4::L; ++j) yr[YOFF + g * M4::L + j] = b[j];
    }
    for (int j = g; j < XLEN - S; j += G) xr[S + j] = 0u;
    for (int j = g; j < YOFF; j += G) yr[j] = 0u;
    for (int j = YOFF + S + g; j < YLEN; j += G) yr[j] = 0u;
  }
  // Limbs change hands between the lanes of a group through LDS at every
  // phase boundary (the operands here, then q1, q3 and r): the fence keeps
  // each lane's stores ahead of the other lanes' loads (as k_mulmod_n2 does).
  wave_sync_mem_();
  // ---- A: T = x y (rounds of 4G columns)
  constexpr int RA = (2 * S + RCOLS - 1) / RCOLS;
  uint32_t T[RA][4];
  uint64_t rc = 0;
#pragma unroll
  for (int r = 0; r < RA; ++r) {
    uint64_t acc[4];
    cols(xr, yr, RCOLS * r, g, S, S, acc);
    rc = norm(acc, T[r], rc, g);
  }
  // q1 = T[S-1 .. 2S-1] (153 limbs) replaces x
#pragma unroll
  for (int r = (S - 1) / RCOLS; r < RA; ++r)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = RCOLS * r + 4 * g + k;
      if (t >= S - 1 && t < 2 * S) xr[t - (S - 1)] = T[r][k];
    }
  for (int j = S + 1 + g; j < XLEN; j += G) xr[j] = 0u;
  wave_sync_mem_();
  // ---- B: q3 = the limbs >= S+1 of q1 mu, from its columns 148 .. 307
  // (>= S-1-3: the truncation costs q3 at most 1, tools/barrett_model.py;
  // q1 mu has no column above 2S, + its carry)
  constexpr int B0 = S - 4, RB = (2 * S + 2 - B0 + RCOLS - 1) / RCOLS;
  static_assert(B0 % 4 == 0 && B0 + RB * RCOLS >= 2 * S + 2, "truncation guard and top columns");
  rc = 0;
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    uint64_t acc[4];
    uint32_t l[4];
    cols(xr, mu, B0 + RCOLS * r, g, S + 1, S + 1, acc);
    rc = norm(acc, l, rc, g);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = B0 + RCOLS * r + 4 * g + k - (S + 1);  // q3 limb index
      if (t >= 0 && t < XLEN) yr[t] = l[k];                // x-role layout (y is no longer needed)
    }
  }
  // q3's x-role row ends in zeros (limbs 153, 154 were written as the zero
  // columns 306, 307; what lies beyond is y's old window)
  for (int j = S + 1 + g; j < XLEN; j += G) yr[j] = 0u;
  wave_sync_mem_();
  // ---- C: r2 = q3 N mod beta^(4G * RC)
  constexpr int RC = (S + 1 + RCOLS - 1) / RCOLS;
  uint32_t R2[RC][4];
  rc = 0;
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    uint64_t acc[4];
    cols(yr, nb, RCOLS * r, g, S + 1, S, acc);
    rc = norm(acc, R2[r], rc, g);
  }
  // ---- D: r = T - r2 mod beta^(4G * RC) (= T - q3 N < 4N), then r -= N while r >= N
  uint32_t bin = 0;
#pragma unroll
  for (int r = 0; r < RC; ++r) bin = bar::sub_round(T[r], R2[r], T[r], bin, g);
#pragma unroll 1
  for (int pass = 0; pass < 4; ++pass) {
    uint32_t D[RC][4];
    bin = 0;
#pragma unroll
    for (int r = 0; r < RC; ++r) {
      uint32_t nl[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) nl[k] = nb[YOFF + RCOLS * r + 4 * g + k];
      bin = bar::sub_round(T[r], nl, D[r], bin, g);
    }
    const bool ge = bin == 0u;  // r >= N: take r - N
    if (__builtin_amdgcn_ballot_w64(ge) == 0) break;
    if (ge) {
#pragma unroll
      for (int r = 0; r < RC; ++r)
#pragma unroll
        for (int k = 0; k < 4; ++k) T[r][k] = D[r][k];
    }
  }
  // ---- out: r's limbs 0 .. S-1 -> packed words (lanes 0-3 of the group)
#pragma unroll
  for (int r = 0; r < RC; ++r)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = RCOLS * r + 4 * g + k;
      if (t < S) xr[t] = T[r][k];
    }
  wave_sync_mem_();
  uint32_t b[M4::L];
#pragma unroll
  for (int j = 0; j < M4::L; ++j) b[j] = xr[(g & 3) * M4::L + j];
  if (live && half == 0) {
    M.store_words(b, out + (size_t)e * key.n2w, key.n2w);
    if (eout && g == 0) {
      const int e1 = ea ? ea[e] : 0, e2 = eb ? eb[e] : 0;
      eout[e] = e1 < e2 ? e1 : e2;
    }
  }
}

}  // namespace xhe
