// Paillier hot-path kernels (gfx950). One residue per TPI-lane group; see
// bn_dev.hpp for the Montgomery representation.
//
// Reference semantics (paths under /root/reference/python):
//   encode            common/crypto/paillier/encoder.py:29-54, paillier.py:279-282
//   raw encrypt       paillier.py:283            c0 = (1 + n*m) mod n^2
//   DJN obfuscation   paillier.py:193-209        c0 * h^a mod n^2 (CRT over p^2, q^2)
//   decrypt           paillier.py:341-368        L(c^(p-1) mod p^2) * hp mod p, CRT
//   decode            encoder.py:56-64, paillier.py:396-403
#pragma once
#include "bn_dev.hpp"
#include "pdigit_dev.hpp"

namespace xhe {

struct ModDev {
  const uint32_t* N;   // S W-limbs (row of S4 words)
  const uint32_t* R1;  // R mod N
  const uint32_t* R2;  // R^2 mod N
  const uint32_t* R3;  // R^3 mod N
  uint32_t n0inv;
  const uint32_t* Rpow;  // n^2 shapes: R^j mod N for j < kRpowRows, rows of S4 limbs (else null)
};

// Segment chunks of plain (non-Montgomery) residues are at most kRawChunk
// long; such a chunk's product comes back to Montgomery form by one product
// with R^(len + 1), so R^j is kept for j <= kRawChunk + 1.
constexpr int kRawChunk = 32;
constexpr int kRpowRows = kRawChunk + 2;

// All pointers are device pointers into the key blob. Limb rows are padded to
// a multiple of 4 words and 16-byte aligned.
struct KeyDev {
  int K, nw, n2w;  // key bits, 32-bit words of n and of n^2
  int priv, djn;
  const uint32_t* n_words;   // n (nw words)
  const uint32_t* n2_words;  // n^2 (n2w words)
  const uint32_t* maxpos;    // n // 3 (nw words)
  const uint32_t* minneg;    // n - n // 3 (nw words)
  const uint32_t* n_lim;     // n as MP2 limbs (raw encryption wide product)
  // ---- mod n^2 (shape MN2): public-key paths and homomorphic operations
  ModDev n2;
  const uint32_t* nR2_n2;     // n * R^2 mod n^2
  const uint32_t* tab_n2;     // [nwin][2^win][S4] h^(d*2^(win*w)) * R mod n^2 (public DJN)
  const uint32_t* ep_words;   // n mod phi(p^2) (nw words), non-DJN private obfuscation exponent
  const uint32_t* eq_words;
  int ep_bits, eq_bits, n_bits;
  // ---- mod p^2 / q^2 (shape MP2)
  ModDev p2, q2;
  ModDev p2L, q2L;            // the same moduli in the 4-lane decrypt shape (S = S4 of p2)
  ModDev p2X, q2X;            // and in the 16-lane (one DPP row) decrypt shape
  ModDev n2X;                 // n^2 in the 16-lane shape (small-batch ciphertext ops)
  const uint32_t* nR2_p2;     // n * R^2 mod p^2
  const uint32_t *nR_p2, *nR_q2;  // n * R mod P^2 (plain n m from a Montgomery product)
  // 16-lane (p2X/q2X, R' = 2^(W*80)) DJN shape on the one-lane tables: every
  // table product scales by R/R', so the start value carries C = (R'/R)^nwin:
  const uint32_t *nR2C_p2X, *nR2C_q2X;  // n * C * R'^2 mod P^2
  const uint32_t *R1C_p2X, *R1C_q2X;    // C * R' mod P^2
  const uint32_t* nR2_q2;     // n * R^2 mod q^2
  const uint32_t* nR2_p2L;    // n * R_L^2 mod p^2 / q^2 in the 4-lane (p2L) shape
  const uint32_t* nR2_q2L;
  const uint32_t* q2invR_p2;  // (q^2)^-1 * R mod p^2
  const uint32_t* q2_lim;     // q^2 (MP2 limbs)
  const uint32_t* p2x4_lim;   // 4 p^2 (MP2 limbs)
  const uint32_t* tab_p2;     // h^(d*2^bit(w)) * R mod p^2, packed rows, windows as win_digit()
  const uint32_t* tab_q2;
  int64_t tab_rs;             // words from one row of tab_p2 / tab_q2 to the next
  int win, nwin, nhi;         // nhi: the first nhi windows are win+1 bits wide (0: uniform)
  // ---- mod p / q (shape MP), decrypt
  ModDev p, q;
  const uint32_t* pm1_words;  // p - 1 (nw/2 words)
  const uint32_t* qm1_words;
  int pm1_bits, qm1_bits;
  const uint32_t* pinv_lim;   // p^-1 mod 2^(W*S) (MP limbs)
  const uint32_t* qinv_lim;
  const uint32_t* hpR;        // hp * R mod p
  const uint32_t* hqR;
  const uint32_t* qinvpR;     // (q^-1 mod p) * R mod p
  const uint32_t* q_lim;      // q (MP limbs)
  const uint32_t* p2x_lim;    // 2 p (MP limbs)
  const uint32_t* p_lim;      // p (MP limbs)
  // ---- Montgomery-digit DJN encryption (k_djn_pmd, 2048-bit keys): the
  // tables hold digit pairs (pmd = 1); MASK + ((1 - R) mod P) limbs per prime
  int pmd;
  const uint32_t *topc_p, *topc_q;
  // ---- Montgomery digits mod n^2 (PMDX, 2048-bit keys, public or private):
  // n as 80 limbs of 27 bits (R = 2^2160), ceil(R/n) n^2 (160 limbs), R - n,
  // the digits of R^2 mod n^2 and of 1 (80 pairs each), MASK + E_i
  int ndig;
  ModDev nd;
  const uint32_t *nd_kn2, *nd_rmn, *nd_topc;
  const uint2 *nd_dw, *nd_d1;
  const uint2* nd_dwt;  // digits of R^2 R_MN2^-1 (public DJN table rows -> digits)
  int pub_nd;           // public DJN tables hold digits of n (k_djn_pub_nd)
  // ---- Montgomery digits mod P^2 over 4 lanes (PMDX, 3072/4096-bit DJN
  // private keys; k_djn_pmdx): P as K limbs of 27 bits, ceil(R/P) P^2, R - P,
  // MASK + E_i, the fold constant Q R^3 mod P (Q the other prime) and the
  // digits of R^2 R_MP2^-1 mod P^2 (the table rows' conversion constant)
  int pmdx;
  ModDev dp, dq;
  const uint32_t *x_kn2_p, *x_kn2_q, *x_rmn_p, *x_rmn_q, *x_topc_p, *x_topc_q, *x_fold_p, *x_fold_q;
  const uint2 *x_dwt_p, *x_dwt_q;
  // the same digits for the decrypt of every 3072/4096-bit private key
  // (k_dec_pmdx_*): the digits of R^2 mod P^2 and hp R mod P (27-bit limbs)
  int pmdx_dec;
  const uint2 *x_dw_p, *x_dw_q;
  const uint32_t *x_hpR_p, *x_hpR_q;
  // ---- one-wave decrypt exponentiation (k_dec_wave, 2048-bit keys): the
  // full Montgomery inverse -P^-2 mod R of the MP2 shape (R = 2^(28*74))
  const uint32_t *p2_nprime, *q2_nprime;
  // ---- RNS small-batch decrypt (k_dec_rns, rns_dev.hpp; 2048-bit private
  // keys): the bases' constant block and one block per prime (null: off)
  const uint32_t *rns, *rns_p, *rns_q;
  // ---- one-block Horner of the mat-vec mod n^2 (k_mexp_horner_wave, 2048-bit
  // keys): n^2 in 154 limbs of 27 bits (R_w = 2^4158), -n^-2 mod R_w and
  // C = R_w^2 R_X^-1 mod n^2 (R_X = 2^(27*160): the 16-lane shape's R)
  const uint32_t *n2w_N, *n2w_np, *n2w_C, *n2w_R2;  // (R2: R_w^2 mod n^2, k_mulmod_wave)
  // ---- Barrett reduction mod n^2 (k_add_barrett, 2048-bit keys):
  // floor(2^(27*304) / n^2) as 153 limbs of 27 bits
  const uint32_t* n2_mu;
};

// ============================================================== encode
// status codes per element (mirrors the exceptions the reference raises)
enum : int32_t { ST_OK = 0, ST_OVERFLOW = 1, ST_VALUE = 2 };

// y = round_half_even(x * 2^-e) as |y| = (v0 + v1 2^32 + v2 2^64) 2^(32 w),
// its sign, the exponent e (mode 0: frexp(x) - 53, i.e. precision None;
// mode 1: fixed e0; clamped by max_exponent when has_max) and the status the
// reference's encode raises for x (encoder.py:29-54).
struct EncVal {
  int32_t st, e;
  int neg, w;
  uint32_t v0, v1, v2;
};

XHE_DEV EncVal encode_value(double v, int mode, int e0, int has_max, int max_exp) {
  EncVal r{ST_OK, 0, 0, 0, 0u, 0u, 0u};
  uint64_t bits = __double_as_longlong(v);
  r.neg = (int)(bits >> 63);
  int bexp = (int)((bits >> 52) & 0x7FF);
  uint64_t frac = bits & ((1ull << 52) - 1);
  int e;
  if (mode == 0) {
    // math.frexp(x)[1] - 53; frexp(0) = (0, 0); frexp(inf/nan) = (x, 0)
    int fe;
    if (bexp == 0x7FF || (bexp == 0 && frac == 0)) fe = 0;
    else if (bexp == 0) fe = -1022 - (__clzll(frac) - 12);  // subnormal: frexp exponent
    else fe = bexp - 1022;
    e = fe - 53;
  } else {
    e = e0;
  }
  if (has_max && max_exp < e) e = max_exp;
  r.e = e;
  // x * (1 << -e): negative shift -> ValueError; shift >= 1024 -> int->float OverflowError
  if (-e < 0) r.st = ST_VALUE;
  else if (-e >= 1024) r.st = ST_OVERFLOW;
  else if (bexp == 0x7FF) r.st = frac ? ST_VALUE : ST_OVERFLOW;  // round(nan) / round(inf)
  // M * 2^E exact decomposition
  uint64_t M;
  int E;
  if (bexp == 0) { M = frac; E = -1074; } else { M = frac | (1ull << 52); E = bexp - 1075; }
  int sh = E - e;  // y = M * 2^sh
  // float product overflow (|y| >= 2^1024) -> inf -> round(inf) OverflowError
  if (r.st == ST_OK && M != 0) {
    int top = 64 - __clzll(M) + sh;  // y < 2^top
    if (top > 1024) r.st = ST_OVERFLOW;
  }
  if (r.st != ST_OK || M == 0) return r;
  if (sh >= 0) {
    int b = sh & 31;
    uint64_t lo = M << b;                                 // bits [w*32, w*32+64)
    r.w = sh >> 5;
    r.v0 = (uint32_t)lo;
    r.v1 = (uint32_t)(lo >> 32);
    r.v2 = b ? (uint32_t)(M >> (64 - b)) : 0u;            // bits [w*32+64, +96)
  } else {
    int rr = -sh;
    uint64_t q, rem, half;
    if (rr >= 64) { q = 0; rem = M; half = (rr == 64) ? (1ull << 63) : ~0ull; if (rr > 64) { q = 0; rem = 0; } }
    else { q = M >> rr; rem = M & ((1ull << rr) - 1); half = 1ull << (rr - 1); }
    if (rr <= 64 && (rem > half || (rem == half && (q & 1)))) q += 1;
    r.v0 = (uint32_t)q;
    r.v1 = (uint32_t)(q >> 32);
  }
  return r;
}

XHE_DEV uint32_t enc_word(const EncVal& y, int k) {
  const int d = k - y.w;
  return d == 0 ? y.v0 : d == 1 ? y.v1 : d == 2 ? y.v2 : 0u;
}

// float64 x -> m = y mod n (n - |y| for negative y, |y| < 2^1077 < n for
// K >= 2048), exponent and status per element. One thread per 16-byte quad
// of m (nw/4 threads per element, nw a multiple of 4): a wave writes whole
// consecutive rows, so the stores are coalesced.
__global__ void k_encode_f64(const double* __restrict__ x, int64_t count, int mode, int e0, int has_max,
                             int max_exp, const uint32_t* __restrict__ n_words, int nw,
                             uint32_t* __restrict__ m_out, int32_t* __restrict__ e_out,
                             int32_t* __restrict__ status) {
  const int nq = nw >> 2;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i = t / nq;
  if (i >= count) return;
  const int q = (int)(t - i * nq);
  const EncVal y = encode_value(x[i], mode, e0, has_max, max_exp);
  if (q == 0) {
    e_out[i] = y.e;
    status[i] = y.st;
  }
  uint32_t o[4] = {0u, 0u, 0u, 0u};
  const bool zero = y.st != ST_OK || (y.v0 | y.v1 | y.v2) == 0u;
  if (!zero) {
    if (!y.neg) {
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = enc_word(y, 4 * q + k);
    } else {
      // n - |y|: the borrow into word 4q comes from words [w, 4q) only
      // (|y| is zero below w), and propagates past w + 2 only through zero words of n
      uint32_t br = 0;
      const int kend = min(4 * q, y.w + 3);
      for (int k = y.w; k < kend; ++k) {  // at most the 3 words of |y|
        const uint32_t nk = n_words[k], yk = enc_word(y, k);
        br = (nk < yk || (nk == yk && br)) ? 1u : 0u;
      }
      for (int k = y.w + 3; k < 4 * q && br; ++k) br = n_words[k] == 0u ? 1u : 0u;  // through zero words only
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t nk = n_words[4 * q + k], yk = enc_word(y, 4 * q + k);
        o[k] = nk - yk - br;
        br = (nk < yk || (nk == yk && br)) ? 1u : 0u;
      }
    }
  }
  uint32_t* dst = m_out + (size_t)i * nw + 4 * q;
  if ((reinterpret_cast<uintptr_t>(m_out) & 15u) == 0u) {
    *reinterpret_cast<uint4*>(dst) = make_uint4(o[0], o[1], o[2], o[3]);
  } else {  // a caller's buffer that is not 16-byte aligned
#pragma unroll
    for (int k = 0; k < 4; ++k) dst[k] = o[k];
  }
}

// ============================================================== ChaCha20
XHE_DEV uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
#define XHE_QR(a, b, c, d) \
  a += b; d ^= a; d = rotl32(d, 16); c += d; b ^= c; b = rotl32(b, 12); \
  a += b; d ^= a; d = rotl32(d, 8);  c += d; b ^= c; b = rotl32(b, 7);

XHE_DEV void chacha20_block(const uint32_t key[8], uint32_t nonce0, uint32_t nonce1, uint64_t ctr, uint32_t out[16]) {
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                    key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                    (uint32_t)ctr, (uint32_t)(ctr >> 32), nonce0, nonce1};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = s[i];
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    XHE_QR(x[0], x[4], x[8], x[12]) XHE_QR(x[1], x[5], x[9], x[13])
    XHE_QR(x[2], x[6], x[10], x[14]) XHE_QR(x[3], x[7], x[11], x[15])
    XHE_QR(x[0], x[5], x[10], x[15]) XHE_QR(x[1], x[6], x[11], x[12])
    XHE_QR(x[2], x[7], x[8], x[13]) XHE_QR(x[3], x[4], x[9], x[14])
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) out[i] = x[i] + s[i];
}

struct ChaChaKey { uint32_t k[8]; uint32_t nonce0, nonce1; };

// Uniform integers in [1, 2^bits) (DJN a, paillier.py:195) when bound == null,
// else in [1, bound) by rejection (non-DJN r in [1, n), paillier.py:215).
// `words` 32-bit words per element; element i (= base + thread) uses counter
// block (i * 64 + attempt) * blocks_per_draw.
XHE_DEV void rand_elem(const ChaChaKey& ck, int64_t i, int words, int bits, const uint32_t* __restrict__ bound,
                       uint32_t* __restrict__ o, int32_t* __restrict__ status, int first_attempt) {
  const int blocks = (words + 15) / 16;
  for (int attempt = first_attempt; attempt < 64; ++attempt) {
    for (int b = 0; b < blocks; ++b) {
      uint32_t ks[16];
      chacha20_block(ck.k, ck.nonce0, ck.nonce1, ((uint64_t)i * 64 + attempt) * blocks + b, ks);
      for (int t = 0; t < 16 && b * 16 + t < words; ++t) o[b * 16 + t] = ks[t];
    }
    // mask to `bits`
    for (int k = 0; k < words; ++k) {
      int lo = 32 * k;
      if (lo >= bits) o[k] = 0;
      else if (bits - lo < 32) o[k] &= (1u << (bits - lo)) - 1u;
    }
    bool zero = true;
    for (int k = 0; k < words; ++k) zero &= o[k] == 0;
    bool ok = !zero;
    if (ok && bound) {  // o < bound ?
      int c = 0;
      for (int k = words - 1; k >= 0 && c == 0; --k) c = o[k] < bound[k] ? -1 : (o[k] > bound[k] ? 1 : 0);
      ok = c < 0;
    }
    if (ok) { if (status) *status = ST_OK; return; }
  }
  if (status) *status = ST_VALUE;
}

__global__ void __launch_bounds__(256) k_rand_below(ChaChaKey ck, int64_t base, int64_t count, int words, int bits,
                             const uint32_t* __restrict__ bound, uint32_t* __restrict__ out,
                             int32_t* __restrict__ status) {
  const int64_t li = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (li >= count) return;
  // stream position base + li: independent of how a batch is split into launches
  rand_elem(ck, base + li, words, bits, bound, out + (size_t)li * words, status ? status + li : nullptr, 0);
}

// The DJN draw (no upper bound) with one thread per ChaCha20 block: the `tpe`
// (a power of two >= blocks) adjacent lanes of one wave make one element, and
// each writes its 64 bytes with 16-byte stores, so a wave writes consecutive
// rows. The same stream and the same words as k_rand_below: attempt 0 is the
// draw unless it is zero (probability 2^-bits), which the group's ballot
// detects and the group's first lane redraws from attempt 1 on.
// (launched with 256 threads: without the bound the compiler assumed
// 1,024-thread blocks, capped the kernel at 128 VGPRs and spilled 262 of
// them around the rare redraw path)
__global__ void __launch_bounds__(256) k_rand_djn(ChaChaKey ck, int64_t base, int64_t count, int words, int bits,
                                                  int tpe, uint32_t* __restrict__ out, int32_t* __restrict__ status) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t li = t / tpe;
  const int b = (int)(t & (tpe - 1));
  const int blocks = (words + 15) / 16;
  const bool mine = li < count && b < blocks;  // every lane reaches the ballot
  uint32_t ks[16];
  bool nz = false;
  if (mine) {
    chacha20_block(ck.k, ck.nonce0, ck.nonce1, (uint64_t)(base + li) * 64 * blocks + b, ks);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int k = b * 16 + u, lo = 32 * k;
      if (k >= words || lo >= bits) ks[u] = 0u;
      else if (bits - lo < 32) ks[u] &= (1u << (bits - lo)) - 1u;
      nz |= ks[u] != 0u;
    }
  }
  const uint64_t ball = __builtin_amdgcn_ballot_w64(nz);
  const int lane = (int)(threadIdx.x & 63);
  const uint64_t gmask = (tpe >= 64 ? ~0ull : ((1ull << tpe) - 1ull)) << (lane & ~(tpe - 1));
  if (!mine) return;
  if (ball & gmask) {
    uint32_t* o = out + (size_t)li * words + 16 * b;
    const int nwb = min(16, words - 16 * b);
    if ((reinterpret_cast<uintptr_t>(out) & 15u) == 0u && (words & 3) == 0) {
      for (int u = 0; u < nwb; u += 4)
        *reinterpret_cast<uint4*>(o + u) = make_uint4(ks[u], ks[u + 1], ks[u + 2], ks[u + 3]);
    } else {
      for (int u = 0; u < nwb; ++u) o[u] = ks[u];
    }
    if (b == 0 && status) status[li] = ST_OK;
  } else if (b == 0) {
    rand_elem(ck, base + li, words, bits, nullptr, out + (size_t)li * words, status ? status + li : nullptr, 1);
  }
}

// ============================================================== encrypt
// A table row is stored packed (RW = K/32 words mod p^2, K/16 mod n^2; 256
// bytes at 2048 bits:
// two whole 128-byte lines) and unpacked to W-bit limbs where it is used.
// One limb of a packed row.
template <int W, int PW>
XHE_DEV uint32_t packed_limb(const uint32_t* p, int l) {
  const int bit = W * l, k = bit >> 5, sh = bit & 31;
  const uint32_t lo = k < PW ? p[k] : 0u;
  const uint32_t hi = k + 1 < PW ? p[k + 1] : 0u;
  return __builtin_amdgcn_alignbit(hi, lo, sh) & ((1u << W) - 1u);
}
// Operand a read from a packed row (limbs beyond the row are zero).
template <int W, int PW>
struct ARowPacked {
  const uint32_t* __restrict__ p;
  XHE_DEV uint4 load4(int i) const {
    return make_uint4(packed_limb<W, PW>(p, i), packed_limb<W, PW>(p, i + 1), packed_limb<W, PW>(p, i + 2),
                      packed_limb<W, PW>(p, i + 3));
  }
};

// The packed row a lane just staged into its slot of a quad-major LDS image
// (word k at slot[(k/4)*256 + k%4]) rewritten in place as S4 limbs (limb i
// at slot[(i/4)*256 + i%4]). Limb quad L reads only words below 4L + 4 (W <
// 32), so walking L downwards never overwrites a word still to be read.
template <class MP2, int PW>
XHE_DEV void unpack_limbs_lds(uint32_t* slot) {
  constexpr int W = MP2::W;
  auto word = [&](int k) -> uint32_t { return k < PW ? slot[(k >> 2) * 256 + (k & 3)] : 0u; };
#pragma unroll
  for (int L = MP2::S4 / 4 - 1; L >= 0; --L) {
    uint32_t v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int l = 4 * L + j, bit = W * l, k = bit >> 5, sh = bit & 31;
      v[j] = l < MP2::S ? (__builtin_amdgcn_alignbit(word(k + 1), word(k), sh) & ((1u << W) - 1u)) : 0u;
    }
    *reinterpret_cast<uint4*>(slot + L * 256) = make_uint4(v[0], v[1], v[2], v[3]);
  }
}

// win-bit digit starting at bit `bit` of a little-endian word array (may
// straddle two words; bits beyond nwords read as zero)
XHE_DEV uint32_t digit_at(const uint32_t* w, int nwords, int bit, int win) {
  int k = bit >> 5, sh = bit & 31;
  uint64_t v = (uint64_t)word_or0(w, k, nwords) | ((uint64_t)word_or0(w, k + 1, nwords) << 32);
  return (uint32_t)(v >> sh) & ((1u << win) - 1u);
}

// Window w of a key's fixed-base tables: the first key.nhi windows are win+1
// bits wide (2^(win+1) rows each), the rest win bits; returns the window's
// digit of the exponent and sets row0 to its first table row. Wave-uniform.
XHE_DEV uint32_t win_digit(const KeyDev& key, const uint32_t* a, int aw, int w, int64_t& row0) {
  const int wide = w < key.nhi ? w : key.nhi;
  row0 = (int64_t)(w + wide) << key.win;
  return digit_at(a, aw, w * key.win + wide, key.win + (w < key.nhi ? 1 : 0));
}

// ---------------------------------------------------------------------------
// Encryption, DJN private key (CRT over p^2, q^2)   (paillier.py:193-209, 283)
//   c_P = (1 + n m) * h_P^a mod P^2        k_djn_pow, grid.y = prime (0: p, 1: q)
//   c   = c_q + q^2 ((c_p + 4p^2 - c_q) (q^2)^-1 mod p^2)    k_crt_enc
// Element rows live in ws as [prime][2*S4 limbs][count] (limb i of element e
// at row[i * count + e]); the second half of each row is wide-product scratch.
// Np2/Nq2: the p^2 / q^2 limb rows passed as separate noalias arguments so
// the modulus limbs are provably read-only and stay in SGPRs (scalar loads).
template <class MP2, int RW>
__global__ void __launch_bounds__(256, 2) k_djn_pow(KeyDev key, const uint32_t* __restrict__ Np2,
                                                    const uint32_t* __restrict__ Nq2,
                                                    const uint32_t* __restrict__ m_words,
                                                    const uint32_t* __restrict__ a_words, int aw, int64_t count,
                                                    uint32_t* __restrict__ ws) {
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MP2::TPI;
  if (e >= count) return;
  const int prime = blockIdx.y;
  const ModDev& md = prime ? key.q2 : key.p2;
  const uint32_t* tab = prime ? key.tab_q2 : key.tab_p2;
  MP2 M;
  M.init(prime ? Nq2 : Np2, md.n0inv);
  uint32_t b[MP2::L];
  M.load_words(b, m_words + (size_t)e * key.nw, key.nw);
  M.mul(b, ARow{prime ? key.nR2_q2 : key.nR2_p2});  // n m R mod P^2
  M.add_row(b, md.R1);                              // (1 + n m) R
  const uint32_t* ae = a_words + (size_t)e * aw;
  for (int w = 0; w < key.nwin; ++w) {
    int64_t row0;
    const uint32_t d = win_digit(key, ae, aw, w, row0);
    M.mul(b, ARowPacked<MP2::W, RW>{tab + (size_t)(row0 + d) * key.tab_rs});
  }
  M.mul(b, AOne{});
  M.reduce_once(b);
  M.store_strided(b, ws + (size_t)prime * 2 * MP2::S4 * count + e, (int)count);
}

// The squaring operand of an exponentiation, parked in LDS instead of a
// global workspace row (a squaring reads back the 74-152 limbs it just
// wrote: through LDS that round trip never leaves the CU). Per wave: 64 / TPI
// residues of S4 words. TPI == 1: quad-major image [quad][lane][4 words]
// (ds_write_b128 / ds_read_b128, conflict-free); TPI > 1: one contiguous row
// per lane group, read by the whole group (broadcast).
template <class M_>
struct SqLds {
  static constexpr int WORDS_PER_WAVE = 64 / M_::TPI * M_::S4;
  uint32_t* slot;
  XHE_DEV explicit SqLds(uint32_t* wave_img) {
    const int lane = threadIdx.x & 63;
    if constexpr (M_::TPI == 1) slot = wave_img + lane * 4;
    else slot = wave_img + (lane / M_::TPI) * M_::S4;
  }
  XHE_DEV void put(const uint32_t (&b)[M_::L]) const {
    if constexpr (M_::TPI == 1) {
#pragma unroll
      for (int q = 0; q < M_::S4 / 4; ++q) {
        uint4 v = make_uint4(4 * q < M_::S ? b[4 * q] : 0u, 4 * q + 1 < M_::S ? b[4 * q + 1] : 0u,
                             4 * q + 2 < M_::S ? b[4 * q + 2] : 0u, 4 * q + 3 < M_::S ? b[4 * q + 3] : 0u);
        *reinterpret_cast<uint4*>(slot + q * 256) = v;
      }
    } else {
      const int g = M_::G::g();
#pragma unroll
      for (int j = 0; j < M_::L; ++j) slot[g * M_::L + j] = b[j];
    }
    wave_sync_mem_();
  }
  XHE_DEV uint4 load4(int i) const {
    if constexpr (M_::TPI == 1) return *reinterpret_cast<const uint4*>(slot + (i >> 2) * 256);
    else return *reinterpret_cast<const uint4*>(slot + i);
  }
  // quad-wise writes (Mont::sqr's upper half, TPI == 1), then sync() before reading
  XHE_DEV void put4(int q, const uint4& v) const { *reinterpret_cast<uint4*>(slot + q * 256) = v; }
  XHE_DEV void sync() const { wave_sync_mem_(); }
};


// k_djn_pow for small batches: one 16-lane DPP row per residue (key.p2X/q2X)
// on the same one-lane tables (rows of RS4 words, Montgomery factor R): with
// the start value (1 + n m) C R', C = (R'/R)^nwin, the nwin table products
// leave (1 + n m) h^a R' exactly as the one-lane kernel leaves (1 + n m) h^a R.
// Output rows as k_djn_pow (RS4 limbs, stride count) for k_crt_enc.
template <class MX, int RS4, int RW>
__global__ void __launch_bounds__(256, 2) k_djn_pow_x(KeyDev key, const uint32_t* __restrict__ m_words,
                                                      const uint32_t* __restrict__ a_words, int aw, int64_t count,
                                                      uint32_t* __restrict__ ws) {
  static_assert(MX::TPI == 16, "16-lane shape");
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MX::TPI;
  if (e >= count) return;
  const int prime = blockIdx.y;
  const ModDev& md = prime ? key.q2X : key.p2X;
  const uint32_t* tab = prime ? key.tab_q2 : key.tab_p2;
  MX M;
  M.init(md.N, md.n0inv);
  uint32_t b[MX::L];
  M.load_words(b, m_words + (size_t)e * key.nw, key.nw);
  M.mul(b, ARow{prime ? key.nR2C_q2X : key.nR2C_p2X});  // n m C R'
  M.add_row(b, prime ? key.R1C_q2X : key.R1C_p2X);     // (1 + n m) C R'
  const uint32_t* ae = a_words + (size_t)e * aw;
  for (int w = 0; w < key.nwin; ++w) {
    int64_t row0;
    const uint32_t d = win_digit(key, ae, aw, w, row0);
    M.mul(b, ARowPacked<MX::W, RW>{tab + (size_t)(row0 + d) * key.tab_rs});
  }
  M.mul(b, AOne{});
  M.reduce_once(b);
  M.store_strided_n(b, ws + (size_t)prime * 2 * RS4 * count + e, (int)count, RS4);
}

#if XHE_LDS_ROWS
// Variant of k_djn_pow (TPI == 1) with each product's table row moved into
// LDS in one burst of LDS-DMA instructions (global_load_lds_dwordx4:
// instruction k moves quad k of every lane's row; image [quad][lane][4
// words], read back with conflict-free ds_read_b128). Every 128-B line of a
// row is then consumed while it is in L2, instead of by 16-B loads spread
// over the whole product.
typedef __attribute__((address_space(3))) void xhe_lds_void;
typedef __attribute__((address_space(1))) void xhe_glb_void;
struct ALdsQ {
  const uint32_t* q;  // this lane's slot of the wave image: limb i at q[(i/4)*256 + i%4]
  XHE_DEV uint4 load4(int i) const { return *reinterpret_cast<const uint4*>(q + (i >> 2) * 256); }
};

// c_P = (1 + n m) h^a mod P^2 for one element and one prime, table rows
// through the wave's LDS image; written as row `prime` of ws.
// XHE_DJN_FOLD: the product starts from the first window's row (h_0 R) and
// (1 + n m) enters once, in plain form, as the last multiplier, so the
// conversion out of Montgomery form is that same product: nwin + 1 products
// instead of nwin + 2 ((1 + n m) R first, a final multiply by 1).
template <class MP2, int RW>
XHE_DEV void djn_prime_lds(const KeyDev& key, const uint32_t* __restrict__ Np, const ModDev& md,
                           const uint32_t* tab, const uint32_t* nR2, const uint32_t* nR,
                           const uint32_t* __restrict__ m_words, const uint32_t* __restrict__ a_words, int aw,
                           int64_t count, int64_t e, int prime, uint32_t* img, const uint32_t* mine,
                           uint32_t* __restrict__ ws) {
  constexpr int NQ = MP2::S4 / 4;
  MP2 M;
  M.init(Np, md.n0inv);
  uint32_t b[MP2::L];
  const uint32_t* ae = a_words + (size_t)e * aw;
  auto stage = [&](int w) XHE_INL {
    int64_t row0;
    const uint32_t d = win_digit(key, ae, aw, w, row0);
    const uint32_t* row = tab + (size_t)(row0 + d) * key.tab_rs;
#pragma unroll
    for (int k = 0; k < RW / 4; ++k)
      __builtin_amdgcn_global_load_lds((xhe_glb_void*)(row + 4 * k), (xhe_lds_void*)(img + k * 256), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unpack_limbs_lds<MP2, RW>(img + (threadIdx.x & 63) * 4);
  };
#if XHE_DJN_FOLD
  (void)nR2;
  stage(0);
#pragma unroll
  for (int k = 0; k < NQ; ++k) {
    const uint4 v = ALdsQ{mine}.load4(4 * k);
    if (4 * k < MP2::S) b[4 * k] = v.x;
    if (4 * k + 1 < MP2::S) b[4 * k + 1] = v.y;
    if (4 * k + 2 < MP2::S) b[4 * k + 2] = v.z;
    if (4 * k + 3 < MP2::S) b[4 * k + 3] = v.w;
  }
  for (int w = 1; w < key.nwin; ++w) {
    stage(w);
    M.mul(b, ALdsQ{mine});
  }
  // park h^a R in this lane's slot of the image (quad-major, as a staged row)
  SqLds<MP2>(img).put(b);
  M.load_words(b, m_words + (size_t)e * key.nw, key.nw);
  M.mul(b, ARow{nR});  // n m mod P^2 (< 2 P^2), plain
  b[0] += 1u;          // 1 + n m: one limb may reach 2^W, inside the lazy-carry bound
  M.mul(b, ALdsQ{mine});  // (1 + n m) h^a mod P^2
#else
  (void)nR;
  M.load_words(b, m_words + (size_t)e * key.nw, key.nw);
  M.mul(b, ARow{nR2});     // n m R mod P^2
  M.add_row(b, md.R1);     // (1 + n m) R
  for (int w = 0; w < key.nwin; ++w) {
    stage(w);
    M.mul(b, ALdsQ{mine});
  }
  M.mul(b, AOne{});
#endif
  M.reduce_once(b);
  M.store_strided(b, ws + (size_t)prime * 2 * MP2::S4 * count + e, (int)count);
}

template <class MP2, int RW>
__global__ void __launch_bounds__(128, 2) k_djn_pow_lds(KeyDev key, const uint32_t* __restrict__ Np2,
                                                        const uint32_t* __restrict__ Nq2,
                                                        const uint32_t* __restrict__ m_words,
                                                        const uint32_t* __restrict__ a_words, int aw, int64_t count,
                                                        uint32_t* __restrict__ ws) {
  static_assert(MP2::TPI == 1, "LDS row staging is per lane");
  __shared__ __attribute__((aligned(16))) uint32_t img_all[2][(MP2::S4 / 4) * 256];
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int prime = blockIdx.y;
  uint32_t* img = img_all[(threadIdx.x >> 6) & 1];
  if (e >= count) return;
  djn_prime_lds<MP2, RW>(key, prime ? Nq2 : Np2, prime ? key.q2 : key.p2, prime ? key.tab_q2 : key.tab_p2,
                     prime ? key.nR2_q2 : key.nR2_p2, prime ? key.nR_q2 : key.nR_p2, m_words, a_words, aw, count, e,
                     prime, img, img + (threadIdx.x & 63) * 4, ws);
}

#endif

#if XHE_PMD && XHE_LDS_ROWS
// ---------------------------------------------------------------------------
// DJN encryption in Montgomery digits (pdigit_dev.hpp PMD; 2048-bit keys,
// K = 37 limbs of P): c_P = (1 + n m) h^a mod P^2 as k_djn_pow_lds computes
// it, with the table products in digit form. The tables hold each row as its
// digits (e, f) < P (k_tab_to_pmd), packed 32 + 32 words. Per prime and
// element: the first window's row is the start value; each further window's
// row is LDS-DMA'd into the wave's image, unpacked into interleaved limb
// pairs, and multiplied in (nwin - 1 digit products, 5 K^2 mads each); the
// result goes back to the 74-limb Montgomery form (R a + P c = h^a R^2 mod
// P^2, to_mont2) for the two Montgomery products that bring in (1 + n m) and
// leave Montgomery form, exactly as in djn_prime_lds. Output rows as
// k_djn_pow_lds (MP2 limbs, [prime][2 S4][count]) for k_crt_enc_w.
//
// G > 1 (small batches, where the chip is not full and the chain of nwin
// dependent products is the latency): G adjacent lanes share an element; lane
// g multiplies windows g, g + G, g + 2G, ... and the G partial products are
// combined by a tree through the lanes' LDS slots (log2 G levels, the writer's
// state streamed as the reader's operand), so the chain is ~nwin/G + log2 G
// products; lane 0 of the group finishes. Products of Montgomery-digit states
// are digit states of the product, so the result is the same residue.
template <class MP2, int KP, int RW, int G = 1>
__global__ void __launch_bounds__(128, 2) k_djn_pmd(KeyDev key, const uint32_t* __restrict__ Pp,
                                                    const uint32_t* __restrict__ Pq, const uint32_t* __restrict__ Np2,
                                                    const uint32_t* __restrict__ Nq2,
                                                    const uint32_t* __restrict__ m_words,
                                                    const uint32_t* __restrict__ a_words, int aw, int64_t count,
                                                    uint32_t* __restrict__ ws) {
  static_assert(MP2::TPI == 1 && MP2::S == 2 * KP && MP2::W == 28, "digits of the one-lane P^2 shape");
  using D = PMD<KP>;
  constexpr int NQ = D::NQ > MP2::S4 / 4 ? D::NQ : MP2::S4 / 4;
  __shared__ __attribute__((aligned(16))) uint32_t img_all[2][NQ * 256];
  __shared__ __attribute__((aligned(16))) uint32_t topc[(KP + 3) & ~3];
  const int prime = blockIdx.y;
  const uint32_t* tc = prime ? key.topc_q : key.topc_p;
  if (threadIdx.x < KP) topc[threadIdx.x] = tc[threadIdx.x];
  __syncthreads();
  static_assert(G >= 1 && G <= 64 && (G & (G - 1)) == 0, "lane groups of a power of two, inside one wave");
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t e = t / G;
  const int g = (int)(threadIdx.x & (G - 1));
  if (e >= count) return;  // whole groups (G divides the wave)
  uint32_t* img = img_all[(threadIdx.x >> 6) & 1];
  uint32_t* slot = img + (threadIdx.x & 63) * 4;
  const uint32_t* tab = prime ? key.tab_q2 : key.tab_p2;
  const uint32_t* ae = a_words + (size_t)e * aw;
  D M;
  M.init(prime ? Pq : Pp, prime ? key.q.n0inv : key.p.n0inv);
  auto stage = [&](int w) XHE_INL {
    int64_t row0;
    const uint32_t d = win_digit(key, ae, aw, w, row0);
    const uint32_t* row = tab + (size_t)(row0 + d) * key.tab_rs;
#pragma unroll
    for (int k = 0; k < RW / 4; ++k)
      __builtin_amdgcn_global_load_lds((xhe_glb_void*)(row + 4 * k), (xhe_lds_void*)(img + k * 256), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unpack_pairs_lds<KP, RW>(slot);
  };
  uint32_t a[KP], c[KP];
  if (G == 1 || g < key.nwin) {
    stage(g);
#pragma unroll
    for (int q = 0; q < D::NQ; ++q) {
      const uint4 v = *reinterpret_cast<const uint4*>(slot + q * 256);
      if (2 * q < KP) a[2 * q] = v.x, c[2 * q] = v.y;
      if (2 * q + 1 < KP) a[2 * q + 1] = v.z, c[2 * q + 1] = v.w;
    }
  }
  for (int w = g + G; w < key.nwin; w += G) {
    stage(w);
    M.mul(a, c, slot, topc);
  }
  if constexpr (G > 1) {
    // tree over the group: at level s, lane g + s (g a multiple of 2s) parks
    // its state in its slot and lane g multiplies it in
#pragma unroll
    for (int s = 1; s < G; s <<= 1) {
      const bool writer = (g & (2 * s - 1)) == s && g < key.nwin;
      const bool reader = (g & (2 * s - 1)) == 0 && g + s < key.nwin;
      if (writer) {
#pragma unroll
        for (int q = 0; q < D::NQ; ++q)
          *reinterpret_cast<uint4*>(slot + q * 256) =
              make_uint4(2 * q < KP ? a[2 * q] : 0u, 2 * q < KP ? c[2 * q] : 0u, 2 * q + 1 < KP ? a[2 * q + 1] : 0u,
                         2 * q + 1 < KP ? c[2 * q + 1] : 0u);
      }
      wave_sync_mem_();
      if (reader) M.mul(a, c, slot + 4 * s, topc);
      wave_sync_mem_();
    }
    if (g != 0) return;
  }
  {
    uint32_t x[2 * KP];
    M.to_mont2(a, c, x);  // h^a R^2 mod P^2, unreduced (< 2^13 P^2)
#pragma unroll
    for (int q = 0; q < MP2::S4 / 4; ++q)
      *reinterpret_cast<uint4*>(slot + q * 256) =
          make_uint4(4 * q < 2 * KP ? x[4 * q] : 0u, 4 * q + 1 < 2 * KP ? x[4 * q + 1] : 0u,
                     4 * q + 2 < 2 * KP ? x[4 * q + 2] : 0u, 4 * q + 3 < 2 * KP ? x[4 * q + 3] : 0u);
  }
  MP2 N;
  N.init(prime ? Nq2 : Np2, prime ? key.q2.n0inv : key.p2.n0inv);
  uint32_t b[MP2::L];
  N.load_words(b, m_words + (size_t)e * key.nw, key.nw);
  N.mul(b, ARow{prime ? key.nR_q2 : key.nR_p2});  // n m mod P^2 (< 2 P^2), plain
  b[0] += 1u;                                     // 1 + n m
  N.mul(b, ALdsQ{slot});                          // (1 + n m) h^a mod P^2
  N.reduce_once(b);
  N.store_strided(b, ws + (size_t)prime * 2 * MP2::S4 * count + e, (int)count);
}

// x <- x^E mod P^2 in Montgomery digits for an exponent E shared by every
// lane (P - 1: the schedule is wave-uniform): 5-bit sliding window as
// pow_uniform_exp, odd powers x^(2t+1), t < 16, in this lane's column of a
// global table (entry t, quad q at tab[(t NQ + q) G], interleaved limb
// pairs). Every product reads its second operand from the lane's LDS slot:
// a squaring parks the state there, a table product copies the entry there
// (19 loads in flight at once); squarings take PMD::sqr (4 K^2 mads).
// (tab: the table's uniform base, lane: this lane's column, G columns; the
// per-lane address is formed at each use, not held across the products)
template <int KP>
XHE_DEV void pmd_pow_uniform(const PMD<KP>& M, uint32_t (&a)[KP], uint32_t (&c)[KP], const uint32_t* ex, int ebits,
                             uint4* __restrict__ tab_base, int lane, int G, uint32_t* slot, const uint32_t* topc) {
  constexpr int NQ = PMD<KP>::NQ;
#define tab (tab_base + opaque_i(lane))
  auto quad = [&](int q) -> uint4 {
    return make_uint4(2 * q < KP ? a[2 * q] : 0u, 2 * q < KP ? c[2 * q] : 0u, 2 * q + 1 < KP ? a[2 * q + 1] : 0u,
                      2 * q + 1 < KP ? c[2 * q + 1] : 0u);
  };
  auto put_slot = [&]() XHE_INL {
#pragma unroll
    for (int q = 0; q < NQ; ++q) *reinterpret_cast<uint4*>(slot + q * 256) = quad(q);
  };
  auto put_tab = [&](int t) XHE_INL {
#pragma unroll
    for (int q = 0; q < NQ; ++q) tab[((size_t)t * NQ + q) * G] = quad(q);
  };
  auto tab_to_slot = [&](int t) XHE_INL {
    uint4 v[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) v[q] = tab[((size_t)t * NQ + q) * G];
#pragma unroll
    for (int q = 0; q < NQ; ++q) *reinterpret_cast<uint4*>(slot + q * 256) = v[q];
  };
  auto tab_to_regs = [&](int t) XHE_INL {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint4 v = tab[((size_t)t * NQ + q) * G];
      if (2 * q < KP) a[2 * q] = v.x, c[2 * q] = v.y;
      if (2 * q + 1 < KP) a[2 * q + 1] = v.z, c[2 * q + 1] = v.w;
    }
  };
  auto bit = [&](int i) { return (ex[i >> 5] >> (i & 31)) & 1u; };
  int i = ebits - 1;
  while (i >= 0 && !bit(i)) --i;
  int pend_sq = 0, pend_mul = -1;
  bool sq = false;  // the next product is a squaring (PMD::sqr) of the parked state
  // the next product of the window schedule: its operand into the slot
  auto next_op = [&]() -> bool {
    while (true) {
      if (pend_sq > 0) {
        put_slot();
        --pend_sq;
        sq = true;
        return true;
      }
      if (pend_mul >= 0) {
        tab_to_slot(pend_mul);
        pend_mul = -1;
        sq = false;
        return true;
      }
      if (i < 0) return false;
      if (!bit(i)) {
        pend_sq = 1;
        --i;
      } else {
        int j = i - 4 < 0 ? 0 : i - 4;
        while (!bit(j)) ++j;  // window [i..j] ends in a set bit
        uint32_t val = 0;
        for (int k = i; k >= j; --k) val = (val << 1) | bit(k);
        pend_sq = i - j + 1;
        pend_mul = (int)(val >> 1);
        i = j - 1;
      }
    }
  };
  // Products in order: x x -> x^2 (then the slot keeps x^2 and the state
  // returns to x), x^(2t-1) x^2 -> tab[t] for t = 1..15, then the window
  // schedule - all through ONE inlined product.
  put_tab(0);
  put_slot();
  sq = true;
  int t = -1;
#pragma unroll 1
  while (true) {
    if (sq) M.sqr(a, c, slot, topc);
    else M.mul(a, c, slot, topc);
    if (t < 15) {
      sq = false;
      if (t < 0) {
        put_slot();
        tab_to_regs(0);
      } else {
        put_tab(t + 1);
      }
      ++t;
      if (t < 15) continue;
      // first window of the exponent: its odd power is the start value
      int j = i - 4 < 0 ? 0 : i - 4;
      while (!bit(j)) ++j;
      uint32_t val = 0;
      for (int k = i; k >= j; --k) val = (val << 1) | bit(k);
      tab_to_regs((int)(val >> 1));
      i = j - 1;
    }
    if (!next_op()) break;
  }
#undef tab
}

// ---------------------------------------------------------------------------
// DJN encryption in Montgomery digits over 4 lanes (PMDX, 3072/4096-bit keys;
// the one-lane k_djn_pmd's construction with the multi-lane product of
// k_ndig_*): the tables hold each row as its digits (e, f) < P (RW/2 words
// each, k_tab_to_pmdx); per prime and element group the first window's row is
// the start state and every further row is unpacked into the group's LDS
// pairs and multiplied in. k_pmdx_enc_out then leaves digits (from_digits),
// folds in (1 + n m) in base P - (1 + n m) y = y0 + P ((y1 + y0 Q m) mod P),
// Q the other prime, as y0 Q m = MontMul(MontMul(y0, REDC(m)), Q R^3) - and
// writes c_P's words; k_words_to_rows puts them into the MP2 rows k_crt_enc
// reads. Digit state between the kernels: st [prime][pair i][count].
template <class D>
struct PmdxKey {
  const ModDev& md;
  const uint32_t *kn2, *rmn, *topc, *fold, *hpR;
  const uint2 *dwt, *dw;
  // prime 0: p, 1: q, 2: n (the digits mod n^2 of k_ndig_*; public DJN tables)
  XHE_DEV PmdxKey(const KeyDev& k, int prime)
      : md(prime == 2 ? k.nd : prime ? k.dq : k.dp),
        kn2(prime == 2 ? k.nd_kn2 : prime ? k.x_kn2_q : k.x_kn2_p),
        rmn(prime == 2 ? k.nd_rmn : prime ? k.x_rmn_q : k.x_rmn_p),
        topc(prime == 2 ? k.nd_topc : prime ? k.x_topc_q : k.x_topc_p),
        fold(prime == 2 ? nullptr : prime ? k.x_fold_q : k.x_fold_p),
        hpR(prime == 2 ? nullptr : prime ? k.x_hpR_q : k.x_hpR_p),
        dwt(prime == 2 ? k.nd_dwt : prime ? k.x_dwt_q : k.x_dwt_p),
        dw(prime == 2 ? k.nd_dw : prime ? k.x_dw_q : k.x_dw_p) {}
};

template <class D, int RW>
__global__ void __launch_bounds__(128, 2) k_djn_pmdx(KeyDev key, const uint32_t* __restrict__ a_words, int aw,
                                                     int64_t count, uint2* __restrict__ st) {
  constexpr int GPB = 128 / D::TPI, L = D::L;
  __shared__ uint2 ops_all[D::K * GPB];
  __shared__ __attribute__((aligned(16))) uint32_t topc[D::K];
  const int prime = blockIdx.y;
  const PmdxKey<D> pk(key, prime);
  for (int i = threadIdx.x; i < D::K; i += blockDim.x) topc[i] = pk.topc[i];
  __syncthreads();
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / D::TPI;
  if (e >= count) return;
  const int g = D::G::g();
  uint2* ops = ops_all + threadIdx.x / D::TPI;
  const uint32_t* tab = prime ? key.tab_q2 : key.tab_p2;
  const uint32_t* ae = a_words + (size_t)e * aw;
  D X;
  X.init(pk.md.N, pk.md.n0inv);
  uint32_t a[L], c[L];
  {
    int64_t row0;
    const uint32_t d = win_digit(key, ae, aw, 0, row0);
    const uint32_t* row = tab + (size_t)(row0 + d) * key.tab_rs;
    pmdx_load<D, 0>(a, row, RW / 2, g);
    pmdx_load<D, 0>(c, row + RW / 2, RW / 2, g);
  }
  for (int w = 1; w < key.nwin; ++w) {
    int64_t row0;
    const uint32_t d = win_digit(key, ae, aw, w, row0);
    pmdx_stage_row<D>(pmdx_launder(tab) + (size_t)(row0 + d) * key.tab_rs, RW / 2, ops, GPB);
    wave_sync_mem_();
    X.template run<false>(a, c, OpLds{ops, GPB}, topc);
    wave_sync_mem_();
  }
  ndig_st_store<D>(a, c, st + (size_t)prime * D::K * count, count, e);
}

template <class D, int RW>
__global__ void __launch_bounds__(128, 2) k_pmdx_enc_out(KeyDev key, const uint32_t* __restrict__ m_words,
                                                         int64_t count, const uint2* __restrict__ st,
                                                         uint32_t* __restrict__ rows27, uint32_t* __restrict__ words) {
  constexpr int L = D::L, S4 = D::MN::S4;
  const int prime = blockIdx.y;
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / D::TPI;
  if (e >= count) return;
  const int g = D::G::g();
  const PmdxKey<D> pk(key, prime);
  D X;
  X.init(pk.md.N, pk.md.n0inv);
  uint32_t y0[L], y1[L];
  {
    uint32_t a[L], c[L];
    ndig_st_load<D>(a, c, st + (size_t)prime * D::K * count, count, e);
    pmdx_from_digits(X, a, c, y0, y1);
  }
  const int cnt = (int)count;
  uint32_t* rows = rows27 + (size_t)prime * 2 * S4 * count + e;
  {  // y1 <- (y1 + y0 Q m) mod P
    uint32_t lo[L], hi[L], mq[L];
    const uint32_t* me = m_words + (size_t)e * key.nw;
    pmdx_load<D, 0>(lo, me, key.nw, g);
    pmdx_load<D, D::K>(hi, me, key.nw, g);
    uint64_t T[L];
#pragma unroll
    for (int j = 0; j < L; ++j) {
      T[j] = lo[j];
      mq[j] = 0;
    }
    X.template redc_q<true>(T, hi, mq);
    D::normalize_top(T, lo);  // m R^-1 mod P (< 2P)
    uint32_t* trow = rows + (size_t)S4 * count;
    X.M.store_strided(lo, trow, cnt);
    wave_sync_mem_();
#pragma unroll
    for (int j = 0; j < L; ++j) lo[j] = y0[j];
    X.M.mul(lo, AStrided{trow, cnt});  // y0 m R^-2
    X.M.mul(lo, ARow{pk.fold});        // y0 m Q (< 2P)
#pragma unroll
    for (int j = 0; j < L; ++j) T[j] = (uint64_t)y1[j] + lo[j];
    D::normalize_top(T, y1);
    X.M.reduce_once(y1);
    X.M.reduce_once(y1);
  }
  X.M.store_strided(y0, rows, cnt);
  wave_sync_mem_();
  X.M.wide_mul_add_store(y1, ARow{pk.md.N}, rows, cnt, words + ((size_t)prime * count + e) * RW, RW);
}

// ---- Decryption of 3072/4096-bit keys in Montgomery digits (PMDX; as
// k_dec_pmd_* for 2048): c mod P^2 as words (k_p2_reduce_words, the 4-lane
// Montgomery shape), its digits (k_dec_pmdx_in), x = c^(P-1) by the
// wave-uniform sliding window in digits (k_dec_pmdx_pow), and on the way out
// (k_dec_pmdx_out) from_digits gives x = y0 + P y1 with y0 = x mod P = 1, so
// L_P(x) = (x - 1) / P = y1 exactly and m_P = y1 hp mod P is one product
// (paillier.py:341-368, context.py:190-194). m_P words -> MP rows
// (k_words_to_rows) -> k_crt_dec.
template <class MP2L, int RW>
__global__ void __launch_bounds__(256, 2) k_p2_reduce_words(KeyDev key, const uint32_t* __restrict__ c_words,
                                                            int64_t count, uint32_t* __restrict__ scr,
                                                            uint32_t* __restrict__ words) {
  const int prime = blockIdx.y;
  const ModDev& md = prime ? key.q2L : key.p2L;
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MP2L::TPI;
  if (e >= count) return;
  const int st = (int)count;
  uint32_t* sq = scr + (size_t)prime * MP2L::S4 * count + e;
  const int n2w = key.n2w;
  const uint32_t* cw = c_words + (size_t)e * n2w;
  MP2L M;
  M.init(md.N, md.n0inv);
  uint32_t b[MP2L::L];
  {  // high limbs [S, 2S) of c into the scratch row (the REDC's upper half)
    const int g = MP2L::G::g();
#pragma unroll
    for (int j = 0; j < MP2L::L; ++j) {
      const int J = MP2L::S + g * MP2L::L + j;
      const int bit = MP2L::W * J, k = bit >> 5, sh = bit & 31;
      const uint32_t lo = word_or0(cw, k, n2w), h2 = word_or0(cw, k + 1, n2w);
      sq[(size_t)(g * MP2L::L + j) * st] = (uint32_t)((((uint64_t)h2 << 32) | lo) >> sh) & MP2L::MASK;
    }
    if (g == 0)
      for (int j = MP2L::S; j < MP2L::S4; ++j) sq[(size_t)j * st] = 0u;
  }
  M.load_words(b, cw, n2w);  // low S limbs
  wave_sync_mem_();
  M.redc_wide(b, AStrided{sq, st});  // c R^-1 mod P^2
  M.mul(b, ARow{md.R2});             // c mod P^2
  M.reduce_once(b);
  wave_sync_mem_();
  store_packed(M, b, sq, st, words + ((size_t)prime * count + e) * RW, RW);
}

template <class D, int RW>
__global__ void __launch_bounds__(128, 2) k_dec_pmdx_in(KeyDev key, const uint32_t* __restrict__ words,
                                                        int64_t count, uint2* __restrict__ st) {
  constexpr int L = D::L;
  __shared__ __attribute__((aligned(16))) uint32_t topc[D::K];
  const int prime = blockIdx.y;
  const PmdxKey<D> pk(key, prime);
  for (int i = threadIdx.x; i < D::K; i += blockDim.x) topc[i] = pk.topc[i];
  __syncthreads();
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / D::TPI;
  if (e >= count) return;
  const int g = D::G::g();
  D X;
  X.init(pk.md.N, pk.md.n0inv);
  uint32_t lo[L], hi[L], a[L], c[L];
  const uint32_t* xe = words + ((size_t)prime * count + e) * RW;
  pmdx_load<D, 0>(lo, xe, RW, g);
  pmdx_load<D, D::K>(hi, xe, RW, g);
  pmdx_to_digits(X, lo, hi, pk.kn2, pk.rmn, pk.dw, topc, a, c);
  ndig_st_store<D>(a, c, st + (size_t)prime * D::K * count, count, e);
}

// st <- st^(P-1) per prime; tab: 16 digit states per group slot and prime
template <class D>
__global__ void __launch_bounds__(128, 2) k_dec_pmdx_pow(KeyDev key, int64_t count, uint2* __restrict__ st,
                                                         uint2* __restrict__ ws) {
  constexpr int GPB = 128 / D::TPI, L = D::L;
  __shared__ uint2 ops_all[D::K * GPB];
  __shared__ __attribute__((aligned(16))) uint32_t topc[D::K];
  const int prime = blockIdx.y;
  const PmdxKey<D> pk(key, prime);
  for (int i = threadIdx.x; i < D::K; i += blockDim.x) topc[i] = pk.topc[i];
  __syncthreads();
  const int gs = (int)gridDim.x * GPB;
  const int gid0 = (int)blockIdx.x * GPB + (int)threadIdx.x / D::TPI;
  uint2* ops = ops_all + threadIdx.x / D::TPI;
  uint2* tab = ws + (size_t)prime * 16 * D::K * gs + gid0;
  uint2* stp = st + (size_t)prime * D::K * count;
  const uint32_t* ex = prime ? key.qm1_words : key.pm1_words;
  const int ebits = prime ? key.qm1_bits : key.pm1_bits;
  for (int64_t e = gid0; e < count; e += gs) {
    D X;
    X.init(pk.md.N, pk.md.n0inv);
    uint32_t a[L], c[L];
    ndig_st_load<D>(a, c, stp, count, e);
    pmdx_pow_uniform(X, a, c, ex, ebits, tab, gs, ops, GPB, topc);
    ndig_st_store<D>(a, c, stp, count, e);
  }
}

// digits of x = c^(P-1) -> m_P = L_P(x) hp mod P as NWH words ([prime][count][NWH])
template <class D, int NWH>
__global__ void __launch_bounds__(128, 2) k_dec_pmdx_out(KeyDev key, int64_t count, const uint2* __restrict__ st,
                                                         uint32_t* __restrict__ scr, uint32_t* __restrict__ words) {
  constexpr int L = D::L;
  const int prime = blockIdx.y;
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / D::TPI;
  if (e >= count) return;
  const PmdxKey<D> pk(key, prime);
  D X;
  X.init(pk.md.N, pk.md.n0inv);
  uint32_t y0[L], y1[L];
  {
    uint32_t a[L], c[L];
    ndig_st_load<D>(a, c, st + (size_t)prime * D::K * count, count, e);
    pmdx_from_digits(X, a, c, y0, y1);
  }
  X.M.mul(y1, ARow{pk.hpR});  // L_P(x) hp mod P (< 2P)
  X.M.reduce_once(y1);
  store_packed(X.M, y1, scr + (size_t)prime * D::MN::S4 * count + e, (int)count,
               words + ((size_t)prime * count + e) * NWH, NWH);
}

// c_P words [prime][count][nwords] -> the MP2 rows of k_crt_enc ([prime][2 S4][count])
template <class MP2>
__global__ void __launch_bounds__(256, 2) k_words_to_rows(const uint32_t* __restrict__ words, int nwords,
                                                          int64_t count, uint32_t* __restrict__ ws) {
  const int prime = blockIdx.y;
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MP2::TPI;
  if (e >= count) return;
  MP2 N;
  uint32_t b[MP2::L];
  N.load_words(b, words + ((size_t)prime * count + e) * nwords, nwords);
  N.store_strided(b, ws + (size_t)prime * 2 * MP2::S4 * count + e, (int)count);
}

// Table rows X = x R_MP2 mod P^2 (packed RW words, reduced) -> the digits
// (e, f) of x, RW/2 words each, in place: to_digits with the constant
// digits of R^2 R_MP2^-1 (one group of TPI lanes per row)
template <class D, int RW>
__global__ void __launch_bounds__(128, 2) k_tab_to_pmdx(KeyDev key, int prime, uint32_t* __restrict__ tab,
                                                        int64_t rows, int64_t rs) {
  constexpr int GPB = 128 / D::TPI, L = D::L;
  __shared__ uint2 ops_all[D::K * GPB];
  __shared__ __attribute__((aligned(16))) uint32_t topc[D::K];
  const PmdxKey<D> pk(key, prime);
  for (int i = threadIdx.x; i < D::K; i += blockDim.x) topc[i] = pk.topc[i];
  __syncthreads();
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / D::TPI;
  if (r >= rows) return;
  const int g = D::G::g();
  uint2* ops = ops_all + threadIdx.x / D::TPI;
  uint32_t* row = tab + (size_t)r * rs;
  D X;
  X.init(pk.md.N, pk.md.n0inv);
  uint32_t a[L], c[L];
  {
    uint32_t lo[L], hi[L];
    pmdx_load<D, 0>(lo, row, RW, g);
    pmdx_load<D, D::K>(hi, row, RW, g);
    pmdx_to_digits(X, lo, hi, pk.kn2, pk.rmn, pk.dwt, topc, a, c);
  }
  // canonical digits for the packed row (a product leaves a < P(1 + 2P/R)
  // and c < R + 4P, which would not fit RW/2 words): a - kP and (c + kR) mod
  // P (R (a - P) + P (c + R) = R a + P c), the latter as MontMul(REDC(c + kR),
  // R^2) = (c + kR) mod P
  {
    const bool k = X.csub(a);
    uint64_t T[L];
    uint32_t zero[L], mq[L];
#pragma unroll
    for (int j = 0; j < L; ++j) {
      T[j] = c[j];
      zero[j] = 0;
      mq[j] = 0;
    }
    if (k && D::last()) T[L - 1] += (uint64_t)1 << D::W;
    X.template redc_q<false>(T, zero, mq);
    D::normalize_top(T, c);
    X.M.mul(c, ARow{pk.md.R2});
    X.M.reduce_once(c);
  }
  pmdx_park<D>(a, c, ops, GPB);
  wave_sync_mem_();
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(ops);
  pack_words_<D::W, D::TPI>(lds, 2 * GPB, D::K, row, RW / 2);
  pack_words_<D::W, D::TPI>(lds + 1, 2 * GPB, D::K, row + RW / 2, RW / 2);
}

// k_dec_pow (one lane per residue) in Montgomery digits, as three kernels so
// that each has the registers to itself: k_dec_pmd_in (c -> c R^2 mod P^2 by
// the 74-limb REDC and a product by R^3, then its digits, pmd_from_mont2),
// k_dec_pmd_pow (x^(P-1) in digits) and k_dec_pmd_out (back through R a + P c
// and one Montgomery product by 1; X_P = x - 1 written to xrows
// [prime][xs4][count] exactly as k_dec_pow<MP2, 0>). The digit state between
// them: st [prime][NQ quads][count] uint4 (interleaved limb pairs).
// k_dec_pmd_in and k_dec_pmd_pow also serve the private non-DJN encryption
// (r mod P^2 -> digits, r^(e_P); k_nodjn_pmd_out finishes it): c_words holds
// nwords words per element (a ciphertext, or a draw r < n).
template <class MP2, int KP>
__global__ void __launch_bounds__(128, 2) k_dec_pmd_in(KeyDev key, const uint32_t* __restrict__ Pp,
                                                       const uint32_t* __restrict__ Pq,
                                                       const uint32_t* __restrict__ Np2,
                                                       const uint32_t* __restrict__ Nq2,
                                                       const uint32_t* __restrict__ c_words, int nwords,
                                                       int64_t count, uint4* __restrict__ st) {
  static_assert(MP2::TPI == 1 && MP2::S == 2 * KP && MP2::W == 28, "digits of the one-lane P^2 shape");
  constexpr int NQ = PMD<KP>::NQ;
  __shared__ __attribute__((aligned(16))) uint32_t img_all[2][(MP2::S4 / 4) * 256];
  const int prime = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  const ModDev& md = prime ? key.q2 : key.p2;
  uint32_t* slot = img_all[(threadIdx.x >> 6) & 1] + (threadIdx.x & 63) * 4;
  const int n2w = nwords;
  const uint32_t* cw = c_words + (size_t)e * n2w;
  uint32_t x[MP2::L];
  {
    MP2 N;
    N.init(prime ? Nq2 : Np2, md.n0inv);
    // high limbs [S, 2S) of c into the slot (the REDC's upper-half source)
#pragma unroll
    for (int q = 0; q < MP2::S4 / 4; ++q) {
      uint32_t v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int J = MP2::S + 4 * q + r, bit = MP2::W * J, k = bit >> 5, sh = bit & 31;
        const uint32_t lo = word_or0(cw, k, n2w), h2 = word_or0(cw, k + 1, n2w);
        v[r] = 4 * q + r < MP2::S ? (uint32_t)((((uint64_t)h2 << 32) | lo) >> sh) & MP2::MASK : 0u;
      }
      *reinterpret_cast<uint4*>(slot + q * 256) = make_uint4(v[0], v[1], v[2], v[3]);
    }
    N.load_words(x, cw, n2w);  // low S limbs
    N.redc_wide(x, ALdsQ{slot});
    N.mul(x, ARow{md.R3});  // c R^2 mod P^2 (< 2 P^2)
  }
  __builtin_amdgcn_sched_barrier(0);
  PMD<KP> M;
  M.init(prime ? Pq : Pp, prime ? key.q.n0inv : key.p.n0inv);
  uint32_t a[KP], c[KP];
  pmd_from_mont2<KP>(M, x, prime ? key.q.R1 : key.p.R1, a, c);
  uint4* so = st + (size_t)prime * NQ * count + e;
#pragma unroll
  for (int q = 0; q < NQ; ++q)
    so[(size_t)q * count] = make_uint4(2 * q < KP ? a[2 * q] : 0u, 2 * q < KP ? c[2 * q] : 0u,
                                       2 * q + 1 < KP ? a[2 * q + 1] : 0u, 2 * q + 1 < KP ? c[2 * q + 1] : 0u);
}

// st <- st^E_P per prime: E = P - 1 (decrypt, mode 0) or e_P = n mod
// phi(P^2) (mode 1: the private non-DJN obfuscator, paillier.py:214-227).
// The exponent is picked from the key inside (4 more pointer/int arguments
// spill SGPRs in this register-bound kernel).
template <int KP>
__global__ void __launch_bounds__(128, 2) k_dec_pmd_pow(KeyDev key, const uint32_t* __restrict__ Pp,
                                                        const uint32_t* __restrict__ Pq, int mode, int64_t count,
                                                        uint4* __restrict__ st, uint4* __restrict__ ws) {
  using D = PMD<KP>;
  constexpr int NQ = D::NQ;
  __shared__ __attribute__((aligned(16))) uint32_t img_all[2][NQ * 256];
  __shared__ __attribute__((aligned(16))) uint32_t topc[(KP + 3) & ~3];
  const int prime = blockIdx.y;
  const uint32_t* tcg = prime ? key.topc_q : key.topc_p;
  if (threadIdx.x < KP) topc[threadIdx.x] = tcg[threadIdx.x];
  __syncthreads();
  const uint32_t* ex = mode ? (prime ? key.eq_words : key.ep_words) : (prime ? key.qm1_words : key.pm1_words);
  const int ebits = mode ? (prime ? key.eq_bits : key.ep_bits) : (prime ? key.qm1_bits : key.pm1_bits);
  // 32-bit indices (count < 2^31 per launch), per-lane addresses formed at
  // use: the product needs every register it can get
  const int G = (int)(gridDim.x * blockDim.x);
  const int gid0 = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  uint4* tab = ws + (size_t)prime * 16 * NQ * G;
  uint4* stp = st + (size_t)prime * NQ * count;
  uint32_t* slot = img_all[(threadIdx.x >> 6) & 1] + (threadIdx.x & 63) * 4;
  D M;
  M.init(prime ? Pq : Pp, prime ? key.q.n0inv : key.p.n0inv);
  for (int e = gid0; e < (int)count; e += G) {
    uint32_t a[KP], c[KP];
    {
      const uint4* se = stp + e;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const uint4 v = se[(size_t)q * count];
        if (2 * q < KP) a[2 * q] = v.x, c[2 * q] = v.y;
        if (2 * q + 1 < KP) a[2 * q + 1] = v.z, c[2 * q + 1] = v.w;
      }
    }
    pmd_pow_uniform<KP>(M, a, c, ex, ebits, tab, gid0, G, slot, topc);
    uint4* so = stp + opaque_i(e);
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      so[(size_t)q * count] = make_uint4(2 * q < KP ? a[2 * q] : 0u, 2 * q < KP ? c[2 * q] : 0u,
                                         2 * q + 1 < KP ? a[2 * q + 1] : 0u, 2 * q + 1 < KP ? c[2 * q + 1] : 0u);
  }
}

template <class MP2, int KP>
__global__ void __launch_bounds__(128, 2) k_dec_pmd_out(KeyDev key, const uint32_t* __restrict__ Pp,
                                                        const uint32_t* __restrict__ Pq,
                                                        const uint32_t* __restrict__ Np2,
                                                        const uint32_t* __restrict__ Nq2, int64_t count,
                                                        const uint4* __restrict__ st, int xs4,
                                                        uint32_t* __restrict__ xrows) {
  constexpr int NQ = PMD<KP>::NQ;
  const int prime = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  const uint4* se = st + (size_t)prime * NQ * count + e;
  uint32_t a[KP], c[KP], x[MP2::L];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const uint4 v = se[(size_t)q * count];
    if (2 * q < KP) a[2 * q] = v.x, c[2 * q] = v.y;
    if (2 * q + 1 < KP) a[2 * q + 1] = v.z, c[2 * q + 1] = v.w;
  }
  {
    PMD<KP> M;
    M.init(prime ? Pq : Pp, prime ? key.q.n0inv : key.p.n0inv);
    M.to_mont2(a, c, x);  // x^(P-1) R^2 mod P^2, unreduced
  }
  // out of Montgomery form: 1 * X R^-2 with X streamed from the lane's LDS
  // slot (as k_djn_pmd's last product)
  __shared__ __attribute__((aligned(16))) uint32_t img_all[2][(MP2::S4 / 4) * 256];
  uint32_t* slot = img_all[(threadIdx.x >> 6) & 1] + (threadIdx.x & 63) * 4;
#pragma unroll
  for (int q = 0; q < MP2::S4 / 4; ++q)
    *reinterpret_cast<uint4*>(slot + q * 256) =
        make_uint4(4 * q < MP2::S ? x[4 * q] : 0u, 4 * q + 1 < MP2::S ? x[4 * q + 1] : 0u,
                   4 * q + 2 < MP2::S ? x[4 * q + 2] : 0u, 4 * q + 3 < MP2::S ? x[4 * q + 3] : 0u);
  wave_sync_mem_();
  __builtin_amdgcn_sched_barrier(0);  // keep the phases apart (interleaved, they spill)
#pragma unroll
  for (int j = 0; j < MP2::L; ++j) x[j] = j == 0 ? 1u : 0u;
  MP2 N;
  N.init(prime ? Nq2 : Np2, prime ? key.q2.n0inv : key.p2.n0inv);
  N.mul(x, ALdsQ{slot});
  N.reduce_once(x);  // c^(P-1) mod P^2, = 1 (mod P)
  // X = x - 1 (x >= 1): a 32-bit borrow chain (the 64-bit add-all-ones form
  // of k_dec_pow spills here)
  uint32_t br = 1u;
  uint32_t* xo = xrows + (size_t)prime * xs4 * count + e;
#pragma unroll
  for (int j = 0; j < MP2::L; ++j) {
    const uint32_t v = x[j] - br;
    br = x[j] < br ? 1u : 0u;
    xo[(size_t)j * count] = v & MP2::MASK;
  }
}

// Private non-DJN encryption, last step: (1 + n m) r^(e_P) mod P^2 from the
// digits of r^(e_P) (k_dec_pmd_pow), as k_djn_pmd finishes: R a + P c is the
// 74-limb Montgomery form, and the product with the plain 1 + n m leaves it.
// Rows as k_crt_enc reads them ([prime][2 S4][count]).
template <class MP2, int KP>
__global__ void __launch_bounds__(128, 2) k_nodjn_pmd_out(KeyDev key, const uint32_t* __restrict__ Pp,
                                                          const uint32_t* __restrict__ Pq,
                                                          const uint32_t* __restrict__ Np2,
                                                          const uint32_t* __restrict__ Nq2,
                                                          const uint32_t* __restrict__ m_words, int64_t count,
                                                          const uint4* __restrict__ st, uint32_t* __restrict__ rows) {
  constexpr int NQ = PMD<KP>::NQ;
  const int prime = blockIdx.y;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  __shared__ __attribute__((aligned(16))) uint32_t img_all[2][(MP2::S4 / 4) * 256];
  uint32_t* slot = img_all[(threadIdx.x >> 6) & 1] + (threadIdx.x & 63) * 4;
  {
    const uint4* se = st + (size_t)prime * NQ * count + e;
    uint32_t a[KP], c[KP], x[2 * KP];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint4 v = se[(size_t)q * count];
      if (2 * q < KP) a[2 * q] = v.x, c[2 * q] = v.y;
      if (2 * q + 1 < KP) a[2 * q + 1] = v.z, c[2 * q + 1] = v.w;
    }
    PMD<KP> M;
    M.init(prime ? Pq : Pp, prime ? key.q.n0inv : key.p.n0inv);
    M.to_mont2(a, c, x);  // r^e R^2 mod P^2, unreduced (< 2^13 P^2)
#pragma unroll
    for (int q = 0; q < MP2::S4 / 4; ++q)
      *reinterpret_cast<uint4*>(slot + q * 256) =
          make_uint4(4 * q < 2 * KP ? x[4 * q] : 0u, 4 * q + 1 < 2 * KP ? x[4 * q + 1] : 0u,
                     4 * q + 2 < 2 * KP ? x[4 * q + 2] : 0u, 4 * q + 3 < 2 * KP ? x[4 * q + 3] : 0u);
  }
  wave_sync_mem_();
  __builtin_amdgcn_sched_barrier(0);
  MP2 N;
  N.init(prime ? Nq2 : Np2, prime ? key.q2.n0inv : key.p2.n0inv);
  uint32_t b[MP2::L];
  N.load_words(b, m_words + (size_t)e * key.nw, key.nw);
  N.mul(b, ARow{prime ? key.nR_q2 : key.nR_p2});  // n m mod P^2 (< 2 P^2), plain
  b[0] += 1u;                                     // 1 + n m
  N.mul(b, ALdsQ{slot});                          // (1 + n m) r^e mod P^2
  N.reduce_once(b);
  N.store_strided(b, rows + (size_t)prime * 2 * MP2::S4 * count + e, (int)count);
}

// Rewrite packed fixed-base table rows X = x R^2 mod P^2 (the 74-limb
// Montgomery form k_tab_combine writes, RW words) as their Montgomery digits
// (e, f) < P, RW/2 words each (pdigit_dev.hpp pmd_from_mont2). One thread per
// row, in place; once per key after the table build.
template <int KP, int RW>
__global__ void __launch_bounds__(256, 2) k_tab_to_pmd(const uint32_t* __restrict__ P, uint32_t n0inv,
                                                       const uint32_t* __restrict__ RmodP, uint32_t* __restrict__ tab,
                                                       int64_t rows, int64_t rs) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  uint32_t* row = tab + (size_t)r * rs;
  uint32_t w[RW];
#pragma unroll
  for (int q = 0; q < RW / 4; ++q) {
    const uint4 v = reinterpret_cast<const uint4*>(row)[q];
    w[4 * q] = v.x, w[4 * q + 1] = v.y, w[4 * q + 2] = v.z, w[4 * q + 3] = v.w;
  }
  uint32_t X[2 * KP];
#pragma unroll
  for (int l = 0; l < 2 * KP; ++l) {
    const int bit = 28 * l, k = bit >> 5, sh = bit & 31;
    const uint32_t lo = word_or0(w, k, RW), hi = word_or0(w, k + 1, RW);
    X[l] = __builtin_amdgcn_alignbit(hi, lo, sh) & ((1u << 28) - 1u);
  }
  PMD<KP> M;
  M.init(P, n0inv);
  uint32_t e[KP], f[KP];
  pmd_from_mont2<KP>(M, X, RmodP, e, f);
  auto word = [&](const uint32_t (&l)[KP], int k) -> uint32_t {
    const int bit = 32 * k, j = bit / 28, sh = bit - 28 * j;
    uint64_t v = (uint64_t)l[j] >> sh;
    if (j + 1 < KP) v |= (uint64_t)l[j + 1] << (28 - sh);
    if (j + 2 < KP) v |= (uint64_t)l[j + 2] << (56 - sh);
    return (uint32_t)v;
  };
#pragma unroll
  for (int q = 0; q < RW / 8; ++q) {
    reinterpret_cast<uint4*>(row)[q] = make_uint4(word(e, 4 * q), word(e, 4 * q + 1), word(e, 4 * q + 2), word(e, 4 * q + 3));
    reinterpret_cast<uint4*>(row)[RW / 8 + q] =
        make_uint4(word(f, 4 * q), word(f, 4 * q + 1), word(f, 4 * q + 2), word(f, 4 * q + 3));
  }
}
#endif

// c = c_q + q^2 ((c_p + 4p^2 - c_q) (q^2)^-1 mod p^2) for element e (utils.py:38-43)
// out == nullptr: the 2S result limbs are left in element e's q row of ws
// (interleaved, limb i at rq[i * count]) for the caller to pack.
template <class MP2>
XHE_DEV void crt_enc_elem(const KeyDev& key, const uint32_t* __restrict__ Np2, int64_t count, int64_t e,
                          uint32_t* __restrict__ ws, uint32_t* __restrict__ out) {
  uint32_t* rp = ws + e;
  uint32_t* rq = ws + (size_t)2 * MP2::S4 * count + e;
  const int st = (int)count;
  MP2 M;
  M.init(Np2, key.p2.n0inv);
  uint32_t b[MP2::L];
  M.load_strided(b, rp, st);
  M.add_sub_rows(b, key.p2x4_lim, rq, st);
  M.mul(b, ARow{key.q2invR_p2});
  M.reduce_once(b);
  M.wide_mul_add_store(b, ARow{key.q2_lim}, rq, st, out ? out + (size_t)e * key.n2w : nullptr, key.n2w);
}

template <class MP2>
__global__ void __launch_bounds__(256, 2) k_crt_enc(KeyDev key, const uint32_t* __restrict__ Np2, int64_t count,
                                                    uint32_t* __restrict__ ws, uint32_t* __restrict__ out) {
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MP2::TPI;
  if (e >= count) return;
  crt_enc_elem<MP2>(key, Np2, count, e, ws, out);
}

// k_crt_enc for one lane per residue, the wide product c_q + q^2 t streamed
// straight into ciphertext words: every limb of the low half is final as
// soon as its row of the operand scan retires, the high half after one
// normalisation, so the limbs are packed into 32-bit words in registers and
// the words go to a per-wave LDS ring (64 words per lane, stride 65); every
// 32 words the ring is stored as whole 128-byte lines of consecutive
// ciphertexts (two per store instruction). Nothing goes back through the
// global workspace (the strided form writes the 2S limbs to ws and reads
// them back to pack them). The word bookkeeping (bits pending, words out) is
// wave-uniform, so its branches are scalar.
template <class MP2, int NW2>
__global__ void __launch_bounds__(256, 2) k_crt_enc_w(KeyDev key, const uint32_t* __restrict__ Np2, int64_t count,
                                                      const uint32_t* __restrict__ ws, uint32_t* __restrict__ out) {
  static_assert(MP2::TPI == 1, "one lane per residue");
  constexpr int S = MP2::S, W = MP2::W, RS = 65;
  static_assert(NW2 % 32 == 0 && 2 * S * W >= 32 * NW2, "ciphertext words");
  __shared__ uint32_t ring_all[4][64 * RS];
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = (int)(threadIdx.x & 63);
  uint32_t* ring = ring_all[(threadIdx.x >> 6) & 3];
  const int64_t e0 = e - lane;
  if (e0 >= count) return;  // whole wave past the end
  const int64_t ec = e < count ? e : count - 1;  // tail lanes recompute the last element, store nothing
  const int st = (int)count;
  const uint32_t* rp = ws + ec;
  const uint32_t* rq = ws + (size_t)2 * MP2::S4 * count + ec;
  MP2 M;
  M.init(Np2, key.p2.n0inv);
  uint32_t b[MP2::L];
  M.load_strided(b, rp, st);
  M.add_sub_rows(b, key.p2x4_lim, rq, st);
  M.mul(b, ARow{key.q2invR_p2});
  M.reduce_once(b);  // t = (c_p - c_q) (q^2)^-1 mod p^2
  uint64_t T[S];
#pragma unroll
  for (int j = 0; j < S; ++j) T[j] = rq[(size_t)j * st];  // + c_q
  uint64_t acc = 0;
  int nb = 0, w = 0;
  auto flush = [&](int base) XHE_INL {
    wave_sync_mem_();
#pragma unroll 4
    for (int r = 0; r < 32; ++r) {
      const int el = 2 * r + (lane >> 5), wd = lane & 31;
      if (e0 + el < count) out[(size_t)(e0 + el) * NW2 + (w - 32) + wd] = ring[el * RS + base + wd];
    }
    wave_sync_mem_();
  };
  auto emit = [&](uint32_t limb) XHE_INL {
    acc |= (uint64_t)limb << nb;
    nb += W;
    if (nb >= 32 && w < NW2) {
      ring[lane * RS + (w & 63)] = (uint32_t)acc;
      acc >>= 32;
      nb -= 32;
      ++w;
      if ((w & 31) == 0) flush((w - 32) & 63);
    }
  };
  for (int i0 = 0; i0 < MP2::S4; i0 += 4) {
    const uint4 a4 = ARow{key.q2_lim}.load4(i0);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (i0 + r < S) {
        const uint32_t ai = comp4(a4, r);
        const uint64_t x0 = mad64(ai, b[0], T[0]);
        mad_shift(T, b, ai);
        T[S - 1] = 0;
        T[0] += x0 >> W;
        emit((uint32_t)x0 & MP2::MASK);
      }
    }
  }
  uint32_t hi[S];
  M.normalize(T, hi);
#pragma unroll
  for (int j = 0; j < S; ++j) emit(hi[j]);
}

// Raw encryption without obfuscation (paillier.py:283): c = 1 + n m  (m < n,
// so the product is already reduced mod n^2). ws: [2*S4][count] rows.
template <class MP2>
__global__ void __launch_bounds__(256, 2) k_raw_enc(KeyDev key, const uint32_t* __restrict__ m_words, int64_t count,
                                                    uint32_t* __restrict__ ws, uint32_t* __restrict__ out) {
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MP2::TPI;
  if (e >= count) return;
  const int st = (int)count;
  uint32_t* row = ws + e;
  MP2 M;
  M.init(key.p2.N, 0);  // only the limb shape is used (no reduction)
  uint32_t b[MP2::L];
  M.load_words(b, m_words + (size_t)e * key.nw, key.nw);
  {
    const int g = MP2::G::g();
#pragma unroll
    for (int j = 0; j < MP2::L; ++j) row[(size_t)(g * MP2::L + j) * st] = (g == 0 && j == 0) ? 1u : 0u;
  }
  wave_sync_mem_();
  M.wide_mul_add_store(b, ARow{key.n_lim}, row, st, out + (size_t)e * key.n2w, key.n2w);
}

// ---------------------------------------------------------------------------
// Decryption (paillier.py:341-368)
// k_dec_pow: X_P = (c^(P-1) mod P^2) - 1 for one prime (grid.y), written to
// xrows [prime][S4][count]. Per-group 4-bit window tables live in wsg
// (17 interleaved rows per group, grid-stride loop over elements).
template <class MP2>
XHE_DEV void pow_uniform_exp(const MP2& M, uint32_t (&b)[MP2::L], const uint32_t* ex, int ebits,
                             uint32_t* tab, uint32_t* sq, int st, uint32_t* sq_lds = nullptr) {
  // 5-bit sliding window over an exponent shared by every lane (p-1 / q-1),
  // so the square/multiply schedule is wave-uniform: odd powers
  // tab[t] = b^(2t+1), t < 16, then ~ebits squarings and ~ebits/6 products
  // (4-bit fixed windows: ebits/4).
  const size_t rs = (size_t)MP2::S4 * st;  // row stride in words
  auto square = [&]() XHE_INL {
    if constexpr (MP2::kSqr) {
      if (sq_lds) {  // the slot carries the square's upper half into the reduction
        M.sqr(b, SqLds<MP2>(sq_lds));
        return;
      }
    }
    if (sq_lds) {
      const SqLds<MP2> L(sq_lds);
      L.put(b);
      M.mul(b, L);
    } else {
      M.store_strided(b, sq, st);
      wave_sync_mem_();
      M.mul(b, AStrided{sq, st});
    }
  };
  auto bit = [&](int i) { return (ex[i >> 5] >> (i & 31)) & 1u; };
  M.store_strided(b, tab, st);  // tab[0] = b
  square();                     // b^2, parked in the sq row
  M.store_strided(b, sq, st);
  wave_sync_mem_();
  M.load_strided(b, tab, st);
#pragma unroll 1
  for (int t = 1; t < 16; ++t) {
    M.mul(b, AStrided{sq, st});  // b^(2t+1) = b^(2t-1) * b^2
    M.store_strided(b, tab + rs * t, st);
  }
  wave_sync_mem_();
  // The window schedule as one loop with one squaring and one product site
  // (each site inlines a whole Montgomery product).
  int i = ebits - 1;
  while (i >= 0 && !bit(i)) --i;
  int pend_sq = 0, pend_mul = -1;
  {  // first window: load its odd power
    int j = i - 4 < 0 ? 0 : i - 4;
    while (!bit(j)) ++j;
    uint32_t val = 0;
    for (int k = i; k >= j; --k) val = (val << 1) | bit(k);
    M.load_strided(b, tab + rs * (val >> 1), st);
    i = j - 1;
  }
#pragma unroll 1
  while (true) {
    if (pend_sq > 0) {
      square();
      --pend_sq;
    } else if (pend_mul >= 0) {
      M.mul(b, AStrided{tab + rs * pend_mul, st});
      pend_mul = -1;
    } else if (i < 0) {
      break;
    } else if (!bit(i)) {
      pend_sq = 1;
      --i;
    } else {
      int j = i - 4 < 0 ? 0 : i - 4;
      while (!bit(j)) ++j;  // window [i..j] ends in a set bit
      uint32_t val = 0;
      for (int k = i; k >= j; --k) val = (val << 1) | bit(k);
      pend_sq = i - j + 1;
      pend_mul = (int)(val >> 1);
      i = j - 1;
    }
  }
}

// SHAPE 0: one lane per residue (key.p2/q2); 1: the 4-lane shape (p2L/q2L);
// 2: the 16-lane shape (p2X/q2X). The wider shapes serve small batches, where
// one lane per residue leaves the chip idle and the ~1,210 dependent products
// of one element set the latency. x rows are written with the one-lane
// shape's row count xs4 (limbs beyond it are zero), so k_dec_fin reads the
// same layout whatever shape produced them.
template <class MP2, int SHAPE = 0>
__global__ void __launch_bounds__(256, 2) k_dec_pow(KeyDev key, const uint32_t* __restrict__ Np2,
                                                    const uint32_t* __restrict__ Nq2,
                                                    const uint32_t* __restrict__ c_words, int64_t count, int xs4,
                                                    uint32_t* __restrict__ xrows, uint32_t* __restrict__ ws) {
  const int prime = blockIdx.y;
  const ModDev& md = SHAPE == 2 ? (prime ? key.q2X : key.p2X)
                     : SHAPE == 1 ? (prime ? key.q2L : key.p2L) : (prime ? key.q2 : key.p2);
  const uint32_t* ex = prime ? key.qm1_words : key.pm1_words;
  const int ebits = prime ? key.qm1_bits : key.pm1_bits;
  const int64_t G_total = (int64_t)gridDim.x * blockDim.x / MP2::TPI;
  const int64_t gid0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MP2::TPI;
  const int st = (int)G_total;
  const size_t rs = (size_t)MP2::S4 * st;
  uint32_t* tab = ws + (size_t)prime * 17 * rs + gid0;  // rows 0..15
  uint32_t* sq = tab + 16 * rs;
  const int n2w = key.n2w;
#if XHE_SQ_LDS
  __shared__ __attribute__((aligned(16))) uint32_t sq_img[4][SqLds<MP2>::WORDS_PER_WAVE];  // 256-thread blocks
  uint32_t* sq_lds = sq_img[(threadIdx.x >> 6) & 3];
#else
  uint32_t* sq_lds = nullptr;
#endif
  for (int64_t e = gid0; e < count; e += G_total) {
    const uint32_t* cw = c_words + (size_t)e * n2w;
    MP2 M;
    M.init(prime ? Nq2 : Np2, md.n0inv);
    uint32_t b[MP2::L];
    // high limbs [S, 2S) of c into the sq row, then REDC(c) * R^3 = c R mod P^2
    {
      const int g = MP2::G::g();
#pragma unroll
      for (int j = 0; j < MP2::L; ++j) {
        int J = MP2::S + g * MP2::L + j;
        int bit = MP2::W * J, k = bit >> 5, sh = bit & 31;
        uint32_t lo = word_or0(cw, k, n2w), h2 = word_or0(cw, k + 1, n2w);
        sq[(size_t)(g * MP2::L + j) * st] = (uint32_t)((((uint64_t)h2 << 32) | lo) >> sh) & MP2::MASK;
      }
      if (g == 0)
        for (int j = MP2::S; j < MP2::S4; ++j) sq[(size_t)j * st] = 0u;
    }
    M.load_words(b, cw, n2w);  // low S limbs
    wave_sync_mem_();
    M.redc_wide(b, AStrided{sq, st});
    M.mul(b, ARow{md.R3});
    pow_uniform_exp(M, b, ex, ebits, tab, sq, st, sq_lds);
    M.mul(b, AOne{});
    M.reduce_once(b);  // x = c^(P-1) mod P^2, x = 1 (mod P)
    // X = x - 1 = x + (2^(W S) - 1) - 2^(W S): add all-ones, drop the top carry
    uint64_t T[MP2::L];
#pragma unroll
    for (int j = 0; j < MP2::L; ++j) T[j] = (uint64_t)b[j] + (uint64_t)MP2::MASK;
    M.normalize(T, b);
    M.store_strided_n(b, xrows + (size_t)prime * xs4 * count + e, (int)count, xs4);
  }
}

// k_dec_fin: m_P = (X_P * P^-1 mod 2^(W*S1)) * hP mod P  (exact division: L_P,
// context.py:190-194), written to mrows [prime][2*S4][count] (MP limbs).
template <class MP2, class MP>
__global__ void __launch_bounds__(256, 2) k_dec_fin(KeyDev key, const uint32_t* __restrict__ Np,
                                                    const uint32_t* __restrict__ Nq, int64_t count,
                                                    const uint32_t* __restrict__ xrows, uint32_t* __restrict__ mrows) {
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MP::TPI;
  if (e >= count) return;
  const int prime = blockIdx.y;
  const ModDev& md = prime ? key.q : key.p;
  const uint32_t* Pinv = prime ? key.qinv_lim : key.pinv_lim;
  const int st = (int)count;
  uint32_t* mrow = mrows + (size_t)prime * 2 * MP::S4 * count + e;
  MP M;
  M.init(prime ? Nq : Np, md.n0inv);
  uint32_t q[MP::L];
  M.load_strided(q, xrows + (size_t)prime * MP2::S4 * count + e, st);  // low S1 limbs of X
  {
    const int g = MP::G::g();
    const bool lead = g == 0;
    uint64_t T[MP::L];
#pragma unroll
    for (int j = 0; j < MP::L; ++j) T[j] = 0;
    for (int i0 = 0; i0 < MP::S4; i0 += 4) {
      uint4 a4 = ARow{Pinv}.load4(i0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (i0 + r < MP::S) {
          uint32_t ai = comp4(a4, r);
          uint64_t x0 = mad64(ai, q[0], T[0]);
          if (lead) mrow[(size_t)(i0 + r) * st] = (uint32_t)x0 & MP::MASK;
          mad_shift(T, q, ai);
          T[MP::L - 1] = MP::G::from_next64(x0);
          T[0] += lead ? (x0 >> MP::W) : 0ull;
        }
      }
    }
  }
  wave_sync_mem_();
  M.load_strided(q, mrow, st);  // L_P(x)
  M.mul(q, ARow{prime ? key.hqR : key.hpR});
  M.reduce_once(q);
  M.store_strided(q, mrow, st);
}

// k_crt_dec: u = (mp + 2p - mq) q^-1 mod p ; m = mq + u q   (utils.py:38-43)
template <class MP>
__global__ void __launch_bounds__(256, 2) k_crt_dec(KeyDev key, const uint32_t* __restrict__ Np, int64_t count,
                                                    uint32_t* __restrict__ mrows, uint32_t* __restrict__ m_out) {
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MP::TPI;
  if (e >= count) return;
  const int st = (int)count;
  uint32_t* rp = mrows + e;
  uint32_t* rq = mrows + (size_t)2 * MP::S4 * count + e;
  MP M;
  M.init(Np, key.p.n0inv);
  uint32_t u[MP::L];
  M.load_strided(u, rp, st);
  M.add_sub_rows(u, key.p2x_lim, rq, st);
  M.mul(u, ARow{key.qinvpR});
  M.reduce_once(u);
  M.wide_mul_add_store(u, ARow{key.q_lim}, rq, st, m_out + (size_t)e * key.nw, key.nw);
}

// ============================================================== mod n^2
// Helpers shared by the n^2 kernels (shape MN2, usually TPI = 4).
#ifndef XHE_STORE_DIRECT
#define XHE_STORE_DIRECT 1  // store_packed straight from the registers (Mont::store_words); 0: via the strided row
#endif
template <class M_>
XHE_DEV void store_packed(const M_& M, const uint32_t (&b)[M_::L], uint32_t* row, int st, uint32_t* out, int nwords) {
#if XHE_STORE_DIRECT
  (void)row;
  (void)st;
  M.store_words(b, out, nwords);
#else
  M.store_strided(b, row, st);
  wave_sync_mem_();
  pack_words_<M_::W, M_::TPI>(row, st, M_::S, out, nwords);
#endif
}

// 4-bit fixed-window power of the Montgomery residue in b. Digits come from
// `digit(w)` (uniform inside a lane group). tab: 16 interleaved rows, sq: one.
template <class M_, class DigitF>
XHE_DEV void pow_window4(const M_& M, uint32_t (&b)[M_::L], const uint32_t* R1, int nwin, DigitF digit,
                         uint32_t* tab, uint32_t* sq, int st, uint32_t* sq_lds = nullptr) {
  const size_t rs = (size_t)M_::S4 * st;
  M.store_strided(b, tab + rs, st);  // tab[1] = b
  {
    uint32_t one[M_::L];
    M.load_row(one, R1);
    M.reduce_once(one);
    M.store_strided(one, tab, st);   // tab[0] = R (Montgomery one)
  }
  wave_sync_mem_();
#pragma unroll 1
  for (int t = 2; t < 16; ++t) {
    M.mul(b, AStrided{tab + rs, st});
    M.store_strided(b, tab + rs * t, st);
  }
  wave_sync_mem_();
  M.load_strided(b, tab + rs * digit(nwin - 1), st);
  for (int w = nwin - 2; w >= 0; --w) {
#pragma unroll 1
    for (int s = 0; s < 4; ++s) {
      if (sq_lds) {
        const SqLds<M_> L(sq_lds);
        L.put(b);
        M.mul(b, L);
      } else {
        M.store_strided(b, sq, st);
        wave_sync_mem_();
        M.mul(b, AStrided{sq, st});
      }
    }
    M.mul(b, AStrided{tab + rs * digit(w), st});
  }
}

XHE_DEV uint32_t nibble(const uint32_t* w, int nwords, int win) {
  int bit = win * 4;
  int k = bit >> 5;
  return (word_or0(w, k, nwords) >> (bit & 31)) & 15u;
}

// out = a * b mod n^2 after aligning exponents: the operand with the larger
// exponent is raised to 2^(e - min(ea, eb)) first (paillier.py:79-86,106-123).
// ws: 2 rows [2*S4][count] per element (second row = pack scratch).
// n^2 constants in the shape of MN2: the 4-lane shape (key.n2) or the
// 16-lane one (key.n2X, small batches).
template <class MN2>
XHE_DEV const ModDev& n2dev(const KeyDev& key) {
  if constexpr (MN2::TPI == 16) return key.n2X;
  else return key.n2;
}

template <class MN2>
__global__ void __launch_bounds__(256, 2) k_mulmod_n2(KeyDev key, const uint32_t* __restrict__ Nn2,
                                                      const uint32_t* __restrict__ a, const int32_t* __restrict__ ea,
                                                      const uint32_t* __restrict__ bw, const int32_t* __restrict__ eb,
                                                      int64_t count, int dmax, uint32_t* __restrict__ out,
                                                      int32_t* __restrict__ eout, uint32_t* __restrict__ ws) {
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MN2::TPI;
  if (e >= count) return;
  const int st = (int)count;
  uint32_t* row = ws + e;
  uint32_t* sq = ws + (size_t)MN2::S4 * count + e;
  MN2 M;
  M.init(Nn2, n2dev<MN2>(key).n0inv);
  const int e1 = ea ? ea[e] : 0, e2 = eb ? eb[e] : 0;
  const int emin = e1 < e2 ? e1 : e2;
  // x = the operand to align (larger exponent; a when equal), y = the other:
  // MontMul(x^(2^d) R, y) = x^(2^d) y, so only x enters Montgomery form and
  // the product leaves it by itself - 2 + d products (was 4 + d: both
  // operands converted, then a product by 1)
  const bool xb = e2 > e1;
  const int dx = (xb ? e2 : e1) - emin;
  const uint32_t* xw = (xb ? bw : a) + (size_t)e * key.n2w;
  const uint32_t* yw = (xb ? a : bw) + (size_t)e * key.n2w;
  uint32_t b[MN2::L];
  // y as plain limbs, parked in `row` (c < n^2, so no reduction is needed)
  M.load_words(b, yw, key.n2w);
  M.store_strided(b, row, st);
  M.load_words(b, xw, key.n2w);
  M.mul(b, ARow{n2dev<MN2>(key).R2});  // x R
  for (int k = 0; k < dmax; ++k) {
    if (k < dx) {
      M.store_strided(b, sq, st);
      wave_sync_mem_();
      M.mul(b, AStrided{sq, st});
    }
  }
  wave_sync_mem_();
  M.mul(b, AStrided{row, st});  // x^(2^d) R * y * R^-1
  M.reduce_once(b);
  store_packed(M, b, row, st, out + (size_t)e * key.n2w, key.n2w);
  if (eout && MN2::G::g() == 0) eout[e] = emin;
}

// Alignment across a gap d >= dneg (1 << d >= min_value_for_negative): the
// reference's _decrease_exponent_to hands _raw_mul the scalar 1 << d, which
// then takes the negative branch and yields c^(2^d - n) instead of c^(2^d)
// (paillier.py:79-86, 173-187). For every element, x = the operand of larger
// exponent when its gap is >= dneg, else 1, and k = n (the caller raises x to
// k and inverts: out *= x^-n). One thread per element; rare path.
__global__ void k_gap_pick(KeyDev key, const uint32_t* __restrict__ a, const int32_t* __restrict__ ea,
                           const uint32_t* __restrict__ b, const int32_t* __restrict__ eb, int64_t count, int dneg,
                           uint32_t* __restrict__ x, uint32_t* __restrict__ k) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  const int64_t d = (int64_t)(ea ? ea[e] : 0) - (int64_t)(eb ? eb[e] : 0);  // NULL: all exponents 0
  const bool big = (d < 0 ? -d : d) >= dneg;
  const uint32_t* src = d > 0 ? a + (size_t)e * key.n2w : b + (size_t)e * key.n2w;
  uint32_t* xo = x + (size_t)e * key.n2w;
  for (int w = 0; w < key.n2w; ++w) xo[w] = big ? src[w] : (w == 0 ? 1u : 0u);
  uint32_t* ko = k + (size_t)e * key.nw;
  for (int w = 0; w < key.nw; ++w) ko[w] = key.n_words[w];
}

// out = c^k mod n^2 with a per-element exponent k (kw words, < 2^kbits).
// Grid-stride; per-group workspace of 17 interleaved rows (4-bit window).
template <class MN2>
__global__ void __launch_bounds__(256, 2) k_powmod_n2(KeyDev key, const uint32_t* __restrict__ Nn2,
                                                      const uint32_t* __restrict__ c, const uint32_t* __restrict__ k,
                                                      int kw, int kbits, int64_t count, uint32_t* __restrict__ out,
                                                      uint32_t* __restrict__ ws) {
  const int64_t G_total = (int64_t)gridDim.x * blockDim.x / MN2::TPI;
  const int64_t gid0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MN2::TPI;
  const int st = (int)G_total;
  const size_t rs = (size_t)MN2::S4 * st;
  uint32_t* tab = ws + gid0;
  uint32_t* sq = tab + 16 * rs;
  const int nwin = kbits <= 0 ? 1 : (kbits + 3) / 4;
#if XHE_SQ_LDS
  __shared__ __attribute__((aligned(16))) uint32_t sq_img[4][SqLds<MN2>::WORDS_PER_WAVE];  // 256-thread blocks
  uint32_t* sq_lds = sq_img[(threadIdx.x >> 6) & 3];
#else
  uint32_t* sq_lds = nullptr;
#endif
  for (int64_t e = gid0; e < count; e += G_total) {
    MN2 M;
    M.init(Nn2, n2dev<MN2>(key).n0inv);
    uint32_t b[MN2::L];
    M.load_words(b, c + (size_t)e * key.n2w, key.n2w);
    M.mul(b, ARow{n2dev<MN2>(key).R2});
    const uint32_t* ke = k + (size_t)e * kw;
    pow_window4(M, b, n2dev<MN2>(key).R1, nwin, [&](int w) { return nibble(ke, kw, w); }, tab, sq, st, sq_lds);
    M.mul(b, AOne{});
    M.reduce_once(b);
    store_packed(M, b, sq, st, out + (size_t)e * key.n2w, key.n2w);
  }
}

// Public-key DJN encryption (paillier.py:210-212,283): (1 + n m) h^a mod n^2
// with the fixed-base table of h mod n^2.
template <class MN2, int RW>
__global__ void __launch_bounds__(256, 2) k_djn_pub(KeyDev key, const uint32_t* __restrict__ Nn2,
                                                    const uint32_t* __restrict__ m_words,
                                                    const uint32_t* __restrict__ a_words, int aw, int64_t count,
                                                    uint32_t* __restrict__ ws, uint32_t* __restrict__ out) {
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MN2::TPI;
  if (e >= count) return;
  MN2 M;
  M.init(Nn2, key.n2.n0inv);
  uint32_t b[MN2::L];
  M.load_words(b, m_words + (size_t)e * key.nw, key.nw);
  M.mul(b, ARow{key.nR2_n2});
  M.add_row(b, key.n2.R1);
  const uint32_t* ae = a_words + (size_t)e * aw;
  for (int w = 0; w < key.nwin; ++w) {
    int64_t row0;
    const uint32_t d = win_digit(key, ae, aw, w, row0);
    M.mul(b, ARowPacked<MN2::W, RW>{key.tab_n2 + (size_t)(row0 + d) * RW});
  }
  M.mul(b, AOne{});
  M.reduce_once(b);
  store_packed(M, b, ws + e, (int)count, out + (size_t)e * key.n2w, key.n2w);
}

#if XHE_NDIG
// Public-key DJN encryption in Montgomery digits of n (2048 bits; the tables
// rewritten as canonical digit pairs by k_tab_to_pmdx at key creation): the
// first window's row is the start state, every further row is unpacked into
// the group's LDS pairs and multiplied in (5 K^2 mads per product instead of
// 2 S^2 on the 152-limb n^2); k_ndig_out folds in (1 + n m). Digit state out:
// st [pair][count].
template <class D, int RW>
__global__ void __launch_bounds__(128, 2) k_djn_pub_nd(KeyDev key, const uint32_t* __restrict__ a_words, int aw,
                                                       int64_t count, uint2* __restrict__ st) {
  constexpr int GPB = 128 / D::TPI, L = D::L;
  __shared__ uint2 ops_all[D::K * GPB];
  __shared__ __attribute__((aligned(16))) uint32_t topc[D::K];
  for (int i = threadIdx.x; i < D::K; i += blockDim.x) topc[i] = key.nd_topc[i];
  __syncthreads();
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / D::TPI;
  if (e >= count) return;
  const int g = D::G::g();
  uint2* ops = ops_all + threadIdx.x / D::TPI;
  const uint32_t* tab = key.tab_n2;
  const uint32_t* ae = a_words + (size_t)e * aw;
  D X;
  X.init(key.nd.N, key.nd.n0inv);
  uint32_t a[L], c[L];
  {
    int64_t row0;
    const uint32_t d = win_digit(key, ae, aw, 0, row0);
    const uint32_t* row = tab + (size_t)(row0 + d) * RW;
    pmdx_load<D, 0>(a, row, RW / 2, g);
    pmdx_load<D, 0>(c, row + RW / 2, RW / 2, g);
  }
  for (int w = 1; w < key.nwin; ++w) {
    int64_t row0;
    const uint32_t d = win_digit(key, ae, aw, w, row0);
    pmdx_stage_row<D>(pmdx_launder(tab) + (size_t)(row0 + d) * RW, RW / 2, ops, GPB);
    wave_sync_mem_();
    X.template run<false>(a, c, OpLds{ops, GPB}, topc);
    wave_sync_mem_();
  }
  ndig_st_store<D>(a, c, st, count, e);
}
#endif

// Non-DJN obfuscation, variable base r with a uniform exponent:
//   public  (paillier.py:228-230): (1 + n m) r^n mod n^2          -> out words
//   private (paillier.py:214-227): (1 + n m) r^e_P mod P^2, P = p/q -> ws rows
//   for k_crt_enc (grid.y = prime).
template <class M_>
XHE_DEV void nodjn_core(const M_& M, uint32_t (&b)[M_::L], const ModDev& md, const uint32_t* nR2,
                        const uint32_t* mw, int nw, const uint32_t* rw, int rwn, const uint32_t* ex, int exw,
                        int ebits, uint32_t* tab, uint32_t* sq, uint32_t* park, int st,
                        uint32_t* sq_lds = nullptr) {
  // c0 R = (1 + n m) R parked first
  M.load_words(b, mw, nw);
  M.mul(b, ARow{nR2});
  M.add_row(b, md.R1);
  M.store_strided(b, park, st);
  // r R, then r^e R
  M.load_words(b, rw, rwn);
  M.mul(b, ARow{md.R2});
  // the exponent (n or e_P) is the same for every lane: wave-uniform 5-bit
  // sliding window (~ebits/6 table products instead of ebits/4)
  pow_uniform_exp(M, b, ex, ebits, tab, sq, st, sq_lds);
  wave_sync_mem_();
  M.mul(b, AStrided{park, st});
  M.mul(b, AOne{});
  M.reduce_once(b);
}

template <class MN2>
__global__ void __launch_bounds__(256, 2) k_nodjn_pub(KeyDev key, const uint32_t* __restrict__ Nn2,
                                                      const uint32_t* __restrict__ m_words,
                                                      const uint32_t* __restrict__ r_words, int rw, int64_t count,
                                                      uint32_t* __restrict__ out, uint32_t* __restrict__ ws) {
  const int64_t G_total = (int64_t)gridDim.x * blockDim.x / MN2::TPI;
  const int64_t gid0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MN2::TPI;
  const int st = (int)G_total;
  const size_t rs = (size_t)MN2::S4 * st;
  uint32_t* tab = ws + gid0;
#if XHE_SQ_LDS
  __shared__ __attribute__((aligned(16))) uint32_t sq_img[4][SqLds<MN2>::WORDS_PER_WAVE];  // 256-thread blocks
  uint32_t* sq_lds = sq_img[(threadIdx.x >> 6) & 3];
#else
  uint32_t* sq_lds = nullptr;
#endif
  for (int64_t e = gid0; e < count; e += G_total) {
    MN2 M;
    M.init(Nn2, key.n2.n0inv);
    uint32_t b[MN2::L];
    nodjn_core(M, b, key.n2, key.nR2_n2, m_words + (size_t)e * key.nw, key.nw, r_words + (size_t)e * rw, rw,
               key.n_words, key.nw, key.n_bits, tab, tab + 16 * rs, tab + 17 * rs, st, sq_lds);
    store_packed(M, b, tab + 16 * rs, st, out + (size_t)e * key.n2w, key.n2w);
  }
}

#if XHE_NDIG
// ---------------------------------------------------------------------------
// Variable-base exponentiations mod n^2 in Montgomery digits (PMDX, 4 lanes
// per element, 2048-bit keys): 4 K^2 mads per squaring and 5 K^2 per product
// at K = 80 instead of 2 S^2 = 46 k at S = 152 (Mont<152, 27, 4>), and half
// as many dependent steps per product. Three kernels, so that each has the
// registers to itself (together they spill): k_ndig_in (plain residue ->
// digits), the exponentiation (k_ndig_pow_n: the exponent n shared by every
// element; k_ndig_pow_k: a per-element exponent), k_ndig_out (digits ->
// plain words, optionally times (1 + n m)). The digit state between them:
// st[pair i][count] uint2. Blocks of 128 threads = 32 element groups.
template <class D>
struct NdigWs {
  static constexpr int GPB = 128 / D::TPI;
  // the exponentiation kernels' per-group-slot table: 16 entries x K pairs
  static constexpr size_t tab_bytes_per_slot() { return (size_t)16 * D::K * 8; }
};

// x (WIDE: n2w ciphertext words, else nwords words of a value < n) -> digits
template <class D, bool WIDE>
__global__ void __launch_bounds__(128, 2) k_ndig_in(KeyDev key, const uint32_t* __restrict__ x, int nwords,
                                                    int64_t count, uint2* __restrict__ st) {
  constexpr int L = D::L;
  __shared__ __attribute__((aligned(16))) uint32_t topc[D::K];
  for (int i = threadIdx.x; i < D::K; i += blockDim.x) topc[i] = key.nd_topc[i];
  __syncthreads();
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / D::TPI;
  if (e >= count) return;
  const int g = D::G::g();
  D X;
  X.init(key.nd.N, key.nd.n0inv);
  uint32_t lo[L], hi[L], a[L], c[L];
  const uint32_t* xe = x + (size_t)e * nwords;
  pmdx_load<D, 0>(lo, xe, nwords, g);
  if constexpr (WIDE) {
    pmdx_load<D, D::K>(hi, xe, nwords, g);
  } else {
#pragma unroll
    for (int j = 0; j < L; ++j) hi[j] = 0;
  }
  pmdx_to_digits(X, lo, hi, key.nd_kn2, key.nd_rmn, key.nd_dw, topc, a, c);
  ndig_st_store<D>(a, c, st, count, e);
}

// st <- st^n (public non-DJN obfuscator r^n, paillier.py:228-230)
template <class D>
__global__ void __launch_bounds__(128, 2) k_ndig_pow_n(KeyDev key, int64_t count, uint2* __restrict__ st,
                                                       uint2* __restrict__ ws) {
  constexpr int GPB = NdigWs<D>::GPB, L = D::L;
  __shared__ uint2 ops_all[D::K * GPB];
  __shared__ __attribute__((aligned(16))) uint32_t topc[D::K];
  for (int i = threadIdx.x; i < D::K; i += blockDim.x) topc[i] = key.nd_topc[i];
  __syncthreads();
  const int gs = (int)gridDim.x * GPB;
  const int gid0 = (int)blockIdx.x * GPB + (int)threadIdx.x / D::TPI;
  uint2* ops = ops_all + threadIdx.x / D::TPI;
  uint2* tab = ws + gid0;
  for (int64_t e = gid0; e < count; e += gs) {
    D X;
    X.init(key.nd.N, key.nd.n0inv);
    uint32_t a[L], c[L];
    ndig_st_load<D>(a, c, st, count, e);
    pmdx_pow_uniform(X, a, c, key.n_words, key.n_bits, tab, gs, ops, GPB, topc);
    ndig_st_store<D>(a, c, st, count, e);
  }
}

// st <- st^k, k per element (kw words, < 2^kbits): _raw_mul's positive
// branch (paillier.py:156-187), 4-bit fixed windows
template <class D>
__global__ void __launch_bounds__(128, 2) k_ndig_pow_k(KeyDev key, const uint32_t* __restrict__ k, int kw, int kbits,
                                                       int64_t count, uint2* __restrict__ st, uint2* __restrict__ ws) {
  constexpr int GPB = NdigWs<D>::GPB, L = D::L;
  __shared__ uint2 ops_all[D::K * GPB];
  __shared__ __attribute__((aligned(16))) uint32_t topc[D::K];
  for (int i = threadIdx.x; i < D::K; i += blockDim.x) topc[i] = key.nd_topc[i];
  __syncthreads();
  const int gs = (int)gridDim.x * GPB;
  const int gid0 = (int)blockIdx.x * GPB + (int)threadIdx.x / D::TPI;
  uint2* ops = ops_all + threadIdx.x / D::TPI;
  uint2* tab = ws + gid0;
  const int nwin = kbits <= 0 ? 1 : (kbits + 3) / 4;
  for (int64_t e = gid0; e < count; e += gs) {
    D X;
    X.init(key.nd.N, key.nd.n0inv);
    uint32_t a[L], c[L];
    ndig_st_load<D>(a, c, st, count, e);
    const uint32_t* ke = k + (size_t)e * kw;
    pmdx_pow_window4(X, a, c, nwin, [&](int w) { return nibble(ke, kw, w); }, key.nd_d1, tab, gs, ops, GPB, topc);
    ndig_st_store<D>(a, c, st, count, e);
  }
}

// digits -> ciphertext words y = y0 + n y1; FOLD: times (1 + n m), m words
// per element (nw): y0 + n ((y1 + y0 m) mod n)   (paillier.py:228-230, 283)
template <class D, bool FOLD>
__global__ void __launch_bounds__(128, 2) k_ndig_out(KeyDev key, const uint2* __restrict__ st,
                                                     const uint32_t* __restrict__ m_words, int64_t count,
                                                     uint32_t* __restrict__ out, uint32_t* __restrict__ ws) {
  constexpr int L = D::L;
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / D::TPI;
  if (e >= count) return;
  const int g = D::G::g();
  D X;
  X.init(key.nd.N, key.nd.n0inv);
  uint32_t y0[L], y1[L];
  {
    uint32_t a[L], c[L];
    ndig_st_load<D>(a, c, st, count, e);
    pmdx_from_digits(X, a, c, y0, y1);
  }
  uint32_t* rows = ws + e;  // 2 x S4 limb rows, stride count
  const int cnt = (int)count;
  if constexpr (FOLD) {
    uint32_t* mrow = rows + (size_t)D::MN::S4 * count;
    uint32_t z[L];
    pmdx_load<D, 0>(z, m_words + (size_t)e * key.nw, key.nw, g);
    X.M.store_strided(z, mrow, cnt);
    wave_sync_mem_();
#pragma unroll
    for (int j = 0; j < L; ++j) z[j] = y0[j];
    X.M.mul(z, AStrided{mrow, cnt});  // y0 m R^-1
    X.M.mul(z, ARow{key.nd.R2});      // y0 m (< 2n)
    uint64_t T[L];
#pragma unroll
    for (int j = 0; j < L; ++j) T[j] = (uint64_t)y1[j] + z[j];
    D::normalize_top(T, y1);
    X.M.reduce_once(y1);
    X.M.reduce_once(y1);
  }
  X.M.store_strided(y0, rows, cnt);
  wave_sync_mem_();
  X.M.wide_mul_add_store(y1, ARow{key.nd.N}, rows, cnt, out + (size_t)e * key.n2w, key.n2w);
}
#endif

// SHAPE 0: the batch shape (key.p2/q2); 1: the 4-lane shape (key.p2L/q2L),
// for key sizes whose batch shape spills in this exponentiation (3072 bits:
// 55 limbs per lane). Rows are written RS4 limbs apart for k_crt_enc.
template <class MP2, int SHAPE = 0, int RS4 = MP2::S4>
__global__ void __launch_bounds__(256, 2) k_nodjn_crt(KeyDev key, const uint32_t* __restrict__ Np2,
                                                      const uint32_t* __restrict__ Nq2,
                                                      const uint32_t* __restrict__ m_words,
                                                      const uint32_t* __restrict__ r_words, int rw, int64_t count,
                                                      uint32_t* __restrict__ rows, uint32_t* __restrict__ ws) {
  const int prime = blockIdx.y;
  const ModDev& md = SHAPE ? (prime ? key.q2L : key.p2L) : (prime ? key.q2 : key.p2);
  const uint32_t* nR2 = SHAPE ? (prime ? key.nR2_q2L : key.nR2_p2L) : (prime ? key.nR2_q2 : key.nR2_p2);
  const int64_t G_total = (int64_t)gridDim.x * blockDim.x / MP2::TPI;
  const int64_t gid0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MP2::TPI;
  const int st = (int)G_total;
  const size_t rs = (size_t)MP2::S4 * st;
  uint32_t* tab = ws + (size_t)prime * 18 * rs + gid0;
#if XHE_SQ_LDS
  __shared__ __attribute__((aligned(16))) uint32_t sq_img[4][SqLds<MP2>::WORDS_PER_WAVE];  // 256-thread blocks
  uint32_t* sq_lds = sq_img[(threadIdx.x >> 6) & 3];
#else
  uint32_t* sq_lds = nullptr;
#endif
  for (int64_t e = gid0; e < count; e += G_total) {
    MP2 M;
    M.init(prime ? Nq2 : Np2, md.n0inv);
    uint32_t b[MP2::L];
    nodjn_core(M, b, md, nR2, m_words + (size_t)e * key.nw, key.nw,
               r_words + (size_t)e * rw, rw, prime ? key.eq_words : key.ep_words, key.nw,
               prime ? key.eq_bits : key.ep_bits, tab, tab + 16 * rs, tab + 17 * rs, st, sq_lds);
    M.store_strided_n(b, rows + (size_t)prime * 2 * RS4 * count + e, (int)count, RS4);
  }
}

// ---- homomorphic sums / histograms (A.9, decision_tree_trainer.py:151-160)
// Each element enters as the plain residue c^(2^d), d = e - e_min of its
// segment (no product when d = 0); the first level of k_chunk_prod chains the
// plain residues and returns each chunk to Montgomery form with one product.
template <class MN2>
__global__ void __launch_bounds__(256, 2) k_align_mont(KeyDev key, const uint32_t* __restrict__ Nn2,
                                                       const uint32_t* __restrict__ c, const int32_t* __restrict__ d,
                                                       int64_t count, int dmax, uint32_t* __restrict__ rows,
                                                       uint32_t* __restrict__ sqws) {
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MN2::TPI;
  if (e >= count) return;
  const int st = (int)count;
  MN2 M;
  M.init(Nn2, n2dev<MN2>(key).n0inv);
  uint32_t b[MN2::L];
  M.load_words(b, c + (size_t)e * key.n2w, key.n2w);
  const int de = (d && dmax) ? d[e] : 0;
  if (de > 0) {  // c^(2^d): into Montgomery form, d squarings, and out again
    M.mul(b, ARow{n2dev<MN2>(key).R2});
    for (int k = 0; k < dmax; ++k) {
      if (k < de) {
        M.store_strided(b, sqws + e, st);
        wave_sync_mem_();
        M.mul(b, AStrided{sqws + e, st});
      }
    }
    M.mul(b, AOne{});
    M.reduce_once(b);
  }
  M.store_strided(b, rows + e, st);
}

// One reduction level: chunk j multiplies `count` rows of a segment, the
// rows first, first + stride, ... (rows [S4][n_in]) into the Montgomery row j
// of out ([S4][n_out]). Chunks are INTERLEAVED over their segment (chunk t of
// nch takes rows t, t + nch, ...): at every step neighbouring lane groups
// read neighbouring columns, one 64-B piece per wave, where contiguous chunks
// of 32 made every group of a wave read its own cache line (20 GB fetched
// per 1 M-row level, `profiles/r4/pmc_ops/`). The product is the same residue
// in any order. plan: (first, stride, count) per chunk; plan == nullptr: every
// segment has seg_len rows and ncs chunks (the mat-vec's uniform segments, no
// upload). raw: the input rows are plain residues and count <= kRawChunk: L
// plain residues chain to P R^-(L-1), and one product by R^(L+1) gives P R -
// one product per element plus one per chunk instead of two per element.
template <class MN2>
__global__ void __launch_bounds__(256, 2) k_chunk_prod(KeyDev key, const uint32_t* __restrict__ Nn2,
                                                       const uint32_t* __restrict__ in, int64_t n_in,
                                                       const int64_t* __restrict__ plan, int64_t seg_len, int64_t ncs,
                                                       int64_t n_out, uint32_t* __restrict__ outp, int raw) {
  const int64_t j = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MN2::TPI;
  if (j >= n_out) return;
  int64_t first, stride, cnt;
  if (plan) {
    first = plan[3 * j];
    stride = plan[3 * j + 1];
    cnt = plan[3 * j + 2];
  } else {
    const int64_t sg = j / ncs, t = j - sg * ncs;
    first = sg * seg_len + t;
    stride = ncs;
    cnt = t < seg_len ? (seg_len - t + ncs - 1) / ncs : 0;
  }
  MN2 M;
  M.init(Nn2, n2dev<MN2>(key).n0inv);
  uint32_t b[MN2::L];
  if (cnt <= 0) {  // empty segment: Montgomery one
    M.load_row(b, n2dev<MN2>(key).R1);
    M.reduce_once(b);
  } else {
    M.load_strided(b, in + first, (int)n_in);
    for (int64_t u = 1; u < cnt; ++u) M.mul(b, AStrided{in + first + u * stride, (int)n_in});
    if (raw) M.mul(b, ARow{n2dev<MN2>(key).Rpow + (size_t)(cnt + 1) * MN2::S4});
    M.reduce_once(b);
  }
  M.store_strided(b, outp + j, (int)n_out);
}

// The first (raw) level straight from the input ciphertexts ([n][PW] words,
// element-major) when no element needs alignment: no k_align_mont pass (a
// 1.2 GB transpose per 1 M elements); the operands are unpacked from their
// words where they are used (ARowPacked), chunks interleaved as above.
template <class MN2, int PW>
__global__ void __launch_bounds__(256, 2) k_chunk_prod_words(KeyDev key, const uint32_t* __restrict__ Nn2,
                                                             const uint32_t* __restrict__ words,
                                                             const int64_t* __restrict__ plan, int64_t seg_len,
                                                             int64_t ncs, int64_t n_out, uint32_t* __restrict__ outp) {
  const int64_t j = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MN2::TPI;
  if (j >= n_out) return;
  int64_t first, stride, cnt;
  if (plan) {
    first = plan[3 * j];
    stride = plan[3 * j + 1];
    cnt = plan[3 * j + 2];
  } else {
    const int64_t sg = j / ncs, t = j - sg * ncs;
    first = sg * seg_len + t;
    stride = ncs;
    cnt = t < seg_len ? (seg_len - t + ncs - 1) / ncs : 0;
  }
  MN2 M;
  M.init(Nn2, n2dev<MN2>(key).n0inv);
  uint32_t b[MN2::L];
  if (cnt <= 0) {
    M.load_row(b, n2dev<MN2>(key).R1);
    M.reduce_once(b);
  } else {
    M.load_words(b, words + (size_t)first * PW, PW);
    for (int64_t u = 1; u < cnt; ++u) M.mul(b, ARowPacked<MN2::W, PW>{words + (size_t)(first + u * stride) * PW});
    M.mul(b, ARow{n2dev<MN2>(key).Rpow + (size_t)(cnt + 1) * MN2::S4});
    M.reduce_once(b);
  }
  M.store_strided(b, outp + j, (int)n_out);
}

// ---- batch modular inversion mod n^2 (Montgomery's trick as a product tree)
// Up-sweep: out[i] = in[2i] * in[2i+1] (Montgomery form, rows [S4][n]).
template <class MN2>
__global__ void __launch_bounds__(256, 2) k_tree_up(KeyDev key, const uint32_t* __restrict__ Nn2,
                                                    const uint32_t* __restrict__ in, int64_t n_in,
                                                    uint32_t* __restrict__ outp, int64_t n_out) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MN2::TPI;
  if (i >= n_out) return;
  MN2 M;
  M.init(Nn2, n2dev<MN2>(key).n0inv);
  uint32_t b[MN2::L];
  M.load_strided(b, in + 2 * i, (int)n_in);
  if (2 * i + 1 < n_in) {
    M.mul(b, AStrided{in + 2 * i + 1, (int)n_in});
    M.reduce_once(b);
  }
  M.store_strided(b, outp + i, (int)n_out);
}

// Down-sweep: inv(child i) = inv(parent i/2) * child(i ^ 1)
template <class MN2>
__global__ void __launch_bounds__(256, 2) k_tree_down(KeyDev key, const uint32_t* __restrict__ Nn2,
                                                      const uint32_t* __restrict__ pinv, int64_t n_par,
                                                      const uint32_t* __restrict__ child, int64_t n_child,
                                                      uint32_t* __restrict__ cinv) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MN2::TPI;
  if (i >= n_child) return;
  MN2 M;
  M.init(Nn2, n2dev<MN2>(key).n0inv);
  uint32_t b[MN2::L];
  M.load_strided(b, pinv + i / 2, (int)n_par);
  const int64_t sib = i ^ 1;
  if (sib < n_child) {
    M.mul(b, AStrided{child + sib, (int)n_child});
    M.reduce_once(b);
  }
  M.store_strided(b, cinv + i, (int)n_child);
}

// n^2 residues (words) -> Montgomery rows [S4][count]; and back.
template <class MN2>
__global__ void __launch_bounds__(256, 2) k_to_mont_rows(KeyDev key, const uint32_t* __restrict__ Nn2,
                                                         const uint32_t* __restrict__ c, int64_t count,
                                                         uint32_t* __restrict__ rows) {
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MN2::TPI;
  if (e >= count) return;
  MN2 M;
  M.init(Nn2, n2dev<MN2>(key).n0inv);
  uint32_t b[MN2::L];
  M.load_words(b, c + (size_t)e * key.n2w, key.n2w);
  M.mul(b, ARow{n2dev<MN2>(key).R2});
  M.reduce_once(b);
  M.store_strided(b, rows + e, (int)count);
}

template <class MN2>
__global__ void __launch_bounds__(256, 2) k_from_mont_rows(KeyDev key, const uint32_t* __restrict__ Nn2,
                                                           uint32_t* __restrict__ rows, int64_t count,
                                                           uint32_t* __restrict__ out) {
  const int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MN2::TPI;
  if (e >= count) return;
  MN2 M;
  M.init(Nn2, n2dev<MN2>(key).n0inv);
  uint32_t b[MN2::L];
  M.load_strided(b, rows + e, (int)count);
  M.mul(b, AOne{});
  M.reduce_once(b);
  store_packed(M, b, rows + e, (int)count, out + (size_t)e * key.n2w, key.n2w);
}

// Root of the product tree <-> plain words for k_inv_single (one group).
template <class MN2>
__global__ void k_row_pack(KeyDev key, const uint32_t* __restrict__ Nn2, uint32_t* __restrict__ row,
                           uint32_t* __restrict__ out) {
  if (blockIdx.x != 0 || threadIdx.x >= MN2::TPI) return;
  pack_words_<MN2::W, MN2::TPI>(row, 1, MN2::S, out, key.n2w);
}
// words y = (P R)^-1 -> Montgomery row of P^-1: y * R^3 * R^-1 = P^-1 R
template <class MN2>
__global__ void k_inv_to_row(KeyDev key, const uint32_t* __restrict__ Nn2, const uint32_t* __restrict__ y,
                             uint32_t* __restrict__ row) {
  if (blockIdx.x != 0 || threadIdx.x >= MN2::TPI) return;
  MN2 M;
  M.init(Nn2, n2dev<MN2>(key).n0inv);
  uint32_t b[MN2::L];
  M.load_words(b, y, key.n2w);
  M.mul(b, ARow{n2dev<MN2>(key).R3});
  M.reduce_once(b);
  M.store_row(b, row);
}

// ---- multi-exponentiation (encrypted mat-vec, np.matmul(enc[B], X[B, D]),
// logistic_regression/trainer.py:166): out[j] = prod_t base[idx[j][t]]^k[j][t].
// Straus-style with per-base window tables shared by every column and a
// parallel product per window:
//   P[j][w] = prod_t tab[idx[j][t]][digit_w(k[j][t])]   (k_mexp_gather + k_chunk_prod)
//   out[j]  = Horner over w: acc = acc^(2^c) * P[j][w]   (k_mexp_horner)
// Tables: tab[b][d] = base_b^d * R mod n^2, d < 2^c, rows of S4 words.
template <class MN2>
__global__ void __launch_bounds__(256, 2) k_mexp_tab(KeyDev key, const uint32_t* __restrict__ Nn2,
                                                     const uint32_t* __restrict__ bases, int64_t nbases, int c,
                                                     uint32_t* __restrict__ tab) {
  const int64_t bi = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MN2::TPI;
  if (bi >= nbases) return;
  MN2 M;
  M.init(Nn2, n2dev<MN2>(key).n0inv);
  uint32_t* t = tab + ((size_t)bi << c) * MN2::S4;
  uint32_t b[MN2::L];
  M.load_row(b, n2dev<MN2>(key).R1);
  M.reduce_once(b);
  M.store_row(b, t);  // base^0 = R
  M.load_words(b, bases + (size_t)bi * key.n2w, key.n2w);
  M.mul(b, ARow{n2dev<MN2>(key).R2});
  M.reduce_once(b);
  M.store_row(b, t + MN2::S4);
  wave_sync_mem_();
  const int rows = 1 << c;
  for (int d = 2; d < rows; ++d) {
    M.mul(b, ARow{t + MN2::S4});
    M.reduce_once(b);
    M.store_row(b, t + (size_t)d * MN2::S4);
  }
}

// The same tables by levels of entries (one launch per level, lvl = 1..c):
// level 1 writes base^0, base^1 and base^2; level l >= 2 writes the entries
// (2^(l-1), 2^l) as tab[2^(l-1)] tab[r] and (l < c) tab[2^l] = tab[2^(l-1)]^2,
// one product per lane group - a chain of c + 1 products per base instead of
// the 2^c - 2 of k_mexp_tab (the mat-vec of a small batch is latency-bound).
template <class MN2>
__global__ void __launch_bounds__(256, 2) k_mexp_tab_lvl(KeyDev key, const uint32_t* __restrict__ Nn2,
                                                         const uint32_t* __restrict__ bases, int64_t nbases, int c,
                                                         int lvl, uint32_t* __restrict__ tab) {
  const int64_t gi = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MN2::TPI;
  MN2 M;
  M.init(Nn2, n2dev<MN2>(key).n0inv);
  uint32_t b[MN2::L];
  if (lvl <= 1) {
    if (gi >= nbases) return;
    uint32_t* t = tab + ((size_t)gi << c) * MN2::S4;
    M.load_row(b, n2dev<MN2>(key).R1);
    M.reduce_once(b);
    M.store_row(b, t);  // base^0 = R
    M.load_words(b, bases + (size_t)gi * key.n2w, key.n2w);
    M.mul(b, ARow{n2dev<MN2>(key).R2});
    M.reduce_once(b);
    M.store_row(b, t + MN2::S4);
    if (c >= 2) {
      wave_sync_mem_();
      M.mul(b, ARow{t + MN2::S4});
      M.reduce_once(b);
      M.store_row(b, t + 2 * MN2::S4);
    }
    return;
  }
  const int64_t h = (int64_t)1 << (lvl - 1);
  const int64_t per = lvl < c ? h : h - 1;  // r = 1..per (r = h: the square)
  const int64_t bi = gi / per, r = gi - bi * per + 1;
  if (bi >= nbases) return;
  uint32_t* t = tab + ((size_t)bi << c) * MN2::S4;
  M.load_row(b, t + h * MN2::S4);
  M.mul(b, ARow{t + r * MN2::S4});
  M.reduce_once(b);
  M.store_row(b, t + (h + r) * MN2::S4);
}

// One lane group per (segment s = j*nwin + w, chunk t): the product of the
// chunk's table rows, stored as a Montgomery row of out [S4][n_out] at
// column s*nchunks + t (the segment order k_chunk_prod reduces).
template <class MN2>
__global__ void __launch_bounds__(256, 2) k_mexp_gather(KeyDev key, const uint32_t* __restrict__ Nn2,
                                                        const uint32_t* __restrict__ tab, int c,
                                                        const int32_t* __restrict__ idx,
                                                        const uint32_t* __restrict__ kx, int kw, int64_t nterms,
                                                        int nwin, int64_t nchunks, int64_t chunk, int64_t n_out,
                                                        uint32_t* __restrict__ out) {
  const int64_t g = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MN2::TPI;
  if (g >= n_out) return;
  const int64_t s = g / nchunks, t = g - s * nchunks;
  const int64_t j = s / nwin;
  const int w = (int)(s - j * nwin);
  const int64_t lo = t * chunk, hi = lo + chunk < nterms ? lo + chunk : nterms;
  MN2 M;
  M.init(Nn2, n2dev<MN2>(key).n0inv);
  uint32_t b[MN2::L];
  const int32_t* ij = idx + j * nterms;
  const uint32_t* kj = kx + (size_t)j * nterms * kw;
  auto row = [&](int64_t i) {
    uint32_t d = digit_at(kj + (size_t)i * kw, kw, w * c, c);
    return tab + (((size_t)ij[i] << c) + d) * MN2::S4;
  };
  M.load_row(b, row(lo));
  for (int64_t i = lo + 1; i < hi; ++i) M.mul(b, ARow{row(i)});
  M.reduce_once(b);
  M.store_strided(b, out + g, (int)n_out);
}

// out[j] = prod_w P[j][w]^(2^(c*w)), P rows [S4][ncols*nwin] (column j*nwin+w);
// sq: one scratch row per column ([S4][ncols]).
template <class MN2>
__global__ void __launch_bounds__(256, 2) k_mexp_horner(KeyDev key, const uint32_t* __restrict__ Nn2,
                                                        const uint32_t* __restrict__ P, int nwin, int c,
                                                        int64_t ncols, uint32_t* __restrict__ sq,
                                                        uint32_t* __restrict__ out) {
  const int64_t j = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MN2::TPI;
  if (j >= ncols) return;
  const int pst = (int)(ncols * nwin);
  const int st = (int)ncols;
  MN2 M;
  M.init(Nn2, n2dev<MN2>(key).n0inv);
  uint32_t b[MN2::L];
  M.load_strided(b, P + j * nwin + (nwin - 1), pst);
  for (int w = nwin - 2; w >= 0; --w) {
    for (int r = 0; r < c; ++r) {
      M.store_strided(b, sq + j, st);
      wave_sync_mem_();
      M.mul(b, AStrided{sq + j, st});
    }
    M.mul(b, AStrided{P + j * nwin + w, pst});
  }
  M.mul(b, AOne{});
  M.reduce_once(b);
  store_packed(M, b, sq + j, st, out + (size_t)j * key.n2w, key.n2w);
}

// ============================================================== tables
// Fixed-base table for h (Montgomery form row `hM`, canonical):
//   tab[w][d] = h^(d * 2^(win*w)) * R mod M, d in [0, 2^win)
// stored packed (RW words per row: K/32 mod p^2, K/16 mod n^2). Every row is a product of a "high"
// and a "low" chain entry (d = hi * 2^half + lo): the chains are built first
// in a limb-form scratch `chain` ([nwin][CH] rows of S4 limbs), then
// k_tab_combine writes every packed row. Chain index of an entry: low d
// (0 <= d <= 2^half) at d, high d (>= 1) at 2^half + d - 1 (high 1 = low 2^half).
XHE_DEV int64_t chain_index(int64_t d, int sh, int half) { return sh == 0 ? d : ((int64_t)1 << half) + d - 1; }
XHE_DEV int64_t chain_rows(int win) { return ((int64_t)1 << (win / 2)) + ((int64_t)1 << (win - win / 2)); }

// k_tab_bases: one group walks the squaring chain, writing low entry 1 of
// every window (h^(2^(win w)) R).
template <class MP2>
__global__ void __launch_bounds__(64, 2) k_tab_bases(ModDev md, const uint32_t* hM, int win, int nwin, uint32_t* chain,
                                                     uint32_t* ws) {
  if (blockIdx.x != 0 || threadIdx.x >= MP2::TPI) return;
  MP2 M;
  M.init(md.N, md.n0inv);
  uint32_t b[MP2::L];
  M.load_row(b, hM);
  const int64_t CH = chain_rows(win);
  for (int w = 0; w < nwin; ++w) {
    M.store_row(b, chain + ((size_t)w * CH + 1) * MP2::S4);
    if (w + 1 == nwin) break;
    for (int s = 0; s < win; ++s) {
      M.store_row(b, ws);
      wave_sync_mem_();
      M.mul(b, ARow{ws});
      M.reduce_once(b);
    }
  }
}

// low entry 0 = R (Montgomery one), one group per window
template <class MP2>
__global__ void __launch_bounds__(256, 2) k_tab_one(ModDev md, int win, int nwin, uint32_t* __restrict__ chain) {
  const int w = (int)(((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MP2::TPI);
  if (w >= nwin) return;
  MP2 M;
  M.init(md.N, md.n0inv);
  uint32_t b[MP2::L];
  M.load_row(b, md.R1);
  M.reduce_once(b);
  M.store_row(b, chain + (size_t)w * chain_rows(win) * MP2::S4);
}

// One doubling level of a chain (sh = 0: low, sh = half: high): entries
// d in [per + 1, 2 per] as entry (d - per) * entry per, d < lim.
template <class MP2>
__global__ void __launch_bounds__(256, 2) k_tab_level(ModDev md, const uint32_t* __restrict__ Nm, int win, int nwin,
                                                       int t, int sh, int lim, uint32_t* __restrict__ chain) {
  const int64_t idx = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MP2::TPI;
  const int64_t per = (int64_t)1 << t;
  if (idx >= (int64_t)nwin * per) return;
  const int w = (int)(idx >> t);
  const int64_t d = per + 1 + (idx & (per - 1));
  if (d >= lim) return;
  const int half = win / 2;
  uint32_t* cw = chain + (size_t)w * chain_rows(win) * MP2::S4;
  MP2 M;
  M.init(Nm, md.n0inv);
  uint32_t b[MP2::L];
  M.load_row(b, cw + (size_t)chain_index(d - per, sh, half) * MP2::S4);
  M.mul(b, ARow{cw + (size_t)chain_index(per, sh, half) * MP2::S4});
  M.reduce_once(b);
  M.store_row(b, cw + (size_t)chain_index(d, sh, half) * MP2::S4);
}

// Every packed row: a chain entry itself (lo == 0 or hi == 0) or the product
// of its high and low entries. The packing goes through a per-group LDS row
// (the group's limbs are spread over TPI lanes).
template <class MP2, int RW>
__global__ void __launch_bounds__(256, 2) k_tab_combine(ModDev md, const uint32_t* __restrict__ Nm, int win,
                                                         int nwin, const uint32_t* __restrict__ chain,
                                                         uint32_t* __restrict__ tab, int64_t rs) {
  __shared__ __attribute__((aligned(16))) uint32_t sc_all[(256 / MP2::TPI) * MP2::S4];
  const int64_t idx = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MP2::TPI;
  const int64_t rows = (int64_t)nwin << win;
  if (idx >= rows) return;
  const int half = win / 2;
  const int w = (int)(idx >> win);
  const int d = (int)(idx & ((1 << win) - 1));
  const int lo = d & ((1 << half) - 1), hi = d >> half;
  const uint32_t* cw = chain + (size_t)w * chain_rows(win) * MP2::S4;
  MP2 M;
  M.init(Nm, md.n0inv);
  uint32_t b[MP2::L];
  if (hi == 0) {
    M.load_row(b, cw + (size_t)chain_index(lo, 0, half) * MP2::S4);
  } else if (lo == 0) {
    M.load_row(b, cw + (size_t)chain_index(hi, half, half) * MP2::S4);
  } else {
    M.load_row(b, cw + (size_t)chain_index(hi, half, half) * MP2::S4);
    M.mul(b, ARow{cw + (size_t)chain_index(lo, 0, half) * MP2::S4});
    M.reduce_once(b);
  }
  uint32_t* sc = sc_all + (size_t)((threadIdx.x % 256) / MP2::TPI) * MP2::S4;
  M.store_row(b, sc);
  wave_sync_mem_();
  pack_words_<MP2::W, MP2::TPI>(sc, 1, MP2::S, tab + (size_t)idx * rs, RW);
}

// Montgomery product of two rows (host-side setup helper / unit tests):
// out = x * y * R^-1 mod M, canonical.
template <class MP2>
__global__ void k_mont_rows(ModDev md, const uint32_t* x, const uint32_t* y, uint32_t* out, int64_t count) {
  int64_t gidx = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / MP2::TPI;
  if (gidx >= count) return;
  MP2 M;
  M.init(md.N, md.n0inv);
  uint32_t b[MP2::L];
  M.load_row(b, x + (size_t)gidx * MP2::S4);
  M.mul(b, ARow{y + (size_t)gidx * MP2::S4});
  M.reduce_once(b);
  M.store_row(b, out + (size_t)gidx * MP2::S4);
}

// ============================================================== decode
// m (nw words) and exponent -> float64 as Paillier.decrypt would hand it to
// astype(np.float32): e < 0: RNE53(v * 2^e) with 2^e a double (0 below
// 2^-1074), subnormals rounded again, overflow to inf (encoder.py:63);
// e >= 0: float(mpz(v << e)) truncated toward zero (gmpy2 2.0.8, measured).
// status: 0 ok, 1 decode OverflowError (max_pos < m < min_neg), 3 mpz too
// large for float (astype OverflowError).
__global__ void k_decode(const uint32_t* __restrict__ m_words, const int32_t* __restrict__ exps, int64_t count,
                         KeyDev key, double* __restrict__ out_f64, float* __restrict__ out_f32,
                         int32_t* __restrict__ status) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int nw = key.nw;
  const uint32_t* m = m_words + (size_t)i * nw;
  int e = exps[i];
  // compare with min_neg / max_pos
  auto cmpw = [&](const uint32_t* a, const uint32_t* b) {
    for (int k = nw - 1; k >= 0; --k) if (a[k] != b[k]) return a[k] < b[k] ? -1 : 1;
    return 0;
  };
  int neg = cmpw(m, key.minneg) >= 0;
  int32_t st = 0;
  if (!neg && cmpw(m, key.maxpos) > 0) st = 1;
  // |v| (neg: n - m) in ONE forward pass over the words, with its borrow
  // chain: the four words ending at the highest nonzero one (w4[3] = word hk)
  // and the OR of every word below them (the rounding's sticky part). (Word
  // by word from the top, each word's borrow needed a scan of the words below
  // it: O(nw^2) loads per element, 0.2 ms for the LR demo's 15 gradients.)
  uint32_t w4[4] = {0u, 0u, 0u, 0u};
  uint32_t low_or = 0u, br = 0u;
  int hk = -1;
  for (int k = 0; k < nw; ++k) {
    uint32_t w;
    if (neg) {
      const uint64_t d = (uint64_t)key.n_words[k] - (uint64_t)m[k] - br;
      w = (uint32_t)d;
      br = (uint32_t)(d >> 63);
    } else {
      w = m[k];
    }
    if (w) {
      const int g = k - hk;  // >= 1: words hk+1 .. k-1 are zero
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (t < g) low_or |= w4[t];  // leaves the window
      uint32_t nw4[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) nw4[t] = t == 3 ? w : (t + g <= 3 ? w4[t + g] : 0u);
#pragma unroll
      for (int t = 0; t < 4; ++t) w4[t] = nw4[t];
      hk = k;
    }
  }
  const int bl = hk < 0 ? 0 : 32 * hk + 32 - __clz(w4[3]);
  auto magw = [&](int k) -> uint32_t {  // word k of |v| for k >= hk - 3
    const int t = 3 - (hk - k);
    return (k > hk || t < 0) ? 0u : w4[t];
  };
  double res;
  if (st != 0) { res = 0.0; }
  else if (bl == 0) {
    res = 0.0;
    if (e < -1074 && neg) res = -0.0;  // never: v == 0 is not negative
  } else {
    // q = RNE53(|v|) as (mant, shift): |v| ~ mant * 2^shift
    uint64_t mant;
    int shift;
    if (bl <= 53) {
      mant = (uint64_t)magw(0) | ((uint64_t)(nw > 1 ? magw(1) : 0) << 32);
      shift = 0;
    } else {
      int s = bl - 53;
      // extract 53 bits starting at bit s, plus round/sticky (all inside the
      // window: s - 1 >= 32 hk - 53)
      auto bitsat = [&](int pos) -> uint64_t {  // 64 bits starting at pos
        int k = pos >> 5, o = pos & 31;
        uint64_t w0 = magw(k), w1 = magw(k + 1), w2 = magw(k + 2);
        uint64_t lo = (w0 | (w1 << 32)) >> o;
        if (o) lo |= w2 << (64 - o);
        return lo;
      };
      mant = bitsat(s) & ((1ull << 53) - 1);
      uint64_t rbit = (bitsat(s - 1) & 1ull);
      bool sticky = low_or != 0;
      for (int k = hk - 3; k < ((s - 1) >> 5); ++k)
        if (k >= 0) sticky |= magw(k) != 0;
      int sb = (s - 1) & 31;
      if (sb) sticky |= (magw((s - 1) >> 5) & ((1u << sb) - 1u)) != 0;
      shift = s;
      if (e >= 0) {
        // gmpy2 mpz->float truncates: keep mant, no rounding
      } else if (rbit && (sticky || (mant & 1))) {
        mant += 1;
        if (mant >> 53) { mant >>= 1; shift += 1; }
      }
    }
    if (e >= 0) {
      int top = bl + e;
      if (top > 1024) { st = 3; res = 0.0; }
      else res = ldexp((double)mant, shift + e);
    } else if (e < -1074) {
      res = 0.0;
    } else {
      int ex2 = shift + e;
      int mb = 64 - __clzll(mant);
      int top = mb + ex2;
      if (top > 1024) res = __longlong_as_double(0x7FF0000000000000ll);
      else if (top <= -1021) {
        int sh2 = -1074 - ex2;  // bits to drop for the subnormal grid
        if (sh2 <= 0) res = ldexp((double)mant, ex2);
        else if (sh2 >= 64) res = 0.0;
        else {
          uint64_t qv = mant >> sh2, rem = mant & ((1ull << sh2) - 1), half = 1ull << (sh2 - 1);
          if (rem > half || (rem == half && (qv & 1))) qv += 1;
          res = ldexp((double)qv, -1074);
        }
      } else res = ldexp((double)mant, ex2);
    }
    if (neg) res = -res;
  }
  if (bl == 0 && e < -1074) res = 0.0;
  if (neg && e < -1074 && st == 0) res = -0.0;
  out_f64[i] = res;
  out_f32[i] = (float)res;
  status[i] = st;
}

}  // namespace xhe
