// Device multi-precision Montgomery arithmetic for gfx950 (CDNA4).
//
// Representation: a residue mod M is S limbs of W bits (W = 27/28) held one
// limb per 32-bit VGPR. A group of TPI consecutive lanes (TPI in {1,2,4,8,16})
// owns one residue, lane g holding limbs [g*L, (g+1)*L), L = S/TPI.
//
// The Montgomery product is operand scanning with LAZY carries: the running
// sum lives in L 64-bit accumulators per lane, every limb product is a single
// v_mad_u64_u32 (32x32+64 -> 64) and no carry is propagated inside the loop.
// With W-bit limbs each accumulator collects at most 2S products of < 2^(2W)
// along its anti-diagonal, so 2S * 2^(2W) < 2^64 is the only constraint
// (static_assert below). The divide-by-2^W shift is folded into the mad
// destinations (T[j-1] = T[j] + a_i*b[j] + m*N[j]) and across lanes it is a
// single DPP move (quad_perm inside 2/4-lane groups, row_shl/row_shr and
// row_newbcast inside a 16-lane DPP row), so the inner loop is 2L mads + O(1)
// per limb of a.
//
// R = 2^(W*S) >= 16*M for every modulus we instantiate, so products of inputs
// below 2M (and up to ~R/M times larger for one operand) stay below 2M and no
// conditional subtraction is needed between products ("almost Montgomery").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace xhe {

#define XHE_DEV __device__ __forceinline__
#define XHE_INL __attribute__((always_inline))  // on lambdas holding Montgomery products: a call would put T[] in scratch

// Build switches (A/B measurement; defaults are the measured-best variant)
#ifndef XHE_NPIPE
#define XHE_NPIPE 1  // TPI==1: modulus limbs loaded one block ahead (Mont::step1)
#endif
#ifndef XHE_MAC_SPLIT
#define XHE_MAC_SPLIT 1  // a*b mads of a block before its m*N mads
#endif
#ifndef XHE_LDS_ROWS
#define XHE_LDS_ROWS 1  // k_djn_pow_lds: table rows staged in LDS by LDS-DMA bursts
#endif
#ifndef XHE_SQ_LDS
#define XHE_SQ_LDS 1  // variable-base exponentiations: squaring operand through LDS (SqLds)
#endif
#ifndef XHE_DJN_FOLD
#define XHE_DJN_FOLD 1  // k_djn_pow_lds: (1 + n m) as the last (plain) multiplier, nwin + 1 products
#endif
#ifndef XHE_SQ_ACC
#define XHE_SQ_ACC 2  // partial sums per column of Mont::sqr's product scan
#endif
#ifndef XHE_PMD
#define XHE_PMD 1  // 2048-bit DJN tables as Montgomery digits, encrypted by k_djn_pmd (pdigit_dev.hpp)
#endif
#ifndef XHE_PMDX
#define XHE_PMDX 1  // 3072/4096-bit DJN tables as Montgomery digits, encrypted by k_djn_pmdx over 4 lanes
#endif
#ifndef XHE_NDIG
#define XHE_NDIG 1  // 2048-bit n^2 exponentiations (public non-DJN r^n, scalar mul c^k) in Montgomery digits mod n^2
#endif
// d = a*b + c with one v_mad_u64_u32. Inline asm keeps a and b 32-bit: the
// C form (uint64_t)a*b + c makes the compiler hold every limb as a
// zero-extended 64-bit register pair, doubling the resident operand.
XHE_DEV uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(c) : "v"(a), "v"(b) : "vcc");
  return c;
}
// T[j-1] = T[j] + a b[j] for j = 1..N-1 (the shift of an operand-scanning
// row), six positions per asm statement: tied accumulators (T[j-1] is
// written after its old value was consumed, no rotation copies), and the
// compiler puts a hazard nop after every asm statement, not inside one
template <int N>
XHE_DEV void mad_shift(uint64_t (&T)[N], const uint32_t (&b)[N], uint32_t a) {
  int j = 1;
#pragma unroll
  for (; j + 6 <= N; j += 6)
    asm("v_mad_u64_u32 %0, vcc, %7, %8, %1\n\t"
        "v_mad_u64_u32 %1, vcc, %7, %9, %2\n\t"
        "v_mad_u64_u32 %2, vcc, %7, %10, %3\n\t"
        "v_mad_u64_u32 %3, vcc, %7, %11, %4\n\t"
        "v_mad_u64_u32 %4, vcc, %7, %12, %5\n\t"
        "v_mad_u64_u32 %5, vcc, %7, %13, %6"
        : "+v"(T[j - 1]), "+v"(T[j]), "+v"(T[j + 1]), "+v"(T[j + 2]), "+v"(T[j + 3]), "+v"(T[j + 4])
        : "v"(T[j + 5]), "v"(a), "v"(b[j]), "v"(b[j + 1]), "v"(b[j + 2]), "v"(b[j + 3]), "v"(b[j + 4]),
          "v"(b[j + 5])
        : "vcc");
#pragma unroll
  for (; j < N; ++j) {
    uint64_t t = T[j];
    asm("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(t) : "v"(a), "v"(b[j]) : "vcc");
    T[j - 1] = t;
  }
}
// same with a wave-uniform b (SGPR operand)
XHE_DEV uint64_t mad64s(uint32_t a, uint32_t b_uniform, uint64_t c) {
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(c) : "v"(a), "s"(b_uniform) : "vcc");
  return c;
}

// w[k] for k < nwords, else 0, with no branch: the load index is clamped
// (nwords >= 1) so every load of an unrolled sequence is in bounds and they
// all issue back to back. The form `k < nwords ? w[k] : 0` with a runtime
// nwords compiled to one branch and one s_waitcnt vmcnt(0) per word: the
// words of a residue were fetched one HBM latency after another (round 5).
XHE_DEV uint32_t word_or0(const uint32_t* __restrict__ w, int k, int nwords) {
  const uint32_t v = w[k < nwords ? k : nwords - 1];
  return k < nwords ? v : 0u;
}

// ------------------------------------------------------------ lane groups
// DPP controls: quad_perm [a,b,c,d] = a | b<<2 | c<<4 | d<<6; row_shl:1 0x101
// (lane i <- lane i+1 of its 16-lane row), row_shr:1 0x111 (lane i <- lane
// i-1), row_newbcast:k 0x150+k (lane k of the row to the whole row, gfx90a+).
template <int TPI>
struct Grp {
  static_assert(TPI == 1 || TPI == 2 || TPI == 4 || TPI == 8 || TPI == 16, "lane groups of 1, 2, 4, 8 or 16");
  static XHE_DEV int g() { return TPI == 1 ? 0 : (int)(threadIdx.x & (TPI - 1)); }
  // 8-lane groups are half rows: a row control reaches both halves, and
  // the upper half (lanes 8-15 of the row) takes the value meant for it
  static XHE_DEV bool upper8() { return (threadIdx.x & 8) != 0; }

  // (mov_dpp with bound_ctrl: a source lane outside the 16-lane row reads 0,
  // and no "old" value has to be materialised first)
  template <int CTRL>
  static XHE_DEV uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
  }
  // value held by lane 0 of the group
  static XHE_DEV uint32_t bcast0(uint32_t v) {
    if constexpr (TPI == 1) return v;
    else if constexpr (TPI == 2) return dpp<0xA0>(v);
    else if constexpr (TPI == 4) return dpp<0x00>(v);
    else if constexpr (TPI == 8) {
      const uint32_t r0 = dpp<0x150>(v), r8 = dpp<0x158>(v);  // row_newbcast:0, :8
      return upper8() ? r8 : r0;
    } else return dpp<0x150>(v);
  }
  // value held by the last lane of the group
  static XHE_DEV uint32_t bcast_last(uint32_t v) {
    if constexpr (TPI == 1) return v;
    else if constexpr (TPI == 2) return dpp<0xF5>(v);
    else if constexpr (TPI == 4) return dpp<0xFF>(v);
    else if constexpr (TPI == 8) {
      const uint32_t r7 = dpp<0x157>(v), r15 = dpp<0x15F>(v);
      return upper8() ? r15 : r7;
    } else return dpp<0x15F>(v);
  }
  // value held by lane g+1 (0 for the last lane)
  static XHE_DEV uint32_t from_next(uint32_t v) {
    if constexpr (TPI == 1) return 0u;
    else if constexpr (TPI == 16) return dpp<0x101>(v);  // lane 15 reads outside the row: 0
    else if constexpr (TPI == 8) {
      const uint32_t r = dpp<0x101>(v);  // row_shl:1; lane 7 of the row reads lane 8
      return g() == 7 ? 0u : r;
    } else {
      uint32_t r = TPI == 2 ? dpp<0xF5>(v) : dpp<0xF9>(v);
      return g() == TPI - 1 ? 0u : r;
    }
  }
  // value held by lane g+1; the last lane's is unspecified (no mask)
  static XHE_DEV uint32_t from_next_any(uint32_t v) {
    if constexpr (TPI == 1) return 0u;
    else if constexpr (TPI == 16 || TPI == 8) return dpp<0x101>(v);
    else return TPI == 2 ? dpp<0xF5>(v) : dpp<0xF9>(v);
  }
  // value held by lane g-1 (0 for lane 0)
  static XHE_DEV uint32_t from_prev(uint32_t v) {
    if constexpr (TPI == 1) return 0u;
    else if constexpr (TPI == 16) return dpp<0x111>(v);  // lane 0 reads outside the row: 0
    else if constexpr (TPI == 8) {
      const uint32_t r = dpp<0x111>(v);  // row_shr:1; lane 8 of the row reads lane 7
      return g() == 0 ? 0u : r;
    } else {
      uint32_t r = TPI == 2 ? dpp<0xA0>(v) : dpp<0x90>(v);
      return g() == 0 ? 0u : r;
    }
  }
  static XHE_DEV uint64_t from_next64(uint64_t v) {
    return (uint64_t)from_next((uint32_t)v) | ((uint64_t)from_next((uint32_t)(v >> 32)) << 32);
  }
  static XHE_DEV uint64_t from_prev64(uint64_t v) {
    return (uint64_t)from_prev((uint32_t)v) | ((uint64_t)from_prev((uint32_t)(v >> 32)) << 32);
  }
};

// ------------------------------------------------------ operand-a sources
// a_i is uniform inside a lane group. load4(i) returns limbs i..i+3 (rows are
// padded to a multiple of 4 words, so i+3 may touch padding).
struct ARow {  // one contiguous row of W-limbs (16-byte aligned)
  const uint32_t* __restrict__ p;
  XHE_DEV uint4 load4(int i) const { return *reinterpret_cast<const uint4*>(p + i); }
};
// Launder a per-lane pointer: the address arithmetic that follows cannot be
// hoisted above this point. Without it LICM precomputes the 64-bit address of
// every limb of an interleaved row (2 VGPRs per limb) outside the loops and
// the Montgomery state spills.
// The zero offset goes through the asm (not the pointer) so the compiler keeps
// the global address space of p (a laundered pointer becomes flat_* accesses).
XHE_DEV const uint32_t* opaque(const uint32_t* p) {
  int zero = 0;
  asm volatile("" : "+s"(zero));
  return p + zero;
}
XHE_DEV uint32_t* opaque(uint32_t* p) {
  int zero = 0;
  asm volatile("" : "+s"(zero));
  return p + zero;
}
XHE_DEV int opaque_i(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

struct AStrided {  // interleaved workspace row: limb i at p[i*stride]
  const uint32_t* p;
  int stride;
  XHE_DEV uint4 load4(int i) const {
    const uint32_t* q = opaque(p) + (size_t)i * stride;
    return make_uint4(q[0], q[stride], q[2 * (size_t)stride], q[3 * (size_t)stride]);
  }
};
struct ALds {  // group row in LDS: limb i at p[i]
  const uint32_t* p;
  XHE_DEV uint4 load4(int i) const { return make_uint4(p[i], p[i + 1], p[i + 2], p[i + 3]); }
};
struct AOne {  // the integer 1 (Montgomery reduction of b)
  XHE_DEV uint4 load4(int i) const { return make_uint4(i == 0 ? 1u : 0u, 0u, 0u, 0u); }
};
struct AZero {
  XHE_DEV uint4 load4(int) const { return make_uint4(0u, 0u, 0u, 0u); }
};

XHE_DEV uint32_t comp4(const uint4& v, int r) { return r == 0 ? v.x : r == 1 ? v.y : r == 2 ? v.z : v.w; }

// Pack `nlimbs` W-bit limbs (one per word, limb i at p[i*stride]) into
// nwords little-endian 32-bit words. Executed by lane `g` of a TPI group for
// words k = g, g+TPI, ...  (limbs beyond nlimbs read as zero).
template <int W, int TPI>
XHE_DEV void pack_words_(const uint32_t* p, int stride, int nlimbs, uint32_t* __restrict__ out, int nwords) {
  const int g = Grp<TPI>::g();
  for (int k = g; k < nwords; k += TPI) {
    int bit = 32 * k;
    int j = bit / W, sh = bit - j * W;
    uint64_t v = 0;
    if (j < nlimbs) v |= (uint64_t)p[(size_t)j * stride];
    if (j + 1 < nlimbs) v |= (uint64_t)p[(size_t)(j + 1) * stride] << W;
    if (j + 2 < nlimbs) v |= (uint64_t)p[(size_t)(j + 2) * stride] << (2 * W);
    out[k] = (uint32_t)(v >> sh);
  }
}

// Workgroup-scope fence: makes this wave's global/LDS writes visible to the
// other lanes of the same wave before they read them.
XHE_DEV void wave_sync_mem_() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

// --------------------------------------------------------------- modulus
template <int S_, int W_, int TPI_>
struct Mont {
  static constexpr int S = S_, W = W_, TPI = TPI_, L = S_ / TPI_;
  static constexpr int S4 = (S_ + 3) & ~3;  // padded row length (words)
  static constexpr uint32_t MASK = (1u << W_) - 1u;
  static_assert(S_ % TPI_ == 0, "S must be a multiple of TPI");
  static_assert(W_ <= 30, "W too large");
  // lazy-carry bound: 2S products of (2^W-1)^2 plus a W-bit carry-in per column
  static_assert((double)(2 * S_ + 2) * (double)(1ull << W_) * (double)(1ull << W_) < 18446744073709551616.0,
                "accumulator would overflow");
  using G = Grp<TPI_>;

  const uint32_t* __restrict__ N;  // S limbs (uniform)
  uint32_t n0inv;                  // -N^-1 mod 2^W
  uint32_t nl[TPI_ == 1 ? 1 : L];  // this lane's modulus limbs (TPI > 1)

  XHE_DEV void init(const uint32_t* Np, uint32_t ninv) {
    N = Np;
    n0inv = ninv;
    if constexpr (TPI > 1) {
      const int g = G::g();
#pragma unroll
      for (int j = 0; j < L; ++j) nl[j] = Np[g * L + j];
    }
  }
  XHE_DEV const uint32_t* np() const { return N; }
  XHE_DEV uint32_t nj(const uint32_t* Np, int j) const {
    if constexpr (TPI == 1) return Np[j];
    else return nl[j];
  }
  // m * N[j] + c
  XHE_DEV uint64_t madN(const uint32_t* Np, uint32_t m, int j, uint64_t c) const {
    if constexpr (TPI == 1) return mad64s(m, Np[j], c);
    else return mad64(m, nl[j], c);
  }

  // T[j-1+k] = T[j+k] + ai*b[j+k] + m*N[j+k], k = 0..3, in place: the block
  // writes T[j-1] first (its old value is already consumed), then T[j] from
  // T[j+1], ... so T[j-1..j+2] are tied in/out operands and each accumulator
  // keeps its register across steps (no rotation copies at the loop edge).
  XHE_DEV void mac4(const uint32_t* Np, uint64_t (&T)[L], const uint32_t (&b)[L], uint32_t ai, uint32_t m,
                    int j) const {
#define XHE_MAC4_ASM                        \
  "v_mad_u64_u32 %0, vcc, %5, %7, %1\n\t"   \
  "v_mad_u64_u32 %0, vcc, %6, %11, %0\n\t"  \
  "v_mad_u64_u32 %1, vcc, %5, %8, %2\n\t"   \
  "v_mad_u64_u32 %1, vcc, %6, %12, %1\n\t"  \
  "v_mad_u64_u32 %2, vcc, %5, %9, %3\n\t"   \
  "v_mad_u64_u32 %2, vcc, %6, %13, %2\n\t"  \
  "v_mad_u64_u32 %3, vcc, %5, %10, %4\n\t"  \
  "v_mad_u64_u32 %3, vcc, %6, %14, %3"
    if constexpr (TPI == 1) {
      asm(XHE_MAC4_ASM
          : "+v"(T[j - 1]), "+v"(T[j]), "+v"(T[j + 1]), "+v"(T[j + 2])
          : "v"(T[j + 3]), "v"(ai), "v"(m), "v"(b[j]), "v"(b[j + 1]), "v"(b[j + 2]), "v"(b[j + 3]),
            "s"(Np[j]), "s"(Np[j + 1]), "s"(Np[j + 2]), "s"(Np[j + 3])
          : "vcc");
    } else {
      asm(XHE_MAC4_ASM
          : "+v"(T[j - 1]), "+v"(T[j]), "+v"(T[j + 1]), "+v"(T[j + 2])
          : "v"(T[j + 3]), "v"(ai), "v"(m), "v"(b[j]), "v"(b[j + 1]), "v"(b[j + 2]), "v"(b[j + 3]),
            "v"(nl[j]), "v"(nl[j + 1]), "v"(nl[j + 2]), "v"(nl[j + 3])
          : "vcc");
    }
#undef XHE_MAC4_ASM
  }
  // 8 limbs (16 mads) per statement: half the statement boundaries (each costs
  // an s_nop the compiler puts after inline asm that writes vcc).
  XHE_DEV void mac8(const uint32_t* Np, uint64_t (&T)[L], const uint32_t (&b)[L], uint32_t ai, uint32_t m,
                    int j) const {
#define XHE_MAC8_ASM                         \
  "v_mad_u64_u32 %0, vcc, %9, %11, %1\n\t"    \
  "v_mad_u64_u32 %0, vcc, %10, %19, %0\n\t"  \
  "v_mad_u64_u32 %1, vcc, %9, %12, %2\n\t"    \
  "v_mad_u64_u32 %1, vcc, %10, %20, %1\n\t"  \
  "v_mad_u64_u32 %2, vcc, %9, %13, %3\n\t"    \
  "v_mad_u64_u32 %2, vcc, %10, %21, %2\n\t"  \
  "v_mad_u64_u32 %3, vcc, %9, %14, %4\n\t"    \
  "v_mad_u64_u32 %3, vcc, %10, %22, %3\n\t"  \
  "v_mad_u64_u32 %4, vcc, %9, %15, %5\n\t"    \
  "v_mad_u64_u32 %4, vcc, %10, %23, %4\n\t"  \
  "v_mad_u64_u32 %5, vcc, %9, %16, %6\n\t"    \
  "v_mad_u64_u32 %5, vcc, %10, %24, %5\n\t"  \
  "v_mad_u64_u32 %6, vcc, %9, %17, %7\n\t"    \
  "v_mad_u64_u32 %6, vcc, %10, %25, %6\n\t"  \
  "v_mad_u64_u32 %7, vcc, %9, %18, %8\n\t"    \
  "v_mad_u64_u32 %7, vcc, %10, %26, %7"
    if constexpr (TPI == 1) {
      asm(XHE_MAC8_ASM
          : "+v"(T[j - 1]), "+v"(T[j]), "+v"(T[j + 1]), "+v"(T[j + 2]), "+v"(T[j + 3]), "+v"(T[j + 4]),
            "+v"(T[j + 5]), "+v"(T[j + 6])
          : "v"(T[j + 7]), "v"(ai), "v"(m), "v"(b[j]), "v"(b[j + 1]), "v"(b[j + 2]), "v"(b[j + 3]),
            "v"(b[j + 4]), "v"(b[j + 5]), "v"(b[j + 6]), "v"(b[j + 7]), "s"(Np[j]), "s"(Np[j + 1]),
            "s"(Np[j + 2]), "s"(Np[j + 3]), "s"(Np[j + 4]), "s"(Np[j + 5]), "s"(Np[j + 6]), "s"(Np[j + 7])
          : "vcc");
    } else {
      asm(XHE_MAC8_ASM
          : "+v"(T[j - 1]), "+v"(T[j]), "+v"(T[j + 1]), "+v"(T[j + 2]), "+v"(T[j + 3]), "+v"(T[j + 4]),
            "+v"(T[j + 5]), "+v"(T[j + 6])
          : "v"(T[j + 7]), "v"(ai), "v"(m), "v"(b[j]), "v"(b[j + 1]), "v"(b[j + 2]), "v"(b[j + 3]),
            "v"(b[j + 4]), "v"(b[j + 5]), "v"(b[j + 6]), "v"(b[j + 7]), "v"(nl[j]), "v"(nl[j + 1]),
            "v"(nl[j + 2]), "v"(nl[j + 3]), "v"(nl[j + 4]), "v"(nl[j + 5]), "v"(nl[j + 6]), "v"(nl[j + 7])
          : "vcc");
    }
#undef XHE_MAC8_ASM
  }

  // ---- TPI == 1 with the modulus limbs in SGPRs loaded one block ahead.
  // Loading N[j..j+7] right before the block that uses it exposes the scalar
  // load latency at every block (an s_waitcnt lgkmcnt(0) per block, five per
  // column); here each block's limbs are requested one block earlier, and the
  // limbs of the first and last blocks of a column stay resident for the
  // whole product.
  static constexpr int J8 = 5 + ((L - 5) / 8) * 8;  // first limb after the 8-limb blocks
  static constexpr int TL = L - J8;                 // tail limbs (0..7)
  struct NRes {
    uint32_t n0, h[4], f[8], t[8];  // N[0], N[1..4], N[5..12], N[J8..L)
  };
  XHE_DEV void load_res(const uint32_t* Np, NRes& r) const {
    r.n0 = Np[0];
#pragma unroll
    for (int k = 0; k < 4; ++k) r.h[k] = Np[1 + k];
#pragma unroll
    for (int k = 0; k < 8; ++k) r.f[k] = Np[5 + k];
#pragma unroll
    for (int k = 0; k < 8; ++k) r.t[k] = k < TL ? Np[J8 + k] : 0u;
  }
#if XHE_MAC_SPLIT
  // all a_i*b products of the block first, then the m*N products: each m*N
  // mad reads an accumulator written 4 (8) instructions earlier instead of
  // by the instruction right before it
#define XHE_MAC4V_ASM                       \
  "v_mad_u64_u32 %0, vcc, %5, %7, %1\n\t"   \
  "v_mad_u64_u32 %1, vcc, %5, %8, %2\n\t"   \
  "v_mad_u64_u32 %2, vcc, %5, %9, %3\n\t"   \
  "v_mad_u64_u32 %3, vcc, %5, %10, %4\n\t"  \
  "v_mad_u64_u32 %0, vcc, %6, %11, %0\n\t"  \
  "v_mad_u64_u32 %1, vcc, %6, %12, %1\n\t"  \
  "v_mad_u64_u32 %2, vcc, %6, %13, %2\n\t"  \
  "v_mad_u64_u32 %3, vcc, %6, %14, %3"
#define XHE_MAC8V_ASM                        \
  "v_mad_u64_u32 %0, vcc, %9, %11, %1\n\t"   \
  "v_mad_u64_u32 %1, vcc, %9, %12, %2\n\t"   \
  "v_mad_u64_u32 %2, vcc, %9, %13, %3\n\t"   \
  "v_mad_u64_u32 %3, vcc, %9, %14, %4\n\t"   \
  "v_mad_u64_u32 %4, vcc, %9, %15, %5\n\t"   \
  "v_mad_u64_u32 %5, vcc, %9, %16, %6\n\t"   \
  "v_mad_u64_u32 %6, vcc, %9, %17, %7\n\t"   \
  "v_mad_u64_u32 %7, vcc, %9, %18, %8\n\t"   \
  "v_mad_u64_u32 %0, vcc, %10, %19, %0\n\t"  \
  "v_mad_u64_u32 %1, vcc, %10, %20, %1\n\t"  \
  "v_mad_u64_u32 %2, vcc, %10, %21, %2\n\t"  \
  "v_mad_u64_u32 %3, vcc, %10, %22, %3\n\t"  \
  "v_mad_u64_u32 %4, vcc, %10, %23, %4\n\t"  \
  "v_mad_u64_u32 %5, vcc, %10, %24, %5\n\t"  \
  "v_mad_u64_u32 %6, vcc, %10, %25, %6\n\t"  \
  "v_mad_u64_u32 %7, vcc, %10, %26, %7"
#else
#define XHE_MAC4V_ASM                       \
  "v_mad_u64_u32 %0, vcc, %5, %7, %1\n\t"   \
  "v_mad_u64_u32 %0, vcc, %6, %11, %0\n\t"  \
  "v_mad_u64_u32 %1, vcc, %5, %8, %2\n\t"   \
  "v_mad_u64_u32 %1, vcc, %6, %12, %1\n\t"  \
  "v_mad_u64_u32 %2, vcc, %5, %9, %3\n\t"   \
  "v_mad_u64_u32 %2, vcc, %6, %13, %2\n\t"  \
  "v_mad_u64_u32 %3, vcc, %5, %10, %4\n\t"  \
  "v_mad_u64_u32 %3, vcc, %6, %14, %3"
#define XHE_MAC8V_ASM                        \
  "v_mad_u64_u32 %0, vcc, %9, %11, %1\n\t"   \
  "v_mad_u64_u32 %0, vcc, %10, %19, %0\n\t"  \
  "v_mad_u64_u32 %1, vcc, %9, %12, %2\n\t"   \
  "v_mad_u64_u32 %1, vcc, %10, %20, %1\n\t"  \
  "v_mad_u64_u32 %2, vcc, %9, %13, %3\n\t"   \
  "v_mad_u64_u32 %2, vcc, %10, %21, %2\n\t"  \
  "v_mad_u64_u32 %3, vcc, %9, %14, %4\n\t"   \
  "v_mad_u64_u32 %3, vcc, %10, %22, %3\n\t"  \
  "v_mad_u64_u32 %4, vcc, %9, %15, %5\n\t"   \
  "v_mad_u64_u32 %4, vcc, %10, %23, %4\n\t"  \
  "v_mad_u64_u32 %5, vcc, %9, %16, %6\n\t"   \
  "v_mad_u64_u32 %5, vcc, %10, %24, %5\n\t"  \
  "v_mad_u64_u32 %6, vcc, %9, %17, %7\n\t"   \
  "v_mad_u64_u32 %6, vcc, %10, %25, %6\n\t"  \
  "v_mad_u64_u32 %7, vcc, %9, %18, %8\n\t"   \
  "v_mad_u64_u32 %7, vcc, %10, %26, %7"
#endif
  XHE_DEV void mac4v(uint64_t (&T)[L], const uint32_t (&b)[L], uint32_t ai, uint32_t m, int j,
                     const uint32_t* n) const {
    asm(XHE_MAC4V_ASM
        : "+v"(T[j - 1]), "+v"(T[j]), "+v"(T[j + 1]), "+v"(T[j + 2])
        : "v"(T[j + 3]), "v"(ai), "v"(m), "v"(b[j]), "v"(b[j + 1]), "v"(b[j + 2]), "v"(b[j + 3]), "s"(n[0]),
          "s"(n[1]), "s"(n[2]), "s"(n[3])
        : "vcc");
  }
  XHE_DEV void mac8v(uint64_t (&T)[L], const uint32_t (&b)[L], uint32_t ai, uint32_t m, int j,
                     const uint32_t* n) const {
    asm(XHE_MAC8V_ASM
        : "+v"(T[j - 1]), "+v"(T[j]), "+v"(T[j + 1]), "+v"(T[j + 2]), "+v"(T[j + 3]), "+v"(T[j + 4]),
          "+v"(T[j + 5]), "+v"(T[j + 6])
        : "v"(T[j + 7]), "v"(ai), "v"(m), "v"(b[j]), "v"(b[j + 1]), "v"(b[j + 2]), "v"(b[j + 3]), "v"(b[j + 4]),
          "v"(b[j + 5]), "v"(b[j + 6]), "v"(b[j + 7]), "s"(n[0]), "s"(n[1]), "s"(n[2]), "s"(n[3]), "s"(n[4]),
          "s"(n[5]), "s"(n[6]), "s"(n[7])
        : "vcc");
  }

  // step() for TPI == 1 (same schedule; N from R and the block pipeline)
  XHE_DEV void step1(const uint32_t* Np, const NRes& R, uint64_t (&T)[L], const uint32_t (&b)[L], uint32_t ai,
                     uint32_t ai_next, uint32_t& m, uint64_t& x0, bool lead) const {
    static_assert(L >= 13, "step1 needs at least one 8-limb block");
    uint64_t xn = 0;
    uint32_t t = 0, mn = 0;
    int stage = 0;
    auto advance = [&]() XHE_INL {
      if (stage == 0) {
        T[0] += lead ? (x0 >> W) : 0ull;
        asm volatile("" : "+v"(T[0]));
      } else if (stage == 1) {
        xn = mad64(ai_next, b[0], T[0]);
        asm volatile("" : "+v"(xn));
      } else if (stage == 2) {
        t = (uint32_t)xn * n0inv;
        asm volatile("" : "+v"(t));
      } else if (stage == 3) {
        mn = t & MASK;
        asm volatile("" : "+v"(mn));
      }
      ++stage;
      __builtin_amdgcn_sched_barrier(0);
    };
    uint32_t nb[2][8];
#pragma unroll
    for (int k = 0; k < 8; ++k) nb[0][k] = R.f[k];
    x0 = mad64s(m, R.n0, x0);
    mac4v(T, b, ai, m, 1, R.h);
    advance();
#pragma unroll
    for (int blk = 0; blk < (J8 - 5) / 8; ++blk) {
      const int j = 5 + 8 * blk;
      const int cur = blk & 1;
      if (j + 16 <= J8) {
        // Scalar loads return out of order, so the only wait is lgkmcnt(0):
        // consume this block's limbs first (the wait lands here, covering
        // only the load issued one block ago), then request the next block's.
        asm volatile("" ::"s"(nb[cur][0]), "s"(nb[cur][1]), "s"(nb[cur][2]), "s"(nb[cur][3]), "s"(nb[cur][4]),
                     "s"(nb[cur][5]), "s"(nb[cur][6]), "s"(nb[cur][7]));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 8; ++k) nb[cur ^ 1][k] = Np[j + 8 + k];
        __builtin_amdgcn_sched_barrier(0);
      }
      mac8v(T, b, ai, m, j, nb[cur]);
      if (stage < 4) advance();
      else __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (TL >= 4) mac4v(T, b, ai, m, J8, R.t);
#pragma unroll
    for (int k = (TL >= 4 ? 4 : 0); k < TL; ++k) T[J8 + k - 1] = mad64s(m, R.t[k], mad64(ai, b[J8 + k], T[J8 + k]));
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (stage < 4) advance();
    T[L - 1] = 0;
    x0 = xn;
    m = mn;
  }

  // ---- squaring (TPI == 1): the square by product scanning, then one
  // Montgomery reduction. Reduction-only blocks: T[j-1+k] = T[j+k] + m*N[j+k].
  XHE_DEV void red4v(uint64_t (&T)[L], uint32_t m, int j, const uint32_t* n) const {
    asm("v_mad_u64_u32 %0, vcc, %5, %6, %1\n\t"
        "v_mad_u64_u32 %1, vcc, %5, %7, %2\n\t"
        "v_mad_u64_u32 %2, vcc, %5, %8, %3\n\t"
        "v_mad_u64_u32 %3, vcc, %5, %9, %4"
        : "+v"(T[j - 1]), "+v"(T[j]), "+v"(T[j + 1]), "+v"(T[j + 2])
        : "v"(T[j + 3]), "v"(m), "s"(n[0]), "s"(n[1]), "s"(n[2]), "s"(n[3])
        : "vcc");
  }
  XHE_DEV void red8v(uint64_t (&T)[L], uint32_t m, int j, const uint32_t* n) const {
    asm("v_mad_u64_u32 %0, vcc, %9, %10, %1\n\t"
        "v_mad_u64_u32 %1, vcc, %9, %11, %2\n\t"
        "v_mad_u64_u32 %2, vcc, %9, %12, %3\n\t"
        "v_mad_u64_u32 %3, vcc, %9, %13, %4\n\t"
        "v_mad_u64_u32 %4, vcc, %9, %14, %5\n\t"
        "v_mad_u64_u32 %5, vcc, %9, %15, %6\n\t"
        "v_mad_u64_u32 %6, vcc, %9, %16, %7\n\t"
        "v_mad_u64_u32 %7, vcc, %9, %17, %8"
        : "+v"(T[j - 1]), "+v"(T[j]), "+v"(T[j + 1]), "+v"(T[j + 2]), "+v"(T[j + 3]), "+v"(T[j + 4]),
          "+v"(T[j + 5]), "+v"(T[j + 6])
        : "v"(T[j + 7]), "v"(m), "s"(n[0]), "s"(n[1]), "s"(n[2]), "s"(n[3]), "s"(n[4]), "s"(n[5]), "s"(n[6]),
          "s"(n[7])
        : "vcc");
  }
  // One reduction row: T <- (T + m*N) / 2^W with limb `hi_i` of the square's
  // upper half entering at the top; the same schedule as step1 (modulus limbs
  // one block ahead, the next row's digit formed under the first blocks).
  XHE_DEV void step1_red(const uint32_t* Np, const NRes& R, uint64_t (&T)[L], uint32_t hi_i, uint32_t& m,
                         uint64_t& x0) const {
    uint64_t xn = 0;
    uint32_t t = 0, mn = 0;
    int stage = 0;
    auto advance = [&]() XHE_INL {
      if (stage == 0) {
        T[0] += x0 >> W;
        asm volatile("" : "+v"(T[0]));
      } else if (stage == 1) {
        xn = T[0];
      } else if (stage == 2) {
        t = (uint32_t)xn * n0inv;
        asm volatile("" : "+v"(t));
      } else if (stage == 3) {
        mn = t & MASK;
        asm volatile("" : "+v"(mn));
      }
      ++stage;
      __builtin_amdgcn_sched_barrier(0);
    };
    uint32_t nb[2][8];
#pragma unroll
    for (int k = 0; k < 8; ++k) nb[0][k] = R.f[k];
    x0 = mad64s(m, R.n0, x0);
    red4v(T, m, 1, R.h);
    advance();
#pragma unroll
    for (int blk = 0; blk < (J8 - 5) / 8; ++blk) {
      const int j = 5 + 8 * blk;
      const int cur = blk & 1;
      if (j + 16 <= J8) {
        asm volatile("" ::"s"(nb[cur][0]), "s"(nb[cur][1]), "s"(nb[cur][2]), "s"(nb[cur][3]), "s"(nb[cur][4]),
                     "s"(nb[cur][5]), "s"(nb[cur][6]), "s"(nb[cur][7]));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 8; ++k) nb[cur ^ 1][k] = Np[j + 8 + k];
        __builtin_amdgcn_sched_barrier(0);
      }
      red8v(T, m, j, nb[cur]);
      if (stage < 4) advance();
      else __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (TL >= 4) red4v(T, m, J8, R.t);
#pragma unroll
    for (int k = (TL >= 4 ? 4 : 0); k < TL; ++k) T[J8 + k - 1] = mad64s(m, R.t[k], T[J8 + k]);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (stage < 4) advance();
    T[L - 1] = hi_i;
    x0 = xn;
    m = mn;
  }
  // Column C of the square into a 64-bit sum: 2 * sum_{i < C-i} a_i a_{C-i}
  // (+ a_{C/2}^2 for even C) + carry; XHE_SQ_ACC partial sums break the mad
  // chain.
  template <int C>
  XHE_DEV uint64_t sq_column(const uint32_t (&a)[L], uint64_t carry) const {
    constexpr int lo = C - (S - 1) > 0 ? C - (S - 1) : 0;
    uint64_t s[XHE_SQ_ACC] = {};
#pragma unroll
    for (int i = lo; 2 * i < C; ++i) s[(i - lo) % XHE_SQ_ACC] = mad64(a[i], a[C - i], s[(i - lo) % XHE_SQ_ACC]);
#pragma unroll
    for (int k = 1; k < XHE_SQ_ACC; ++k) s[0] += s[k];
    uint64_t x = (s[0] << 1) + carry;
    if constexpr ((C & 1) == 0) x = mad64(a[C / 2], a[C / 2], x);
    return x;
  }
  template <int C, class HI>
  XHE_DEV void sq_columns(const uint32_t (&a)[L], uint32_t (&lo)[L], uint64_t carry, uint4& q, const HI& hi) const {
    if constexpr (C < 2 * S) {
      const uint64_t x = C < 2 * S - 1 ? sq_column<C < 2 * S - 1 ? C : 0>(a, carry) : carry;
      const uint32_t limb = (uint32_t)x & MASK;
      if constexpr (C < S) {
        lo[C] = limb;
      } else {
        constexpr int h = C - S;
        if constexpr ((h & 3) == 0) q.x = limb;
        else if constexpr ((h & 3) == 1) q.y = limb;
        else if constexpr ((h & 3) == 2) q.z = limb;
        else q.w = limb;
        if constexpr ((h & 3) == 3 || C == 2 * S - 1) {
          if constexpr ((h & 3) < 3) q.w = 0;
          if constexpr ((h & 3) < 2) q.z = 0;
          if constexpr ((h & 3) < 1) q.y = 0;
          hi.put4(h >> 2, q);
        }
      }
      sq_columns<C + 1, HI>(a, lo, x >> W, q, hi);
    }
  }
  // b <- b^2 R^-1 mod N (TPI == 1 shapes with the SGPR modulus pipeline; others
  // fall back to mul with `a` = a copy of b). The square's S(S+1)/2 column
  // products replace the S^2 a_i*b_k mads of a general product; its upper S
  // limbs go through `hi` (the caller's per-lane LDS slot: put4 / load4) into
  // the reduction. Bounds: a column sum is below (S/2+1) 2^(2W+1) + carry; the
  // reduction adds S terms below 2^(2W) to limbs below 2^W - as in mul().
  static constexpr bool kSqr = TPI == 1 && L >= 13 && XHE_NPIPE;
  template <class HI>
  XHE_DEV void sqr(uint32_t (&b)[L], const HI& hi) const {
    uint32_t lo[L];
    uint4 q = make_uint4(0u, 0u, 0u, 0u);
    sq_columns<0, HI>(b, lo, 0ull, q, hi);
    uint64_t T[L];
#pragma unroll
    for (int j = 0; j < L; ++j) T[j] = lo[j];
    hi.sync();
    const uint32_t* Np = np();
    NRes R;
    load_res(Np, R);
    uint64_t x0 = T[0];
    uint32_t m = ((uint32_t)x0 * n0inv) & MASK;
    uint4 cur = hi.load4(0);
    int i = 0;
    for (; i + 4 <= S; i += 4) {
      uint4 nxt = hi.load4(i + 4 < S4 ? i + 4 : i);
      __builtin_amdgcn_sched_barrier(0);
      step1_red(Np, R, T, cur.x, m, x0);
      __builtin_amdgcn_sched_barrier(0);
      step1_red(Np, R, T, cur.y, m, x0);
      __builtin_amdgcn_sched_barrier(0);
      step1_red(Np, R, T, cur.z, m, x0);
      __builtin_amdgcn_sched_barrier(0);
      step1_red(Np, R, T, cur.w, m, x0);
      __builtin_amdgcn_sched_barrier(0);
      cur = nxt;
    }
#pragma unroll
    for (int r = 0; r < (S & 3); ++r) step1_red(Np, R, T, comp4(cur, r), m, x0);
    normalize(T, b);
  }

  // One column of the product: T <- (T + a_i*b + m*N) / 2^W, software-
  // pipelined: on entry x0 = a_i*b[0] + T[0] and m (its Montgomery digit) are
  // already known; as soon as the first block has produced the new T[0] the
  // next column's x0 and m are formed, so the mul_lo -> and -> broadcast chain
  // overlaps the remaining mads instead of stalling the start of every column.
  XHE_DEV void step(const uint32_t* Np, uint64_t (&T)[L], const uint32_t (&b)[L], uint32_t ai, uint32_t ai_next,
                    uint32_t& m, uint64_t& x0, bool lead) const {
    static_assert(L >= 5, "pipelined step needs L >= 5");
    // The next column's chain (carry into T[0] -> x0' -> x0' * n0inv -> mask +
    // broadcast) is dependent end to end, and a wave issues in order: each
    // link is placed after its own block of independent mads (sched_barrier)
    // so its latency is covered instead of stalling the wave.
    uint64_t xn = 0;
    uint32_t t = 0, mn = 0;
    int stage = 0;
    auto advance = [&]() XHE_INL {
      // (the empty volatile asm pins each link between its barriers; plain
      // arithmetic would otherwise be sunk to its use at IR level)
      if (stage == 0) {
        // every lane keeps the carry of the limb it hands down (position
        // g*L-1 -> g*L is this lane's new T[0]); lane 0's limb is dropped
        T[0] += x0 >> W;
        asm volatile("" : "+v"(T[0]));
      } else if (stage == 1) {
        xn = mad64(ai_next, b[0], T[0]);
        asm volatile("" : "+v"(xn));
      } else if (stage == 2) {
        t = (uint32_t)xn * n0inv;
        asm volatile("" : "+v"(t));
      } else if (stage == 3) {
        mn = G::bcast0(t & MASK);
        asm volatile("" : "+v"(mn));
      }
      ++stage;
      __builtin_amdgcn_sched_barrier(0);
    };
    x0 = madN(Np, m, 0, x0);
    mac4(Np, T, b, ai, m, 1);
    advance();
    int j = 5;
#pragma unroll
    for (; j + 8 <= L; j += 8) {
      mac8(Np, T, b, ai, m, j);
      if (stage < 4) advance();
    }
#pragma unroll
    for (; j + 4 <= L; j += 4) {
      mac4(Np, T, b, ai, m, j);
      if (stage < 4) advance();
    }
#pragma unroll
    for (; j < L; ++j) T[j - 1] = madN(Np, m, j, mad64(ai, b[j], T[j]));
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (stage < 4) advance();
    T[L - 1] = (uint64_t)G::from_next((uint32_t)x0 & MASK);  // its carry stayed in lane g+1
    x0 = xn;
    m = mn;
  }

  // Carry-normalise the accumulators into W-bit limbs.
  XHE_DEV void normalize(const uint64_t (&T)[L], uint32_t (&b)[L]) const {
    // sched_barrier per limb keeps the scheduler from hoisting every 64-bit
    // partial sum ahead of its mask (which doubles the live registers).
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      uint64_t x = T[j] + c;
      b[j] = (uint32_t)x & MASK;
      c = x >> W;
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (TPI >= 4) {
      // One round of lane-to-lane carries (c < 2^36 into L >= 5 limbs), after
      // which every lane's carry-out is 0 or 1 and passes through a lane only
      // when all its limbs are MASK: the remaining ripple is a carry-lookahead
      // on the wave's lane masks (generate g, propagate p; carries into the
      // lanes = (g + (g|p)) ^ g ^ (g|p)), with the group's top lane cleared so
      // no carry crosses into the next group. TPI-1 ripple rounds -> 2 passes.
      uint64_t cin = G::from_prev64(c);
      uint32_t all = 1u;
#pragma unroll
      for (int j = 0; j < L; ++j) {
        uint64_t x = (uint64_t)b[j] + cin;
        b[j] = (uint32_t)x & MASK;
        cin = x >> W;
        all &= (b[j] == MASK) ? 1u : 0u;
        __builtin_amdgcn_sched_barrier(0);
      }
      constexpr uint64_t top = TPI == 16 ? 0x8000800080008000ull : TPI == 8 ? 0x8080808080808080ull
                                                                            : 0x8888888888888888ull;
      const uint64_t gm = __builtin_amdgcn_ballot_w64(cin != 0) & ~top;
      const uint64_t tm = (gm | __builtin_amdgcn_ballot_w64(all != 0)) & ~top;
      const uint64_t cm = (gm + tm) ^ gm ^ tm;
      uint32_t ci = (uint32_t)(cm >> (threadIdx.x & 63)) & 1u;
#pragma unroll
      for (int j = 0; j < L; ++j) {
        uint32_t x = b[j] + ci;
        b[j] = x & MASK;
        ci = x >> W;
      }
    } else if constexpr (TPI > 1) {
#pragma unroll
      for (int r = 1; r < TPI; ++r) {
        uint64_t cin = G::from_prev64(c);
#pragma unroll
        for (int j = 0; j < L; ++j) {
          uint64_t x = (uint64_t)b[j] + cin;
          b[j] = (uint32_t)x & MASK;
          cin = x >> W;
          __builtin_amdgcn_sched_barrier(0);
        }
        c = cin;
      }
    }
  }

  // b <- a * b * R^-1 mod N  (result < 2N for inputs in range)
  template <class A>
  XHE_DEV void mul(uint32_t (&b)[L], const A& a) const {
    uint64_t T[L];
#pragma unroll
    for (int j = 0; j < L; ++j) T[j] = 0;
    run<A>(T, b, a);
    normalize(T, b);
  }

  template <class A>
  XHE_DEV void run(uint64_t (&T)[L], const uint32_t (&b)[L], const A& a) const {
    const bool lead = G::g() == 0;
    const uint32_t* Np = np();
    uint4 cur = a.load4(0);
    uint64_t x0 = mad64(cur.x, b[0], T[0]);
    uint32_t m = G::bcast0(((uint32_t)x0 * n0inv) & MASK);
    int i = 0;
#if XHE_NPIPE
    if constexpr (TPI == 1 && L >= 13) {
      NRes R;
      load_res(Np, R);
      for (; i + 4 <= S; i += 4) {
        uint4 nxt = a.load4(i + 4 < S4 ? i + 4 : i);
        __builtin_amdgcn_sched_barrier(0);
        step1(Np, R, T, b, cur.x, cur.y, m, x0, lead);
        __builtin_amdgcn_sched_barrier(0);
        step1(Np, R, T, b, cur.y, cur.z, m, x0, lead);
        __builtin_amdgcn_sched_barrier(0);
        step1(Np, R, T, b, cur.z, cur.w, m, x0, lead);
        __builtin_amdgcn_sched_barrier(0);
        step1(Np, R, T, b, cur.w, nxt.x, m, x0, lead);
        __builtin_amdgcn_sched_barrier(0);
        cur = nxt;
      }
#pragma unroll
      for (int r = 0; r < (S & 3); ++r)
        step1(Np, R, T, b, comp4(cur, r), r + 1 < (S & 3) ? comp4(cur, r + 1) : 0u, m, x0, lead);
      return;
    }
#endif
    for (; i + 4 <= S; i += 4) {
      uint4 nxt = a.load4(i + 4 < S4 ? i + 4 : i);
      __builtin_amdgcn_sched_barrier(0);
      step(Np, T, b, cur.x, cur.y, m, x0, lead);
      __builtin_amdgcn_sched_barrier(0);
      step(Np, T, b, cur.y, cur.z, m, x0, lead);
      __builtin_amdgcn_sched_barrier(0);
      step(Np, T, b, cur.z, cur.w, m, x0, lead);
      __builtin_amdgcn_sched_barrier(0);
      step(Np, T, b, cur.w, nxt.x, m, x0, lead);
      __builtin_amdgcn_sched_barrier(0);
      cur = nxt;
    }
#pragma unroll
    for (int r = 0; r < (S & 3); ++r)
      step(Np, T, b, comp4(cur, r), r + 1 < (S & 3) ? comp4(cur, r + 1) : 0u, m, x0, lead);
  }

  // Montgomery reduction of a double-length value: lo = limbs [0,S) in b,
  // hi limbs [S, 2S) supplied by `hi` (uniform a-source). Returns
  // (hi*2^(WS) + lo) * R^-1 mod N in b (< 2N when the input < R*N).
  template <class A>
  XHE_DEV void redc_wide(uint32_t (&b)[L], const A& hi) const {
    uint64_t T[L];
#pragma unroll
    for (int j = 0; j < L; ++j) T[j] = b[j];
    const bool lead = G::g() == 0;
    const bool last = G::g() == TPI - 1;
    const uint32_t* Np = np();
    for (int i0 = 0; i0 < S4; i0 += 4) {
      uint4 h4 = hi.load4(i0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (i0 + r < S) {
          uint64_t x0 = T[0];
          uint32_t m = ((uint32_t)x0 * n0inv) & MASK;
          m = G::bcast0(m);
          x0 = madN(Np, m, 0, x0);
#pragma unroll
          for (int j = 1; j < L; ++j) T[j - 1] = madN(Np, m, j, T[j]);
          uint64_t up = G::from_next64(x0);
          T[L - 1] = last ? (uint64_t)comp4(h4, r) : up;
          T[0] += lead ? (x0 >> W) : 0ull;
        }
      }
    }
    normalize(T, b);
  }

  // b in [0, 2N) -> [0, N)
  XHE_DEV void reduce_once(uint32_t (&b)[L]) const {
    uint32_t d[L];
    uint32_t br = 0;
    const uint32_t* Np = np();
#pragma unroll
    for (int j = 0; j < L; ++j) {
      int64_t x = (int64_t)b[j] - (int64_t)nj(Np, j) - (int64_t)br;
      br = x < 0 ? 1u : 0u;
      d[j] = (uint32_t)(x + ((int64_t)br << W));
    }
    if constexpr (TPI > 1) {
      // each round moves borrows one lane up; the top lane's total borrow is
      // its local borrow plus every borrow it generates while absorbing them
      uint32_t total = br;
#pragma unroll
      for (int r = 1; r < TPI; ++r) {
        uint32_t bin = G::from_prev(br);
#pragma unroll
        for (int j = 0; j < L; ++j) {
          int64_t x = (int64_t)d[j] - (int64_t)bin;
          bin = x < 0 ? 1u : 0u;
          d[j] = (uint32_t)(x + ((int64_t)bin << W));
        }
        br = bin;
        total |= bin;
      }
      br = G::bcast_last(total);
    }
    if (!br) {
#pragma unroll
      for (int j = 0; j < L; ++j) b[j] = d[j];
    }
  }

  // b <- b + addend - subtrahend (all as W-limb values, result must be >= 0)
  // addend limbs from a group row (ARow-like pointer), subtrahend from `sub`.
  XHE_DEV void add_sub_rows(uint32_t (&b)[L], const uint32_t* add, const uint32_t* subp, int sub_stride) const {
    const int g = G::g();
    int64_t c = 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      int64_t x = (int64_t)b[j] + (int64_t)add[g * L + j] - (int64_t)subp[(size_t)(g * L + j) * sub_stride] + c;
      c = x >> W;  // arithmetic shift: floor division
      b[j] = (uint32_t)(x & MASK);
    }
    if constexpr (TPI > 1) {
#pragma unroll
      for (int r = 1; r < TPI; ++r) {
        int64_t cin = (int64_t)G::from_prev64((uint64_t)c);
#pragma unroll
        for (int j = 0; j < L; ++j) {
          int64_t x = (int64_t)b[j] + cin;
          cin = x >> W;
          b[j] = (uint32_t)(x & MASK);
        }
        c = cin;
      }
    }
  }

  // b <- b + row (W-limb row, uniform pointer); carries normalised
  XHE_DEV void add_row(uint32_t (&b)[L], const uint32_t* row) const {
    const int g = G::g();
    uint64_t T[L];
#pragma unroll
    for (int j = 0; j < L; ++j) T[j] = (uint64_t)b[j] + row[g * L + j];
    normalize(T, b);
  }

  // Wide product with addend: out = init + b * a, where a is a uniform row of
  // S limbs, init an interleaved row of S limbs at ws (stride). The 2S result
  // limbs are written to the same interleaved row (ws must hold 2*S4 limbs),
  // then packed into nwords little-endian words at `out`.
  template <class A>
  XHE_DEV void wide_mul_add_store(const uint32_t (&b)[L], const A& a, uint32_t* ws, int stride,
                                  uint32_t* __restrict__ out, int nwords) const {
    const int g = G::g();
    const bool lead = g == 0;
    uint64_t T[L];
#pragma unroll
    for (int j = 0; j < L; ++j) T[j] = ws[(size_t)(g * L + j) * stride];
    wave_sync_mem_();
    for (int i0 = 0; i0 < S4; i0 += 4) {
      uint4 a4 = a.load4(i0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (i0 + r < S) {
          uint32_t ai = comp4(a4, r);
          uint64_t x0 = mad64(ai, b[0], T[0]);
          if (lead) ws[(size_t)(i0 + r) * stride] = (uint32_t)x0 & MASK;
          mad_shift(T, b, ai);
          T[L - 1] = G::from_next64(x0);
          T[0] += lead ? (x0 >> W) : 0ull;
        }
      }
    }
    uint32_t hi[L];
    normalize(T, hi);
#pragma unroll
    for (int j = 0; j < L; ++j) ws[(size_t)(S + g * L + j) * stride] = hi[j];
    wave_sync_mem_();
    if (out) pack_words_<W, TPI>(ws, stride, 2 * S, out, nwords);
  }

  // ---------------------------------------------------------------- I/O
  // Load W-limbs from a little-endian 32-bit word array of nwords words.
  // Limbs of a packed little-endian word array (zero beyond nwords). The lane
  // index is dispatched to compile-time copies so every word is loaded once
  // and every shift is an immediate (a runtime lane offset made the compiler
  // keep 2 loads + a 64-bit address per limb live and spill).
  template <int GG>
  XHE_DEV void load_words_g(uint32_t (&b)[L], const uint32_t* __restrict__ w, int nwords) const {
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const int bit = W * (GG * L + j);
      const int k = bit >> 5, sh = bit & 31;
      const uint32_t lo = word_or0(w, k, nwords);
      const uint32_t hi = sh + W > 32 ? word_or0(w, k + 1, nwords) : 0u;
      b[j] = (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) & MASK;
    }
  }
  template <int GG>
  XHE_DEV void load_words_from(uint32_t (&b)[L], const uint32_t* __restrict__ w, int nwords, int g) const {
    if constexpr (GG == TPI - 1) {
      load_words_g<GG>(b, w, nwords);
    } else {
      if (g == GG) load_words_g<GG>(b, w, nwords);
      else load_words_from<GG + 1>(b, w, nwords, g);
    }
  }
  XHE_DEV void load_words(uint32_t (&b)[L], const uint32_t* __restrict__ w, int nwords) const {
    load_words_from<0>(b, w, nwords, G::g());
  }
  // Store limbs [0, nlimbs) of the residue into an interleaved row (the
  // residue's limbs beyond nlimbs must be zero).
  XHE_DEV void store_strided_n(const uint32_t (&b)[L], uint32_t* p, int stride, int nlimbs) const {
    p = opaque(p);
    const int g = G::g();
#pragma unroll
    for (int j = 0; j < L; ++j)
      if (g * L + j < nlimbs) p[(size_t)(g * L + j) * stride] = b[j];
  }
  // b (normalised limbs) packed to nwords little-endian 32-bit words straight
  // from the registers: lane g writes the words that START in its limbs, the
  // next lane's first two limbs (DPP) complete the last of them - the same
  // words as store_strided + pack_words_, without the round trip through a
  // strided row (a write and a read of S4 words per element).
  // The code is the same for every lane: the lane's bits (and the next
  // lane's first two limbs) packed into local words u[] at compile-time
  // positions, then one funnel shift by the lane's runtime bit offset per
  // output word and a predicated store. (A first form branched per lane
  // position with compile-time offsets; the compiler merged the branches'
  // last stores into a shared tail and put one operand copy on the wrong
  // lane's path - wrong top words of the 3072-bit mod-p^2 outputs, DESIGN.md
  // round 4.)
  XHE_DEV void store_words(const uint32_t (&b)[L], uint32_t* __restrict__ out, int nwords) const {
    constexpr int LB = L * W;                // bits per lane
    constexpr int NWM = (LB + 31) / 32 + 1;  // bound on the words starting in one lane
    const uint32_t n0 = G::from_next(b[0]);
    const uint32_t n1 = G::from_next(L > 1 ? b[1] : 0u);
    auto limb = [&](int x) -> uint64_t {
      return x < L ? (uint64_t)b[x] : x == L ? (uint64_t)n0 : x == L + 1 ? (uint64_t)n1 : 0ull;
    };
    uint32_t u[NWM + 1];
#pragma unroll
    for (int i = 0; i <= NWM; ++i) {
      const int bit = 32 * i, jl = bit / W, sh = bit - jl * W;
      const uint64_t v = limb(jl) | (limb(jl + 1) << W) | (limb(jl + 2) << (2 * W));
      u[i] = (uint32_t)(v >> sh);
    }
    const int b0 = G::g() * LB, ks = (b0 + 31) >> 5;
    const int off = (ks << 5) - b0;  // [0, 32): local bit of the lane's first word
    const int ke = (b0 + LB + 31) >> 5, kend = ke < nwords ? ke : nwords;
    uint32_t* o = out + ks;
#pragma unroll
    for (int i = 0; i < NWM; ++i) {
      const uint32_t w = (uint32_t)((((uint64_t)u[i + 1] << 32) | u[i]) >> off);
      if (ks + i < kend) o[i] = w;
    }
  }
  // Store this lane's limbs one per word into an interleaved row.
  XHE_DEV void store_strided(const uint32_t (&b)[L], uint32_t* p, int stride) const {
    p = opaque(p);
    const int g = G::g();
#pragma unroll
    for (int j = 0; j < L; ++j) p[(size_t)(g * L + j) * stride] = b[j];
  }
  XHE_DEV void load_strided(uint32_t (&b)[L], const uint32_t* p, int stride) const {
    p = opaque(p);
    const int g = G::g();
#pragma unroll
    for (int j = 0; j < L; ++j) b[j] = p[(size_t)(g * L + j) * stride];
  }
  XHE_DEV void load_row(uint32_t (&b)[L], const uint32_t* p) const {
    const int g = G::g();
#pragma unroll
    for (int j = 0; j < L; ++j) b[j] = p[g * L + j];
  }
  XHE_DEV void store_row(const uint32_t (&b)[L], uint32_t* p) const {
    const int g = G::g();
#pragma unroll
    for (int j = 0; j < L; ++j) p[g * L + j] = b[j];
  }
};

}  // namespace xhe
