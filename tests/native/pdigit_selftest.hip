// Device self-test and timing of the Montgomery-digit arithmetic mod P^2
// (xfl_amd/csrc/pdigit_dev.hpp PMD): run on the GPU box by
// tests/test_gpu_native_selftests.py.
//
// 1. "mul": chains of PMD<37>::mul on random states and random table rows
//    (packed words staged in LDS and unpacked by unpack_pairs_lds, as the
//    kernel does), each product checked against host big integers:
//    R a' + P c' = (R a + P c)(R e + P f) R^-2 (mod P^2), a' < 2P, c' < R + 8P.
// 2. "to_mont2": R a + P c as 74 limbs.  3. "from_mont2": a reduced residue
//    X < P^2 into digits (e, f) < P with R e + P f = X (mod P^2).
// 4. Throughput: ITER dependent products per lane on the whole chip (2 waves
//    per SIMD), PMD<37>::mul against Mont<74, 28, 1>::mul, hipEvent-timed.
// Prints JSON lines; exits 1 on any mismatch.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <random>
#include <vector>

#include "../../xfl_amd/csrc/bn_dev.hpp"
#include "../../xfl_amd/csrc/hostbn.hpp"
#include "../../xfl_amd/csrc/pdigit_dev.hpp"

using namespace xhe;
constexpr int K = 37, RW = 64;
using PM = PMD<K>;
constexpr int NQ = PM::NQ;
using MP = Mont<74, 28, 1>;

// mode 0: state <- state (x) row; 1: out = to_mont2(state); 2: out = from_mont2(state as 74 limbs)
__global__ void __launch_bounds__(128, 2) k_check(const uint32_t* P, uint32_t n0inv, const uint32_t* topc_g,
                                                  const uint32_t* RmodP, const uint32_t* rows, uint32_t* state,
                                                  uint32_t* out, int count, int mode) {
  __shared__ __attribute__((aligned(16))) uint32_t img_all[2][NQ * 256];
  __shared__ __attribute__((aligned(16))) uint32_t topc[40];
  if (threadIdx.x < 40) topc[threadIdx.x] = threadIdx.x < K ? topc_g[threadIdx.x] : 0u;
  __syncthreads();
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  uint32_t* slot = img_all[(threadIdx.x >> 6) & 1] + (threadIdx.x & 63) * 4;
  PM M;
  M.init(P, n0inv);
  if (mode == 0) {
#pragma unroll
    for (int q = 0; q < RW / 4; ++q)
      *reinterpret_cast<uint4*>(slot + q * 256) = *reinterpret_cast<const uint4*>(rows + (size_t)e * RW + 4 * q);
    unpack_pairs_lds<K, RW>(slot);
    uint32_t a[K], c[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      a[j] = state[(size_t)e * 2 * K + j];
      c[j] = state[(size_t)e * 2 * K + K + j];
    }
    M.mul(a, c, slot, topc);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      state[(size_t)e * 2 * K + j] = a[j];
      state[(size_t)e * 2 * K + K + j] = c[j];
    }
  } else if (mode == 3) {  // state <- state^2 (the state parked in the slot, as the decrypt does)
    uint32_t a[K], c[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      a[j] = state[(size_t)e * 2 * K + j];
      c[j] = state[(size_t)e * 2 * K + K + j];
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q)
      *reinterpret_cast<uint4*>(slot + q * 256) =
          make_uint4(2 * q < K ? a[2 * q] : 0u, 2 * q < K ? c[2 * q] : 0u, 2 * q + 1 < K ? a[2 * q + 1] : 0u,
                     2 * q + 1 < K ? c[2 * q + 1] : 0u);
    M.sqr(a, c, slot, topc);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      state[(size_t)e * 2 * K + j] = a[j];
      state[(size_t)e * 2 * K + K + j] = c[j];
    }
  } else if (mode == 1) {
    uint32_t a[K], c[K], x[2 * K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      a[j] = state[(size_t)e * 2 * K + j];
      c[j] = state[(size_t)e * 2 * K + K + j];
    }
    M.to_mont2(a, c, x);
#pragma unroll
    for (int j = 0; j < 2 * K; ++j) out[(size_t)e * 2 * K + j] = x[j];
  } else {
    uint32_t x[2 * K], f0[K], f1[K];
#pragma unroll
    for (int j = 0; j < 2 * K; ++j) x[j] = state[(size_t)e * 2 * K + j];
    pmd_from_mont2<K>(M, x, RmodP, f0, f1);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      out[(size_t)e * 2 * K + j] = f0[j];
      out[(size_t)e * 2 * K + K + j] = f1[j];
    }
  }
}

// ITER dependent products of each lane's state with its own row (staged once)
__global__ void __launch_bounds__(128, 2) k_time_pmd(const uint32_t* P, uint32_t n0inv, const uint32_t* topc_g,
                                                     const uint32_t* rows, const uint32_t* state, uint32_t* sink,
                                                     int count, int iters) {
  __shared__ __attribute__((aligned(16))) uint32_t img_all[2][NQ * 256];
  __shared__ __attribute__((aligned(16))) uint32_t topc[40];
  if (threadIdx.x < 40) topc[threadIdx.x] = threadIdx.x < K ? topc_g[threadIdx.x] : 0u;
  __syncthreads();
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  const int s = e % 256;
  uint32_t* slot = img_all[(threadIdx.x >> 6) & 1] + (threadIdx.x & 63) * 4;
#pragma unroll
  for (int q = 0; q < RW / 4; ++q)
    *reinterpret_cast<uint4*>(slot + q * 256) = *reinterpret_cast<const uint4*>(rows + (size_t)s * RW + 4 * q);
  unpack_pairs_lds<K, RW>(slot);
  PM M;
  M.init(P, n0inv);
  uint32_t a[K], c[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    a[j] = state[(size_t)s * 2 * K + j];
    c[j] = state[(size_t)s * 2 * K + K + j];
  }
  for (int t = 0; t < iters; ++t) M.mul(a, c, slot, topc);
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) acc ^= a[j] ^ c[j];
  sink[e] = acc;
}

// The production product for comparison: Mont<74, 28, 1>::mul with the row
// staged in the lane's LDS slot (k_djn_pow_lds's ALdsQ operand, modulus limbs
// through the SGPR pipeline)
struct ALdsQ {
  const uint32_t* q;
  XHE_DEV uint4 load4(int i) const { return *reinterpret_cast<const uint4*>(q + (i >> 2) * 256); }
};
__global__ void __launch_bounds__(128, 2) k_time_mont(const uint32_t* __restrict__ N, uint32_t n0, const uint32_t* x,
                                                      const uint32_t* y, uint32_t* out, int count, int iters) {
  __shared__ __attribute__((aligned(16))) uint32_t img_all[2][(MP::S4 / 4) * 256];
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  uint32_t* slot = img_all[(threadIdx.x >> 6) & 1] + (threadIdx.x & 63) * 4;
  const int s = e % 256;
#pragma unroll
  for (int q = 0; q < MP::S4 / 4; ++q)
    *reinterpret_cast<uint4*>(slot + q * 256) = *reinterpret_cast<const uint4*>(y + (size_t)s * MP::S4 + 4 * q);
  MP M;
  M.init(N, n0);
  uint32_t b[MP::L];
  M.load_row(b, x + (size_t)s * MP::S4);
  for (int t = 0; t < iters; ++t) M.mul(b, ALdsQ{slot});
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < MP::L; ++i) acc ^= b[i];
  out[e] = acc;
}

static BigU rand_big(std::mt19937_64& rng, int bits) {
  std::vector<uint32_t> w((bits + 31) / 32);
  for (auto& v : w) v = (uint32_t)rng();
  if (bits % 32) w.back() &= (1u << (bits % 32)) - 1;
  return BigU::from_words(w.data(), w.size());
}

static void put_limbs(std::vector<uint32_t>& v, const BigU& a, int n) {
  auto l = a.to_limbs(28, n);
  v.insert(v.end(), l.begin(), l.end());
}
// K limbs with the top one unmasked (values up to ~2^(28K+1))
static void put_limbs_loose(std::vector<uint32_t>& v, const BigU& a, int n) {
  std::vector<uint32_t> l(n);
  for (int j = 0; j < n; ++j) {
    size_t bit = (size_t)28 * j, k = bit >> 5, sh = bit & 31;
    uint64_t x = (uint64_t)a.word(k) | ((uint64_t)a.word(k + 1) << 32);
    l[j] = j + 1 < n ? (uint32_t)((x >> sh) & 0xFFFFFFFu) : (uint32_t)(x >> sh);
  }
  v.insert(v.end(), l.begin(), l.end());
}
static BigU from_limbs(const uint32_t* l, int n) {
  BigU r;
  for (int j = n - 1; j >= 0; --j) r = add(shl(r, 28), BigU(l[j]));
  return r;
}

int main() {
  std::mt19937_64 rng(4321);
  BigU P;
  {
    auto pw = rand_big(rng, 1024).to_limbs(32, 32);
    pw[31] |= 0x80000000u;
    pw[0] |= 1u;
    P = BigU::from_words(pw.data(), 32);
  }
  const BigU P2 = mul(P, P);
  const BigU R = pow2(28 * K);
  const BigU Rp = mod(R, P);
  const BigU Rinv = modinv(Rp, P);
  const BigU E = submod(BigU(1), Rp, P);  // (1 - R) mod P
  const BigU R2inv = modinv(mod(mul(R, R), P2), P2);
  const uint32_t n0 = mont_ninv(P.word(0), 28);
  std::vector<uint32_t> hP, hE, hRp, topc;
  put_limbs(hP, P, K);
  put_limbs(hE, E, K);
  put_limbs(hRp, Rp, K);
  for (int i = 0; i < K; ++i) topc.push_back(0xFFFFFFFu + hE[i]);
  // digits (e, f) < P of x R^2 mod P^2
  auto digits = [&](const BigU& x, BigU* e, BigU* f) {
    BigU X = mulmod(x, mod(mul(R, R), P2), P2);
    *e = mulmod(mod(X, P), Rinv, P);
    BigU V = sub(add(X, mul(R, P)), mul(R, *e));  // X + R P - R e > 0, = 0 (mod P)
    BigU q, r;
    divmod(V, P, &q, &r);
    *f = submod(mod(q, P), Rp, P);
  };
  auto value = [&](const BigU& a, const BigU& c) { return mulmod(mod(add(mul(R, a), mul(P, c)), P2), R2inv, P2); };
  auto pack_row = [&](std::vector<uint32_t>& v, const BigU& e, const BigU& f) {
    for (int k = 0; k < RW / 2; ++k) v.push_back(e.word(k));
    for (int k = 0; k < RW / 2; ++k) v.push_back(f.word(k));
  };

  const int count = 4096, chain = 8;
  std::vector<BigU> xs(count), sa(count), sc(count);
  std::vector<uint32_t> hstate;
  for (int i = 0; i < count; ++i) {
    xs[i] = mod(rand_big(rng, 2048), P2);
    if (i == 0) xs[i] = sub(P2, BigU(1));
    if (i == 1) xs[i] = BigU(1);
    digits(xs[i], &sa[i], &sc[i]);
    put_limbs_loose(hstate, sa[i], K);
    put_limbs_loose(hstate, sc[i], K);
  }
  uint32_t *dP, *dtopc, *dRp, *drows, *dstate, *dout;
  hipMalloc(&dP, hP.size() * 4);
  hipMalloc(&dtopc, topc.size() * 4);
  hipMalloc(&dRp, hRp.size() * 4);
  hipMalloc(&drows, (size_t)count * RW * 4);
  hipMalloc(&dstate, (size_t)count * 2 * K * 4);
  hipMalloc(&dout, (size_t)count * 2 * K * 4);
  hipMemcpy(dP, hP.data(), hP.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dtopc, topc.data(), topc.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dRp, hRp.data(), hRp.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dstate, hstate.data(), hstate.size() * 4, hipMemcpyHostToDevice);
  int rc = 0;
  // 1. product chains
  {
    int bad = 0, range = 0;
    std::vector<BigU> acc = xs;
    std::vector<uint32_t> hrows;
    std::vector<BigU> ys(count);
    for (int t = 0; t < chain; ++t) {
      hrows.clear();
      for (int i = 0; i < count; ++i) {
        ys[i] = mod(rand_big(rng, 2048), P2);
        if (t == 0 && i == 2) ys[i] = sub(P2, BigU(1));
        if (t == 1 && i == 3) ys[i] = BigU(0);
        BigU e, f;
        digits(ys[i], &e, &f);
        pack_row(hrows, e, f);
        acc[i] = mulmod(acc[i], ys[i], P2);
      }
      hipMemcpy(drows, hrows.data(), hrows.size() * 4, hipMemcpyHostToDevice);
      hipLaunchKernelGGL(k_check, dim3(count / 128), dim3(128), 0, 0, dP, n0, dtopc, dRp, drows, dstate, dout, count,
                         0);
      if (hipMemcpy(hstate.data(), dstate, hstate.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) {
        printf("{\"error\": \"hip\"}\n");
        return 1;
      }
      const BigU cmax = add(R, mul(P, BigU(8)));
      const BigU amax = mul(P, BigU(2));
      for (int i = 0; i < count; ++i) {
        BigU a = from_limbs(&hstate[(size_t)i * 2 * K], K), c = from_limbs(&hstate[(size_t)i * 2 * K + K], K);
        if (cmp(value(a, c), acc[i]) != 0) {
          if (++bad < 4) printf("  chain %d elem %d: wrong value\n", t, i);
        }
        if (cmp(a, amax) >= 0 || cmp(c, cmax) >= 0) ++range;
      }
    }
    printf("{\"check\": \"mul\", \"bad\": %d, \"out_of_range\": %d, \"of\": %d}\n", bad, range, count * chain);
    rc |= bad != 0 || range != 0;
    // squaring chains continue from the product chains' states
    bad = range = 0;
    for (int t = 0; t < chain; ++t) {
      for (int i = 0; i < count; ++i) acc[i] = mulmod(acc[i], acc[i], P2);
      hipLaunchKernelGGL(k_check, dim3(count / 128), dim3(128), 0, 0, dP, n0, dtopc, dRp, drows, dstate, dout, count,
                         3);
      if (hipMemcpy(hstate.data(), dstate, hstate.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) {
        printf("{\"error\": \"hip\"}\n");
        return 1;
      }
      const BigU cmax = add(R, mul(P, BigU(8)));
      const BigU amax = mul(P, BigU(2));
      for (int i = 0; i < count; ++i) {
        BigU a = from_limbs(&hstate[(size_t)i * 2 * K], K), c = from_limbs(&hstate[(size_t)i * 2 * K + K], K);
        if (cmp(value(a, c), acc[i]) != 0 && ++bad < 4) printf("  sqr chain %d elem %d: wrong value\n", t, i);
        if (cmp(a, amax) >= 0 || cmp(c, cmax) >= 0) ++range;
      }
    }
    printf("{\"check\": \"sqr\", \"bad\": %d, \"out_of_range\": %d, \"of\": %d}\n", bad, range, count * chain);
    rc |= bad != 0 || range != 0;
  }
  // 2. to_mont2 of the final states: R a + P c (74 limbs, exact integer)
  {
    hipLaunchKernelGGL(k_check, dim3(count / 128), dim3(128), 0, 0, dP, n0, dtopc, dRp, drows, dstate, dout, count, 1);
    std::vector<uint32_t> ho((size_t)count * 2 * K);
    hipMemcpy(ho.data(), dout, ho.size() * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < count; ++i) {
      BigU a = from_limbs(&hstate[(size_t)i * 2 * K], K), c = from_limbs(&hstate[(size_t)i * 2 * K + K], K);
      if (cmp(from_limbs(&ho[(size_t)i * 2 * K], 2 * K), add(mul(R, a), mul(P, c))) != 0 && ++bad < 4)
        printf("  to_mont2 elem %d wrong\n", i);
    }
    printf("{\"check\": \"to_mont2\", \"bad\": %d, \"of\": %d}\n", bad, count);
    rc |= bad != 0;
  }
  // 3. from_mont2: X < P^2 -> (e, f)
  {
    std::vector<BigU> X(count);
    std::vector<uint32_t> hx;
    for (int i = 0; i < count; ++i) {
      X[i] = mod(rand_big(rng, 2048), P2);
      if (i == 0) X[i] = BigU(0);
      if (i == 1) X[i] = sub(P2, BigU(1));
      if (i == 2) X[i] = mul(R, sub(P, BigU(1)));  // t near P
      X[i] = mod(X[i], P2);
      put_limbs(hx, X[i], 2 * K);
    }
    hipMemcpy(dstate, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_check, dim3(count / 128), dim3(128), 0, 0, dP, n0, dtopc, dRp, drows, dstate, dout, count, 2);
    std::vector<uint32_t> ho((size_t)count * 2 * K);
    hipMemcpy(ho.data(), dout, ho.size() * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < count; ++i) {
      BigU e = from_limbs(&ho[(size_t)i * 2 * K], K), f = from_limbs(&ho[(size_t)i * 2 * K + K], K);
      const bool ok = cmp(e, P) < 0 && cmp(f, P) < 0 && cmp(mod(add(mul(R, e), mul(P, f)), P2), X[i]) == 0;
      if (!ok && ++bad < 4) printf("  from_mont2 elem %d wrong\n", i);
    }
    printf("{\"check\": \"from_mont2\", \"bad\": %d, \"of\": %d}\n", bad, count);
    rc |= bad != 0;
  }
  // 4. throughput
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int lanes = cus * 4 * 2 * 64, iters = 64;
  uint32_t* dsink;
  hipMalloc(&dsink, (size_t)lanes * 4);
  std::vector<uint32_t> mx, my, hN = P2.to_limbs(28, MP::S);
  hN.resize(MP::S4, 0);
  for (int i = 0; i < 256; ++i) {
    auto a = xs[i].to_limbs(28, MP::S), b = xs[(i + 1) % count].to_limbs(28, MP::S);
    a.resize(MP::S4, 0);
    b.resize(MP::S4, 0);
    mx.insert(mx.end(), a.begin(), a.end());
    my.insert(my.end(), b.begin(), b.end());
  }
  uint32_t *dN, *dmx, *dmy;
  hipMalloc(&dN, hN.size() * 4);
  hipMalloc(&dmx, mx.size() * 4);
  hipMalloc(&dmy, my.size() * 4);
  hipMemcpy(dN, hN.data(), hN.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dmx, mx.data(), mx.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dmy, my.data(), my.size() * 4, hipMemcpyHostToDevice);
  const uint32_t n0m = mont_ninv(P2.word(0), 28);
  hipEvent_t ta, tb;
  hipEventCreate(&ta);
  hipEventCreate(&tb);
  auto time_it = [&](auto launch) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(ta);
    launch();
    hipEventRecord(tb);
    hipEventSynchronize(tb);
    float ms = 0;
    hipEventElapsedTime(&ms, ta, tb);
    return (double)lanes * iters / (ms * 1e-3);
  };
  const double mont = time_it([&] {
    hipLaunchKernelGGL(k_time_mont, dim3(lanes / 128), dim3(128), 0, 0, dN, n0m, dmx, dmy, dsink, lanes, iters);
  });
  const double pmd = time_it([&] {
    hipLaunchKernelGGL(k_time_pmd, dim3(lanes / 128), dim3(128), 0, 0, dP, n0, dtopc, drows, dstate, dsink, lanes,
                       iters);
  });
  printf("{\"products_per_s\": {\"montgomery_mod_P2\": %.4g, \"montgomery_digits\": %.4g}, "
         "\"digits_vs_montgomery\": %.3f, \"lanes\": %d, \"iters\": %d}\n",
         mont, pmd, pmd / mont, lanes, iters);
  return rc;
}
