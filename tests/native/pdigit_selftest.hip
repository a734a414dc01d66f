// Device self-test and timing of the base-P digit arithmetic mod P^2
// (xfl_amd/csrc/pdigit_dev.hpp): run on the GPU box.
//
// 1. PDig<37>::mul / sqr on random digits (and edge values) against host
//    big-integer arithmetic (hostbn.hpp): every result digit bit-exact.
// 2. Throughput: each lane runs ITER dependent products (or squarings) on its
//    own residue, PDig<37> in digit form against Mont<74, 28, 1>::mul (the
//    current product mod P^2 of k_djn_pow / k_dec_pow), same grid (2 waves
//    per SIMD, the whole chip), hipEvent-timed.
// Prints JSON lines; exits 1 on any mismatch.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <random>
#include <vector>

#include "../../xfl_amd/csrc/bn_dev.hpp"
#include "../../xfl_amd/csrc/hostbn.hpp"
#include "../../xfl_amd/csrc/pdigit_dev.hpp"

using namespace xhe;
constexpr int K = 37;
using PD = PDig<K>;
using MP = Mont<74, 28, 1>;

__global__ void __launch_bounds__(256, 2) k_check(const uint32_t* P, const uint32_t* MU, const uint32_t* x,
                                                  const uint32_t* y, uint32_t* out, int count, int mode) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  PD D{P, MU};
  uint32_t x0[K], x1[K], y0[K], y1[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    x0[i] = x[(size_t)e * 2 * K + i];
    x1[i] = x[(size_t)e * 2 * K + K + i];
    y0[i] = y[(size_t)e * 2 * K + i];
    y1[i] = y[(size_t)e * 2 * K + K + i];
  }
  if (mode == 0) D.mul(x0, x1, y0, y1);
  else D.sqr(x0, x1);
#pragma unroll
  for (int i = 0; i < K; ++i) {
    out[(size_t)e * 2 * K + i] = x0[i];
    out[(size_t)e * 2 * K + K + i] = x1[i];
  }
}

// ITER products (MODE 0) or squarings (MODE 1) of each lane's residue with its
// own fixed second operand (one kernel per mode: registers are allocated for
// that code path alone)
template <int MODE>
__global__ void __launch_bounds__(256, 2) k_time_digit(const uint32_t* P, const uint32_t* MU, const uint32_t* x,
                                                       const uint32_t* y, uint32_t* out, int count, int iters) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  PD D{P, MU};
  uint32_t x0[K], x1[K], y0[K], y1[K];
  const int s = e % 256;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    x0[i] = x[(size_t)s * 2 * K + i];
    x1[i] = x[(size_t)s * 2 * K + K + i];
    y0[i] = y[(size_t)s * 2 * K + i];
    y1[i] = y[(size_t)s * 2 * K + K + i];
  }
  for (int t = 0; t < iters; ++t) {
    if constexpr (MODE == 0) D.mul(x0, x1, y0, y1);
    else D.sqr(x0, x1);
  }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < K; ++i) acc ^= x0[i] ^ x1[i];
  out[e] = acc;
}

__global__ void __launch_bounds__(256, 2) k_time_mont(const uint32_t* N, uint32_t n0, const uint32_t* x,
                                                      const uint32_t* y, uint32_t* out, int count, int iters) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  MP M;
  M.init(N, n0);
  uint32_t b[MP::L];
  const int s = e % 256;
  M.load_row(b, x + (size_t)s * MP::S4);
  for (int t = 0; t < iters; ++t) M.mul(b, ARow{y + (size_t)s * MP::S4});
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

int main() {
  std::mt19937_64 rng(4321);
  BigU P = rand_big(rng, 1024);
  P = add(P, BigU(0));
  {
    std::vector<uint32_t> w((1024 + 31) / 32);
    auto pw = P.to_limbs(32, 32);
    pw[31] |= 0x80000000u;
    pw[0] |= 1u;
    P = BigU::from_words(pw.data(), 32);
  }
  const BigU P2 = mul(P, P);
  BigU MU, rem;
  divmod(pow2(28 * 2 * K), P, &MU, &rem);
  std::vector<uint32_t> hP, hMU;
  put_limbs(hP, P, K);
  put_limbs(hMU, MU, K + 1);
  const int count = 4096;
  std::vector<BigU> xs, ys;
  std::vector<uint32_t> hx, hy;
  for (int i = 0; i < count; ++i) {
    BigU a = mod(rand_big(rng, 2048), P2), b = mod(rand_big(rng, 2048), P2);
    if (i == 0) a = sub(P2, BigU(1));
    if (i == 1) a = b = sub(P2, BigU(1));
    if (i == 2) a = sub(P, BigU(1));
    if (i == 3) b = P;
    if (i == 4) a = BigU(0);
    xs.push_back(a);
    ys.push_back(b);
    BigU a1, a0, b1, b0;
    divmod(a, P, &a1, &a0);
    divmod(b, P, &b1, &b0);
    put_limbs(hx, a0, K);
    put_limbs(hx, a1, K);
    put_limbs(hy, b0, K);
    put_limbs(hy, b1, K);
  }
  uint32_t *dP, *dMU, *dx, *dy, *dout;
  hipMalloc(&dP, hP.size() * 4);
  hipMalloc(&dMU, hMU.size() * 4);
  hipMalloc(&dx, hx.size() * 4);
  hipMalloc(&dy, hy.size() * 4);
  hipMalloc(&dout, hx.size() * 4);
  hipMemcpy(dP, hP.data(), hP.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dMU, hMU.data(), hMU.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dx, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dy, hy.data(), hy.size() * 4, hipMemcpyHostToDevice);
  int rc = 0;
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(k_check, dim3(count / 256), dim3(256), 0, 0, dP, dMU, dx, dy, dout, count, mode);
    std::vector<uint32_t> ho(hx.size());
    if (hipMemcpy(ho.data(), dout, ho.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) {
      printf("{\"error\": \"hip\"}\n");
      return 1;
    }
    int bad = 0;
    for (int i = 0; i < count; ++i) {
      BigU want = mode == 0 ? mulmod(xs[i], ys[i], P2) : mulmod(xs[i], xs[i], P2);
      BigU w1, w0;
      divmod(want, P, &w1, &w0);
      std::vector<uint32_t> wl;
      put_limbs(wl, w0, K);
      put_limbs(wl, w1, K);
      for (int j = 0; j < 2 * K; ++j)
        if (wl[j] != ho[(size_t)i * 2 * K + j]) {
          if (++bad < 4) printf("  elem %d limb %d got %07x want %07x\n", i, j, ho[(size_t)i * 2 * K + j], wl[j]);
          break;
        }
    }
    printf("{\"check\": \"%s\", \"bad\": %d, \"of\": %d}\n", mode ? "sqr" : "mul", bad, count);
    rc |= bad != 0;
  }
  // throughput: 2 waves per SIMD on every CU, ITER products per lane
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int lanes = cus * 4 * 2 * 64, iters = 64;
  uint32_t* dsink;
  hipMalloc(&dsink, (size_t)lanes * 4);
  // Montgomery operands: the same residues, as 74-limb rows
  std::vector<uint32_t> mx, my;
  for (int i = 0; i < 256; ++i) {
    auto a = xs[i].to_limbs(28, MP::S), b = ys[i].to_limbs(28, MP::S);
    a.resize(MP::S4, 0);
    b.resize(MP::S4, 0);
    mx.insert(mx.end(), a.begin(), a.end());
    my.insert(my.end(), b.begin(), b.end());
  }
  std::vector<uint32_t> hN = P2.to_limbs(28, MP::S);
  hN.resize(MP::S4, 0);
  uint32_t *dN, *dmx, *dmy;
  hipMalloc(&dN, hN.size() * 4);
  hipMalloc(&dmx, mx.size() * 4);
  hipMalloc(&dmy, my.size() * 4);
  hipMemcpy(dN, hN.data(), hN.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dmx, mx.data(), mx.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dmy, my.data(), my.size() * 4, hipMemcpyHostToDevice);
  const uint32_t n0 = mont_ninv(P2.word(0), 28);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto time_it = [&](auto launch) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(a);
    launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return (double)lanes * iters / (ms * 1e-3);
  };
  const double mont = time_it([&] {
    hipLaunchKernelGGL(k_time_mont, dim3(lanes / 256), dim3(256), 0, 0, dN, n0, dmx, dmy, dsink, lanes, iters);
  });
  const double dmul = time_it([&] {
    hipLaunchKernelGGL(k_time_digit<0>, dim3(lanes / 256), dim3(256), 0, 0, dP, dMU, dx, dy, dsink, lanes, iters);
  });
  const double dsqr = time_it([&] {
    hipLaunchKernelGGL(k_time_digit<1>, dim3(lanes / 256), dim3(256), 0, 0, dP, dMU, dx, dy, dsink, lanes, iters);
  });
  printf("{\"products_per_s\": {\"montgomery_mod_P2\": %.4g, \"digit_mul\": %.4g, \"digit_sqr\": %.4g}, "
         "\"digit_mul_vs_montgomery\": %.3f, \"lanes\": %d, \"iters\": %d}\n",
         mont, dmul, dsqr, dmul / mont, lanes, iters);
  return rc;
}
