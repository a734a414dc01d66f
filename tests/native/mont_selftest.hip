// Device Montgomery primitive self-test (run on the GPU box):
// compares Mont<S,W,TPI>::mul / reduce_once / normalize against host BigU
// arithmetic for random odd moduli. Prints one line per shape and exits 1
// on any mismatch.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <random>
#include "../../xfl_amd/csrc/bn_dev.hpp"
#include "../../xfl_amd/csrc/hostbn.hpp"

using namespace xhe;

template <class MP>
__global__ void k_test(const uint32_t* N, uint32_t n0, const uint32_t* x, const uint32_t* y, uint32_t* out, int count,
                       int mode) {
  int e = (blockIdx.x * blockDim.x + threadIdx.x) / MP::TPI;
  if (e >= count) return;
  MP M;
  M.init(N, n0);
  uint32_t b[MP::L];
  M.load_row(b, x + (size_t)e * MP::S4);
  if (mode != 2) M.mul(b, ARow{y + (size_t)e * MP::S4});
  if (mode != 1) M.reduce_once(b);
  M.store_row(b, out + (size_t)e * MP::S4);
}

template <class MP>
int run(int bits, std::mt19937_64& rng, int mode) {
  const int count = 256;
  BigU N;
  {
    std::vector<uint32_t> w((bits + 31) / 32);
    for (auto& v : w) v = (uint32_t)rng();
    if (bits % 32) w.back() &= (1u << (bits % 32)) - 1;
    w.back() |= 1u << ((bits - 1) % 32);
    w[0] |= 1;
    N = BigU::from_words(w.data(), w.size());
  }
  std::vector<uint32_t> hx, hy, hN = N.to_limbs(MP::W, MP::S);
  hN.resize(MP::S4, 0);
  std::vector<BigU> xs, ys;
  for (int i = 0; i < count; ++i) {
    std::vector<uint32_t> w((bits + 31) / 32);
    for (auto& v : w) v = (uint32_t)rng();
    BigU a = mod(BigU::from_words(w.data(), w.size()), N);
    for (auto& v : w) v = (uint32_t)rng();
    BigU b = mod(BigU::from_words(w.data(), w.size()), N);
    if (i == 0) a = sub(N, BigU(1));
    if (i == 1) { a = sub(N, BigU(1)); b = sub(N, BigU(1)); }
    xs.push_back(a);
    ys.push_back(b);
    auto la = a.to_limbs(MP::W, MP::S), lb = b.to_limbs(MP::W, MP::S);
    la.resize(MP::S4, 0);
    lb.resize(MP::S4, 0);
    hx.insert(hx.end(), la.begin(), la.end());
    hy.insert(hy.end(), lb.begin(), lb.end());
  }
  uint32_t *dN, *dx, *dy, *dout;
  hipMalloc(&dN, hN.size() * 4);
  hipMalloc(&dx, hx.size() * 4);
  hipMalloc(&dy, hy.size() * 4);
  hipMalloc(&dout, hx.size() * 4);
  hipMemcpy(dN, hN.data(), hN.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dx, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dy, hy.data(), hy.size() * 4, hipMemcpyHostToDevice);
  uint32_t n0 = mont_ninv(N.word(0), MP::W);
  int blocks = (count * MP::TPI + 255) / 256;
  hipLaunchKernelGGL(k_test<MP>, dim3(blocks), dim3(256), 0, 0, dN, n0, dx, dy, dout, count, mode);
  std::vector<uint32_t> ho(hx.size());
  if (hipMemcpy(ho.data(), dout, ho.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) {
    printf("hip error\n");
    return 1;
  }
  BigU R = pow2((size_t)MP::W * MP::S);
  BigU Rinv = modinv(mod(R, N), N);
  int bad = 0;
  for (int i = 0; i < count; ++i) {
    BigU want = mulmod(mulmod(xs[i], ys[i], N), Rinv, N);
    if (mode == 2) want = xs[i];
    if (mode == 1) {  // unreduced product: compare mod N
      std::vector<uint32_t> got(ho.begin() + (size_t)i * MP::S4, ho.begin() + (size_t)i * MP::S4 + MP::S);
      BigU g;
      for (int j = MP::S - 1; j >= 0; --j) g = add(shl(g, MP::W), BigU(got[j]));
      if (cmp(mod(g, N), want) != 0 || cmp(g, shl(N, 1)) >= 0) { bad++; if (bad < 4) printf("  elem %d mismatch (unreduced)\n", i); }
      continue;
    }
    auto wl = want.to_limbs(MP::W, MP::S);
    for (int j = 0; j < MP::S; ++j)
      if (wl[j] != ho[(size_t)i * MP::S4 + j]) { bad++; if (bad < 4) printf("  elem %d limb %d got %08x want %08x\n", i, j, ho[(size_t)i * MP::S4 + j], wl[j]); break; }
  }
  printf("{\"shape\": \"S=%d W=%d TPI=%d bits=%d\", \"mode\": %d, \"bad\": %d, \"of\": %d}\n", MP::S, MP::W, MP::TPI, bits, mode, bad, count);
  hipFree(dN); hipFree(dx); hipFree(dy); hipFree(dout);
  return bad != 0;
}

int main() {
  std::mt19937_64 rng(1234);
  int rc = 0;
  for (int mode = 0; mode < 3; ++mode) {
    rc |= run<Mont<74, 28, 1>>(2048, rng, mode);
    rc |= run<Mont<74, 28, 2>>(2048, rng, mode);
    rc |= run<Mont<110, 28, 2>>(3072, rng, mode);
    rc |= run<Mont<56, 28, 2>>(1536, rng, mode);
    rc |= run<Mont<152, 27, 4>>(4096, rng, mode);
    rc |= run<Mont<76, 27, 4>>(2048, rng, mode);
    rc |= run<Mont<160, 27, 16>>(4096, rng, mode);
    rc |= run<Mont<304, 27, 16>>(8192, rng, mode);
    rc |= run<Mont<640, 26, 16>>(16384, rng, mode);
  }
  return rc;
}
