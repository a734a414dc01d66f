// Differential probe of WaveDig::mul (dec_wave.hpp): one digit product per
// block on given operands; the host side (tools/dbg/wavedig_probe.py) checks
// every result residue against Python integers. Debug tool, not product code.
//   wavedig_probe IN OUT N     IN: P, P', topc (3 x 37 words) then N x (a, c, e, f) x 37 words
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../xfl_amd/csrc/xhe_kernels.hpp"
#include "../../xfl_amd/csrc/dec_wave.hpp"
using namespace xhe;
constexpr int K = 37;
__global__ void __launch_bounds__(256) k_probe(const uint32_t* consts, const uint32_t* in, uint32_t* out, uint64_t* cols, int n) {
  using WD = WaveDig<K, 4>;
  __shared__ __attribute__((aligned(16))) WD::Lds s;
  const int l = threadIdx.x;
  const int e = blockIdx.x;
  uint32_t* w = reinterpret_cast<uint32_t*>(&s);
  for (int j = l; j < (int)(sizeof(s) / 4); j += WD::NT) w[j] = 0u;
  __syncthreads();
  const uint32_t* x = in + (size_t)e * 4 * K;
  for (int j = l; j < K; j += WD::NT) {
    s.zp[WD::ZO + j] = consts[j];
    s.zpp[WD::ZO + j] = consts[K + j];
    s.topc[j] = consts[2 * K + j];
    s.a[j] = x[j];
    s.c[j] = x[K + j];
    s.ze[WD::ZO + j] = x[2 * K + j];
    s.zf[WD::ZO + j] = x[3 * K + j];
  }
  __syncthreads();
  int cur = 0;
  WD::mul(s, cur, s.a, s.c, s.a, s.c, false);
  for (int j = l; j < K; j += WD::NT) {
    out[(size_t)e * 2 * K + j] = s.a[j];
    out[(size_t)e * 2 * K + K + j] = s.c[j];
  }
  constexpr int NC = WD::G + 2 * K;
  for (int j = l; j < 2 * NC; j += WD::NT) cols[(size_t)e * 2 * NC + j] = j < NC ? s.col1[cur][j] : s.col2[cur][j - NC];
}
int main(int argc, char** argv) {
  if (argc < 4) return 2;
  const int n = atoi(argv[3]);
  std::vector<uint32_t> h((size_t)3 * K + (size_t)n * 4 * K), o((size_t)n * 2 * K);
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(h.data(), 4, h.size(), f) != h.size()) return 3;
  fclose(f);
  uint32_t *dc, *di, *dout;
  uint64_t* dcol;
  constexpr int NC = 3 + 2 * K;
  std::vector<uint64_t> oc((size_t)n * 2 * NC);
  if (hipMalloc(&dc, 3 * K * 4) || hipMalloc(&di, (size_t)n * 4 * K * 4) || hipMalloc(&dout, o.size() * 4) || hipMalloc(&dcol, oc.size() * 8)) return 4;
  hipMemcpy(dc, h.data(), 3 * K * 4, hipMemcpyHostToDevice);
  hipMemcpy(di, h.data() + 3 * K, (size_t)n * 4 * K * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_probe, dim3(n), dim3(256), 0, 0, dc, di, dout, dcol, n);
  if (hipDeviceSynchronize() != hipSuccess) return 5;
  hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(oc.data(), dcol, oc.size() * 8, hipMemcpyDeviceToHost);
  if (argc > 4) {
    FILE* fc = fopen(argv[4], "wb");
    fwrite(oc.data(), 8, oc.size(), fc);
    fclose(fc);
  }
  f = fopen(argv[2], "wb");
  fwrite(o.data(), 4, o.size(), f);
  fclose(f);
  printf("probe done %d\n", n);
  return 0;
}
