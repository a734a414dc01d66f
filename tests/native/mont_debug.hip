// printf trace of one Montgomery product with TPI=2 (debug aid)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../../xfl_amd/csrc/bn_dev.hpp"
#include "../../xfl_amd/csrc/hostbn.hpp"
using namespace xhe;
using MP = Mont<8, 28, 2>;
__global__ void k(const uint32_t* N, uint32_t n0, const uint32_t* x, const uint32_t* y, uint32_t* out) {
  if (threadIdx.x >= 2) return;
  MP M;
  M.init(N, n0);
  uint32_t b[MP::L];
  M.load_row(b, x);
  uint64_t T[MP::L];
  for (int j = 0; j < MP::L; ++j) T[j] = 0;
  const bool lead = MP::G::g() == 0;
  for (int i = 0; i < MP::S; ++i) {
    M.step(M.np(), T, b, y[i], lead);
    printf("i=%d lane=%d T=%llx %llx %llx %llx\n", i, (int)threadIdx.x, (unsigned long long)T[0], (unsigned long long)T[1], (unsigned long long)T[2], (unsigned long long)T[3]);
  }
  M.normalize(T, b);
  M.store_row(b, out);
}
int main() {
  uint32_t hN[8], hx[8], hy[8];
  for (int i = 0; i < 8; i++) { hN[i] = (0x9e3779b9u * (i + 1)) & 0xfffffff; hx[i] = (0x85ebca6bu * (i + 3)) & 0xfffffff; hy[i] = (0xc2b2ae35u * (i + 7)) & 0xfffffff; }
  hN[0] |= 1; hN[7] |= 0x8000000; hx[7] &= 0x3ffffff; hy[7] &= 0x3ffffff;
  uint32_t n0 = mont_ninv(hN[0], 28);
  uint32_t *dN, *dx, *dy, *dout;
  (void)hipMalloc(&dN, 32); (void)hipMalloc(&dx, 32); (void)hipMalloc(&dy, 32); (void)hipMalloc(&dout, 32);
  (void)hipMemcpy(dN, hN, 32, hipMemcpyHostToDevice); (void)hipMemcpy(dx, hx, 32, hipMemcpyHostToDevice); (void)hipMemcpy(dy, hy, 32, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dN, n0, dx, dy, dout);
  uint32_t ho[8];
  (void)hipMemcpy(ho, dout, 32, hipMemcpyDeviceToHost);
  printf("N="); for (int i = 0; i < 8; i++) printf("%07x ", hN[i]); printf("\nx="); for (int i = 0; i < 8; i++) printf("%07x ", hx[i]);
  printf("\ny="); for (int i = 0; i < 8; i++) printf("%07x ", hy[i]); printf("\nn0=%x\nout="); for (int i = 0; i < 8; i++) printf("%07x ", ho[i]); printf("\n");
  return 0;
}
