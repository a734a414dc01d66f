// Integer / FP64 VALU throughput microbenchmark for gfx950.
// Measures lane-ops per second for the instructions a multi-precision
// Montgomery product can be built from; the peak P_int used by bench.py's
// roofline is the v_mad_u64_u32 rate measured here.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 16384
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// 8 independent 64-bit accumulators per lane.
__global__ void __launch_bounds__(256) k_mad64(uint32_t* out, uint32_t s) {
  uint64_t acc[8];
  uint32_t a = threadIdx.x * 2654435761u + s, b = a ^ 0x9e3779b9u;
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++)
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b) : "vcc");
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r ^= (uint32_t)acc[i] ^ (uint32_t)(acc[i] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

// mad with carry-out counted: the product-scanning MAC step.
__global__ void __launch_bounds__(256) k_mad64_addc(uint32_t* out, uint32_t s) {
  uint64_t acc[8];
  uint32_t c2[8];
  uint32_t a = threadIdx.x * 2654435761u + s, b = a ^ 0x9e3779b9u;
#pragma unroll
  for (int i = 0; i < 8; i++) { acc[i] = a + i; c2[i] = 0; }
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++)
      asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc"
                   : "+v"(acc[i]), "+v"(c2[i]) : "v"(a), "v"(b) : "vcc");
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r ^= (uint32_t)acc[i] ^ (uint32_t)(acc[i] >> 32) ^ c2[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void __launch_bounds__(256) k_mullo(uint32_t* out, uint32_t s) {
  uint32_t acc[8];
  uint32_t a = threadIdx.x * 2654435761u + s;
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++)
      asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(a));
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void __launch_bounds__(256) k_mulhi(uint32_t* out, uint32_t s) {
  uint32_t acc[8];
  uint32_t a = threadIdx.x * 2654435761u + s;
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++)
      asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(a));
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void __launch_bounds__(256) k_addc(uint32_t* out, uint32_t s) {
  uint32_t acc[8];
  uint32_t a = threadIdx.x * 2654435761u + s;
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++)
      asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(acc[i]) : "v"(a) : "vcc");
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void __launch_bounds__(256) k_u24(uint32_t* out, uint32_t s) {
  uint32_t acc[8];
  uint32_t a = (threadIdx.x * 2654435761u + s) & 0xffffff;
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++)
      asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(acc[i]) : "v"(a));
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void __launch_bounds__(256) k_fma64(uint32_t* out, uint32_t s) {
  double acc[8];
  double a = 1.0000001 + threadIdx.x * 1e-9 + s * 1e-12, b = 0.9999999;
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++)
      asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(acc[i]) : "v"(a), "v"(b));
  }
  double r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r);
}

__global__ void __launch_bounds__(256) k_fma32(uint32_t* out, uint32_t s) {
  float acc[8];
  float a = 1.0000001f + threadIdx.x * 1e-9f + s * 1e-12f, b = 0.9999999f;
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++)
      asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(acc[i]) : "v"(a), "v"(b));
  }
  float r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(r);
}


__global__ void __launch_bounds__(256) k_mad64_s(uint32_t* out, uint32_t s) {
  uint64_t acc[8];
  uint32_t a = threadIdx.x * 2654435761u + s, b = a ^ 0x9e3779b9u;
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      uint64_t cc;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[i]), "=s"(cc) : "v"(a), "v"(b));
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r ^= (uint32_t)acc[i] ^ (uint32_t)(acc[i] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void __launch_bounds__(256) k_mad64_addc_s(uint32_t* out, uint32_t s) {
  uint64_t acc[8];
  uint32_t c2[8];
  uint32_t a = threadIdx.x * 2654435761u + s, b = a ^ 0x9e3779b9u;
#pragma unroll
  for (int i = 0; i < 8; i++) { acc[i] = a + i; c2[i] = 0; }
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      uint64_t cc, cc2;
      asm volatile("v_mad_u64_u32 %0, %2, %4, %5, %0\n\tv_addc_co_u32_e64 %1, %3, 0, %1, %2"
                   : "+v"(acc[i]), "+v"(c2[i]), "=&s"(cc), "=s"(cc2) : "v"(a), "v"(b));
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r ^= (uint32_t)acc[i] ^ (uint32_t)(acc[i] >> 32) ^ c2[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void __launch_bounds__(256) k_addc_s(uint32_t* out, uint32_t s) {
  uint32_t acc[8];
  uint32_t a = threadIdx.x * 2654435761u + s;
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      uint64_t cc, cc2;
      asm volatile("v_add_co_u32_e64 %0, %1, %0, %3\n\tv_addc_co_u32_e64 %0, %2, %0, %3, %1" : "+v"(acc[i]), "=&s"(cc), "=s"(cc2) : "v"(a));
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void __launch_bounds__(256) k_add32(uint32_t* out, uint32_t s) {
  uint32_t acc[8];
  uint32_t a = threadIdx.x * 2654435761u + s;
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++)
      asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(a));
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void __launch_bounds__(256) k_add64(uint32_t* out, uint32_t s) {
  uint64_t acc[8];
  uint64_t a = threadIdx.x * 2654435761u + s;
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++)
      asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[i]) : "v"(a));
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r ^= (uint32_t)acc[i] ^ (uint32_t)(acc[i] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

typedef void (*kfn)(uint32_t*, uint32_t);

static int run(const char* name, kfn f, double ops_per_iter_per_lane, uint32_t* d) {
  int blocks = 256 * 8, threads = 256;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; r++) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(f, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)r);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  double lane_ops = (double)blocks * threads * ITERS * 8 * ops_per_iter_per_lane;
  double rate = lane_ops / (best * 1e-3);
  // cycles per wave64 instruction per SIMD at 2.4 GHz: 1024 SIMDs * 64 lanes
  double cyc = 1024.0 * 64 * 2.4e9 / rate;
  printf("{\"op\": \"%s\", \"lane_ops_per_s\": %.4e, \"ms\": %.3f, \"cyc_per_wave_instr_at_2.4GHz\": %.2f}\n", name, rate, best, cyc);
  return 0;
}

int main() {
  uint32_t* d;
  CHECK(hipMalloc(&d, 256 * 8 * 256 * 4));
  run("v_fma_f32", k_fma32, 1, d);
  run("v_add_u32", k_add32, 1, d);
  run("v_mad_u64_u32(vcc)", k_mad64, 1, d);
  run("v_mad_u64_u32(sgpr carry)", k_mad64_s, 1, d);
  run("v_mad_u64_u32+v_addc_co_u32(pair, sgpr carry)", k_mad64_addc_s, 1, d);
  run("v_add_co_u32+v_addc_co_u32(pair, sgpr carry)", k_addc_s, 1, d);
  run("v_lshl_add_u64", k_add64, 1, d);
  run("v_mad_u64_u32+v_addc_co_u32(pair)", k_mad64_addc, 1, d);
  run("v_mul_lo_u32", k_mullo, 1, d);
  run("v_mul_hi_u32", k_mulhi, 1, d);
  run("v_add_co_u32+v_addc_co_u32(pair)", k_addc, 1, d);
  run("v_mad_u32_u24", k_u24, 1, d);
  run("v_fma_f64", k_fma64, 1, d);
  run("v_fma_f32", k_fma32, 1, d);
  CHECK(hipFree(d));
  return 0;
}
