// FP32 VALU FMA throughput on gfx950: what a register-resident fmaf loop sustains at 1, 2 and 4 waves per SIMD,
// scalar v_fmac_f32 vs packed v_pk_fma_f32 (the ceiling for the VQ distance kernel).
// build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/probe/valu_fma_probe.hip -o /tmp/valu_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int NACC>
__global__ void fma_scalar(float* out, int iters, float a, float b) {
  float acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = threadIdx.x * 1e-3f + i;
  float x = a + threadIdx.x * 1e-7f, y = b;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = fmaf(x, y, acc[i]);
    x = __builtin_amdgcn_readfirstlane(__float_as_uint(x)) ? x : y;  // keep x live, loop-carried
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NACC>
__global__ void fma_packed(float* out, int iters, float a, float b) {
  f2 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = f2{threadIdx.x * 1e-3f + i, (float)i};
  f2 x = f2{a + threadIdx.x * 1e-7f, a}, y = f2{b, b};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_elementwise_fma(x, y, acc[i]);
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i].x + acc[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
void run(const char* name, K kern, int threads, int blocks, int lds_bytes, double fma_per_thread_iter, int iters) {
  float* out;
  hipMalloc(&out, (size_t)blocks * threads * 4);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), lds_bytes, 0, out, iters, 1.0001f, 0.9999f);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r)
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), lds_bytes, 0, out, iters, 1.0001f, 0.9999f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  const double flop = 2.0 * fma_per_thread_iter * iters * threads * (double)blocks;
  printf("%-34s threads %4d blocks %5d: %8.3f ms  %7.1f TFLOP/s\n", name, threads, blocks, ms, flop / ms / 1e9);
  hipFree(out);
}

int main() {
  const int iters = 20000;
  // 1 workgroup per CU forced by 96 KB of dynamic LDS; waves per SIMD = threads / 256
  for (int th : {256, 512, 1024}) {
    run("scalar v_fmac, 32 acc", fma_scalar<32>, th, 256, 96 * 1024, 32, iters);
    run("packed v_pk_fma, 16 acc (32 fma)", fma_packed<16>, th, 256, 96 * 1024, 32, iters);
  }
  run("scalar v_fmac, 32 acc, 8 WG/CU", fma_scalar<32>, 256, 2048, 0, 32, iters);
  run("packed v_pk_fma, 16 acc, 8 WG/CU", fma_packed<16>, 256, 2048, 0, 32, iters);
  return 0;
}
