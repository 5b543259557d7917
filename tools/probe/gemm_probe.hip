#define AW_GEMM_STAMPS 1
// Standalone timing probe for the GEMM fixed cost (diagnostic only; not part of the library).
// Builds the production gemm.hip into this translation unit and compares it with stripped probe kernels of the
// same grid / LDS footprint.   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/gemm_probe.hip \
//   vq-vae-transformer-arc-welding_amd/csrc/runtime.hip -o tools/bin/gemm_probe
#include "../../vq-vae-transformer-arc-welding_amd/csrc/gemm.hip"
#include "../../vq-vae-transformer-arc-welding_amd/csrc/gemm_fast_fwd.hip"
#include "../../vq-vae-transformer-arc-welding_amd/csrc/gemm_fast_bwd.hip"
#include <vector>
#include <string.h>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

__global__ __launch_bounds__(256, 2) void probe_empty(float* out) {
  __shared__ char smem[67584];
  if (threadIdx.x == 999) { smem[threadIdx.x] = 1; out[0] = smem[blockIdx.x]; }
}
// every block writes its 128x128 f32 tile: thread -> 4 consecutive columns x 16 rows
__global__ __launch_bounds__(256, 2) void probe_store(float* C, int N, int tiles_n) {
  __shared__ char smem[67584];
  const int tid = threadIdx.x;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int c4 = (tid & 31) * 4, r0 = tid >> 5;
  if (tid == 999) smem[tid] = 0;
  for (int lr = r0; lr < 128; lr += 8) {
    float4 v = make_float4(lr, c4, 1.f, 2.f);
    *reinterpret_cast<float4*>(C + (int64_t)(tm * 128 + lr) * N + tn * 128 + c4) = v;
  }
}

__global__ void probe_fill(bf16* x, size_t n, uint32_t seed) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    x[i] = (bf16)(((float)(h & 0xFFFF) / 65536.f - 0.5f) * 2.f);
  }
}

template <typename F> float timeit(F f, int reps = 50) {
  for (int i = 0; i < 5; ++i) f();
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / reps;
}

int main(int argc, char** argv) {
  const int M = 16384, N = 512, Kmax = 2048;
  const bool only_conv = argc > 1 && strcmp(argv[1], "conv") == 0;
  bf16 *A, *B; float* C; bf16* Cb;
  CK(hipMalloc(&A, (size_t)M * Kmax * 2)); CK(hipMalloc(&B, (size_t)N * Kmax * 2));
  CK(hipMalloc(&C, (size_t)M * N * 4)); CK(hipMalloc(&Cb, (size_t)M * N * 2));
  probe_fill<<<1024, 256>>>(A, (size_t)M * Kmax, 1); probe_fill<<<1024, 256>>>(B, (size_t)N * Kmax, 2);
  const int tiles = (M / 128) * (N / 128);
  if (only_conv) {   // PMC target: the decoder forward conv GEMM (K = 3 x 512, bias + GELU operand epilogue)
    bf16* C2; float* bias;
    CK(hipMalloc(&C2, (size_t)M * N * 2)); CK(hipMalloc(&bias, N * 4)); CK(hipMemset(bias, 0, N * 4));
    aw_gemm_args a; memset(&a, 0, sizeof(a));
    a.M = M; a.N = N; a.K = 3 * 512; a.a_dtype = AW_BF16; a.A = A; a.lda = 512; a.B = B; a.ldb = 3 * 512;
    a.conv_cin = 512; a.conv_seg = 16; a.conv_dir = 1; a.conv_operand = 0;
    a.alpha = 1.f; a.C = Cb; a.ldc = N; a.c_dtype = AW_BF16; a.col_mul = 1; a.bias = bias;
    a.C2 = C2; a.ldc2 = N; a.c2_dtype = AW_BF16; a.c2_mode = 1;
    printf("conv fwd K1536 bias + C bf16 + C2 gelu bf16: %.2f us\n", timeit([&] { aw_gemm(&a, 0); }, 50));
    a.C2 = nullptr; a.c2_mode = 0; a.bias = nullptr;
    printf("conv fwd K1536 C bf16 only: %.2f us\n", timeit([&] { aw_gemm(&a, 0); }, 50));
    return 0;
  }
  printf("empty kernel (512 blocks, 66 KiB LDS)     %8.2f us\n", timeit([&] { probe_empty<<<tiles, 256>>>(C); }));
  printf("store-only 128x128 f32 tiles (32 MiB)      %8.2f us\n", timeit([&] { probe_store<<<tiles, 256>>>(C, N, N / 128); }));
  for (int K : {64, 512, 2048}) {
    for (int cd : {AW_F32, AW_BF16}) {
      aw_gemm_args a; memset(&a, 0, sizeof(a));
      a.M = M; a.N = N; a.K = K; a.a_dtype = AW_BF16; a.A = A; a.lda = K; a.B = B; a.ldb = K;
      a.alpha = 1.f; a.C = cd == AW_F32 ? (void*)C : (void*)Cb; a.ldc = N; a.c_dtype = cd; a.col_mul = 1;
      float us = timeit([&] { aw_gemm(&a, 0); });
      printf("aw_gemm M16384 N512 K%-5d C %s          %8.2f us  (%.0f TF)\n", K, cd == AW_F32 ? "f32 " : "bf16", us,
             2.0 * M * N * K / us / 1e6);
    }
  }
  // fixed-cost attribution at K=64: block count (M) and the store phase (C = null)
  for (int Mx : {2048, 4096, 8192, 16384}) {
    for (int st : {1, 0}) {
      aw_gemm_args a; memset(&a, 0, sizeof(a));
      a.M = Mx; a.N = N; a.K = 64; a.a_dtype = AW_BF16; a.A = A; a.lda = 64; a.B = B; a.ldb = 64;
      a.alpha = 1.f; a.C = st ? (void*)C : nullptr; a.ldc = N; a.c_dtype = AW_F32; a.col_mul = 1;
      printf("aw_gemm M%-5d N512 K64 %s  %8.2f us\n", Mx, st ? "C f32    " : "no store ", timeit([&] { aw_gemm(&a, 0); }));
    }
  }
  {
    float* bias; float* pre; bf16* C2;
    CK(hipMalloc(&bias, N * 4)); CK(hipMalloc(&pre, (size_t)M * N * 4)); CK(hipMalloc(&C2, (size_t)M * N * 2));
    CK(hipMemset(bias, 0, N * 4)); CK(hipMemset(pre, 0, (size_t)M * N * 4));
    for (int v = 0; v < 4; ++v) {
      aw_gemm_args a; memset(&a, 0, sizeof(a));
      a.M = M; a.N = N; a.K = 512; a.a_dtype = AW_BF16; a.A = A; a.lda = 512; a.B = B; a.ldb = 512;
      a.alpha = 1.f; a.C = C; a.ldc = N; a.c_dtype = AW_F32; a.col_mul = 1; a.bias = bias;
      const char* nm = "bias + C f32 + C2 gelu bf16";
      if (v >= 1) { a.C2 = C2; a.ldc2 = N; a.c2_dtype = AW_BF16; a.c2_mode = 1; }
      else nm = "bias + C f32";
      if (v >= 2) { a.resid = pre; a.ld_resid = N; a.drop_p = 0.1f; a.drop_seed = 5; nm = "bias+drop+resid+C+C2 gelu"; }
      if (v == 3) { a.b_trans = 1; a.bias = nullptr; a.drop_p = 0.f; a.pre = pre; a.ld_pre = N; a.c2_mode = 3;
                    a.drop2_p = 0.1f; a.drop2_seed = 3; nm = "bwd: pre'+resid+C+C2 dropcopy"; }
      printf("aw_gemm M16384 N512 K512 %-30s %8.2f us\n", nm, timeit([&] { aw_gemm(&a, 0); }));
    }
  }
  // weight-gradient form: 16 grouped problems of 512x512, K = 16384 tokens
  {
    const int Mw = 512, Nw = 512, Kw = 16384, G = 16;
    bf16 *X; float* Wg;
    CK(hipMalloc(&X, (size_t)Kw * Mw * 2 * 2)); CK(hipMalloc(&Wg, (size_t)G * Mw * Nw * 4 * 3));
    probe_fill<<<1024, 256>>>(X, (size_t)Kw * Mw * 2, 7);
    float* rows; CK(hipMalloc(&rows, G * Mw * 4));
    for (int form = 0; form < 2; ++form) {
      std::vector<aw_gemm_args> v(G);
      for (int g = 0; g < G; ++g) {
        aw_gemm_args& a = v[g]; memset(&a, 0, sizeof(a));
        a.M = Mw; a.N = Nw; a.K = Kw; a.a_dtype = AW_BF16; a.alpha = 1.f; a.c_dtype = AW_F32; a.accumulate = 1;
        a.C = Wg + (size_t)g * Mw * Nw * 3; a.ldc = 3 * Nw; a.col_mul = 3; a.col_off = 1;
        if (form == 0) a.a_rowsum = rows + g * Mw;
        if (form == 0) { a.A = X; a.lda = Mw; a.a_trans = 1; a.B = X + (size_t)Kw * Mw; a.ldb = Nw; a.b_trans = 1; }
        else { a.A = X; a.lda = Kw; a.B = X + (size_t)Kw * Mw; a.ldb = Kw; }
      }
      aw_gemm_set_tile(128);
      float u128 = timeit([&] { aw_gemm_grouped(v.data(), G, 0); }, 10);
      aw_gemm_set_tile(256);
      float u256 = timeit([&] { aw_gemm_grouped(v.data(), G, 0); }, 10);
      aw_gemm_set_tile(0);
      printf("  (forced tile 128: %.2f us, forced 256: %.2f us)\n", u128, u256);
      float us = timeit([&] { aw_gemm_grouped(v.data(), G, 0); }, 10);
      printf("grouped x16 512x512xK16384 %s  %8.2f us  (%.0f TF)\n", form == 0 ? "TT (tokens-major, tr reads)" :
             "NN (K-contiguous)          ", us, 2.0 * G * Mw * Nw * Kw / us / 1e6);
      float us1 = timeit([&] { aw_gemm_grouped(v.data(), 8, 0); }, 10);
      printf("grouped x8  512x512xK16384 %s  %8.2f us  (%.0f TF)\n", form == 0 ? "TT" : "NN", us1,
             2.0 * 8 * Mw * Nw * Kw / us1 / 1e6);
    }
  }
  // power-of-two row strides: transformer-like grouped wgrad M=2048 (A = [K][2048] bf16), N=512, K=16371, 8 groups
  {
    const int Mw = 2048, Nw = 512, Kw = 16371, G = 8;
    for (int pad : {0, 64}) {
      const int lda = Mw + pad, ldb = Nw + pad;
      bf16 *Xa, *Xb; float* Wg; float* rows;
      CK(hipMalloc(&Xa, (size_t)Kw * lda * 2 * G)); CK(hipMalloc(&Xb, (size_t)Kw * ldb * 2 * G));
      CK(hipMalloc(&Wg, (size_t)G * Mw * Nw * 4)); CK(hipMalloc(&rows, (size_t)G * Mw * 4));
      probe_fill<<<1024, 256>>>(Xa, (size_t)Kw * lda * G, 11); probe_fill<<<1024, 256>>>(Xb, (size_t)Kw * ldb * G, 12);
      std::vector<aw_gemm_args> v(G);
      for (int g = 0; g < G; ++g) {
        aw_gemm_args& a = v[g]; memset(&a, 0, sizeof(a));
        a.M = Mw; a.N = Nw; a.K = Kw; a.a_dtype = AW_BF16; a.alpha = 1.f; a.c_dtype = AW_F32; a.accumulate = 1;
        a.A = Xa + (size_t)g * Kw * lda; a.lda = lda; a.a_trans = 1; a.B = Xb + (size_t)g * Kw * ldb; a.ldb = ldb; a.b_trans = 1;
        a.C = Wg + (size_t)g * Mw * Nw; a.ldc = Nw; a.col_mul = 1; a.a_rowsum = rows + g * Mw;
      }
      float us = timeit([&] { aw_gemm_grouped(v.data(), G, 0); }, 10);
      printf("transformer-like grouped wgrad x8 2048x512xK16371 lda pad %2d: %8.2f us (%.0f TF)\n", pad, us,
             2.0 * G * Mw * Nw * Kw / us / 1e6);
      CK(hipFree(Xa)); CK(hipFree(Xb)); CK(hipFree(Wg)); CK(hipFree(rows));
    }
  }
  // tile A/B (aw_gemm_set_tile): 128x128 two-stage vs 256x128 three-stage
  for (int bmv : {128, 256}) {
    aw_gemm_set_tile(bmv);
    for (int K : {512, 1536, 2048}) {
      aw_gemm_args a; memset(&a, 0, sizeof(a));
      a.M = M; a.N = N; a.K = K; a.a_dtype = AW_BF16; a.A = A; a.lda = K; a.B = B; a.ldb = K;
      a.alpha = 1.f; a.C = Cb; a.ldc = N; a.c_dtype = AW_BF16; a.col_mul = 1;
      float us = timeit([&] { aw_gemm(&a, 0); });
      printf("tile %d: M16384 N512 K%-5d C bf16  %8.2f us  (%.0f TF)\n", bmv, K, us, 2.0 * M * N * K / us / 1e6);
    }
  }
  aw_gemm_set_tile(0);
  // phase stamps (s_memrealtime, 10 ns ticks) of one launch
  for (int Kx : {64, 512, 1536}) {
    aw_gemm_args a; memset(&a, 0, sizeof(a));
    a.M = M; a.N = N; a.K = Kx; a.a_dtype = AW_BF16; a.A = A; a.lda = Kx; a.B = B; a.ldb = Kx;
    a.alpha = 1.f; a.C = C; a.ldc = N; a.c_dtype = AW_F32; a.col_mul = 1;
    for (int i = 0; i < 3; ++i) aw_gemm(&a, 0);
    CK(hipDeviceSynchronize());
    std::vector<uint64_t> st(512 * 8);
    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(g_gemm_stamps), st.size() * 8));
    uint64_t t0min = ~0ull, t0max = 0, t4max = 0;
    double ph[4] = {0, 0, 0, 0};
    for (int b = 0; b < 512; ++b) {
      const uint64_t* s = &st[b * 8];
      t0min = std::min(t0min, s[0]); t0max = std::max(t0max, s[0]); t4max = std::max(t4max, s[4]);
      for (int q = 0; q < 4; ++q) ph[q] += (double)(s[q + 1] - s[q]) * 10.0 / 512;
    }
    printf("K%-5d stamps: block-start spread %.2f us, span %.2f us; per-block avg: prologue %.2f  mainloop %.2f  "
           "epi-stage %.2f  epi-store %.2f us\n", Kx, (t0max - t0min) * 0.01, (t4max - t0min) * 0.01, ph[0] / 1000,
           ph[1] / 1000, ph[2] / 1000, ph[3] / 1000);
  }
  return 0;
}
