// BatchNorm1d inside the VQ-VAE ResBlocks (`--batchnorm 1`, model/vq_vae_patch_embedd.py:60-74):
//   GELU -> Conv -> BN -> GELU -> Conv -> BN -> Dropout, plus the residual.
// Activations are token-major [N rows][H channels].  Statistics are per (group, channel) with group = row % G:
// the decoder normalises over all rows (G = 1, n = B*S); the encoder runs its ResBlocks on every token slice
// separately (CNNBlock(seperate=True), :104-110), so each of the S token positions has its own batch statistics
// (G = S, n = B) and every forward moves the running statistics S times, in token order.
// The convolutions stay on aw_gemm (plain bias epilogue, f32 pre-BN output); these kernels do the statistics,
// the normalise(+GELU / +dropout+residual) passes and the two-pass BatchNorm backward.
#include "common.h"

namespace {

constexpr int BN_ROWS = 64;   // rows of one group per statistics block

// sums[0][g][c] += sum h, sums[1][g][c] += sum h^2 over rows r = g + G*k
__global__ __launch_bounds__(256) void bn_stats_kernel(const float* __restrict__ h, int64_t N, int H, int G,
                                                       double* __restrict__ sums) {
  const int g = blockIdx.y;
  const int64_t per = (N - g + G - 1) / G;          // rows of group g
  const int64_t k0 = (int64_t)blockIdx.x * BN_ROWS, k1 = min(per, k0 + BN_ROWS);
  for (int c = threadIdx.x; c < H; c += blockDim.x) {
    float s = 0.f, q = 0.f;
    for (int64_t k = k0; k < k1; ++k) {
      const float v = h[(g + k * G) * H + c];
      s += v;
      q = fmaf(v, v, q);
    }
    if (k1 > k0) {
      atomicAdd(sums + (int64_t)g * H + c, (double)s);
      atomicAdd(sums + ((int64_t)G + g) * H + c, (double)q);
    }
  }
}

// stats [4][G][H]: mean, invstd, gamma, beta.  Training: batch statistics per group (biased variance), running
// statistics updated once per group in group order with the unbiased variance (torch BatchNorm1d), nbt += G.
__global__ void bn_finalize_groups_kernel(const double* __restrict__ sums, int64_t n, int H, int G,
                                          const float* gamma, const float* beta, float* rm, float* rv, int64_t* nbt,
                                          float eps, float mom, int training, float* __restrict__ stats) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= H) return;
  const int64_t GH = (int64_t)G * H;
  for (int g = 0; g < G; ++g) {
    float mean, invstd;
    if (training) {
      const double m = sums[(int64_t)g * H + c] / (double)n;
      double var = sums[GH + (int64_t)g * H + c] / (double)n - m * m;
      if (var < 0) var = 0;
      mean = (float)m;
      invstd = (float)(1.0 / sqrt(var + (double)eps));
      if (rm) rm[c] = (1.f - mom) * rm[c] + mom * mean;
      if (rv) rv[c] = (1.f - mom) * rv[c] + mom * (float)(var * (double)n / (double)(n > 1 ? n - 1 : 1));
    } else {
      mean = rm[c];
      invstd = 1.0f / sqrtf(rv[c] + eps);
    }
    stats[(int64_t)g * H + c] = mean;
    stats[GH + (int64_t)g * H + c] = invstd;
    stats[2 * GH + (int64_t)g * H + c] = gamma ? gamma[c] : 1.f;
    stats[3 * GH + (int64_t)g * H + c] = beta ? beta[c] : 0.f;
  }
  if (training && c == 0 && nbt) nbt[0] += G;
}

template <typename TO>
__device__ __forceinline__ float op_gelu(float x) {
  return sizeof(TO) == 2 ? gelu_erf_fast(x) : gelu_erf(x);   // as the GEMM epilogues of the same operand dtype
}

// mode 0: out = BN(h), op = GELU(out).   mode 1: out = resid + drop(BN(h)), op = GELU(out) (op may be NULL).
// mode 2: as mode 1 with op = out (the last block's output feeds a conv directly, without GELU)
template <typename TO>
__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ h, int64_t N, int H, int G,
                                                       const float* __restrict__ st, int mode,
                                                       const float* __restrict__ resid, float p, uint64_t seed,
                                                       const uint64_t* __restrict__ seed_ptr, float* __restrict__ out,
                                                       TO* __restrict__ op) {
  const uint64_t ds = aw_seed_mix(seed, seed_ptr);
  const int64_t GH = (int64_t)G * H, total = N * H;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / H;
    const int c = (int)(e - r * H);
    const int64_t gi = (r % G) * H + c;
    float v = (h[e] - st[gi]) * st[GH + gi] * st[2 * GH + gi] + st[3 * GH + gi];
    if (mode != 0) v = resid[e] + v * aw_dropout_scale(ds, (uint64_t)e, p);
    out[e] = v;
    if (op) op[e] = from_f32<TO>(mode == 2 ? v : op_gelu<TO>(v));
  }
}

// sums[0][g][c] += sum t, sums[1][g][c] += sum t * xhat, t = g_in * dropout mask
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const float* __restrict__ h, int64_t N, int H, int G,
                                                            const float* __restrict__ st,
                                                            const float* __restrict__ gin, float p, uint64_t seed,
                                                            const uint64_t* __restrict__ seed_ptr,
                                                            double* __restrict__ sums) {
  const uint64_t ds = aw_seed_mix(seed, seed_ptr);
  const int g = blockIdx.y;
  const int64_t GH = (int64_t)G * H;
  const int64_t per = (N - g + G - 1) / G;
  const int64_t k0 = (int64_t)blockIdx.x * BN_ROWS, k1 = min(per, k0 + BN_ROWS);
  for (int c = threadIdx.x; c < H; c += blockDim.x) {
    const int64_t gi = (int64_t)g * H + c;
    const float mean = st[gi], inv = st[GH + gi];
    float s = 0.f, q = 0.f;
    for (int64_t k = k0; k < k1; ++k) {
      const int64_t e = (g + k * G) * H + c;
      const float t = gin[e] * aw_dropout_scale(ds, (uint64_t)e, p);
      s += t;
      q = fmaf(t, (h[e] - mean) * inv, q);
    }
    if (k1 > k0) {
      atomicAdd(sums + gi, (double)s);
      atomicAdd(sums + GH + gi, (double)q);
    }
  }
}

// dh = gamma*invstd*(t - S1/n - xhat*S2/n) (training) or gamma*invstd*t (eval); the first block also adds the
// BN parameter gradients dgamma += sum_g S2, dbeta += sum_g S1
template <typename TO>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float* __restrict__ h, int64_t N, int H, int G,
                                                           const float* __restrict__ st,
                                                           const float* __restrict__ gin, float p, uint64_t seed,
                                                           const uint64_t* __restrict__ seed_ptr,
                                                           const double* __restrict__ sums, int64_t n, int training,
                                                           TO* __restrict__ dh, float* __restrict__ dgamma,
                                                           float* __restrict__ dbeta) {
  const uint64_t ds = aw_seed_mix(seed, seed_ptr);
  const int64_t GH = (int64_t)G * H, total = N * H;
  if (blockIdx.x == 0) {
    for (int c = threadIdx.x; c < H; c += blockDim.x) {
      double a = 0.0, b = 0.0;
      for (int g = 0; g < G; ++g) {
        a += sums[GH + (int64_t)g * H + c];
        b += sums[(int64_t)g * H + c];
      }
      if (dgamma) dgamma[c] += (float)a;
      if (dbeta) dbeta[c] += (float)b;
    }
  }
  const float invn = 1.0f / (float)n;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / H;
    const int c = (int)(e - r * H);
    const int64_t gi = (r % G) * H + c;
    const float inv = st[GH + gi];
    const float t = gin[e] * aw_dropout_scale(ds, (uint64_t)e, p);
    float v;
    if (training) {
      const float xh = (h[e] - st[gi]) * inv;
      v = st[2 * GH + gi] * inv * (t - (float)sums[gi] * invn - xh * (float)sums[GH + gi] * invn);
    } else {
      v = st[2 * GH + gi] * inv * t;
    }
    dh[e] = from_f32<TO>(v);
  }
}

int grid_elems(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" int aw_bn_group_stats(const float* h, int64_t N, int H, int G, double* sums, void* stream) {
  AW_REQUIRE(h && sums && N >= 0 && H > 0 && G > 0, "aw_bn_group_stats: bad args");
  if (N == 0) return AW_OK;
  const int64_t per = (N + G - 1) / G;
  dim3 grid((unsigned)((per + BN_ROWS - 1) / BN_ROWS), (unsigned)G);
  hipLaunchKernelGGL(bn_stats_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), h, N, H, G, sums);
  return aw::check_launch("aw_bn_group_stats");
}

extern "C" int aw_bn_group_finalize(const double* sums, int64_t n, int H, int G, const float* gamma,
                                    const float* beta, float* running_mean, float* running_var, int64_t* nbt,
                                    float eps, float momentum, int training, float* stats, void* stream) {
  AW_REQUIRE(stats && H > 0 && G > 0, "aw_bn_group_finalize: bad args");
  AW_REQUIRE(!training || sums, "aw_bn_group_finalize: training needs the sums");
  // torch.nn.BatchNorm1d in training mode refuses a batch of one value per channel (nn.functional.batch_norm:
  // "Expected more than 1 value per channel when training"); a zero variance would silently collapse to beta
  AW_REQUIRE(!training || n > 1, "Expected more than 1 value per channel when training, got %lld per group",
             (long long)n);
  AW_REQUIRE(training || (running_mean && running_var), "aw_bn_group_finalize: eval needs running statistics");
  hipLaunchKernelGGL(bn_finalize_groups_kernel, dim3(aw_cdiv(H, 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), sums, n, H, G, gamma, beta, running_mean, running_var,
                     nbt, eps, momentum, training, stats);
  return aw::check_launch("aw_bn_group_finalize");
}

extern "C" int aw_bn_apply(const float* h, int64_t N, int H, int G, const float* stats, int mode,
                           const float* resid, float drop_p, uint64_t drop_seed, const uint64_t* seed_ptr,
                           float* out, void* op, int op_dtype, void* stream) {
  AW_REQUIRE(h && stats && out && N >= 0 && H > 0 && G > 0 && mode >= 0 && mode <= 2 && (mode == 0 || resid),
             "aw_bn_apply: bad args");
  if (N == 0) return AW_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (op_dtype == AW_BF16)
    hipLaunchKernelGGL(bn_apply_kernel<bf16>, dim3(grid_elems(N * H)), dim3(256), 0, s, h, N, H, G, stats, mode,
                       resid, drop_p, drop_seed, reinterpret_cast<const uint64_t*>(seed_ptr), out, (bf16*)op);
  else
    hipLaunchKernelGGL(bn_apply_kernel<float>, dim3(grid_elems(N * H)), dim3(256), 0, s, h, N, H, G, stats, mode,
                       resid, drop_p, drop_seed, reinterpret_cast<const uint64_t*>(seed_ptr), out, (float*)op);
  return aw::check_launch("aw_bn_apply");
}

extern "C" int aw_bn_bwd_reduce(const float* h, int64_t N, int H, int G, const float* stats, const float* g_in,
                                float drop_p, uint64_t drop_seed, const uint64_t* seed_ptr, double* sums,
                                void* stream) {
  AW_REQUIRE(h && stats && g_in && sums && N >= 0 && H > 0 && G > 0, "aw_bn_bwd_reduce: bad args");
  if (N == 0) return AW_OK;
  const int64_t per = (N + G - 1) / G;
  dim3 grid((unsigned)((per + BN_ROWS - 1) / BN_ROWS), (unsigned)G);
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), h, N, H, G,
                     stats, g_in, drop_p, drop_seed, seed_ptr, sums);
  return aw::check_launch("aw_bn_bwd_reduce");
}

extern "C" int aw_bn_bwd_apply(const float* h, int64_t N, int H, int G, const float* stats, const float* g_in,
                               float drop_p, uint64_t drop_seed, const uint64_t* seed_ptr, const double* sums,
                               int64_t n, int training, void* dh, int dh_dtype, float* dgamma, float* dbeta,
                               void* stream) {
  AW_REQUIRE(h && stats && g_in && sums && dh && N >= 0 && H > 0 && G > 0 && n > 0, "aw_bn_bwd_apply: bad args");
  if (N == 0) return AW_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dh_dtype == AW_BF16)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<bf16>, dim3(grid_elems(N * H)), dim3(256), 0, s, h, N, H, G, stats, g_in,
                       drop_p, drop_seed, seed_ptr, sums, n, training, (bf16*)dh, dgamma, dbeta);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<float>, dim3(grid_elems(N * H)), dim3(256), 0, s, h, N, H, G, stats,
                       g_in, drop_p, drop_seed, seed_ptr, sums, n, training, (float*)dh, dgamma, dbeta);
  return aw::check_launch("aw_bn_bwd_apply");
}
