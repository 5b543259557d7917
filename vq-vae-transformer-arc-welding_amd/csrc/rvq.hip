// Residual VQ with EMA codebooks (ResidualVQLightning, reference model/vector_quantizer.py:9-56, which wraps
// vector-quantize-pytorch's ResidualVQ -> VectorQuantize -> EuclideanCodebook; the library is not installed here, so
// this restates its published algorithm -- parity unpinned).  The nearest-code search is aw_vq_forward
// (csrc/vq.hip) on each layer's residual; these kernels add what the EMA codebook needs around it:
//   * aw_vq_cluster_sums: per-code sums of the assigned rows (the embed_sum of the EMA, and of a k-means step);
//   * aw_kmeans_update:   means <- sums / counts where counts > 0 (k-means init, kmeans_iters Lloyd steps);
//   * aw_rvq_ema_update:  cluster_size / embed_avg EMA, Laplace-smoothed normalisation, dead-code replacement by
//                         batch rows -- all on the device, so a captured training-step graph can replay it;
//   * aw_rvq_residual:    quantized_out += q_i, residual_{i+1} = residual_i - q_i;
//   * aw_rvq_backward:    straight-through + commitment gradient of the whole stack.
// Everything is fp32 and HBM-bound (K x D and N x D streams), with per-code sums by float atomics (L2-resident
// K x D table).
#include "common.h"

namespace {

constexpr int RQ_THREADS = 256;

__global__ __launch_bounds__(RQ_THREADS) void cluster_sums_kernel(const float* __restrict__ z,
                                                                  const int64_t* __restrict__ idx, int64_t N, int D,
                                                                  float* __restrict__ sums) {
  // one thread per 4 consecutive elements of a row (D % 4 == 0)
  const int64_t n4 = N * D / 4;
  const int d4 = D / 4;
  for (int64_t t = (int64_t)blockIdx.x * RQ_THREADS + threadIdx.x; t < n4; t += (int64_t)gridDim.x * RQ_THREADS) {
    const int64_t row = t / d4;
    const int c = (int)(t - row * d4) * 4;
    const float4 v = *reinterpret_cast<const float4*>(z + row * D + c);
    float* dst = sums + idx[row] * D + c;
    atomicAdd(dst + 0, v.x);
    atomicAdd(dst + 1, v.y);
    atomicAdd(dst + 2, v.z);
    atomicAdd(dst + 3, v.w);
  }
}

__global__ __launch_bounds__(RQ_THREADS) void kmeans_update_kernel(float* __restrict__ means,
                                                                   const float* __restrict__ sums,
                                                                   const float* __restrict__ counts, int K, int D,
                                                                   float* __restrict__ avg) {
  const int64_t n = (int64_t)K * D;
  for (int64_t e = (int64_t)blockIdx.x * RQ_THREADS + threadIdx.x; e < n; e += (int64_t)gridDim.x * RQ_THREADS) {
    const float c = counts[e / D];
    float m = means[e];
    if (c > 0.f) m = sums[e] / c;            // empty clusters keep their mean (torch.where(zero_mask, means, new))
    means[e] = m;
    if (avg) avg[e] = m * c;                 // the init's embed_avg = means * bins
  }
}

// Phase 1 (one workgroup): cluster_size EMA, the smoothed sizes the codebook is normalised by, and which codes expire
// and which batch row replaces each of them.  Expired code of rank j (of n_exp) takes a uniformly random row of the
// j-th of n_exp equal strata of the N rows (distinct rows, like the library's randperm(N)[:n_exp]); n_exp > N draws
// rows with replacement (its randint branch).
__global__ __launch_bounds__(1024) void ema_phase1_kernel(float* __restrict__ cs, const float* __restrict__ counts,
                                                          int K, int64_t N, float decay, float eps, float threshold,
                                                          uint64_t salt, const uint64_t* __restrict__ ctr,
                                                          float* __restrict__ smooth, int* __restrict__ sample) {
  __shared__ float red[1024];
  __shared__ int ired[1024];
  const int tid = threadIdx.x;
  float tot = 0.f;
  int nexp = 0;
  for (int k = tid; k < K; k += 1024) {
    const float c = cs[k] * decay + counts[k] * (1.f - decay);
    smooth[k] = c;                              // staged: the EMA'd size
    tot += c;
    nexp += (threshold > 0.f && c < threshold) ? 1 : 0;
  }
  red[tid] = tot;
  ired[tid] = nexp;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if (tid < o) {
      red[tid] += red[tid + o];
      ired[tid] += ired[tid + o];
    }
    __syncthreads();
  }
  const float total = red[0];
  const int n_exp = ired[0];
  __syncthreads();
  const uint64_t seed = ctr ? aw_seed_mix(salt, ctr) : salt;
  // expired ranks in code order: chunked exclusive scan over the 1024 threads
  int base = 0;
  for (int k0 = 0; k0 < K; k0 += 1024) {
    const int k = k0 + tid;
    const float c = k < K ? smooth[k] : 0.f;
    const int ex = (k < K && threshold > 0.f && c < threshold) ? 1 : 0;
    ired[tid] = ex;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {        // Hillis-Steele inclusive scan
      const int v = tid >= o ? ired[tid - o] : 0;
      __syncthreads();
      ired[tid] += v;
      __syncthreads();
    }
    const int rank = base + ired[tid] - ex;
    const int chunk = ired[1023];
    if (k < K) {
      // Laplace smoothing (x + eps) / (sum + K eps) * sum of the EMA'd sizes, before any reset
      smooth[k] = (c + eps) / (total + (float)K * eps) * total;
      int row = -1;
      if (ex) {
        const uint64_t h = aw_hash_group(seed, (uint64_t)rank);
        if ((int64_t)n_exp <= N) {
          const int64_t lo = (int64_t)rank * N / n_exp, hi = (int64_t)(rank + 1) * N / n_exp;
          row = (int)(lo + (int64_t)(h % (uint64_t)(hi - lo)));
        } else {
          row = (int)(h % (uint64_t)N);
        }
      }
      sample[k] = row;
      cs[k] = ex ? threshold : c;               // reset_cluster_size = threshold_ema_dead_code
    }
    base += chunk;
    __syncthreads();
  }
}

// Phase 2 (K x D): embed_avg EMA, embed = embed_avg / smoothed size; expired codes take their batch row
// (embed = row, embed_avg = row * threshold).
__global__ __launch_bounds__(RQ_THREADS) void ema_phase2_kernel(float* __restrict__ embed, float* __restrict__ eavg,
                                                                const float* __restrict__ sums,
                                                                const float* __restrict__ smooth,
                                                                const int* __restrict__ sample,
                                                                const float* __restrict__ z, int K, int D, float decay,
                                                                float threshold) {
  const int64_t n = (int64_t)K * D;
  for (int64_t e = (int64_t)blockIdx.x * RQ_THREADS + threadIdx.x; e < n; e += (int64_t)gridDim.x * RQ_THREADS) {
    const int64_t k = e / D;
    const int d = (int)(e - k * D);
    const int row = sample[k];
    if (row >= 0) {
      const float v = z[(int64_t)row * D + d];
      embed[e] = v;
      eavg[e] = v * threshold;
    } else {
      const float a = eavg[e] * decay + sums[e] * (1.f - decay);
      eavg[e] = a;
      embed[e] = a / smooth[k];
    }
  }
}

__global__ __launch_bounds__(RQ_THREADS) void rvq_residual_kernel(const float* __restrict__ r,
                                                                  const float* __restrict__ zq, int64_t n,
                                                                  float* __restrict__ out, int first,
                                                                  float* __restrict__ r_next) {
  for (int64_t e = (int64_t)blockIdx.x * RQ_THREADS + threadIdx.x; e < n; e += (int64_t)gridDim.x * RQ_THREADS) {
    const float q = zq[e];
    out[e] = first ? q : out[e] + q;
    if (r_next) r_next[e] = r[e] - q;
  }
}

__global__ __launch_bounds__(RQ_THREADS) void rvq_backward_kernel(const float* __restrict__ res,
                                                                  const float* __restrict__ q,
                                                                  const float* __restrict__ gzq,
                                                                  const float* __restrict__ gloss, int nq, int64_t n,
                                                                  float inv_nd, float commit,
                                                                  float* __restrict__ dz) {
  for (int64_t e = (int64_t)blockIdx.x * RQ_THREADS + threadIdx.x; e < n; e += (int64_t)gridDim.x * RQ_THREADS) {
    float g = gzq ? (float)nq * gzq[e] : 0.f;
    for (int i = 0; i < nq; ++i) g += gloss[i] * commit * 2.f * (res[i * n + e] - q[i * n + e]) * inv_nd;
    dz[e] = g;
  }
}

int grid_of(int64_t n) {
  const int64_t g = (n + RQ_THREADS - 1) / RQ_THREADS;
  return (int)(g < 1 ? 1 : (g > 16384 ? 16384 : g));
}

}  // namespace

extern "C" int aw_vq_cluster_sums(const float* z, const int64_t* idx, int64_t N, int K, int D, float* sums,
                                  void* stream) {
  AW_REQUIRE(z && idx && sums && N >= 0 && K > 0 && D > 0 && D % 4 == 0, "aw_vq_cluster_sums: bad args (D %% 4 == 0)");
  AW_REQUIRE(((uintptr_t)z % 16) == 0, "aw_vq_cluster_sums: z must be 16-B aligned");
  if (N == 0) return AW_OK;
  hipLaunchKernelGGL(cluster_sums_kernel, dim3(grid_of(N * D / 4)), dim3(RQ_THREADS), 0,
                     reinterpret_cast<hipStream_t>(stream), z, idx, N, D, sums);
  return aw::check_launch("aw_vq_cluster_sums");
}

extern "C" int aw_kmeans_update(float* means, const float* sums, const float* counts, int K, int D, float* avg,
                                void* stream) {
  AW_REQUIRE(means && sums && counts && K > 0 && D > 0, "aw_kmeans_update: bad args");
  hipLaunchKernelGGL(kmeans_update_kernel, dim3(grid_of((int64_t)K * D)), dim3(RQ_THREADS), 0,
                     reinterpret_cast<hipStream_t>(stream), means, sums, counts, K, D, avg);
  return aw::check_launch("aw_kmeans_update");
}

extern "C" int aw_rvq_ema_update(float* embed, float* embed_avg, float* cluster_size, const float* counts,
                                 const float* sums, const float* z, int64_t N, int K, int D, float decay, float eps,
                                 float threshold, uint64_t salt, const uint64_t* seed_ptr, float* ws, void* stream) {
  AW_REQUIRE(embed && embed_avg && cluster_size && counts && sums && z && ws && N > 0 && K > 0 && D > 0,
             "aw_rvq_ema_update: bad args");
  AW_REQUIRE(decay >= 0.f && decay <= 1.f && eps >= 0.f && threshold >= 0.f, "aw_rvq_ema_update: bad hyper-parameters");
  AW_REQUIRE(N < (int64_t)1 << 31, "aw_rvq_ema_update: N must be < 2^31");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* smooth = ws;
  int* sample = reinterpret_cast<int*>(ws + K);
  hipLaunchKernelGGL(ema_phase1_kernel, dim3(1), dim3(1024), 0, s, cluster_size, counts, K, N, decay, eps, threshold,
                     salt, seed_ptr, smooth, sample);
  hipLaunchKernelGGL(ema_phase2_kernel, dim3(grid_of((int64_t)K * D)), dim3(RQ_THREADS), 0, s, embed, embed_avg, sums,
                     smooth, sample, z, K, D, decay, threshold);
  return aw::check_launch("aw_rvq_ema_update");
}

extern "C" int aw_rvq_residual(const float* r, const float* zq, int64_t n, float* out, int first, float* r_next,
                               void* stream) {
  AW_REQUIRE(r && zq && out && n >= 0, "aw_rvq_residual: bad args");
  if (n == 0) return AW_OK;
  hipLaunchKernelGGL(rvq_residual_kernel, dim3(grid_of(n)), dim3(RQ_THREADS), 0, reinterpret_cast<hipStream_t>(stream),
                     r, zq, n, out, first, r_next);
  return aw::check_launch("aw_rvq_residual");
}

extern "C" int aw_rvq_backward(const float* res, const float* q, const float* g_zq, const float* g_loss, int nq,
                               int64_t N, int D, float commitment, float* dz, void* stream) {
  AW_REQUIRE(res && q && g_loss && dz && nq >= 1 && N >= 0 && D > 0, "aw_rvq_backward: bad args");
  if (N == 0) return AW_OK;
  const int64_t n = N * D;
  hipLaunchKernelGGL(rvq_backward_kernel, dim3(grid_of(n)), dim3(RQ_THREADS), 0, reinterpret_cast<hipStream_t>(stream),
                     res, q, g_zq, g_loss, nq, n, 1.f / (float)n, commitment, dz);
  return aw::check_launch("aw_rvq_backward");
}
