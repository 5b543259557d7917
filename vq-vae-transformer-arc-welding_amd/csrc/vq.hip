// Vector quantizer (model/vector_quantizer.py:59-131) for gfx950.
//
// Forward: one workgroup = 64 rows (one row per lane, the row held in VGPRs) x 4 waves that split the codes.
// The codebook is staged through LDS in 64 KiB tiles (K=512 x D=64 is two tiles) and read as wave-uniform
// float4 broadcasts.  Distances follow the reference expression exactly in fp32:
//     d_k = fl( fl(|z|^2 + |e_k|^2) - 2 * dot(z, e_k) ),  dot = k-ordered fmaf chain over the embedding dim
// (torch's CPU sgemm on this shape is bit-identical to that chain -- measured), so the
// argmin (lexicographic (d, k) minimum == torch.argmin first-index tie rule) is bit-exact.
// No MFMA: the work is 1 MFLOP/window, dominated by staging, not arithmetic.
#include "common.h"

namespace {

constexpr int VQ_THREADS = 256;
constexpr int VQ_ROWS = 64;

template <int D>
__global__ __launch_bounds__(VQ_THREADS) void vq_fwd_kernel(const float* __restrict__ z, const float* __restrict__ E,
                                                            int64_t N, int K, float* __restrict__ zq,
                                                            int64_t* __restrict__ idx, float* __restrict__ counts,
                                                            double* __restrict__ sqerr) {
  constexpr int KT = 16384 / D;  // codes per 64 KiB LDS tile
  __shared__ __attribute__((aligned(16))) float Es[KT * D];
  __shared__ float ee[KT];
  __shared__ float bd[4][VQ_ROWS];
  __shared__ int bk[4][VQ_ROWS];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t row = (int64_t)blockIdx.x * VQ_ROWS + lane;
  const bool valid = row < N;

  float zr[D];
  {
    const float4* zp = reinterpret_cast<const float4*>(z + (valid ? row : 0) * D);
#pragma unroll
    for (int q = 0; q < D / 4; ++q) {
      float4 v = valid ? zp[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      zr[4 * q + 0] = v.x;
      zr[4 * q + 1] = v.y;
      zr[4 * q + 2] = v.z;
      zr[4 * q + 3] = v.w;
    }
  }
  float zz = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) zz = __fadd_rn(zz, __fmul_rn(zr[d], zr[d]));

  float best = __builtin_huge_valf();
  int bestk = 0x7fffffff;
  for (int t0 = 0; t0 < K; t0 += KT) {
    const int kt = min(KT, K - t0);
    __syncthreads();
    const float4* src = reinterpret_cast<const float4*>(E + (int64_t)t0 * D);
    {
      // all of this thread's tile loads first, then the LDS stores: a load -> store loop paid one L2 round trip
      // per float4 (16 in a row per tile)
      constexpr int PER = KT * D / 4 / VQ_THREADS;
      const int n4 = kt * D / 4;
      float4 tmp[PER];
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int i = tid + u * VQ_THREADS;
        tmp[u] = i < n4 ? src[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int i = tid + u * VQ_THREADS;
        if (i < n4) reinterpret_cast<float4*>(Es)[i] = tmp[u];
      }
    }
    for (int c = tid; c < kt; c += VQ_THREADS) {  // |e_k|^2 from global (L2) rows: avoids strided LDS reads
      const float4* ep = reinterpret_cast<const float4*>(E + (int64_t)(t0 + c) * D);
      float s = 0.f;
#pragma unroll 4
      for (int q = 0; q < D / 4; ++q) {
        float4 v = ep[q];
        s = __fadd_rn(s, __fmul_rn(v.x, v.x));
        s = __fadd_rn(s, __fmul_rn(v.y, v.y));
        s = __fadd_rn(s, __fmul_rn(v.z, v.z));
        s = __fadd_rn(s, __fmul_rn(v.w, v.w));
      }
      ee[c] = s;
    }
    __syncthreads();
    const int per = (kt + 3) / 4;
    const int kb = wid * per, ke = min(kt, kb + per);
    // four codes per iteration: four independent in-order fmaf chains (each chain is the reference's dot
    // product bit for bit; the chains only interleave to hide the fma latency), compared in code order
    int k = kb;
    constexpr int NC = D <= 64 ? 4 : 1;   // wide embeddings: the row itself fills the register file
    for (; NC == 4 && k + 4 <= ke; k += 4) {
      const float4* e0 = reinterpret_cast<const float4*>(Es + k * D);
      float dt[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < D / 4; ++q) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float4 e = e0[c * (D / 4) + q];
          dt[c] = fmaf(zr[4 * q + 0], e.x, dt[c]);
          dt[c] = fmaf(zr[4 * q + 1], e.y, dt[c]);
          dt[c] = fmaf(zr[4 * q + 2], e.z, dt[c]);
          dt[c] = fmaf(zr[4 * q + 3], e.w, dt[c]);
        }
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float dist = __fsub_rn(__fadd_rn(zz, ee[k + c]), __fmul_rn(2.f, dt[c]));
        const int gk = t0 + k + c;
        if (dist < best || (dist == best && gk < bestk)) {
          best = dist;
          bestk = gk;
        }
      }
    }
    for (; k < ke; ++k) {
      const float4* e4 = reinterpret_cast<const float4*>(Es + k * D);
      float dot = 0.f;
#pragma unroll
      for (int q = 0; q < D / 4; ++q) {
        const float4 e = e4[q];
        dot = fmaf(zr[4 * q + 0], e.x, dot);
        dot = fmaf(zr[4 * q + 1], e.y, dot);
        dot = fmaf(zr[4 * q + 2], e.z, dot);
        dot = fmaf(zr[4 * q + 3], e.w, dot);
      }
      const float dist = __fsub_rn(__fadd_rn(zz, ee[k]), __fmul_rn(2.f, dot));
      const int gk = t0 + k;
      if (dist < best || (dist == best && gk < bestk)) {
        best = dist;
        bestk = gk;
      }
    }
  }
  bd[wid][lane] = best;
  bk[wid][lane] = bestk;
  __syncthreads();
  if (wid != 0) return;
#pragma unroll
  for (int w = 1; w < 4; ++w) {
    const float d = bd[w][lane];
    const int k = bk[w][lane];
    if (d < best || (d == best && k < bestk)) {
      best = d;
      bestk = k;
    }
  }
  double se = 0.0;
  if (valid) {
    if (bestk < 0 || bestk >= K) bestk = 0;  // all-NaN row guard (torch would return the NaN position)
    idx[row] = bestk;
    atomicAdd(counts + bestk, 1.0f);
    const float4* ep = reinterpret_cast<const float4*>(E + (int64_t)bestk * D);
    float4* op = reinterpret_cast<float4*>(zq + row * D);
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < D / 4; ++q) {
      const float4 e = ep[q];
      float4 o;
      float d0 = __fsub_rn(e.x, zr[4 * q + 0]), d1 = __fsub_rn(e.y, zr[4 * q + 1]);
      float d2 = __fsub_rn(e.z, zr[4 * q + 2]), d3 = __fsub_rn(e.w, zr[4 * q + 3]);
      o.x = __fadd_rn(zr[4 * q + 0], d0);  // z + (z_q - z).detach()
      o.y = __fadd_rn(zr[4 * q + 1], d1);
      o.z = __fadd_rn(zr[4 * q + 2], d2);
      o.w = __fadd_rn(zr[4 * q + 3], d3);
      op[q] = o;
      s += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
    }
    se = s;
  }
  se = wave_sum_d(se);
  if (lane == 0) atomicAdd(sqerr, se);
}

__global__ void vq_finalize_kernel(const float* counts, const double* sqerr, int64_t N, int K, int D, float beta,
                                   float* loss, float* perp) {
  __shared__ float part[256];
  const float invN = 1.0f / (float)N;
  float s = 0.f;
  for (int k = threadIdx.x; k < K; k += 256) {
    const float p = counts[k] * invN;
    s += p * logf(p + 1e-10f);
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float m = (float)(sqerr[0] / ((double)N * (double)D));
    loss[0] = m + beta * m;
    perp[0] = expf(-part[0]);
  }
}

__global__ void vq_bwd_kernel(const float* __restrict__ z, const float* __restrict__ E, const int64_t* __restrict__ idx,
                              const float* __restrict__ g_zq, const float* __restrict__ g_loss, int64_t N, int D,
                              float beta, float* __restrict__ dz, float* __restrict__ dE) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * D) return;
  const int64_t r = i / D;
  const int d = (int)(i - r * D);
  const int64_t k = idx[r];
  const float g = g_loss ? g_loss[0] : 0.f;
  const float scale = 2.0f / (float)((double)N * (double)D);
  const float diff = E[k * D + d] - z[i];  // z_q - z
  dz[i] = (g_zq ? g_zq[i] : 0.f) - g * scale * diff;
  if (g != 0.f) atomicAdd(dE + k * D + d, g * beta * scale * diff);
}

__global__ void vq_onehot_kernel(const int64_t* idx, int64_t N, int K, float* onehot) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * (int64_t)K) return;
  const int64_t r = i / K;
  onehot[i] = (idx[r] == (i - r * K)) ? 1.f : 0.f;
}

__global__ void vq_gather_kernel(const float* E, const int64_t* idx, int64_t N, int D, float* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * D) return;
  const int64_t r = i / D;
  out[i] = E[idx[r] * D + (i - r * D)];
}

}  // namespace

extern "C" int aw_vq_forward(const float* z, const float* E, int64_t N, int K, int D, float* zq, int64_t* idx,
                             float* counts, double* sqerr, void* stream) {
  AW_REQUIRE(z && E && zq && idx && counts && sqerr, "aw_vq_forward: null pointer");
  AW_REQUIRE(N >= 0 && K > 0, "aw_vq_forward: bad N/K");
  AW_REQUIRE(((uintptr_t)z % 16) == 0 && ((uintptr_t)E % 16) == 0 && ((uintptr_t)zq % 16) == 0,
             "aw_vq_forward: z/E/zq must be 16-B aligned");
  if (N == 0) return AW_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(aw_cdiv(N, VQ_ROWS));
  switch (D) {
    case 16: hipLaunchKernelGGL(vq_fwd_kernel<16>, grid, dim3(VQ_THREADS), 0, s, z, E, N, K, zq, idx, counts, sqerr); break;
    case 32: hipLaunchKernelGGL(vq_fwd_kernel<32>, grid, dim3(VQ_THREADS), 0, s, z, E, N, K, zq, idx, counts, sqerr); break;
    case 64: hipLaunchKernelGGL(vq_fwd_kernel<64>, grid, dim3(VQ_THREADS), 0, s, z, E, N, K, zq, idx, counts, sqerr); break;
    case 128: hipLaunchKernelGGL(vq_fwd_kernel<128>, grid, dim3(VQ_THREADS), 0, s, z, E, N, K, zq, idx, counts, sqerr); break;
    case 256: hipLaunchKernelGGL(vq_fwd_kernel<256>, grid, dim3(VQ_THREADS), 0, s, z, E, N, K, zq, idx, counts, sqerr); break;
    default: aw::set_error("aw_vq_forward: unsupported embedding dim %d (16/32/64/128/256)", D); return AW_ERR_ARG;
  }
  return aw::check_launch("aw_vq_forward");
}

extern "C" int aw_vq_finalize(const float* counts, const double* sqerr, int64_t N, int K, int D, float beta,
                              float* loss, float* perplexity, void* stream) {
  AW_REQUIRE(counts && sqerr && loss && perplexity && N > 0 && K > 0 && D > 0, "aw_vq_finalize: bad args");
  hipLaunchKernelGGL(vq_finalize_kernel, dim3(1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), counts, sqerr,
                     N, K, D, beta, loss, perplexity);
  return aw::check_launch("aw_vq_finalize");
}

extern "C" int aw_vq_backward(const float* z, const float* E, const int64_t* idx, const float* g_zq,
                              const float* g_loss, int64_t N, int K, int D, float beta, float* dz, float* dE,
                              void* stream) {
  AW_REQUIRE(z && E && idx && dz && dE && N >= 0 && K > 0 && D > 0, "aw_vq_backward: bad args");
  if (N == 0) return AW_OK;
  const int64_t n = N * D;
  hipLaunchKernelGGL(vq_bwd_kernel, dim3(aw_cdiv(n, 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), z,
                     E, idx, g_zq, g_loss, N, D, beta, dz, dE);
  return aw::check_launch("aw_vq_backward");
}

extern "C" int aw_vq_onehot(const int64_t* idx, int64_t N, int K, float* onehot, void* stream) {
  AW_REQUIRE(idx && onehot && N >= 0 && K > 0, "aw_vq_onehot: bad args");
  if (N == 0) return AW_OK;
  const int64_t n = N * (int64_t)K;
  hipLaunchKernelGGL(vq_onehot_kernel, dim3(aw_cdiv(n, 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), idx,
                     N, K, onehot);
  return aw::check_launch("aw_vq_onehot");
}

extern "C" int aw_vq_gather(const float* E, const int64_t* idx, int64_t N, int D, float* out, void* stream) {
  AW_REQUIRE(E && idx && out && N >= 0 && D > 0, "aw_vq_gather: bad args");
  if (N == 0) return AW_OK;
  const int64_t n = N * D;
  hipLaunchKernelGGL(vq_gather_kernel, dim3(aw_cdiv(n, 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), E,
                     idx, N, D, out);
  return aw::check_launch("aw_vq_gather");
}
