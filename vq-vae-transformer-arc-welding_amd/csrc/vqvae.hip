#include <stdlib.h>
// VQ-VAE-Patch layout and un-patch head kernels (model/vq_vae_patch_embedd.py) for gfx950.
// HBM-bound byte/elementwise work: coalesced float4 traffic, one wave per row where a row reduction is needed.
#include "common.h"
#include <algorithm>

namespace {

// ---------------------------------------------------------------- patchify (vq_vae_patch_embedd.py:13-17)
template <typename T>
__global__ void patchify_kernel(const float* __restrict__ x, int64_t B, int L, int C, int P, T* __restrict__ out,
                                int64_t ldp) {
  const int S = L * C / P;
  const int64_t n = B * S * ldp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t tok = i / ldp;
    const int j = (int)(i - tok * ldp);
    float v = 0.f;
    if (j < P) {
      const int64_t b = tok / S;
      const int t = (int)(tok - b * S);
      const int f = t * P + j;          // channel-major flat index within the window
      const int c = f / L, l = f - c * L;
      v = x[(b * L + l) * C + c];
    }
    out[i] = from_f32<T>(v);
  }
}

// ---------------------------------------------------------------- weight relayouts (+cast)
template <typename T>
__global__ void relayout_kernel(const float* __restrict__ W, int O, int I, int k, int tap, int mode,
                                T* __restrict__ out, int64_t ldo) {
  int64_t n;
  switch (mode) {
    case 0: n = (int64_t)O * I; break;
    case 1: n = (int64_t)O * 3 * I; break;
    case 2: n = (int64_t)3 * O * I; break;
    case 3: n = (int64_t)k * O * I; break;  // W is (I, O, k) here: "O" = out channels of the ConvT
    default: n = (int64_t)O * ldo; break;
  }
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    if (mode == 0) {
      const int64_t o = e / I, i = e - o * I;
      v = W[(o * I + i) * k + tap];
    } else if (mode == 1) {
      const int64_t o = e / (3 * I), r = e - o * 3 * I;
      const int64_t j = r / I, i = r - j * I;
      v = W[(o * I + i) * 3 + j];
    } else if (mode == 2) {
      const int64_t jo = e / I, i = e - jo * I;
      const int64_t j = jo / O, o = jo - j * O;
      v = W[(o * I + i) * 3 + j];
    } else if (mode == 3) {
      const int64_t jo = e / I, i = e - jo * I;
      const int64_t j = jo / O, o = jo - j * O;
      v = W[(i * O + o) * k + j];
    } else {
      const int64_t o = e / ldo, j = e - o * ldo;
      v = j < k ? W[o * k + j] : 0.f;
    }
    out[e] = from_f32<T>(v);
  }
}

// many relayouts in one launch: blockIdx.y = job; jobs travel in the kernel arguments
struct RelayoutJobs {
  aw_relayout_job j[AW_RELAYOUT_MAX_JOBS];
};

__device__ __forceinline__ int64_t relayout_count(const aw_relayout_job& jb) {
  switch (jb.mode) {
    case 0: return (int64_t)jb.O * jb.I;
    case 1: return (int64_t)jb.O * 3 * jb.I;
    case 2: return (int64_t)3 * jb.O * jb.I;
    case 3: return (int64_t)jb.k * jb.O * jb.I;
    case 4: return (int64_t)jb.O * jb.ldo;
    case 7: return (int64_t)3 * jb.O * jb.I;
    default: return (int64_t)jb.O * jb.I;   // 5 (copy), 6 (K-step-major tap)
  }
}

template <typename T>
__global__ __launch_bounds__(256) void relayout_batch_kernel(RelayoutJobs J) {
  // 32-bit unsigned index math (every job is < 2^31 elements, checked on the host): the int64 divisions by
  // runtime extents cost more than the copy itself
  const aw_relayout_job& jb = J.j[blockIdx.y];
  const float* __restrict__ W = jb.W;
  T* __restrict__ out = reinterpret_cast<T*>(jb.out);
  const uint32_t O = jb.O, I = jb.I, k = jb.k, tap = jb.tap, ldo = (uint32_t)jb.ldo;
  const int mode = jb.mode;
  const uint32_t n = (uint32_t)relayout_count(jb);
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
    float v;
    if (mode == 0) {
      const uint32_t o = e / I, i = e - o * I;
      v = W[(o * I + i) * k + tap];
    } else if (mode == 1) {
      const uint32_t o = e / (3 * I), r = e - o * 3 * I;
      const uint32_t j = r / I, i = r - j * I;
      v = W[(o * I + i) * 3 + j];
    } else if (mode == 2) {
      const uint32_t jo = e / I, i = e - jo * I;
      const uint32_t j = jo / O, o = jo - j * O;
      v = W[(o * I + i) * 3 + j];
    } else if (mode == 3) {
      const uint32_t jo = e / I, i = e - jo * I;
      const uint32_t j = jo / O, o = jo - j * O;
      v = W[(i * O + o) * k + j];
    } else if (mode == 4) {
      const uint32_t o = e / ldo, j = e - o * ldo;
      v = j < k ? W[o * k + j] : 0.f;
    } else if (mode == 7) {    // tap-major storage (O, 3, I) -> [3O][I], row j O + o (declare_tap_major)
      const uint32_t jo = e / I, i = e - jo * I;
      const uint32_t j = jo / O, o = jo - j * O;
      v = W[(o * 3 + j) * I + i];
    } else {
      v = W[e];
    }
    out[e] = from_f32<T>(v);
  }
}

__global__ void grad_scatter_kernel(const float* __restrict__ g, int O, int I, int k, int tap, int mode, int64_t ldg,
                                    float* __restrict__ G) {
  int64_t n;
  switch (mode) {
    case 0: n = (int64_t)O * I; break;
    case 1: n = (int64_t)O * 3 * I; break;
    case 3: n = (int64_t)k * O * I; break;
    default: n = (int64_t)O * k; break;
  }
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    if (mode == 0) {
      const int64_t o = e / I, i = e - o * I;
      G[(o * I + i) * k + tap] += g[o * ldg + i];
    } else if (mode == 1) {
      const int64_t o = e / (3 * I), r = e - o * 3 * I;
      const int64_t j = r / I, i = r - j * I;
      G[(o * I + i) * 3 + j] += g[o * ldg + r];
    } else if (mode == 3) {
      const int64_t jo = e / I, i = e - jo * I;
      const int64_t j = jo / O, o = jo - j * O;
      G[(i * O + o) * k + j] += g[jo * ldg + i];
    } else {
      const int64_t o = e / k, j = e - o * k;
      G[o * k + j] += g[o * ldg + j];
    }
  }
}

template <typename T>
__global__ void cast_kernel(const float* __restrict__ in, int64_t n, T* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = from_f32<T>(in[i]);
}

// ---------------------------------------------------------------- BatchNorm finalize
__global__ void bn_finalize_kernel(const double* __restrict__ cs, int64_t n, int H, const float* gamma,
                                   const float* beta, float* rm, float* rv, int64_t* nbt, float eps, float mom,
                                   int training, float* stats) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= H) return;
  float mean, invstd;
  if (training) {
    const double m = cs[o] / (double)n;
    double var = cs[H + o] / (double)n - m * m;
    if (var < 0) var = 0;
    mean = (float)m;
    invstd = (float)(1.0 / sqrt(var + (double)eps));
    if (rm) rm[o] = (1.f - mom) * rm[o] + mom * mean;
    if (rv) rv[o] = (1.f - mom) * rv[o] + mom * (float)(var * (double)n / (double)(n > 1 ? n - 1 : 1));
    if (o == 0 && nbt) nbt[0] += 1;
  } else {
    mean = rm[o];
    invstd = 1.0f / sqrtf(rv[o] + eps);
  }
  stats[o] = mean;
  stats[H + o] = invstd;
  stats[2 * H + o] = gamma ? gamma[o] : 1.f;
  stats[3 * H + o] = beta ? beta[o] : 0.f;
}

// ---------------------------------------------------------------- un-patch head
// One wave per position row; lane L owns channels o = 4L + 256s (s < NS): its BN statistics and ConvT2 taps
// stay in registers for every row the wave visits, so the row loop is a pure float4 stream of y.
constexpr int HEAD_MAXV = 4;  // NS <= 4 -> H <= 1024

template <int NS>
struct HeadParams {
  float mean[NS][4], inv[NS][4], gam[NS][4], bet[NS][4], w[NS][4][5];
  bool on[NS];
  __device__ __forceinline__ void load(const float* st, const float* w2, int H, int lane) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int o4 = lane * 4 + 256 * s;
      on[s] = o4 < H;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int o = on[s] ? o4 + e : 0;
        mean[s][e] = st[o];
        inv[s][e] = st[H + o];
        gam[s][e] = st[2 * H + o];
        bet[s][e] = st[3 * H + o];
#pragma unroll
        for (int j = 0; j < 5; ++j) w[s][e][j] = on[s] ? w2[o * 5 + j] : 0.f;
      }
    }
  }
};

__device__ __forceinline__ float pick5(const float (&v)[5], int lane) {
  float r = v[0];
#pragma unroll
  for (int j = 1; j < 5; ++j)
    if (lane == j) r = v[j];
  return r;
}

// Sum over the wave into lane 63 with DPP adds (quad xor 1/2, row rotate 4/8, row_bcast 15/31): six VALU ops per
// value, against six LDS-crossbar ds_bpermute round trips (plus their index math) for the shfl_xor butterfly.
template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWMASK, 0xF, false));
}
__device__ __forceinline__ float wave_sum_to_last(float v) {
  v += dpp_f<0xB1>(v);         // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);         // quad_perm [2,3,0,1]
  v += dpp_f<0x124>(v);        // row_ror:4
  v += dpp_f<0x128>(v);        // row_ror:8   -> every lane holds its 16-lane row sum
  v += dpp_f<0x142, 0xA>(v);   // row_bcast:15 into rows 1, 3
  v += dpp_f<0x143, 0xC>(v);   // row_bcast:31 into rows 2, 3 -> lane 63 holds the wave sum
  return v;
}

// 4 consecutive channels of y as f32 (y f32, or bf16: the ConvT output stored in the operand dtype)
__device__ __forceinline__ float4 head_load4(const float* y, int64_t e) { return *reinterpret_cast<const float4*>(y + e); }
__device__ __forceinline__ float4 head_load4(const bf16* y, int64_t e) {
  const uint2 h = *reinterpret_cast<const uint2*>(y + e);
  return make_float4(__uint_as_float(h.x << 16), __uint_as_float(h.x & 0xFFFF0000u), __uint_as_float(h.y << 16),
                     __uint_as_float(h.y & 0xFFFF0000u));
}
__device__ __forceinline__ float2 head_load2(const float* y, int64_t e) { return *reinterpret_cast<const float2*>(y + e); }
__device__ __forceinline__ float2 head_load2(const bf16* y, int64_t e) {
  const uint32_t h = *reinterpret_cast<const uint32_t*>(y + e);
  return make_float2(__uint_as_float(h << 16), __uint_as_float(h & 0xFFFF0000u));
}

template <int NS, typename TY = float>
__global__ __launch_bounds__(256) void head_fwd_kernel(const TY* __restrict__ y, int64_t R, int H, int Q,
                                                       const float* __restrict__ st, const float* __restrict__ w2,
                                                       const float* __restrict__ b2, float* __restrict__ x_hat) {
  const int lane = threadIdx.x & 63;
  // the row index is wave-uniform: kept in SGPRs, the y loads are SGPR base + lane offset
  const int64_t wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  HeadParams<NS> hp;
  hp.load(st, w2, H, lane);
  // BN folded into one FMA per element: bn = v * A + B with A = inv * gam, B = bet - mean * A
  float A[NS][4], B[NS][4];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      A[s][e] = hp.inv[s][e] * hp.gam[s][e];
      B[s][e] = fmaf(-hp.mean[s][e], A[s][e], hp.bet[s][e]);
    }
  const float bias = b2[0];
  // software pipeline: the next FD rows' loads are in flight while this row is reduced (no look-ahead left the
  // loads latency-bound at ~2 TB/s; FD 2 measured no better than 1 at 5 waves/SIMD)
  constexpr int FD = 1;
  float4 nv[FD][NS];
  auto load_row = [&](int d, int64_t r) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
      nv[d][s] = (hp.on[s] && r < R) ? head_load4(y, r * H + lane * 4 + 256 * s) : make_float4(0.f, 0.f, 0.f, 0.f);
  };
#pragma unroll
  for (int d = 0; d < FD; ++d) load_row(d, wave + d * nw);
  for (int64_t rb = wave; rb < R; rb += FD * nw)
#pragma unroll
  for (int d = 0; d < FD; ++d) {
    const int64_t r = rb + d * nw;
    float4 v[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) v[s] = nv[d][s];
    load_row(d, r + FD * nw);
    if (r >= R) continue;    // wave-uniform
    float part[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (!hp.on[s]) continue;
      const float vv[4] = {v[s].x, v[s].y, v[s].z, v[s].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a = gelu_erf_fast(fmaf(vv[e], A[s][e], B[s][e]));
#pragma unroll
        for (int j = 0; j < 5; ++j) part[j] = fmaf(a, hp.w[s][e][j], part[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < 5; ++j) part[j] = wave_sum_to_last(part[j]);
    if (lane == 63) {   // row r = b*Q + q -> x_hat[b][5q + j]
#pragma unroll
      for (int j = 0; j < 5; ++j) x_hat[r * 5 + j] = part[j] + bias;
    }
  }
}

// pass 1: per-channel sums for the BN backward + ConvT2 weight/bias grads + gamma/beta grads.
template <int NS>
__global__ __launch_bounds__(256) void head_bwd1_kernel(const float* __restrict__ y, int64_t R, int H, int Q,
                                                        const float* __restrict__ st, const float* __restrict__ w2,
                                                        const float* __restrict__ gx, double* __restrict__ gsums,
                                                        float* __restrict__ gw2, float* __restrict__ gb2,
                                                        float* __restrict__ ggamma, float* __restrict__ gbeta) {
  extern __shared__ float red[];  // 7*H floats: gw2 (5H), sum g (H), sum g*xn (H)
  for (int i = threadIdx.x; i < 7 * H; i += blockDim.x) red[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  HeadParams<NS> hp;
  hp.load(st, w2, H, lane);
  float accw[NS][4][5], accg[NS][4], accgx[NS][4];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      accg[s][e] = accgx[s][e] = 0.f;
#pragma unroll
      for (int j = 0; j < 5; ++j) accw[s][e][j] = 0.f;
    }
  float gbsum = 0.f;
  // software pipeline over rows (see head_fwd_kernel): the next row's y and g are loaded before this row's math
  float4 nv[NS];
  float ngo[5];
  auto load_row = [&](int64_t r) {
    const bool in = r < R;
    const int64_t rr = in ? r : 0;
    const float* gp = gx + rr * 5;          // row r = b*Q + q -> g_xhat[b][5q + j]
#pragma unroll
    for (int j = 0; j < 5; ++j) ngo[j] = in ? gp[j] : 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      nv[s] = (hp.on[s] && in) ? *reinterpret_cast<const float4*>(y + rr * H + lane * 4 + 256 * s)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  load_row(wave);
  for (int64_t r = wave; r < R; r += nw) {
    float go[5];
    float4 vrow[NS];
#pragma unroll
    for (int j = 0; j < 5; ++j) go[j] = ngo[j];
#pragma unroll
    for (int s = 0; s < NS; ++s) vrow[s] = nv[s];
    load_row(r + nw);
    gbsum += go[0] + go[1] + go[2] + go[3] + go[4];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (!hp.on[s]) continue;
      const float4 v = vrow[s];
      const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xn = (vv[e] - hp.mean[s][e]) * hp.inv[s][e];
        const float bn = xn * hp.gam[s][e] + hp.bet[s][e];
        const float a = gelu_erf_fast(bn);
        float ga = 0.f;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          ga = fmaf(go[j], hp.w[s][e][j], ga);
          accw[s][e][j] = fmaf(a, go[j], accw[s][e][j]);
        }
        const float gbn = ga * gelu_erf_grad_fast(bn);
        accg[s][e] += gbn;
        accgx[s][e] = fmaf(gbn, xn, accgx[s][e]);
      }
    }
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (!hp.on[s]) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int o = lane * 4 + 256 * s + e;
#pragma unroll
      for (int j = 0; j < 5; ++j) atomicAdd(&red[o * 5 + j], accw[s][e][j]);
      atomicAdd(&red[5 * H + o], accg[s][e]);
      atomicAdd(&red[6 * H + o], accgx[s][e]);
    }
  }
  if (lane == 0) atomicAdd(gb2, gbsum);
  __syncthreads();
  for (int i = threadIdx.x; i < 5 * H; i += blockDim.x) atomicAdd(gw2 + i, red[i]);
  for (int o = threadIdx.x; o < H; o += blockDim.x) {
    atomicAdd(gsums + o, (double)red[5 * H + o]);
    atomicAdd(gsums + H + o, (double)red[6 * H + o]);
    if (gbeta) atomicAdd(gbeta + o, red[5 * H + o]);
    if (ggamma) atomicAdd(ggamma + o, red[6 * H + o]);
  }
}

// pass 2: g_y = BN backward of g*gelu'(bn); db_y = channel sums of g_y.
template <typename T, int NS>
__global__ __launch_bounds__(256) void head_bwd2_kernel(const float* __restrict__ y, int64_t R, int H, int Q,
                                                        const float* __restrict__ st, const float* __restrict__ w2,
                                                        const float* __restrict__ gx,
                                                        const double* __restrict__ gsums, int training,
                                                        T* __restrict__ gy, float* __restrict__ dby) {
  extern __shared__ float red[];  // H
  for (int i = threadIdx.x; i < H; i += blockDim.x) red[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  HeadParams<NS> hp;
  hp.load(st, w2, H, lane);
  const float invn = 1.0f / (float)R;
  float sg[NS][4], sgx[NS][4], accd[NS][4];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int o = hp.on[s] ? lane * 4 + 256 * s + e : 0;
      sg[s][e] = training ? (float)gsums[o] * invn : 0.f;
      sgx[s][e] = training ? (float)gsums[H + o] * invn : 0.f;
      accd[s][e] = 0.f;
    }
  float4 nv[NS];
  float ngo[5];
  auto load_row = [&](int64_t r) {   // software pipeline over rows, as in head_bwd1_kernel
    const bool in = r < R;
    const int64_t rr = in ? r : 0;
    const float* gp = gx + rr * 5;          // row r = b*Q + q -> g_xhat[b][5q + j]
#pragma unroll
    for (int j = 0; j < 5; ++j) ngo[j] = in ? gp[j] : 0.f;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      nv[s] = (hp.on[s] && in) ? *reinterpret_cast<const float4*>(y + rr * H + lane * 4 + 256 * s)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  load_row(wave);
  for (int64_t r = wave; r < R; r += nw) {
    float go[5];
    float4 vrow[NS];
#pragma unroll
    for (int j = 0; j < 5; ++j) go[j] = ngo[j];
#pragma unroll
    for (int s = 0; s < NS; ++s) vrow[s] = nv[s];
    load_row(r + nw);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (!hp.on[s]) continue;
      const int o4 = lane * 4 + 256 * s;
      const float4 v = vrow[s];
      const float vv[4] = {v.x, v.y, v.z, v.w};
      float g4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xn = (vv[e] - hp.mean[s][e]) * hp.inv[s][e];
        const float bn = xn * hp.gam[s][e] + hp.bet[s][e];
        float ga = 0.f;
#pragma unroll
        for (int j = 0; j < 5; ++j) ga = fmaf(go[j], hp.w[s][e][j], ga);
        const float gbn = ga * gelu_erf_grad_fast(bn);
        const float g = hp.gam[s][e] * hp.inv[s][e] * (gbn - sg[s][e] - xn * sgx[s][e]);
        accd[s][e] += g;
        g4[e] = g;
      }
      if constexpr (sizeof(T) == 2) {
        bf16 h[4] = {(bf16)g4[0], (bf16)g4[1], (bf16)g4[2], (bf16)g4[3]};
        uint2 u;
        memcpy(&u, h, 8);
        *reinterpret_cast<uint2*>(gy + r * H + o4) = u;
      } else {
        *reinterpret_cast<float4*>(gy + r * H + o4) = make_float4(g4[0], g4[1], g4[2], g4[3]);
      }
    }
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (!hp.on[s]) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) atomicAdd(&red[lane * 4 + 256 * s + e], accd[s][e]);
  }
  __syncthreads();
  for (int o = threadIdx.x; o < H; o += blockDim.x) atomicAdd(dby + o, red[o]);
}

// Channel-split forms of the two backward passes (H a power of two, 64..2048): a row is covered by H/2
// threads with two channels each, so the per-thread state (BN parameters, ConvT2 taps, accumulators of two
// channels) stays small enough for 1024-thread workgroups: 16 waves per workgroup keep y streaming at HBM rate
// while the number of workgroups -- each ends with its per-channel global atomics -- stays at 512.
struct Head2 {   // the two channels c0, c0+1 of a thread as register pairs
  f32x2 inv, c, gam, bet, w[5];   // c = -mean * inv: xn = v * inv + c in one packed FMA
  __device__ __forceinline__ void load(const float* st, const float* w2, int H, int c0) {
    const f32x2 mean = {st[c0], st[c0 + 1]};
    inv = (f32x2){st[H + c0], st[H + c0 + 1]};
    gam = (f32x2){st[2 * H + c0], st[2 * H + c0 + 1]};
    bet = (f32x2){st[3 * H + c0], st[3 * H + c0 + 1]};
    c = -mean * inv;
#pragma unroll
    for (int j = 0; j < 5; ++j) w[j] = (f32x2){w2[c0 * 5 + j], w2[(c0 + 1) * 5 + j]};
  }
};

// Rows in flight per thread in the channel-split passes: each thread streams only 8 bytes of y per row, so one row
// of look-ahead kept ~8 KB per CU in flight (1.9-3.3 TB/s); HEAD_CS_DEPTH rows are loaded ahead instead.
constexpr int HEAD_CS_DEPTH = 2;

template <typename TY, bool UNI>
__global__ __launch_bounds__(1024) void head_bwd1_cs_kernel(const TY* __restrict__ y, int64_t R, int H, int Q,
                                                           const float* __restrict__ st, const float* __restrict__ w2,
                                                           const float* __restrict__ gx, double* __restrict__ gsums,
                                                           float* __restrict__ gw2, float* __restrict__ gb2,
                                                           float* __restrict__ ggamma, float* __restrict__ gbeta) {
  extern __shared__ float red[];  // 7*H floats: gw2 (5H), sum g (H), sum g*xn (H)
  for (int i = threadIdx.x; i < 7 * H; i += blockDim.x) red[i] = 0.f;
  __syncthreads();
  const int tpr = H >> 1, rpb = blockDim.x / tpr;
  const int c0 = (threadIdx.x % tpr) * 2;
  // UNI (H >= 128: a row spans whole waves): the row index is wave-uniform, so the row's five g_xhat values come
  // by scalar loads instead of five broadcast vector loads per row and wave
  const int rg = UNI ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x / tpr)) : (int)(threadIdx.x / tpr);
  Head2 hp;
  hp.load(st, w2, H, c0);
  f32x2 accw[5], accg = aw_splat2(0.f), accgx = aw_splat2(0.f);
#pragma unroll
  for (int j = 0; j < 5; ++j) accw[j] = aw_splat2(0.f);
  float gbsum = 0.f;
  const int64_t step = (int64_t)gridDim.x * rpb;
  constexpr int D = HEAD_CS_DEPTH;
  float2 nv[D];
  float ngo[D][5];
  auto load_row = [&](int d, int64_t r) {   // rows past R load as zeros
    const bool in = r < R;
    const int64_t rr = in ? r : 0;
    const float* gp = gx + rr * 5;          // row r = b*Q + q -> g_xhat[b][5q + j]
#pragma unroll
    for (int j = 0; j < 5; ++j) ngo[d][j] = in ? gp[j] : 0.f;
    nv[d] = in ? head_load2(y, rr * H + c0) : make_float2(0.f, 0.f);
  };
  const int64_t r0 = (int64_t)blockIdx.x * rpb + rg;
#pragma unroll
  for (int d = 0; d < D; ++d) load_row(d, r0 + d * step);
  for (int64_t rb = r0; rb < R; rb += D * step)
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const int64_t r = rb + d * step;
    float go[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) go[j] = ngo[d][j];
    const f32x2 v = {nv[d].x, nv[d].y};
    load_row(d, r + D * step);
    __builtin_amdgcn_sched_barrier(0);   // one row's math at a time: the unrolled rows must not interleave (spills)
    // a row past R has g = 0 and y = 0: every accumulator below gains exactly zero from it
    if (c0 == 0) gbsum += go[0] + go[1] + go[2] + go[3] + go[4];
    const f32x2 xn = __builtin_elementwise_fma(v, hp.inv, hp.c);
    const f32x2 bn = __builtin_elementwise_fma(xn, hp.gam, hp.bet);
    f32x2 a, dg;
    gelu_erf_fast2_and_grad(bn, a, dg);
    f32x2 ga = aw_splat2(0.f);
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      ga = __builtin_elementwise_fma(aw_splat2(go[j]), hp.w[j], ga);
      accw[j] = __builtin_elementwise_fma(a, aw_splat2(go[j]), accw[j]);
    }
    const f32x2 gbn = ga * dg;
    accg += gbn;
    accgx = __builtin_elementwise_fma(gbn, xn, accgx);
  }
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int o = c0 + e;
#pragma unroll
    for (int j = 0; j < 5; ++j) atomicAdd(&red[o * 5 + j], accw[j][e]);
    atomicAdd(&red[5 * H + o], accg[e]);
    atomicAdd(&red[6 * H + o], accgx[e]);
  }
  if (c0 == 0) atomicAdd(gb2, gbsum);
  __syncthreads();
  for (int i = threadIdx.x; i < 5 * H; i += blockDim.x) atomicAdd(gw2 + i, red[i]);
  for (int o = threadIdx.x; o < H; o += blockDim.x) {
    atomicAdd(gsums + o, (double)red[5 * H + o]);
    atomicAdd(gsums + H + o, (double)red[6 * H + o]);
    if (gbeta) atomicAdd(gbeta + o, red[5 * H + o]);
    if (ggamma) atomicAdd(ggamma + o, red[6 * H + o]);
  }
}

template <typename T, typename TY, bool UNI>
__global__ __launch_bounds__(1024) void head_bwd2_cs_kernel(const TY* __restrict__ y, int64_t R, int H, int Q,
                                                           const float* __restrict__ st, const float* __restrict__ w2,
                                                           const float* __restrict__ gx,
                                                           const double* __restrict__ gsums, int training,
                                                           T* __restrict__ gy, float* __restrict__ dby) {
  extern __shared__ float red[];  // H
  for (int i = threadIdx.x; i < H; i += blockDim.x) red[i] = 0.f;
  __syncthreads();
  const int tpr = H >> 1, rpb = blockDim.x / tpr;
  const int c0 = (threadIdx.x % tpr) * 2;
  // UNI (H >= 128: a row spans whole waves): the row index is wave-uniform, so the row's five g_xhat values come
  // by scalar loads instead of five broadcast vector loads per row and wave
  const int rg = UNI ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x / tpr)) : (int)(threadIdx.x / tpr);
  Head2 hp;
  hp.load(st, w2, H, c0);
  const float invn = 1.0f / (float)R;
  f32x2 sg = aw_splat2(0.f), sgx = aw_splat2(0.f), accd = aw_splat2(0.f);
  if (training) {
    sg = (f32x2){(float)gsums[c0], (float)gsums[c0 + 1]} * aw_splat2(invn);
    sgx = (f32x2){(float)gsums[H + c0], (float)gsums[H + c0 + 1]} * aw_splat2(invn);
  }
  const f32x2 P = hp.gam * hp.inv;
  const int64_t step = (int64_t)gridDim.x * rpb;
  constexpr int D = HEAD_CS_DEPTH;
  float2 nv[D];
  float ngo[D][5];
  auto load_row = [&](int d, int64_t r) {   // rows past R load as zeros
    const bool in = r < R;
    const int64_t rr = in ? r : 0;
    const float* gp = gx + rr * 5;          // row r = b*Q + q -> g_xhat[b][5q + j]
#pragma unroll
    for (int j = 0; j < 5; ++j) ngo[d][j] = in ? gp[j] : 0.f;
    nv[d] = in ? head_load2(y, rr * H + c0) : make_float2(0.f, 0.f);
  };
  const int64_t r0 = (int64_t)blockIdx.x * rpb + rg;
#pragma unroll
  for (int d = 0; d < D; ++d) load_row(d, r0 + d * step);
  for (int64_t rb = r0; rb < R; rb += D * step)
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const int64_t r = rb + d * step;
    float go[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) go[j] = ngo[d][j];
    const f32x2 v = {nv[d].x, nv[d].y};
    load_row(d, r + D * step);
    __builtin_amdgcn_sched_barrier(0);   // one row's math at a time: the unrolled rows must not interleave (spills)
    const f32x2 xn = __builtin_elementwise_fma(v, hp.inv, hp.c);
    const f32x2 bn = __builtin_elementwise_fma(xn, hp.gam, hp.bet);
    f32x2 ga = aw_splat2(0.f);
#pragma unroll
    for (int j = 0; j < 5; ++j) ga = __builtin_elementwise_fma(aw_splat2(go[j]), hp.w[j], ga);
    const f32x2 gbn = ga * gelu_erf_grad_fast2(bn);
    const f32x2 g = P * (gbn - __builtin_elementwise_fma(xn, sgx, sg));
    if (r >= R) continue;
    accd += g;
    if constexpr (sizeof(T) == 2) {
      bf16 h[2] = {(bf16)g.x, (bf16)g.y};
      uint32_t u;
      memcpy(&u, h, 4);
      if (AW_WT_MISC) aw_st_wt(gy + r * H + c0, u);
      else *reinterpret_cast<uint32_t*>(gy + r * H + c0) = u;
    } else if (AW_WT_MISC) {
      u32x2 u = {__float_as_uint(g.x), __float_as_uint(g.y)};
      aw_st_wt(gy + r * H + c0, u);
    } else {
      *reinterpret_cast<float2*>(gy + r * H + c0) = make_float2(g.x, g.y);
    }
  }
#pragma unroll
  for (int e = 0; e < 2; ++e) atomicAdd(&red[c0 + e], accd[e]);
  __syncthreads();
  for (int o = threadIdx.x; o < H; o += blockDim.x) atomicAdd(dby + o, red[o]);
}

// ---------------------------------------------------------------- fused head forward + pass 1 (training step)
// The training step's loss is mse(x_hat, x) + the embedding loss (autencoder_lightning_base.py:80-97), so a row's
// gradient g_xhat = c (x_hat - x) (c = 2 / numel * loss scale: aw_mse_bwd's formula) is known the moment its x_hat
// is: one pass over y computes the forward (BN -> GELU -> ConvT2), the MSE sum and gradient, and pass 1's sums and
// gradients (aw_unpatch_head_bwd1), from one Phi / exp per element -- y is read once instead of twice.
// H = 512.  One wave per row; lane l owns 8 channels: f32 y -> 4l..4l+3 and 256+4l..+3 (the two 1-KiB halves of a
// 2-KiB row), bf16 y -> 8l..8l+7 (one 1-KiB row).  Rows reach the wave's OWN slice of LDS by LDS-DMA in batches of
// HB rows through a ring of three batches (two in flight while one computes), without VGPRs held by loads and
// without barriers (nothing is shared between waves until the final per-channel reduction).  The x row (5 floats)
// comes the same way.
#ifndef AW_ATOMIC_ROTATE
#define AW_ATOMIC_ROTATE 1
#endif
constexpr int HB = 4;          // rows per wave below which the grid shrinks
constexpr int HFW = 8;         // waves per workgroup (one workgroup per CU: its per-channel atomics end the launch)
template <typename TY> struct HeadRows {
  static constexpr int ROWB = 512 * (int)sizeof(TY);   // bytes per y row
  static constexpr int NP = ROWB / 1024;                // 1-KiB DMA pieces per row
  static constexpr int XB = 32;                         // bytes per x slot (5 floats used)
  static constexpr int HB = sizeof(TY) == 4 ? 2 : 4;    // rows per batch (even: the fused pass takes them in pairs)
  static constexpr int PB = HB * (NP + 1);              // DMA instructions per batch and wave
  static constexpr int NBUF = 3;                        // batches in the wave's ring (two in flight)
  static constexpr int BATCH = HB * (ROWB + XB);
  static constexpr int WAVE = NBUF * BATCH;
  static constexpr int NG = sizeof(TY) == 4 ? 4 : 8;   // channels of a lane that are contiguous in a row
  __device__ static int chan(int lane, int k) {
    return sizeof(TY) == 4 ? (k < 4 ? 4 * lane + k : 256 + 4 * lane + k - 4) : 8 * lane + k;
  }
  __device__ static void row(const char* p, int lane, float (&v)[8]) {   // this lane's 8 channels of an LDS row
    if constexpr (sizeof(TY) == 4) {
      const float4 a = *reinterpret_cast<const float4*>(p + 16 * lane);
      const float4 b = *reinterpret_cast<const float4*>(p + 1024 + 16 * lane);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
      const uint4 u = *reinterpret_cast<const uint4*>(p + 16 * lane);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
      }
    }
  }
};

template <typename TY>
__global__ __launch_bounds__(64 * HFW, 1) void head_fwd_bwd1_kernel(
    const TY* __restrict__ y, int64_t R, const float* __restrict__ st, const float* __restrict__ w2,
    const float* __restrict__ b2, const float* __restrict__ x, const float* __restrict__ gscale, float gmul,
    float* __restrict__ x_hat, float* __restrict__ g_xhat, double* __restrict__ sqerr, double* __restrict__ gsums,
    float* __restrict__ gw2, float* __restrict__ gb2, float* __restrict__ ggamma, float* __restrict__ gbeta) {
  using HR = HeadRows<TY>;
  constexpr int H = 512;
  // the waves' row buffers; after the row loop, their per-channel partial sums [wave][7H] (gw2 5H, sum g, sum g*xhat)
  constexpr int LB = HFW * HR::WAVE > HFW * 7 * H * 4 ? HFW * HR::WAVE : HFW * 7 * H * 4;
  __shared__ __attribute__((aligned(16))) char L[LB];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t wave = (int64_t)blockIdx.x * HFW + wv, nw = (int64_t)gridDim.x * HFW;
  const char* Lw = L + wv * HR::WAVE;
  const uint32_t lw = aw_lds_addr(Lw);
  const aw_v4i32 dy = aw_rdesc(y, (uint32_t)(R * HR::ROWB));
  const aw_v4i32 dx = aw_rdesc(x, (uint32_t)(R * 20));
  auto issue = [&](int64_t bt) {   // batch bt of this wave's rows into buffer bt % NBUF; rows past R load zeros
    const uint32_t base = lw + (uint32_t)((bt % HR::NBUF) * HR::BATCH);
#pragma unroll
    for (int k = 0; k < HR::HB; ++k) {
      const int64_t r0 = wave + (bt * HR::HB + k) * nw;
      const int r = (int)(r0 < R ? r0 : R);
#pragma unroll
      for (int pc = 0; pc < HR::NP; ++pc) aw_dma16(base + k * HR::ROWB + pc * 1024, r * HR::ROWB + pc * 1024 + 16 * lane, dy);
      if (lane < 5) aw_dma4(base + HR::HB * HR::ROWB + k * HR::XB, r * 20 + 4 * lane, dx);
    }
  };
  // per-channel state as pairs (channels chan(2p), chan(2p+1)): xn = v * inv + c, bn = xn * gam + bet
  f32x2 inv[4], cc[4], gam[4], bet[4], w[4][5];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int o0 = HR::chan(lane, 2 * p), o1 = HR::chan(lane, 2 * p + 1);
    inv[p] = (f32x2){st[H + o0], st[H + o1]};
    cc[p] = -(f32x2){st[o0], st[o1]} * inv[p];
    gam[p] = (f32x2){st[2 * H + o0], st[2 * H + o1]};
    bet[p] = (f32x2){st[3 * H + o0], st[3 * H + o1]};
#pragma unroll
    for (int j = 0; j < 5; ++j) w[p][j] = (f32x2){w2[o0 * 5 + j], w2[o1 * 5 + j]};
  }
  f32x2 accw[4][5], accg[4], accgx[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    accg[p] = accgx[p] = aw_splat2(0.f);
#pragma unroll
    for (int j = 0; j < 5; ++j) accw[p][j] = aw_splat2(0.f);
  }
  const float c = gmul * gscale[0];
  const float bias = b2[0];
  double sq = 0.0;
  float gbs = 0.f;
  const int64_t nrows = wave < R ? (R - 1 - wave) / nw + 1 : 0;
  const int64_t nb = (nrows + HR::HB - 1) / HR::HB;
  // a batch's x_hat / g_xhat values are stored right after the NEXT batch's wait: the wait covers stores too (vmcnt),
  // and stored at once they would expose their write latency at every batch
  float hx[HR::HB], hg[HR::HB];
  int64_t hb = -1;   // batch whose values are held
  auto flush = [&]() {
    if (hb < 0) return;
#pragma unroll
    for (int k = 0; k < HR::HB; ++k) {
      const int64_t r = wave + (hb * HR::HB + k) * nw;
      if (r < R && lane < 5) {   // row r = b*Q + q -> x_hat[b][5q + j]
        x_hat[r * 5 + lane] = hx[k];
        g_xhat[r * 5 + lane] = hg[k];
      }
    }
    hb = -1;
  };
  // counted waits: loads retire in order, so vmcnt <= PB (the newest batch) means batch bt has landed; the few stores
  // between them only make the wait longer, never shorter
  if (nb > 0) issue(0);
  if (nb > 1) issue(1);
  for (int64_t bt = 0; bt < nb; ++bt) {
    if (bt + 1 < nb)
      aw_vm_wait<HR::PB>();
    else
      aw_vm_wait<0>();
    flush();
    if (bt + 2 < nb) issue(bt + 2);
    hb = bt;
    const char* Lb = Lw + (bt % HR::NBUF) * HR::BATCH;
    // two rows at a time: their forward halves, their 10 wave reductions and their backward halves interleave
    // (at two waves per SIMD one row alone left the VALU waiting on its own dependency chains)
#pragma unroll
    for (int k0 = 0; k0 < HR::HB; k0 += 2) {
      const int64_t r0 = wave + (bt * HR::HB + k0) * nw;
      if (r0 >= R) break;   // wave-uniform
      const bool two = r0 + nw < R;
      f32x2 a[2][4], dg[2][4], xn[2][4];
      float part[2][5];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float v[8];
        HR::row(Lb + (k0 + u) * HR::ROWB, lane, v);
        f32x2 pj[5];
#pragma unroll
        for (int j = 0; j < 5; ++j) pj[j] = aw_splat2(0.f);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          xn[u][p] = __builtin_elementwise_fma((f32x2){v[2 * p], v[2 * p + 1]}, inv[p], cc[p]);
          const f32x2 bn = __builtin_elementwise_fma(xn[u][p], gam[p], bet[p]);
          f32x2 e;
          const f32x2 phi = aw_phi_e2(bn, e);
          a[u][p] = bn * phi;
          dg[u][p] = __builtin_elementwise_fma(bn * aw_splat2(AW_INV_SQRT2PI), e, phi);
#pragma unroll
          for (int j = 0; j < 5; ++j) pj[j] = __builtin_elementwise_fma(a[u][p], w[p][j], pj[j]);
        }
#pragma unroll
        for (int j = 0; j < 5; ++j) part[u][j] = pj[j].x + pj[j].y;
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int j = 0; j < 5; ++j) part[u][j] = wave_sum_to_last(part[u][j]);
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (u == 1 && !two) break;   // wave-uniform
        const float* xs = reinterpret_cast<const float*>(Lb + HR::HB * HR::ROWB + (k0 + u) * HR::XB);
        float go[5], xo = 0.f, gsel = 0.f, d2 = 0.f, gsum = 0.f;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          const float xh = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(part[u][j]), 63)) + bias;
          const float d = xh - xs[j];
          go[j] = c * d;
          d2 = fmaf(d, d, d2);
          gsum += go[j];
          if (lane == j) {
            xo = xh;
            gsel = go[j];
          }
        }
        hx[k0 + u] = xo;
        hg[k0 + u] = gsel;
        sq += (double)d2;
        gbs += gsum;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          f32x2 ga = aw_splat2(0.f);
#pragma unroll
          for (int j = 0; j < 5; ++j) {
            ga = __builtin_elementwise_fma(aw_splat2(go[j]), w[p][j], ga);
            accw[p][j] = __builtin_elementwise_fma(a[u][p], aw_splat2(go[j]), accw[p][j]);
          }
          const f32x2 gbn = ga * dg[u][p];
          accg[p] += gbn;
          accgx[p] = __builtin_elementwise_fma(gbn, xn[u][p], accgx[p]);
        }
      }
    }
  }
  flush();
  aw_vm_wait<0>();   // every DMA of this wave has landed before its buffer is reused (or the LDS released)
  __syncthreads();
  // per-channel sums: each wave writes its partials, then every entry is summed over the waves in fixed order and
  // added to the gradients with one global atomic per workgroup (LDS atomics from 8 waves on the same channels
  // measured 22 us of the 106 us launch)
  float* part = reinterpret_cast<float*>(L);
  float* mine = part + wv * 7 * H;
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int o = HR::chan(lane, 2 * p + e);
#pragma unroll
      for (int j = 0; j < 5; ++j) mine[o * 5 + j] = accw[p][j][e];
      mine[5 * H + o] = accg[p][e];
      mine[6 * H + o] = accgx[p][e];
    }
  // the two scalar sums per workgroup (one atomic each), not per wave: 2 x 2048 same-address atomics serialised
  // into ~12 us of the launch's tail (fused head 88.7 -> 74.8-76.6 us isolated, tools/probe/head_probe.py)
  __shared__ double scal[HFW][2];
  if (lane == 0) {
    scal[wv][0] = sq;
    scal[wv][1] = (double)gbs;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0;
#pragma unroll
    for (int q = 0; q < HFW; ++q) {
      a += scal[q][0];
      b += scal[q][1];
    }
    atomicAdd(sqerr, a);
    atomicAdd(gb2, (float)b);
  }
  // per-channel sums: every workgroup adds into the same 7H addresses; starting each workgroup's walk at its own
  // offset keeps them on different addresses at any moment (AW_ATOMIC_ROTATE=0 in the build: all from entry 0)
  for (int i0 = threadIdx.x; i0 < 7 * H; i0 += 64 * HFW) {
#if AW_ATOMIC_ROTATE
    const int i = (i0 + (int)(blockIdx.x % 7) * H) % (7 * H);
#else
    const int i = i0;
#endif
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < HFW; ++q) t += part[q * 7 * H + i];
    if (i < 5 * H) {
      atomicAdd(gw2 + i, t);
    } else if (i < 6 * H) {
      atomicAdd(gsums + (i - 5 * H), (double)t);
      if (gbeta) atomicAdd(gbeta + (i - 5 * H), t);
    } else {
      atomicAdd(gsums + (i - 5 * H), (double)t);
      if (ggamma) atomicAdd(ggamma + (i - 6 * H), t);
    }
  }
}

// Pass 2 on the same row stream (H = 512): g_y = BN backward of g * gelu'(bn) per row, its channel sums db_y.  The
// row's five g_xhat values come by LDS-DMA beside its y row.
template <typename T, typename TY>
__global__ __launch_bounds__(64 * HFW, 1) void head_bwd2_rows_kernel(const TY* __restrict__ y, int64_t R,
                                                                    const float* __restrict__ st,
                                                                    const float* __restrict__ w2,
                                                                    const float* __restrict__ gx,
                                                                    const double* __restrict__ gsums, int training,
                                                                    T* __restrict__ gy, float* __restrict__ dby) {
  using HR = HeadRows<TY>;
  constexpr int H = 512;
  __shared__ __attribute__((aligned(16))) char L[HFW * HR::WAVE];   // row buffers, then the partial sums [wave][H]
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t wave = (int64_t)blockIdx.x * HFW + wv, nw = (int64_t)gridDim.x * HFW;
  const char* Lw = L + wv * HR::WAVE;
  const uint32_t lw = aw_lds_addr(Lw);
  const aw_v4i32 dy = aw_rdesc(y, (uint32_t)(R * HR::ROWB));
  const aw_v4i32 dg = aw_rdesc(gx, (uint32_t)(R * 20));
  auto issue = [&](int64_t bt) {
    const uint32_t base = lw + (uint32_t)((bt % HR::NBUF) * HR::BATCH);
#pragma unroll
    for (int k = 0; k < HR::HB; ++k) {
      const int64_t r0 = wave + (bt * HR::HB + k) * nw;
      const int r = (int)(r0 < R ? r0 : R);
#pragma unroll
      for (int pc = 0; pc < HR::NP; ++pc) aw_dma16(base + k * HR::ROWB + pc * 1024, r * HR::ROWB + pc * 1024 + 16 * lane, dy);
      if (lane < 5) aw_dma4(base + HR::HB * HR::ROWB + k * HR::XB, r * 20 + 4 * lane, dg);
    }
  };
  const float invn = 1.0f / (float)R;
  f32x2 inv[4], cc[4], gam[4], bet[4], P[4], sg[4], sgx[4], w[4][5], accd[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int o0 = HR::chan(lane, 2 * p), o1 = HR::chan(lane, 2 * p + 1);
    inv[p] = (f32x2){st[H + o0], st[H + o1]};
    cc[p] = -(f32x2){st[o0], st[o1]} * inv[p];
    gam[p] = (f32x2){st[2 * H + o0], st[2 * H + o1]};
    bet[p] = (f32x2){st[3 * H + o0], st[3 * H + o1]};
    P[p] = gam[p] * inv[p];
    sg[p] = training ? (f32x2){(float)gsums[o0], (float)gsums[o1]} * aw_splat2(invn) : aw_splat2(0.f);
    sgx[p] = training ? (f32x2){(float)gsums[H + o0], (float)gsums[H + o1]} * aw_splat2(invn) : aw_splat2(0.f);
    accd[p] = aw_splat2(0.f);
#pragma unroll
    for (int j = 0; j < 5; ++j) w[p][j] = (f32x2){w2[o0 * 5 + j], w2[o1 * 5 + j]};
  }
  const int64_t nrows = wave < R ? (R - 1 - wave) / nw + 1 : 0;
  const int64_t nb = (nrows + HR::HB - 1) / HR::HB;
  // a batch's g_y rows are stored right after the NEXT batch's wait (the wait covers stores too)
  float hold[HR::HB][8];
  int64_t hb = -1;
  auto flush = [&]() {
    if (hb < 0) return;
#pragma unroll
    for (int k = 0; k < HR::HB; ++k) {
      const int64_t r = wave + (hb * HR::HB + k) * nw;
      if (r >= R) break;
      const float* out = hold[k];
      // this lane's channels: f32 y -> 4l.. and 256+4l.. (two groups of 4), bf16 y -> 8l.. (one group of 8)
      T* dst = gy + r * H;
#pragma unroll
      for (int q = 0; q < 8 / HR::NG; ++q) {
        const int o = HR::chan(lane, q * HR::NG);
        if constexpr (sizeof(T) == 2) {
          if constexpr (HR::NG == 4) {
            bf16 h[4] = {(bf16)out[4 * q], (bf16)out[4 * q + 1], (bf16)out[4 * q + 2], (bf16)out[4 * q + 3]};
            u32x2 u;
            memcpy(&u, h, 8);
            aw_st_wt(dst + o, u);
          } else {
            bf16 h[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) h[i] = (bf16)out[i];
            f32x4 u;
            memcpy(&u, h, 16);
            aw_st_wt(dst + o, u);
          }
        } else {
#pragma unroll
          for (int i = 0; i < HR::NG; i += 4)
            aw_st_wt(dst + o + i, (f32x4){out[q * HR::NG + i], out[q * HR::NG + i + 1], out[q * HR::NG + i + 2],
                                          out[q * HR::NG + i + 3]});
        }
      }
    }
    hb = -1;
  };
  // counted waits: loads retire in order, so vmcnt <= PB (the newest batch) means batch bt has landed; the few stores
  // between them only make the wait longer, never shorter
  if (nb > 0) issue(0);
  if (nb > 1) issue(1);
  for (int64_t bt = 0; bt < nb; ++bt) {
    if (bt + 1 < nb)
      aw_vm_wait<HR::PB>();
    else
      aw_vm_wait<0>();
    flush();
    if (bt + 2 < nb) issue(bt + 2);
    hb = bt;
    const char* Lb = Lw + (bt % HR::NBUF) * HR::BATCH;
#pragma unroll
    for (int k = 0; k < HR::HB; ++k) {
      const int64_t r = wave + (bt * HR::HB + k) * nw;
      if (r >= R) break;   // wave-uniform
      float v[8];
      HR::row(Lb + k * HR::ROWB, lane, v);
      const float* gs = reinterpret_cast<const float*>(Lb + HR::HB * HR::ROWB + k * HR::XB);
      float go[5];
#pragma unroll
      for (int j = 0; j < 5; ++j) go[j] = gs[j];
      float* out = hold[k];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const f32x2 xn = __builtin_elementwise_fma((f32x2){v[2 * p], v[2 * p + 1]}, inv[p], cc[p]);
        const f32x2 bn = __builtin_elementwise_fma(xn, gam[p], bet[p]);
        f32x2 e;
        const f32x2 phi = aw_phi_e2(bn, e);
        const f32x2 d = __builtin_elementwise_fma(bn * aw_splat2(AW_INV_SQRT2PI), e, phi);
        f32x2 ga = aw_splat2(0.f);
#pragma unroll
        for (int j = 0; j < 5; ++j) ga = __builtin_elementwise_fma(aw_splat2(go[j]), w[p][j], ga);
        const f32x2 g = P[p] * (ga * d - __builtin_elementwise_fma(xn, sgx[p], sg[p]));
        accd[p] += g;
        out[2 * p] = g.x;
        out[2 * p + 1] = g.y;
      }
    }
  }
  flush();
  aw_vm_wait<0>();
  __syncthreads();
  float* part = reinterpret_cast<float*>(L);
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    part[wv * H + HR::chan(lane, 2 * p)] = accd[p].x;
    part[wv * H + HR::chan(lane, 2 * p + 1)] = accd[p].y;
  }
  __syncthreads();
  for (int o0 = threadIdx.x; o0 < H; o0 += 64 * HFW) {
#if AW_ATOMIC_ROTATE
    const int o = (o0 + (int)(blockIdx.x & 7) * (H / 8)) % H;   // see head_fwd_bwd1_kernel
#else
    const int o = o0;
#endif
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < HFW; ++q) t += part[q * H + o];
    atomicAdd(dby + o, t);
  }
}

// n4 float4 groups (0 when a or b is not 16-B aligned) then the scalar tail.  Four float4 loads of each input in
// flight per thread: the one-element loop waited on a load per element (13.6 us at the bench's 409,600 elements).
// Each thread sums a group of four float4 products in f32, the groups and waves in f64.
__global__ __launch_bounds__(256) void mse_fwd_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                      int64_t n, int64_t n4, double* sqerr) {
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x, t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t q0 = t; q0 < n4; q0 += 4 * stride) {
    float4 va[4], vb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t q = q0 + u * stride;
      const bool in = q < n4;
      va[u] = in ? reinterpret_cast<const float4*>(a)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
      vb[u] = in ? reinterpret_cast<const float4*>(b)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float sm = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float dx = va[u].x - vb[u].x, dy = va[u].y - vb[u].y, dz = va[u].z - vb[u].z, dw = va[u].w - vb[u].w;
      sm += (dx * dx + dy * dy) + (dz * dz + dw * dw);
    }
    acc += (double)sm;
  }
  for (int64_t i = 4 * n4 + t; i < n; i += stride) {
    const float d = a[i] - b[i];
    acc += (double)(d * d);
  }
  __shared__ double red[4];
  acc = wave_sum_d(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(sqerr, red[0] + red[1] + red[2] + red[3]);
}

__global__ void mse_bwd_kernel(const float* __restrict__ a, const float* __restrict__ b, int64_t n,
                               const float* __restrict__ g, float* __restrict__ ga) {
  const float c = 2.0f / (float)n * g[0];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    ga[i] = c * (a[i] - b[i]);
}

__global__ void scalar_add_kernel(const float* a, const float* b, float* out) { out[0] = a[0] + b[0]; }
__global__ void mse_finalize_kernel(const double* s, int64_t n, float* out) { out[0] = (float)(s[0] / (double)n); }
// the training step's loss in the same launch: recon = mse, loss = recon + addend (the embedding loss)
__global__ void mse_finalize_add_kernel(const double* s, int64_t n, const float* addend, float* out, float* sum) {
  const float r = (float)(s[0] / (double)n);
  out[0] = r;
  sum[0] = r + addend[0];
}

// channel-split head backward: H / 2 threads per row must divide the 1024-thread workgroup
int head_cus() {   // the row-stream head passes run one workgroup per CU
  static const int n = [] {
    int dev = 0, c = 0;
    return hipGetDevice(&dev) == hipSuccess &&
                   hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && c > 0
               ? c : 256;
  }();
  return n;
}

int head_wgs() {   // workgroups of the channel-split head passes (AW_HEAD_WGS: tuning override)
  // 256 measured best at H 512, B 1024: fewer starve the CUs of rows in flight, more serialise on the per-channel
  // global atomics every workgroup ends with
  static const int n = [] { const char* e = getenv("AW_HEAD_WGS"); return e ? atoi(e) : 256; }();
  return n;
}

bool head_cs_ok(int H) { return H >= 64 && H <= 2048 && (H & (H - 1)) == 0; }

int grid_for(int64_t n, int threads = 256, int cap = 8192) {
  int64_t g = (n + threads - 1) / threads;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" int aw_patchify(const float* x, int64_t B, int L, int C, int P, void* patches, int64_t ldp, int dtype,
                           void* stream) {
  AW_REQUIRE(x && patches && B >= 0 && L > 0 && C > 0 && P > 0 && ldp >= P, "aw_patchify: bad args");
  AW_REQUIRE((L * C) % P == 0, "aw_patchify: L*C must be a multiple of P");
  if (B == 0) return AW_OK;
  const int64_t n = B * (L * C / P) * ldp;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == AW_BF16)
    hipLaunchKernelGGL(patchify_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, s, x, B, L, C, P, (bf16*)patches, ldp);
  else
    hipLaunchKernelGGL(patchify_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, x, B, L, C, P, (float*)patches, ldp);
  return aw::check_launch("aw_patchify");
}

extern "C" int aw_weight_relayout(const float* W, int O, int I, int k, int tap, int mode, void* out, int64_t ldo,
                                  int dtype, void* stream) {
  AW_REQUIRE(W && out && O > 0 && I > 0 && k > 0 && mode >= 0 && mode <= 4, "aw_weight_relayout: bad args");
  AW_REQUIRE(!(mode == 4 && ldo < k), "aw_weight_relayout: ldo < k");
  int64_t n = mode == 4 ? (int64_t)O * ldo : (int64_t)O * I * (mode == 0 ? 1 : (mode == 3 ? k : 3));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == AW_BF16)
    hipLaunchKernelGGL(relayout_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, s, W, O, I, k, tap, mode, (bf16*)out, ldo);
  else
    hipLaunchKernelGGL(relayout_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, W, O, I, k, tap, mode, (float*)out, ldo);
  return aw::check_launch("aw_weight_relayout");
}

extern "C" int aw_weight_relayout_batch(const aw_relayout_job* jobs, int n, int dtype, void* stream) {
  AW_REQUIRE(jobs && n >= 0 && n <= AW_RELAYOUT_MAX_JOBS, "aw_weight_relayout_batch: need 0..%d jobs",
             AW_RELAYOUT_MAX_JOBS);
  AW_REQUIRE(dtype == AW_BF16 || dtype == AW_F32, "aw_weight_relayout_batch: bad dtype");
  if (n == 0) return AW_OK;
  RelayoutJobs J;
  memset(&J, 0, sizeof(J));
  int64_t most = 0;
  for (int i = 0; i < n; ++i) {
    const aw_relayout_job& jb = jobs[i];
    AW_REQUIRE(jb.W && jb.out && jb.O > 0 && jb.I > 0 && jb.k > 0 && jb.mode >= 0 && jb.mode <= 7 && jb.mode != 6,
               "aw_weight_relayout_batch: bad job %d", i);
    AW_REQUIRE(!(jb.mode == 4 && jb.ldo < jb.k), "aw_weight_relayout_batch: job %d ldo < k", i);
    AW_REQUIRE((int64_t)jb.O * jb.I * (jb.k > 3 ? jb.k : 3) < (1ll << 31) && (int64_t)jb.O * jb.ldo < (1ll << 31),
               "aw_weight_relayout_batch: job %d exceeds 2^31 elements", i);
    J.j[i] = jb;
    const int64_t c = jb.mode == 4 ? (int64_t)jb.O * jb.ldo
                                    : (int64_t)jb.O * jb.I * ((jb.mode == 0 || jb.mode == 5) ? 1
                                                              : (jb.mode == 3 ? jb.k : 3));
    most = c > most ? c : most;
  }
  int gx = (int)((most + 255) / 256);
  gx = gx < 1 ? 1 : (gx > 256 ? 256 : gx);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == AW_BF16)
    hipLaunchKernelGGL(relayout_batch_kernel<bf16>, dim3(gx, n), dim3(256), 0, s, J);
  else
    hipLaunchKernelGGL(relayout_batch_kernel<float>, dim3(gx, n), dim3(256), 0, s, J);
  return aw::check_launch("aw_weight_relayout_batch");
}

extern "C" int aw_weight_grad_scatter(const float* g, int O, int I, int k, int tap, int mode, int64_t ldg, float* G,
                                      void* stream) {
  AW_REQUIRE(g && G && O > 0 && I > 0 && k > 0 && (mode == 0 || mode == 1 || mode == 3 || mode == 4),
             "aw_weight_grad_scatter: bad args");
  int64_t n = mode == 4 ? (int64_t)O * k : (int64_t)O * I * (mode == 0 ? 1 : (mode == 3 ? k : 3));
  hipLaunchKernelGGL(grad_scatter_kernel, dim3(grid_for(n)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), g, O,
                     I, k, tap, mode, ldg, G);
  return aw::check_launch("aw_weight_grad_scatter");
}

extern "C" int aw_cast(const float* in, int64_t n, void* out, int dtype, void* stream) {
  AW_REQUIRE(in && out && n >= 0, "aw_cast: bad args");
  if (n == 0) return AW_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == AW_BF16)
    hipLaunchKernelGGL(cast_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, s, in, n, (bf16*)out);
  else
    hipLaunchKernelGGL(cast_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, in, n, (float*)out);
  return aw::check_launch("aw_cast");
}

extern "C" int aw_bn_finalize(const double* colstats, int64_t n, int H, const float* gamma, const float* beta,
                              float* running_mean, float* running_var, int64_t* nbt, float eps, float momentum,
                              int training, float* stats, void* stream) {
  AW_REQUIRE(stats && H > 0, "aw_bn_finalize: bad args");
  AW_REQUIRE(!training || colstats, "aw_bn_finalize: training needs colstats");
  AW_REQUIRE(!training || n > 1, "Expected more than 1 value per channel when training, got %lld", (long long)n);
  AW_REQUIRE(training || (running_mean && running_var), "aw_bn_finalize: eval needs running stats");
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(aw_cdiv(H, 256)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     colstats, n, H, gamma, beta, running_mean, running_var, nbt, eps, momentum, training, stats);
  return aw::check_launch("aw_bn_finalize");
}

extern "C" int aw_unpatch_head_fwd_ex(const void* yv, int y_dtype, int64_t R, int H, int Q, const float* stats,
                                      const float* w2, const float* b2, float* x_hat, void* stream) {
  AW_REQUIRE(yv && stats && w2 && b2 && x_hat && R >= 0 && Q > 0 && H > 0, "aw_unpatch_head_fwd: bad args");
  AW_REQUIRE(H % 4 == 0 && H <= 256 * HEAD_MAXV, "aw_unpatch_head_fwd: H must be a multiple of 4 and <= 1024");
  AW_REQUIRE(R % Q == 0, "aw_unpatch_head_fwd: rows must be whole windows");
  AW_REQUIRE(y_dtype == AW_F32 || y_dtype == AW_BF16, "aw_unpatch_head_fwd: bad y_dtype %d", y_dtype);
  if (R == 0) return AW_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // one resident round of workgroups: a grid larger than what fits at the kernel's occupancy runs a second, partly
  // filled round of row-loop waves (2048 workgroups at 5 waves/SIMD left ~40% of the chip idle in the tail)
  static const int fwd_wgs = [] {
    const char* e = getenv("AW_HEAD_FWD_WGS");
    if (e) return atoi(e);
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, head_fwd_kernel<2>, 256, 0) != hipSuccess)
      return 2048;
    return per > 0 && cus > 0 ? per * cus : 2048;
  }();
  dim3 grid(grid_for(R * 64, 256, fwd_wgs));
#define AW_HF(NSV, TY) \
  hipLaunchKernelGGL((head_fwd_kernel<NSV, TY>), grid, dim3(256), 0, s, (const TY*)yv, R, H, Q, stats, w2, b2, x_hat)
  const int ns = (H + 255) / 256;
  if (y_dtype == AW_BF16) {
    if (ns == 1) AW_HF(1, bf16); else if (ns == 2) AW_HF(2, bf16); else if (ns == 3) AW_HF(3, bf16); else AW_HF(4, bf16);
  } else {
    if (ns == 1) AW_HF(1, float); else if (ns == 2) AW_HF(2, float); else if (ns == 3) AW_HF(3, float); else AW_HF(4, float);
  }
#undef AW_HF
  return aw::check_launch("aw_unpatch_head_fwd");
}

extern "C" int aw_unpatch_head_fwd(const float* y, int64_t R, int H, int Q, const float* stats, const float* w2,
                                   const float* b2, float* x_hat, void* stream) {
  return aw_unpatch_head_fwd_ex(y, AW_F32, R, H, Q, stats, w2, b2, x_hat, stream);
}

extern "C" int aw_unpatch_head_bwd1_ex(const void* yv, int y_dtype, int64_t R, int H, int Q, const float* stats,
                                       const float* w2, const float* g_xhat, double* gsums, float* gw2, float* gb2,
                                       float* ggamma, float* gbeta, void* stream) {
  AW_REQUIRE(yv && stats && w2 && g_xhat && gsums && gw2 && gb2, "aw_unpatch_head_bwd1: null pointer");
  AW_REQUIRE(H % 4 == 0 && H <= 256 * HEAD_MAXV && R % Q == 0, "aw_unpatch_head_bwd1: bad shape");
  AW_REQUIRE(y_dtype == AW_F32 || (y_dtype == AW_BF16 && head_cs_ok(H)),
             "aw_unpatch_head_bwd1: y_dtype %d (bf16 y needs H a power of two in 64..2048)", y_dtype);
  if (R == 0) return AW_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t sh = 7 * H * sizeof(float);
  if (head_cs_ok(H)) {
    const dim3 g1(grid_for(R * (H / 2), 1024, head_wgs()));
#define AW_H1C(TY, UNI)                                                                                            \
  hipLaunchKernelGGL((head_bwd1_cs_kernel<TY, UNI>), g1, dim3(1024), sh, s, (const TY*)yv, R, H, Q, stats, w2, g_xhat, \
                     gsums, gw2, gb2, ggamma, gbeta)
    const bool uni = H >= 128;
    if (y_dtype == AW_BF16) {
      if (uni) AW_H1C(bf16, true); else AW_H1C(bf16, false);
    } else {
      if (uni) AW_H1C(float, true); else AW_H1C(float, false);
    }
#undef AW_H1C
    return aw::check_launch("aw_unpatch_head_bwd1");
  }
  const float* y = (const float*)yv;
  dim3 grid(grid_for(R * 64, 256, 512));
#define AW_H1(NSV) \
  hipLaunchKernelGGL(head_bwd1_kernel<NSV>, grid, dim3(256), sh, s, y, R, H, Q, stats, w2, g_xhat, gsums, gw2, gb2, \
                     ggamma, gbeta)
  switch ((H + 255) / 256) {
    case 1: AW_H1(1); break;
    case 2: AW_H1(2); break;
    case 3: AW_H1(3); break;
    default: AW_H1(4); break;
  }
#undef AW_H1
  return aw::check_launch("aw_unpatch_head_bwd1");
}

extern "C" int aw_unpatch_head_bwd1(const float* y, int64_t R, int H, int Q, const float* stats, const float* w2,
                                    const float* g_xhat, double* gsums, float* gw2, float* gb2, float* ggamma,
                                    float* gbeta, void* stream) {
  return aw_unpatch_head_bwd1_ex(y, AW_F32, R, H, Q, stats, w2, g_xhat, gsums, gw2, gb2, ggamma, gbeta, stream);
}

extern "C" int aw_unpatch_head_bwd2_ex(const void* yv, int y_dtype, int64_t R, int H, int Q, const float* stats,
                                       const float* w2, const float* g_xhat, const double* gsums, int training,
                                       void* g_y, int gy_dtype, float* db_y, void* stream) {
  AW_REQUIRE(yv && stats && w2 && g_xhat && gsums && g_y && db_y, "aw_unpatch_head_bwd2: null pointer");
  AW_REQUIRE(H % 4 == 0 && H <= 256 * HEAD_MAXV && R % Q == 0, "aw_unpatch_head_bwd2: bad shape");
  AW_REQUIRE(y_dtype == AW_F32 || (y_dtype == AW_BF16 && head_cs_ok(H)),
             "aw_unpatch_head_bwd2: y_dtype %d (bf16 y needs H a power of two in 64..2048)", y_dtype);
  if (R == 0) return AW_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t sh = H * sizeof(float);
  if (H == 512 && R * 512 * (y_dtype == AW_F32 ? 4 : 2) < (1ll << 31)) {
    const dim3 g2((unsigned)std::max<int64_t>(1, std::min<int64_t>(head_cus(), (R + HB * HFW - 1) / (HB * HFW))));
#define AW_H2R(T, TY)                                                                                              \
  hipLaunchKernelGGL((head_bwd2_rows_kernel<T, TY>), g2, dim3(64 * HFW), 0, s, (const TY*)yv, R, stats, w2, g_xhat, \
                     gsums, training, (T*)g_y, db_y)
    if (gy_dtype == AW_BF16) {
      if (y_dtype == AW_BF16) AW_H2R(bf16, bf16); else AW_H2R(bf16, float);
    } else {
      if (y_dtype == AW_BF16) AW_H2R(float, bf16); else AW_H2R(float, float);
    }
#undef AW_H2R
    return aw::check_launch("aw_unpatch_head_bwd2");
  }
  if (head_cs_ok(H)) {
    dim3 g2(grid_for(R * (H / 2), 1024, head_wgs()));
#define AW_H2C(T, TY)                                                                                               \
  do {                                                                                                              \
    if (H >= 128)                                                                                                   \
      hipLaunchKernelGGL((head_bwd2_cs_kernel<T, TY, true>), g2, dim3(1024), sh, s, (const TY*)yv, R, H, Q, stats,  \
                         w2, g_xhat, gsums, training, (T*)g_y, db_y);                                               \
    else                                                                                                            \
      hipLaunchKernelGGL((head_bwd2_cs_kernel<T, TY, false>), g2, dim3(1024), sh, s, (const TY*)yv, R, H, Q, stats, \
                         w2, g_xhat, gsums, training, (T*)g_y, db_y);                                               \
  } while (0)
    if (gy_dtype == AW_BF16) {
      if (y_dtype == AW_BF16) AW_H2C(bf16, bf16); else AW_H2C(bf16, float);
    } else {
      if (y_dtype == AW_BF16) AW_H2C(float, bf16); else AW_H2C(float, float);
    }
#undef AW_H2C
    return aw::check_launch("aw_unpatch_head_bwd2");
  }
  const float* y = (const float*)yv;
  dim3 grid(grid_for(R * 64, 256, 1024));
#define AW_H2(TY, NSV) \
  hipLaunchKernelGGL((head_bwd2_kernel<TY, NSV>), grid, dim3(256), sh, s, y, R, H, Q, stats, w2, g_xhat, gsums, \
                     training, (TY*)g_y, db_y)
  const int ns = (H + 255) / 256;
  if (gy_dtype == AW_BF16) {
    if (ns == 1) AW_H2(bf16, 1); else if (ns == 2) AW_H2(bf16, 2); else if (ns == 3) AW_H2(bf16, 3); else AW_H2(bf16, 4);
  } else {
    if (ns == 1) AW_H2(float, 1); else if (ns == 2) AW_H2(float, 2); else if (ns == 3) AW_H2(float, 3); else AW_H2(float, 4);
  }
#undef AW_H2
  return aw::check_launch("aw_unpatch_head_bwd2");
}

extern "C" int aw_unpatch_head_fwd_bwd1(const void* yv, int y_dtype, int64_t R, int H, int Q, const float* stats,
                                        const float* w2, const float* b2, const float* x, const float* gscale,
                                        float* x_hat, float* g_xhat, double* sqerr, double* gsums, float* gw2,
                                        float* gb2, float* ggamma, float* gbeta, void* stream) {
  AW_REQUIRE(yv && stats && w2 && b2 && x && gscale && x_hat && g_xhat && sqerr && gsums && gw2 && gb2,
             "aw_unpatch_head_fwd_bwd1: null pointer");
  AW_REQUIRE(H == 512 && Q > 0 && R % Q == 0, "aw_unpatch_head_fwd_bwd1: needs H == 512 and whole windows");
  AW_REQUIRE(y_dtype == AW_F32 || y_dtype == AW_BF16, "aw_unpatch_head_fwd_bwd1: bad y_dtype %d", y_dtype);
  AW_REQUIRE(R * 512 * (y_dtype == AW_F32 ? 4 : 2) < (1ll << 31), "aw_unpatch_head_fwd_bwd1: y exceeds 2 GiB");
  if (R == 0) return AW_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(head_cus(), (R + HB * HFW - 1) / (HB * HFW))));
  const float gmul = 2.0f / (float)(R * 5);   // aw_mse_bwd: 2 / numel
  if (y_dtype == AW_BF16)
    hipLaunchKernelGGL(head_fwd_bwd1_kernel<bf16>, grid, dim3(64 * HFW), 0, s, (const bf16*)yv, R, stats, w2, b2, x,
                       gscale, gmul, x_hat, g_xhat, sqerr, gsums, gw2, gb2, ggamma, gbeta);
  else
    hipLaunchKernelGGL(head_fwd_bwd1_kernel<float>, grid, dim3(64 * HFW), 0, s, (const float*)yv, R, stats, w2, b2, x,
                       gscale, gmul, x_hat, g_xhat, sqerr, gsums, gw2, gb2, ggamma, gbeta);
  return aw::check_launch("aw_unpatch_head_fwd_bwd1");
}

extern "C" int aw_unpatch_head_bwd2(const float* y, int64_t R, int H, int Q, const float* stats, const float* w2,
                                    const float* g_xhat, const double* gsums, int training, void* g_y, int gy_dtype,
                                    float* db_y, void* stream) {
  return aw_unpatch_head_bwd2_ex(y, AW_F32, R, H, Q, stats, w2, g_xhat, gsums, training, g_y, gy_dtype, db_y,
                                 stream);
}

extern "C" int aw_mse_fwd(const float* a, const float* b, int64_t n, double* sqerr, void* stream) {
  AW_REQUIRE(a && b && sqerr && n >= 0, "aw_mse_fwd: bad args");
  if (n == 0) return AW_OK;
  // few workgroups: each ends with one f64 atomic on the same address (1024 of them serialised into ~14 us)
  const int64_t n4 = (((uintptr_t)a | (uintptr_t)b) & 15) ? 0 : n / 4;
  hipLaunchKernelGGL(mse_fwd_kernel, dim3(grid_for(n4 ? n4 : n, 256, 64)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), a, b, n, n4, sqerr);
  return aw::check_launch("aw_mse_fwd");
}

extern "C" int aw_mse_bwd(const float* a, const float* b, int64_t n, const float* g, float* ga, void* stream) {
  AW_REQUIRE(a && b && g && ga && n >= 0, "aw_mse_bwd: bad args");
  if (n == 0) return AW_OK;
  hipLaunchKernelGGL(mse_bwd_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     a, b, n, g, ga);
  return aw::check_launch("aw_mse_bwd");
}

extern "C" int aw_scalar_add(const float* a, const float* b, float* out, void* stream) {
  AW_REQUIRE(a && b && out, "aw_scalar_add: null pointer");
  hipLaunchKernelGGL(scalar_add_kernel, dim3(1), dim3(1), 0, reinterpret_cast<hipStream_t>(stream), a, b, out);
  return aw::check_launch("aw_scalar_add");
}

extern "C" int aw_mse_finalize(const double* sqerr, int64_t numel, float* out, void* stream) {
  AW_REQUIRE(sqerr && out && numel > 0, "aw_mse_finalize: bad args");
  hipLaunchKernelGGL(mse_finalize_kernel, dim3(1), dim3(1), 0, reinterpret_cast<hipStream_t>(stream), sqerr, numel, out);
  return aw::check_launch("aw_mse_finalize");
}

extern "C" int aw_mse_finalize_add(const double* sqerr, int64_t numel, const float* addend, float* out, float* sum,
                                   void* stream) {
  AW_REQUIRE(sqerr && addend && out && sum && numel > 0, "aw_mse_finalize_add: bad args");
  hipLaunchKernelGGL(mse_finalize_add_kernel, dim3(1), dim3(1), 0, reinterpret_cast<hipStream_t>(stream), sqerr, numel,
                     addend, out, sum);
  return aw::check_launch("aw_mse_finalize_add");
}
