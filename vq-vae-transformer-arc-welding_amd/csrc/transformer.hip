// Latent-Transformer kernels (model/transformer_block.py, model/transformer_decoder.py, model/embedding.py)
// for gfx950: LayerNorm, token+position embedding, causal attention (flash-style: the T x T score matrix is
// never materialised, softmax statistics are kept per query row and the backward recomputes P from the
// saved log-sum-exp), and cross-entropy with ignore_index.
#include <stdlib.h>

#include "common.h"
#include <algorithm>

namespace aw {  // attention.hip: MFMA path for bf16, head size 64
bool attn_mfma_supported(int dtype, int hs, int d, int64_t T);
void attn_fwd_mfma(const void* qkv, int64_t B, int T, int nh, int d, void* y, float* lse, hipStream_t s);
void attn_bwd_mfma(const void* qkv, const void* y, const void* dy, const float* lse, float* delta, int64_t B, int T,
                   int nh, int d, void* dqkv, hipStream_t s);   // delta computed by its dQ launch
}  // namespace aw

#ifndef AW_ATOMIC_ROTATE
#define AW_ATOMIC_ROTATE 1
#endif

namespace {

// ---------------------------------------------------------------- LayerNorm (one wave per row)
template <typename T>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ x, int64_t R, int D,
                                                     const float* __restrict__ w, const float* __restrict__ b,
                                                     float eps, T* __restrict__ y, float* __restrict__ mean,
                                                     float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= R) return;
  const float* xr = x + r * D;
  float s = 0.f;
  for (int i = lane; i < D; i += 64) s += xr[i];
  const float mu = wave_sum(s) / (float)D;
  float v = 0.f;
  for (int i = lane; i < D; i += 64) {
    const float d = xr[i] - mu;
    v += d * d;
  }
  const float rs = rsqrtf(wave_sum(v) / (float)D + eps);
  for (int i = lane; i < D; i += 64) y[r * D + i] = from_f32<T>((xr[i] - mu) * rs * w[i] + b[i]);
  if (lane == 0) {
    mean[r] = mu;
    rstd[r] = rs;
  }
}

template <typename T2>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                     int64_t R, int D, const float* __restrict__ w,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     float* __restrict__ dx, int accumulate, float* __restrict__ dw,
                                                     float* __restrict__ db, T2* __restrict__ dx2, float drop_p,
                                                     uint64_t drop_seed, const uint64_t* __restrict__ seed_ptr) {
  drop_seed = aw_seed_mix(drop_seed, seed_ptr);
  extern __shared__ float red[];  // 2*D
  for (int i = threadIdx.x; i < 2 * D; i += blockDim.x) red[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = wave; r < R; r += nw) {
    const float mu = mean[r], rs = rstd[r];
    const float* xr = x + r * D;
    const float* dyr = dy + r * D;
    float s1 = 0.f, s2 = 0.f;
    for (int i = lane; i < D; i += 64) {
      const float xh = (xr[i] - mu) * rs;
      const float g = dyr[i] * w[i];
      s1 += g;
      s2 += g * xh;
      atomicAdd(&red[i], dyr[i] * xh);
      atomicAdd(&red[D + i], dyr[i]);
    }
    s1 = wave_sum(s1) / (float)D;
    s2 = wave_sum(s2) / (float)D;
    for (int i = lane; i < D; i += 64) {
      const float xh = (xr[i] - mu) * rs;
      const float g = dyr[i] * w[i];
      float v = rs * (g - s1 - xh * s2);
      if (accumulate) v += dx[r * D + i];
      dx[r * D + i] = v;
      if (dx2) dx2[r * D + i] = from_f32<T2>(v * aw_dropout_scale(drop_seed, (uint64_t)r * D + i, drop_p));
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < D; i += blockDim.x) {
    atomicAdd(dw + i, red[i]);
    atomicAdd(db + i, red[D + i]);
  }
}

// Vectorised forms for D % 256 == 0 (d_model 512): lane owns float4 columns 4*lane + 256*j, j < NV; the row
// statistics come from one pass over registers.  Backward keeps the dw/db partial sums of its columns in
// registers across all rows the wave visits, then reduces the block's waves through LDS: one atomic per
// column per block instead of two LDS atomics per element.
template <typename T, int NV>
__global__ __launch_bounds__(256) void ln_fwd_vec_kernel(const float* __restrict__ x, int64_t R, int D,
                                                         const float* __restrict__ w, const float* __restrict__ b,
                                                         float eps, T* __restrict__ y, float* __restrict__ mean,
                                                         float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= R) return;
  float4 v[NV], w4[NV], b4[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = *reinterpret_cast<const float4*>(x + r * D + 4 * lane + 256 * j);
  // the affine parameters load beside the row (issued after the load of x, waited for only after the reductions;
  // loaded after the reductions, their latency followed the two wave sums of every row)
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    w4[j] = *reinterpret_cast<const float4*>(w + 4 * lane + 256 * j);
    b4[j] = *reinterpret_cast<const float4*>(b + 4 * lane + 256 * j);
  }
  __builtin_amdgcn_sched_barrier(0);   // keep the loads issued here, ahead of the reductions
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
  const float mu = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const float a = v[j].x - mu, bb = v[j].y - mu, c = v[j].z - mu, e = v[j].w - mu;
    q += (a * a + bb * bb) + (c * c + e * e);
  }
  const float rs = rsqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = 4 * lane + 256 * j;
    const float o[4] = {(v[j].x - mu) * rs * w4[j].x + b4[j].x, (v[j].y - mu) * rs * w4[j].y + b4[j].y,
                        (v[j].z - mu) * rs * w4[j].z + b4[j].z, (v[j].w - mu) * rs * w4[j].w + b4[j].w};
    if constexpr (sizeof(T) == 2) {
      bf16 h[4] = {(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
      uint2 u;
      memcpy(&u, h, 8);
      *reinterpret_cast<uint2*>(y + r * D + c) = u;
    } else {
      *reinterpret_cast<float4*>(y + r * D + c) = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
  if (lane == 0) {
    mean[r] = mu;
    rstd[r] = rs;
  }
}

template <typename T2, int NV>
__global__ __launch_bounds__(512) void ln_bwd_vec_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                         int64_t R, int D, const float* __restrict__ w,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, float* __restrict__ dx,
                                                         int accumulate, float* __restrict__ dw,
                                                         float* __restrict__ db, T2* __restrict__ dx2, float drop_p,
                                                         uint64_t drop_seed, const uint64_t* __restrict__ seed_ptr) {
  // per-wave dw / db partials [wave][2][256 NV] (dynamic: blockDim.x / 64 waves), reduced in wave order at the end
  extern __shared__ float red[];
  const int nwv = blockDim.x >> 6;
  drop_seed = aw_seed_mix(drop_seed, seed_ptr);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  float4 w4[NV], pdw[NV], pdb[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    w4[j] = *reinterpret_cast<const float4*>(w + 4 * lane + 256 * j);
    pdw[j] = pdb[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // Each wave walks ~R/nw rows; the next row's x / dy / statistics are loaded before this row's two wave
  // reductions and stores, so the loads stay in flight across the dependent work.
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  float4 xc[NV], dc[NV], oc[NV];
  float muc = 0.f, rsc = 0.f;
  if (wave < R) {
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      xc[j] = *reinterpret_cast<const float4*>(x + wave * D + 4 * lane + 256 * j);
      dc[j] = *reinterpret_cast<const float4*>(dy + wave * D + 4 * lane + 256 * j);
      oc[j] = accumulate ? *reinterpret_cast<const float4*>(dx + wave * D + 4 * lane + 256 * j) : z4;
    }
    muc = mean[wave];
    rsc = rstd[wave];
  }
  for (int64_t r = wave; r < R; r += nw) {
    const float mu = muc, rs = rsc;
    float4 xcur[NV], dcur[NV], ocur[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      xcur[j] = xc[j];
      dcur[j] = dc[j];
      ocur[j] = oc[j];
    }
    const int64_t rn = r + nw;
    if (rn < R) {
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        xc[j] = *reinterpret_cast<const float4*>(x + rn * D + 4 * lane + 256 * j);
        dc[j] = *reinterpret_cast<const float4*>(dy + rn * D + 4 * lane + 256 * j);
        oc[j] = accumulate ? *reinterpret_cast<const float4*>(dx + rn * D + 4 * lane + 256 * j) : z4;
      }
      muc = mean[rn];
      rsc = rstd[rn];
    }
    float4 xh[NV], g[NV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const float4 xv = xcur[j];
      const float4 dv = dcur[j];
      xh[j] = make_float4((xv.x - mu) * rs, (xv.y - mu) * rs, (xv.z - mu) * rs, (xv.w - mu) * rs);
      g[j] = make_float4(dv.x * w4[j].x, dv.y * w4[j].y, dv.z * w4[j].z, dv.w * w4[j].w);
      pdw[j].x += dv.x * xh[j].x; pdw[j].y += dv.y * xh[j].y; pdw[j].z += dv.z * xh[j].z; pdw[j].w += dv.w * xh[j].w;
      pdb[j].x += dv.x; pdb[j].y += dv.y; pdb[j].z += dv.z; pdb[j].w += dv.w;
      s1 += (g[j].x + g[j].y) + (g[j].z + g[j].w);
      s2 += (g[j].x * xh[j].x + g[j].y * xh[j].y) + (g[j].z * xh[j].z + g[j].w * xh[j].w);
    }
    s1 = wave_sum(s1) / (float)D;
    s2 = wave_sum(s2) / (float)D;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c = 4 * lane + 256 * j;
      float v[4] = {rs * (g[j].x - s1 - xh[j].x * s2), rs * (g[j].y - s1 - xh[j].y * s2),
                    rs * (g[j].z - s1 - xh[j].z * s2), rs * (g[j].w - s1 - xh[j].w * s2)};
      if (accumulate) {
        v[0] += ocur[j].x; v[1] += ocur[j].y; v[2] += ocur[j].z; v[3] += ocur[j].w;
      }
      *reinterpret_cast<float4*>(dx + r * D + c) = make_float4(v[0], v[1], v[2], v[3]);
      if (dx2) {
        float m[4] = {v[0], v[1], v[2], v[3]};
        if (drop_p > 0.f) {
          float ds[4];
          aw_dropout_scale4(drop_seed, (uint64_t)r * D + c, drop_p, ds);
#pragma unroll
          for (int e = 0; e < 4; ++e) m[e] *= ds[e];
        }
        if constexpr (sizeof(T2) == 2) {
          bf16 h[4] = {(bf16)m[0], (bf16)m[1], (bf16)m[2], (bf16)m[3]};
          uint2 u;
          memcpy(&u, h, 8);
          *reinterpret_cast<uint2*>(dx2 + r * D + c) = u;
        } else {
          *reinterpret_cast<float4*>(dx2 + r * D + c) = make_float4(m[0], m[1], m[2], m[3]);
        }
      }
    }
  }
  constexpr int C = 256 * NV;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    *reinterpret_cast<float4*>(&red[(wv * 2 + 0) * C + 4 * lane + 256 * j]) = pdw[j];
    *reinterpret_cast<float4*>(&red[(wv * 2 + 1) * C + 4 * lane + 256 * j]) = pdb[j];
  }
  __syncthreads();
  // every workgroup adds into the same 2C addresses: each starts its walk at its own offset, so that at any moment
  // they queue on different addresses (AW_ATOMIC_ROTATE=0 in the build: all from column 0)
  for (int i0 = threadIdx.x; i0 < C; i0 += blockDim.x) {
#if AW_ATOMIC_ROTATE
    const int i = (i0 + (int)(blockIdx.x & 7) * (C / 8)) % C;
#else
    const int i = i0;
#endif
    float a = 0.f, b = 0.f;
    for (int v = 0; v < nwv; ++v) {
      a += red[(v * 2 + 0) * C + i];
      b += red[(v * 2 + 1) * C + i];
    }
    atomicAdd(dw + i, a);
    atomicAdd(db + i, b);
  }
}

// ---------------------------------------------------------------- embedding (model/embedding.py:57-59)
__global__ void embed_fwd_kernel(const int64_t* __restrict__ ids, int64_t B, int T, int D,
                                 const float* __restrict__ wtok, const float* __restrict__ pe, float* __restrict__ x) {
  const int64_t n = B * T * D;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / D;
    const int i = (int)(e - r * D);
    const int t = (int)(r % T);
    x[e] = wtok[ids[r] * D + i] + pe[(int64_t)t * D + i];
  }
}

// Vectorised form (D % 4 == 0, 16-B aligned tables): one wave per row, float4 columns; the row's id and position are
// computed once per row instead of per element (the element-wise form: 21 us at 16371 x 512, 1.6 TB/s).
__global__ __launch_bounds__(256) void embed_fwd_rows_kernel(const int64_t* __restrict__ ids, int64_t R, int T, int D,
                                                             const float* __restrict__ wtok,
                                                             const float* __restrict__ pe, float* __restrict__ x) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int d4 = D >> 2;
  for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < R; r += nw) {
    const float4* a = reinterpret_cast<const float4*>(wtok + ids[r] * D);
    const float4* b = reinterpret_cast<const float4*>(pe + (r % T) * D);
    float4* o = reinterpret_cast<float4*>(x + r * D);
    for (int c = lane; c < d4; c += 64) {
      const float4 u = a[c], v = b[c];
      o[c] = make_float4(u.x + v.x, u.y + v.y, u.z + v.z, u.w + v.w);
    }
  }
}

// The embedding with the first block's ln_1 fused (D = 256 NV, one wave per row): x = wtok[id] + pe[t] as
// embed_fwd_rows_kernel, then LayerNorm(x) from the same registers, in ln_fwd_vec_kernel's order of operations
// (bit-identical to the two launches; the LayerNorm's read of x is saved)
template <typename T, int NV>
__global__ __launch_bounds__(256) void embed_ln_fwd_kernel(const int64_t* __restrict__ ids, int64_t R, int Tn, int D,
                                                           const float* __restrict__ wtok, const float* __restrict__ pe,
                                                           float* __restrict__ x, const float* __restrict__ w,
                                                           const float* __restrict__ b, float eps, T* __restrict__ y,
                                                           float* __restrict__ mean, float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63;
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= R) return;
  const float* a = wtok + ids[r] * D;
  const float* p = pe + (r % Tn) * D;
  float4 v[NV], w4[NV], b4[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const float4 u = *reinterpret_cast<const float4*>(a + 4 * lane + 256 * j);
    const float4 q = *reinterpret_cast<const float4*>(p + 4 * lane + 256 * j);
    v[j] = make_float4(u.x + q.x, u.y + q.y, u.z + q.z, u.w + q.w);
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    w4[j] = *reinterpret_cast<const float4*>(w + 4 * lane + 256 * j);
    b4[j] = *reinterpret_cast<const float4*>(b + 4 * lane + 256 * j);
    *reinterpret_cast<float4*>(x + r * D + 4 * lane + 256 * j) = v[j];
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
  const float mu = wave_sum(s) / (float)D;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const float a0 = v[j].x - mu, a1 = v[j].y - mu, a2 = v[j].z - mu, a3 = v[j].w - mu;
    q += (a0 * a0 + a1 * a1) + (a2 * a2 + a3 * a3);
  }
  const float rs = rsqrtf(wave_sum(q) / (float)D + eps);
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = 4 * lane + 256 * j;
    const float o[4] = {(v[j].x - mu) * rs * w4[j].x + b4[j].x, (v[j].y - mu) * rs * w4[j].y + b4[j].y,
                        (v[j].z - mu) * rs * w4[j].z + b4[j].z, (v[j].w - mu) * rs * w4[j].w + b4[j].w};
    if constexpr (sizeof(T) == 2) {
      bf16 h[4] = {(bf16)o[0], (bf16)o[1], (bf16)o[2], (bf16)o[3]};
      uint2 u;
      memcpy(&u, h, 8);
      *reinterpret_cast<uint2*>(y + r * D + c) = u;
    } else {
      *reinterpret_cast<float4*>(y + r * D + c) = make_float4(o[0], o[1], o[2], o[3]);
    }
  }
  if (lane == 0) {
    mean[r] = mu;
    rstd[r] = rs;
  }
}

__global__ void embed_bwd_kernel(const int64_t* __restrict__ ids, int64_t B, int T, int D, const float* __restrict__ dx,
                                 float* __restrict__ dw) {
  const int64_t n = B * T * D;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / D;
    atomicAdd(dw + ids[r] * D + (e - r * D), dx[e]);
  }
}

// One workgroup per row (grid-stride): the row's id is one scalar load, its D columns are consecutive lanes (every
// wave-instruction of atomics covers 256 contiguous bytes), and there is no per-element 64-bit division or id load.
__global__ __launch_bounds__(256) void embed_bwd_rows_kernel(const int64_t* __restrict__ ids, int64_t R, int D,
                                                             const float* __restrict__ dx, float* __restrict__ dw) {
  for (int64_t r = blockIdx.x; r < R; r += gridDim.x) {
    const float* src = dx + r * D;
    float* dst = dw + ids[r] * D;
    for (int c = threadIdx.x; c < D; c += blockDim.x) atomicAdd(dst + c, src[c]);
  }
}

// The table gradient without global atomics (the decoder's ~32 rows per table row made the atomic form contend on the
// same addresses: 46.7 us per decoder step for 16371 x 512).  (1) One workgroup counting-sorts the row indices by
// id in LDS: off[v] .. off[v + 1] - 1 are the slots of ord holding the rows of table row v (ids outside [0, V) are
// dropped).  (2) One workgroup per table row sums its rows' gradients in registers and adds the sum to the table row with
// one plain read-modify-write (each element has one owner).  The order of a row's terms follows the
// sort's LDS atomics, so -- as with the atomic form -- the f32 summation order is not fixed from run to run.
constexpr int ESORT_THREADS = 1024;
constexpr int ESORT_MAX_V = 15360;   // LDS: (V + 1024) ints, within 64 KB of dynamic LDS
constexpr int ESORT_U = 8;           // ids in flight per thread (the loads go out before the LDS atomics)

__global__ __launch_bounds__(ESORT_THREADS) void embed_sort_kernel(const int64_t* __restrict__ ids, int R, int V,
                                                                   int* __restrict__ off, int* __restrict__ ord) {
  extern __shared__ int esh[];
  int* cnt = esh;
  int* part = esh + V;
  const int tid = threadIdx.x;
  for (int i = tid; i < V; i += ESORT_THREADS) cnt[i] = 0;
  __syncthreads();
  for (int r0 = tid; r0 < R; r0 += ESORT_U * ESORT_THREADS) {
    int64_t v[ESORT_U];
#pragma unroll
    for (int u = 0; u < ESORT_U; ++u) {   // clamped address, then a select: no branch (and wait) per load
      const int r = r0 + u * ESORT_THREADS;
      const int64_t x = ids[min(r, R - 1)];
      v[u] = r < R ? x : -1;
    }
#pragma unroll
    for (int u = 0; u < ESORT_U; ++u)
      if ((uint64_t)v[u] < (uint64_t)V) atomicAdd(&cnt[v[u]], 1);
  }
  __syncthreads();
  // exclusive scan of the counts: a serial chunk per thread, then the 1024 chunk sums
  const int per = (V + ESORT_THREADS - 1) / ESORT_THREADS, b0 = min(V, tid * per), b1 = min(V, b0 + per);
  int s = 0;
  for (int i = b0; i < b1; ++i) s += cnt[i];
  part[tid] = s;
  __syncthreads();
  for (int o = 1; o < ESORT_THREADS; o <<= 1) {
    const int add = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += add;
    __syncthreads();
  }
  int run = part[tid] - s;
  for (int i = b0; i < b1; ++i) {
    const int c = cnt[i];
    off[i] = run;
    cnt[i] = run;   // becomes the row's fill cursor
    run += c;
  }
  if (tid == ESORT_THREADS - 1) off[V] = part[ESORT_THREADS - 1];
  __syncthreads();
  for (int r0 = tid; r0 < R; r0 += ESORT_U * ESORT_THREADS) {
    int64_t v[ESORT_U];
#pragma unroll
    for (int u = 0; u < ESORT_U; ++u) {   // clamped address, then a select: no branch (and wait) per load
      const int r = r0 + u * ESORT_THREADS;
      const int64_t x = ids[min(r, R - 1)];
      v[u] = r < R ? x : -1;
    }
#pragma unroll
    for (int u = 0; u < ESORT_U; ++u)
      if ((uint64_t)v[u] < (uint64_t)V) ord[atomicAdd(&cnt[v[u]], 1)] = r0 + u * ESORT_THREADS;
  }
}

// One workgroup (4 waves) per table row v, D = 256 NV: wave w sums the row's entries w, w + 4, ... (8 at a time; lane: float4
// columns 4 lane + 256 j); the segment's row indices come 64 at a time in one load and are read per entry from a
// lane (no dependent index load per entry); the 4 partial sums meet in LDS and one read-modify-write adds them.
constexpr int ESEG_U = 8;   // entries in flight per wave (the decoder's ~32 rows per table row: one round per wave)
template <int NV>
__global__ __launch_bounds__(256) void embed_segsum_kernel(const int* __restrict__ off, const int* __restrict__ ord,
                                                           int D, const float* __restrict__ dx,
                                                           float* __restrict__ dw) {
  __shared__ float4 red[3][64 * NV];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int v = blockIdx.x;
  const int i0 = off[v], i1 = off[v + 1];
  if (i0 == i1) return;   // workgroup-uniform
  float4 a[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) a[j] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int b0 = i0; b0 < i1; b0 += 64) {
    const int n = min(64, i1 - b0);
    const int myr = lane < n ? ord[b0 + lane] : 0;
    for (int e = w; e < n; e += 4 * ESEG_U) {
      float4 u[ESEG_U][NV];
#pragma unroll
      for (int k = 0; k < ESEG_U; ++k) {
        const int ek = e + 4 * k;
        // past the segment: the entry's own row again, its value dropped by a select (a branch around each load
        // made every load wait for the one before)
        const int r = __shfl(myr, ek < n ? ek : e, 64);
        const float m = ek < n ? 1.f : 0.f;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          const float4 x = *reinterpret_cast<const float4*>(dx + (int64_t)r * D + 4 * lane + 256 * j);
          u[k][j] = make_float4(x.x * m, x.y * m, x.z * m, x.w * m);
        }
      }
#pragma unroll
      for (int k = 0; k < ESEG_U; ++k)
#pragma unroll
        for (int j = 0; j < NV; ++j)
          a[j] = make_float4(a[j].x + u[k][j].x, a[j].y + u[k][j].y, a[j].z + u[k][j].z, a[j].w + u[k][j].w);
    }
  }
  if (w > 0)
#pragma unroll
    for (int j = 0; j < NV; ++j) red[w - 1][64 * j + lane] = a[j];
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const float4 p1 = red[0][64 * j + lane], p2 = red[1][64 * j + lane], p3 = red[2][64 * j + lane];
      float4* o = reinterpret_cast<float4*>(dw + (int64_t)v * D + 4 * lane + 256 * j);
      const float4 p = *o;
      *o = make_float4(p.x + ((a[j].x + p1.x) + (p2.x + p3.x)), p.y + ((a[j].y + p1.y) + (p2.y + p3.y)),
                       p.z + ((a[j].z + p1.z) + (p2.z + p3.z)), p.w + ((a[j].w + p1.w) + (p2.w + p3.w)));
    }
  }
}

// ---------------------------------------------------------------- causal attention
// Two lanes per query (or key) row, each holding half of the head dimension; partial dot products are combined
// with one xor-1 shuffle.  Key/value (resp. query) tiles of 32 rows are staged in LDS and read as broadcasts.
// 64 rows per 128-thread workgroup; grid = (ceil(T/64), n_head, B).  EXACT kernels are compiled for head sizes
// 16/32/64/128; any other head size (hs <= 128, e.g. d_model 32 with 4 heads) runs the HS-capacity kernel with
// the runtime size: lane 0 of a pair holds ceil(hs/2) values, lane 1 the rest.
constexpr int ATT_ROWS = 64;
constexpr int ATT_TILE = 32;

template <int HS, bool EXACT> struct HeadSplit {
  int hs, h2, mine, off;    // head size, lane-0 share, this lane's share, this lane's first element
  __device__ __forceinline__ HeadSplit(int hs_rt, int half) {
    hs = EXACT ? HS : hs_rt;
    h2 = EXACT ? HS / 2 : (hs + 1) / 2;
    mine = half ? hs - h2 : h2;
    off = half * h2;
  }
  __device__ __forceinline__ bool has(int e) const { return EXACT || e < mine; }
};

// Attention-probability dropout (CausalSelfAttention.attn_dropout, model/transformer_block.py:44-57; DROP): P_ij of
// (b, h) is kept with probability 1 - p and scaled by 1/(1 - p), the mask of element ((b*nh + h)*T + i)*T + j
// regenerated from (seed, element) by the backward; the row normaliser and delta_i = dy_i . y_i are unchanged.
struct AttnDrop {
  float p;
  uint64_t seed;
  __device__ __forceinline__ float scale(int64_t bh, int T_, int i, int j) const {
    return aw_dropout_scale(seed, ((uint64_t)bh * T_ + i) * T_ + j, p);
  }
};

template <typename T, int HS, bool EXACT = true, bool DROP = false>
__global__ __launch_bounds__(128) void attn_fwd_kernel(const T* __restrict__ qkv, int T_, int nh, int d, int hs_rt,
                                                       T* __restrict__ y, float* __restrict__ lse, float scale,
                                                       float drop_p, uint64_t drop_seed,
                                                       const uint64_t* __restrict__ seed_ptr) {
  constexpr int H2 = HS / 2;
  __shared__ float Ks[ATT_TILE][HS + 1];
  __shared__ float Vs[ATT_TILE][HS + 1];
  const int b = blockIdx.z, h = blockIdx.y;
  const int tid = threadIdx.x, half = tid & 1;
  const HeadSplit<HS, EXACT> hd(hs_rt, half);
  const int hs = hd.hs;
  const int qi = blockIdx.x * ATT_ROWS + (tid >> 1);
  const int64_t ld = 3 * (int64_t)d;
  const T* base = qkv + (int64_t)b * T_ * ld;
  const bool valid = qi < T_;
  AttnDrop dr{drop_p, DROP ? aw_seed_mix(drop_seed, seed_ptr) : 0ull};
  const int64_t bh = (int64_t)b * nh + h;
  float q[H2], o[H2];
#pragma unroll
  for (int e = 0; e < H2; ++e) {
    q[e] = valid && hd.has(e) ? to_f32<T>(base[(int64_t)qi * ld + h * hs + hd.off + e]) * scale : 0.f;
    o[e] = 0.f;
  }
  float m = -__builtin_huge_valf(), l = 0.f;
  const int kend = min(T_, (blockIdx.x + 1) * ATT_ROWS);  // keys beyond the block's last query are masked
  for (int k0 = 0; k0 < kend; k0 += ATT_TILE) {
    __syncthreads();
    for (int i = tid; i < ATT_TILE * hs; i += 128) {
      const int kr = i / hs, e = i - kr * hs;
      const int kk = k0 + kr;
      float kv = 0.f, vv = 0.f;
      if (kk < T_) {
        kv = to_f32<T>(base[(int64_t)kk * ld + d + h * hs + e]);
        vv = to_f32<T>(base[(int64_t)kk * ld + 2 * d + h * hs + e]);
      }
      Ks[kr][e] = kv;
      Vs[kr][e] = vv;
    }
    __syncthreads();
    float s[ATT_TILE];
    float tmax = -__builtin_huge_valf();
#pragma unroll
    for (int j = 0; j < ATT_TILE; ++j) {
      float a = 0.f;
#pragma unroll
      for (int e = 0; e < H2; ++e)
        if (hd.has(e)) a = fmaf(q[e], Ks[j][hd.off + e], a);
      a += __shfl_xor(a, 1, 64);
      const bool ok = (k0 + j) <= qi && (k0 + j) < T_;
      s[j] = ok ? a : -__builtin_huge_valf();
      tmax = fmaxf(tmax, s[j]);
    }
    const float mn = fmaxf(m, tmax);
    if (mn == -__builtin_huge_valf()) continue;  // nothing visible yet (padded row)
    const float corr = __expf(m - mn);
    l *= corr;
#pragma unroll
    for (int e = 0; e < H2; ++e) o[e] *= corr;
#pragma unroll
    for (int j = 0; j < ATT_TILE; ++j) {
      const float pj = __expf(s[j] - mn);
      l += pj;
      const float pv = DROP ? pj * dr.scale(bh, T_, qi, k0 + j) : pj;
#pragma unroll
      for (int e = 0; e < H2; ++e)
        if (hd.has(e)) o[e] = fmaf(pv, Vs[j][hd.off + e], o[e]);
    }
    m = mn;
  }
  if (!valid) return;
  const float inv = 1.f / l;
  T* yr = y + ((int64_t)b * T_ + qi) * d + h * hs + hd.off;
#pragma unroll
  for (int e = 0; e < H2; ++e)
    if (hd.has(e)) yr[e] = from_f32<T>(o[e] * inv);
  if (half == 0) lse[((int64_t)b * nh + h) * T_ + qi] = m + logf(l);
}

// delta_i = sum_e dy_i,e * y_i,e   (per (b, h, i))
template <typename T>
__global__ void attn_delta_kernel(const T* __restrict__ y, const T* __restrict__ dy, int64_t B, int T_, int nh, int d,
                                  float* __restrict__ delta) {
  const int64_t n = B * nh * T_;
  const int hs = d / nh;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t bh = r / T_;
    const int t = (int)(r - bh * T_);
    const int64_t b = bh / nh;
    const int h = (int)(bh - b * nh);
    const int64_t off = (b * T_ + t) * d + h * hs;
    float s = 0.f;
#pragma unroll 8
    for (int e = 0; e < hs; ++e) s += to_f32<T>(dy[off + e]) * to_f32<T>(y[off + e]);
    delta[r] = s;
  }
}

// dq_i = scale * sum_{j<=i} P_ij (dP_ij - delta_i) k_j     (query-stationary)
template <typename T, int HS, bool EXACT = true, bool DROP = false>
__global__ __launch_bounds__(128) void attn_bwd_dq_kernel(const T* __restrict__ qkv, const T* __restrict__ dy,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ delta, int T_, int nh, int d,
                                                          int hs_rt, T* __restrict__ dqkv, float scale, float drop_p,
                                                          uint64_t drop_seed, const uint64_t* __restrict__ seed_ptr) {
  constexpr int H2 = HS / 2;
  __shared__ float Ks[ATT_TILE][HS + 1];
  __shared__ float Vs[ATT_TILE][HS + 1];
  const int b = blockIdx.z, h = blockIdx.y;
  const int tid = threadIdx.x, half = tid & 1;
  const HeadSplit<HS, EXACT> hd(hs_rt, half);
  const int hs = hd.hs;
  const int qi = blockIdx.x * ATT_ROWS + (tid >> 1);
  const int64_t ld = 3 * (int64_t)d;
  const T* base = qkv + (int64_t)b * T_ * ld;
  const bool valid = qi < T_;
  AttnDrop dr{drop_p, DROP ? aw_seed_mix(drop_seed, seed_ptr) : 0ull};
  const int64_t bh = (int64_t)b * nh + h;
  float q[H2], g[H2], dq[H2];
  const int64_t yo = ((int64_t)b * T_ + (valid ? qi : 0)) * d + h * hs + hd.off;
#pragma unroll
  for (int e = 0; e < H2; ++e) {
    q[e] = valid && hd.has(e) ? to_f32<T>(base[(int64_t)qi * ld + h * hs + hd.off + e]) * scale : 0.f;
    g[e] = valid && hd.has(e) ? to_f32<T>(dy[yo + e]) : 0.f;
    dq[e] = 0.f;
  }
  const int64_t st = ((int64_t)b * nh + h) * T_ + (valid ? qi : 0);
  const float L = valid ? lse[st] : 0.f, Dl = valid ? delta[st] : 0.f;
  const int kend = min(T_, (blockIdx.x + 1) * ATT_ROWS);
  for (int k0 = 0; k0 < kend; k0 += ATT_TILE) {
    __syncthreads();
    for (int i = tid; i < ATT_TILE * hs; i += 128) {
      const int kr = i / hs, e = i - kr * hs;
      const int kk = k0 + kr;
      float kv = 0.f, vv = 0.f;
      if (kk < T_) {
        kv = to_f32<T>(base[(int64_t)kk * ld + d + h * hs + e]);
        vv = to_f32<T>(base[(int64_t)kk * ld + 2 * d + h * hs + e]);
      }
      Ks[kr][e] = kv;
      Vs[kr][e] = vv;
    }
    __syncthreads();
#pragma unroll 4
    for (int j = 0; j < ATT_TILE; ++j) {
      float a = 0.f, dp = 0.f;
#pragma unroll
      for (int e = 0; e < H2; ++e)
        if (hd.has(e)) {
          a = fmaf(q[e], Ks[j][hd.off + e], a);
          dp = fmaf(g[e], Vs[j][hd.off + e], dp);
        }
      a += __shfl_xor(a, 1, 64);
      dp += __shfl_xor(dp, 1, 64);
      const bool ok = valid && (k0 + j) <= qi && (k0 + j) < T_;
      const float p = ok ? __expf(a - L) : 0.f;
      const float ds = p * ((DROP ? dp * dr.scale(bh, T_, qi, k0 + j) : dp) - Dl);
#pragma unroll
      for (int e = 0; e < H2; ++e)
        if (hd.has(e)) dq[e] = fmaf(ds, Ks[j][hd.off + e], dq[e]);
    }
  }
  if (!valid) return;
  T* out = dqkv + ((int64_t)b * T_ + qi) * ld + h * hs + hd.off;
#pragma unroll
  for (int e = 0; e < H2; ++e)
    if (hd.has(e)) out[e] = from_f32<T>(dq[e] * scale);
}

// dk_j = scale * sum_{i>=j} dS_ij q_i ;  dv_j = sum_{i>=j} P_ij dy_i      (key-stationary)
template <typename T, int HS, bool EXACT = true, bool DROP = false>
__global__ __launch_bounds__(128) void attn_bwd_dkv_kernel(const T* __restrict__ qkv, const T* __restrict__ dy,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ delta, int T_, int nh, int d,
                                                           int hs_rt, T* __restrict__ dqkv, float scale, float drop_p,
                                                           uint64_t drop_seed, const uint64_t* __restrict__ seed_ptr) {
  constexpr int H2 = HS / 2;
  __shared__ float Qs[ATT_TILE][HS + 1];
  __shared__ float Gs[ATT_TILE][HS + 1];
  __shared__ float Ls[ATT_TILE], Ds[ATT_TILE];
  const int b = blockIdx.z, h = blockIdx.y;
  const int tid = threadIdx.x, half = tid & 1;
  const HeadSplit<HS, EXACT> hd(hs_rt, half);
  const int hs = hd.hs;
  const int kj = blockIdx.x * ATT_ROWS + (tid >> 1);
  const int64_t ld = 3 * (int64_t)d;
  const T* base = qkv + (int64_t)b * T_ * ld;
  const bool valid = kj < T_;
  AttnDrop dr{drop_p, DROP ? aw_seed_mix(drop_seed, seed_ptr) : 0ull};
  const int64_t bh = (int64_t)b * nh + h;
  float k[H2], v[H2], dk[H2], dv[H2];
#pragma unroll
  for (int e = 0; e < H2; ++e) {
    k[e] = valid && hd.has(e) ? to_f32<T>(base[(int64_t)kj * ld + d + h * hs + hd.off + e]) : 0.f;
    v[e] = valid && hd.has(e) ? to_f32<T>(base[(int64_t)kj * ld + 2 * d + h * hs + hd.off + e]) : 0.f;
    dk[e] = dv[e] = 0.f;
  }
  const int qstart = blockIdx.x * ATT_ROWS;  // queries before the block's first key see none of its keys
  for (int q0 = (qstart / ATT_TILE) * ATT_TILE; q0 < T_; q0 += ATT_TILE) {
    __syncthreads();
    for (int i = tid; i < ATT_TILE * hs; i += 128) {
      const int qr = i / hs, e = i - qr * hs;
      const int qq = q0 + qr;
      float qv = 0.f, gv = 0.f;
      if (qq < T_) {
        qv = to_f32<T>(base[(int64_t)qq * ld + h * hs + e]) * scale;
        gv = to_f32<T>(dy[((int64_t)b * T_ + qq) * d + h * hs + e]);
      }
      Qs[qr][e] = qv;
      Gs[qr][e] = gv;
    }
    for (int i = tid; i < ATT_TILE; i += 128) {
      const int qq = q0 + i;
      const int64_t st = ((int64_t)b * nh + h) * T_ + qq;
      Ls[i] = qq < T_ ? lse[st] : 0.f;
      Ds[i] = qq < T_ ? delta[st] : 0.f;
    }
    __syncthreads();
#pragma unroll 4
    for (int i = 0; i < ATT_TILE; ++i) {
      float a = 0.f, dp = 0.f;
#pragma unroll
      for (int e = 0; e < H2; ++e)
        if (hd.has(e)) {
          a = fmaf(Qs[i][hd.off + e], k[e], a);
          dp = fmaf(Gs[i][hd.off + e], v[e], dp);
        }
      a += __shfl_xor(a, 1, 64);
      dp += __shfl_xor(dp, 1, 64);
      const int qq = q0 + i;
      const bool ok = valid && qq >= kj && qq < T_;
      const float p = ok ? __expf(a - Ls[i]) : 0.f;
      const float ms = DROP ? dr.scale(bh, T_, qq, kj) : 1.f;
      const float ds = p * (dp * ms - Ds[i]);
      const float pd = p * ms;
#pragma unroll
      for (int e = 0; e < H2; ++e)
        if (hd.has(e)) {
          dv[e] = fmaf(pd, Gs[i][hd.off + e], dv[e]);
          dk[e] = fmaf(ds, Qs[i][hd.off + e], dk[e]);  // Qs already carries the scale
        }
    }
  }
  if (!valid) return;
  T* out = dqkv + ((int64_t)b * T_ + kj) * ld + h * hs + hd.off;
#pragma unroll
  for (int e = 0; e < H2; ++e)
    if (hd.has(e)) {
      out[d + e] = from_f32<T>(dk[e]);
      out[2 * d + e] = from_f32<T>(dv[e]);
    }
}

// ---------------------------------------------------------------- cross entropy (one wave per row)
// Rows of up to 64 * NC logits: one wave per row with all of the row's loads issued at once and the next row's in
// flight while this one reduces (ce_fwd_kernel below, kept for V > 1024, walks a row twice -- max, then sum -- and waits
// on its loads each time: 45 vs 16.5 us at 16371 x 514); 16-wave workgroups, one pair of f64 atomics per workgroup.
template <int NC>
__global__ __launch_bounds__(1024) void ce_fwd_rows_kernel(const float* __restrict__ logits, int64_t R, int V,
                                                           int64_t ldl, const int64_t* __restrict__ y, int ignore,
                                                           double* loss_sum, double* count, float* __restrict__ lse) {
  __shared__ double part[16][2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t nw = (int64_t)gridDim.x * 16;
  double ls = 0.0, cnt = 0.0;
  float nv[NC];
  int64_t ny = ignore;
  // the row's logits AND its target id load one row ahead; the target logit is then taken from the registers (its
  // own dependent load after the target id's, both exposed per row, was most of this kernel's time)
  auto load = [&](int64_t r) {
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int i = lane + 64 * k;
      nv[k] = (r < R && i < V) ? logits[r * ldl + i] : -__builtin_huge_valf();
    }
    ny = r < R ? y[r] : ignore;
  };
  int64_t r = (int64_t)blockIdx.x * 16 + wv;
  load(r);
  for (; r < R; r += nw) {
    float v[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) v[k] = nv[k];
    const int64_t t = ny;
    load(r + nw);
    float mx = -__builtin_huge_valf();
#pragma unroll
    for (int k = 0; k < NC; ++k) mx = fmaxf(mx, v[k]);
    mx = wave_max(mx);
    float sm = 0.f;
#pragma unroll
    for (int k = 0; k < NC; ++k) sm += __expf(v[k] - mx);   // -inf (past V) -> 0
    sm = wave_sum(sm);
    const float L = mx + logf(sm);
    if (lane == 0) lse[r] = L;
    if (t != ignore) {   // wave-uniform; the lane holding column t adds the row's term
      const int tk = (int)(t >> 6);
      float tv = v[0];
#pragma unroll
      for (int k = 1; k < NC; ++k) tv = k == tk ? v[k] : tv;
      if (lane == (int)(t & 63)) ls += (double)(L - tv);
      cnt += 1.0;
    }
  }
  ls = wave_sum_d(ls);
  if (lane == 0) {
    part[wv][0] = ls;
    part[wv][1] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, c = 0.0;
    for (int w = 0; w < 16; ++w) {
      a += part[w][0];
      c += part[w][1];
    }
    atomicAdd(loss_sum, a);
    atomicAdd(count, c);
  }
}

__global__ __launch_bounds__(256) void ce_fwd_kernel(const float* __restrict__ logits, int64_t R, int V, int64_t ldl,
                                                     const int64_t* __restrict__ y, int ignore, double* loss_sum,
                                                     double* count, float* __restrict__ lse) {
  // one wave per row, grid-strided; per-block partial sums -> one pair of f64 atomics per block (thousands of
  // same-address atomics, one per row, serialise)
  __shared__ double part[4][2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  double ls = 0.0, cnt = 0.0;
  for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < R; r += nw) {
    const float* lr = logits + r * ldl;
    float mx = -__builtin_huge_valf();
    for (int i = lane; i < V; i += 64) mx = fmaxf(mx, lr[i]);
    mx = wave_max(mx);
    float s = 0.f;
    for (int i = lane; i < V; i += 64) s += __expf(lr[i] - mx);
    s = wave_sum(s);
    const float L = mx + logf(s);
    if (lane == 0) {
      lse[r] = L;
      const int64_t t = y[r];
      if (t != ignore) {
        ls += (double)(L - lr[t]);
        cnt += 1.0;
      }
    }
  }
  if (lane == 0) {
    part[wv][0] = ls;
    part[wv][1] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(loss_sum, (part[0][0] + part[1][0]) + (part[2][0] + part[3][0]));
    atomicAdd(count, (part[0][1] + part[1][1]) + (part[2][1] + part[3][1]));
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ce_bwd_kernel(const float* __restrict__ logits, int64_t R, int V, int64_t ldl,
                                                     const int64_t* __restrict__ y, int ignore,
                                                     const float* __restrict__ lse, const double* __restrict__ count,
                                                     const float* __restrict__ g, T* __restrict__ dl, int64_t ldd) {
  const int lane = threadIdx.x & 63;
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= R) return;
  const int64_t t = y[r];
  const float c = t == ignore ? 0.f : g[0] / (float)count[0];
  const float L = lse[r];
  for (int i = lane; i < V; i += 64) {
    const float p = __expf(logits[r * ldl + i] - L);
    dl[r * ldd + i] = from_f32<T>(c * (p - (i == t ? 1.f : 0.f)));
  }
  for (int i = V + lane; i < ldd; i += 64) dl[r * ldd + i] = from_f32<T>(0.f);
}

// ---------------------------------------------------------------- classification head
__global__ __launch_bounds__(256) void class_s_kernel(const float* __restrict__ xf, int64_t R, int D,
                                                      const float* __restrict__ w1, const float* __restrict__ b1,
                                                      float* __restrict__ s) {
  const int lane = threadIdx.x & 63;
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= R) return;
  float a = 0.f;
  for (int i = lane; i < D; i += 64) a = fmaf(xf[r * D + i], w1[i], a);
  a = wave_sum(a);
  if (lane == 0) s[r] = a + (b1 ? b1[0] : 0.f);
}

__global__ __launch_bounds__(64) void class_out_kernel(const float* __restrict__ s, int64_t B, int T,
                                                       const float* __restrict__ W2, const float* __restrict__ b2,
                                                       float* __restrict__ out) {
  const int lane = threadIdx.x;
  const int64_t b = blockIdx.x;
  float a0 = 0.f, a1 = 0.f;
  for (int t = lane; t < T; t += 64) {
    const float g = gelu_erf(s[b * T + t]);
    a0 = fmaf(g, W2[t], a0);
    a1 = fmaf(g, W2[T + t], a1);
  }
  a0 = wave_sum(a0);
  a1 = wave_sum(a1);
  if (lane == 0) {
    out[b * 2 + 0] = a0 + (b2 ? b2[0] : 0.f);
    out[b * 2 + 1] = a1 + (b2 ? b2[1] : 0.f);
  }
}

// per row r: ds = (sum_c dout[b][c] W2[c][t]) * gelu'(s); dxf[r] = ds * w1; dw1 += ds * xf[r]; db1 += ds
__global__ __launch_bounds__(256) void class_bwd_rows_kernel(const float* __restrict__ xf, const float* __restrict__ s,
                                                             const float* __restrict__ dout, int64_t R, int T, int D,
                                                             const float* __restrict__ w1, const float* __restrict__ W2,
                                                             float* __restrict__ dxf, float* __restrict__ dw1,
                                                             float* __restrict__ db1) {
  extern __shared__ float red[];  // D + 1
  for (int i = threadIdx.x; i <= D; i += blockDim.x) red[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  float dbsum = 0.f;
  for (int64_t r = wave; r < R; r += nw) {
    const int64_t b = r / T;
    const int t = (int)(r - b * T);
    const float dg = dout[b * 2] * W2[t] + dout[b * 2 + 1] * W2[T + t];
    const float ds = dg * gelu_erf_grad(s[r]);
    dbsum += ds;
    for (int i = lane; i < D; i += 64) {
      dxf[r * D + i] = ds * w1[i];
      if (dw1) atomicAdd(&red[i], ds * xf[r * D + i]);
    }
  }
  if (lane == 0) atomicAdd(&red[D], dbsum);
  __syncthreads();
  for (int i = threadIdx.x; i < D; i += blockDim.x)
    if (dw1) atomicAdd(dw1 + i, red[i]);
  if (threadIdx.x == 0 && db1) atomicAdd(db1, red[D]);
}

// dW2[c][t] += sum_b dout[b][c] g[b,t];  db2[c] += sum_b dout[b][c]
__global__ void class_bwd_w2_kernel(const float* __restrict__ s, const float* __restrict__ dout, int64_t B, int T,
                                    float* __restrict__ dW2, float* __restrict__ db2) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < T) {
    float a0 = 0.f, a1 = 0.f;
    for (int64_t b = 0; b < B; ++b) {
      const float g = gelu_erf(s[b * T + t]);
      a0 = fmaf(dout[b * 2], g, a0);
      a1 = fmaf(dout[b * 2 + 1], g, a1);
    }
    if (dW2) {
      dW2[t] += a0;
      dW2[T + t] += a1;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && db2) {
    float c0 = 0.f, c1 = 0.f;
    for (int64_t b = 0; b < B; ++b) {
      c0 += dout[b * 2];
      c1 += dout[b * 2 + 1];
    }
    db2[0] += c0;
    db2[1] += c1;
  }
}

__global__ void ce_finalize_kernel(const double* s, const double* c, float* out) { out[0] = (float)(s[0] / c[0]); }

int gridcap(int64_t n, int threads = 256, int cap = 8192) {
  int64_t g = (n + threads - 1) / threads;
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

}  // namespace

extern "C" int aw_layernorm_fwd(const float* x, int64_t R, int D, const float* w, const float* b, float eps, void* y,
                                int y_dtype, float* mean, float* rstd, void* stream) {
  AW_REQUIRE(x && w && b && y && mean && rstd && R >= 0 && D > 0, "aw_layernorm_fwd: bad args");
  if (R == 0) return AW_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(aw_cdiv(R, 4));
#define AW_LNF(NV)                                                                                              \
  if (y_dtype == AW_BF16)                                                                                       \
    hipLaunchKernelGGL((ln_fwd_vec_kernel<bf16, NV>), grid, dim3(256), 0, s, x, R, D, w, b, eps, (bf16*)y, mean, \
                       rstd);                                                                                   \
  else                                                                                                          \
    hipLaunchKernelGGL((ln_fwd_vec_kernel<float, NV>), grid, dim3(256), 0, s, x, R, D, w, b, eps, (float*)y,     \
                       mean, rstd);                                                                             \
  return aw::check_launch("aw_layernorm_fwd");
  const bool al = (((uintptr_t)x | (uintptr_t)w | (uintptr_t)b | (uintptr_t)y) & 15) == 0;
  if (al && D == 256) { AW_LNF(1) }
  if (al && D == 512) { AW_LNF(2) }
  if (al && D == 768) { AW_LNF(3) }
  if (al && D == 1024) { AW_LNF(4) }
#undef AW_LNF
  if (y_dtype == AW_BF16)
    hipLaunchKernelGGL(ln_fwd_kernel<bf16>, grid, dim3(256), 0, s, x, R, D, w, b, eps, (bf16*)y, mean, rstd);
  else
    hipLaunchKernelGGL(ln_fwd_kernel<float>, grid, dim3(256), 0, s, x, R, D, w, b, eps, (float*)y, mean, rstd);
  return aw::check_launch("aw_layernorm_fwd");
}

extern "C" int aw_layernorm_bwd(const float* x, const float* dy, int64_t R, int D, const float* w, const float* mean,
                                const float* rstd, float* dx, int accumulate, float* dw, float* db, void* dx2,
                                int dx2_dtype, float drop_p, uint64_t drop_seed, const uint64_t* seed_ptr,
                                void* stream) {
  AW_REQUIRE(x && dy && w && mean && rstd && dx && dw && db && R >= 0 && D > 0 && D <= 8192,
             "aw_layernorm_bwd: bad args");
  if (R == 0) return AW_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // workgroups of the row walk (AW_LN_BWD_BLOCKS: tuning override); each ends with one atomic per dw / db column,
  // so more workgroups contend on those 2D addresses: 256 measured best at 16371 x 512 (29.4 us, 5.1 TB/s; 512:
  // 32.5 us, 1024: 40.1 us; tools/probe/ln_probe.py)
  static const int cap = [] { const char* e = getenv("AW_LN_BWD_BLOCKS"); return e ? atoi(e) : 256; }();
  // waves per workgroup of the vectorised kernel (AW_LN_BWD_WAVES: 8, the kernel's launch bound, or 4): more waves
  // keep more row loads in flight per CU at the same number of end-of-kernel dw / db atomics (8 vs 4: decoder step
  // 5.462 vs 5.520 ms, same box)
  static const int lnw = [] {
    const char* e = getenv("AW_LN_BWD_WAVES");
    return e && atoi(e) == 4 ? 4 : 8;
  }();
  dim3 grid(gridcap(R * 64, 64 * lnw, cap));
#define AW_LNB(NV)                                                                                               \
  if (dx2_dtype == AW_BF16)                                                                                      \
    hipLaunchKernelGGL((ln_bwd_vec_kernel<bf16, NV>), grid, dim3(64 * lnw), lnw * 2 * 256 * NV * 4, s, x, dy, R, \
                       D, w, mean, rstd, dx, accumulate, dw, db, (bf16*)dx2, drop_p, drop_seed, seed_ptr);         \
  else                                                                                                           \
    hipLaunchKernelGGL((ln_bwd_vec_kernel<float, NV>), grid, dim3(64 * lnw), lnw * 2 * 256 * NV * 4, s, x, dy,   \
                       R, D, w, mean, rstd, dx, accumulate, dw, db, (float*)dx2, drop_p, drop_seed, seed_ptr);    \
  return aw::check_launch("aw_layernorm_bwd");
  const bool al = (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)w | (uintptr_t)dx | (uintptr_t)dx2) & 15) == 0;
  if (al && D == 256) { AW_LNB(1) }
  if (al && D == 512) { AW_LNB(2) }
  if (al && D == 768) { AW_LNB(3) }
  if (al && D == 1024) { AW_LNB(4) }
#undef AW_LNB
  // the generic kernel runs 256-thread workgroups: its grid is sized for them, not for the 64*lnw-thread vector form
  const dim3 grid1(gridcap(R * 64, 256, cap));
  if (dx2_dtype == AW_BF16)
    hipLaunchKernelGGL(ln_bwd_kernel<bf16>, grid1, dim3(256), 2 * D * sizeof(float), s, x, dy, R, D, w, mean, rstd, dx,
                       accumulate, dw, db, (bf16*)dx2, drop_p, drop_seed, seed_ptr);
  else
    hipLaunchKernelGGL(ln_bwd_kernel<float>, grid1, dim3(256), 2 * D * sizeof(float), s, x, dy, R, D, w, mean, rstd, dx,
                       accumulate, dw, db, (float*)dx2, drop_p, drop_seed, seed_ptr);
  return aw::check_launch("aw_layernorm_bwd");
}

extern "C" int aw_embed_fwd(const int64_t* ids, int64_t B, int T, int D, const float* wtok, const float* pe, float* x,
                            void* stream) {
  AW_REQUIRE(ids && wtok && pe && x && B >= 0 && T > 0 && D > 0, "aw_embed_fwd: bad args");
  if (B == 0) return AW_OK;
  if ((D & 3) == 0 && (((uintptr_t)wtok | (uintptr_t)pe | (uintptr_t)x) & 15) == 0) {
    const int64_t R = B * T;
    hipLaunchKernelGGL(embed_fwd_rows_kernel, dim3((unsigned)std::min<int64_t>((R + 3) / 4, 4096)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), ids, R, T, D, wtok, pe, x);
    return aw::check_launch("aw_embed_fwd");
  }
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(gridcap(B * T * D)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     ids, B, T, D, wtok, pe, x);
  return aw::check_launch("aw_embed_fwd");
}

extern "C" int aw_embed_ln_fwd(const int64_t* ids, int64_t B, int T, int D, const float* wtok, const float* pe, float* x,
                               const float* w, const float* b, float eps, void* y, int y_dtype, float* mean,
                               float* rstd, void* stream) {
  AW_REQUIRE(ids && wtok && pe && x && w && b && y && mean && rstd && B >= 0 && T > 0 &&
                 (D == 256 || D == 512 || D == 768 || D == 1024) && (y_dtype == AW_BF16 || y_dtype == AW_F32) &&
                 (((uintptr_t)wtok | (uintptr_t)pe | (uintptr_t)x | (uintptr_t)w | (uintptr_t)b | (uintptr_t)y) & 15) == 0,
             "aw_embed_ln_fwd: bad args (D must be 256, 512, 768 or 1024; 16-B aligned tensors)");
  if (B == 0) return AW_OK;
  const int64_t R = B * T;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid(aw_cdiv(R, 4));
#define AW_ELN(NV)                                                                                                   \
  if (y_dtype == AW_BF16)                                                                                            \
    hipLaunchKernelGGL((embed_ln_fwd_kernel<bf16, NV>), grid, dim3(256), 0, s, ids, R, T, D, wtok, pe, x, w, b, eps, \
                       (bf16*)y, mean, rstd);                                                                        \
  else                                                                                                               \
    hipLaunchKernelGGL((embed_ln_fwd_kernel<float, NV>), grid, dim3(256), 0, s, ids, R, T, D, wtok, pe, x, w, b, eps,\
                       (float*)y, mean, rstd);                                                                       \
  return aw::check_launch("aw_embed_ln_fwd");
  if (D == 256) { AW_ELN(1) }
  if (D == 512) { AW_ELN(2) }
  if (D == 768) { AW_ELN(3) }
  AW_ELN(4)
#undef AW_ELN
}

extern "C" int aw_embed_sort(const int64_t* ids, int64_t R, int V, int* work, void* stream) {
  AW_REQUIRE(ids && work && R >= 0 && R < (int64_t)1 << 31 && V > 0 && V <= ESORT_MAX_V,
             "aw_embed_sort: bad args (V must be 1..15360)");
  hipLaunchKernelGGL(embed_sort_kernel, dim3(1), dim3(ESORT_THREADS), (V + ESORT_THREADS) * sizeof(int),
                     reinterpret_cast<hipStream_t>(stream), ids, (int)R, V, work, work + V + 1);
  return aw::check_launch("aw_embed_sort");
}

extern "C" int aw_embed_bwd_segsum(const int* work, int V, int D, const float* dx, float* dwtok, void* stream) {
  AW_REQUIRE(work && dx && dwtok && V > 0 && V <= ESORT_MAX_V && (D == 256 || D == 512 || D == 768 || D == 1024) &&
                 (((uintptr_t)dx | (uintptr_t)dwtok) & 15) == 0,
             "aw_embed_bwd_segsum: bad args (D must be 256, 512, 768 or 1024; 16-B aligned dx / dwtok)");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int* off = work;
  const int* ord = work + V + 1;
#define AW_SEG(NV) hipLaunchKernelGGL(embed_segsum_kernel<NV>, dim3(V), dim3(256), 0, s, off, ord, D, dx, dwtok);
  if (D == 256) AW_SEG(1) else if (D == 512) AW_SEG(2) else if (D == 768) AW_SEG(3) else AW_SEG(4)
#undef AW_SEG
  return aw::check_launch("aw_embed_bwd_segsum");
}

extern "C" int aw_embed_bwd_sorted(const int64_t* ids, int64_t B, int T, int D, int V, const float* dx, float* dwtok,
                                   int* work, void* stream) {
  AW_REQUIRE(ids && dx && dwtok && work && B >= 0 && T > 0 && D > 0 && V > 0 && B * T < (int64_t)1 << 31,
             "aw_embed_bwd_sorted: bad args");
  if (B == 0) return AW_OK;
  if (V > ESORT_MAX_V || (D != 256 && D != 512 && D != 768 && D != 1024) || (((uintptr_t)dx | (uintptr_t)dwtok) & 15))
    return aw_embed_bwd(ids, B, T, D, dx, dwtok, stream);
  const int rc = aw_embed_sort(ids, B * T, V, work, stream);
  return rc != AW_OK ? rc : aw_embed_bwd_segsum(work, V, D, dx, dwtok, stream);
}

extern "C" int aw_embed_bwd(const int64_t* ids, int64_t B, int T, int D, const float* dx, float* dwtok, void* stream) {
  AW_REQUIRE(ids && dx && dwtok && B >= 0 && T > 0 && D > 0, "aw_embed_bwd: bad args");
  if (B == 0) return AW_OK;
  // AW_EMBED_BWD_ROWS=0: the element-wise form (A/B)
  static const bool rows = [] { const char* e = getenv("AW_EMBED_BWD_ROWS"); return !(e && atoi(e) == 0); }();
  if (rows) {
    const int64_t R = B * T;
    hipLaunchKernelGGL(embed_bwd_rows_kernel, dim3((unsigned)(R < 4096 ? R : 4096)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), ids, R, D, dx, dwtok);
  } else {
    hipLaunchKernelGGL(embed_bwd_kernel, dim3(gridcap(B * T * D)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), ids, B, T, D, dx, dwtok);
  }
  return aw::check_launch("aw_embed_bwd");
}

#define AW_ATT_DISPATCH(KERNEL, HSV, ...)                                                        \
  do {                                                                                           \
    if (dtype == AW_BF16) hipLaunchKernelGGL((KERNEL<bf16, HSV>), __VA_ARGS__);                  \
    else hipLaunchKernelGGL((KERNEL<float, HSV>), __VA_ARGS__);                                  \
  } while (0)

// ---------------------------------------------------------------- KV-cache decode (generate)
// cache (B, Tmax, 2d) rows [K | V]; the new rows' K and V are appended first (their own launch, so no wave reads
// a cache row another wave of the same launch is writing), then one wave per (query row, head) attends over
// positions 0..pos0+i: pass 1 scores one key per lane into LDS with the running max, pass 2 exponentiates and
// sums, pass 3 gives each lane one head dimension and walks the keys (p broadcast from LDS).  f32 arithmetic.
template <typename T>
__global__ void kv_append_kernel(const T* __restrict__ qkv, int64_t B, int n_new, int pos0, int d,
                                 T* __restrict__ cache, int Tmax) {
  const int64_t total = B * n_new * 2 * (int64_t)d;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / (2 * d);                 // new row b*n_new + i
    const int c = (int)(e - r * 2 * d);            // column within [K | V]
    const int64_t b = r / n_new;
    const int i = (int)(r - b * n_new);
    cache[(b * Tmax + pos0 + i) * 2 * d + c] = qkv[r * 3 * d + d + c];
  }
}

template <typename T>
__global__ __launch_bounds__(64) void attn_decode_kernel(const T* __restrict__ qkv, int n_new, int pos0, int nh,
                                                         int d, const T* __restrict__ cache, int Tmax,
                                                         T* __restrict__ y, float scale) {
  extern __shared__ float sc[];                    // Tmax scores
  const int lane = threadIdx.x;
  const int64_t r = blockIdx.x;                    // new row b*n_new + i
  const int h = blockIdx.y;
  const int64_t b = r / n_new;
  const int i = (int)(r - b * n_new);
  const int hs = d / nh;
  const int nk = pos0 + i + 1;                     // causal: keys 0 .. pos0 + i
  const T* q = qkv + r * 3 * d + h * hs;
  const T* kv = cache + b * (int64_t)Tmax * 2 * d;
  float mx = -__builtin_huge_valf();
  for (int j = lane; j < nk; j += 64) {
    const T* k = kv + (int64_t)j * 2 * d + h * hs;
    float dot = 0.f;
    for (int e = 0; e < hs; ++e) dot = fmaf(to_f32<T>(q[e]), to_f32<T>(k[e]), dot);
    const float s = dot * scale;
    sc[j] = s;
    mx = fmaxf(mx, s);
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = lane; j < nk; j += 64) {
    const float p = __expf(sc[j] - mx);
    sc[j] = p;
    sum += p;
  }
  sum = wave_sum(sum);
  __syncthreads();
  const float inv = 1.f / sum;
  for (int e = lane; e < hs; e += 64) {
    float acc = 0.f;
    for (int j = 0; j < nk; ++j) acc = fmaf(sc[j], to_f32<T>(kv[(int64_t)j * 2 * d + d + h * hs + e]), acc);
    y[r * d + h * hs + e] = from_f32<T>(acc * inv);
  }
}

extern "C" int aw_attn_decode(const void* qkv_new, int64_t B, int n_new, int pos0, int n_head, int d, int dtype,
                              void* kv_cache, int Tmax, void* y, void* stream) {
  AW_REQUIRE(qkv_new && kv_cache && y && B >= 0 && n_new > 0 && pos0 >= 0 && n_head > 0 && d % n_head == 0 &&
                 pos0 + n_new <= Tmax,
             "aw_attn_decode: bad args (pos0 + n_new must fit the cache of Tmax positions)");
  if (B == 0) return AW_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t tot = B * n_new * 2 * (int64_t)d;
  const int g = (int)((tot + 255) / 256 > 4096 ? 4096 : (tot + 255) / 256);
  const float scale = 1.0f / sqrtf((float)(d / n_head));
  dim3 grid((unsigned)(B * n_new), n_head);
  const size_t sh = (size_t)Tmax * sizeof(float);
  if (dtype == AW_BF16) {
    hipLaunchKernelGGL(kv_append_kernel<bf16>, dim3(g), dim3(256), 0, s, (const bf16*)qkv_new, B, n_new, pos0, d,
                       (bf16*)kv_cache, Tmax);
    hipLaunchKernelGGL(attn_decode_kernel<bf16>, grid, dim3(64), sh, s, (const bf16*)qkv_new, n_new, pos0, n_head, d,
                       (const bf16*)kv_cache, Tmax, (bf16*)y, scale);
  } else {
    hipLaunchKernelGGL(kv_append_kernel<float>, dim3(g), dim3(256), 0, s, (const float*)qkv_new, B, n_new, pos0, d,
                       (float*)kv_cache, Tmax);
    hipLaunchKernelGGL(attn_decode_kernel<float>, grid, dim3(64), sh, s, (const float*)qkv_new, n_new, pos0, n_head,
                       d, (const float*)kv_cache, Tmax, (float*)y, scale);
  }
  return aw::check_launch("aw_attn_decode");
}

extern "C" int aw_attn_fwd_dropout(const void* qkv, int64_t B, int T, int n_head, int d, int dtype, void* y,
                                   float* lse, float drop_p, uint64_t drop_seed, const uint64_t* seed_ptr,
                                   void* stream) {
  AW_REQUIRE(qkv && y && lse && B >= 0 && T > 0 && n_head > 0 && d % n_head == 0, "aw_attn_fwd: bad args");
  AW_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "aw_attn_fwd: dropout probability must be in [0, 1)");
  const int hs = d / n_head;
  AW_REQUIRE(hs >= 1 && hs <= 128, "aw_attn_fwd: head size %d unsupported (1..128)", hs);
  if (B == 0) return AW_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (drop_p == 0.f && aw::attn_mfma_supported(dtype, hs, d, T)) {
    aw::attn_fwd_mfma(qkv, B, T, n_head, d, y, lse, s);
    return aw::check_launch("aw_attn_fwd");
  }
  dim3 grid(aw_cdiv(T, ATT_ROWS), n_head, (unsigned)B);
  const float scale = 1.0f / sqrtf((float)hs);
#define AW_F(HSV, EX, DR)                                                                                          \
  if (dtype == AW_BF16)                                                                                            \
    hipLaunchKernelGGL((attn_fwd_kernel<bf16, HSV, EX, DR>), grid, dim3(128), 0, s, (const bf16*)qkv, T, n_head, d, \
                       hs, (bf16*)y, lse, scale, drop_p, drop_seed, seed_ptr);                                     \
  else                                                                                                             \
    hipLaunchKernelGGL((attn_fwd_kernel<float, HSV, EX, DR>), grid, dim3(128), 0, s, (const float*)qkv, T, n_head, \
                       d, hs, (float*)y, lse, scale, drop_p, drop_seed, seed_ptr);
  if (drop_p > 0.f) {         // dropout: the runtime-size kernels (non-default; reference att_dropout = 0.0)
    if (hs <= 16) { AW_F(16, false, true) } else if (hs <= 32) { AW_F(32, false, true) }
    else if (hs <= 64) { AW_F(64, false, true) } else { AW_F(128, false, true) }
  } else {
    switch (hs) {
      case 16: AW_F(16, true, false) break;
      case 32: AW_F(32, true, false) break;
      case 64: AW_F(64, true, false) break;
      case 128: AW_F(128, true, false) break;
      default:
        if (hs < 16) { AW_F(16, false, false) } else if (hs < 32) { AW_F(32, false, false) }
        else if (hs < 64) { AW_F(64, false, false) } else { AW_F(128, false, false) }
    }
  }
#undef AW_F
  return aw::check_launch("aw_attn_fwd");
}

extern "C" int aw_attn_fwd(const void* qkv, int64_t B, int T, int n_head, int d, int dtype, void* y, float* lse,
                           void* stream) {
  return aw_attn_fwd_dropout(qkv, B, T, n_head, d, dtype, y, lse, 0.f, 0ull, nullptr, stream);
}

extern "C" int aw_attn_bwd_dropout(const void* qkv, const void* y, const void* dy, const float* lse, int64_t B, int T,
                                   int n_head, int d, int dtype, void* dqkv, float* ws, float drop_p,
                                   uint64_t drop_seed, const uint64_t* seed_ptr, void* stream) {
  AW_REQUIRE(qkv && y && dy && lse && dqkv && ws && B >= 0 && T > 0 && n_head > 0 && d % n_head == 0,
             "aw_attn_bwd: bad args");
  AW_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "aw_attn_bwd: dropout probability must be in [0, 1)");
  const int hs = d / n_head;
  AW_REQUIRE(hs >= 1 && hs <= 128, "aw_attn_bwd: head size %d unsupported (1..128)", hs);
  if (B == 0) return AW_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(aw_cdiv(T, ATT_ROWS), n_head, (unsigned)B);
  const float scale = 1.0f / sqrtf((float)hs);
  const int64_t nrows = B * n_head * T;
  if (drop_p == 0.f && aw::attn_mfma_supported(dtype, hs, d, T)) {
    aw::attn_bwd_mfma(qkv, y, dy, lse, ws, B, T, n_head, d, dqkv, s);
    return aw::check_launch("aw_attn_bwd");
  }
#define AW_B(HSV, EX, DR)                                                                                          \
  if (dtype == AW_BF16) {                                                                                          \
    hipLaunchKernelGGL((attn_delta_kernel<bf16>), dim3(gridcap(nrows)), dim3(256), 0, s, (const bf16*)y,             \
                       (const bf16*)dy, B, T, n_head, d, ws);                                                      \
    hipLaunchKernelGGL((attn_bwd_dq_kernel<bf16, HSV, EX, DR>), grid, dim3(128), 0, s, (const bf16*)qkv,             \
                       (const bf16*)dy, lse, ws, T, n_head, d, hs, (bf16*)dqkv, scale, drop_p, drop_seed, seed_ptr); \
    hipLaunchKernelGGL((attn_bwd_dkv_kernel<bf16, HSV, EX, DR>), grid, dim3(128), 0, s, (const bf16*)qkv,            \
                       (const bf16*)dy, lse, ws, T, n_head, d, hs, (bf16*)dqkv, scale, drop_p, drop_seed, seed_ptr); \
  } else {                                                                                                         \
    hipLaunchKernelGGL((attn_delta_kernel<float>), dim3(gridcap(nrows)), dim3(256), 0, s, (const float*)y,           \
                       (const float*)dy, B, T, n_head, d, ws);                                                     \
    hipLaunchKernelGGL((attn_bwd_dq_kernel<float, HSV, EX, DR>), grid, dim3(128), 0, s, (const float*)qkv,           \
                       (const float*)dy, lse, ws, T, n_head, d, hs, (float*)dqkv, scale, drop_p, drop_seed,         \
                       seed_ptr);                                                                                  \
    hipLaunchKernelGGL((attn_bwd_dkv_kernel<float, HSV, EX, DR>), grid, dim3(128), 0, s, (const float*)qkv,          \
                       (const float*)dy, lse, ws, T, n_head, d, hs, (float*)dqkv, scale, drop_p, drop_seed,         \
                       seed_ptr);                                                                                  \
  }
  if (drop_p > 0.f) {
    if (hs <= 16) { AW_B(16, false, true) } else if (hs <= 32) { AW_B(32, false, true) }
    else if (hs <= 64) { AW_B(64, false, true) } else { AW_B(128, false, true) }
  } else {
    switch (hs) {
      case 16: AW_B(16, true, false) break;
      case 32: AW_B(32, true, false) break;
      case 64: AW_B(64, true, false) break;
      case 128: AW_B(128, true, false) break;
      default:
        if (hs < 16) { AW_B(16, false, false) } else if (hs < 32) { AW_B(32, false, false) }
        else if (hs < 64) { AW_B(64, false, false) } else { AW_B(128, false, false) }
    }
  }
#undef AW_B
  return aw::check_launch("aw_attn_bwd");
}

extern "C" int aw_attn_bwd(const void* qkv, const void* y, const void* dy, const float* lse, int64_t B, int T,
                           int n_head, int d, int dtype, void* dqkv, float* ws, void* stream) {
  return aw_attn_bwd_dropout(qkv, y, dy, lse, B, T, n_head, d, dtype, dqkv, ws, 0.f, 0ull, nullptr, stream);
}

extern "C" int aw_ce_fwd(const float* logits, int64_t R, int V, int64_t ldl, const int64_t* y, int ignore_index,
                         double* loss_sum, double* count, float* lse, void* stream) {
  AW_REQUIRE(logits && y && loss_sum && count && lse && R >= 0 && V > 0 && ldl >= V, "aw_ce_fwd: bad args");
  if (R == 0) return AW_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 gr((unsigned)std::min<int64_t>((R + 63) / 64, 256));   // <= 256 workgroups of 16 waves, ~4 rows per wave
#define AW_CEF(NC)                                                                                                \
  hipLaunchKernelGGL(ce_fwd_rows_kernel<NC>, gr, dim3(1024), 0, s, logits, R, V, ldl, y, ignore_index, loss_sum, \
                     count, lse);                                                                                  \
  return aw::check_launch("aw_ce_fwd");
  if (V <= 256) { AW_CEF(4) }
  if (V <= 512) { AW_CEF(8) }
  if (V <= 576) { AW_CEF(9) }
  if (V <= 1024) { AW_CEF(16) }
#undef AW_CEF
  hipLaunchKernelGGL(ce_fwd_kernel, dim3(gridcap(R * 64, 256, 1024)), dim3(256), 0, s, logits, R, V, ldl, y,
                     ignore_index, loss_sum, count, lse);
  return aw::check_launch("aw_ce_fwd");
}

extern "C" int aw_ce_bwd(const float* logits, int64_t R, int V, int64_t ldl, const int64_t* y, int ignore_index,
                         const float* lse, const double* count, const float* g, void* dlogits, int64_t ldd, int dtype,
                         void* stream) {
  AW_REQUIRE(logits && y && lse && count && g && dlogits && R >= 0 && V > 0 && ldd >= V, "aw_ce_bwd: bad args");
  if (R == 0) return AW_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == AW_BF16)
    hipLaunchKernelGGL(ce_bwd_kernel<bf16>, dim3(aw_cdiv(R, 4)), dim3(256), 0, s, logits, R, V, ldl, y, ignore_index,
                       lse, count, g, (bf16*)dlogits, ldd);
  else
    hipLaunchKernelGGL(ce_bwd_kernel<float>, dim3(aw_cdiv(R, 4)), dim3(256), 0, s, logits, R, V, ldl, y, ignore_index,
                       lse, count, g, (float*)dlogits, ldd);
  return aw::check_launch("aw_ce_bwd");
}

extern "C" int aw_class_head_fwd(const float* xf, int64_t B, int T, int D, const float* w1, const float* b1,
                                 const float* W2, const float* b2, float* s, float* out, void* stream) {
  AW_REQUIRE(xf && w1 && W2 && s && out && B >= 0 && T > 0 && D > 0, "aw_class_head_fwd: bad args");
  if (B == 0) return AW_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t R = B * T;
  hipLaunchKernelGGL(class_s_kernel, dim3(aw_cdiv(R, 4)), dim3(256), 0, st, xf, R, D, w1, b1, s);
  hipLaunchKernelGGL(class_out_kernel, dim3((unsigned)B), dim3(64), 0, st, s, B, T, W2, b2, out);
  return aw::check_launch("aw_class_head_fwd");
}

extern "C" int aw_class_head_bwd(const float* xf, const float* s, const float* dout, int64_t B, int T, int D,
                                 const float* w1, const float* W2, float* dxf, float* dw1, float* db1, float* dW2,
                                 float* db2, void* stream) {
  AW_REQUIRE(xf && s && dout && w1 && W2 && dxf && B >= 0 && T > 0 && D > 0, "aw_class_head_bwd: bad args");
  if (B == 0) return AW_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t R = B * T;
  hipLaunchKernelGGL(class_bwd_rows_kernel, dim3(gridcap(R * 64, 256, 256)), dim3(256), (D + 1) * sizeof(float), st,
                     xf, s, dout, R, T, D, w1, W2, dxf, dw1, db1);
  hipLaunchKernelGGL(class_bwd_w2_kernel, dim3(aw_cdiv(T, 256)), dim3(256), 0, st, s, dout, B, T, dW2, db2);
  return aw::check_launch("aw_class_head_bwd");
}

extern "C" int aw_ce_finalize(const double* loss_sum, const double* count, float* out, void* stream) {
  AW_REQUIRE(loss_sum && count && out, "aw_ce_finalize: bad args");
  hipLaunchKernelGGL(ce_finalize_kernel, dim3(1), dim3(1), 0, reinterpret_cast<hipStream_t>(stream), loss_sum, count,
                     out);
  return aw::check_launch("aw_ce_finalize");
}
