// Multi-tensor RAdam + global-norm clip over one flat parameter/gradient buffer (gfx950).
// torch.optim.RAdam semantics (L2 weight decay added to the gradient, lerp first moment, rectification
// once rho_t > 5) as configured by model/autencoder_lightning_base.py:122-124 and
// model/transformer_decoder.py:64-114; clip = Lightning gradient_clip_val -> clip_grad_norm_ (L2).
#include <math.h>

#include "common.h"

namespace {

constexpr int MAXSEG_LDS = 1024;

struct RAdamScalars {
  float lr, beta1, beta2, eps;
  float bc1, sqrt_bc2, rect;
  int rectified;
};

// Bias corrections and rectification for step t, in double (torch computes them as python floats).
__host__ __device__ inline RAdamScalars radam_scalars(int64_t step, float lr, float beta1, float beta2, float eps) {
  const double b1 = beta1, b2 = beta2, t = (double)step;
  const double bc1 = 1.0 - pow(b1, t), bc2 = 1.0 - pow(b2, t);
  const double rho_inf = 2.0 / (1.0 - b2) - 1.0;
  const double rho_t = rho_inf - 2.0 * t * pow(b2, t) / bc2;
  RAdamScalars S;
  S.lr = lr;
  S.beta1 = beta1;
  S.beta2 = beta2;
  S.eps = eps;
  S.bc1 = (float)bc1;
  S.sqrt_bc2 = (float)sqrt(bc2);
  S.rectified = rho_t > 5.0;
  S.rect = S.rectified ? (float)sqrt((rho_t - 4) * (rho_t - 2) * rho_inf / ((rho_inf - 4) * (rho_inf - 2) * rho_t)) : 1.f;
  return S;
}

__global__ void counter_add_kernel(int64_t* c, int64_t v, int64_t* snap) {
  const int64_t n = c[0] + v;
  c[0] = n;
  if (snap) snap[0] = n;
}

// the same, plus zeroing a small f64 block (a forward's accumulators) in the one launch
__global__ __launch_bounds__(256) void counter_add_zero_kernel(int64_t* c, int64_t v, int64_t* snap, double* z,
                                                               int64_t nz) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t n = c[0] + v;
    c[0] = n;
    snap[0] = n;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nz; i += (int64_t)gridDim.x * blockDim.x)
    z[i] = 0.0;
}

__device__ __forceinline__ int find_seg(const int64_t* off, int nseg, int64_t e) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {  // last segment with off <= e
    int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= e) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Segment of element e for a thread whose elements only increase (grid-stride loops): advance from the last one
// (amortised O(1); the binary search per element it replaces made both kernels ALU-bound).
template <typename Off>
__device__ __forceinline__ int next_seg(const Off* off, int nseg, int s, int64_t e) {
  while (s + 1 < nseg && off[s + 1] <= e) ++s;
  return s;
}

// Segment table of the grad-norm pass in LDS (offsets and the end of the live part -- the segment's start when the
// segment is inactive, so one compare decides): the per-element tests are LDS reads, so an iteration's gradient loads
// no longer wait on global reads of the table (35.8 -> 23.8 us).  The operand-writing update kernel keeps the same
// table as 32-bit offsets (load_segs32, 8 KB of LDS: 125 -> 120.5 us, same-box A/B; the 16 KB int64 table cost it
// more in occupancy than the lookups saved, 123 -> 142 us).
__device__ __forceinline__ void load_segs(const int64_t* __restrict__ off, const int64_t* __restrict__ len,
                                          const int* __restrict__ active, int nseg, int64_t* s_off, int64_t* s_end) {
  for (int i = threadIdx.x; i < nseg; i += blockDim.x) {
    s_off[i] = off[i];
    s_end[i] = active[i] ? off[i] + len[i] : off[i];
  }
}

// The same table as 32-bit element offsets (total < 2^31): the update kernels' LDS stays 8 KB.
__device__ __forceinline__ void load_segs32(const int64_t* __restrict__ off, const int64_t* __restrict__ len,
                                            const int* __restrict__ active, int nseg, int* s_off, int* s_end) {
  for (int i = threadIdx.x; i < nseg; i += blockDim.x) {
    s_off[i] = (int)off[i];
    s_end[i] = (int)(active[i] ? off[i] + len[i] : off[i]);
  }
}

__device__ __forceinline__ float radam_one(float gr, float& pv, float& mv, float& vv, float wd, float gs,
                                           const RAdamScalars& S) {
  gr = gs == 1.0f ? gr : gr * gs;
  if (wd != 0.f) gr = gr + wd * pv;
  mv = mv + (1.0f - S.beta1) * (gr - mv);  // exp_avg.lerp_(grad, 1-beta1)
  vv = vv * S.beta2 + (1.0f - S.beta2) * (gr * gr);
  const float mhat = mv / S.bc1;
  if (S.rectified) {
    const float adaptive = S.sqrt_bc2 / (sqrtf(vv) + S.eps);
    pv = pv - ((mhat * S.lr) * adaptive) * S.rect;
  } else {
    pv = pv - mhat * S.lr;
  }
  return pv;
}

// float4 grid-stride over the flat buffers (segments are 256-B aligned: a float4 never straddles two; the
// alignment padding past seg_len is zero in p, g, m and v and stays zero).
__global__ __launch_bounds__(256) void radam_kernel(float* __restrict__ p, float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    const int64_t* __restrict__ seg_off,
                                                    const int64_t* __restrict__ seg_len,
                                                    const float* __restrict__ seg_wd, const int* __restrict__ seg_active,
                                                    int nseg, int64_t total, RAdamScalars S,
                                                    const float* __restrict__ gscale,
                                                    const int64_t* __restrict__ step_ptr, int zero_g) {
  __shared__ int64_t s_off[MAXSEG_LDS];
  __shared__ RAdamScalars s_S;
  for (int i = threadIdx.x; i < nseg; i += blockDim.x) s_off[i] = seg_off[i];
  if (step_ptr && threadIdx.x == 0) s_S = radam_scalars(*step_ptr, S.lr, S.beta1, S.beta2, S.eps);
  __syncthreads();
  if (step_ptr) S = s_S;
  const float gs = gscale ? gscale[0] : 1.0f;
  const int64_t n4 = total >> 2;
  int s = 0;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = q << 2;
    s = next_seg(s_off, nseg, s, e);
    if (e >= s_off[s] + seg_len[s] || !seg_active[s]) continue;
    const float wd = seg_wd[s];
    const float4 g4 = reinterpret_cast<const float4*>(g)[q];
    float4 p4 = reinterpret_cast<const float4*>(p)[q];
    float4 m4 = reinterpret_cast<const float4*>(m)[q];
    float4 v4 = reinterpret_cast<const float4*>(v)[q];
    radam_one(g4.x, p4.x, m4.x, v4.x, wd, gs, S);
    radam_one(g4.y, p4.y, m4.y, v4.y, wd, gs, S);
    radam_one(g4.z, p4.z, m4.z, v4.z, wd, gs, S);
    radam_one(g4.w, p4.w, m4.w, v4.w, wd, gs, S);
    if (AW_WT_MISC) {
      aw_st_wt(reinterpret_cast<float4*>(p) + q, (f32x4){p4.x, p4.y, p4.z, p4.w});
      aw_st_wt(reinterpret_cast<float4*>(m) + q, (f32x4){m4.x, m4.y, m4.z, m4.w});
      aw_st_wt(reinterpret_cast<float4*>(v) + q, (f32x4){v4.x, v4.y, v4.z, v4.w});
      if (zero_g) aw_st_wt(reinterpret_cast<float4*>(g) + q, (f32x4){0.f, 0.f, 0.f, 0.f});
    } else {
      reinterpret_cast<float4*>(p)[q] = p4;
      reinterpret_cast<float4*>(m)[q] = m4;
      reinterpret_cast<float4*>(v)[q] = v4;
      if (zero_g) reinterpret_cast<float4*>(g)[q] = make_float4(0.f, 0.f, 0.f, 0.f);   // zero_grad, fused
    }
  }
}

// Operand copy of an updated element: index of flat element l of a segment (the parameter in its storage order,
// (O, I, k) contiguous) in the operand `d` (aw_weight_relayout modes), or -1 when the element is not part of it.
__device__ __forceinline__ int64_t op_dst(const aw_operand_desc& d, uint32_t l) {
  const uint32_t O = (uint32_t)d.O, I = (uint32_t)d.I, k = (uint32_t)d.k;
  switch (d.mode) {
    case 0: {   // (O, I, k) tap t -> [O][I]
      const uint32_t oi = l / k, j = l - oi * k;
      return j == (uint32_t)d.tap ? (int64_t)oi : -1;
    }
    case 1: {   // (O, I, 3) -> [O][3 I], col j I + i
      const uint32_t oi = l / 3u, j = l - oi * 3u, o = oi / I, i = oi - o * I;
      return (int64_t)o * 3 * I + (int64_t)j * I + i;
    }
    case 2: {   // (O, I, 3) -> [3 O][I], row j O + o
      const uint32_t oi = l / 3u, j = l - oi * 3u, o = oi / I, i = oi - o * I;
      return ((int64_t)j * O + o) * I + i;
    }
    case 3: {   // convT (I_in, O, k) -> [k O][I_in], row j O + o
      const uint32_t io = l / k, j = l - io * k, i = io / O, o = io - i * O;
      return ((int64_t)j * O + o) * I + i;
    }
    case 4: {   // (O, 1, k) -> [O][ldo] (the zero padding columns are never touched)
      const uint32_t o = l / k, j = l - o * k;
      return (int64_t)o * d.ldo + j;
    }
    case 5:
      return (int64_t)l;
    case 7: {   // tap-major storage (O, 3, I) -> [3 O][I], row j O + o
      const uint32_t oj = l / I, i = l - oj * I, o = oj / 3u, j = oj - o * 3u;
      return ((int64_t)j * O + o) * I + i;
    }
    default:
      return -1;
  }
}

__device__ __forceinline__ void op_store(const aw_operand_desc& d, uint32_t l, float v) {
  const int64_t t = op_dst(d, l);
  if (t < 0) return;
  if (d.dtype == AW_BF16)
    reinterpret_cast<bf16*>(d.out)[t] = (bf16)v;
  else
    reinterpret_cast<float*>(d.out)[t] = v;
}

// The four elements l0..l0+3 of one float4 (l0 % 4 == 0, all inside the segment): one 8-B (bf16) or 16-B (f32)
// store when their operand positions are consecutive -- plain casts (mode 5, a k = 1 matrix in mode 0) and the
// tap-major input-gradient copy (mode 7, rows of I % 4 == 0) -- else four element stores.  The element stores
// left the copies at under 1 TB/s (a 2-B store per lane).
__device__ __forceinline__ void op_store4(const aw_operand_desc& d, uint32_t l0, const float (&pv)[4]) {
  int64_t t0 = -1;
  if (d.mode == 5 || (d.mode == 0 && d.k == 1 && d.tap == 0)) t0 = l0;
  else if (d.mode == 7 && (d.I & 3) == 0) t0 = op_dst(d, l0);
  if (t0 >= 0 && ((uintptr_t)d.out & 15) == 0) {
    if (d.dtype == AW_BF16) {
      typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
      bf16x4 h = {(bf16)pv[0], (bf16)pv[1], (bf16)pv[2], (bf16)pv[3]};
      if (AW_WT_MISC) {
        u32x2 u;
        memcpy(&u, &h, 8);
        aw_st_wt(reinterpret_cast<bf16x4*>(d.out) + (t0 >> 2), u);
      } else {
        reinterpret_cast<bf16x4*>(d.out)[t0 >> 2] = h;
      }
    } else if (AW_WT_MISC) {
      aw_st_wt(reinterpret_cast<float4*>(d.out) + (t0 >> 2), (f32x4){pv[0], pv[1], pv[2], pv[3]});
    } else {
      reinterpret_cast<float4*>(d.out)[t0 >> 2] = make_float4(pv[0], pv[1], pv[2], pv[3]);
    }
    return;
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) op_store(d, l0 + c, pv[c]);
}

// radam_kernel that also refreshes the operand copies of every updated element (up to AW_OPS_PER_SEG per segment,
// ops[AW_OPS_PER_SEG * s + j], mode < 0 = unused): the per-step relayout launch of the forward disappears and the
// updated weights are cast while still in registers.
__global__ __launch_bounds__(256) void radam_ops_kernel(float* __restrict__ p, float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        const int64_t* __restrict__ seg_off,
                                                        const int64_t* __restrict__ seg_len,
                                                        const float* __restrict__ seg_wd,
                                                        const int* __restrict__ seg_active, int nseg, int64_t total,
                                                        RAdamScalars S, const float* __restrict__ gscale,
                                                        const int64_t* __restrict__ step_ptr,
                                                        const aw_operand_desc* __restrict__ ops, int zero_g) {
  __shared__ int s_off[MAXSEG_LDS], s_end[MAXSEG_LDS];
  __shared__ RAdamScalars s_S;
  load_segs32(seg_off, seg_len, seg_active, nseg, s_off, s_end);
  if (step_ptr && threadIdx.x == 0) s_S = radam_scalars(*step_ptr, S.lr, S.beta1, S.beta2, S.eps);
  __syncthreads();
  if (step_ptr) S = s_S;
  const float gs = gscale ? gscale[0] : 1.0f;
  const int n4 = (int)(total >> 2);
  int s = 0;
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += gridDim.x * blockDim.x) {
    const int e = q << 2;
    s = next_seg(s_off, nseg, s, e);
    const int end = s_end[s];
    if (e >= end) continue;   // past the segment's live part (or an inactive segment): no global read decides it
    const float wd = seg_wd[s];
    const float4 g4 = reinterpret_cast<const float4*>(g)[q];
    float4 p4 = reinterpret_cast<const float4*>(p)[q];
    float4 m4 = reinterpret_cast<const float4*>(m)[q];
    float4 v4 = reinterpret_cast<const float4*>(v)[q];
    radam_one(g4.x, p4.x, m4.x, v4.x, wd, gs, S);
    radam_one(g4.y, p4.y, m4.y, v4.y, wd, gs, S);
    radam_one(g4.z, p4.z, m4.z, v4.z, wd, gs, S);
    radam_one(g4.w, p4.w, m4.w, v4.w, wd, gs, S);
    if (AW_WT_MISC) {
      aw_st_wt(reinterpret_cast<float4*>(p) + q, (f32x4){p4.x, p4.y, p4.z, p4.w});
      aw_st_wt(reinterpret_cast<float4*>(m) + q, (f32x4){m4.x, m4.y, m4.z, m4.w});
      aw_st_wt(reinterpret_cast<float4*>(v) + q, (f32x4){v4.x, v4.y, v4.z, v4.w});
      if (zero_g) aw_st_wt(reinterpret_cast<float4*>(g) + q, (f32x4){0.f, 0.f, 0.f, 0.f});
    } else {
      reinterpret_cast<float4*>(p)[q] = p4;
      reinterpret_cast<float4*>(m)[q] = m4;
      reinterpret_cast<float4*>(v)[q] = v4;
      if (zero_g) reinterpret_cast<float4*>(g)[q] = make_float4(0.f, 0.f, 0.f, 0.f);   // zero_grad, fused
    }
    const uint32_t l0 = (uint32_t)(e - s_off[s]);
    const int64_t len = end - s_off[s];
    const float pv[4] = {p4.x, p4.y, p4.z, p4.w};
#pragma unroll
    for (int j = 0; j < AW_OPS_PER_SEG; ++j) {
      const aw_operand_desc d = ops[AW_OPS_PER_SEG * s + j];
      if (d.mode < 0) continue;
      if ((int64_t)l0 + 4 <= len) {
        op_store4(d, l0, pv);
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if ((int64_t)l0 + c < len) op_store(d, l0 + c, pv[c]);   // past seg_len: alignment padding
      }
    }
  }
}

// Sum of squares of the active segments over the flat buffer (float4 grid-stride as radam_kernel).
template <int NT>
__global__ __launch_bounds__(NT) void sumsq_kernel(const float* __restrict__ g, const int64_t* __restrict__ seg_off,
                                                    const int64_t* __restrict__ seg_len,
                                                    const int* __restrict__ seg_active, int nseg, int64_t total,
                                                    double* ws) {
  __shared__ int64_t s_off[MAXSEG_LDS], s_end[MAXSEG_LDS];
  load_segs(seg_off, seg_len, seg_active, nseg, s_off, s_end);
  __syncthreads();
  float acc = 0.f;
  const int64_t n4 = total >> 2;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int s = 0;
  // four float4 loads in flight per thread (one dependent load per iteration left the pass latency-bound)
  for (int64_t q0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q0 < n4; q0 += 4 * stride) {
    float4 v[4];
    bool use[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t q = q0 + u * stride;
      const int64_t e = q << 2;
      use[u] = false;
      if (q < n4) {
        s = next_seg(s_off, nseg, s, e);
        use[u] = e < s_end[s];
      }
      v[u] = use[u] ? reinterpret_cast<const float4*>(g)[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)   // past seg_len inside a float4: alignment padding, always zero
      acc += (v[u].x * v[u].x + v[u].y * v[u].y) + (v[u].z * v[u].z + v[u].w * v[u].w);
  }
  __shared__ double red[NT / 64];
  double d = wave_sum_d((double)acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = d;
  __syncthreads();
  // one partial per workgroup, summed in a fixed order by clip_coef_kernel: no same-address atomics (1024 of
  // them serialised into ~40 us) and a deterministic norm
  if (threadIdx.x == 0) {
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += red[i];
    ws[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(64) void clip_coef_kernel(const double* ws, int nws, float max_norm, float* out_norm,
                                                       float* out_coef) {
  double a = 0.0;
  for (int i = threadIdx.x; i < nws; i += 64) a += ws[i];
  a = wave_sum_d(a);
  if (threadIdx.x != 0) return;
  const float norm = (float)sqrt(a);
  out_norm[0] = norm;
  float c = max_norm / (norm + 1e-6f);
  out_coef[0] = c < 1.0f ? c : 1.0f;
}

__global__ void scale_kernel(float* x, int64_t n, const float* s) {
  const float c = s[0];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] *= c;
}

}  // namespace

extern "C" int aw_radam_step(float* param, float* grad, float* exp_avg, float* exp_avg_sq,
                             const int64_t* seg_off, const int64_t* seg_len, const float* seg_wd, const int* seg_active,
                             int nseg, int64_t total, int64_t step, float lr, float beta1, float beta2, float eps,
                             const float* gscale, const int64_t* step_ptr, int zero_grad, void* stream) {
  AW_REQUIRE(param && grad && exp_avg && exp_avg_sq && seg_off && seg_len && seg_wd && seg_active,
             "aw_radam_step: null pointer");
  AW_REQUIRE(nseg > 0 && nseg <= MAXSEG_LDS, "aw_radam_step: nseg must be in [1, %d]", MAXSEG_LDS);
  AW_REQUIRE((step_ptr || step >= 1) && total >= 0, "aw_radam_step: step counts from 1");
  // scalars in double, as torch's _single_tensor_radam computes them (python floats); on the device when the
  // step number lives there
  const RAdamScalars S = radam_scalars(step_ptr ? 1 : step, lr, beta1, beta2, eps);
  AW_REQUIRE(total % 4 == 0 && ((uintptr_t)param & 15) == 0 && ((uintptr_t)grad & 15) == 0 &&
                 ((uintptr_t)exp_avg & 15) == 0 && ((uintptr_t)exp_avg_sq & 15) == 0,
             "aw_radam_step: flat buffers must be 16-B aligned with total %% 4 == 0");
  if (total == 0) return AW_OK;
  int64_t g = (total / 4 + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(radam_kernel, dim3((int)g), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), param, grad,
                     exp_avg, exp_avg_sq, seg_off, seg_len, seg_wd, seg_active, nseg, total, S, gscale, step_ptr,
                     zero_grad);
  return aw::check_launch("aw_radam_step");
}

extern "C" int aw_radam_step_ops(float* param, float* grad, float* exp_avg, float* exp_avg_sq,
                                 const int64_t* seg_off, const int64_t* seg_len, const float* seg_wd,
                                 const int* seg_active, int nseg, int64_t total, int64_t step, float lr, float beta1,
                                 float beta2, float eps, const float* gscale, const int64_t* step_ptr,
                                 const aw_operand_desc* ops, int zero_grad, void* stream) {
  AW_REQUIRE(param && grad && exp_avg && exp_avg_sq && seg_off && seg_len && seg_wd && seg_active && ops,
             "aw_radam_step_ops: null pointer");
  AW_REQUIRE(nseg > 0 && nseg <= MAXSEG_LDS, "aw_radam_step_ops: nseg must be in [1, %d]", MAXSEG_LDS);
  AW_REQUIRE((step_ptr || step >= 1) && total >= 0, "aw_radam_step_ops: step counts from 1");
  AW_REQUIRE(total < ((int64_t)1 << 31), "aw_radam_step_ops: total must be < 2^31 elements");
  AW_REQUIRE(total % 4 == 0 && ((uintptr_t)param & 15) == 0 && ((uintptr_t)grad & 15) == 0 &&
                 ((uintptr_t)exp_avg & 15) == 0 && ((uintptr_t)exp_avg_sq & 15) == 0,
             "aw_radam_step_ops: flat buffers must be 16-B aligned with total %% 4 == 0");
  const RAdamScalars S = radam_scalars(step_ptr ? 1 : step, lr, beta1, beta2, eps);
  if (total == 0) return AW_OK;
  int64_t g = (total / 4 + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(radam_ops_kernel, dim3((int)g), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), param,
                     grad, exp_avg, exp_avg_sq, seg_off, seg_len, seg_wd, seg_active, nseg, total, S, gscale, step_ptr,
                     ops, zero_grad);
  return aw::check_launch("aw_radam_step_ops");
}

extern "C" int aw_counter_add(int64_t* counter, int64_t v, void* stream) {
  AW_REQUIRE(counter, "aw_counter_add: null counter");
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(1), 0, reinterpret_cast<hipStream_t>(stream), counter, v,
                     nullptr);
  return aw::check_launch("aw_counter_add");
}

extern "C" int aw_counter_add_snapshot(int64_t* counter, int64_t v, int64_t* snapshot, void* stream) {
  AW_REQUIRE(counter && snapshot, "aw_counter_add_snapshot: null pointer");
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(1), 0, reinterpret_cast<hipStream_t>(stream), counter, v,
                     snapshot);
  return aw::check_launch("aw_counter_add_snapshot");
}

extern "C" int aw_counter_add_snapshot_zero(int64_t* counter, int64_t v, int64_t* snapshot, double* zero,
                                            int64_t nzero, void* stream) {
  AW_REQUIRE(counter && snapshot && nzero >= 0 && (zero || nzero == 0), "aw_counter_add_snapshot_zero: bad args");
  int64_t g = (nzero + 255) / 256;
  if (g > 1024) g = 1024;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(counter_add_zero_kernel, dim3((int)g), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     counter, v, snapshot, zero, nzero);
  return aw::check_launch("aw_counter_add_snapshot_zero");
}

extern "C" int aw_grad_norm_clip(const float* grad, const int64_t* seg_off, const int64_t* seg_len,
                                 const int* seg_active, int nseg, int64_t total, float max_norm, double* ws,
                                 float* out_norm, float* out_coef, void* stream) {
  AW_REQUIRE(grad && seg_off && seg_len && seg_active && ws && out_norm && out_coef && nseg > 0 &&
                 nseg <= MAXSEG_LDS && total >= 0 && total % 4 == 0 && ((uintptr_t)grad & 15) == 0,
             "aw_grad_norm_clip: bad args (segments <= %d, 16-B aligned, total %% 4 == 0)", MAXSEG_LDS);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // 512-thread workgroups (AW_NORM_THREADS=256: the old shape): the same 1024 partials, half the grid-stride
  // iterations per thread -- 24.4 -> 23.2 us, same-box A/B
  static const int nt = [] { const char* e = getenv("AW_NORM_THREADS"); return e && atoi(e) == 256 ? 256 : 512; }();
  int64_t g = (total / 4 + nt - 1) / nt;
  if (g > AW_NORM_WS) g = AW_NORM_WS;
  if (g < 1) g = 1;
  if (nt == 512)
    hipLaunchKernelGGL(sumsq_kernel<512>, dim3((int)g), dim3(512), 0, s, grad, seg_off, seg_len, seg_active, nseg,
                       total, ws);
  else
    hipLaunchKernelGGL(sumsq_kernel<256>, dim3((int)g), dim3(256), 0, s, grad, seg_off, seg_len, seg_active, nseg,
                       total, ws);
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(64), 0, s, ws, (int)g, max_norm, out_norm, out_coef);
  return aw::check_launch("aw_grad_norm_clip");
}

extern "C" int aw_scale(float* x, int64_t n, const float* sc, void* stream) {
  AW_REQUIRE(x && sc && n >= 0, "aw_scale: bad args");
  if (n == 0) return AW_OK;
  int64_t g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(scale_kernel, dim3((int)g), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), x, n, sc);
  return aw::check_launch("aw_scale");
}
