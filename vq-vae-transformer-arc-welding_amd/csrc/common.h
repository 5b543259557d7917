// Shared device helpers for the arc-welding VQ-VAE / Transformer HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>

#include "../../include/arcweld_amd.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

// Write-through (sc1) global stores for large streamed outputs: the written lines leave the XCD's L2 at once instead
// of staying dirty until the end-of-kernel release writes them back (which the next launch waits for).  Vector
// stores only (MI355X_MICROARCH.md: a 16-B sc1 store costs about a plain one).  AW_WT_MISC selects them in the
// non-GEMM kernels that stream out tens of MB (RAdam, un-patch head backward; same-box A/B: neutral to +0.3 %).
#ifndef AW_WT_MISC
#define AW_WT_MISC 1
#endif
__device__ __forceinline__ void aw_st_wt(void* p, f32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void aw_st_wt(void* p, u32x2 v) {
  asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void aw_st_wt(void* p, uint32_t v) {
  asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
typedef __bf16 bf16;

// ---------------------------------------------------------------- LDS-DMA (gfx950 buffer_load ... lds)
// Lane l of one wave-instruction writes its 16 (dwordx4) or 4 (dword) bytes at M0 + 16 l / M0 + 4 l; the source is a
// raw buffer whose range check returns zeros past nbytes (every mask and tail).  The inline asm is invisible to the
// compiler's wait-count tracking: callers retire the loads with aw_vm_wait (a counted or a full vmcnt).
// (The asm writes M0, declared clobbered; no compiler-generated code in these kernels uses M0, so the "reserved
// register" warning is silenced.)
#pragma clang diagnostic ignored "-Winline-asm"
typedef int aw_v4i32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ aw_v4i32 aw_rdesc(const void* base, uint32_t nbytes) {
  const uint64_t p = (uint64_t)(uintptr_t)base;
  return aw_v4i32{(int)__builtin_amdgcn_readfirstlane((uint32_t)p),
                  (int)__builtin_amdgcn_readfirstlane((uint32_t)(p >> 32) & 0xFFFFu),
                  (int)__builtin_amdgcn_readfirstlane(nbytes), 0x00020000};
}
__device__ __forceinline__ void aw_dma16(uint32_t m0, int off, aw_v4i32 desc) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0), "v"(off), "s"(desc)
               : "memory", "m0");
}
__device__ __forceinline__ void aw_dma4(uint32_t m0, int off, aw_v4i32 desc) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dword %1, %2, 0 offen lds" ::"s"(m0), "v"(off), "s"(desc)
               : "memory", "m0");
}
template <int N> __device__ __forceinline__ void aw_vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ uint32_t aw_lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)p;
}

// ---------------------------------------------------------------- error plumbing (host side)
namespace aw {
void set_error(const char* fmt, ...);
int check_launch(const char* what);
}  // namespace aw

#define AW_REQUIRE(cond, ...)                 \
  do {                                        \
    if (!(cond)) {                            \
      aw::set_error(__VA_ARGS__);             \
      return AW_ERR_ARG;                      \
    }                                         \
  } while (0)

// ---------------------------------------------------------------- numerics
#define AW_INV_SQRT2 0.70710678118654752440f
#define AW_INV_SQRT2PI 0.39894228040143267794f

// GELU with the exact erf form (torch nn.GELU() default; model/vq_vae_patch_embedd.py:62,65 and
// model/transformer_decoder.py:34).
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * AW_INV_SQRT2)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  return 0.5f * (1.0f + erff(x * AW_INV_SQRT2)) + x * AW_INV_SQRT2PI * __expf(-0.5f * x * x);
}
// Branch-free GELU(erf) for the bf16-operand paths and the un-patch head.  Phi(x) = 1 - erfc(x / sqrt 2) / 2 by
// Abramowitz & Stegun 7.1.26: erfc(z) = t (a1 + t (a2 + t (a3 + t (a4 + t a5)))) exp(-z^2), t = 1 / (1 + p z), z >= 0,
// absolute error <= 1.5e-7 (so |Phi error| <= 7.5e-8).  One exponential serves both GELU and its derivative:
// exp(-z^2) = exp(-x^2 / 2) = sqrt(2 pi) phi(x), so GELU'(x) = Phi(x) + x phi(x) costs one FMA more.  About 7 VALU
// operations + rcp + exp per element, against 15 + rcp + 2 exp for the Numerical Recipes erfc (whose polynomial sat
// inside its exponential, leaving a second exp for phi).  Phi = 1/2 + copysign(1/2 - erfc/2, x): one v_bfi_b32 in place
// of a compare + select.  The exact-f32 (parity / tokenization) GEMMs keep erff so that the codebook indices stay
// bit-exact.
#define AW_AS_P 0.23164189758f          /* p / sqrt 2, p = 0.3275911 */
#define AW_AS_B1 0.127414796f           /* a_i / 2 */
#define AW_AS_B2 -0.142248368f
#define AW_AS_B3 0.7107068705f
#define AW_AS_B4 -0.7265760135f
#define AW_AS_B5 0.5307027145f
#define AW_NHALF_LOG2E -0.72134752044f  /* -log2(e) / 2 */
__device__ __forceinline__ float aw_phi_e(float x, float& e) {   // Phi(x); e = exp(-x^2 / 2)
  const float t = __builtin_amdgcn_rcpf(fmaf(fabsf(x), AW_AS_P, 1.0f));   // v_rcp_f32 (1 ulp)
  float q = fmaf(t, AW_AS_B5, AW_AS_B4);
  q = fmaf(q, t, AW_AS_B3);
  q = fmaf(q, t, AW_AS_B2);
  q = fmaf(q, t, AW_AS_B1);
  e = __builtin_amdgcn_exp2f(x * (x * AW_NHALF_LOG2E));
  const float r = (q * t) * e;   // erfc(|x| / sqrt 2) / 2
  return 0.5f + copysignf(0.5f - r, x);
}
__device__ __forceinline__ float aw_phi_cdf(float x) {    // P(N(0,1) <= x) = 0.5 * (1 + erf(x / sqrt 2))
  float e;
  return aw_phi_e(x, e);
}
__device__ __forceinline__ float gelu_erf_fast(float x) { return x * aw_phi_cdf(x); }
__device__ __forceinline__ float gelu_erf_grad_fast(float x) {
  float e;
  const float phi = aw_phi_e(x, e);
  return fmaf(x * AW_INV_SQRT2PI, e, phi);
}

// The same functions on a pair of values (the two channels a thread owns): the polynomial and the products run as
// v_pk_fma_f32 / v_pk_mul_f32 (two values per instruction), only rcp / exp / the sign insert stay scalar.  Same
// operations in the same order per element as the scalar forms above (up to FMA contraction).
__device__ __forceinline__ f32x2 aw_splat2(float c) { return (f32x2){c, c}; }
__device__ __forceinline__ f32x2 aw_phi_e2(f32x2 x, f32x2& e) {
  const f32x2 t = {__builtin_amdgcn_rcpf(fmaf(fabsf(x.x), AW_AS_P, 1.0f)),
                   __builtin_amdgcn_rcpf(fmaf(fabsf(x.y), AW_AS_P, 1.0f))};
  f32x2 q = __builtin_elementwise_fma(t, aw_splat2(AW_AS_B5), aw_splat2(AW_AS_B4));
  q = __builtin_elementwise_fma(q, t, aw_splat2(AW_AS_B3));
  q = __builtin_elementwise_fma(q, t, aw_splat2(AW_AS_B2));
  q = __builtin_elementwise_fma(q, t, aw_splat2(AW_AS_B1));
  const f32x2 a = x * (x * aw_splat2(AW_NHALF_LOG2E));
  e = (f32x2){__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
  const f32x2 h = aw_splat2(0.5f) - (q * t) * e;
  return aw_splat2(0.5f) + (f32x2){copysignf(h.x, x.x), copysignf(h.y, x.y)};
}
__device__ __forceinline__ f32x2 aw_phi_cdf2(f32x2 x) {
  f32x2 e;
  return aw_phi_e2(x, e);
}
__device__ __forceinline__ f32x2 gelu_erf_fast2(f32x2 x) { return x * aw_phi_cdf2(x); }
// GELU and its derivative from one Phi evaluation (one exponential per element)
__device__ __forceinline__ void gelu_erf_fast2_and_grad(f32x2 x, f32x2& g, f32x2& dg) {
  f32x2 e;
  const f32x2 phi = aw_phi_e2(x, e);
  g = x * phi;
  dg = __builtin_elementwise_fma(x * aw_splat2(AW_INV_SQRT2PI), e, phi);
}
__device__ __forceinline__ f32x2 gelu_erf_grad_fast2(f32x2 x) {
  f32x2 g, dg;
  gelu_erf_fast2_and_grad(x, g, dg);
  return dg;
}

// Four values at a time (two packed pairs): the form the bf16 GEMM epilogues and the fused encoder chain share, so
// that both round identically (tests/test_res_chain.py compares them bit for bit).
__device__ __forceinline__ void aw_gelu4(const float (&x)[4], float (&y)[4]) {
  const f32x2 a = gelu_erf_fast2((f32x2){x[0], x[1]}), b = gelu_erf_fast2((f32x2){x[2], x[3]});
  y[0] = a.x, y[1] = a.y, y[2] = b.x, y[3] = b.y;
}
__device__ __forceinline__ void aw_gelu_grad4(const float (&x)[4], float (&g)[4]) {
  const f32x2 a = gelu_erf_grad_fast2((f32x2){x[0], x[1]}), b = gelu_erf_grad_fast2((f32x2){x[2], x[3]});
  g[0] = a.x, g[1] = a.y, g[2] = b.x, g[3] = b.y;
}

// GELU tanh form (model/transformer_block.py:8-15): 0.5*x*(1 + tanh(u)) == x * sigmoid(2u), u = sqrt(2/pi)(x +
// 0.044715 x^3) -- one exp and one division instead of tanhf (same value to fp32 rounding).
#define AW_SQRT_2_OVER_PI 0.79788456080286535588f
__device__ __forceinline__ float gelu_tanh(float x) {
  const float u = AW_SQRT_2_OVER_PI * (x + 0.044715f * x * x * x);
  return x * __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * u));
}
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float u = AW_SQRT_2_OVER_PI * (x + 0.044715f * x * x * x);
  const float s = __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * u));   // = 0.5 * (1 + tanh(u))
  const float du = AW_SQRT_2_OVER_PI * (1.0f + 3.0f * 0.044715f * x * x);
  return s + 2.0f * x * s * (1.0f - s) * du;
}
// a pair of them as packed f32 (v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32; exp and rcp stay scalar): the same
// operations per element up to FMA contraction
__device__ __forceinline__ void gelu_tanh_and_grad2(f32x2 x, f32x2& g, f32x2& dg) {
  const f32x2 x2 = x * x;
  const f32x2 u = aw_splat2(AW_SQRT_2_OVER_PI) * __builtin_elementwise_fma(aw_splat2(0.044715f) * x2, x, x);
  const f32x2 a = aw_splat2(-2.0f * 1.44269504088896340736f) * u;
  const f32x2 s = {__builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(a.x)),
                   __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(a.y))};
  const f32x2 du = aw_splat2(AW_SQRT_2_OVER_PI) * __builtin_elementwise_fma(aw_splat2(3.0f * 0.044715f), x2,
                                                                             aw_splat2(1.0f));
  g = x * s;
  dg = __builtin_elementwise_fma((x + x) * s * (aw_splat2(1.0f) - s), du, s);
}
// both from one exponential: g = gelu_tanh(x), dg = gelu_tanh_grad(x), the same operations as the two above
__device__ __forceinline__ void gelu_tanh_and_grad(float x, float& g, float& dg) {
  const float u = AW_SQRT_2_OVER_PI * (x + 0.044715f * x * x * x);
  const float s = __builtin_amdgcn_rcpf(1.0f + __expf(-2.0f * u));
  const float du = AW_SQRT_2_OVER_PI * (1.0f + 3.0f * 0.044715f * x * x);
  g = x * s;
  dg = s + 2.0f * x * s * (1.0f - s) * du;
}

// The GEMM epilogue's  x * m + r  (m = the last of act' / dropout scale, r = the residual): fused when both are
// present, so the rounding does not depend on the compiler's contraction choices (gemm_core.h and the fused encoder
// chain, reschain.hip, must agree bit for bit).
__device__ __forceinline__ float aw_epi_mad(float x, float m, bool has_m, float r, bool has_r) {
  if (has_m && has_r) return __builtin_fmaf(x, m, r);
  if (has_m) x = __fmul_rn(x, m);
  if (has_r) x = __fadd_rn(x, r);
  return x;
}

// ---------------------------------------------------------------- counter-based RNG (dropout masks)
// One splitmix64 draw per aligned group of 4 elements (g = e >> 2) of a launch with seed s; element e takes the
// 16-bit uniform in bits [16*(e & 3), 16*(e & 3) + 16) and is dropped iff u < round(p * 65536).  Forward and
// backward regenerate the identical mask from (seed, element); a row of 4 aligned columns costs one hash.
__device__ __forceinline__ uint64_t aw_hash_group(uint64_t seed, uint64_t g) {
  uint64_t z = seed + (g + 1ull) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint32_t aw_drop_threshold(float p) { return (uint32_t)(p * 65536.f + 0.5f); }
// Effective seed when a device-side per-step counter is supplied (seed_ptr in the ABI).
__device__ __forceinline__ uint64_t aw_seed_mix_value(uint64_t salt, uint64_t ctr) {
  uint64_t z = salt ^ (ctr * 0xD1B54A32D192ED03ull + 0x8CB92BA72F3D8DD7ull);
  z = (z ^ (z >> 32)) * 0xD6E8FEB86659FD93ull;
  return z ^ (z >> 32);
}
__device__ __forceinline__ uint64_t aw_seed_mix(uint64_t salt, const uint64_t* ctr) {
  return ctr ? aw_seed_mix_value(salt, *ctr) : salt;
}
__device__ __forceinline__ float aw_dropout_scale(uint64_t seed, uint64_t e, float p) {
  if (p <= 0.f) return 1.f;
  const uint32_t u = (uint32_t)(aw_hash_group(seed, e >> 2) >> (16 * (e & 3))) & 0xFFFFu;
  return u < aw_drop_threshold(p) ? 0.f : 1.f / (1.f - p);
}
// scales of elements e0 .. e0+3 (one hash when e0 is group-aligned)
__device__ __forceinline__ void aw_dropout_scale4(uint64_t seed, uint64_t e0, float p, float (&s)[4]) {
  if ((e0 & 3) == 0) {
    const uint64_t h = aw_hash_group(seed, e0 >> 2);
    const uint32_t t = aw_drop_threshold(p);
    const float k = 1.f / (1.f - p);
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] = ((uint32_t)(h >> (16 * i)) & 0xFFFFu) < t ? 0.f : k;
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] = aw_dropout_scale(seed, e0 + i, p);
  }
}

// ---------------------------------------------------------------- typed load/store helpers
template <typename T> __device__ __forceinline__ float to_f32(T v);
template <> __device__ __forceinline__ float to_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f32<bf16>(bf16 v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v);
template <> __device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float v) { return (bf16)v; }

__device__ __forceinline__ float load_as_f32(const void* p, int dtype, int64_t i) {
  return dtype == AW_BF16 ? (float)((const bf16*)p)[i] : ((const float*)p)[i];
}
__device__ __forceinline__ void store_from_f32(void* p, int dtype, int64_t i, float v) {
  if (dtype == AW_BF16)
    ((bf16*)p)[i] = (bf16)v;
  else
    ((float*)p)[i] = v;
}

// ---------------------------------------------------------------- wave reductions (wave64)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

static inline int aw_cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
