// Specialised-epilogue instantiations of the MFMA GEMM for the forward layouts (A row-major [M][K], B [N][K];
// plain and implicit-conv A).  One kernel per epilogue code the hot path issues (gemm.hip: epi_code):
//   VQ-VAE:  conv/ResBlock pre-activation + GELU operand, residual + dropout, sep conv, ConvT + BN statistics
//            (model/vq_vae_patch_embedd.py:11,65,68,87,143,27), exact-f32 tokenization forms;
//   Transformer: c_attn, c_proj/MLP projection + dropout + residual, c_fc + tanh-GELU, lm_head
//            (model/transformer_block.py:30,32,78-79; model/transformer_decoder.py:29).
#include "gemm_core.h"

namespace awg {

#define AW_FWD_CODES(X, T, LY)                                              \
  X(T, LY, EP_BIAS | EP_C | EP_C2ACT | EP_C2BF)                             \
  X(T, LY, EP_BIAS | EP_C | EP_CBF | EP_C2ACT | EP_C2BF)                    \
  X(T, LY, EP_BIAS | EP_DROP | EP_RESID | EP_C | EP_C2ACT | EP_C2BF)        \
  X(T, LY, EP_BIAS | EP_RESID | EP_C | EP_C2ACT | EP_C2BF)                  \
  X(T, LY, EP_BIAS | EP_DROP | EP_RESID | EP_C | EP_CBF)                    \
  X(T, LY, EP_BIAS | EP_RESID | EP_C | EP_CBF)

#define AW_FWD_PLAIN_CODES(X, T, LY)                                        \
  X(T, LY, EP_BIAS | EP_C)                                                  \
  X(T, LY, EP_BIAS | EP_BIASMOD | EP_C | EP_STATS)                          \
  X(T, LY, EP_BIAS | EP_BIASMOD | EP_C)                                     \
  X(T, LY, EP_BIAS | EP_BIASMOD | EP_C | EP_CBF | EP_STATS)                 \
  X(T, LY, EP_BIAS | EP_BIASMOD | EP_C | EP_CBF)                            \
  X(T, LY, EP_BIAS | EP_C | EP_CBF)                                         \
  X(T, LY, EP_BIAS | EP_DROP | EP_RESID | EP_C)                             \
  X(T, LY, EP_BIAS | EP_RESID | EP_C)                                       \
  X(T, LY, EP_BIAS | EP_TANH | EP_C | EP_C2ACT | EP_C2BF)                   \
  X(T, LY, EP_BIAS | EP_TANH | EP_C | EP_CBF | EP_C2ACT | EP_C2BF)          \
  X(T, LY, EP_C)                                                            \
  X(T, LY, EP_C | EP_CBF)

// exact-f32 operand forms (parity mode and the frozen-encoder tokenization: f32 C2)
#define AW_FWD_F32_CODES(X, T, LY)                                          \
  X(T, LY, EP_BIAS | EP_C | EP_C2ACT)                                       \
  X(T, LY, EP_BIAS | EP_RESID | EP_C | EP_C2ACT)                            \
  X(T, LY, EP_BIAS | EP_RESID | EP_C)                                       \
  X(T, LY, EP_BIAS | EP_C)

bool launch_fast_fwd(const GemmP& P, hipStream_t s, bool is_bf16, Layout ly, uint32_t code) {
  if (is_bf16 && ly == L_NN) {
    switch (code) {
      AW_FWD_CODES(AW_FAST_CASE, bf16, L_NN)
      AW_FWD_PLAIN_CODES(AW_FAST_CASE, bf16, L_NN)
      default: return false;
    }
  }
  if (is_bf16 && ly == L_NN_CONV) {
    switch (code) {
      AW_FWD_CODES(AW_FAST_CASE, bf16, L_NN_CONV)
      default: return false;
    }
  }
  if (!is_bf16 && ly == L_NN) {
    switch (code) {
      AW_FWD_F32_CODES(AW_FAST_CASE, float, L_NN)
      default: return false;
    }
  }
  return false;
}

}  // namespace awg
