// Epilogue codes that get a specialised GEMM instantiation (gemm.hip: epi_code), shared by the 128-row
// (gemm_fast_fwd.hip, gemm_fast_bwd.hip) and the 256-row ping-pong (gemm_fast_256.hip) translation units.
#pragma once
#include "gemm_core.h"

// forward layouts (A row-major [M][K], B [N][K]; plain and implicit-conv A):
//   VQ-VAE:  conv/ResBlock pre-activation + GELU operand, residual + dropout, sep conv, ConvT + BN statistics
//            (model/vq_vae_patch_embedd.py:11,65,68,87,143,27), exact-f32 tokenization forms;
//   Transformer: c_attn, c_proj/MLP projection + dropout + residual, c_fc + tanh-GELU (and its derivative), lm_head
//            (model/transformer_block.py:30,32,78-79; model/transformer_decoder.py:29).
#define AW_FWD_CODES(X, T, LY)                                              \
  X(T, LY, EP_BIAS | EP_C | EP_C2ACT | EP_C2BF)                             \
  X(T, LY, EP_BIAS | EP_C | EP_CBF | EP_C2ACT | EP_C2BF)                    \
  X(T, LY, EP_BIAS | EP_DROP | EP_RESID | EP_C | EP_C2ACT | EP_C2BF)        \
  X(T, LY, EP_BIAS | EP_RESID | EP_C | EP_C2ACT | EP_C2BF)                  \
  X(T, LY, EP_BIAS | EP_DROP | EP_RESID | EP_C | EP_CBF)                    \
  X(T, LY, EP_BIAS | EP_RESID | EP_C | EP_CBF)                             \
  X(T, LY, EP_BIAS | EP_DROP | EP_RESID | EP_RESIDBF | EP_C | EP_CBF | EP_C2ACT | EP_C2BF) \
  X(T, LY, EP_BIAS | EP_RESID | EP_RESIDBF | EP_C | EP_CBF | EP_C2ACT | EP_C2BF)         \
  X(T, LY, EP_BIAS | EP_DROP | EP_RESID | EP_RESIDBF | EP_C | EP_CBF)                    \
  X(T, LY, EP_BIAS | EP_RESID | EP_RESIDBF | EP_C | EP_CBF)

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
  X(T, LY, EP_BIAS | EP_TANH | EP_C | EP_CBF | EP_C2DACT | EP_C2BF)         \
  X(T, LY, EP_C)                                                            \
  X(T, LY, EP_C | EP_CBF)

#define AW_FWD_F32_CODES(X, T, LY)                                          \
  X(T, LY, EP_BIAS | EP_C | EP_C2ACT)                                       \
  X(T, LY, EP_BIAS | EP_RESID | EP_C | EP_C2ACT)                            \
  X(T, LY, EP_BIAS | EP_RESID | EP_C)                                       \
  X(T, LY, EP_BIAS | EP_C)

// input-gradient layouts (A row-major [M][K], B [K][N]; plain and implicit-conv A): GELU' of the saved
// pre-activation (erf: model/vq_vae_patch_embedd.py:62,65; tanh: transformer_block.py:8-15), residual-gradient
// accumulation, dropout-masked operand copy for the next GEMM, plain f32/bf16 gradients.
#define AW_BWD_CONV_CODES(X, T, LY)                                         \
  X(T, LY, EP_PRE | EP_C | EP_CBF)                                          \
  X(T, LY, EP_PRE | EP_PREBF | EP_C | EP_CBF)                               \
  X(T, LY, EP_PRE | EP_RESID | EP_C | EP_C2DROP | EP_C2BF)                  \
  X(T, LY, EP_PRE | EP_RESID | EP_C | EP_C2COPY | EP_C2BF)                  \
  X(T, LY, EP_PRE | EP_PREBF | EP_RESID | EP_RESIDBF | EP_C | EP_CBF | EP_C2DROP | EP_C2BF) \
  X(T, LY, EP_PRE | EP_PREBF | EP_RESID | EP_RESIDBF | EP_C | EP_CBF | EP_C2COPY | EP_C2BF)

#define AW_BWD_PLAIN_CODES(X, T, LY)                                        \
  X(T, LY, EP_C | EP_C2DROP | EP_C2BF)                                      \
  X(T, LY, EP_C | EP_C2COPY | EP_C2BF)                                      \
  X(T, LY, EP_C | EP_CBF | EP_C2DROP | EP_C2BF)                             \
  X(T, LY, EP_C | EP_CBF | EP_C2COPY | EP_C2BF)                             \
  X(T, LY, EP_C)                                                            \
  X(T, LY, EP_C | EP_CBF)                                                   \
  X(T, LY, EP_PRE | EP_TANH | EP_C | EP_CBF)                               \
  X(T, LY, EP_PRE | EP_PREBF | EP_TANH | EP_C | EP_CBF)                    \
  X(T, LY, EP_PRE | EP_PREBF | EP_DERIV | EP_C | EP_CBF)
