// Specialised-epilogue instantiations of the MFMA GEMM for the input-gradient layouts (A row-major [M][K],
// B [K][N]; plain and implicit-conv A).  Epilogue codes the backward issues (gemm.hip: epi_code):
//   GELU' of the saved pre-activation (erf: model/vq_vae_patch_embedd.py:62,65; tanh: transformer_block.py:8-15),
//   residual-gradient accumulation, dropout-masked operand copy for the next GEMM, plain f32/bf16 gradients.
#include "gemm_core.h"

namespace awg {

#define AW_BWD_CONV_CODES(X, T, LY)                                         \
  X(T, LY, EP_PRE | EP_C | EP_CBF)                                          \
  X(T, LY, EP_PRE | EP_PREBF | EP_C | EP_CBF)                               \
  X(T, LY, EP_PRE | EP_RESID | EP_C | EP_C2DROP | EP_C2BF)                  \
  X(T, LY, EP_PRE | EP_RESID | EP_C | EP_C2COPY | EP_C2BF)

#define AW_BWD_PLAIN_CODES(X, T, LY)                                        \
  X(T, LY, EP_C | EP_C2DROP | EP_C2BF)                                      \
  X(T, LY, EP_C | EP_C2COPY | EP_C2BF)                                      \
  X(T, LY, EP_C)                                                            \
  X(T, LY, EP_C | EP_CBF)                                                   \
  X(T, LY, EP_PRE | EP_TANH | EP_C | EP_CBF)                               \
  X(T, LY, EP_PRE | EP_PREBF | EP_TANH | EP_C | EP_CBF)

bool launch_fast_bwd(const GemmP& P, hipStream_t s, bool is_bf16, Layout ly, uint32_t code) {
  if (is_bf16 && ly == L_NT) {
    switch (code) {
      AW_BWD_CONV_CODES(AW_FAST_CASE, bf16, L_NT)
      AW_BWD_PLAIN_CODES(AW_FAST_CASE, bf16, L_NT)
      default: return false;
    }
  }
  if (is_bf16 && ly == L_NT_CONV) {
    switch (code) {
      AW_BWD_CONV_CODES(AW_FAST_CASE, bf16, L_NT_CONV)
      default: return false;
    }
  }
  return false;
}

}  // namespace awg
