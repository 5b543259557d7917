"""MI355X-native runtime behind the reference module surface (model/*.py mirrors).

arcweld._native   ctypes binding of lib/libarcweld_amd.so (the C ABI in include/arcweld_amd.h)
arcweld.kernels   thin typed wrappers (one per C entry point) taking torch device tensors
arcweld.vqvae     autograd Functions + the fused VQ-VAE-Patch step engine
arcweld.optim     flat-buffer RAdam / clip (multi-tensor, HIP)
arcweld.trainer   the Lightning-equivalent fit loop (clip, accumulate, DDP over RCCL)
"""
