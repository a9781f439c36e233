"""MI355X (gfx950) implementation of the ML-VAE training step.

_lib     ctypes binding of libmlvae.so (C ABI: include/mlvae.h)
engine   VAEEngine: the fused train step (flat params/grads/Adam state, fixed launch order)
ops      torch.autograd.Functions for the drop-in nn.Modules
optim    Adam / clip_grad_norm_ on the device, EngineOptimizer facade
dist     data parallel on batch (one process per GPU, RCCL all-reduce)
build    hipcc build of libmlvae.so
"""
