"""Drop-in replacements for the reference's VAE modules (ref:src/modules/), backed by
libmlvae.so.  Constructor signatures, parameter names/shapes (state_dict keys) and
forward() return dicts follow the reference; the arithmetic runs in HIP kernels."""
