"""Conv1d-encoder variant of the VAE recipe (BASELINE.json configs[3]): the test_vanilla_vae
SBModel (ref:src/models/test_vanilla_vae/model.py:12-55) over modules.conv_vae.ConvVAE; the fused
engine runs it with VAEConfig.enc_conv (csrc/conv.hip)."""
from models.test_vanilla_vae.model import SBModel  # noqa: F401
