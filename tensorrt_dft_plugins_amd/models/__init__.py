"""Model families built on the DFT ops: FourCastNet AFNO and FNO."""
from .afno import AFNOConfig, AFNONet, afno2d_reference, flops_per_sample, fourcastnet_config  # noqa: F401
from .fno import FNO2d, FNOBlock, FNOConfig, SpectralConv2d, fno_block_flops, spectral_conv2d_reference  # noqa: F401
