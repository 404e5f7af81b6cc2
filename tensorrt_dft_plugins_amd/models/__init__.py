"""Model families built on the DFT ops: FourCastNet AFNO and FNO."""
from .afno import AFNOConfig, AFNONet, afno2d_reference, flops_per_sample, fourcastnet_config  # noqa: F401
