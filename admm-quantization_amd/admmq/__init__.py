"""admmq — MI355X-native ADMM quantized CP/low-rank factorization.

Drop-in replacements for KamikaziZen/admm-quantization's hot path:

    source.admm.admm_iteration / init_factors / squared_relative_diff -> admmq.admm
    source.quantization.quantize_tensor (+ _mse, min_max_quantize)     -> admmq.quantization
    source.utils.unfold                                                 -> admmq.utils
    source.parafac_epc.parafac_epc                                      -> admmq.parafac_epc
    scripts/factorize.py (ALS driver + CLI)                             -> admmq.factorize
      (Gram∘Gram / MTTKRP / reconstruction error on the device)         -> admmq.als
    scripts/factorize_lowrank.py (quant + low-rank ADMM + CLI)          -> admmq.lowrank
    source.models.build_cp_layer / build_cp2conv_layer / ... (export)   -> admmq.export

Compute runs in libadmmq.so (hand-written HIP for gfx950) through a C ABI
(include/admmq.h); there is no CPU fallback.
"""
from .admm import admm_iteration, admm_iteration_batched, init_factors, init_factors_many, squared_relative_diff  # noqa: F401
from .quantization import quantize_tensor, quantize_tensor_mse, min_max_quantize, quantize_batched  # noqa: F401
from .utils import unfold  # noqa: F401

__version__ = "0.1.0"
