"""vrvq_amd — MI355X (gfx950) implementation of the VRVQ encode -> RVQ -> decode hot path.

Drop-in surface of the reference (lixinghe1999/VRVQ): `DAC_VRVQ` and its sub-modules, the
`generate_mask_hard / generate_mask_ste / cal_bpf_from_mask` helpers, and `conf/*.yml`
loading. Every op runs in the in-tree HIP library `libvrvq_hip.so` (C-ABI: include/vrvq.h).
"""
from .model import (DAC_VRVQ, Decoder, Encoder, ImportanceSubnet, ResidualVectorQuantize,
                    VBRResidualVectorQuantize, VectorQuantize)
from .layers import (DecoderBlock, EncoderBlock, ResidualUnit, Snake1d, WNConv1d,
                     WNConvTranspose1d)
from .utils import (cal_bpf_from_mask, cal_bpf_tensor, check_errors, generate_mask_hard,
                    generate_mask_ste, level_sweep, masked_sum, scale_importance)
from .config import from_config, load_config, model_kwargs

__all__ = [
    "DAC_VRVQ", "Encoder", "Decoder", "ImportanceSubnet", "VectorQuantize",
    "ResidualVectorQuantize", "VBRResidualVectorQuantize", "Snake1d", "WNConv1d",
    "WNConvTranspose1d", "ResidualUnit", "EncoderBlock", "DecoderBlock",
    "generate_mask_hard", "generate_mask_ste", "cal_bpf_from_mask", "cal_bpf_tensor",
    "masked_sum", "scale_importance", "level_sweep", "load_config", "model_kwargs",
    "from_config", "check_errors",
]
