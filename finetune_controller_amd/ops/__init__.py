"""Hot ops of the worker runtime: gfx950 HIP kernels with torch reference paths.

See ``_backend`` for the dispatch policy (HIP on GPU, loud failure if the extension is missing,
``FTC_KERNELS=torch`` for the stock-PyTorch baseline).
"""
from ._backend import ext_available, kernel_mode, load_ext, use_hip  # noqa: F401
from .activation import gelu_tanh, swiglu  # noqa: F401
from .attention import (RopeGrad, Segments, attention_packed, attention_reference, model_tile_len,  # noqa: F401
                        pad_batch_to, segments_from_eos)
from .decode import KVCache, decode_attention  # noqa: F401
from .cross_entropy import cross_entropy_reference, fused_linear_cross_entropy  # noqa: F401
from .linear import lora_linear  # noqa: F401
from .norm import add_rms_norm, layer_norm, rms_norm  # noqa: F401
from .rope import RotaryTable, apply_rope_packed  # noqa: F401
