"""Autograd-level ops.  GPU tensors → gfx950 HIP kernels (``replicann_amd/_C.so``);
CPU tensors → plain ATen with the same math.  No other backends."""

from .activation import dropout, gelu, relu, softmax
from .attention import attention, attention_decode, attention_is_mfma, attention_packed, attention_reference, mask_to_bias
from .conv import GradJoin, conv2d_nhwc, conv_implicit_ok
from .embedding import embedding, vit_join
from .fp8 import Fp8State, dequantize_bf8, dequantize_fp8, fp8_dgrad, fp8_wgrad, linear_fp8, quantize_bf8, quantize_fp8
from .linear import ACT_GELU, ACT_NONE, ACT_RELU, gemm, linear, linear_kv_append, mlp
from .loss import cross_entropy, linear_cross_entropy
from .norm import batch_norm_nhwc, layer_norm
from .pool import avgpool_nhwc, maxpool_nhwc

__all__ = [
    "attention", "attention_decode", "attention_is_mfma", "attention_packed", "attention_reference", "mask_to_bias", "avgpool_nhwc",
    "batch_norm_nhwc", "conv2d_nhwc", "GradJoin", "conv_implicit_ok", "cross_entropy", "dropout", "embedding", "vit_join", "gelu", "gemm",
    "layer_norm", "linear", "linear_kv_append", "mlp", "linear_cross_entropy", "linear_fp8", "Fp8State", "quantize_fp8", "dequantize_fp8", "quantize_bf8", "dequantize_bf8", "fp8_wgrad", "fp8_dgrad", "maxpool_nhwc", "relu", "softmax", "ACT_GELU", "ACT_NONE", "ACT_RELU",
]
