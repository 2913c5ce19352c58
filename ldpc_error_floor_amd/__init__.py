"""MI355X-native neural min-sum (NMS / quantized NMS) LDPC decoder.

Drop-in replacement for the decoding path of ghy1228/LDPC_Error_Floor
(``build_neural_network`` run by ``compute_results``): HIP kernels for gfx950 behind a C ABI
(``include/ldpc_nms.h``) with a thin pybind11 binding.  See DESIGN.md.
"""
from .code import CodeParams, TannerGraph, load_base_graph, snr_to_sigma, code_rate
from .config import NMSConfig, ConfigError, check_params
from .weights import (DecoderWeights, read_weight_file, load_weights_reference_order,
                      expand_weights, flat_weights)
from .channel import create_mix_epoch, quantize_host, read_uncor_llr, write_uncor_file
from .metrics import calc_ber_fer, Counters, loss_forward

__all__ = [
    "CodeParams", "TannerGraph", "load_base_graph", "snr_to_sigma", "code_rate",
    "NMSConfig", "ConfigError", "check_params",
    "DecoderWeights", "read_weight_file", "load_weights_reference_order", "expand_weights",
    "flat_weights", "create_mix_epoch", "quantize_host", "read_uncor_llr", "write_uncor_file",
    "calc_ber_fer", "Counters", "loss_forward", "NMSDecoder", "Decoder", "Session", "build_session",
    "compute_results", "fer_sweep",
]


def __getattr__(name):
    # GPU-facing pieces import torch + the HIP extension lazily.
    if name in ("NMSDecoder", "Decoder", "DecodeResult"):
        from . import decoder
        return getattr(decoder, name)
    if name in ("Session", "build_session", "make_net_dict"):
        from . import session
        return getattr(session, name)
    if name in ("compute_results", "fer_sweep"):
        from . import fer
        return getattr(fer, name)
    raise AttributeError(name)
