"""Typed decoder / evaluation configuration mirroring the reference's module globals.

The reference configures everything through edited globals (``main_Base.py:22-63``,
``main_Post.py:22-63``) and validates them with ``check_params``
(``Main_Functions.py:498-523``), which calls ``sys.exit`` on a violation.  ``NMSConfig``
keeps the same names and meaning; ``validate`` enforces the same rules but raises
``ConfigError``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

__all__ = ["NMSConfig", "ConfigError", "check_params", "DECODING_SP", "DECODING_MS",
           "DECODING_QMS", "DECODING_MS_NONUDGE", "VALID_Q_BITS"]

DECODING_SP = 0          # sum-product (tanh/atanh), flood kernel (Main_Functions.py:238-245)
DECODING_MS = 1          # min-sum, fp32, clip +-clip_LLR
DECODING_QMS = 2         # quantized min-sum (q_bit grid)
DECODING_MS_NONUDGE = 3  # min-sum without the 0 -> 1e-4 nudge (Main_Functions.py:229,247)
VALID_Q_BITS = (6, 5, -5, 4, 3)


class ConfigError(ValueError):
    """Raised where the reference's ``check_params`` would ``sys.exit``."""


def check_params(sampling_type: int, snr_matrix, sharing: Sequence[int], iters_max: int,
                 fixed_iter: int, iter_step: int):
    """``Main_Functions.py:498-523`` with exceptions instead of ``sys.exit``."""
    snr_matrix = np.atleast_1d(np.asarray(snr_matrix, dtype=np.float64))
    if sampling_type == 1:
        if snr_matrix.size > 1:
            snr_matrix = np.array([0.0])
    elif sampling_type == 2:
        if snr_matrix.size > 1:
            raise ConfigError("sampling_type == 2 and len(SNR_Matrix) > 1")
    if int(np.sum(sharing)) == 0:
        raise ConfigError("np.sum(sharing) == 0")
    if any(v in (4, 5) for v in sharing) and (iters_max - fixed_iter) % iter_step > 0:
        raise ConfigError("any(value in [4,5] for value in sharing) and "
                          "(iters_max - fixed_iter) % iter_step > 0")
    if sharing[2] in (1, 4):
        raise ConfigError("sharing[2] in [1,4]")
    if sharing[1] != 0 and sharing[0] != sharing[1]:
        raise ConfigError("sharing[1] != 0 and sharing[0]!=sharing[1])")
    return snr_matrix


@dataclass
class NMSConfig:
    filename: str = "wman_N0576_R34_z24"
    sharing: tuple = (3, 0, 3)
    sampling_type: int = 0
    decoding_type: int = DECODING_QMS
    q_bit: int = 5
    systematic: int = 0
    z_value: int = 24
    punct_start: int = 0
    punct_end: int = 0
    short_start: int = 0
    short_end: int = 0
    iters_max: int = 20
    fixed_iter: int = 0
    fixed_init: int = 0
    iter_step: int = 20
    loss_type: int = 2
    etha: float = 0.0
    batch_size: int = 20
    clip_LLR: float = 20.0
    seed_in: int = 2
    SNR_Matrix: Sequence[float] = field(default_factory=lambda: [2.0, 2.5, 3.0, 3.5, 4.0])
    weights_file: Optional[str] = None

    def validate(self):
        self.SNR_Matrix = check_params(self.sampling_type, self.SNR_Matrix, self.sharing,
                                       self.iters_max, self.fixed_iter, self.iter_step)
        if self.decoding_type not in (DECODING_SP, DECODING_MS, DECODING_QMS, DECODING_MS_NONUDGE):
            raise ConfigError(f"decoding_type {self.decoding_type} is not supported")
        if self.decoding_type == DECODING_QMS and self.q_bit not in VALID_Q_BITS:
            raise ConfigError(f"q_bit {self.q_bit} not in {VALID_Q_BITS}")
        return self

    @property
    def word_seed(self) -> int:
        return 2042 + self.seed_in          # main_Base.py:71

    @property
    def noise_seed(self) -> int:
        return 1074 + self.seed_in          # main_Base.py:72

    def target_node(self, N: int, M: int) -> int:
        return N - M if self.systematic == 1 else N     # main_Base.py:83-86
