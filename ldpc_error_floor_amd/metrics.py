"""Frame/bit error metrics with the reference's contract.

``calc_ber_fer`` <- ``Print_Functions.py:100-118`` (vectorized; same return values and types):
per iteration t a frame is wrong when any hard decision ``(y >= 0)`` differs from ``Y``;
FER = fraction of frames wrong at *every* iteration; FER_last / BER_last use t = T-1 and
BER divides by ``B * N*z`` even when only the first ``Nt*z`` bits are output.

``Counters`` holds the device-side equivalent for the all-zero codeword: int64
{bit errors at T-1, frames wrong at T-1, frames wrong at every iteration, 2*loss} where
the loss is the forward value of loss_type 2 with etha = 0 (``Main_Functions.py:337-356``):
per frame 1/2 (1 - sign(min_k(-y_k))) in {0, 1/2, 1}.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

__all__ = ["calc_ber_fer", "Counters", "loss_forward"]

C_BITERR_LAST, C_FRAME_ERR_LAST, C_FRAME_ERR_ALL, C_LOSS2 = range(4)


def calc_ber_fer(y_pred_all, iters_max, Y_test, batch_size):
    y = np.asarray(y_pred_all)
    length = y.shape[1]
    Y = np.asarray(Y_test)[:, :length]
    pred = (y.reshape(iters_max, batch_size, length) >= 0).astype(np.int64)
    wrong = (np.abs(pred - Y[None]).sum(axis=2) > 0)                 # [T, B]
    uncor_flag = np.min(wrong.astype(np.float64), axis=0)
    fer = uncor_flag.sum() * 1.0 / batch_size
    error_num = (pred[iters_max - 1] - Y).sum(axis=1)
    ber_last = np.abs(error_num.sum()) / (Y_test.shape[0] * Y_test.shape[1])
    fer_last = wrong[iters_max - 1].sum() * 1.0 / Y_test.shape[0]
    return ber_last, fer_last, fer, uncor_flag, error_num


def loss_forward(y_all, T, B, loss_type=2, etha=0.0, labels=None, t_first=None):
    """Forward value of ``lossa`` (``Main_Functions.py:337-356``) from ``ya_output_all``.

    ``y_all`` is [T*B, Nt*z]; the sum runs over t = T-1 down to ``t_first`` (default T-1,
    which is what etha = 0 selects since 0**k = 0 for k > 0) weighted by etha**(T-1-t).
    loss_type 2 uses the exact forward value of sign_through (the reference's STE adds
    float rounding of order 1e-8).
    """
    y = np.asarray(y_all, np.float32).reshape(T, B, -1)
    if t_first is None:
        t_first = T - 1
    total = 0.0
    coeff = 0.0
    for t in range(T - 1, t_first - 1, -1):
        w = np.float32(etha) ** (T - 1 - t)
        x = y[t]
        if loss_type == 0:
            z = np.zeros_like(x) if labels is None else np.asarray(labels, np.float32)[:, :x.shape[1]]
            term = np.maximum(x, 0) - x * z + np.log1p(np.exp(-np.abs(x)))
        elif loss_type == 1:
            term = 1.0 / (1.0 + np.exp(-x))
        elif loss_type == 2:
            term = 0.5 * (1.0 - np.sign(np.min(-x, axis=1)))
        else:
            raise ValueError(f"loss_type {loss_type}")
        total = total + w * term
        coeff += w
    return float(np.mean(total / coeff))


@dataclass
class Counters:
    """Accumulated device counters for one SNR point (all-zero codeword)."""
    bit_err_last: int = 0
    frame_err_last: int = 0
    frame_err_all: int = 0
    loss2: int = 0
    frames: int = 0
    bits_per_frame: int = 0

    @classmethod
    def from_array(cls, arr, frames: int, bits_per_frame: int) -> "Counters":
        a = [int(x) for x in np.asarray(arr).reshape(-1)[:4]]
        return cls(a[0], a[1], a[2], a[3], frames, bits_per_frame)

    @property
    def ber_last(self) -> float:
        return self.bit_err_last / max(1, self.frames * self.bits_per_frame)

    @property
    def fer_last(self) -> float:
        return self.frame_err_last / max(1, self.frames)

    @property
    def fer(self) -> float:
        return self.frame_err_all / max(1, self.frames)

    @property
    def loss(self) -> float:
        return 0.5 * self.loss2 / max(1, self.frames)
