"""Eager numpy stand-in for the subset of ``tensorflow.compat.v1`` the reference uses.

Fixture-generation infrastructure only (used by ``make_golden.py`` in the build container,
never shipped to or run on the GPU box).  TensorFlow is not installed in this image and
there is no network, so the reference's graph code (``Main_Functions.build_neural_network``)
is executed op-by-op with numpy float32 equivalents of the TF ops it calls.  In QMS mode
every intermediate is a small half-integer, so all sums/products are exact and the result
equals TF's by construction; ``tf.round`` and ``np.round`` both round half to even.
In MS mode TF's fp32 matmul summation order is unknown, hence the stated tolerance.

Placeholders are eager: the caller puts concrete arrays in ``net_dict`` before building.
"""
from __future__ import annotations

import sys
import types

import numpy as np

F32 = np.float32


def _f(x):
    return np.asarray(x, dtype=F32) if not isinstance(x, np.ndarray) or x.dtype != F32 else x


def _make_module():
    tf = types.ModuleType("tensorflow.compat.v1")
    tf.float32 = F32
    tf.disable_v2_behavior = lambda: None
    tf.transpose = lambda x, perm=None: np.transpose(x, perm)
    tf.multiply = lambda a, b: np.multiply(a, b)
    tf.add = lambda a, b: np.add(a, b)
    tf.reshape = lambda x, shape, name=None: np.reshape(x, shape)
    tf.to_float = lambda x: np.asarray(x).astype(F32)
    tf.matmul = lambda a, b: np.matmul(_f(a), _f(b))
    tf.tile = lambda x, multiples: np.tile(x, multiples)
    tf.reduce_prod = lambda x, axis=None, reduction_indices=None: np.prod(
        x, axis=axis if axis is not None else reduction_indices).astype(F32)
    tf.reduce_min = lambda x, axis=None: np.min(x, axis=axis)
    tf.reduce_mean = lambda x, axis=None, name=None: np.mean(x, axis=axis, dtype=F32)
    tf.zeros = lambda shape, dtype=F32: np.zeros(shape, dtype=F32)
    tf.ones = lambda shape, dtype=F32: np.ones(shape, dtype=F32)
    tf.clip_by_value = lambda x, clip_value_min, clip_value_max: np.clip(
        x, clip_value_min, clip_value_max).astype(F32)
    tf.abs = np.abs
    tf.sign = np.sign
    tf.round = np.round
    tf.stop_gradient = lambda x: x
    tf.tanh = np.tanh
    tf.atanh = np.arctanh
    tf.exp = np.exp
    tf.concat = lambda values, axis: np.concatenate(values, axis=axis)

    math = types.SimpleNamespace(sigmoid=lambda x: (1.0 / (1.0 + np.exp(-x))).astype(F32))
    tf.math = math

    def sce(labels, logits):
        x = _f(logits)
        z = _f(labels)
        return (np.maximum(x, 0) - x * z + np.log1p(np.exp(-np.abs(x)))).astype(F32)
    tf.nn = types.SimpleNamespace(sigmoid_cross_entropy_with_logits=sce)

    class _Adam:
        def __init__(self, learning_rate=None):
            pass

        def minimize(self, loss, var_list=None):
            return None
    tf.train = types.SimpleNamespace(AdamOptimizer=_Adam, Saver=lambda *a, **k: None)

    def constant_initializer(value):
        return ("const", np.asarray(value, dtype=np.float64))

    def truncated_normal_initializer(mean=0.0, stddev=1.0):
        return ("tnorm", mean, stddev)

    def get_variable(name, dtype=F32, shape=None, initializer=None, constraint=None):
        if initializer[0] != "const":
            raise NotImplementedError("random initializers are not used by the fixtures")
        return np.broadcast_to(initializer[1].astype(F32), (shape,)).copy()

    tf.constant_initializer = constant_initializer
    tf.truncated_normal_initializer = truncated_normal_initializer
    tf.get_variable = get_variable
    tf.placeholder = lambda *a, **k: None
    return tf


def install():
    """Register the stand-in as ``tensorflow`` / ``tensorflow.compat`` / ``.compat.v1``."""
    v1 = _make_module()
    compat = types.ModuleType("tensorflow.compat")
    compat.v1 = v1
    root = types.ModuleType("tensorflow")
    root.compat = compat
    sys.modules["tensorflow"] = root
    sys.modules["tensorflow.compat"] = compat
    sys.modules["tensorflow.compat.v1"] = v1
    return v1
