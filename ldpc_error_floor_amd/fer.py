"""FER evaluation loops: the reference's ``compute_results`` contract and a device sweep.

* ``compute_results`` <- ``Print_Functions.py:130-165``: batches x SNRs (SNR innermost, which
  fixes the host RNG consumption order), host LLRs (``create_mix_epoch``) or uncorrected
  words (``read_uncor_llr``), ``sess.run`` of ``ya_output_all`` [+ ``lossa``],
  ``calc_ber_fer``, and ``Results[4, nSNR]`` accumulated as float32 ``/ batch_num``.  It
  works with this package's ``Session`` or any object with the same ``run``.
* ``fer_sweep``: throughput mode for long error-floor sweeps.  LLRs are generated on the
  GPU (``NMSDecoder.awgn``), counters stay on the device (int64), and with
  ``torch.distributed`` initialised each rank decodes a disjoint contiguous range of the
  global codeword stream; the only communication is one ``all_reduce(SUM)`` of the
  [nSNR, 4] counter block at the end (SURVEY.md §8 e).
"""
from __future__ import annotations

import math
import time

import numpy as np

from .channel import append_uncor_rows, create_mix_epoch, read_uncor_llr, write_uncor_file
from .metrics import Counters, calc_ber_fer

__all__ = ["compute_results", "fer_sweep", "shard_range"]


def compute_results(sample_num, input_llr, input_codeword, SNR_sigma, wordRandom, noiseRandom,
                    batch_size, sampling_type, N_proto, M_proto, z_value, train_on_zero_word,
                    training_iter_end, sess, net_dict, etha_curr, decoding_type, punct_start,
                    punct_end, short_start, short_end, q_bit, clip_LLR, uncor_path="Uncor.txt"):
    start_time = time.time()
    SNR_sigma = np.atleast_1d(SNR_sigma)
    Results = np.zeros((4, SNR_sigma.size), dtype=np.float32)   # BER, FER_last, FER, loss
    batch_num = math.floor(sample_num / batch_size)
    for batch_idx in range(batch_num):
        for SNR_idx in range(SNR_sigma.size):
            SNR_point = np.array([SNR_sigma[SNR_idx]])
            if sampling_type in (0, 2):
                X, Y = create_mix_epoch(SNR_point, wordRandom, noiseRandom, batch_size, N_proto,
                                        N_proto - M_proto, z_value, [], train_on_zero_word,
                                        decoding_type, punct_start, punct_end, short_start,
                                        short_end, q_bit, clip_LLR)
            elif sampling_type == 1:
                X, Y = read_uncor_llr(input_llr, input_codeword, batch_idx, batch_size, N_proto,
                                      z_value)
            else:
                raise ValueError(f"sampling_type {sampling_type}")
            feed = {net_dict["xa"]: X, net_dict["ya"]: Y, net_dict["etha"]: etha_curr,
                    net_dict["learn_rate"]: 0}
            if sampling_type == 2:
                y_pred_all = sess.run(fetches=net_dict["ya_output_all"], feed_dict=feed)
                loss_batch = 0
            else:
                y_pred_all, loss_batch = sess.run(fetches=[net_dict["ya_output_all"],
                                                           net_dict["lossa"]], feed_dict=feed)
            ber_last, fer_last, fer, uncor_flag, _ = calc_ber_fer(y_pred_all, training_iter_end,
                                                                  Y, batch_size)
            if sampling_type == 2 and np.sum(uncor_flag == 1) > 0:
                write_uncor_file(uncor_flag, X, N_proto * z_value, uncor_path)
            Results[0, SNR_idx] += ber_last / batch_num
            Results[1, SNR_idx] += fer_last / batch_num
            Results[2, SNR_idx] += fer / batch_num
            Results[3, SNR_idx] += loss_batch / batch_num
    return Results, time.time() - start_time


def shard_range(total: int, rank: int, world: int):
    """Contiguous [begin, end) share of ``total`` codewords for ``rank``."""
    per = total // world
    rem = total % world
    begin = rank * per + min(rank, rem)
    return begin, begin + per + (1 if rank < rem else 0)


def fer_sweep(decoder, sigmas, n_codewords: int, batch: int, seed: int = 1076, T=None,
              punct=(0, 0), short=(0, 0), kernel=None, group=None, progress=None,
              uncor_path=None):
    """Decode ``n_codewords`` per SNR point (split across ranks) with GPU LLRs and device
    counters.  Returns a list of ``Counters`` (global totals on every rank).

    ``uncor_path``: append the frames wrong at every iteration to this file in the
    ``Uncor.txt`` format (``sampling_type == 2``, ``Print_Functions.py:155-156``), collected on
    the GPU; with several ranks each rank writes ``<uncor_path>.rank<r>``."""
    import torch
    import torch.distributed as dist
    dist_on = dist.is_available() and dist.is_initialized()
    rank = dist.get_rank(group) if dist_on else 0
    world = dist.get_world_size(group) if dist_on else 1
    sigmas = np.atleast_1d(np.asarray(sigmas, np.float64))
    dev = decoder.device
    counters = torch.zeros((sigmas.size, 4), dtype=torch.int64, device=dev)
    begin, end = shard_range(int(n_codewords), rank, world)
    fused_channel = uncor_path is None and hasattr(decoder, "decode_awgn")
    llr = None if fused_channel else torch.empty((batch, decoder.n_vars), dtype=torch.float32,
                                                 device=dev)
    flags = torch.empty(batch, dtype=torch.uint8, device=dev) if uncor_path else None
    upath = uncor_path if (uncor_path is None or world == 1) else f"{uncor_path}.rank{rank}"
    for si, sigma in enumerate(sigmas):
        pos = begin
        while pos < end:
            b = min(batch, end - pos)
            if fused_channel:
                # LLRs generated inside the decoder (ldpc_decode_awgn): no HBM round trip
                decoder.decode_awgn(b, float(sigma), seed + 7919 * si, offset=pos, punct=punct,
                                    short=short, T=T, counters=counters[si], kernel=kernel)
            else:
                decoder.awgn(b, float(sigma), seed + 7919 * si, offset=pos, punct=punct,
                             short=short, out=llr[:b])
                decoder.decode(llr[:b], T=T, app=False, counters=counters[si], kernel=kernel,
                               flags=None if flags is None else flags[:b])
                if flags is not None:
                    rows = decoder.collect_uncorrected(flags[:b], llr[:b])
                    if rows.shape[0]:
                        append_uncor_rows(rows, upath)
            pos += b
            if progress:
                progress(si, pos - begin, end - begin)
    if dist_on and world > 1:
        dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group)
    host = counters.cpu().numpy()
    return [Counters.from_array(host[i], int(n_codewords), decoder.n_vars)
            for i in range(sigmas.size)]
