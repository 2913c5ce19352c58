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

import json
import math
import os
import time

import numpy as np

from .channel import append_uncor_rows, create_mix_epoch, read_uncor_llr, write_uncor_file
from .metrics import Counters, calc_ber_fer

__all__ = ["compute_results", "fer_sweep", "shard_range", "SweepCheckpoint", "collect_uncor_inputs",
           "decoder_fingerprint"]


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


CKPT_VERSION = 3        # 2: key holds point_seeds and the decoder fingerprint; rank 0's file
                        # is <path> at every world size; 3: the key holds the channel stream
                        # (CHANNEL_STREAM) and the state the uncorrected-word file's per-point
                        # marks (the multi-rank merge)
# The on-GPU channel's stream (csrc/ldpc_awgn.h, oracle/philox_oracle.py), part of a checkpoint's
# key: a resume across a change of the generator (round 4 replaced QMS Box-Muller by the exact
# level sampler) would add counters from another codeword stream.  Bump it with the stream.
CHANNEL_STREAM = "philox4x32-10/qms-level-v1/box-muller-v1"


class SweepCheckpoint:
    """One rank's sweep state as a small JSON file, replaced atomically (write + rename).

    ``key`` holds everything that fixes the codeword stream and its partition (seed, sigmas,
    total codewords, batch, T, puncture/shorten, rank/world, the decoder's fingerprint); a
    resume against a different key is refused.  Rank 0 keeps ``<path>`` at every world size
    (rank r > 0: ``<path>.rank<r>``), so a resume at another world size finds rank 0's file
    and is refused by its key instead of silently starting over.  ``si`` / ``pos`` = the SNR index and global codeword index to decode next,
    ``counters`` = this rank's (not yet all-reduced) int64 counter block, ``uncor_bytes`` = the
    length of the uncorrected-word file at that point (truncated back to it on resume, so rows
    written after the checkpoint are not duplicated)."""

    def __init__(self, path):
        self.path = path

    def load(self):
        if not os.path.exists(self.path):
            return None
        with open(self.path) as f:
            st = json.load(f)
        if st.get("version") != CKPT_VERSION:
            why = (" (version 3 keys the on-GPU channel stream, "
                   f"{CHANNEL_STREAM!r}: an older checkpoint cannot say which codewords it decoded)"
                   if st.get("version") in (1, 2) else "")
            raise ValueError(f"{self.path}: checkpoint version {st.get('version')} != {CKPT_VERSION}{why}")
        return st

    def save(self, key, si, pos, counters, uncor_bytes=None, done=False, uncor_marks=None,
             uncor_base=None):
        st = {"version": CKPT_VERSION, "key": key, "si": int(si), "pos": int(pos),
              "counters": [[int(v) for v in row] for row in counters],
              "uncor_bytes": uncor_bytes, "uncor_marks": uncor_marks, "uncor_base": uncor_base,
              "done": bool(done), "time": time.time()}
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(st, f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, self.path)


def decoder_fingerprint(decoder, T=None):
    """What a checkpointed sweep decoded with: graph, lifting, mode, clip, weights, iterations
    (a resume with another decoder would add its counters to the old ones)."""
    import hashlib
    h = hashlib.sha256()
    proto = getattr(getattr(decoder, "graph", None), "proto", None)
    if proto is None:
        proto = getattr(decoder, "proto", None)
    if proto is not None:
        h.update(np.ascontiguousarray(np.asarray(proto, np.int64)).tobytes())
    W = getattr(decoder, "weights", None) or getattr(decoder, "W", None)
    for a in (getattr(W, "alpha", None), getattr(W, "alpha_ucn", None), getattr(W, "beta", None)):
        if a is not None:
            h.update(np.ascontiguousarray(np.asarray(a, np.float32)).tobytes())
        h.update(b"|")
    return {"graph_weights_sha256": h.hexdigest()[:32], "z": int(getattr(decoder, "z", 0)),
            "decoding_type": int(getattr(decoder, "decoding_type", getattr(decoder, "dt", -1))),
            "q_bit": int(getattr(decoder, "q_bit", getattr(decoder, "q", 0))),
            "clip": float(getattr(decoder, "clip", 20.0)),
            "target_bits": int(getattr(decoder, "target_bits", 0)),
            "T": int(getattr(decoder, "T", 0) if T is None else T)}


def fer_sweep(decoder, sigmas, n_codewords: int, batch: int, seed: int = 1076, T=None,
              punct=None, short=None, kernel=None, group=None, progress=None,
              uncor_path=None, checkpoint=None, checkpoint_every: int = 64,
              resume: bool = False, point_seeds=None, overlap: bool = False):
    """Decode ``n_codewords`` per SNR point (split across ranks) with GPU LLRs and device
    counters.  Returns a list of ``Counters`` (global totals on every rank).

    ``punct`` / ``short``: 1-based inclusive ranges of the channel (``create_mix_epoch``,
    ``Print_Functions.py:29-72``); ``None`` uses the decoder's own (``Decoder(..., punct,
    short)`` / ``build_session``).  SNR point ``si`` uses the Philox stream ``seed + 7919 si``
    (or ``point_seeds[si]``: callers that sweep the same SNR in separate runs give each point
    its own stream) indexed by the global codeword number, so any partition of the codewords
    (ranks, batches, a resume) decodes the same words.

    ``uncor_path``: append the frames wrong at every iteration to this file in the
    ``Uncor.txt`` format (``sampling_type == 2``, ``Print_Functions.py:155-156``), collected on
    the GPU.  With several ranks each rank writes ``<uncor_path>.rank<r>`` during the sweep and
    records where each SNR point's rows end in it; after the final all-reduce rank 0 appends
    them to ``uncor_path`` point by point, ranks in order -- the shards are contiguous, so the
    file is byte for byte the one a single process writes (global codeword order), the one file
    ``main_Post.py`` reads (``Main_Functions.py:529-532``).  The file is
    appended to, as the reference appends (``Print_Functions.py:122``): a fresh start
    (``resume=False``) keeps whatever the file already holds, including the rows of an attempt
    that died before its first checkpoint -- delete it first for a clean run.  A resume
    truncates it back to the length its checkpoint recorded.

    ``checkpoint``: path of this sweep's checkpoint -- rank 0 writes ``<path>``, rank r > 0
    ``<path>.rank<r>`` -- written every ``checkpoint_every`` batches and after every SNR point;
    ``resume=True`` continues from it (a missing file starts from the beginning).  Its key
    holds the channel stream (``CHANNEL_STREAM``), the decoder and the partition, so a resume
    with anything else is refused.

    ``overlap``: when the decoding kernel reads its LLRs from HBM (the float modes' ffl and
    flood: their channel is a kernel of its own; the QMS bit-sliced and v5 kernels generate it in
    their prologue), generate batch j + 1 on a second stream while batch j decodes
    (``pipelined_channel_decode``); the counters are the same either way.  Off by default:
    measured on one MI355X when the bit-sliced kernels still read HBM LLRs
    (``tools/overlap_probe.py``, ``profiles/r3/overlap``), it gained nothing (C2 6.36 against
    6.29 ms per 2^20-codeword step, C4 / C5 equal, C3 1.6 % slower) — the channel kernel is
    VALU-bound too and finds no idle issue slots beside the decode's waves."""
    import torch
    import torch.distributed as dist
    dist_on = dist.is_available() and dist.is_initialized()
    rank = dist.get_rank(group) if dist_on else 0
    world = dist.get_world_size(group) if dist_on else 1
    sigmas = np.atleast_1d(np.asarray(sigmas, np.float64))
    if point_seeds is None:
        point_seeds = [seed + 7919 * si for si in range(sigmas.size)]
    point_seeds = [int(x) for x in point_seeds]
    if len(point_seeds) != sigmas.size:
        raise ValueError("point_seeds needs one seed per SNR point")
    dev = decoder.device
    punct = tuple(getattr(decoder, "punct", (0, 0)) if punct is None else punct)
    short = tuple(getattr(decoder, "short", (0, 0)) if short is None else short)
    counters = torch.zeros((sigmas.size, 4), dtype=torch.int64, device=dev)
    begin, end = shard_range(int(n_codewords), rank, world)
    # the channel generated inside the decoder (ldpc_decode_awgn) unless the decoder cannot;
    # collecting uncorrected words then regenerates only the failing frames' rows
    # (collect_uncorrected_awgn: the same values the HBM channel would hold)
    fused_channel = hasattr(decoder, "decode_awgn") and (
        uncor_path is None or hasattr(decoder, "collect_uncorrected_awgn"))
    llr = None if fused_channel else torch.empty((batch, decoder.n_vars), dtype=torch.float32,
                                                 device=dev)
    flags = torch.empty(batch, dtype=torch.uint8, device=dev) if uncor_path else None
    upath = uncor_path if (uncor_path is None or world == 1) else f"{uncor_path}.rank{rank}"
    fsize = lambda path: os.path.getsize(path) if os.path.exists(path) else 0   # noqa: E731
    # the multi-rank merge: marks[si + 1] = this rank's file length after point si (marks[0]: at
    # the sweep's start); base = the merged file's length at the start (rank 0)
    marks = [None] * (sigmas.size + 1)
    base = None
    if upath is not None:
        marks[0] = fsize(upath)
        if world > 1 and rank == 0:
            base = fsize(uncor_path)
    ck = None
    si0, pos0 = 0, begin
    if checkpoint is not None:
        ck = SweepCheckpoint(checkpoint if rank == 0 else f"{checkpoint}.rank{rank}")
        key = {"seed": int(seed), "point_seeds": point_seeds, "sigmas": [float(x) for x in sigmas],
               "n_codewords": int(n_codewords), "batch": int(batch),
               "T": None if T is None else int(T), "punct": list(punct), "short": list(short),
               "rank": rank, "world": world, "uncor": upath is not None,
               "decoder": decoder_fingerprint(decoder, T), "channel": CHANNEL_STREAM}
        err = ""
        try:
            st = ck.load() if resume else None
            if st is not None and st["key"] != key:
                err = f"{ck.path}: checkpoint is for {st['key']}, this sweep is {key}"
        except ValueError as e:
            st, err = None, str(e)
        if dist_on:
            # every rank raises together (one failing rank alone would leave the others waiting
            # in the final all_reduce)
            flag = torch.tensor([1 if err else 0], dtype=torch.int64, device=counters.device)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
            if int(flag.item()) and not err:
                err = "another rank refused its checkpoint"
        if err:
            raise ValueError(err)
        if st is not None:
            si0, pos0 = st["si"], st["pos"]
            counters.copy_(torch.tensor(st["counters"], dtype=torch.int64))
            if upath is not None and st.get("uncor_bytes") is not None and os.path.exists(upath):
                with open(upath, "r+b") as f:
                    f.truncate(int(st["uncor_bytes"]))
            if upath is not None and st.get("uncor_marks") is not None:
                marks = list(st["uncor_marks"])
            if st.get("uncor_base") is not None:
                base = int(st["uncor_base"])

    def save(si, pos, done=False):
        ub = fsize(upath) if upath else None
        ck.save(key, si, pos, counters.cpu().tolist(), ub, done, marks if upath else None, base)

    if ck is not None and st is None:
        # a fresh start records the uncorrected-word file's current length at once: a resume
        # truncates back to it (rows of an attempt that died before its first checkpoint go),
        # and rows earlier sweeps appended to a shared file stay (Print_Functions.py:122 appends)
        save(si0, pos0)

    if fused_channel and upath is None and overlap and _pipelines(decoder, T, kernel):
        # the channel of batch j + 1 on a second stream while batch j decodes (the decoder reads
        # its LLRs from HBM, so ldpc_decode_awgn would run the two kernels back to back)
        jobs = [(si, pos, min(batch, end - pos)) for si in range(si0, sigmas.size)
                for pos in range(pos0 if si == si0 else begin, end, batch)]
        nbs = {}

        def done(j, si, pos, b):
            nbs[si] = nbs.get(si, 0) + 1
            if ck is not None and checkpoint_every > 0 and nbs[si] % checkpoint_every == 0 and pos + b < end:
                save(si, pos + b)
            if progress:
                progress(si, pos + b - begin, end - begin)
            if pos + b >= end and ck is not None:
                save(si + 1, begin, done=(si + 1 == sigmas.size))

        pipelined_channel_decode(decoder, jobs, lambda si: (float(sigmas[si]), point_seeds[si]),
                                 lambda si: counters[si], T=T, kernel=kernel, punct=punct,
                                 short=short, on_done=done)
        for si in range(si0, sigmas.size):          # points with no codewords on this rank
            if ck is not None and si not in nbs:
                save(si + 1, begin, done=(si + 1 == sigmas.size))
        si0 = sigmas.size
    # the collection on the in-kernel channel: batch j's failing rows are regenerated, copied and
    # written (side stream, host) while batch j + 1 decodes; two frame-flag buffers
    side, flag_bufs, pending = None, None, []
    if fused_channel and flags is not None:
        side = torch.cuda.Stream(dev)
        flag_bufs = [flags, torch.empty_like(flags)]

    def flush():
        while pending:
            fb, sg, ps, p0, ev = pending.pop(0)
            side.wait_event(ev)
            rows = decoder.collect_uncorrected_awgn(fb, sg, ps, offset=p0, punct=punct, short=short,
                                                    stream=side)
            if rows.shape[0]:
                append_uncor_rows(rows, upath, formatter=decoder.format_uncor_rows)

    for si, sigma in enumerate(sigmas):
        if si < si0:
            continue
        pos = pos0 if si == si0 else begin
        nb = 0
        while pos < end:
            b = min(batch, end - pos)
            if fused_channel:
                # LLRs generated inside the decoder (ldpc_decode_awgn): no HBM round trip
                fb = None if flag_bufs is None else flag_bufs[nb % 2][:b]
                decoder.decode_awgn(b, float(sigma), point_seeds[si], offset=pos, punct=punct,
                                    short=short, T=T, counters=counters[si], kernel=kernel, flags=fb)
                if fb is not None:
                    ev = torch.cuda.Event()
                    ev.record(torch.cuda.current_stream(dev))
                    flush()                       # the previous batch, while this one decodes
                    pending.append((fb, float(sigma), point_seeds[si], pos, ev))
            else:
                decoder.awgn(b, float(sigma), point_seeds[si], offset=pos, punct=punct,
                             short=short, out=llr[:b])
                decoder.decode(llr[:b], T=T, app=False, counters=counters[si], kernel=kernel,
                               flags=None if flags is None else flags[:b])
                if flags is not None:
                    rows = decoder.collect_uncorrected(flags[:b], llr[:b])
                    if rows.shape[0]:
                        append_uncor_rows(rows, upath, formatter=decoder.format_uncor_rows)
            pos += b
            nb += 1
            if ck is not None and checkpoint_every > 0 and nb % checkpoint_every == 0 and pos < end:
                flush()                           # (the file holds every batch up to pos)
                save(si, pos)
            if progress:
                progress(si, pos - begin, end - begin)
        flush()
        if upath is not None:
            marks[si + 1] = fsize(upath)
        if ck is not None:
            save(si + 1, begin, done=(si + 1 == sigmas.size))
    if dist_on:
        # (a world of one included: the same collective the multi-GPU job runs)
        dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group)
    if upath is not None and world > 1:
        _merge_uncor_files(uncor_path, marks, base, rank, world, group, counters.device)
    host = counters.cpu().numpy()
    return [Counters.from_array(host[i], int(n_codewords), decoder.n_vars)
            for i in range(sigmas.size)]


def _merge_uncor_files(uncor_path, marks, base, rank, world, group, device):
    """The multi-rank uncorrected-word collection's last step: every rank's per-point marks
    (byte offsets into ``<uncor_path>.rank<r>``) to rank 0, which appends point by point, ranks
    in order, the rows each rank wrote for it to ``uncor_path`` (truncated back to its length at
    the sweep's start first, so a resumed finished sweep merges again to the same file).  The
    shards are contiguous in global codeword order (``shard_range``), so the result is the
    single-process file byte for byte.  One all_gather of an int64 tensor (gloo and RCCL alike)
    and a barrier, so no rank leaves before the file is complete."""
    import torch
    import torch.distributed as dist
    mine = torch.tensor([-1 if m is None else int(m) for m in marks], dtype=torch.int64, device=device)
    allm = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allm, mine, group=group)
    if rank == 0:
        rows = [m.cpu().tolist() for m in allm]
        if any(x < 0 for r in rows for x in r):
            raise RuntimeError("uncorrected-word merge: a rank did not finish every SNR point")
        with open(uncor_path, "ab") as out:
            out.truncate(int(base or 0))
            out.seek(0, os.SEEK_END)
            srcs = [open(f"{uncor_path}.rank{r}", "rb") if os.path.exists(f"{uncor_path}.rank{r}") else None
                    for r in range(world)]
            try:
                for si in range(len(marks) - 1):
                    for r, f in enumerate(srcs):
                        a, b = rows[r][si], rows[r][si + 1]
                        if b > a:
                            f.seek(a)
                            out.write(f.read(b - a))
            finally:
                for f in srcs:
                    if f is not None:
                        f.close()
    dist.barrier(group=group)


def _pipelines(decoder, T, kernel) -> bool:
    """Whether ``decoder`` runs on a GPU and ``ldpc_decode_awgn`` would generate its LLRs with
    the channel kernel into HBM (flood and ffl; the fused v5 and the QMS bit-sliced kernels
    generate in their prologue)."""
    dev = getattr(decoder, "device", None)
    if getattr(dev, "type", None) != "cuda" or not hasattr(decoder, "generates_channel_in_kernel"):
        return False
    return not decoder.generates_channel_in_kernel(T, kernel)


def pipelined_channel_decode(decoder, jobs, point, cnt, T=None, kernel=None, punct=None,
                             short=None, on_done=None):
    """Decode a sequence of on-GPU channel batches, the channel of batch j + 1 generated on a
    second stream while batch j decodes on the current stream (two LLR buffers; an event orders
    each buffer's next generation after the decode that read it).  The codewords and counters are
    those of ``decoder.decode_awgn`` batch by batch (``ldpc_channel_awgn`` + ``ldpc_decode``).

    ``jobs``: (si, pos, b) = SNR point, global offset of the batch's first codeword, batch size;
    ``point(si)`` -> (sigma, Philox seed); ``cnt(si)`` -> the int64[4] device counters of point
    si; ``on_done(j, si, pos, b)`` runs on the host after decode j is queued."""
    import torch
    jobs = list(jobs)
    if not jobs:
        return
    dev = decoder.device
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    bmax = max(b for _, _, b in jobs)
    bufs = [torch.empty((bmax, decoder.n_vars), dtype=torch.float32, device=dev) for _ in range(2)]
    gen_ev, dec_ev = [None, None], [None, None]

    def gen(j):
        si, pos, b = jobs[j]
        k = j % 2
        sigma, seed = point(si)
        if dec_ev[k] is None:
            side.wait_stream(main)            # a fresh buffer: after the main stream's earlier work
        else:
            side.wait_event(dec_ev[k])        # after the decode that read this buffer
        decoder.awgn(b, sigma, seed, offset=pos, punct=punct, short=short, out=bufs[k][:b],
                     stream=side)
        gen_ev[k] = torch.cuda.Event()
        gen_ev[k].record(side)

    try:
        gen(0)
        for j, (si, pos, b) in enumerate(jobs):
            if j + 1 < len(jobs):
                gen(j + 1)
            k = j % 2
            main.wait_event(gen_ev[k])
            decoder.decode(bufs[k][:b], T=T, app=False, counters=cnt(si), kernel=kernel, stream=main)
            dec_ev[k] = torch.cuda.Event()
            dec_ev[k].record(main)
            if on_done:
                on_done(j, si, pos, b)
    finally:
        # (also when on_done raises): the buffers return to the main stream's pool only after
        # every generation queued on the side stream
        main.wait_stream(side)


def collect_uncor_inputs(decoder, sigma, filename, counts=(10000, 5000, 5000), out_dir="Inputs",
                         batch: int = 1 << 16, seed: int = 1076, T=None, punct=None, short=None,
                         max_codewords: int = 1 << 34):
    """Regenerate the post-decoder's inputs ``<out_dir>/[Uncor]_<filename>{,_Valid,_Test}.txt``
    (``process_data``, ``Main_Functions.py:526-576``; stripped from the reference snapshot,
    ``.MISSING_LARGE_BLOBS:1-3``): the reference's ``sampling_type == 2`` pass —
    ``compute_results`` -> ``calc_ber_fer``'s ``uncor_flag`` -> ``write_uncor_file``
    (``Print_Functions.py:144-156``, ``:120-126``) — run as a GPU sweep of the base decoder.

    Split k (training, _Valid, _Test) decodes the Philox stream ``seed + k`` at ``sigma`` in
    batches and appends the frames wrong at every iteration (compacted on the GPU) in the
    ``Uncor.txt`` row format (3 zero columns, negated LLRs, ``%.1f``) until it holds
    ``counts[k]`` rows.  Returns {path: (rows, codewords decoded)}."""
    import torch
    punct = tuple(getattr(decoder, "punct", (0, 0)) if punct is None else punct)
    short = tuple(getattr(decoder, "short", (0, 0)) if short is None else short)
    os.makedirs(out_dir, exist_ok=True)
    dev = decoder.device
    llr = torch.empty((batch, decoder.n_vars), dtype=torch.float32, device=dev)
    flags = torch.empty(batch, dtype=torch.uint8, device=dev)
    out = {}
    for k, (suffix, need) in enumerate(zip(("", "_Valid", "_Test"), counts)):
        path = os.path.join(out_dir, f"[Uncor]_{filename}{suffix}.txt")
        if os.path.exists(path):
            os.remove(path)
        have, pos = 0, 0
        while have < need:
            if pos >= max_codewords:
                raise RuntimeError(f"{path}: only {have} uncorrected words in {pos} codewords")
            decoder.awgn(batch, float(sigma), seed + k, offset=pos, punct=punct, short=short,
                         out=llr)
            decoder.decode(llr, T=T, app=False, flags=flags)
            rows = decoder.collect_uncorrected(flags, llr)
            if rows.shape[0]:
                rows = rows[:need - have]
                append_uncor_rows(rows, path, formatter=decoder.format_uncor_rows)
                have += rows.shape[0]
            pos += batch
        if need == 0:
            open(path, "w").close()
        out[path] = (have, pos)
    return out
