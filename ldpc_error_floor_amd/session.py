"""TF1-``Session``-compatible facade so the reference's FER loops run unchanged.

The reference evaluates its decoder with
``sess.run(fetches=net_dict["ya_output_all"] [, net_dict["lossa"]], feed_dict={net_dict['xa']:
X, net_dict['ya']: Y, net_dict['etha']: e, net_dict['learn_rate']: 0})``
(``Print_Functions.py:147-151``).  ``build_session`` returns ``(sess, net_dict)`` where
``net_dict`` maps the same keys to string handles and ``sess.run`` accepts those handles
(a single one or a list) plus ``ya_output{t}`` / ``ya_output_target{t}``.  The batch size is
fixed like the reference's placeholders (``main_Base.py:124-125``): a different B raises.

Parity mode on several GPUs (SURVEY §8 e: "host-generated LLRs, sliced by rank"), opt-in
with ``shard=True``: every rank runs the same host loop (``compute_results`` with the same
seeds, so every rank holds the same ``xa``), decodes its contiguous slice of the batch
(``fer.shard_range``) and ``all_gather``s the APP slices, so ``sess.run`` returns the whole
``ya_output_all`` on every rank and every rank computes the same ``Results``.  Each call first
checks (one all_reduce MIN/MAX of a checksum of ``xa``) that every rank fed the same batch and
raises otherwise.  Every rank must make the same sequence of ``run`` calls.  Without
``shard`` a Session never communicates, whatever ``torch.distributed`` holds: the reference
itself runs one process per GPU with no exchange (``main_Base.py:14-15``), and ranks under
torchrun may evaluate different configs or seeds.
"""
from __future__ import annotations

import numpy as np

from .code import TannerGraph, load_base_graph
from .config import NMSConfig
from .decoder import NMSDecoder
from .metrics import loss_forward
from .weights import DecoderWeights, expand_weights, read_weight_file

__all__ = ["Session", "build_session", "make_net_dict"]

FEED_KEYS = ("xa", "ya", "etha", "learn_rate")


def make_net_dict(T: int):
    d = {k: k for k in FEED_KEYS + ("ya_output_all", "lossa")}
    for t in range(T):
        d[f"ya_output{t}"] = f"ya_output{t}"
        d[f"ya_output_target{t}"] = f"ya_output_target{t}"
    return d


class Session:
    def __init__(self, decoder: NMSDecoder, batch_size: int, T=None, loss_type: int = 2,
                 loss_t_first=None, group=None, shard: bool = False):
        self.decoder = decoder
        self.batch_size = int(batch_size)
        self.T = decoder.T if T is None else int(T)
        self.loss_type = loss_type
        self.loss_t_first = loss_t_first
        self.group = group
        self.shard = bool(shard)
        self.calls = 0

    def _decode_app(self, X, target_bits=None):
        """APP [T, B, bits] of the host batch X on the host.  Sharded (``shard=True`` with
        more than one rank): this rank's slice decoded, the others gathered (one all_gather of
        equal-size padded slices)."""
        import torch
        import torch.distributed as dist
        from .fer import shard_range
        B = X.shape[0]
        dist_on = self.shard and dist.is_available() and dist.is_initialized()
        world = dist.get_world_size(self.group) if dist_on else 1
        if world == 1:
            return self.decoder.decode(X, T=self.T, app=True, target_bits=target_bits).app.cpu().numpy()
        rank = dist.get_rank(self.group)
        b0, b1 = shard_range(B, rank, world)
        nb = target_bits or self.decoder.target_bits
        per = -(-B // world)
        # RCCL gathers device tensors; gloo (CPU rehearsal) host tensors
        on_dev = dist.get_backend(self.group) == "nccl"
        dev = self.decoder.device if on_dev else torch.device("cpu")
        self._check_same_batch(X, dev)
        part = torch.zeros((self.T, per, nb), dtype=torch.float32, device=dev)
        if b1 > b0:
            app = self.decoder.decode(X[b0:b1], T=self.T, app=True, target_bits=target_bits).app
            part[:, :b1 - b0] = app.to(dev)
        parts = [torch.empty_like(part) for _ in range(world)]
        dist.all_gather(parts, part, group=self.group)
        out = np.empty((self.T, B, nb), np.float32)
        for r in range(world):
            r0, r1 = shard_range(B, r, world)
            out[:, r0:r1] = parts[r][:, :r1 - r0].cpu().numpy()
        return out

    def _check_same_batch(self, X, dev):
        """Raise unless every rank of the group fed the same ``xa`` (a sharded Session gathers
        the other ranks' APP rows, which are only this rank's answer if they decoded this
        rank's batch)."""
        import hashlib
        import torch
        import torch.distributed as dist
        h = hashlib.blake2b(np.ascontiguousarray(X).tobytes(), digest_size=7).digest()
        v = int.from_bytes(h, "little")                  # < 2^56: exact in int64
        lo = torch.tensor([v, -v], dtype=torch.int64, device=dev)
        dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=self.group)
        if int(lo[0]) != v or int(lo[1]) != -v:
            raise RuntimeError("Session(shard=True): the ranks fed different xa batches to "
                               "sess.run; a sharded parity run needs the same host stream on "
                               "every rank")

    def run(self, fetches, feed_dict):
        single = not isinstance(fetches, (list, tuple))
        keys = [fetches] if single else list(fetches)
        feed = {(k if isinstance(k, str) else str(k)): v for k, v in feed_dict.items()}
        if "xa" not in feed:
            raise KeyError("feed_dict must provide 'xa'")
        X = np.asarray(feed["xa"], dtype=np.float32)
        B = X.shape[0]
        if B != self.batch_size:
            raise ValueError(f"xa batch {B} != placeholder batch {self.batch_size} "
                             "(the reference's placeholders have a fixed batch size)")
        app = self._decode_app(X.reshape(B, -1))              # [T, B, Nt*z]
        self.calls += 1
        out = []
        T = self.T
        full = None
        for k in keys:
            if k == "ya_output_all":
                out.append(app.reshape(T * B, -1))
            elif k == "lossa":
                out.append(np.float32(loss_forward(app.reshape(T * B, -1), T, B, self.loss_type,
                                                   float(feed.get("etha", 0.0)), feed.get("ya"),
                                                   self.loss_t_first)))
            elif k.startswith("ya_output_target"):
                out.append(app[int(k[len("ya_output_target"):])])
            elif k.startswith("ya_output"):
                t = int(k[len("ya_output"):])
                if self.decoder.target_bits == self.decoder.n_vars:
                    out.append(app[t])
                else:
                    if full is None:
                        full = self._decode_app(X.reshape(B, -1), target_bits=self.decoder.n_vars)
                    out.append(full[t])
            else:
                raise KeyError(f"unsupported fetch {k!r}")
        return out[0] if single else out


def build_session(cfg: NMSConfig, proto=None, weights: DecoderWeights = None, device=None,
                  kernel: str = "auto", graph_dir=None, group=None, shard: bool = False):
    """Decoder + Session + net_dict for a reference-style config.  ``shard=True``: a
    multi-GPU parity run that splits each batch over the ranks of ``group`` (default: the
    default group); off by default, so every rank decodes its own batches alone."""
    import os
    from .code import default_graph_dir
    cfg.validate()
    if proto is None:
        gd = graph_dir or os.path.join(default_graph_dir(), "BaseGraph")
        proto = load_base_graph(os.path.join(gd, cfg.filename + ".txt"))
    g = TannerGraph(proto, cfg.z_value)
    T = cfg.iters_max
    if weights is None:
        if cfg.weights_file is None:
            raise ValueError("weights or cfg.weights_file required")
        wf = read_weight_file(cfg.weights_file)
        weights = expand_weights(cfg.sharing, wf.blocks, T, g, cfg.fixed_iter)
    dec = NMSDecoder(proto, cfg.z_value, weights, cfg.decoding_type, cfg.q_bit,
                     cfg.target_node(g.N, g.M), cfg.clip_LLR, device=device, kernel=kernel)
    # the channel's puncture / shorten ranges (create_mix_epoch, Print_Functions.py:29-72) become
    # the defaults of dec.awgn / dec.decode_awgn / fer_sweep(dec, ...)
    dec.punct = (int(cfg.punct_start), int(cfg.punct_end))
    dec.short = (int(cfg.short_start), int(cfg.short_end))
    t_first = max(cfg.iters_max - cfg.iter_step - cfg.fixed_init, cfg.fixed_iter)
    sess = Session(dec, cfg.batch_size, T, cfg.loss_type, t_first, group=group, shard=shard)
    return sess, make_net_dict(T)
