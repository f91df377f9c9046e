"""Multi-GPU data parallelism for the hot path: corpus shards + replica averaging.

The reference parallelises only with OpenMP threads sharing one model
(Word2Vec.cpp:375-394). Across GPUs this framework runs one process per GPU
(torchrun), gives each rank a contiguous shard of the sentences and a full
model replica in its HBM, trains the shard with the Hogwild kernels, and at
the end of every round (every `sync_every` sentences of the largest shard, the
same round count on every rank) averages the replicas with an RCCL all-reduce over xGMI
(backend "nccl" is RCCL on ROCm). The alpha schedule follows the GLOBAL word
count: after each averaging round the per-rank counters are summed and every
rank resumes from the sum, with train_words the global raw-token total
(Word2Vec.cpp:362-363,379-380).

Works unchanged on the gloo backend with CPU tensors (the CPU tests use that).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist


def shard_range(n_items: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced [lo, hi) of n_items for `rank` (sizes differ by at most 1)."""
    base, extra = divmod(n_items, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def n_rounds(n_total: int, world: int, sync_every: int) -> int:
    """Averaging rounds per epoch, the same on every rank (a rank that ran a
    different number of collectives would deadlock the group): enough rounds
    that the largest shard syncs at least every `sync_every` sentences."""
    largest = -(-n_total // world)
    if sync_every <= 0 or largest == 0:
        return 1
    return max(1, -(-largest // sync_every))


def round_slices(n: int, rounds: int) -> list[tuple[int, int]]:
    """Cut [0, n) into `rounds` consecutive near-equal slices (some may be empty)."""
    return [(n * k // rounds, n * (k + 1) // rounds) for k in range(rounds)]


@dataclass
class ReplicaGroup:
    """The replicas of W / C / synapses1 held by this rank (torch tensors that
    the device handle was bound to with w2v_dev_bind_model)."""

    tensors: list
    world: int
    group: object = None

    def average(self) -> None:
        """In-place mean over ranks. One all-reduce per matrix: each is one
        large contiguous buffer (V x pitch fp32), the message size RCCL's
        ring/tree algorithms over xGMI run at full link rate."""
        if self.world == 1:
            return
        for t in self.tensors:
            if dist.get_backend(self.group) == "nccl":
                dist.all_reduce(t, op=dist.ReduceOp.AVG, group=self.group)
            else:  # gloo has no AVG
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
                t.div_(self.world)

    def global_progress(self, local_words: int, device) -> int:
        """Sum of the ranks' in-vocab word counters (the reference's current_words)."""
        if self.world == 1:
            return int(local_words)
        v = torch.tensor([int(local_words)], dtype=torch.int64, device=device)
        dist.all_reduce(v, op=dist.ReduceOp.SUM, group=self.group)
        return int(v.item())


def train_rounds(trainer, replicas: ReplicaGroup, order_dev: torch.Tensor, epoch: int, rounds: int,
                 device, progress_base: int, events: list | None = None) -> int:
    """One epoch of this rank's shard in rounds: train a slice of the order on
    the device, average the replicas, move every rank to the global progress.
    `progress_base` is the global word count at epoch start; returns the new one.
    The kernels and the collectives are ordered on the current stream; if
    `events` is a list, a (start, end) timing-event pair around every kernel
    launch is appended to it."""
    n = order_dev.numel()
    global_words = progress_base
    for lo, hi in round_slices(n, rounds):
        trainer.set_progress(global_words)
        if hi > lo:
            ev = None
            if events is not None:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            trainer.train_sentences_async(epoch, order_dev.data_ptr() + 8 * lo, hi - lo)
            if ev is not None:
                ev[1].record()
                events.append(ev)
        replicas.average()
        local = trainer.get_progress() - global_words
        global_words += replicas.global_progress(local, device)
    return global_words
