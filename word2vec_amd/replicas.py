"""Multi-GPU data parallelism for the hot path: corpus shards + replica averaging.

The reference parallelises only with OpenMP threads sharing one model
(Word2Vec.cpp:375-394). Across GPUs this framework runs one process per GPU
(torchrun), gives each rank a contiguous shard of the sentences and a full
model replica in its HBM, trains the shard with the Hogwild kernels, and at
the end of every round (every `sync_every` sentences of the largest shard, the
same round count on every rank) exchanges what the replicas learned.

The exchange is native: `NativeAverager` wraps the C-ABI's RCCL group
(include/w2v_dev.h w2v_group_*: the replicas' updates since the last exchange
summed with one ncclAllReduce per matrix over xGMI, then combined per `mode`:
"sum" (every update once, as one shared model), "average" (model averaging:
the mean), "row_average" (per row, the mean over the replicas that changed
it), "adaptive", or the per-row divisors of set_split / set_saturation;
optionally overlapped with the next round's training). The constructor's
default is "sum" with overlap off (the primitive, as the tests drive it);
bench.py and Word2Vec::replica_mode pick "auto": the mean for up to four
replicas of long shards (>= 64 x 4 M words: configs[3]'s scale), else the sum
for two replicas and adaptive for more (summing R >= 3 replicas diverges on
the frequent rows, plain averaging of short shards loses the rare rows'
progress; measured tables in DESIGN.md §6), with the exchange overlapped.
`TorchAverager` (model averaging
over torch.distributed) is what the CPU tests run on the gloo backend to
exercise the round logic, which is the same object code. `make_averager` is
bench.py's per-rank construction (the group id broadcast included); the CPU
tests drive it against a stub of the C-ABI's group calls, and on a one-GPU box
it builds the `RehearsalAverager`.

The alpha schedule stays global without a collective per round: each rank
knows every rank's words per round (exchanged once, `global_round_words`), sets
its device counter to (global words at the round start) / world and its
train_words to (global raw tokens) / world, so alpha follows the reference's
schedule of the global count (Word2Vec.cpp:362-363,379-380) while the ranks
progress in step.
"""
from __future__ import annotations

import ctypes as C
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


def agree_rounds(rounds: int, world: int, group=None) -> int:
    """The largest of the ranks' round counts (every rank must run the same
    number of exchanges; shards of a synthetic or real corpus differ by a few
    words, and a per-rank ceil near an integer would split them)."""
    if world <= 1:
        return rounds
    t = torch.tensor([int(rounds)], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def round_slices(n: int, rounds: int) -> list[tuple[int, int]]:
    """Cut [0, n) into `rounds` consecutive near-equal slices (some may be empty)."""
    return [(n * k // rounds, n * (k + 1) // rounds) for k in range(rounds)]


def local_round_words(sent_offsets, order, rounds: int) -> list[int]:
    """In-vocab words of each round's slice of `order` (sentence ids into
    sent_offsets): what the device counter advances by in that round."""
    import numpy as np

    off = np.asarray(sent_offsets, dtype=np.int64)
    o = np.asarray(order, dtype=np.int64)
    lens = off[o + 1] - off[o]
    cum = np.concatenate([[0], np.cumsum(lens)])
    return [int(cum[hi] - cum[lo]) for lo, hi in round_slices(o.size, rounds)]


def global_round_words(local: list[int], world: int, group=None, device="cpu") -> list[int]:
    """Sum over ranks of each round's words (one small all-reduce, once)."""
    if world == 1:
        return list(local)
    t = torch.tensor(local, dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return [int(x) for x in t.cpu().tolist()]


@dataclass
class TorchAverager:
    """In-place mean of this rank's replica tensors over torch.distributed
    (the CPU tests' gloo backend; gloo has no AVG: sum then divide)."""

    tensors: list
    world: int
    group: object = None

    def average(self) -> None:
        if self.world == 1:
            return
        for t in self.tensors:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            t.div_(self.world)

    def finish(self) -> None:
        pass


def _handle(trainer):
    return trainer.h.value if isinstance(trainer.h, C.c_void_p) else trainer.h


class NativeAverager:
    """The C-ABI's RCCL replica group (w2v_group_*) over this process's device
    handles; `unique_id` (W2V_GROUP_ID_BYTES bytes from group_unique_id() on
    rank 0) joins the handles to a multi-process group as ranks
    [first_rank, first_rank + len(trainers)) of `nranks`."""

    def __init__(self, trainers, unique_id: bytes | None = None, nranks: int | None = None, first_rank: int = 0,
                 overlap: bool = False, mode: str = "sum"):
        from . import _native as N

        self.N = N
        self.lib = N.load_dev_lib()
        arr = (C.c_void_p * len(trainers))(*[t.h.value if isinstance(t.h, C.c_void_p) else t.h for t in trainers])
        g = C.c_void_p()
        uid = None if unique_id is None else (C.c_uint8 * N.W2V_GROUP_ID_BYTES).from_buffer_copy(unique_id)
        N.check(self.lib, self.lib.w2v_group_create(arr, len(trainers), uid, int(nranks or len(trainers)),
                                                    int(first_rank), C.byref(g)), "w2v_group_create")
        self.g = g
        self.trainers = trainers
        N.check(self.lib, self.lib.w2v_group_set_overlap(self.g, int(bool(overlap))), "w2v_group_set_overlap")
        modes = {"row_average": N.W2V_GROUP_ROW_AVERAGE, "sum": N.W2V_GROUP_SUM, "average": N.W2V_GROUP_AVERAGE,
                 "adaptive": N.W2V_GROUP_ADAPTIVE}
        N.check(self.lib, self.lib.w2v_group_set_mode(self.g, modes[mode]), "w2v_group_set_mode")

    def set_split(self, tokens_per_round: int, saturated_updates: float) -> int:
        """W2V_GROUP_SPLIT: the mean of the replicas' updates for rows expected to be updated >=
        saturated_updates times per replica in a round of tokens_per_round tokens, the sum for the rest.
        Returns the number of averaged rows."""
        self.N.check(self.lib, self.lib.w2v_group_set_split(self.g, int(tokens_per_round), float(saturated_updates)),
                     "w2v_group_set_split")
        n = C.c_int64()
        self.N.check(self.lib, self.lib.w2v_group_split_rows(self.g, C.byref(n)), "w2v_group_split_rows")
        return n.value

    def set_saturation(self, tokens_per_round: int, beta: float) -> int:
        """W2V_GROUP_SATURATION: the summed update divided per row by R(1-(1-beta)^u)/(1-(1-beta)^(Ru)), u =
        the row's expected updates per replica in a round of tokens_per_round tokens (the sum for rarely
        updated rows, the mean for rows every replica saturates within the round). Returns the rows with a
        divisor above 1."""
        self.N.check(self.lib, self.lib.w2v_group_set_saturation(self.g, int(tokens_per_round), float(beta)),
                     "w2v_group_set_saturation")
        n = C.c_int64()
        self.N.check(self.lib, self.lib.w2v_group_split_rows(self.g, C.byref(n)), "w2v_group_split_rows")
        return n.value

    def row_divisors(self, which: int, rows: int):
        """The per-row divisors of matrix `which` the exchange applies (all 1 outside SPLIT / SATURATION)."""
        import numpy as np

        out = np.empty(rows, np.float32)
        self.N.check(self.lib, self.lib.w2v_group_row_divisors(self.g, int(which), out.ctypes.data_as(C.POINTER(C.c_float)),
                                                               int(rows)), "w2v_group_row_divisors")
        return out

    def average(self, rows: int = 0) -> None:
        """Exchange all rows (rows == 0) or only the `rows` hottest (W / C rows [0, rows), the nodes nearest
        the Huffman root)."""
        if rows:
            self.N.check(self.lib, self.lib.w2v_group_average_rows_async(self.g, int(rows)),
                         "w2v_group_average_rows_async")
        else:
            self.N.check(self.lib, self.lib.w2v_group_average_async(self.g), "w2v_group_average_async")

    def finish(self) -> None:
        self.N.check(self.lib, self.lib.w2v_group_finish(self.g), "w2v_group_finish")

    def info(self) -> dict:
        n, loc, ov, r = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64()
        self.N.check(self.lib, self.lib.w2v_group_info(self.g, C.byref(n), C.byref(loc), C.byref(ov), C.byref(r)),
                     "w2v_group_info")
        return {"nranks": n.value, "local": bool(loc.value), "overlap": bool(ov.value), "rounds": r.value}

    def close(self) -> None:
        if getattr(self, "g", None):
            self.lib.w2v_group_destroy(self.g)
            self.g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def group_unique_id() -> bytes:
    from . import _native as N

    lib = N.load_dev_lib()
    buf = (C.c_uint8 * N.W2V_GROUP_ID_BYTES)()
    N.check(lib, lib.w2v_group_unique_id(buf), "w2v_group_unique_id")
    return bytes(buf)


class RehearsalAverager:
    """The N > 1 path rehearsed with every rank on ONE GPU (RCCL refuses two
    ranks on one device: "Duplicate GPU detected"). Each rank runs the native
    exchange on a one-rank RCCL communicator — the same group calls per round
    (delta kernel, ncclAllReduce on the communication stream, fold; with one
    rank an identity on the model) — and the cross-process combination is the
    mean over torch.distributed (gloo). Only ncclCommInitRank with more than
    one rank, and the multi-rank all-reduce, are new on a multi-GPU node."""

    def __init__(self, native: NativeAverager, torch_avg: TorchAverager):
        self.native, self.torch_avg = native, torch_avg

    def average(self) -> None:
        self.native.average()
        self.torch_avg.average()

    def finish(self) -> None:
        self.native.finish()

    def info(self) -> dict:
        return self.native.info()

    def close(self) -> None:
        self.native.close()


def make_averager(trainer, mats, world: int, rank: int, mode: str, overlap: bool, share_gpu: bool = False):
    """The replica exchange of bench.py --gpus N, one call per rank (world > 1
    needs torch.distributed initialised: the group id travels over it):
      * world 1: a no-op;
      * one rank per GPU: the native RCCL group over all ranks (rank 0 makes
        the unique id, broadcast to the others) in `mode`;
      * share_gpu (the one-GPU rehearsal): RehearsalAverager — rank 0 makes one
        id per rank, broadcast the same way, each rank a one-rank native group,
        the mean over torch.distributed across the processes.
    Returns (averager, description)."""
    if world == 1:
        return TorchAverager(mats, 1), "dp1"
    if not share_gpu:
        uid = [group_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        return NativeAverager([trainer], uid[0], world, rank, overlap=overlap, mode=mode), f"{mode} (w2v_group)"
    uids = [[group_unique_id() for _ in range(world)] if rank == 0 else None]
    dist.broadcast_object_list(uids, src=0)
    native = NativeAverager([trainer], uids[0][rank], 1, 0, overlap=overlap, mode=mode)
    # the one-rank group told the handle "1 replica": the rehearsal trains with
    # the policy an N-GPU run uses
    native.N.check(native.lib, native.lib.w2v_dev_set_replica_count(_handle(trainer), int(world)),
                   "w2v_dev_set_replica_count")
    return RehearsalAverager(native, TorchAverager(mats, world)), "rehearsal: one-rank w2v_group per process + gloo mean"


def train_rounds(trainer, averager, order_dev: torch.Tensor, epoch: int, rounds: int, progress_base: int,
                 round_words: list[int], world: int, events: list | None = None) -> int:
    """One epoch of this rank's shard in `rounds` rounds, all enqueued on the
    trainer's stream without a host sync: per round, the device counter is set
    to (global words at the round start) / world, the slice trains, and the
    replicas are averaged. `progress_base` is the global word count at epoch
    start, round_words[r] the words all ranks train in round r; returns the
    global count at epoch end. If `events` is a list, a (start, end)
    torch.cuda.Event pair around every kernel launch is appended to it (they
    are recorded on torch's current stream, which must be the trainer's)."""
    n = order_dev.numel()
    g = progress_base
    for r, (lo, hi) in enumerate(round_slices(n, rounds)):
        trainer.set_progress_async(g // world)
        if hi > lo:
            ev = None
            if events is not None:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            trainer.train_sentences_async(epoch, order_dev.data_ptr() + 8 * lo, hi - lo)
            if ev is not None:
                ev[1].record()
                events.append(ev)
        averager.average()
        g += round_words[r]
    return g
