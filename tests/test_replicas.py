"""Multi-rank logic of word2vec_amd/replicas.py on CPU with gloo (world 2 and 3):
shards partition the corpus, averaging is the exact mean, the per-round global
word counts are the sum over ranks, and the round loop drives a trainer the
way the GPU path does (a fake trainer stands in for the HIP handle, the
torch/gloo averager for the native RCCL group)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from word2vec_amd.replicas import (TorchAverager, global_round_words, local_round_words, n_rounds, round_slices,
                                   shard_range, train_rounds)


def test_shard_range_partitions():
    for n in (0, 1, 7, 100, 1001):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_round_slices_and_counts():
    assert round_slices(10, 3) == [(0, 3), (3, 6), (6, 10)]
    assert round_slices(2, 3) == [(0, 0), (0, 1), (1, 2)]
    assert round_slices(0, 2) == [(0, 0), (0, 0)]
    assert n_rounds(15, 2, 3) == 3 and n_rounds(15, 2, 0) == 1 and n_rounds(7, 3, 1) == 3
    # uneven shards still get the same number of rounds on every rank
    for n in (7, 15, 100):
        for world in (2, 3, 8):
            r = n_rounds(n, world, 4)
            for rank in range(world):
                lo, hi = shard_range(n, rank, world)
                assert len(round_slices(hi - lo, r)) == r


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_local_round_words():
    off = [0, 3, 5, 9, 10]  # sentence lengths 3, 2, 4, 1
    assert local_round_words(off, [2, 0, 3, 1], 2) == [7, 3]
    assert local_round_words(off, [0, 1, 2, 3], 3) == [3, 2, 5]
    assert sum(local_round_words(off, [3, 2, 1, 0], 1)) == 10


class FakeTrainer:
    """Adds (rank+1) to every replica element per trained sentence and counts
    10 words per sentence, like a device handle bound to the tensors; records
    the progress values the round loop sets."""

    def __init__(self, tensors, rank):
        self.t, self.rank, self.words = tensors, rank, 0
        self.seen, self.progress = [], []

    def set_progress_async(self, w):
        self.words = w
        self.progress.append(w)

    def train_sentences_async(self, epoch, ptr, count):
        self.seen.append(count)
        for t in self.t:
            t.add_(float((self.rank + 1) * count))
        self.words += 10 * count


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        W = torch.full((4, 8), float(rank), dtype=torch.float32)
        C = torch.arange(32, dtype=torch.float32).reshape(4, 8) * (rank + 1)
        g = TorchAverager([W, C], world)
        g.average()
        mean_rank = sum(range(world)) / world
        assert torch.allclose(W, torch.full_like(W, mean_rank))
        assert torch.allclose(C, torch.arange(32, dtype=torch.float32).reshape(4, 8) * (world + 1) / 2)
        # round loop: uneven shards of 15 sentences of 10 words, sync every 3 of the largest
        lo, hi = shard_range(15, rank, world)
        order = torch.arange(lo, hi, dtype=torch.int64)
        R = n_rounds(15, world, 3)
        off = [10 * k for k in range(16)]
        rw = global_round_words(local_round_words(off, order.tolist(), R), world)
        W.zero_()
        tr = FakeTrainer([W], rank)
        total = train_rounds(tr, TorchAverager([W], world), order, 0, R, 100, rw, world)
        out.put((rank, tr.seen, total, W[0, 0].item(), tr.progress, rw))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_replica_averaging_and_rounds(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # every rank ran the same number of rounds; progress = 100 + 10 words x 15 sentences
    totals = {r[2] for r in res}
    assert totals == {100 + 10 * 15}
    # the counter each rank starts a round from is the global count / world
    rw = res[0][5]
    assert sum(rw) == 150 and all(r[5] == rw for r in res)
    starts = [100 + sum(rw[:k]) for k in range(len(rw))]
    assert all(r[4] == [s // world for s in starts] for r in res)
    # the replica after the rounds is identical on every rank and equals the
    # sequence of averaged round updates
    vals = {round(r[3], 4) for r in res}
    assert len(vals) == 1
    expect = 0.0
    R = n_rounds(15, world, 3)
    rounds = [round_slices(shard_range(15, r, world)[1] - shard_range(15, r, world)[0], R) for r in range(world)]
    for k in range(len(rounds[0])):
        expect += sum((r + 1) * (rounds[r][k][1] - rounds[r][k][0]) for r in range(world)) / world
    assert abs(vals.pop() - expect) < 1e-4
