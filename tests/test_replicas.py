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

from word2vec_amd.replicas import (TorchAverager, agree_rounds, global_round_words, local_round_words, n_rounds, round_slices,
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
        # bench.py's per-rank round counts (a ceil of each rank's own shard) agree on the largest
        agreed = agree_rounds(5 + rank, world)
        out.put((rank, tr.seen, total, W[0, 0].item(), tr.progress, rw, agreed))
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
    assert {r[6] for r in res} == {5 + world - 1}
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


# ---- bench.py's per-rank exchange (make_averager) against a stub group -------
class StubGroupLib:
    """Stands in for libw2v_hip.so's w2v_group_* calls (include/w2v_dev.h) on
    CPU: the "group" is the process's gloo world, the handles' models are the
    FakeTrainer tensors (looked up by handle value). average_async sums the
    replicas' changes since the last exchange (D = M - P) over gloo and folds
    them per the mode, as the native group does (w2v_group.hip: sum c = 1,
    average c = nranks); every call is logged for the assertions."""

    def __init__(self, models):
        self.models, self.calls, self.groups = models, [], {}

    def w2v_group_unique_id(self, buf):
        self.calls.append(("unique_id",))
        for i in range(len(buf)):
            buf[i] = (7 * i + 3) % 256
        return 0

    def w2v_group_create(self, arr, n, uid, nranks, first_rank, pg):
        hs = [arr[i] for i in range(n)]
        self.calls.append(("create", hs, bytes(uid) if uid is not None else None, nranks, first_rank))
        gid = 100 + len(self.groups)
        self.groups[gid] = {"handles": hs, "nranks": nranks, "mode": 0, "overlap": 0, "rounds": 0,
                            "snap": [[t.clone() for t in self.models[h]] for h in hs]}
        pg._obj.value = gid
        return 0

    def w2v_group_set_overlap(self, g, on):
        self.groups[g.value]["overlap"] = on
        return 0

    def w2v_group_set_mode(self, g, mode):
        self.groups[g.value]["mode"] = mode
        return 0

    def w2v_group_average_async(self, g):
        from word2vec_amd import _native as N

        st = self.groups[g.value]
        st["rounds"] += 1
        self.calls.append(("average", g.value))
        c = st["nranks"] if st["mode"] == N.W2V_GROUP_AVERAGE else 1
        for h, snap in zip(st["handles"], st["snap"]):
            for m, p in zip(self.models[h], snap):
                d = m - p
                if st["nranks"] > 1:
                    dist.all_reduce(d)
                m.copy_(p + d / c)
                p.copy_(m)
        return 0

    def w2v_group_finish(self, g):
        self.calls.append(("finish", g.value))
        return 0

    def w2v_group_info(self, g, n, loc, ov, r):
        st = self.groups[g.value]
        n._obj.value, loc._obj.value, ov._obj.value, r._obj.value = st["nranks"], 0, st["overlap"], st["rounds"]
        return 0

    def w2v_group_destroy(self, g):
        self.calls.append(("destroy", g.value))

    def w2v_dev_set_replica_count(self, h, n):
        self.calls.append(("replica_count", h, n))
        return 0

    def w2v_dev_last_error(self):
        return b"stub"


class _Handle:
    def __init__(self, tr, h):
        import ctypes

        self.tr, self.h = tr, ctypes.c_void_p(h)

    def __getattr__(self, k):
        return getattr(self.tr, k)


def _worker_make_averager(rank, world, port, out, share):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from word2vec_amd import _native as N
        from word2vec_amd import replicas

        W = torch.zeros(4, 8)
        handle = 0x1000 + rank
        stub = StubGroupLib({handle: [W]})
        N.load_dev_lib = lambda path=None: stub  # this spawned process only
        tr = _Handle(FakeTrainer([W], rank), handle)
        mode = "average"
        avg, desc = replicas.make_averager(tr, [W], world, rank, mode, True, share)
        lo, hi = shard_range(16, rank, world)
        order = torch.arange(lo, hi, dtype=torch.int64)
        R = n_rounds(16, world, 3)
        off = [10 * k for k in range(17)]
        rw = global_round_words(local_round_words(off, order.tolist(), R), world)
        total = train_rounds(tr, avg, order, 0, R, 0, rw, world)
        avg.finish()
        info = avg.info()
        avg.close()
        out.put((rank, desc, stub.calls, info, total, W[0, 0].item(), R))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("share", [False, True])
def test_make_averager_stub_group_world2(share):
    """bench.py --gpus 2's exchange on CPU with a stub of the native group:
    rank 0 makes the group id(s), gloo carries them, every rank creates its
    group with the right (nranks, first_rank) — (2, rank) across GPUs, (1, 0)
    with its own id in the one-GPU rehearsal — runs one exchange per round,
    and the replicas end identical (the mean of the ranks' updates, by the
    group across GPUs, by gloo in the rehearsal)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_make_averager, args=(r, world, port, q, share)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    uid0 = bytes((7 * i + 3) % 256 for i in range(128))
    for rank, desc, calls, info, total, w, R in res:
        creates = [c for c in calls if c[0] == "create"]
        assert len(creates) == 1
        _, hs, uid, nranks, first = creates[0]
        assert hs == [0x1000 + rank] and uid == uid0
        assert (nranks, first) == ((1, 0) if share else (world, rank))
        # the rehearsal's policy assumes the run's replica count, not its one-rank group's
        rc = [c for c in calls if c[0] == "replica_count"]
        assert rc == ([("replica_count", 0x1000 + rank, world)] if share else [])
        if share:
            assert calls.index(rc[0]) > calls.index(creates[0])
        # only rank 0 makes ids: one per rank in the rehearsal, one for the group otherwise
        n_ids = sum(c[0] == "unique_id" for c in calls)
        assert n_ids == ((world if share else 1) if rank == 0 else 0)
        assert sum(c[0] == "average" for c in calls) == R == info["rounds"]
        assert info["overlap"] == 1 and info["nranks"] == nranks
        assert calls[-1][0] == "destroy"
        assert ("rehearsal" in desc) == share
        assert total == 160
    assert res[0][5] == res[1][5]
    # each round adds (rank + 1) x sentences on each rank; the mean over the ranks
    rounds = [round_slices(shard_range(16, r, world)[1] - shard_range(16, r, world)[0], res[0][6]) for r in range(world)]
    expect = sum(sum((r + 1) * (rounds[r][k][1] - rounds[r][k][0]) for r in range(world)) / world
                 for k in range(res[0][6]))
    assert abs(res[0][5] - expect) < 1e-4
