"""bench.py's N-rank bookkeeping, rehearsed on CPU: which engines each rank
drives, which lines each engine holds, and the collective sequence of the
timed regions (barriers, max-over-ranks clock), at world size 8 over gloo.

The driver launches `bench.py --gpus 8` as 8 ranks of torch.distributed.run;
in node mode rank 0 drives every GPU through one bjx_node and ranks 1-7 only
join the barriers.  A rank that calls one collective fewer than the others
hangs the job, so every rank here runs bench.timed_region itself (the function
main() uses) with a stand-in step, and the test checks that all ranks made the
same collective calls and read the same clock."""
import os
import socket
import time

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench

WORLD = 8


def test_rank_plan_node_mode_world8():
    n = 1000
    plans = [bench.rank_plan(WORLD, r, r, 0, "node", 8, n) for r in range(WORLD)]
    assert plans[0]["drives"] and not any(p["drives"] for p in plans[1:])
    assert all(p["node_mode"] and p["n_parts"] == WORLD and p["devices"] == list(range(8)) for p in plans)
    chunks = plans[0]["chunks"]
    assert [c[0] for c in chunks] == list(range(8))  # engine k on GPU k
    covered = sorted((lo, lo + m) for _, lo, m in chunks)
    assert covered[0][0] == 0 and covered[-1][1] == WORLD * n
    assert all(a[1] == b[0] for a, b in zip(covered, covered[1:]))  # every line exactly once
    assert all(p["chunks"] == [] for p in plans[1:])


def test_rank_plan_rccl_and_single_process():
    n = 500
    plans = [bench.rank_plan(WORLD, r, r, 0, "rccl", 8, n) for r in range(WORLD)]
    assert all(p["drives"] and not p["node_mode"] for p in plans)
    assert [p["chunks"] for p in plans] == [[(r, r * n, n)] for r in range(WORLD)]
    # --node-engines 2 on a one-GPU box: one process, two engines on device 0
    p = bench.rank_plan(1, 0, 0, 2, "node", 1, n)
    assert p["node_mode"] and p["drives"] and p["devices"] == [0, 0]
    assert p["chunks"] == [(0, 0, n), (0, n, n)]
    p = bench.rank_plan(1, 0, 0, 0, "node", 1, n)
    assert not p["node_mode"] and p["chunks"] == [(0, 0, n)]


def test_rank_plan_single_process_gpus8():
    """`python3 bench.py --gpus 8` with no launcher (WORLD_SIZE unset): one
    process drives 8 engines on 8 distinct devices through one bjx_node."""
    n = 700
    p = bench.rank_plan(1, 0, 0, 0, "node", 8, n, gpus=8)
    assert p["node_mode"] and p["drives"] and p["n_parts"] == 8
    assert p["devices"] == list(range(8)) and len(set(p["devices"])) == 8
    assert p["chunks"] == [(k, k * n, n) for k in range(8)]
    # --gpus 1 is the plain single-engine run
    p = bench.rank_plan(1, 0, 0, 0, "node", 8, n, gpus=1)
    assert not p["node_mode"] and p["chunks"] == [(0, 0, n)]
    # fewer devices than asked for: refuse instead of timing fewer GPUs
    with pytest.raises(SystemExit):
        bench.rank_plan(1, 0, 0, 0, "node", 4, n, gpus=8)
    with pytest.raises(SystemExit):
        bench.rank_plan(1, 0, 0, 2, "node", 8, n, gpus=8)
    # under a launcher every rank sees WORLD_SIZE and the node of rank 0 is unchanged
    p = bench.rank_plan(8, 0, 0, 0, "node", 8, n, gpus=8)
    assert p["devices"] == list(range(8)) and p["drives"]


class _Counted:
    """torch.distributed with its collectives counted (in call order)."""

    def __init__(self):
        self.calls = []
        self.ReduceOp = dist.ReduceOp

    def barrier(self):
        self.calls.append("barrier")
        dist.barrier()

    def all_reduce(self, t, op):
        self.calls.append("all_reduce")
        dist.all_reduce(t, op=op)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    D = _Counted()
    P = bench.rank_plan(WORLD, rank, rank, 0, "node", 8, 1000)
    done = []

    def step():  # the driving rank does the work of all 8 engines
        if P["drives"]:
            time.sleep(0.02)
            done.append(len(P["chunks"]))
        return None

    el, outs = bench.timed_region(D, step, lambda: None, 3, "cpu")
    el2, _ = bench.timed_region(D, step, lambda: None, 2, "cpu")  # the decision-emission re-timing
    D.barrier()
    q.put((rank, el, el2, D.calls, len(outs), sum(done)))
    dist.destroy_process_group()


def test_timed_regions_world8_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    calls = [r[3] for r in res]
    assert all(c == calls[0] for c in calls)  # same collectives in the same order on every rank
    assert calls[0].count("barrier") == 5 and calls[0].count("all_reduce") == 2
    # every rank reports the driving rank's time (max over ranks), which covers its 3 + 2 steps
    assert len({r[1] for r in res}) == 1 and len({r[2] for r in res}) == 1
    assert res[0][1] >= 3 * 0.02 and res[0][2] >= 2 * 0.02
    assert res[0][5] == 5 * WORLD and all(r[5] == 0 for r in res[1:])  # rank 0 stepped all 8 engines
    assert all(r[4] == 3 for r in res)
