"""Communicator bootstrap agreement (parallel/comm.py ``_Agreement``) over a 2-rank gloo group: votes
go through the rendezvous store with a deadline, a rank's early failure is visible to its peers (so a
peer inside a non-blocking RCCL init aborts it), and a missing vote ends the job instead of a hang."""
import os
import tempfile

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.timeout(300)


def _worker(rank, world, path, mode, q):
    import torch.distributed as dist
    from dbx_distributed_pytorch_examples_amd.parallel.comm import CommAgreementTimeout, _Agreement
    dist.init_process_group("gloo", init_method=f"file://{path}", rank=rank, world_size=world)
    try:
        ag = _Agreement(None)
        if mode == "vote":
            q.put((rank, ag.all_true(True, "a", 30), ag.all_true(rank == 0, "b", 30)))
        elif mode == "fail":
            if rank == 1:
                ag.post_failure("construction raised")
            dist.barrier()
            q.put((rank, ag.peer_failed()))
        elif mode == "missing":
            if rank == 0:
                try:
                    ag.all_true(True, "c", 3)
                    q.put((rank, "no timeout"))
                except CommAgreementTimeout as e:
                    q.put((rank, "timeout" if "'c'" in str(e) else str(e)))
            else:
                q.put((rank, "skipped"))
        # a second agreement gets a fresh key space (generation counter)
        ag2 = _Agreement(None)
        assert ag2.prefix != ag.prefix
    finally:
        dist.destroy_process_group()


def _run(mode):
    path = os.path.join(tempfile.mkdtemp(), "pg")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, path, mode, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict()
    for _ in range(2):
        r, *v = q.get(timeout=120)
        out[r] = v
    for p in ps:
        p.join(60)
    return out


def test_votes_agree():
    out = _run("vote")
    assert out[0] == [True, False] and out[1] == [True, False]


def test_early_failure_is_visible_to_peers():
    out = _run("fail")
    assert out[0] == [True] and out[1] == [True]


def test_missing_vote_times_out():
    out = _run("missing")
    assert out[0] == ["timeout"]
