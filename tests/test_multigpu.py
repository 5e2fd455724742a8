"""The multi-GPU code paths on one MI355X.

* RCCL itself, with a one-rank communicator: what RCCL reports, the all-reduce used as
  the timing barrier and max, the all-gathers, and bh_prove_witness_partial_comm.
* The per-rank code of a multi-GPU run with N ranks as N contexts and host threads on
  one device (bh_prove_witness_partials_ranks): each rank holding its own Parameters with
  only its shard's window-table slices and, with the H block distributed, its gathered
  share of the h vector -- exactly the memory layout of the processes of an N-GPU run.
  The recombined proof equals the single-device proof byte for byte.
* bench.py --gpus N on a box with fewer devices fails loudly (non-zero exit).
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R, S = 27134, 17146


def _bh():
    import bellman_hip as bh
    return bh


def test_rccl_single_rank_communicator(ctx):
    bh = _bh()
    comm = bh.Comm(ctx, bh.Comm.unique_id(), 1, 0)
    try:
        assert comm.info() == (1, 0, 0)
        assert comm.allreduce_max(3.25) == 3.25
        assert comm.allgather_bytes(b"abcdefgh") == [b"abcdefgh"]
        params = bh.Parameters.chain(ctx, 15)
        w = bh.Witness.chain(ctx, 15)
        single = bh.prove_witness(ctx, params, w, R, S)
        part = comm.prove_partial(ctx, params, w)
        assert part == bh.prove_witness_partial(ctx, params, w, 0, 1)
        parts = comm.allgather(part)
        assert bh.proof_from_partials(params.vk_bytes(), parts, 1, R, S) == single
    finally:
        comm.close()


@pytest.mark.parametrize("logc,nranks", [(12, 2), (14, 4), (18, 4), (18, 8)])
def test_ranks_with_shard_tables_equal_single_proof(ctx, logc, nranks):
    """Each rank: own context, own Parameters prepared with bh_params_prepare_shard (slices of
    l/a/b_g1/b_g2 and, for N >= 4, the gathered h share), then all ranks run concurrently
    with device-copy all-to-alls.  At 2^18 / 4 ranks every shard is large enough for tables."""
    bh = _bh()
    rounds = (1 << (logc - 1)) - 1
    params = bh.Parameters.chain(ctx, rounds)
    w = bh.Witness.chain(ctx, rounds)
    single = bh.prove_witness(ctx, params, w, R, S)
    ctxs = [bh.Context(0) for _ in range(nranks)]
    try:
        ps = [bh.Parameters.chain(c, rounds) for c in ctxs]
        for k, p in enumerate(ps):
            p.prepare_shard(w, k, nranks, distributed_h=True)
        parts = bh.prove_witness_partials_ranks(ctxs, ps, w)
        assert bh.proof_from_partials(params.vk_bytes(), parts, nranks, R, S) == single
        st = ctxs[0].last_stats()
        if (1 << logc) // nranks >= 1 << 16:  # shards this large use window tables
            assert st[10] == st[11] > 0  # every large multiexp of rank 0 used its table slice
            assert st[12] > 0
        # and once more (tables resident, nothing rebuilt)
        assert bh.prove_witness_partials_ranks(ctxs, ps, w) == parts
    finally:
        for c in ctxs:
            c.close()


def test_shard_tables_are_a_slice(ctx):
    """A rank's tables hold ~1/N of the single-GPU table bytes (capacity 1/N)."""
    bh = _bh()
    rounds = (1 << 18) - 1
    w = bh.Witness.chain(ctx, rounds)
    full = bh.Parameters.chain(ctx, rounds)
    full.prepare(w, 4)
    bh.prove_witness_partial(ctx, full, w, 1, 4)
    full_bytes = ctx.last_stats()[12]
    shard = bh.Parameters.chain(ctx, rounds)
    shard.prepare_shard(w, 1, 4, distributed_h=False)
    bh.prove_witness_partial(ctx, shard, w, 1, 4)
    st = ctx.last_stats()
    assert st[10] == st[11] > 0
    assert 0 < st[12] < 0.3 * full_bytes


def test_bench_gpus_more_than_devices_fails_loudly():
    bh = _bh()
    n = bh.device_count() + 1
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--log-constraints", "10",
                        "--steps", "1", "--warmup", "0"], capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "devices" in p.stderr


def _gloo_rank(rank, world, port, rounds, q):
    sys.path.insert(0, os.path.join(ROOT, "bellman-mpc_amd"))
    import torch
    import torch.distributed as dist
    import bellman_hip as bh
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ctx = bh.Context(0)
    try:
        params = bh.Parameters.chain(ctx, rounds)
        w = bh.Witness.chain(ctx, rounds)
        rec = bh.prove_witness_partial(ctx, params, w, rank, world)
        t = torch.frombuffer(bytearray(rec), dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(out, t)
        if rank == 0:
            parts = b"".join(x.numpy().tobytes() for x in out)
            proof = bh.proof_from_partials(params.vk_bytes(), parts, world, R, S)
            q.put(proof == bh.prove_witness(ctx, params, w, R, S))
        dist.barrier()
    finally:
        ctx.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("world,logc", [(2, 12), (3, 16)])
def test_rank_processes_exchange_partials_over_gloo(world, logc):
    """The product's per-rank path in separate processes (one context each, as bench.py's
    ranks run), partial records exchanged by a real collective (gloo all-gather, standing in
    for the ncclAllGather of bh_prove_witness_partial_comm), recombined by rank 0: equal to the
    single-device proof.  Ranks share cuda:0 here; 2-3 processes on the card."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mctx = mp.get_context("spawn")
    q = mctx.Queue()
    procs = [mctx.Process(target=_gloo_rank, args=(r, world, port, (1 << (logc - 1)) - 1, q))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        ok = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert ok
    assert all(p.exitcode == 0 for p in procs)
