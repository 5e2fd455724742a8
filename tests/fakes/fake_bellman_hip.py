"""CPU stand-in for `bellman_hip`, used ONLY by tests/test_bench_ranks_cpu.py.

It lets bench.py's multi-rank orchestration run on CPU: launcher environment, the
rendezvous of the RCCL unique id, the per-rank records (devices, ms, window-table use),
max-over-ranks timing, partial exchange and rank 0's combine, and the C5 split.  Proofs
are deterministic hashes and the "communicator" is a directory of files; nothing here
computes anything of the product, and no product code imports it.
"""
import hashlib
import os
import time

BH_G1, BH_G2 = 0, 1
PARTIAL_BYTES = 960


def device_count():
    return int(os.environ.get("FAKE_DEVICES", "8"))


def _h(*parts, n=192):
    out, i = b"", 0
    while len(out) < n:
        out += hashlib.sha256(repr((i,) + parts).encode()).digest()
        i += 1
    return out[:n]


class Context:
    def __init__(self, device=0):
        self.device = device
        self.tables = True
        self._stats = [0.0] * 13

    def synchronize(self):
        pass

    def set_tables(self, on):
        self.tables = bool(on)

    def last_timings(self):
        return self._stats[:10]

    def last_stats(self):
        return list(self._stats)

    def _proved(self, n, table_bytes=0.0):
        time.sleep(0.001)
        self._stats = [1.0, 0.5, 0.8, 6, 6.0 * n, 0.2, 2, 1.0 * n, 13.0 * n, 2.0 * n,
                       5 if self.tables else 0, 5, table_bytes if self.tables else 0.0]

    def scratch_report(self):
        """bh_scratch_report's keys (bellman_hip.Context.scratch_report) with a fitting budget."""
        return {"limit_max": 1 << 33, "limit_current": 0, "worst_bytes_per_lane": 0, "worst_per_queue": 0,
                "queues": 7, "total_need": 0, "fits": True, "kernels_checked": 0, "worst_per_queue_resident": 0,
                "live_contexts": 1, "worst_kernel": ""}

    def close(self):
        pass


FULL_TABLE_BYTES = 31.4e9  # the 2^22 proof's window tables on one device


class Parameters:
    """Records which window tables were prepared (`prepared`): ("full", nshards) for
    bh_params_prepare, ("shard", shard, nshards, distributed_h) for bh_params_prepare_shard."""

    def __init__(self, ctx, rounds):
        self.ctx, self.rounds, self.prepared = ctx, rounds, None

    @classmethod
    def chain(cls, ctx, rounds):
        return cls(ctx, rounds)

    def prepare(self, witness, nshards=1):
        self.prepared = ("full", nshards)

    def prepare_shard(self, witness, shard, nshards, distributed_h=True):
        self.prepared = ("shard", shard, nshards, bool(distributed_h))

    def table_bytes(self):
        if not self.prepared:
            return 0.0
        return FULL_TABLE_BYTES / self.prepared[2] if self.prepared[0] == "shard" else FULL_TABLE_BYTES

    def vk_bytes(self):
        return _h("vk", self.rounds, n=96 * 3 + 192 * 3 + 4 + 96 * 2)


class Witness:
    def __init__(self, ctx, rounds, seed, preimage_seed):
        self.ctx, self.rounds, self.seed, self.preimage_seed = ctx, rounds, seed, preimage_seed

    @classmethod
    def chain(cls, ctx, rounds, seed=7, preimage_seed=None):
        return cls(ctx, rounds, seed, preimage_seed)


def prove_witness(ctx, params, w, r, s):
    ctx._proved(2 * params.rounds + 2, params.table_bytes())
    return _h("proof", params.rounds, w.seed, w.preimage_seed, r, s)


def prove_batch(ctx, params, ws, r, s, lanes=0):
    return [prove_witness(ctx, params, w, r, s) for w in ws]


def proof_from_partials(vk, parts, nshards, r, s):
    assert len(parts) == PARTIAL_BYTES * nshards, "one 960-byte record per rank"
    return _h("combined", vk, parts, r, s)


class Comm:
    """file-backed all-gather among the FAKE_COMM_DIR ranks (stands in for RCCL)"""

    @staticmethod
    def unique_id():
        return os.urandom(128)

    def __init__(self, ctx, uid, nranks, rank):
        assert len(uid) == 128
        self.ctx, self.nranks, self.rank, self.gen = ctx, nranks, rank, 0
        self.dir = os.environ["FAKE_COMM_DIR"]
        self._gather(uid)  # like ncclCommInitRank: returns once every rank has joined

    def _gather(self, payload):
        self.gen += 1
        tmp = os.path.join(self.dir, f".{self.gen}_{self.rank}")
        with open(tmp, "wb") as f:
            f.write(payload)
        os.replace(tmp, os.path.join(self.dir, f"{self.gen}_{self.rank}"))
        out, t_end = [], time.monotonic() + 60
        for k in range(self.nranks):
            path = os.path.join(self.dir, f"{self.gen}_{k}")
            while not os.path.exists(path):
                assert time.monotonic() < t_end, f"rank {k} never arrived at gather {self.gen}"
                time.sleep(0.005)
            with open(path, "rb") as f:
                out.append(f.read())
        return out

    def info(self):
        return (self.nranks, self.rank, self.ctx.device)

    def prove_partial(self, ctx, params, witness):
        # a rank proves with exactly the per-rank tables the one-GPU rehearsal times
        # (tools/shard_rehearsal.py: prepare_shard(w, rank, N, distributed_h=True)), never the
        # full-vector tables of bh_params_prepare
        want = ("shard", self.rank, self.nranks, True)
        assert params.prepared == want, f"rank {self.rank} prepared {params.prepared}, expected {want}"
        ctx._proved((2 * params.rounds + 2) // self.nranks, params.table_bytes())
        return _h("partial", params.rounds, self.rank, n=PARTIAL_BYTES)

    def allgather(self, partial):
        assert len(partial) == PARTIAL_BYTES
        return b"".join(self._gather(partial))

    def allgather_bytes(self, rec):
        recs = self._gather(rec)
        assert len({len(x) for x in recs}) == 1, "RCCL all-gather needs equal-size records"
        return recs

    def allreduce_max(self, x):
        return max(float(v.decode()) for v in self._gather(repr(float(x)).encode()))

    def close(self):
        pass
