"""bench.py's multi-rank orchestration on CPU (the path the driver's 8-GPU run takes).

Each rank is a fresh interpreter with the launcher's variables (WORLD_SIZE / RANK /
LOCAL_RANK, as torch.distributed.run sets them) running bench.py with `bellman_hip`
replaced by tests/fakes/fake_bellman_hip.py (hash "proofs", a file-backed all-gather).
Checked: the rendezvous of the unique id, RCCL's reported ranks and devices, the per-rank
records in the BENCH line, the max-over-ranks timing, the C5 split, and that only rank 0
prints.  The device work itself is covered by the -m gpu tests."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNNER = (
    "import sys, runpy; sys.path.insert(0, {fakes!r}); import fake_bellman_hip as f; "
    "sys.modules['bellman_hip'] = f; sys.argv = ['bench.py'] + sys.argv[1:]; "
    "runpy.run_path({bench!r}, run_name='__main__')"
)


@pytest.mark.parametrize("world", [2, 4])
def test_bench_multirank_line(tmp_path, world):
    code = RUNNER.format(fakes=os.path.join(ROOT, "tests", "fakes"), bench=os.path.join(ROOT, "bench.py"))
    args = ["--gpus", str(world), "--log-constraints", "6", "--steps", "3", "--warmup", "1",
            "--cpu-baseline", "0", "--dropin", "0", "--c5", "8", "--c5-log-constraints", "4"]
    comm = tmp_path / "comm"
    comm.mkdir()
    procs = []
    for rank in range(world):
        env = dict(os.environ, WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank),
                   BH_RDZV_DIR=str(tmp_path / "rdzv"), FAKE_COMM_DIR=str(comm), FAKE_DEVICES=str(world))
        procs.append(subprocess.Popen([sys.executable, "-c", code] + args, env=env, cwd=ROOT,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    try:
        outs = [p.communicate(timeout=60) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e
    lines = [l for l in outs[0][0].splitlines() if l.startswith("{")]
    assert len(lines) == 1
    for o, _ in outs[1:]:
        assert not [l for l in o.splitlines() if l.startswith("{")]  # only rank 0 prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["steps"] == 3 and d["warmup"] == 1
    assert d["rccl"] == {"ranks": world, "devices": list(range(world))}
    assert len(d["per_rank_ms_per_step"]) == world
    assert d["ms_per_step"] >= max(d["per_rank_ms_per_step"]) * 0.999  # max over ranks
    assert d["srs_window_tables"]["used"] == [5] * world
    # every rank built only its own table slices (bh_params_prepare_shard), as rehearsed
    assert d["srs_window_tables"]["prepare"] == ["shard"] * world
    assert all(abs(gb - 31.4 / world) < 0.01 for gb in d["srs_window_tables"]["GB"])
    assert d["config"]["parallelism"] == f"msm-shard{world}" and d["config"]["exchange"] == "rccl"
    assert d["c5"]["proofs"] == 8 and d["c5"]["proofs_match_single"] is True
    assert d["value"] > 0 and d["proof_sha_prefix"]


def test_bench_single_gpu_prepares_full_tables(tmp_path):
    """N = 1: the full-vector tables (bh_params_prepare), reported as such."""
    code = RUNNER.format(fakes=os.path.join(ROOT, "tests", "fakes"), bench=os.path.join(ROOT, "bench.py"))
    env = dict(os.environ, FAKE_COMM_DIR=str(tmp_path), FAKE_DEVICES="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "-c", code, "--log-constraints", "6", "--steps", "2", "--warmup", "1",
                        "--cpu-baseline", "0", "--dropin", "0", "--c5", "0"], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    d = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][0])
    assert d["n_gpus"] == 1 and d["srs_window_tables"]["prepare"] == "full"
    assert abs(d["srs_window_tables"]["GB"] - 31.4) < 0.01


def test_bench_rank_fails_on_missing_devices(tmp_path):
    """A rank whose node shows fewer devices than --gpus exits non-zero (no silent 1-GPU run)."""
    code = RUNNER.format(fakes=os.path.join(ROOT, "tests", "fakes"), bench=os.path.join(ROOT, "bench.py"))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", BH_RDZV_DIR=str(tmp_path),
               FAKE_COMM_DIR=str(tmp_path), FAKE_DEVICES="1")
    p = subprocess.run([sys.executable, "-c", code, "--gpus", "2", "--log-constraints", "6"], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 3 and "needs 2 devices" in p.stderr
