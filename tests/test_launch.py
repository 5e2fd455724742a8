"""CPU tests of the multi-GPU launcher (bellman-mpc_amd/bh_launch.py) that
`bench.py --gpus N` uses: rank environment rules, the parent spawning one
process per rank with LOCAL_RANK = device, the out-of-band rendezvous of the
RCCL unique id, and failure propagation.  No GPU and no HIP library involved."""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bellman-mpc_amd"))
import bh_launch  # noqa: E402


def test_rank_env_plain_run():
    assert bh_launch.rank_env(1, {}) == (1, 0, 0, False)
    assert bh_launch.rank_env(8, {}) == (8, 0, 0, True)  # the parent must spawn


def test_rank_env_under_launcher():
    env = {"WORLD_SIZE": "4", "RANK": "2", "LOCAL_RANK": "2"}
    assert bh_launch.rank_env(4, env) == (4, 2, 2, False)
    with pytest.raises(bh_launch.LaunchError):
        bh_launch.rank_env(8, env)  # launcher and --gpus disagree: never a silent other run
    with pytest.raises(bh_launch.LaunchError):
        bh_launch.rank_env(4, {"WORLD_SIZE": "4", "RANK": "4", "LOCAL_RANK": "0"})
    with pytest.raises(bh_launch.LaunchError):
        bh_launch.rank_env(0, {})


def test_rendezvous_dir_keys():
    a = bh_launch.rendezvous_dir({"MASTER_PORT": "29500", "TMPDIR": "/tmp"})
    b = bh_launch.rendezvous_dir({"MASTER_PORT": "29501", "TMPDIR": "/tmp"})
    assert a != b and str(os.getppid()) in a
    assert bh_launch.rendezvous_dir({"BH_RDZV_DIR": "/x/y"}) == "/x/y"


def test_publish_wait_roundtrip(tmp_path):
    d = str(tmp_path / "rdzv")
    bh_launch.publish(d, "uid", b"\x01" * 128)
    assert bh_launch.wait_for(d, "uid", timeout=1) == b"\x01" * 128
    bh_launch.cleanup(d)
    assert not os.path.exists(d)
    with pytest.raises(bh_launch.LaunchError):
        bh_launch.wait_for(d, "uid", timeout=0.2)


_CHILD = textwrap.dedent("""
    import json, os, sys
    sys.path.insert(0, {pkg!r})
    import bh_launch
    world, rank, local, spawn = bh_launch.rank_env(int(sys.argv[1]))
    assert not spawn
    d = bh_launch.rendezvous_dir()
    if rank == 0:
        bh_launch.publish(d, "uid", b"uid-%d" % os.getpid())
        uid = bh_launch.wait_for(d, "uid")
    else:
        uid = bh_launch.wait_for(d, "uid", timeout=30)
    with open(os.path.join({out!r}, "rank%d.json" % rank), "w") as f:
        json.dump({{"world": world, "rank": rank, "local": local, "uid": uid.decode(), "dir": d}}, f)
    sys.exit(int(os.environ.get("FAIL_RANK", "-1")) == rank and 7 or 0)
""")


def _child(tmp_path):
    script = tmp_path / "child.py"
    script.write_text(_CHILD.format(pkg=os.path.join(ROOT, "bellman-mpc_amd"), out=str(tmp_path)))
    return str(script)


def test_spawn_ranks_one_process_per_device(tmp_path):
    import json
    rc = bh_launch.spawn_ranks(4, [_child(tmp_path), "4"], environ=dict(os.environ, TMPDIR=str(tmp_path)))
    assert rc == 0
    recs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(4)]
    assert [r["rank"] for r in recs] == [0, 1, 2, 3]
    assert [r["local"] for r in recs] == [0, 1, 2, 3]  # LOCAL_RANK = device, each rank its own
    assert all(r["world"] == 4 for r in recs)
    assert len({r["uid"] for r in recs}) == 1  # every rank read rank 0's id
    assert not os.path.exists(recs[0]["dir"])  # rendezvous directory removed


def test_spawn_ranks_propagates_failure(tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path), FAIL_RANK="1")
    assert bh_launch.spawn_ranks(2, [_child(tmp_path), "2"], environ=env) == 7


def test_bench_rejects_mismatched_launcher():
    """bench.py under a launcher whose WORLD_SIZE differs from --gpus exits non-zero before
    loading the HIP library."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2 and "WORLD_SIZE=2" in p.stderr
