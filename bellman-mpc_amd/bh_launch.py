"""One process per GPU for the multi-GPU prover, without torch.

`bench.py --gpus N` either runs under a launcher that already set RANK /
LOCAL_RANK / WORLD_SIZE (``python -m torch.distributed.run --nproc-per-node N``)
or, started as a plain ``python bench.py --gpus N``, starts the N rank processes
itself with this module before anything in the parent touches HIP.  The ranks
exchange nothing but the 128-byte RCCL unique id out of band (a file written by
rank 0 in a directory every rank derives from its common parent process); all
device traffic, the timing barrier and the max-over-ranks reduction then go
over RCCL inside libbellman_hip.so.  torch is deliberately not imported: it
bundles its own HIP runtime and RCCL, and one process must not load two.

This module imports nothing that loads the HIP library, so the launcher parent
stays free of GPU state (a process that has initialised the GPU must not start
rank processes by exec, and must not hold the device while they run).
"""
import os
import subprocess
import sys
import time

RANK_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE")


class LaunchError(RuntimeError):
    pass


def rank_env(gpus, environ=None):
    """(world, rank, local_rank, spawn) for `--gpus gpus` in this environment.

    spawn is True when this process must start the ranks itself (no launcher
    variables and gpus > 1).  A launcher whose WORLD_SIZE differs from --gpus is
    an error, never silently a different run."""
    env = os.environ if environ is None else environ
    if gpus < 1:
        raise LaunchError(f"--gpus must be >= 1 (got {gpus})")
    if "WORLD_SIZE" not in env:
        return gpus, 0, 0, gpus > 1
    world = int(env["WORLD_SIZE"])
    rank = int(env.get("RANK", "0"))
    local = int(env.get("LOCAL_RANK", str(rank)))
    if world != gpus:
        raise LaunchError(f"WORLD_SIZE={world} from the launcher but --gpus {gpus}")
    if not 0 <= rank < world or not 0 <= local < world:
        raise LaunchError(f"RANK={rank} LOCAL_RANK={local} outside WORLD_SIZE={world}")
    return world, rank, local, False


def rendezvous_dir(environ=None):
    """Directory shared by the ranks of ONE run: keyed by the common parent process
    (the torchrun agent, or spawn_ranks' parent) and the run id / master port, so
    back-to-back runs never read each other's id."""
    env = os.environ if environ is None else environ
    if env.get("BH_RDZV_DIR"):
        return env["BH_RDZV_DIR"]
    key = "_".join([str(os.getppid()), env.get("TORCHELASTIC_RUN_ID", "none"), env.get("MASTER_PORT", "0")])
    return os.path.join(env.get("TMPDIR", "/tmp"), f"bh_rdzv_{key}")


def publish(directory, name, payload: bytes):
    """Atomically write `payload` as directory/name (rank 0)."""
    os.makedirs(directory, exist_ok=True)
    tmp = os.path.join(directory, f".{name}.{os.getpid()}")
    with open(tmp, "wb") as f:
        f.write(payload)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, os.path.join(directory, name))


def wait_for(directory, name, timeout=120.0, poll=0.02):
    """Block until directory/name exists (written by publish) and return its bytes."""
    path = os.path.join(directory, name)
    t_end = time.monotonic() + timeout
    while True:
        try:
            with open(path, "rb") as f:
                return f.read()
        except FileNotFoundError:
            if time.monotonic() > t_end:
                raise LaunchError(f"rendezvous: {path} did not appear within {timeout:.0f} s")
            time.sleep(poll)


def cleanup(directory):
    try:
        for f in os.listdir(directory):
            os.unlink(os.path.join(directory, f))
        os.rmdir(directory)
    except OSError:
        pass


def spawn_ranks(n, argv, environ=None, python=None, timeout=None):
    """Start n rank processes `python argv...` with RANK / LOCAL_RANK / WORLD_SIZE set
    (LOCAL_RANK = the device) and a fresh rendezvous directory; wait for all of them.

    Returns the exit code to propagate: 0 if every rank succeeded, else the first
    non-zero one.  If one rank fails the others are terminated (a rank blocked in a
    collective would otherwise wait for its dead peer forever)."""
    env0 = dict(os.environ if environ is None else environ)
    rdzv = os.path.join(env0.get("TMPDIR", "/tmp"), f"bh_rdzv_{os.getpid()}_{int(time.time() * 1e6)}")
    cleanup(rdzv)
    procs = []
    for r in range(n):
        env = dict(env0)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), BH_RDZV_DIR=rdzv)
        env.setdefault("MASTER_ADDR", "127.0.0.1")
        procs.append(subprocess.Popen([python or sys.executable] + list(argv), env=env))
    t_end = None if timeout is None else time.monotonic() + timeout
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in live:
                        q.terminate()
            if t_end is not None and time.monotonic() > t_end and live:
                for q in live:
                    q.kill()
                rc = rc or 124
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        cleanup(rdzv)
    return rc
