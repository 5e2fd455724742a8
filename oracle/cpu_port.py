"""ORACLE / CPU BASELINE wrapper (test + bench infrastructure only).

ctypes binding of oracle/cpu/libbellman_port.so, the C++ restatement of
bellman's multicore prover core (see oracle/cpu/bellman_port.cpp header).
Used by tests/ (as a checker) and by bench.py's cpu_baseline leg."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "cpu", "libbellman_port.so")


def build():
    subprocess.run(["make", "-s", "-C", os.path.join(HERE, "cpu")], check=True)


def _lib():
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    P, S, U64, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int
    lib.bp_chain_prove.restype = I
    lib.bp_chain_prove.argtypes = [P, S, S, U64, I, I, P, P, P, P, P]
    lib.bp_hardware_threads.restype = I
    lib.bp_multiexp_g1.restype = I
    lib.bp_multiexp_g1.argtypes = [P, S, P, S, I, P, P]
    lib.bp_multiexp.restype = I
    lib.bp_multiexp.argtypes = [I, P, S, S, P, P, S, I, P, P]
    return lib


def hardware_threads():
    return _lib().bp_hardware_threads()


def chain_prove(params_bytes, rounds, seed=7, threads=0, reps=1, r=27134, s=17146):
    """Synthesize the MiMC chain and run the bellman-algorithm prover core.
    Returns (proof bytes, median core ms, synthesis ms)."""
    lib = _lib()
    buf = np.frombuffer(params_bytes, dtype=np.uint8)
    rr = np.array([r, 0, 0, 0], dtype=np.uint64)
    ss = np.array([s, 0, 0, 0], dtype=np.uint64)
    out = np.zeros(192, dtype=np.uint8)
    ms = ctypes.c_double()
    ms_syn = ctypes.c_double()
    st = lib.bp_chain_prove(buf.ctypes.data_as(ctypes.c_void_p), len(params_bytes), rounds, seed, threads, reps,
                            rr.ctypes.data_as(ctypes.c_void_p), ss.ctypes.data_as(ctypes.c_void_p),
                            out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ms), ctypes.byref(ms_syn))
    if st != 0:
        raise RuntimeError(f"bellman port failed with status {st}")
    return out.tobytes(), ms.value, ms_syn.value


def multiexp_g1(bases_uncompressed, exps_limbs, threads=0):
    """bellman's multiexp (FullDensity) on the host cores: bases = concatenated 96-byte
    uncompressed encodings, exps = (n,4) uint64 canonical limbs.  Returns (bytes, ms)."""
    lib = _lib()
    b = np.frombuffer(bases_uncompressed, dtype=np.uint8)
    e = np.ascontiguousarray(exps_limbs, dtype=np.uint64).reshape(-1, 4)
    out = np.zeros(96, dtype=np.uint8)
    ms = ctypes.c_double()
    st = lib.bp_multiexp_g1(b.ctypes.data_as(ctypes.c_void_p), len(bases_uncompressed) // 96,
                            e.ctypes.data_as(ctypes.c_void_p), e.shape[0], threads,
                            out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ms))
    if st:
        raise RuntimeError(f"bp_multiexp_g1 failed: {st}")
    return out.tobytes(), ms.value


def multiexp(group, bases_uncompressed, exps_limbs, base_offset=0, density_words=None, threads=0):
    """bellman's multiexp over G1 (group 1) or G2 (group 2) with a base offset and an optional
    density bitvec (uint64 words): (uncompressed bytes, ms)."""
    lib = _lib()
    pb = 96 if group == 1 else 192
    b = np.frombuffer(bases_uncompressed, dtype=np.uint8)
    e = np.ascontiguousarray(exps_limbs, dtype=np.uint64).reshape(-1, 4)
    d = None if density_words is None else np.ascontiguousarray(density_words, dtype=np.uint64)
    out = np.zeros(pb, dtype=np.uint8)
    ms = ctypes.c_double()
    st = lib.bp_multiexp(group, b.ctypes.data_as(ctypes.c_void_p), len(bases_uncompressed) // pb, base_offset,
                         None if d is None else d.ctypes.data_as(ctypes.c_void_p),
                         e.ctypes.data_as(ctypes.c_void_p), e.shape[0], threads,
                         out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(ms))
    if st:
        raise RuntimeError(f"bp_multiexp failed: {st}")
    return out.tobytes(), ms.value
