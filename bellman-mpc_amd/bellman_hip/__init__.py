"""bellman_hip -- Python host layer over the MI355X Groth16 prover core.

Mirrors the reference crate's API for the hot path (paths relative to
/root/reference/bellman/src):

  multiexp(ctx, bases, offset, density, exponents)   multiexp.rs:252-281
  EvaluationDomain.{fft, ifft, coset_fft, ...}        domain.rs:42-190
  Parameters.read / .write                            groth16/mod.rs:260-400
  ProvingAssignment / create_proof / create_random_proof
                                                       groth16/prover.rs:19-350
  Circuit / ConstraintSystem / LinearCombination      lib.rs:203-623

All arithmetic runs in libbellman_hip.so (HIP kernels for gfx950) through the
C ABI declared in include/bellman_hip.h; this module only marshals.  If the
shared library is missing this module raises at import time -- there is no
CPU fallback.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.environ.get("BH_LIB_OVERRIDE") or os.path.join(_HERE, "libbellman_hip.so")  # override: A/B builds

R_MODULUS = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
_MONT_R = pow(2, 256, R_MODULUS)
_MONT_RINV = pow(_MONT_R, -1, R_MODULUS)

BH_OK = 0
BH_ERR_INVALID_ARGUMENT = 10
BH_G1, BH_G2 = 1, 2
BH_SCALARS_CANONICAL, BH_SCALARS_MONTGOMERY = 0, 1


class SynthesisError(Exception):
    """Mirrors lib.rs:355-364; .code is the bh_status."""

    def __init__(self, code, msg=""):
        super().__init__(f"{msg} (status {code}: {_status_string(code)})")
        self.code = code


class UnexpectedIdentity(SynthesisError):
    pass


class UnexpectedEof(SynthesisError):
    pass


class PolynomialDegreeTooLarge(SynthesisError):
    pass


class DensitySizeMismatch(SynthesisError):
    pass


class AssignmentMissing(SynthesisError):
    def __init__(self):
        super().__init__(6, "assignment missing")


_ERRS = {1: UnexpectedIdentity, 2: UnexpectedEof, 3: PolynomialDegreeTooLarge, 4: DensitySizeMismatch}


def _load():
    if not os.path.exists(_LIB_PATH):
        raise ImportError(f"bellman_hip: {_LIB_PATH} not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_LIB_PATH)
    P, S, U64, I, U8 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32
    sig = {
        "bh_status_string": (ctypes.c_char_p, [I]),
        "bh_version": (I, []),
        "bh_verify_proof": (I, [P, S, P, P, S, P]),
        "bh_verify_batch": (I, [P, S, P, P, S, S, P, P]),
        "bh_ctx_create": (I, [I, P]),
        "bh_ctx_destroy": (I, [P]),
        "bh_ctx_reserve": (I, [P, S, U8]),
        "bh_ctx_set_window": (I, [P, I]),
        "bh_srs_upload": (I, [P, I, P, S, I, P]),
        "bh_srs_free": (I, [P]),
        "bh_srs_len": (S, [P]),
        "bh_srs_get": (I, [P, S, P]),
        "bh_multiexp": (I, [P, P, S, P, S, P, S, I, P]),
        "bh_domain_size": (I, [S, P, P]),
        "bh_fft": (I, [P, P, U8]),
        "bh_ifft": (I, [P, P, U8]),
        "bh_coset_fft": (I, [P, P, U8]),
        "bh_icoset_fft": (I, [P, P, U8]),
        "bh_distribute_powers": (I, [P, P, S, P]),
        "bh_divide_by_z_on_coset": (I, [P, P, U8]),
        "bh_mul_assign": (I, [P, P, P, S]),
        "bh_sub_assign": (I, [P, P, P, S]),
        "bh_compute_h": (I, [P, P, P, P, S, P, P]),
        "bh_params_load": (I, [P, P, S, I, P]),
        "bh_params_free": (I, [P]),
        "bh_params_sizes": (I, [P, P]),
        "bh_params_write": (I, [P, P, S, P]),
        "bh_prove": (I, [P, P, P, P, P, S, P, S, P, S, P, P, P, P, P, P]),
        "bh_witness_upload": (I, [P, P, P, P, S, P, S, P, S, P, P, P, P]),
        "bh_witness_free": (I, [P]),
        "bh_prove_witness": (I, [P, P, P, P, P, P]),
        "bh_chain_witness": (I, [P, S, U64, P]),
        "bh_chain_params": (I, [P, S, U64, U64, U64, U64, U64, U64, P]),
        "bh_last_timings": (I, [P, P]),
        "bh_shard_range": (I, [S, S, S, P, P]),
        "bh_prove_witness_partial": (I, [P, P, P, S, S, P]),
        "bh_vk_write": (I, [P, P, S, P]),
        "bh_proof_from_partials": (I, [P, S, P, S, P, P, P]),
        "bh_comm_unique_id": (I, [P]),
        "bh_comm_init": (I, [P, P, I, I, P]),
        "bh_comm_allgather_partials": (I, [P, P, P]),
        "bh_comm_destroy": (I, [P]),
        "bh_ctx_synchronize": (I, [P]),
        "bh_device_count": (I, []),
        "bh_ctx_set_tables": (I, [P, I]),
        "bh_params_prepare": (I, [P, P, P, S]),
        "bh_chain_witness_preimage": (I, [P, S, U64, U64, P]),
        "bh_prove_witness_partial_comm": (I, [P, P, P, P, P]),
        "bh_prove_witness_partials_local": (I, [P, P, P, S, P]),
        "bh_comm_allgather": (I, [P, P, S, P]),
        "bh_params_prepare_shard": (I, [P, P, P, S, S, I]),
        "bh_last_stats": (I, [P, P, S]),
        "bh_prove_witness_partials_ranks": (I, [P, P, P, S, P]),
        "bh_chain_sizes": (I, [S, P]),
        "bh_rehearse_rank": (I, [P, P, P, S, S, P]),
        "bh_multiexp_submit": (I, [P, P, S, P, S, P, S, I, P]),
        "bh_multiexp_wait": (I, [P, P]),
        "bh_prove_batch": (I, [P, P, P, S, P, P, I, P]),
        "bh_chain_assignment": (I, [S, U64, U64, P, P, P, P, P, P, P, P]),
        "bh_comm_allreduce_max": (I, [P, P]),
        "bh_comm_info": (I, [P, P]),
        "bh_params_vector": (I, [P, I, P]),
        "bh_scalars_upload": (I, [P, P, S, I, P]),
        "bh_compute_h_scalars": (I, [P, P, P, P, S, P]),
        "bh_scalars_len": (S, [P]),
        "bh_scalars_free": (I, [P]),
        "bh_multiexp_submit_scalars": (I, [P, P, S, P, S, P, P]),
        "bh_scalars_sync": (I, [P]),
        "bh_scalars_stamps": (I, [P, P]),
        "bh_scratch_report": (I, [P, P, S, ctypes.c_char_p, S]),
        "bh_evdom_from_coeffs": (I, [P, P, S, P]),
        "bh_evdom_size": (I, [P, P, P]),
        "bh_evdom_fft": (I, [P]),
        "bh_evdom_ifft": (I, [P]),
        "bh_evdom_coset_fft": (I, [P]),
        "bh_evdom_icoset_fft": (I, [P]),
        "bh_evdom_distribute_powers": (I, [P, P]),
        "bh_evdom_divide_by_z_on_coset": (I, [P]),
        "bh_evdom_mul_assign": (I, [P, P]),
        "bh_evdom_sub_assign": (I, [P, P]),
        "bh_evdom_read": (I, [P, P, S]),
        "bh_evdom_write": (I, [P, P, S]),
        "bh_evdom_into_scalars": (I, [P, S, P]),
        "bh_evdom_sync": (I, [P]),
        "bh_evdom_free": (I, [P]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


_lib = _load()

# every symbol declared in include/bellman_hip.h
EXPORTED_SYMBOLS = [
    "bh_status_string", "bh_version", "bh_ctx_create", "bh_ctx_destroy", "bh_ctx_reserve", "bh_ctx_set_window",
    "bh_srs_upload", "bh_srs_free", "bh_srs_len", "bh_srs_get", "bh_multiexp", "bh_domain_size", "bh_fft",
    "bh_ifft", "bh_coset_fft", "bh_icoset_fft", "bh_distribute_powers", "bh_divide_by_z_on_coset",
    "bh_mul_assign", "bh_sub_assign", "bh_compute_h", "bh_params_load", "bh_params_free", "bh_params_sizes",
    "bh_prove", "bh_witness_upload", "bh_witness_free", "bh_prove_witness", "bh_chain_witness",
    "bh_chain_params", "bh_params_write", "bh_last_timings", "bh_shard_range", "bh_prove_witness_partial",
    "bh_vk_write", "bh_proof_from_partials", "bh_comm_unique_id", "bh_comm_init", "bh_comm_allgather_partials",
    "bh_comm_destroy", "bh_ctx_synchronize", "bh_device_count", "bh_ctx_set_tables", "bh_params_prepare",
    "bh_chain_witness_preimage", "bh_prove_witness_partial_comm", "bh_prove_witness_partials_local",
    "bh_comm_allgather", "bh_comm_allreduce_max", "bh_comm_info", "bh_params_prepare_shard", "bh_last_stats",
    "bh_prove_witness_partials_ranks", "bh_chain_sizes", "bh_chain_assignment", "bh_rehearse_rank",
    "bh_multiexp_submit", "bh_multiexp_wait", "bh_prove_batch", "bh_verify_proof", "bh_verify_batch",
    "bh_params_vector", "bh_scalars_upload", "bh_compute_h_scalars", "bh_scalars_len", "bh_scalars_free",
    "bh_multiexp_submit_scalars", "bh_scalars_sync", "bh_scratch_report", "bh_scalars_stamps",
    "bh_evdom_from_coeffs", "bh_evdom_size", "bh_evdom_fft", "bh_evdom_ifft", "bh_evdom_coset_fft",
    "bh_evdom_icoset_fft", "bh_evdom_distribute_powers", "bh_evdom_divide_by_z_on_coset", "bh_evdom_mul_assign",
    "bh_evdom_sub_assign", "bh_evdom_read", "bh_evdom_write", "bh_evdom_into_scalars", "bh_evdom_sync",
    "bh_evdom_free",
]
BH_VEC_H, BH_VEC_L, BH_VEC_A, BH_VEC_B_G1, BH_VEC_B_G2 = range(5)
PARTIAL_BYTES = 960


def lib():
    return _lib


def _status_string(code):
    s = _lib.bh_status_string(int(code))
    return s.decode() if s else "?"


def _check(code, what=""):
    if code != BH_OK:
        raise _ERRS.get(code, SynthesisError)(code, what)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


# ------------------------------------------------------------------ Fr encodings
def fr_to_mont(values):
    """ints -> (n,4) uint64 bls12_381 Montgomery limbs."""
    out = np.zeros((len(values), 4), dtype=np.uint64)
    for i, v in enumerate(values):
        x = (int(v) % R_MODULUS) * _MONT_R % R_MODULUS
        out[i] = [(x >> (64 * k)) & 0xFFFFFFFFFFFFFFFF for k in range(4)]
    return out


def fr_from_mont(arr):
    out = []
    for row in np.asarray(arr, dtype=np.uint64).reshape(-1, 4):
        x = sum(int(row[k]) << (64 * k) for k in range(4))
        out.append(x * _MONT_RINV % R_MODULUS)
    return out


def fr_to_canonical_limbs(values):
    """ints -> (n,4) uint64 canonical (Scalar::to_le_bits words)."""
    out = np.zeros((len(values), 4), dtype=np.uint64)
    for i, v in enumerate(values):
        x = int(v) % R_MODULUS
        out[i] = [(x >> (64 * k)) & 0xFFFFFFFFFFFFFFFF for k in range(4)]
    return out


class DensityWords:
    """A DensityTracker already in bitvec Lsb0 words (n bits), e.g. chain_assignment's maps."""

    def __init__(self, words, n):
        self.words, self.n = np.ascontiguousarray(words, dtype=np.uint64), int(n)

    def total(self):
        full, rem = self.n // 64, self.n % 64
        t = sum(bin(int(x)).count("1") for x in self.words[:full])
        if rem:
            t += bin(int(self.words[full]) & ((1 << rem) - 1)).count("1")
        return t


def _density(density):
    """-> (words or None, nbits)"""
    if density is None or isinstance(density, FullDensity) or density is FullDensity:
        return None, 0
    if isinstance(density, DensityWords):
        return density.words, density.n
    bits = density.bv if hasattr(density, "bv") else list(density)
    return density_words(bits), len(bits)


def density_words(bits):
    """list[bool] -> uint64 words (bitvec Lsb0)."""
    n = len(bits)
    w = np.zeros(max(1, (n + 63) // 64), dtype=np.uint64)
    for i, b in enumerate(bits):
        if b:
            w[i >> 6] |= np.uint64(1) << np.uint64(i & 63)
    return w


# ------------------------------------------------------------------ context / bases
class Context:
    """One MI355X device: streams + workspaces (replaces multicore::Worker)."""

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        _check(_lib.bh_ctx_create(device, ctypes.byref(h)), "bh_ctx_create")
        self.h = h

    def reserve(self, max_msm_len, max_log_domain=0):
        _check(_lib.bh_ctx_reserve(self.h, max_msm_len, max_log_domain), "bh_ctx_reserve")

    def set_window(self, c):
        _check(_lib.bh_ctx_set_window(self.h, c), "bh_ctx_set_window")

    def set_tables(self, enable):
        """Prover SRS window tables on/off (results never depend on it)."""
        _check(_lib.bh_ctx_set_tables(self.h, int(bool(enable))), "bh_ctx_set_tables")

    def synchronize(self):
        _check(_lib.bh_ctx_synchronize(self.h))

    def last_timings(self):
        """bh_last_timings: see include/bellman_hip.h for the 10 fields."""
        out = (ctypes.c_double * 10)()
        _check(_lib.bh_last_timings(self.h, out))
        return list(out)

    def last_stats(self):
        """bh_last_stats: the 10 timing fields, then tables used / large multiexps / table bytes, then
        (after prove() from host buffers) the upload landing times of aux, a, b, c and H's end, ms, then
        (after an EvaluationDomain transform) its upload / transform / download ms, then the wall time of
        the G1 and of the G2 accumulations (the union of their launches, which can overlap)."""
        out = (ctypes.c_double * 23)()
        _check(_lib.bh_last_stats(self.h, out, 23))
        return list(out)

    def scratch_report(self):
        """bh_scratch_report: the scratch budget of the library's kernels against the device limit."""
        out = (ctypes.c_uint64 * 10)()
        name = ctypes.create_string_buffer(64)
        _check(_lib.bh_scratch_report(self.h, out, 10, name, 64))
        keys = ["limit_max", "limit_current", "worst_bytes_per_lane", "worst_per_queue", "queues", "total_need",
                "fits", "kernels_checked", "worst_per_queue_resident", "live_contexts"]
        d = dict(zip(keys, list(out)))
        d["fits"] = bool(d["fits"])
        d["worst_kernel"] = name.value.decode()
        return d

    def close(self):
        if self.h:
            _lib.bh_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Bases:
    """Device-resident Arc<Vec<G1Affine|G2Affine>> (the multiexp SourceBuilder)."""

    def __init__(self, ctx, group, uncompressed: bytes, checked=True):
        pb = 96 if group == BH_G1 else 192
        assert len(uncompressed) % pb == 0
        n = len(uncompressed) // pb
        buf = np.frombuffer(uncompressed, dtype=np.uint8) if n else np.zeros(1, np.uint8)
        h = ctypes.c_void_p()
        _check(_lib.bh_srs_upload(ctx.h, group, _ptr(buf), n, int(checked), ctypes.byref(h)), "bh_srs_upload")
        self.h, self.group, self.ctx = h, group, ctx

    def __len__(self):
        return _lib.bh_srs_len(self.h)

    def get(self, i):
        out = np.zeros(96 if self.group == BH_G1 else 192, dtype=np.uint8)
        _check(_lib.bh_srs_get(self.h, i, _ptr(out)))
        return out.tobytes()

    def __del__(self):
        try:
            _lib.bh_srs_free(self.h)
        except Exception:
            pass


class FullDensity:
    """multiexp.rs:96-115"""


def multiexp(ctx, bases, offset, density, exponents, montgomery=False):
    """multiexp::multiexp (multiexp.rs:252-281).  density: FullDensity/None or
    a DensityTracker / list of bools; exponents: list of ints or an (n,4)
    uint64 array (canonical, or Montgomery when montgomery=True).
    Returns the uncompressed encoding of the affine result."""
    if isinstance(exponents, np.ndarray):
        ex = np.ascontiguousarray(exponents, dtype=np.uint64).reshape(-1, 4)
    else:
        ex = fr_to_mont(exponents) if montgomery else fr_to_canonical_limbs(exponents)
    n = ex.shape[0]
    dw, nbits = _density(density)
    out = np.zeros(96 if bases.group == BH_G1 else 192, dtype=np.uint8)
    _check(_lib.bh_multiexp(ctx.h, bases.h, offset, _ptr(dw), nbits,
                            _ptr(ex) if n else None, n,
                            BH_SCALARS_MONTGOMERY if montgomery else BH_SCALARS_CANONICAL, _ptr(out)),
           "bh_multiexp")
    return out.tobytes()


class Waiter:
    """multicore.rs:94-110: the pending result of multiexp_async; wait() returns the
    uncompressed affine point (or raises the multiexp's SynthesisError)."""

    def __init__(self, handle, group, ctx=None, bases=None):
        # the context and bases stay referenced until the wait: garbage collection cannot
        # destroy them under a multiexp in flight (an explicit ctx.close() detaches the job:
        # wait() then raises)
        self.h, self.group, self._ctx, self._bases = handle, group, ctx, bases

    def wait(self):
        if self.h is None:
            raise RuntimeError("Waiter already waited")
        out = np.zeros(96 if self.group == BH_G1 else 192, dtype=np.uint8)
        h, self.h = self.h, None
        try:
            _check(_lib.bh_multiexp_wait(h, _ptr(out)), "bh_multiexp_wait")
        finally:
            self._ctx = self._bases = None
        return out.tobytes()

    def __del__(self):
        if getattr(self, "h", None) is not None:
            try:
                _lib.bh_multiexp_wait(self.h, None)
            except Exception:
                pass


class Scalars:
    """A device-resident Arc<Vec<Fr::Repr>> (bh_scalars): uploaded once (bh_scalars_upload) or
    produced on the device (compute_h_scalars), read by any number of multiexp_async calls."""

    def __init__(self, ctx, exponents=None, montgomery=False, _handle=None):
        self.ctx = ctx
        if _handle is not None:
            self.h = _handle
            return
        if isinstance(exponents, np.ndarray):
            ex = np.ascontiguousarray(exponents, dtype=np.uint64).reshape(-1, 4)
        else:
            ex = fr_to_mont(exponents) if montgomery else fr_to_canonical_limbs(exponents)
        h = ctypes.c_void_p()
        _check(_lib.bh_scalars_upload(ctx.h, _ptr(ex) if ex.shape[0] else None, ex.shape[0],
                                      BH_SCALARS_MONTGOMERY if montgomery else BH_SCALARS_CANONICAL,
                                      ctypes.byref(h)), "bh_scalars_upload")
        self.h = h

    def __len__(self):
        return _lib.bh_scalars_len(self.h)

    def sync(self):
        """bh_scalars_sync: the producer has read its host buffers (and reports the H status)."""
        _check(_lib.bh_scalars_sync(self.h), "bh_scalars_sync")
        self._keep = None

    def stamps(self):
        """bh_scalars_stamps: the producer's stage times (ms since compute_h_scalars): a, b, c copies
        enqueued, H enqueued, deferred multiexps enqueued, and how many were deferred."""
        out = (ctypes.c_double * 6)()
        _check(_lib.bh_scalars_stamps(self.h, out), "bh_scalars_stamps")
        return [round(x, 3) for x in out]

    def close(self):
        if getattr(self, "h", None):
            _lib.bh_scalars_free(self.h)  # returns once a producer no longer reads _keep
            self.h = None
        self._keep = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def compute_h_scalars(ctx, a, b, c):
    """The H block (prover.rs:210-231) leaving h on the device: a Scalars of m-1 entries.
    a, b, c: (n,4) Montgomery arrays (or lists of ints); computed asynchronously."""
    A, B, C = (np.ascontiguousarray(x, dtype=np.uint64).reshape(-1, 4) if isinstance(x, np.ndarray)
               else fr_to_mont(x) for x in (a, b, c))
    n = A.shape[0]
    assert B.shape[0] == n and C.shape[0] == n
    h = ctypes.c_void_p()
    _check(_lib.bh_compute_h_scalars(ctx.h, _ptr(A), _ptr(B), _ptr(C), n, ctypes.byref(h)), "bh_compute_h_scalars")
    out = Scalars(ctx, _handle=h)
    out._keep = (A, B, C)  # read asynchronously: referenced until sync() or close()
    return out


class ParamsBases:
    """A Parameters vector as multiexp bases (ParameterSource::get_*, groth16/mod.rs:414-477):
    borrowed from the Parameters, which it keeps referenced."""

    def __init__(self, params, which):
        h = ctypes.c_void_p()
        _check(_lib.bh_params_vector(params.h, which, ctypes.byref(h)), "bh_params_vector")
        self.h, self.params = h, params
        self.group = BH_G2 if which == BH_VEC_B_G2 else BH_G1

    def __len__(self):
        return _lib.bh_srs_len(self.h)


def multiexp_async(ctx, bases, offset, density, exponents, montgomery=False):
    """multiexp::multiexp returning a Waiter (bh_multiexp_submit); arguments as multiexp(), or
    exponents = a Scalars (device-resident; bh_multiexp_submit_scalars)."""
    if isinstance(exponents, Scalars):
        dw, nbits = _density(density)
        h = ctypes.c_void_p()
        _check(_lib.bh_multiexp_submit_scalars(ctx.h, bases.h, offset, _ptr(dw), nbits, exponents.h,
                                               ctypes.byref(h)), "bh_multiexp_submit_scalars")
        return Waiter(h, bases.group, ctx, (bases, exponents))
    if isinstance(exponents, np.ndarray):
        ex = np.ascontiguousarray(exponents, dtype=np.uint64).reshape(-1, 4)
    else:
        ex = fr_to_mont(exponents) if montgomery else fr_to_canonical_limbs(exponents)
    n = ex.shape[0]
    dw, nbits = _density(density)
    h = ctypes.c_void_p()
    _check(_lib.bh_multiexp_submit(ctx.h, bases.h, offset, _ptr(dw), nbits,
                                   _ptr(ex) if n else None, n,
                                   BH_SCALARS_MONTGOMERY if montgomery else BH_SCALARS_CANONICAL, ctypes.byref(h)),
           "bh_multiexp_submit")
    return Waiter(h, bases.group, ctx, bases)


# ------------------------------------------------------------------ EvaluationDomain
class EvaluationDomain:
    """domain.rs:21-190 over Scalar<Fr>; coefficients live as (m,4) Montgomery limbs."""

    def __init__(self, ctx, coeffs):
        """from_coeffs (domain.rs:47-79): coeffs = list of ints or (n,4) Montgomery array."""
        arr = coeffs if isinstance(coeffs, np.ndarray) else fr_to_mont(coeffs)
        arr = np.ascontiguousarray(arr, dtype=np.uint64).reshape(-1, 4)
        m = ctypes.c_size_t()
        e = ctypes.c_uint32()
        _check(_lib.bh_domain_size(arr.shape[0], ctypes.byref(m), ctypes.byref(e)), "from_coeffs")
        self.m, self.exp = m.value, e.value
        self.coeffs = np.zeros((self.m, 4), dtype=np.uint64)
        self.coeffs[: arr.shape[0]] = arr
        self.ctx = ctx

    from_coeffs = classmethod(lambda cls, ctx, coeffs: cls(ctx, coeffs))

    def _run(self, f):
        _check(f(self.ctx.h, _ptr(self.coeffs), self.exp))

    def fft(self):
        self._run(_lib.bh_fft)

    def ifft(self):
        self._run(_lib.bh_ifft)

    def coset_fft(self):
        self._run(_lib.bh_coset_fft)

    def icoset_fft(self):
        self._run(_lib.bh_icoset_fft)

    def divide_by_z_on_coset(self):
        self._run(_lib.bh_divide_by_z_on_coset)

    def distribute_powers(self, g):
        gm = fr_to_mont([g])[0]
        _check(_lib.bh_distribute_powers(self.ctx.h, _ptr(self.coeffs), self.m, _ptr(gm)))

    def mul_assign(self, other):
        assert self.m == other.m
        _check(_lib.bh_mul_assign(self.ctx.h, _ptr(self.coeffs), _ptr(other.coeffs), self.m))

    def sub_assign(self, other):
        assert self.m == other.m
        _check(_lib.bh_sub_assign(self.ctx.h, _ptr(self.coeffs), _ptr(other.coeffs), self.m))

    def into_coeffs(self):
        return fr_from_mont(self.coeffs)


class ResidentEvaluationDomain:
    """EvaluationDomain (domain.rs:21-190) whose coefficients stay in HBM between calls
    (bh_evdom_*): the methods enqueue device work, only as_ref / into_coeffs / into_scalars read
    back.  from_coeffs reads the host array asynchronously (kept referenced until sync)."""

    def __init__(self, ctx, coeffs):
        arr = coeffs if isinstance(coeffs, np.ndarray) else fr_to_mont(coeffs)
        arr = np.ascontiguousarray(arr, dtype=np.uint64).reshape(-1, 4)
        h = ctypes.c_void_p()
        _check(_lib.bh_evdom_from_coeffs(ctx.h, _ptr(arr) if arr.shape[0] else None, arr.shape[0], ctypes.byref(h)),
               "from_coeffs")
        self.ctx, self.h, self._keep = ctx, h, arr
        m = ctypes.c_size_t()
        e = ctypes.c_uint32()
        _check(_lib.bh_evdom_size(h, ctypes.byref(m), ctypes.byref(e)))
        self.m, self.exp = m.value, e.value

    from_coeffs = classmethod(lambda cls, ctx, coeffs: cls(ctx, coeffs))

    def _run(self, f, *args):
        _check(f(self.h, *args))

    def fft(self):
        self._run(_lib.bh_evdom_fft)

    def ifft(self):
        self._run(_lib.bh_evdom_ifft)

    def coset_fft(self):
        self._run(_lib.bh_evdom_coset_fft)

    def icoset_fft(self):
        self._run(_lib.bh_evdom_icoset_fft)

    def divide_by_z_on_coset(self):
        self._run(_lib.bh_evdom_divide_by_z_on_coset)

    def distribute_powers(self, g):
        gm = fr_to_mont([g])[0]
        self._run(_lib.bh_evdom_distribute_powers, _ptr(gm))

    def mul_assign(self, other):
        self._run(_lib.bh_evdom_mul_assign, other.h)

    def sub_assign(self, other):
        self._run(_lib.bh_evdom_sub_assign, other.h)

    def sync(self):
        """bh_evdom_sync: the upload has read the host array."""
        self._run(_lib.bh_evdom_sync)
        self._keep = None

    def as_mont(self, n=None, out=None):
        """as_ref (domain.rs:28-32): the first n (default m) coefficients, (n,4) Montgomery
        (into `out` when given: a caller's reused buffer)."""
        n = self.m if n is None else n
        if out is None:
            out = np.zeros((max(n, 1), 4), dtype=np.uint64)
        assert out.dtype == np.uint64 and out.flags.c_contiguous and out.shape[0] >= n
        self._run(_lib.bh_evdom_read, _ptr(out), n)
        return out[:n]

    def as_ref(self):
        return fr_from_mont(self.as_mont())

    def into_coeffs(self):
        return self.as_ref()

    def write(self, coeffs):
        """as_mut written back (domain.rs:34-38): replaces the coefficients (zero padded)."""
        arr = coeffs if isinstance(coeffs, np.ndarray) else fr_to_mont(coeffs)
        arr = np.ascontiguousarray(arr, dtype=np.uint64).reshape(-1, 4)
        self._run(_lib.bh_evdom_write, _ptr(arr) if arr.shape[0] else None, arr.shape[0])
        self._keep = arr

    def into_scalars(self, n):
        """prover.rs:226-231 on the device: the first n coefficients as a Scalars vector
        (canonical), ready for multiexp_async; consumes the domain."""
        h = ctypes.c_void_p()
        self._run(_lib.bh_evdom_into_scalars, n, ctypes.byref(h))
        return Scalars(self.ctx, _handle=h)

    def close(self):
        if getattr(self, "h", None):
            _lib.bh_evdom_free(self.h)
            self.h = None
        self._keep = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def compute_h_resident(ctx, a, b, c, scalars=False):
    """The H block through the resident EvaluationDomain exactly as create_proof drives it
    (prover.rs:210-231, ten calls): h as a list of m-1 ints, or as a device Scalars."""
    da, db, dc = (ResidentEvaluationDomain(ctx, x) for x in (a, b, c))
    try:
        da.ifft()
        da.coset_fft()
        db.ifft()
        db.coset_fft()
        dc.ifft()
        dc.coset_fft()
        da.mul_assign(db)
        da.sub_assign(dc)
        da.divide_by_z_on_coset()
        da.icoset_fft()
        if scalars:
            return da.into_scalars(da.m - 1)
        return fr_from_mont(da.as_mont(da.m - 1))
    finally:
        for d in (da, db, dc):
            d.close()


def compute_h(ctx, a, b, c):
    """H block of create_proof (prover.rs:210-231) -> list of m-1 ints."""
    A, B, C = (x if isinstance(x, np.ndarray) else fr_to_mont(x) for x in (a, b, c))
    n = A.shape[0]
    m = ctypes.c_size_t()
    _check(_lib.bh_domain_size(n, ctypes.byref(m), None))
    out = np.zeros((max(m.value - 1, 1), 4), dtype=np.uint64)
    hl = ctypes.c_size_t()
    _check(_lib.bh_compute_h(ctx.h, _ptr(A), _ptr(B), _ptr(C), n, _ptr(out), ctypes.byref(hl)))
    return fr_from_mont(out[: hl.value])


# ------------------------------------------------------------------ Parameters
class Parameters:
    """Device-resident Parameters<Bls12> (groth16/mod.rs:224-247)."""

    def __init__(self, ctx, handle):
        self.ctx, self.h = ctx, handle

    @classmethod
    def read(cls, ctx, data: bytes, checked=True):
        buf = np.frombuffer(data, dtype=np.uint8)
        h = ctypes.c_void_p()
        _check(_lib.bh_params_load(ctx.h, _ptr(buf), len(data), int(checked), ctypes.byref(h)), "Parameters::read")
        return cls(ctx, h)

    @classmethod
    def chain(cls, ctx, rounds, seed=7, alpha=6, beta=24, gamma=6, delta=24, tau=2):
        h = ctypes.c_void_p()
        _check(_lib.bh_chain_params(ctx.h, rounds, seed, alpha, beta, gamma, delta, tau, ctypes.byref(h)),
               "bh_chain_params")
        return cls(ctx, h)

    def sizes(self):
        out = (ctypes.c_size_t * 6)()
        _check(_lib.bh_params_sizes(self.h, out))
        return dict(zip(["h", "l", "a", "b_g1", "b_g2", "ic"], list(out)))

    def write(self):
        n = ctypes.c_size_t()
        _check(_lib.bh_params_write(self.h, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, dtype=np.uint8)
        _check(_lib.bh_params_write(self.h, _ptr(out), n.value, ctypes.byref(n)))
        return out.tobytes()

    def vector(self, which):
        """ParameterSource::get_h/get_l/get_a/get_b_g1/get_b_g2: BH_VEC_* -> multiexp bases."""
        return ParamsBases(self, which)

    def prepare(self, witness, nshards=1):
        """Build the prover window tables now rather than inside the first proof."""
        _check(_lib.bh_params_prepare(self.ctx.h, self.h, witness.h, nshards), "bh_params_prepare")

    def prepare_shard(self, witness, shard, nshards, distributed_h=True):
        """Build only the table slices shard `shard` of `nshards` uses (a rank's 1/N share)."""
        _check(_lib.bh_params_prepare_shard(self.ctx.h, self.h, witness.h, shard, nshards, int(bool(distributed_h))),
               "bh_params_prepare_shard")

    def vk_bytes(self):
        """VerifyingKey::write (groth16/mod.rs:146-159)."""
        n = ctypes.c_size_t()
        _check(_lib.bh_vk_write(self.h, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, dtype=np.uint8)
        _check(_lib.bh_vk_write(self.h, _ptr(out), n.value, ctypes.byref(n)))
        return out.tobytes()

    def __del__(self):
        try:
            _lib.bh_params_free(self.h)
        except Exception:
            pass


# ------------------------------------------------------------------ R1CS host API (lib.rs)
class Variable:
    __slots__ = ("kind", "index")

    def __init__(self, kind, index):
        self.kind, self.index = kind, index


ONE = Variable("input", 0)


class LinearCombination:
    """lib.rs:240-350"""

    def __init__(self, terms=None):
        self.terms = list(terms or [])

    @staticmethod
    def zero():
        return LinearCombination()

    def __add__(self, o):
        if isinstance(o, Variable):
            return LinearCombination(self.terms + [(o, 1)])
        if isinstance(o, LinearCombination):
            return LinearCombination(self.terms + o.terms)
        coeff, x = o
        if isinstance(x, LinearCombination):
            return LinearCombination(self.terms + [(v, c * coeff) for v, c in x.terms])
        return LinearCombination(self.terms + [(x, coeff)])

    def __sub__(self, o):
        if isinstance(o, Variable):
            return LinearCombination(self.terms + [(o, -1)])
        if isinstance(o, LinearCombination):
            return LinearCombination(self.terms + [(v, -c) for v, c in o.terms])
        coeff, x = o
        if isinstance(x, LinearCombination):
            return LinearCombination(self.terms + [(v, -c * coeff) for v, c in x.terms])
        return LinearCombination(self.terms + [(x, -coeff)])


class DensityTracker:
    """multiexp.rs:117-157"""

    def __init__(self):
        self.bv = []

    def add_element(self):
        self.bv.append(False)

    def inc(self, i):
        self.bv[i] = True

    def get_total_density(self):
        return sum(self.bv)


class ProvingAssignment:
    """prover.rs:55-156 (host-side witness assignment and density tracking)."""

    def __init__(self):
        self.a_aux_density, self.b_input_density, self.b_aux_density = DensityTracker(), DensityTracker(), DensityTracker()
        self.a, self.b, self.c = [], [], []
        self.input_assignment, self.aux_assignment = [], []

    @staticmethod
    def one():
        return ONE

    def namespace(self, name):
        return self

    def alloc(self, name, f):
        v = f()
        if v is None:
            raise AssignmentMissing()
        self.aux_assignment.append(int(v) % R_MODULUS)
        self.a_aux_density.add_element()
        self.b_aux_density.add_element()
        return Variable("aux", len(self.aux_assignment) - 1)

    def alloc_input(self, name, f):
        v = f()
        if v is None:
            raise AssignmentMissing()
        self.input_assignment.append(int(v) % R_MODULUS)
        self.b_input_density.add_element()
        return Variable("input", len(self.input_assignment) - 1)

    def _eval(self, lc, in_d, aux_d):
        acc = 0
        for v, coeff in lc.terms:
            if v.kind == "input":
                t = self.input_assignment[v.index]
                if in_d is not None:
                    in_d.inc(v.index)
            else:
                t = self.aux_assignment[v.index]
                if aux_d is not None:
                    aux_d.inc(v.index)
            acc += t * coeff
        return acc % R_MODULUS

    def enforce(self, name, la, lb, lc):
        z = LinearCombination.zero
        self.a.append(self._eval(la(z()), None, self.a_aux_density))
        self.b.append(self._eval(lb(z()), self.b_input_density, self.b_aux_density))
        self.c.append(self._eval(lc(z()), None, None))


def synthesize(circuit):
    """prover.rs:187-204"""
    p = ProvingAssignment()
    p.alloc_input("", lambda: 1)
    circuit.synthesize(p)
    for i in range(len(p.input_assignment)):
        p.enforce("", lambda lc, i=i: lc + Variable("input", i), lambda lc: lc, lambda lc: lc)
    return p


class Witness:
    """A complete assignment resident in HBM (bh_witness)."""

    def __init__(self, ctx, handle, num_constraints):
        self.ctx, self.h, self.num_constraints = ctx, handle, num_constraints

    @classmethod
    def from_assignment(cls, ctx, p):
        arrs = [fr_to_mont(x) for x in (p.a, p.b, p.c, p.input_assignment, p.aux_assignment)]
        dens = [density_words(d.bv) for d in (p.a_aux_density, p.b_input_density, p.b_aux_density)]
        h = ctypes.c_void_p()
        _check(_lib.bh_witness_upload(ctx.h, _ptr(arrs[0]), _ptr(arrs[1]), _ptr(arrs[2]), len(p.a),
                                      _ptr(arrs[3]), len(p.input_assignment), _ptr(arrs[4]),
                                      len(p.aux_assignment), _ptr(dens[0]), _ptr(dens[1]), _ptr(dens[2]),
                                      ctypes.byref(h)), "bh_witness_upload")
        return cls(ctx, h, len(p.a))

    @classmethod
    def chain(cls, ctx, rounds, seed=7, preimage_seed=None):
        """Native MiMC-chain synthesis: constants from seed, preimage from preimage_seed
        (default seed + 1)."""
        h = ctypes.c_void_p()
        ps = seed + 1 if preimage_seed is None else preimage_seed
        _check(_lib.bh_chain_witness_preimage(ctx.h, rounds, seed, ps, ctypes.byref(h)), "bh_chain_witness")
        return cls(ctx, h, 2 * rounds + 2)

    def __del__(self):
        try:
            _lib.bh_witness_free(self.h)
        except Exception:
            pass


def prove_witness(ctx, params, witness, r, s):
    """create_proof after synthesis (prover.rs:206-349) -> Proof::write bytes (192)."""
    out = np.zeros(192, dtype=np.uint8)
    rr, ss = fr_to_canonical_limbs([r])[0], fr_to_canonical_limbs([s])[0]
    _check(_lib.bh_prove_witness(ctx.h, params.h, witness.h, _ptr(rr), _ptr(ss), _ptr(out)), "create_proof")
    return out.tobytes()


def chain_assignment(rounds, seed=7, preimage_seed=None):
    """The MiMC chain's ProvingAssignment on the host (bh_chain_assignment) in the layouts of
    bh_prove: a/b/c/inputs/aux as (n,4) uint64 Montgomery, densities as uint64 bit words."""
    sz = (ctypes.c_size_t * 3)()
    _check(_lib.bh_chain_sizes(rounds, sz), "bh_chain_sizes")
    nc, ni, na = sz
    out = {k: np.zeros((n, 4), dtype=np.uint64) for k, n in (("a", nc), ("b", nc), ("c", nc), ("inputs", ni),
                                                              ("aux", na))}
    out["a_aux_density"] = np.zeros((na + 63) // 64, dtype=np.uint64)
    out["b_input_density"] = np.zeros((ni + 63) // 64, dtype=np.uint64)
    out["b_aux_density"] = np.zeros((na + 63) // 64, dtype=np.uint64)
    ps = seed + 1 if preimage_seed is None else preimage_seed
    _check(_lib.bh_chain_assignment(rounds, seed, ps, *[_ptr(out[k]) for k in (
        "a", "b", "c", "inputs", "aux", "a_aux_density", "b_input_density", "b_aux_density")]), "bh_chain_assignment")
    return out


def prove(ctx, params, asg, r, s):
    """bh_prove: create_proof after synthesis straight from host buffers (the drop-in entry
    point of INTEGRATION.md section 1).  asg: dict as returned by chain_assignment."""
    out = np.zeros(192, dtype=np.uint8)
    rr, ss = fr_to_canonical_limbs([r])[0], fr_to_canonical_limbs([s])[0]
    A = [np.ascontiguousarray(asg[k], dtype=np.uint64) for k in ("a", "b", "c", "inputs", "aux")]
    D = [np.ascontiguousarray(asg[k], dtype=np.uint64) for k in ("a_aux_density", "b_input_density", "b_aux_density")]
    _check(_lib.bh_prove(ctx.h, params.h, _ptr(A[0]), _ptr(A[1]), _ptr(A[2]), A[0].shape[0], _ptr(A[3]),
                         A[3].shape[0], _ptr(A[4]), A[4].shape[0], _ptr(D[0]), _ptr(D[1]), _ptr(D[2]), _ptr(rr),
                         _ptr(ss), _ptr(out)), "bh_prove")
    return out.tobytes()


def prove_seam(ctx, params, asg, r, s, profile=None, h_via_domain=False):
    """create_proof after synthesis (prover.rs:206-349) through the multiexp seam alone, as a
    Rust caller that swaps only multiexp() and the H block sees it: h on the device
    (bh_compute_h_scalars), the assignments uploaded once (the Arcs of prover.rs:233-250), the
    eight multiexps in flight on the Parameters' own vectors (get_h ... get_b_g2, so their window
    tables apply), waited, and the proof assembled on the host (prover.rs:315-349).
    asg: dict as returned by chain_assignment.  Byte-equal to prove().  h_via_domain: the H block
    through the resident EvaluationDomain's ten calls instead (compute_h_resident), h handed to
    the multiexp as a device vector (into_scalars), as a caller swapping EvaluationDomain too."""
    ni, na = asg["inputs"].shape[0], asg["aux"].shape[0]
    if h_via_domain:
        h = compute_h_resident(ctx, asg["a"], asg["b"], asg["c"], scalars=True)
    else:
        h = compute_h_scalars(ctx, asg["a"], asg["b"], asg["c"])
    inp = Scalars(ctx, asg["inputs"], montgomery=True)
    aux = Scalars(ctx, asg["aux"], montgomery=True)
    a_aux = DensityWords(asg["a_aux_density"], na)
    b_in = DensityWords(asg["b_input_density"], ni)
    b_aux = DensityWords(asg["b_aux_density"], na)
    b_in_total = b_in.total()
    H, L, A, B1, B2 = (params.vector(k) for k in (BH_VEC_H, BH_VEC_L, BH_VEC_A, BH_VEC_B_G1, BH_VEC_B_G2))
    waiters = [multiexp_async(ctx, H, 0, None, h), multiexp_async(ctx, L, 0, None, aux),
               multiexp_async(ctx, A, 0, None, inp), multiexp_async(ctx, A, ni, a_aux, aux),
               multiexp_async(ctx, B1, 0, b_in, inp), multiexp_async(ctx, B1, b_in_total, b_aux, aux),
               multiexp_async(ctx, B2, 0, b_in, inp), multiexp_async(ctx, B2, b_in_total, b_aux, aux)]
    partial = b"".join(w.wait() for w in waiters)
    if profile is not None and not h_via_domain:  # the h producer's stage times (bh_scalars_stamps)
        profile.append(h.stamps())
    return proof_from_partials(params.vk_bytes(), partial, 1, r, s)


def prove_batch(ctx, params, witnesses, r, s, lanes=0):
    """Throughput mode: len(witnesses) independent proofs pipelined on one device
    (bh_prove_batch) -> list of Proof::write bytes."""
    k = len(witnesses)
    wa = (ctypes.c_void_p * max(k, 1))(*[w.h.value for w in witnesses])
    out = np.zeros(max(k, 1) * 192, dtype=np.uint8)
    rr, ss = fr_to_canonical_limbs([r])[0], fr_to_canonical_limbs([s])[0]
    _check(_lib.bh_prove_batch(ctx.h, params.h, wa, k, _ptr(rr), _ptr(ss), lanes, _ptr(out)), "bh_prove_batch")
    return [out[192 * i:192 * (i + 1)].tobytes() for i in range(k)]


def create_proof(ctx, circuit, params, r, s):
    """prover.rs:175-350: synthesize on the host, prove on the device."""
    p = synthesize(circuit)
    w = Witness.from_assignment(ctx, p)
    return prove_witness(ctx, params, w, r, s)


def create_random_proof(ctx, circuit, params, rng=None):
    """prover.rs:158-173: the fork ignores rng and uses r = 27134, s = 17146."""
    return create_proof(ctx, circuit, params, 27134, 17146)


# ------------------------------------------------------------------ multi-GPU (MSM sharding)
def shard_range(n, shard, nshards):
    lo, hi = ctypes.c_size_t(), ctypes.c_size_t()
    _check(_lib.bh_shard_range(n, shard, nshards, ctypes.byref(lo), ctypes.byref(hi)))
    return lo.value, hi.value


def prove_witness_partial(ctx, params, witness, shard, nshards):
    """This rank's partial sums of the 8 multiexps (960 bytes)."""
    out = np.zeros(PARTIAL_BYTES, dtype=np.uint8)
    _check(_lib.bh_prove_witness_partial(ctx.h, params.h, witness.h, shard, nshards, _ptr(out)), "partial")
    return out.tobytes()


def prove_witness_partials_local(ctx, params, witness, nshards):
    """All nshards partial records on this one device (distributed H emulated with device
    copies): the multi-GPU algorithm end to end without a second GPU."""
    out = np.zeros(nshards * PARTIAL_BYTES, dtype=np.uint8)
    _check(_lib.bh_prove_witness_partials_local(ctx.h, params.h, witness.h, nshards, _ptr(out)), "partials_local")
    return out.tobytes()


def prove_witness_partials_ranks(ctxs, params_list, witness):
    """N ranks of one device with their own contexts and Parameters (bh_prove_witness_partials_ranks)."""
    n = len(ctxs)
    assert len(params_list) == n
    ca = (ctypes.c_void_p * n)(*[c.h.value for c in ctxs])
    pa = (ctypes.c_void_p * n)(*[p.h.value for p in params_list])
    out = np.zeros(n * PARTIAL_BYTES, dtype=np.uint8)
    _check(_lib.bh_prove_witness_partials_ranks(ca, pa, witness.h, n, _ptr(out)), "partials_ranks")
    return out.tobytes()


def rehearse_rank(ctx, params, witness, rank, nranks):
    """Rank `rank` of an nranks-GPU run on this device (bh_rehearse_rank): host ms of its proof."""
    ms = ctypes.c_double()
    _check(_lib.bh_rehearse_rank(ctx.h, params.h, witness.h, rank, nranks, ctypes.byref(ms)), "rehearse_rank")
    return ms.value


def proof_from_partials(vk_bytes, partials, nshards, r, s):
    """Host-only: sum the gathered partials (shard order) and assemble the proof."""
    vk = np.frombuffer(vk_bytes, dtype=np.uint8)
    parts = np.frombuffer(partials, dtype=np.uint8)
    assert parts.size == nshards * PARTIAL_BYTES
    out = np.zeros(192, dtype=np.uint8)
    rr, ss = fr_to_canonical_limbs([r])[0], fr_to_canonical_limbs([s])[0]
    _check(_lib.bh_proof_from_partials(_ptr(vk), vk.size, _ptr(parts), nshards, _ptr(rr), _ptr(ss), _ptr(out)),
           "proof_from_partials")
    return out.tobytes()


def verify_proof(vk_bytes, proof, public_inputs):
    """verify_proof (verifier.rs:11-62) on the host: vk = VerifyingKey::write bytes (or the
    head of Parameters::write), proof = Proof::write bytes, public_inputs = ints without ONE.
    Raises on malformed data (e.g. the wrong number of inputs); returns bool."""
    vk = np.frombuffer(bytes(vk_bytes), dtype=np.uint8)
    pf = np.frombuffer(bytes(proof), dtype=np.uint8)
    assert pf.size == 192
    ins = fr_to_canonical_limbs(public_inputs) if public_inputs else np.zeros((1, 4), dtype=np.uint64)
    ok = ctypes.c_int()
    _check(_lib.bh_verify_proof(_ptr(vk), vk.size, _ptr(pf), _ptr(ins), len(public_inputs), ctypes.byref(ok)),
           "verify_proof")
    return bool(ok.value)


def verify_batch(vk_bytes, proofs, public_inputs, zs):
    """Batch verifier (verifier/batch.rs:95-169): proofs = list of 192-byte proofs,
    public_inputs = list (one per proof) of input lists, zs = the random nonzero scalars."""
    k = len(proofs)
    vk = np.frombuffer(bytes(vk_bytes), dtype=np.uint8)
    pf = np.frombuffer(b"".join(bytes(p) for p in proofs) or b"\0", dtype=np.uint8)
    ni = len(public_inputs[0]) if k else 0
    flat = [x for row in public_inputs for x in row]
    ins = fr_to_canonical_limbs(flat) if flat else np.zeros((1, 4), dtype=np.uint64)
    z = fr_to_canonical_limbs(zs) if zs else np.zeros((1, 4), dtype=np.uint64)
    ok = ctypes.c_int()
    _check(_lib.bh_verify_batch(_ptr(vk), vk.size, _ptr(pf), _ptr(ins), ni, k, _ptr(z), ctypes.byref(ok)),
           "verify_batch")
    return bool(ok.value)


def device_count():
    return _lib.bh_device_count()


class Comm:
    """RCCL communicator for the partial-sum exchange (bh_comm_*)."""

    @staticmethod
    def unique_id():
        out = np.zeros(128, dtype=np.uint8)
        _check(_lib.bh_comm_unique_id(_ptr(out)), "ncclGetUniqueId")
        return out.tobytes()

    def __init__(self, ctx, uid, nranks, rank):
        b = np.frombuffer(uid, dtype=np.uint8)
        h = ctypes.c_void_p()
        _check(_lib.bh_comm_init(ctx.h, _ptr(b), nranks, rank, ctypes.byref(h)), "ncclCommInitRank")
        self.h, self.nranks = h, nranks

    def prove_partial(self, ctx, params, witness):
        """This rank's partial record with the H block distributed over the communicator
        (bh_prove_witness_partial_comm)."""
        out = np.zeros(PARTIAL_BYTES, dtype=np.uint8)
        _check(_lib.bh_prove_witness_partial_comm(ctx.h, params.h, witness.h, self.h, _ptr(out)), "partial_comm")
        return out.tobytes()

    def allgather(self, partial):
        src = np.frombuffer(partial, dtype=np.uint8)
        out = np.zeros(self.nranks * PARTIAL_BYTES, dtype=np.uint8)
        _check(_lib.bh_comm_allgather_partials(self.h, _ptr(src), _ptr(out)), "ncclAllGather")
        return out.tobytes()

    def allgather_bytes(self, rec):
        """Every rank's equal-length record, rank order (bh_comm_allgather)."""
        src = np.frombuffer(bytes(rec), dtype=np.uint8)
        out = np.zeros(self.nranks * src.size, dtype=np.uint8)
        _check(_lib.bh_comm_allgather(self.h, _ptr(src), src.size, _ptr(out)), "ncclAllGather")
        return [out[k * src.size:(k + 1) * src.size].tobytes() for k in range(self.nranks)]

    def allreduce_max(self, x):
        """Max of x over the ranks; also a barrier (bh_comm_allreduce_max)."""
        v = ctypes.c_double(float(x))
        _check(_lib.bh_comm_allreduce_max(self.h, ctypes.byref(v)), "ncclAllReduce")
        return v.value

    def info(self):
        """(rank count, this rank, HIP device) as RCCL reports them."""
        out = (ctypes.c_int * 3)()
        _check(_lib.bh_comm_info(self.h, out), "bh_comm_info")
        return tuple(out)

    def close(self):
        if self.h:
            _lib.bh_comm_destroy(self.h)
            self.h = None
