"""CPU checks of the drop-in boundary: the shared library loads and exports
every symbol include/bellman_hip.h declares (no compute calls without a GPU)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "bellman_hip.h")).read()
    return sorted(set(re.findall(r"\b(bh_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "bellman-mpc_amd", "bellman_hip", "libbellman_hip.so"))
    syms = header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_python_layer_binds_every_header_symbol():
    import bellman_hip as bh
    assert sorted(bh.EXPORTED_SYMBOLS) == header_symbols()
    assert bh.lib().bh_version() == 1
    assert bh._status_string(2).startswith("I/O error")


def test_domain_size_rule():
    # EvaluationDomain::from_coeffs sizing (domain.rs:47-60), pure host logic
    import ctypes
    import bellman_hip as bh
    m = ctypes.c_size_t()
    e = ctypes.c_uint32()
    for n, (mm, ee) in {0: (1, 0), 1: (1, 0), 2: (2, 1), 3: (4, 2), 1025: (2048, 11)}.items():
        assert bh.lib().bh_domain_size(n, ctypes.byref(m), ctypes.byref(e)) == 0
        assert (m.value, e.value) == (mm, ee)
    assert bh.lib().bh_domain_size((1 << 32) + 1, ctypes.byref(m), ctypes.byref(e)) == 3
