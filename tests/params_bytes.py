"""Slicing of Parameters::write bytes (groth16/mod.rs:260-290) into its vectors, for tests."""


def split_params(data):
    """-> dict with vk bytes and the raw uncompressed vectors h, l, a, b_g1 (96-B points) and
    b_g2 (192-B points) as bytes, plus their lengths."""
    off = 96 * 3 + 192 * 3
    n_ic = int.from_bytes(data[off:off + 4], "big")
    off += 4 + 96 * n_ic
    out = {"vk": data[:off]}
    for name, width in (("h", 96), ("l", 96), ("a", 96), ("b_g1", 96), ("b_g2", 192)):
        n = int.from_bytes(data[off:off + 4], "big")
        off += 4
        out[name] = data[off:off + n * width]
        out[name + "_len"] = n
        off += n * width
    assert off == len(data)
    return out
