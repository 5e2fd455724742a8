"""Debug: tiny G2/G1 multiexps with known answers (oracle-checked)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "bellman-mpc_amd"))
sys.path.insert(0, ROOT)
import bellman_hip as bh
from oracle import bls12_381 as O

g = json.load(open(os.path.join(ROOT, "tests/golden/golden.json")))
ctx = bh.Context(0)
for grp, key, C, dec, enc in ((bh.BH_G1, "msm_g1", O.G1, O.g1_from_uncompressed, O.g1_to_uncompressed),
                              (bh.BH_G2, "msm_g2", O.G2, O.g2_from_uncompressed, O.g2_to_uncompressed)):
    hexes = g[key]["bases"][:4]
    bases = bh.Bases(ctx, grp, b"".join(bytes.fromhex(h) for h in hexes))
    pts = [C.from_affine(dec(bytes.fromhex(h))[1]) for h in hexes]
    for exps in ([1], [2], [3], [1, 1], [5, 7], [255], [256], [2**20 + 3]):
        got = bh.multiexp(ctx, bases, 0, None, exps)
        acc = C.sum([C.mul(p, e) for e, p in zip(exps, pts)])
        exp = enc(C.to_affine(acc))
        print(key, exps, "OK" if got == exp else "BAD", flush=True)
