"""Two recorded hit sets of the same cohort (exhaustive_hits_*.npz of tools/full_triangle.py), e.g.
the exhaustive scan refined with the fp64 MFMA kernel (refine_kernel) against the one refined on int8
slices (refine8_kernel): identical (i, j) sets and the largest relative difference of eff / var /
chi / p.   python tools/compare_hits.py OLD.npz NEW.npz [OUT.json]"""
import json
import sys

import numpy as np


def main():
    a, b = (np.load(p) for p in sys.argv[1:3])
    ka = set(zip(a["i"].tolist(), a["j"].tolist()))
    kb = set(zip(b["i"].tolist(), b["j"].tolist()))
    out = {"old": sys.argv[1], "new": sys.argv[2], "old_hits": len(ka), "new_hits": len(kb),
           "symmetric_difference": len(ka ^ kb), "same_fingerprint": bytes(a["fingerprint"]) == bytes(b["fingerprint"])}
    if not ka ^ kb:
        oa = np.lexsort((a["j"], a["i"]))
        ob = np.lexsort((b["j"], b["i"]))
        for k in ("eff", "var", "chi", "p"):
            x, y = a[k][oa], b[k][ob]
            out["max_rel_diff_" + k] = float(np.max(np.abs(x - y) / np.maximum(np.abs(x), 1e-300)))
    print(json.dumps(out))
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)
    return 0 if not ka ^ kb else 3


if __name__ == "__main__":
    sys.exit(main())
