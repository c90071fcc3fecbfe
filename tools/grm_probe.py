"""GRM kernel timing over panel sizes (random imputed codes, no missing): the int8 SYRK's time per
call (gmat_grm_stats), its issued-ops rate against the int8 peak and the whole call's device time, so
the per-stage cost and the fixed (slot / epilogue) cost can be separated.
   python tools/grm_probe.py [N:M ...]   (default 2000:20000 2000:80000 5000:100000)
A checksum of the additive GRM of the first size is printed for A/Bs (the result is exact integers
scaled in fp64, so it must not change)."""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

INT8_PEAK_TOPS = 5000.0


def body_of(rng, n, m):
    codes = rng.choice(np.array([0, 2, 3], dtype=np.uint8), size=(m, (n + 3) // 4 * 4))
    codes[:, n:] = 0
    c = codes.reshape(m, -1, 4)
    return (c[:, :, 0] | (c[:, :, 1] << 2) | (c[:, :, 2] << 4) | (c[:, :, 3] << 6)).astype(np.uint8).ravel()


def main():
    from gmat_amd import _native as N
    from gmat_amd.plink import Geno
    lib = N.ensure_device()
    sizes = [tuple(map(int, a.split(":"))) for a in sys.argv[1:]] or [(2000, 20000), (2000, 80000), (5000, 100000)]
    rng = np.random.default_rng(1)
    out = {"lib": os.environ.get("GMAT_HIP_LIB", "gmat_amd/libgmat_hip.so")}
    for n, m in sizes:
        g = Geno(body=body_of(rng, n, m), n_id=n, n_snp=m)
        k = np.empty((n, n))
        sc = ctypes.c_double()
        st = np.zeros(4)
        rec = {}
        for kind in ((1, 0, 1, 0) if os.environ.get("GRM_PROBE_ORDER") == "interleave" else (0, 1)):
            ts = []
            for r in range(6):
                N.check(lib.gmat_grm(g.handle, kind, 0.001, N.ptr(k), ctypes.byref(sc)), "gmat_grm")
                N.check(lib.gmat_grm_stats(N.ptr(st)), "gmat_grm_stats")
                if r:
                    ts.append((st[0], st[3]))
            kern = float(np.median([t[0] for t in ts]))
            rec[("add" if kind == 0 else "dom") + ("" if ("add" if kind == 0 else "dom") not in rec else "2")] = {
                "kernel_us": kern * 1e6, "device_us": float(np.median([t[1] for t in ts])) * 1e6,
                "int8_frac": st[1] / kern / 1e12 / INT8_PEAK_TOPS,
                "sha": hashlib.sha256(k.tobytes()).hexdigest()[:16]}
        g.close()
        out["%dx%d" % (n, m)] = rec
    print(json.dumps(out))


if __name__ == "__main__":
    main()
