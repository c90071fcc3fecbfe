"""Random SNP pairs -- drop-in for gmat.remma.random_pair (random_pair.py:6-65), with an
optional ``seed`` (the reference draws from the unseeded global np.random)."""
import logging

import numpy as np

from .. import dist


def _draw(num_snp, out_file, num_pair, num_each_pair, accept, seed):
    rng = np.random.default_rng(seed) if seed is not None else np.random
    got, seen = [], set()
    while len(got) < num_pair:
        arr = rng.integers(num_snp, size=(num_each_pair, 2)) if seed is not None else \
            rng.randint(num_snp, size=(num_each_pair, 2))
        arr = arr[accept(arr)]
        for a, b in arr.tolist():
            if (a, b) not in seen:
                seen.add((a, b))
                got.append((a, b))
    res = np.array(got[:num_pair], dtype=np.int64)
    with open(out_file, "w") as f:
        f.write("snp_0 snp_1\n")
        f.write("".join("%d %d\n" % (a, b) for a, b in res.tolist()))
    return res


@dist.on_root
def random_pair(num_snp, out_file="random_pair", num_pair=100000, num_each_pair=5000, seed=None):
    """Unique random pairs i < j (AA / DD); writes out_file and returns the (num_pair, 2) array."""
    if num_pair > num_snp * (num_snp - 1) / 2:
        raise ValueError("num_pair must be not greater than: " + str(num_snp * (num_snp - 1) / 2))
    if num_pair < num_each_pair:
        raise ValueError("num_pair must be greater than num_each_pair")
    return _draw(num_snp, out_file, num_pair, num_each_pair, lambda a: a[:, 0] < a[:, 1], seed)


@dist.on_root
def random_pairAD(num_snp, out_file="random_pair", num_pair=100000, num_each_pair=5000, seed=None):
    """Unique random ordered pairs i != j (AD)."""
    if num_pair > num_snp * (num_snp - 1):
        raise ValueError("num_pair must be not greater than: " + str(num_snp * (num_snp - 1)))
    if num_pair < num_each_pair:
        raise ValueError("num_pair must be greater than num_each_pair")
    return _draw(num_snp, out_file, num_pair, num_each_pair, lambda a: a[:, 0] != a[:, 1], seed)
